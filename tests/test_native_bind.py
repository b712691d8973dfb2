"""gsr_bind (csrc/gsr_bind.cpp) against _C.py's ctypes marshalling (-m gpu): the same library calls,
so the same outputs bit for bit, and the same error texts for the inputs _C.py rejects."""
import pytest
import torch

import splat_scenes as S
import splat_step
from diff_gaussian_rasterization import GaussianRasterizer, _C

pytestmark = pytest.mark.gpu


@pytest.fixture
def parts():
    prev = _C._NATIVE_PARTS
    if _C._native() is None:
        pytest.skip("gsr_bind.so not built")
    yield
    _C._NATIVE_PARTS = prev


def _summed_step(cfg, cams, act, dl, cuda, leaf):
    """The summed multi-view step: leaf inputs (deferred pass: forward, render half, multi-view call)
    or non-leaf ones (immediate backward)."""
    if leaf:
        leaves = {k: v.detach().clone().requires_grad_(True) for k, v in act.items()}
        st = splat_step.RenderStep(cuda, cams, lambda ci: dict(leaves, means2D=torch.zeros_like(
            leaves["means3D"], requires_grad=True)), dl, [torch.cuda.current_stream()], threads=False)
        imgs = st(list(range(len(cams))))
        st.close()
        torch.cuda.synchronize()
        return imgs, {k: v.grad.clone() for k, v in leaves.items()}
    params = {k: torch.nn.Parameter(v.detach().clone()) for k, v in act.items()}
    imgs = []
    for rs in cams:  # non-leaf inputs (as create_render_arguments makes them): the immediate backward
        args = {k: v * 1.0 for k, v in params.items()}
        args["means2D"] = torch.zeros_like(params["means3D"], requires_grad=True) + 0
        imgs.append(GaussianRasterizer(raster_settings=rs)(**args)[0])
    torch.stack([(i * dl).sum() for i in imgs]).sum().backward()
    torch.cuda.synchronize()
    return [i.detach() for i in imgs], {k: v.grad.clone() for k, v in params.items()}


@pytest.mark.parametrize("leaf", [True, False])
@pytest.mark.parametrize("sh_degree", [-1, 3])
def test_native_equals_ctypes(cuda, parts, leaf, sh_degree):
    cfg = S.CONFIGS["C2"]
    p = S.synthetic_cloud(20_000, cfg.s0, sh_degree=sh_degree, seed=3, device=cuda)
    with torch.no_grad():
        act = S.activated_inputs(p, sh_degree)
    act = {k: v for k, v in act.items() if v is not None and k != "means2D"}
    if sh_degree >= 0:
        act.pop("colors_precomp", None)
    W, H = 320, 240
    cams = [S.render_settings(W, H, S.intrinsics(300.0, W, H), S.look_at(yaw, 0.2, 5.0), device=cuda,
                              sh_degree=max(sh_degree, 0)) for yaw in (0, 90, 180)]
    dl = S.upstream_grad(H, W, device=cuda)
    out = {}
    for mode in (0, 15, 0, 15):  # twice each: the second pass of a mode speculates from the history
        _C._NATIVE_PARTS = mode
        out.setdefault(mode, []).append(_summed_step(cfg, cams, act, dl, cuda, leaf))
    for a, b in zip(out[0], out[15]):
        for x, y in zip(a[0], b[0]):
            assert torch.equal(x, y)
        assert a[1].keys() == b[1].keys()
        for k in a[1]:
            assert torch.equal(a[1][k], b[1][k]), k


def test_native_error_texts(cuda, parts):
    p = S.synthetic_cloud(500, 0.02, seed=1, device=cuda)
    with torch.no_grad():
        a = S.activated_inputs(p, -1)
    rs = S.render_settings(64, 48, S.intrinsics(64.0, 64, 48), S.look_at(0, 0.1, 4.0), device=cuda)
    e = torch.empty(0, device=cuda)

    def call(**over):
        x = dict(a, **over)
        return _C.rasterize_gaussians(rs.bg, x["means3D"], x["colors_precomp"], x["opacities"], x["scales"],
                                      x["rotations"], 1.0, e, rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy,
                                      rs.image_height, rs.image_width, e, 0, rs.campos, False)

    cases = [dict(means3D=a["means3D"][:, :2]), dict(opacities=a["opacities"].double()),
             dict(scales=a["scales"].cpu())]
    for over in cases:
        msgs = []
        for mode in (0, 15):
            _C._NATIVE_PARTS = mode
            with pytest.raises(RuntimeError) as ei:
                call(**over)
            msgs.append(str(ei.value))
        assert msgs[0] == msgs[1], msgs
