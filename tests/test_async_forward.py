"""Asynchronous forward (-m gpu; gsr_forward_async / gsr_forward_resolve / gsr_forward_release, ABI 17).

A forward whose (device, P, W, H) has pair-count history returns as soon as its kernels are queued,
without reading num_rendered back.  The device checks the speculative BINNING capacity after the tile
scan; when it fails, the library's resolver thread redoes the post-scan kernels exactly on its own
stream and the forward's last kernel (k_fwd_gate) holds the caller's stream until then.  Every output
must be bitwise the exact path's (images, radii, IMAGE arrays, and the backward, which reads BINNING
through the resolution), whether the speculation stood or was redone, and whatever the host does
next (an immediate device synchronisation included: the resolver needs nothing from the caller).
"""
import gc
import time

import pytest
import torch

import splat_scenes as S
import diff_gaussian_rasterization as dgr
from diff_gaussian_rasterization import GaussianRasterizer, _C

pytestmark = pytest.mark.gpu


def _forward(a, rs, mode):
    e = torch.empty(0, device=a["means3D"].device)
    info = {}
    out = _C.rasterize_gaussians(rs.bg, a["means3D"], a.get("colors_precomp", e), a["opacities"], a["scales"],
                                 a["rotations"], 1.0, e, rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy,
                                 rs.image_height, rs.image_width, a.get("shs", e), rs.sh_degree, rs.campos, False,
                                 prepare_backward=True, speculate=mode != "exact", info=info,
                                 nonblocking=mode == "async")
    return info, out


def _backward(a, rs, out, info, dl):
    e = torch.empty(0, device=a["means3D"].device)
    K, color, radii, geom, binning, img, depth = out
    layout, ptr = info["binning_layout"], None
    if info["pending"] is not None:
        K, layout, ptr = info["pending"].resolve()
    return _C.rasterize_gaussians_backward(rs.bg, a["means3D"], radii, a.get("colors_precomp", e), a["scales"],
                                           a["rotations"], 1.0, e, rs.viewmatrix, rs.projmatrix, rs.tanfovx,
                                           rs.tanfovy, dl, a.get("shs", e), rs.sh_degree, rs.campos, geom, K,
                                           binning, img, prepare_backward=True, binning_layout=layout,
                                           binning_ptr=ptr), K


def _run(a, rs, mode, dl, sync_first=False):
    info, out = _forward(a, rs, mode)
    if sync_first:  # the host blocks on the device before anything resolves the forward
        torch.cuda.synchronize()
    g, K = _backward(a, rs, out, info, dl)
    torch.cuda.synchronize()
    P = a["means3D"].shape[0]
    W, H = rs.image_width, rs.image_height
    dec = _C.decode_buffers(P, W, H, K, out[3], out[4], out[5], binning_layout=info["binning_layout"])
    return {"info": info, "K": K, "color": out[1], "depth": out[6], "radii": out[2], "g": g,
            "image": {k: dec[k].clone() for k in ("ranges", "n_contrib", "pix_end", "tile_maxc", "seg_off")}}


def _same(x, y):
    assert x["K"] == y["K"]
    for k in ("color", "depth", "radii"):
        assert torch.equal(x[k], y[k]), k
    for k, v in x["image"].items():
        assert torch.equal(v, y["image"][k]), k
    for p, q in zip(x["g"], y["g"]):
        assert (p is None and q is None) or torch.equal(p, q)


def _cloud(cuda, P=60_000):
    a = {k: v for k, v in S.activated_inputs(S.synthetic_cloud(P, 0.01, sh_degree=3, seed=21, device=cuda), 3).items()
         if k != "means2D" and v is not None}
    a.pop("colors_precomp", None)
    return a


def test_async_forward_stands_and_is_redone_bitwise(cuda):
    P, W, H = 60_000, 640, 480
    a = _cloud(cuda, P)
    dense = dict(a, scales=a["scales"] * 4.0)  # K 111873 -> 256884 (CPU oracle): past the capacity
    cam = S.render_settings(W, H, S.intrinsics(500.0, W, H), S.look_at(30, 0.2, 9.0), device=cuda, sh_degree=3)
    dl = S.upstream_grad(H, W, device=cuda)
    _C.speculation_stats(reset=True)
    exact_far = _run(a, cam, "exact", dl)
    exact_near = _run(dense, cam, "exact", dl)
    _C.speculation_stats(reset=True)
    _run(a, cam, "exact", dl)                      # history: the sparse cloud
    info, out = _forward(a, cam, "async")
    assert out[0] == -1 and info["pending"] is not None and info["speculated"]
    del info, out
    stood = _run(a, cam, "async", dl)              # within the capacity: the queued kernels stand
    assert stood["info"]["pending"].redone is False
    _same(stood, exact_far)
    redone = _run(dense, cam, "async", dl)         # capacity exceeded: the resolver redoes it
    assert redone["info"]["pending"].redone is True
    _same(redone, exact_near)
    _C.speculation_stats(reset=True)
    _run(a, cam, "exact", dl)
    held = _run(dense, cam, "async", dl, sync_first=True)  # device sync before any resolve call
    assert held["info"]["pending"].redone is True
    _same(held, exact_near)


def test_async_redo_on_many_streams(cuda):
    """Failed speculations on 8 caller streams (more streams than the process's hardware queues, so
    they share queues): a redo must never queue behind the waiting forward's held queue -- the
    resolver's stream has a hardware queue of its own.  Every forward completes with the exact image
    (a stuck redo would trip the 5 s gate timeout and report an error)."""
    P, W, H = 60_000, 640, 480
    a = _cloud(cuda, P)
    dense = dict(a, scales=a["scales"] * 4.0)  # K 111873 -> 256884: past the capacity
    cam = S.render_settings(W, H, S.intrinsics(500.0, W, H), S.look_at(30, 0.2, 9.0), device=cuda, sh_degree=3)
    ref = _forward(dense, cam, "exact")[1][1].clone()
    streams = [torch.cuda.Stream() for _ in range(8)]
    for k, st in enumerate(streams):
        _C.speculation_stats(reset=True)
        _forward(a, cam, "exact")  # sparse history: the dense forward below exceeds its capacity
        torch.cuda.synchronize()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            info, out = _forward(dense, cam, "async")
            busy = [torch.randn(1 << 20, device=cuda) * 2.0 for _ in range(4)]  # queued behind the forward
        torch.cuda.synchronize()
        assert info["pending"].resolve()[0] > 0 and info["pending"].redone, k
        assert torch.equal(out[1], ref), k
        del busy


def test_async_forward_redo_with_long_lists(cuda):
    """A failed speculation whose tiles need the host-sized merge sort (> 4096 pairs): the resolver's
    redo runs the chunk sorts + merge passes with their temporary buffer."""
    g = torch.Generator().manual_seed(4)
    P = 12_000
    m = torch.zeros(P, 3)
    m[:, 0] = torch.rand(P, generator=g) * 0.02 - 0.01
    m[:, 1] = torch.rand(P, generator=g) * 0.02 - 0.01
    m[:, 2] = torch.rand(P, generator=g) * 2 - 1
    a = {"means3D": m, "colors_precomp": torch.rand(P, 3, generator=g), "opacities": torch.full((P, 1), 0.05),
         "scales": torch.full((P, 3), 0.004), "rotations": torch.tensor([[1.0, 0, 0, 0]]).repeat(P, 1)}
    a = {k: v.to(cuda) for k, v in a.items()}
    rs = S.render_settings(64, 64, S.intrinsics(64.0, 64, 64), S.look_at(0, 0, 4), device=cuda)
    dl = S.upstream_grad(64, 64, device=cuda)
    exact = _run(a, rs, "exact", dl)
    spread = dict(a, means3D=a["means3D"] * torch.tensor([300.0, 300.0, 1.0], device=cuda))
    _C.speculation_stats(reset=True)
    _run(spread, rs, "exact", dl)
    got = _run(a, rs, "async", dl)
    assert got["info"]["pending"].redone is True
    _same(got, exact)
    nxt = _run(a, rs, "async", dl)  # long lists in the history: no capacity, the blocking exact path
    assert nxt["info"]["pending"] is None
    _same(nxt, exact)


def test_async_forwards_released_unresolved(cuda):
    """No-grad forwards queued back to back and dropped without a resolve (inference, train.py:778):
    every image is the exact one, and the library drops every record once it resolved."""
    P, W, H = 40_000, 320, 240
    a = _cloud(cuda, P)
    cam = S.render_settings(W, H, S.intrinsics(260.0, W, H), S.look_at(10, 0.1, 9.0), device=cuda, sh_degree=3)
    dense = dict(a, scales=a["scales"] * 3.0)
    ref = [_forward(x, cam, "exact")[1][1].clone() for x in (a, dense)]
    _C.speculation_stats(reset=True)
    _forward(a, cam, "exact")
    imgs = []
    for k in range(40):  # the first dense one exceeds the capacity the sparse history gives (redone)
        x = dense if k % 8 == 5 else a
        info, out = _forward(x, cam, "async")
        imgs.append((k % 8 == 5, out[1]))
        del info, out
    torch.cuda.synchronize()
    for dense_k, img in imgs:
        assert torch.equal(img, ref[1] if dense_k else ref[0])
    gc.collect()
    t0 = time.time()
    while _C.async_stats()[1] and time.time() - t0 < 5:
        time.sleep(0.01)
    assert _C.async_stats()[1] == 0


@pytest.mark.parametrize("leaf", [True, False])
def test_autograd_step_async_equals_blocking(cuda, leaf):
    """The drop-in module's summed multi-view step (train.py:402-418): leaf inputs (deferred multi-view
    pass, render halves held back while a forward is unresolved) and the reference's non-leaf
    create_render_arguments inputs (immediate per-view backward) -- images and gradients bitwise those
    of the blocking forward."""
    P, W, H = 80_000, 480, 320
    base = S.synthetic_cloud(P, 0.01, seed=5, device=cuda)
    cams = [S.render_settings(W, H, S.intrinsics(400.0, W, H), S.look_at(yaw, 0.2, 8.0), device=cuda)
            for yaw in (0, 40, 80, 120, 160)]
    dl = S.upstream_grad(H, W, device=cuda)

    def step():
        params = {k: torch.nn.Parameter(v.clone()) for k, v in base.items()}
        if leaf:
            with torch.no_grad():
                act = S.activated_inputs(params, -1)
            leaves = {k: v.detach().clone().requires_grad_(True) for k, v in act.items()}
        imgs = []
        for rs in cams:
            args = dict(leaves, means2D=torch.zeros_like(leaves["means3D"], requires_grad=True)) if leaf \
                else S.render_arguments(params)
            imgs.append(GaussianRasterizer(raster_settings=rs)(**args)[0])
        torch.stack([(i * dl).sum() for i in imgs]).sum().backward()
        torch.cuda.synchronize()
        src = leaves if leaf else params
        return [i.detach() for i in imgs], {k: v.grad for k, v in src.items() if v.grad is not None}

    prev = dgr.set_async_forward(False)
    try:
        step()  # history for every view's key
        ref = step()
        dgr.set_async_forward(True)
        got = step()
        assert _C.async_stats()[0] > 0
    finally:
        dgr.set_async_forward(prev)
    for x, y in zip(ref[0], got[0]):
        assert torch.equal(x, y)
    assert ref[1].keys() == got[1].keys()
    for k in ref[1]:
        assert torch.equal(ref[1][k], got[1][k]), k


@pytest.mark.parametrize("miss", [False, True])
def test_speculative_render_half_bitwise(cuda, miss):
    """Deferred views whose asynchronous forward is still unresolved when the backward reaches them
    (the GPU is held busy ahead of the forwards) queue their render half at once against the forward's
    capacity (ABI 19).  When the speculation stands the half is final; when the forward is redone
    (``miss``: a denser cloud than the pair-count history, so the capacity is exceeded) its kernels
    return at once and the end-of-pass callback redoes it.  Images and gradients are bitwise those of
    blocking forwards either way."""
    P, W, H = 80_000, 480, 320
    base = S.synthetic_cloud(P, 0.01, seed=7, device=cuda)
    cams = [S.render_settings(W, H, S.intrinsics(400.0, W, H), S.look_at(yaw, 0.2, 8.0), device=cuda)
            for yaw in (0, 72, 144, 216, 288)]
    dl = S.upstream_grad(H, W, device=cuda)
    with torch.no_grad():
        act = S.activated_inputs(base, -1)

    def step(scale, busy):
        leaves = {k: v.detach().clone().requires_grad_(True) for k, v in act.items()}
        with torch.no_grad():
            leaves["scales"].mul_(scale)
        if busy:  # the forwards queue behind ~20 ms of device work: none is resolved at the backward
            torch.cuda._sleep(50_000_000)
        imgs = [GaussianRasterizer(raster_settings=rs)(**dict(leaves, means2D=torch.zeros_like(
            leaves["means3D"], requires_grad=True)))[0] for rs in cams]
        torch.stack([(i * dl).sum() for i in imgs]).sum().backward()
        torch.cuda.synchronize()
        return [i.detach() for i in imgs], {k: v.grad for k, v in leaves.items() if v.grad is not None}

    scale = 3.0 if miss else 1.0
    prev_async, prev_half = dgr.set_async_forward(False), dgr._defer["spec_half"]
    try:
        dgr._defer["spec_half"] = True
        ref = step(scale, False)
        _C.speculation_stats(reset=True)
        step(1.0, False)  # pair-count history of the sparse cloud for every view's key
        dgr.set_async_forward(True)
        q0, r0 = dgr._spec_half_stats["queued"], dgr._spec_half_stats["redone"]
        got = step(scale, True)
        queued, redone = dgr._spec_half_stats["queued"] - q0, dgr._spec_half_stats["redone"] - r0
    finally:
        dgr.set_async_forward(prev_async)
        dgr._defer["spec_half"] = prev_half
    assert queued > 0
    assert (redone > 0) == miss, (queued, redone)
    for x, y in zip(ref[0], got[0]):
        assert torch.equal(x, y)
    assert ref[1].keys() == got[1].keys()
    for k in ref[1]:
        assert torch.equal(ref[1][k], got[1][k]), k


def test_external_stream_of_handle_zero_is_the_default_stream(cuda):
    """The deferred backward's stream lookup: raw handle 0 must give torch's default stream (the same
    queue as the forward), a real handle the stream it names (round 6)."""
    assert _C._external_stream(0, cuda) == torch.cuda.default_stream(cuda)
    s = torch.cuda.Stream(device=cuda)
    e = _C._external_stream(s.cuda_stream, cuda)
    assert e.cuda_stream == s.cuda_stream


@pytest.mark.parametrize("half", [False, True])
def test_held_back_render_half_on_default_stream(cuda, half):
    """A deferred view whose asynchronous forward is unresolved at its backward node, on the DEFAULT
    stream: its render half is queued by the end-of-pass callback (held back, or redone after a missed
    speculation) on the view's stream, handle 0.  torch.cuda.ExternalStream(0) is a separate queue on
    ROCm (round 6: those halves raced the forward and the per-Gaussian pass -- NaN or wrong gradients in
    ~every held-back step, tools/spec_half_repro.py); the view's stream must be the default stream
    itself.  One view, a denser cloud than the pair-count history, the GPU held busy: bitwise equal to
    blocking forwards, three times over (the allocator's reuse made the race show from the second)."""
    P, W, H = 80_000, 480, 320
    base = S.synthetic_cloud(P, 0.01, seed=7, device=cuda)
    rs = S.render_settings(W, H, S.intrinsics(400.0, W, H), S.look_at(0, 0.2, 8.0), device=cuda)
    dl = S.upstream_grad(H, W, device=cuda)
    with torch.no_grad():
        act = S.activated_inputs(base, -1)

    def step(scale, busy):
        leaves = {k: v.detach().clone().requires_grad_(True) for k, v in act.items()}
        with torch.no_grad():
            leaves["scales"].mul_(scale)
        if busy:
            torch.cuda._sleep(50_000_000)
        img = GaussianRasterizer(raster_settings=rs)(**dict(leaves, means2D=torch.zeros_like(
            leaves["means3D"], requires_grad=True)))[0]
        (img * dl).sum().backward()
        torch.cuda.synchronize()
        return img.detach(), {k: v.grad for k, v in leaves.items() if v.grad is not None}

    assert torch.cuda.current_stream().cuda_stream == 0
    prev_async, prev_half = dgr.set_async_forward(False), dgr._defer["spec_half"]
    try:
        dgr._defer["spec_half"] = half
        ref = step(3.0, False)
        for _ in range(3):
            dgr.set_async_forward(False)
            _C.speculation_stats(reset=True)
            step(1.0, False)  # pair-count history of the sparse cloud: the capacity stands, K unknown
            dgr.set_async_forward(True)
            got = step(3.0, True)
            assert torch.equal(ref[0], got[0])
            assert ref[1].keys() == got[1].keys()
            for k in ref[1]:
                assert torch.equal(ref[1][k], got[1][k]), k
    finally:
        dgr.set_async_forward(prev_async)
        dgr._defer["spec_half"] = prev_half


@pytest.mark.parametrize("shape", ["call", "autograd"])
def test_gate_timeout_fails_that_steps_backward(cuda, shape):
    """A failed speculation whose redo the resolver holds back longer than the gate's timeout (test hook
    gsr_debug_async_fault: 300 ms hold, 20 ms timeout): the speculative render abandons the gate, the
    work queued after the forward runs on outputs that are not final -- and that SAME step must fail:
    the forward's resolution (at the step's backward) raises.  Afterwards the library recovers (no
    sticky error): the next asynchronous step equals the blocking one bitwise."""
    P, W, H = 60_000, 640, 480
    a = _cloud(cuda, P)
    dense = dict(a, scales=a["scales"] * 4.0)  # past the sparse cloud's capacity (see above)
    cam = S.render_settings(W, H, S.intrinsics(500.0, W, H), S.look_at(30, 0.2, 9.0), device=cuda, sh_degree=3)
    dl = S.upstream_grad(H, W, device=cuda)
    _C.speculation_stats(reset=True)
    _run(a, cam, "exact", dl)  # history: the sparse cloud
    _C.debug_async_fault(hold_next_redo_ms=300, gate_timeout_ms=20)
    try:
        if shape == "call":
            info, out = _forward(dense, cam, "async")
            torch.cuda.synchronize()  # the stream passes the abandoned gate (20 ms)
            with pytest.raises(RuntimeError, match="gate timed out"):
                _backward(dense, cam, out, info, dl)
            del info, out
        else:
            leaves = {k: v.detach().clone().requires_grad_(True) for k, v in dense.items()}
            with dgr.async_forward(True):
                img = GaussianRasterizer(raster_settings=cam)(
                    **dict(leaves, means2D=torch.zeros_like(leaves["means3D"], requires_grad=True)))[0]
            torch.cuda.synchronize()
            with pytest.raises(RuntimeError, match="gate timed out"):
                (img * dl).sum().backward()
            del img
    finally:
        _C.debug_async_fault(0, 0, clear=True)
    gc.collect()
    torch.cuda.synchronize()
    _C.speculation_stats(reset=True)
    _run(a, cam, "exact", dl)
    _same(_run(dense, cam, "async", dl), _run(dense, cam, "exact", dl))
