"""Fused Adam against the reference's own optimizer, torch.optim.Adam.

The reference optimises the Gaussians with torch.optim.Adam (densify.py:68-86: one named group per
parameter, lr = 0.0 default, eps = 1e-15), which IS the parity target here: the GPU tests run both on
identical parameters / gradients for several steps, including a group with lr = 0 (segmentation
masks), groups without gradients (camera_*), sizes that are not multiples of 4, a learning-rate
change between steps, and densification surgery in between.  Parameters, both moments and step
counts must be BITWISE equal: the kernel reproduces _multi_tensor_adam's operation order and its
compiler's FMA contractions (lerp, addcmul, addcdiv), verified with tools/adam_probe.py.
"""
import numpy as np
import pytest
import torch

LR = {"means": 0.00016 * 3.0, "colors": 0.0025, "segmentation_masks": 0.0, "rotation_quaternions": 0.001,
      "opacity_logits": 0.05, "log_scales": 0.001, "camera_matrices": 1e-4, "camera_center": 1e-4}
WIDTH = {"means": 3, "colors": 3, "segmentation_masks": 3, "rotation_quaternions": 4, "opacity_logits": 1,
         "log_scales": 3}


def _params(P, dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    p = {k: torch.randn(P, w, generator=g) for k, w in WIDTH.items()}
    p["camera_matrices"] = torch.zeros(50, 3)
    p["camera_center"] = torch.zeros(50, 3)
    return {k: torch.nn.Parameter(v.to(dev)) for k, v in p.items()}


def _opt(cls, params):
    return cls([{"params": [v], "name": k, "lr": LR[k]} for k, v in params.items()], lr=0.0, eps=1e-15)


def _close(a, b, what):
    """Bitwise equal: the fused kernel follows torch's foreach operation order and contractions."""
    np.testing.assert_array_equal(a.detach().cpu().numpy(), b.detach().cpu().numpy(), err_msg=what)


def test_fused_adam_refuses_cpu_and_unsupported():
    import splat_adam
    with pytest.raises(NotImplementedError):
        splat_adam.FusedAdam([torch.nn.Parameter(torch.zeros(3))], weight_decay=0.1)
    p = torch.nn.Parameter(torch.zeros(3))
    opt = splat_adam.FusedAdam([p])
    p.grad = torch.ones(3)
    with pytest.raises(RuntimeError, match="no CPU path"):
        opt.step()


@pytest.mark.gpu
@pytest.mark.parametrize("P", [1, 1001, 65536 + 3])
def test_gpu_fused_adam_matches_torch_adam(cuda, P):
    import splat_adam
    pa, pb = _params(P, cuda), _params(P, cuda)
    oa, ob = _opt(torch.optim.Adam, pa), _opt(splat_adam.FusedAdam, pb)
    g = torch.Generator().manual_seed(1)
    for it in range(6):
        if it == 3:  # a scheduler-style lr change
            for o in (oa, ob):
                for grp in o.param_groups:
                    grp["lr"] *= 0.5
        for k in WIDTH:
            gr = (0.01 * torch.randn(pa[k].shape, generator=g)).to(cuda)
            pa[k].grad, pb[k].grad = gr.clone(), gr.clone()
        oa.step()
        ob.step()
    torch.cuda.synchronize()
    for k in pa:
        _close(pb[k], pa[k], k)
        if k in WIDTH:
            sa, sb = oa.state[pa[k]], ob.state[pb[k]]
            assert float(sa["step"]) == float(sb["step"]) == 6.0
            _close(sb["exp_avg"], sa["exp_avg"], k + ".exp_avg")
            _close(sb["exp_avg_sq"], sa["exp_avg_sq"], k + ".exp_avg_sq")
        else:
            assert len(ob.state[pb[k]]) == 0  # never had a gradient: no state, like torch
    np.testing.assert_array_equal(pb["segmentation_masks"].detach().cpu().numpy(),
                                  _params(P, "cpu")["segmentation_masks"].detach().numpy())  # lr = 0


@pytest.mark.gpu
def test_gpu_fused_adam_through_densification(cuda):
    """Adam state surgery by splat_densify works on FusedAdam exactly as on torch.optim.Adam."""
    import splat_adam
    import splat_densify
    P = 5000
    runs = []
    for cls in (torch.optim.Adam, splat_adam.FusedAdam):
        params = _params(P, cuda, seed=3)
        with torch.no_grad():
            params["log_scales"].mul_(0.5).add_(float(np.log(0.03)))
        opt = _opt(cls, params)
        g = torch.Generator().manual_seed(4)
        for k in WIDTH:
            params[k].grad = (0.01 * torch.randn(params[k].shape, generator=g)).to(cuda)
        opt.step()
        dv = splat_densify.DensificationVariables(
            visibility_count=torch.full((P,), 2.0, device=cuda),
            mean_2d_gradients_accumulated=(8e-4 * torch.rand(P, generator=g)).to(cuda),
            max_2d_radii=torch.zeros(P, device=cuda),
            gaussian_is_visible_mask=torch.zeros(P, dtype=torch.bool, device=cuda),
            means_2d=torch.zeros(P, 3, device=cuda, requires_grad=True))
        dv.means_2d.grad = torch.zeros(P, 3, device=cuda)
        torch.manual_seed(9)
        info = splat_densify.densify_gaussians(params, dv, 3.0, opt, 1000)
        for k in WIDTH:
            params[k].grad = (0.01 * torch.randn(params[k].shape, generator=g)).to(cuda)
        opt.step()
        runs.append((params, opt, info))
    (pa, oa, ia), (pb, ob, ib) = runs
    assert ia == ib and ia["n_split"] > 0 and ia["n_keep_clone"] > 0
    for k in WIDTH:
        _close(pb[k], pa[k], k)
        _close(ob.state[pb[k]]["exp_avg"], oa.state[pa[k]]["exp_avg"], k)
        assert float(ob.state[pb[k]]["step"]) == float(oa.state[pa[k]]["step"]) == 2.0
