"""Fused L1 + SSIM loss: oracle pinned to the reference, HIP kernels vs oracle.

CPU: the float64 oracle (oracle/ssim_oracle.py) reproduces the reference's own calc_ssim values and
autograd gradients (tests/golden, produced by importing external.py) and torch.autograd of a
float64 restatement.  GPU (-m gpu): splat_loss through the C ABI of libgsr.so against the oracle on
the golden inputs, ragged / tiny / batched shapes and a 1080p render-sized pair.  Tolerances: the
scalar means within 1e-5 relative (fp32 separable blur + double block sums vs float64), gradients
within 1e-4 relative + 1e-6 of the largest magnitude.
"""
import os

import numpy as np
import pytest
import torch

from oracle import ssim_oracle as SO

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "reference_harness.npz"))


def _grad_close(got, ref, rtol=1e-4, atol_frac=1e-6):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    tol = rtol * np.abs(ref) + atol_frac * np.abs(ref).max()
    bad = np.abs(got - ref) > tol
    assert not bad.any(), f"{bad.sum()} of {bad.size} gradient values off, worst {np.abs(got - ref).max():.3e}"


def test_oracle_window_matches_reference_definition():
    w = SO.window_1d()
    assert w.dtype == np.float32 and w.shape == (11,)
    assert abs(float(w.sum()) - 1.0) < 1e-6 and np.all(w == w[::-1])


def test_oracle_matches_reference_ssim_value_and_grad():
    a, b = GOLD["ssim_in_img1"], GOLD["ssim_in_img2"]
    _, ssim, st = SO.l1_ssim(a, b)
    assert abs(ssim - float(GOLD["ssim_out"])) < 2e-6
    _grad_close(SO.l1_ssim_grad(st, 0.0, 1.0), GOLD["ssim_out_grad"], rtol=2e-4, atol_frac=2e-5)


def test_oracle_matches_reference_combined_loss():
    """0.8 l1 + 0.2 (1 - ssim) of densify.py:149-151 on a ragged binary-target pair."""
    a, b = GOLD["loss_in_img1"], GOLD["loss_in_img2"]
    l1, ssim, st = SO.l1_ssim(a, b)
    assert abs(l1 - float(GOLD["loss_out_l1"])) < 2e-6
    assert abs(ssim - float(GOLD["loss_out_ssim"])) < 2e-6
    _grad_close(SO.l1_ssim_grad(st, 0.8, -0.2), GOLD["loss_out_grad"], rtol=2e-4, atol_frac=2e-5)


def test_oracle_grad_matches_torch_autograd_float64():
    g = torch.Generator().manual_seed(3)
    a = torch.rand(2, 3, 19, 23, generator=g, dtype=torch.float64)
    b = torch.rand(2, 3, 19, 23, generator=g, dtype=torch.float64)
    x = a.clone().requires_grad_(True)
    w = torch.from_numpy(SO.window_1d().astype(np.float64))
    w2 = torch.outer(w, w)[None, None].expand(6, 1, 11, 11)

    def blur(t):
        return torch.nn.functional.conv2d(t.reshape(1, 6, 19, 23), w2, padding=5, groups=6).reshape(t.shape)

    mu1, mu2 = blur(x), blur(b)
    s = ((2 * mu1 * mu2 + SO.C1) * (2 * (blur(x * b) - mu1 * mu2) + SO.C2)) / (
        (mu1 ** 2 + mu2 ** 2 + SO.C1) * ((blur(x * x) - mu1 ** 2) + (blur(b * b) - mu2 ** 2) + SO.C2))
    loss = 0.3 * (x - b).abs().mean() + 0.7 * s.mean()
    loss.backward()
    l1, ssim, st = SO.l1_ssim(a.numpy(), b.numpy())
    assert abs(0.3 * l1 + 0.7 * ssim - loss.detach().item()) < 1e-12
    np.testing.assert_allclose(SO.l1_ssim_grad(st, 0.3, 0.7), x.grad.numpy(), rtol=1e-9, atol=1e-14)


# ------------------------------------------------------------------------------------------------
def _gpu_case(cuda, a, b, g_l1=0.8, g_ssim=-0.2):
    import splat_loss
    x = torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(cuda).requires_grad_(True)
    y = torch.from_numpy(np.ascontiguousarray(b, np.float32)).to(cuda)
    l1, ssim = splat_loss.l1_and_ssim(x, y)
    (g_l1 * l1 + g_ssim * ssim).backward()
    torch.cuda.synchronize()
    rl1, rssim, st = SO.l1_ssim(a.astype(np.float32), b.astype(np.float32))
    assert abs(float(l1) - rl1) <= 1e-5 * abs(rl1) + 1e-7, (float(l1), rl1)
    assert abs(float(ssim) - rssim) <= 1e-5 * abs(rssim) + 1e-7, (float(ssim), rssim)
    ref = SO.l1_ssim_grad(st, g_l1, g_ssim)
    # |x - y| == 0 exactly is where sign() is 0 in both; elsewhere the sign terms agree bitwise
    _grad_close(x.grad.cpu().numpy(), ref)


@pytest.mark.gpu
def test_gpu_loss_matches_reference_goldens(cuda):
    import splat_loss
    x = torch.from_numpy(GOLD["ssim_in_img1"]).to(cuda).requires_grad_(True)
    y = torch.from_numpy(GOLD["ssim_in_img2"]).to(cuda)
    s = splat_loss.calc_ssim(x, y)
    s.backward()
    assert abs(s.detach().item() - float(GOLD["ssim_out"])) < 2e-6
    _grad_close(x.grad.cpu().numpy(), GOLD["ssim_out_grad"], rtol=2e-4, atol_frac=2e-5)
    x = torch.from_numpy(GOLD["loss_in_img1"]).to(cuda).requires_grad_(True)
    y = torch.from_numpy(GOLD["loss_in_img2"]).to(cuda)
    loss = splat_loss.image_loss(x, y)
    loss.backward()
    ref = 0.8 * float(GOLD["loss_out_l1"]) + 0.2 * (1 - float(GOLD["loss_out_ssim"]))
    assert abs(loss.detach().item() - ref) < 2e-6
    _grad_close(x.grad.cpu().numpy(), GOLD["loss_out_grad"], rtol=2e-4, atol_frac=2e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(3, 1, 1), (3, 5, 7), (1, 33, 65), (3, 64, 32), (3, 37, 130),
                                   (2, 3, 40, 70), (3, 100, 200)])
def test_gpu_loss_parity_shapes(cuda, shape):
    rng = np.random.default_rng(sum(shape))
    a = rng.random(shape, dtype=np.float32)
    b = np.clip(a + 0.2 * rng.standard_normal(shape).astype(np.float32), 0, 1)
    _gpu_case(cuda, a, b)


@pytest.mark.gpu
def test_gpu_loss_parity_1080p(cuda):
    rng = np.random.default_rng(7)
    a = rng.random((3, 1080, 1920), dtype=np.float32)
    b = (rng.random((3, 1080, 1920)) > 0.5).astype(np.float32)
    _gpu_case(cuda, a, b, 1.0, 1.0)


@pytest.mark.gpu
def test_gpu_loss_single_output_grads(cuda):
    """Only one of the two outputs used: the other upstream gradient is absent (NULL in the ABI)."""
    import splat_loss
    rng = np.random.default_rng(11)
    a, b = rng.random((3, 30, 40), dtype=np.float32), rng.random((3, 30, 40), dtype=np.float32)
    _, _, st = SO.l1_ssim(a, b)
    for which, (gl, gs) in (("ssim", (0.0, 1.0)), ("l1", (1.0, 0.0))):
        x = torch.from_numpy(a).to(cuda).requires_grad_(True)
        l1, ssim = splat_loss.l1_and_ssim(x, torch.from_numpy(b).to(cuda))
        (ssim if which == "ssim" else l1).backward()
        _grad_close(x.grad.cpu().numpy(), SO.l1_ssim_grad(st, gl, gs))


@pytest.mark.gpu
def test_gpu_loss_errors(cuda):
    import splat_loss
    x = torch.rand(3, 8, 8, device=cuda)
    with pytest.raises(NotImplementedError):
        splat_loss.l1_and_ssim(x, x.clone().requires_grad_(True))
    with pytest.raises(RuntimeError, match="shapes differ"):
        splat_loss.l1_and_ssim(x, torch.rand(3, 8, 9, device=cuda))
    with pytest.raises(NotImplementedError):
        splat_loss.calc_ssim(x, x, window_size=7)


def test_loss_refuses_cpu_tensors():
    import splat_loss
    with pytest.raises(RuntimeError, match="no CPU path"):
        splat_loss.l1_and_ssim(torch.rand(3, 8, 8), torch.rand(3, 8, 8))
