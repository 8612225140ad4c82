"""Fused device SSIM / L1 + 0.3·(1 − SSIM) loss (mx_ssim.hip; train_restoration.py:142-178 ssim() and
CombinedLoss) against the float64 evaluation of the reference formula (oracle/ssim_ref.py, torch CPU):
loss within 1e-5 (absolute; the loss is O(0.1-1)) and the gradient w.r.t. the prediction within 1e-5
relative (norm) on 256x256x8 patches -- the bar the kernels are built for (f64 window sums); plus odd
sizes smaller than the window, other window sizes, the mean-SSIM entry, channels-last inputs (the HIP
U-Net's output layout) and determinism."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _pair(shape, seed, noise=0.08):
    g = torch.Generator().manual_seed(seed)
    clean = torch.rand(shape, generator=g, dtype=torch.float64)
    # smooth + flat regions too: the variance terms cancel there
    clean[..., : shape[2] // 3, :] = 0.5
    pred = (clean + noise * torch.randn(shape, generator=g, dtype=torch.float64)).clamp(0, 1)
    return pred, clean


def _ref(pred64, clean64, weight, window=11, combined=True):
    from oracle import ssim_ref
    p = pred64.clone().requires_grad_(True)
    loss = ssim_ref.combined_loss(p, clean64, weight) if combined else ssim_ref.ssim(p, clean64, window)
    loss.backward()
    return float(loss), p.grad


@pytest.mark.parametrize("shape,window", [((8, 3, 256, 256), 11), ((2, 3, 37, 53), 11), ((1, 3, 7, 9), 11),
                                          ((2, 1, 64, 70), 7)])
def test_ssim_l1_loss_and_gradient_vs_f64(dev, shape, window):
    from mx_det import ops
    p64, c64 = _pair(shape, 3)
    pred = p64.float().to(dev).requires_grad_(True)
    clean = c64.float().to(dev)
    # the f32 inputs themselves differ from the f64 ones by <= 2^-25; evaluate the reference at them
    if window == 11:
        lr, gr = _ref(pred.detach().cpu().double(), clean.cpu().double(), 0.3)
        loss = ops.ssim_l1_loss(pred, clean, 0.3)
    else:
        lr, gr = _ref(pred.detach().cpu().double(), clean.cpu().double(), 0.0, window, combined=False)
        loss = ops.ssim(pred, clean, window)
    loss.backward()
    assert abs(float(loss) - lr) <= 1e-5, (float(loss), lr)
    e = ((pred.grad.double().cpu() - gr).norm() / gr.norm()).item()
    assert e <= 1e-5, e


def test_channels_last_and_restoration_entry_points(dev):
    from mx_det import ops
    from mx_det.restoration import CombinedLoss, compute_psnr, ssim
    p64, c64 = _pair((4, 3, 48, 40), 5)
    a = p64.float().to(dev)
    b = c64.float().to(dev)
    cl = a.contiguous(memory_format=torch.channels_last)
    assert float(ops.ssim(cl, b)) == float(ops.ssim(a, b))
    from oracle import ssim_ref
    assert abs(float(ssim(a, b)) - float(ssim_ref.ssim(a.cpu().double(), b.cpu().double()))) < 1e-6
    x = cl.clone().requires_grad_(True)
    y = a.clone().requires_grad_(True)
    CombinedLoss(0.3)(x, b).backward()
    CombinedLoss(0.3)(y, b).backward()
    assert torch.equal(x.grad.contiguous(), y.grad.contiguous())
    mse = float(((a.double() - b.double()) ** 2).mean())
    import math
    assert abs(compute_psnr(a, b) - 10 * math.log10(1 / mse)) < 1e-4
    assert compute_psnr(b, b) == 100.0


def test_deterministic_and_rejects_target_grad(dev):
    from mx_det import ops
    p64, c64 = _pair((8, 3, 96, 96), 9)
    a, b = p64.float().to(dev), c64.float().to(dev)
    r = [float(ops.ssim_l1_loss(a, b)) for _ in range(3)]
    assert r[0] == r[1] == r[2]
    with pytest.raises(RuntimeError):
        ops.ssim(a, b.clone().requires_grad_(True))
    with pytest.raises(RuntimeError):
        ops.ssim(a, b, window_size=10)
