"""TEST INFRASTRUCTURE ONLY (oracle): CPU restatement of the reference's restoration loss
(scripts/train_restoration.py:135-178 -- Gaussian window, ssim(), CombinedLoss) on torch CPU, in any
dtype (float64 is the parity anchor for the fused HIP kernels of mx_ssim.hip). Only tests/ import this.

The statistic: per pixel, Gaussian-weighted window means (11 x 11, σ 1.5, 2-D weights normalised to
sum 1, zero padding so every pixel has a window) of x, y, x², y², xy; variances/covariance as
E[ab] − E[a]E[b]; SSIM = (2μxμy + C1)(2σxy + C2) / ((μx² + μy² + C1)(σx² + σy² + C2)) with
C1 = 0.01², C2 = 0.03²; the loss is mean|x − y| + w·(1 − mean SSIM)."""
import torch
import torch.nn.functional as F


def window_2d(size=11, sigma=1.5, dtype=torch.float32):
    """The reference builds the 1-D profile (exp of −d²/2σ²), takes its outer product and divides by
    the total (train_restoration.py:135-139) -- in float32 there; here in `dtype` throughout, so the
    float64 evaluation is the formula's exact reading."""
    d = torch.arange(size, dtype=dtype) - size // 2
    prof = torch.exp(-(d * d) / (2 * sigma * sigma))
    w = prof[:, None] * prof[None, :]
    return w / w.sum()


def _wmean(t, w):
    c = t.shape[1]
    return F.conv2d(t, w.expand(c, 1, *w.shape).contiguous(), padding=w.shape[-1] // 2, groups=c)


def ssim(pred, target, window_size=11):
    w = window_2d(window_size, dtype=pred.dtype)
    mx, my = _wmean(pred, w), _wmean(target, w)
    vx = _wmean(pred * pred, w) - mx * mx
    vy = _wmean(target * target, w) - my * my
    cxy = _wmean(pred * target, w) - mx * my
    c1, c2 = 0.01 ** 2, 0.03 ** 2
    num = (2 * mx * my + c1) * (2 * cxy + c2)
    den = (mx * mx + my * my + c1) * (vx + vy + c2)
    return (num / den).mean()


def combined_loss(pred, target, ssim_weight=0.3):
    return (pred - target).abs().mean() + ssim_weight * (1 - ssim(pred, target))
