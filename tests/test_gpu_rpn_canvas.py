"""RPNHead small levels as one zero-framed canvas conv chain (frcnn.RPNHead.forward) on the HIP
backend: equal to the per-level chains (torchvision's loop) in f32 (bf16x3 convs) for outputs, feature
gradients and the shared weights' gradients. Tolerances: outputs within 1e-5 of the tensor norm and
1e-4 of its largest element (a different split-K choice for the canvas shape changes the f32
summation order of an output element through two chained convs); feature gradients 1e-4 of the norm
(a ReLU derivative flips where a pre-activation sits at ~0 in one order and not the other); weight gradients
1e-4 relative (the canvas wgrad sums the five levels' pixels in one pass instead of accumulating
per-level gradients)."""
import pytest
import torch

from test_model_cpu import _rpn_head_run


@pytest.mark.gpu
@pytest.mark.parametrize("hw0", [(200, 336), (96, 168)])
def test_rpn_head_canvas_equals_per_level_hip(dev, hw0, monkeypatch):
    from mx_det.backend import HipBackend
    H, W = hw0
    hw = [(H, W)]
    for _ in range(4):
        H, W = (H + 1) // 2, (W + 1) // 2
        hw.append((H, W))
    torch.manual_seed(2)
    feats = [torch.randn(2, h, w, 256, device=dev) for h, w in hw]
    be = HipBackend("f32")
    a = _rpn_head_run(be, feats, True, monkeypatch)
    b = _rpn_head_run(be, feats, False, monkeypatch)
    for x, y in zip(a[0], b[0]):  # logits / deltas
        assert x.shape == y.shape
        assert (x - y).norm() <= 1e-5 * y.norm()
        assert (x - y).abs().max() <= 1e-4 * y.abs().max()
    for x, y in zip(a[1], b[1]):  # feature gradients: a ReLU mask bit may flip where a pre-activation ~ 0
        assert x.shape == y.shape
        assert (x - y).norm() <= 1e-4 * y.norm()
    for k in a[2]:
        g1, g2 = a[2][k], b[2][k]
        assert (g1 - g2).norm() <= 1e-4 * g2.norm(), k


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_mask_pixels_matches_broadcast_multiply(dev, dtype):
    """mx_mask_pixels = t * mask[None, :, :, None] bit for bit (NaN, inf and -0 included), its backward
    g * mask, and (f32) the planes it writes equal split_planes of the output."""
    from mx_det import ops
    g = torch.Generator().manual_seed(2)
    t = torch.randn(2, 19, 23, 64, generator=g)
    t[0, 0, 0, :3] = torch.tensor([float("nan"), float("inf"), -0.0])
    t[1, 5, 7, :2] = torch.tensor([float("-inf"), -3.0])
    mask = (torch.rand(1, 19, 23, 1, generator=g) < 0.7).float()
    mask[0, 0, 0, 0] = 0.0
    x = t.to(dev, dtype).requires_grad_(True)
    y = ops.mask_pixels(x, mask.reshape(-1).to(dev), planes_krs=1 if dtype == torch.float32 else 0)
    want = x.detach() * mask.to(dev, dtype)
    iv = torch.int16 if dtype == torch.bfloat16 else torch.int32
    nan = torch.isnan(want)
    assert torch.equal(torch.isnan(y.detach()), nan)  # NaN payloads may differ (bf16 rounding of a NaN)
    assert torch.equal(y.detach()[~nan].view(iv), want[~nan].view(iv))
    gy = torch.randn(y.shape, generator=g).to(dev, dtype)
    y.backward(gy)
    assert torch.equal(x.grad.view(iv), (gy * mask.to(dev, dtype)).view(iv))
    if dtype == torch.float32:
        pl = getattr(y, "_mx_planes", None)
        assert pl is None  # below MX_X3_PLANES_MIN: no planes for this small map


@pytest.mark.gpu
def test_mask_pixels_planes(dev, monkeypatch):
    from mx_det import conv as mc
    from mx_det import ops
    monkeypatch.setenv("MX_X3_PLANES_MIN", "0")
    x = torch.randn(2, 31, 37, 64, device=dev)
    mask = (torch.rand(31 * 37, device=dev) < 0.5).float()
    y = ops.mask_pixels(x, mask, planes_krs=4096)
    assert torch.equal(y._mx_planes.view(torch.int16), mc.split_planes(y).view(torch.int16))
