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
