"""mx_det's torch.library operators (mx_det/torch_ops.py): torchvision's schemas, the fake (meta)
implementations, and -- on the GPU -- numerics through torch.ops against the oracle (torchvision's
CPU algorithm restated in oracle/), autograd through the registered _roi_align_backward, and
torch.library.opcheck."""
import numpy as np
import pytest
import torch

# torchvision 0.20.1 (the reference's pin) schemas, torchvision/csrc/ops/{nms,roi_align}.cpp
TV_SCHEMAS = {
    "nms": "nms(Tensor dets, Tensor scores, float iou_threshold) -> Tensor",
    "roi_align": ("roi_align(Tensor input, Tensor rois, float spatial_scale, SymInt pooled_height, "
                  "SymInt pooled_width, int sampling_ratio, bool aligned) -> Tensor"),
    "_roi_align_backward": ("_roi_align_backward(Tensor grad, Tensor rois, float spatial_scale, "
                            "SymInt pooled_height, SymInt pooled_width, SymInt batch_size, SymInt channels, "
                            "SymInt height, SymInt width, int sampling_ratio, bool aligned) -> Tensor"),
}


def _ops():
    from mx_det import torch_ops
    return torch_ops


def test_schemas_match_torchvision():
    _ops()
    for name, sch in TV_SCHEMAS.items():
        op = getattr(torch.ops.mx_det, name).default
        assert str(op._schema) == "mx_det::" + sch, (str(op._schema), sch)


def test_fake_shapes():
    _ops()
    from torch._subclasses.fake_tensor import FakeTensorMode
    from torch.fx.experimental.symbolic_shapes import ShapeEnv
    with FakeTensorMode(shape_env=ShapeEnv()):
        x = torch.empty(2, 64, 30, 40)
        r = torch.empty(17, 5)
        y = torch.ops.mx_det.roi_align(x, r, 0.25, 7, 7, 2, False)
        assert tuple(y.shape) == (17, 64, 7, 7)
        g = torch.ops.mx_det._roi_align_backward(y, r, 0.25, 7, 7, 2, 64, 30, 40, 2, False)
        assert tuple(g.shape) == (2, 64, 30, 40)
        k = torch.ops.mx_det.nms(torch.empty(9, 4), torch.empty(9), 0.5)
        assert k.dim() == 1 and k.dtype == torch.int64


def test_cpu_tensors_have_no_fallback():
    _ops()
    with pytest.raises(NotImplementedError):
        torch.ops.mx_det.nms(torch.zeros(3, 4), torch.zeros(3), 0.5)


def _boxes(rng, n, H, W, med):
    xy = rng.uniform(0, 1, (n, 2)) * [W, H]
    wh = np.exp(rng.normal(np.log(med), 0.6, (n, 2)))
    return np.concatenate([xy, xy + wh], 1).astype(np.float32)


@pytest.mark.gpu
def test_nms_matches_oracle(dev):
    from oracle import oracle as orc
    ops = _ops()
    rng = np.random.default_rng(21)
    b = _boxes(rng, 3000, 800, 1333, 40)
    s = rng.uniform(0, 1, 3000).astype(np.float32)
    got = ops.nms(torch.from_numpy(b).to(dev), torch.from_numpy(s).to(dev), 0.7).cpu().numpy()
    ref = orc.nms(b, s, 0.7)
    assert np.array_equal(got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("aligned", [False, True])
def test_roi_align_nchw_and_autograd_match_oracle(dev, aligned):
    from oracle import oracle as orc
    ops = _ops()
    rng = np.random.default_rng(22 + aligned)
    N, C, H, W, scale = 2, 64, 40, 52, 0.25
    feat = rng.standard_normal((N, C, H, W)).astype(np.float32)
    bx = _boxes(rng, 150, H / scale, W / scale, 30)
    bx[0] = [-20, -30, 40, 40]
    rois = np.concatenate([rng.integers(0, N, (150, 1)).astype(np.float32), bx], 1)
    x = torch.from_numpy(feat).to(dev).requires_grad_(True)
    r = torch.from_numpy(rois).to(dev)
    y = ops.roi_align(x, r, 7, scale, 2, aligned)
    assert y.shape == (150, C, 7, 7)
    assert np.array_equal(y.detach().cpu().numpy(), orc.roi_align(feat, rois, scale, (7, 7), 2, aligned))
    g = rng.standard_normal((150, C, 7, 7)).astype(np.float32)
    y.backward(torch.from_numpy(g).to(dev))
    ref = orc.roi_align_backward(g, rois, scale, (N, C, H, W), 2, aligned)
    assert np.array_equal(x.grad.cpu().numpy(), ref)  # deterministic gather: torchvision's CPU order
    gi = torch.ops.mx_det._roi_align_backward(torch.from_numpy(g).to(dev), r, scale, 7, 7, N, C, H, W, 2, aligned)
    assert torch.equal(gi, x.grad)


@pytest.mark.gpu
def test_opcheck(dev):
    ops = _ops()
    rng = np.random.default_rng(23)
    x = torch.from_numpy(rng.standard_normal((1, 32, 20, 24)).astype(np.float32)).to(dev).requires_grad_(True)
    bx = _boxes(rng, 12, 80, 96, 20)
    r = torch.from_numpy(np.concatenate([np.zeros((12, 1), np.float32), bx], 1)).to(dev)
    torch.library.opcheck(torch.ops.mx_det.roi_align.default, (x, r, 0.25, 7, 7, 2, False),
                          test_utils=("test_schema", "test_autograd_registration", "test_faketensor"))
    b = torch.from_numpy(_boxes(rng, 50, 100, 100, 20)).to(dev)
    s = torch.rand(50, device=dev)
    torch.library.opcheck(torch.ops.mx_det.nms.default, (b, s, 0.5), test_utils=("test_schema",))
    assert ops is not None


@pytest.mark.gpu
@pytest.mark.parametrize("aligned", [False, True])
def test_roi_align_adaptive_sampling_and_list_boxes(dev, aligned):
    """torchvision.ops.roi_align's defaults: sampling_ratio=-1 (per-RoI ceil(roi_h/ph) x ceil(roi_w/pw)
    grid) and boxes as a list of per-image Tensor[L, 4]. Forward bit-exact vs the oracle's adaptive
    grid; backward (atomics, as torchvision's CUDA kernel) within 1e-5 of it."""
    from oracle import oracle as orc
    ops = _ops()
    rng = np.random.default_rng(31 + aligned)
    N, C, H, W, scale = 2, 32, 36, 44, 0.25
    feat = rng.standard_normal((N, C, H, W)).astype(np.float32)
    per = [_boxes(rng, n, H / scale, W / scale, med) for n, med in ((40, 30), (25, 90))]
    per[1][0] = [-20, -30, 170, 150]  # partly outside, large grid (ceil(~45/7) = 7 samples a side)
    rois = np.concatenate([np.concatenate([np.full((len(b), 1), i, np.float32), b], 1) for i, b in enumerate(per)])
    x = torch.from_numpy(feat).to(dev).requires_grad_(True)
    y = ops.roi_align(x, [torch.from_numpy(b).to(dev) for b in per], (5, 6), scale, -1, aligned)
    ref = orc.roi_align(feat, rois, scale, (5, 6), -1, aligned)
    assert np.array_equal(y.detach().cpu().numpy(), ref)
    y0 = ops.roi_align(x, torch.from_numpy(rois).to(dev), (5, 6), scale, 0, aligned)  # 0 is adaptive too
    assert torch.equal(y0, y)
    g = rng.standard_normal(y.shape).astype(np.float32)
    y.backward(torch.from_numpy(g).to(dev))
    gr = orc.roi_align_backward(g, rois, scale, (N, C, H, W), -1, aligned)
    err = np.abs(x.grad.cpu().numpy() - gr).max() / np.abs(gr).max()
    assert err < 1e-5, err
    with pytest.raises(RuntimeError):
        ops.roi_align(x, torch.zeros(3, 4, device=dev), 7, scale, 2, aligned)
    assert ops.roi_align(x, [], 7, scale, -1, aligned).shape == (0, C, 7, 7)
