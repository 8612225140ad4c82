"""Host logic of the detection model (CPU, no GPU): torchvision-compatible module tree and the
reference's train/eval call contract, run end-to-end on the CPU restatement backend
(oracle/cpu_backend.py) at a small image size."""
import pytest
import torch

from oracle.cpu_backend import CpuBackend


def _model(nc=7, trainable=3):
    from mx_det import frcnn
    m = frcnn.fasterrcnn_resnet50_fpn_v2(weights=None)
    m.roi_heads.box_predictor = frcnn.FastRCNNPredictor(m.roi_heads.box_predictor.cls_score.in_features, nc)
    frcnn.set_trainable_layers(m.backbone.body, trainable)
    return m.set_backend(CpuBackend())


def test_state_dict_matches_torchvision_layout():
    from mx_det import frcnn
    m = frcnn.fasterrcnn_resnet50_fpn_v2(weights=None)
    assert sum(p.numel() for p in m.parameters()) == 43712278  # torchvision fasterrcnn_resnet50_fpn_v2
    sd = m.state_dict()
    for k, shape in [("backbone.body.conv1.weight", (64, 3, 7, 7)),
                     ("backbone.body.layer4.2.bn3.running_var", (2048,)),
                     ("backbone.body.layer2.0.downsample.0.weight", (512, 256, 1, 1)),
                     ("backbone.fpn.inner_blocks.3.0.weight", (256, 2048, 1, 1)),
                     ("backbone.fpn.layer_blocks.0.1.num_batches_tracked", ()),
                     ("rpn.head.conv.1.0.bias", (256,)),
                     ("rpn.head.bbox_pred.weight", (12, 256, 1, 1)),
                     ("roi_heads.box_head.3.1.weight", (256,)),
                     ("roi_heads.box_head.5.weight", (1024, 12544)),
                     ("roi_heads.box_predictor.bbox_pred.weight", (364, 1024))]:
        assert tuple(sd[k].shape) == shape, k
    m2 = _model()
    assert sum(p.numel() for p in m2.parameters() if p.requires_grad) == 43056434  # 43.06M


def test_train_step_contract_cpu():
    from mx_det.data import synth_batch
    torch.manual_seed(0)
    m = _model().train()
    imgs, tg = synth_batch(0, 2, H=128, W=192)
    images = [im.permute(2, 0, 1).float() / 255 for im in imgs]
    losses = m(images, tg)
    assert list(losses) == ["loss_classifier", "loss_box_reg", "loss_objectness", "loss_rpn_box_reg"]
    total = sum(losses.values())
    assert torch.isfinite(total)
    total.backward()
    assert m.backbone.body.layer2[0].conv1.weight.grad is not None
    assert m.backbone.body.layer1[0].conv1.weight.grad is None  # frozen (trainable_backbone_layers=3)
    assert m.roi_heads.box_head[5].weight.grad.abs().sum() > 0
    assert int(m.backbone.body.bn1.num_batches_tracked) == 1  # BN stays in train mode when frozen


def test_eval_contract_cpu():
    from mx_det.data import synth_batch
    m = _model().eval()
    imgs, _ = synth_batch(3, 1, H=128, W=160)
    with torch.no_grad():
        out = m([imgs[0].permute(2, 0, 1).float() / 255])
    assert len(out) == 1 and set(out[0]) == {"boxes", "labels", "scores"}
    assert out[0]["boxes"].shape[0] <= 100 and out[0]["boxes"].shape[1] == 4


def test_degenerate_boxes_rejected():
    m = _model().train()
    img = [torch.rand(3, 64, 64)]
    with pytest.raises(ValueError):
        m(img, [{"boxes": torch.tensor([[10., 10., 5., 20.]]), "labels": torch.tensor([1])}])


def _rpn_head_run(be, feats, canvas, monkeypatch, seed=0):
    from mx_det import frcnn
    monkeypatch.setenv("MX_RPN_CANVAS", "1" if canvas else "0")
    torch.manual_seed(seed)
    head = frcnn.RPNHead(256, 3)
    for p in head.parameters():
        torch.nn.init.normal_(p, std=0.05)
    head = head.to(feats[0].device)
    fs = [f.clone().requires_grad_(True) for f in feats]
    obj, dls, npl = head(fs, be)
    logits, deltas = list(obj.split(npl, 1)), list(dls.split(npl, 1))
    loss = sum((lg * (i + 1)).sin().sum() + dl.cos().sum() for i, (lg, dl) in enumerate(zip(logits, deltas)))
    loss.backward()
    return ([t.detach() for t in logits + deltas], [f.grad for f in fs],
            {k: p.grad for k, p in head.named_parameters()})


def test_rpn_head_canvas_equals_per_level(monkeypatch):
    """RPNHead's small levels run as one conv chain over a zero-framed canvas (frcnn.RPNHead.forward):
    logits / deltas, feature gradients and the shared weights' gradients equal the per-level chains
    (torchvision's loop), here on the CPU restatement backend."""
    torch.manual_seed(1)
    hw = [(40, 52), (20, 26), (10, 13), (5, 7), (3, 4)]
    feats = [torch.randn(2, h, w, 256) for h, w in hw]
    a = _rpn_head_run(CpuBackend(), feats, True, monkeypatch)
    b = _rpn_head_run(CpuBackend(), feats, False, monkeypatch)
    for x, y in zip(a[0] + a[1], b[0] + b[1]):
        assert x.shape == y.shape
        torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-4)
    for k in a[2]:
        torch.testing.assert_close(a[2][k], b[2][k], rtol=1e-4, atol=1e-3)


def test_rpn_canvas_layout_frames_levels():
    from mx_det import frcnn
    hws = [(100, 168), (50, 84), (25, 42), (13, 21)]
    pos, Hc, Wc = frcnn.RPNHead.canvas_layout(hws)
    occ = torch.zeros(Hc + 2, Wc + 2, dtype=torch.int32)
    for (h, w), (y, x) in zip(hws, pos):
        assert y + h <= Hc and x + w <= Wc
        occ[y:y + h + 2, x:x + w + 2] += 1  # the level plus a one-pixel frame on every side
    inner = torch.zeros_like(occ)
    for (h, w), (y, x) in zip(hws, pos):
        inner[y + 1:y + h + 1, x + 1:x + w + 1] += 1
    assert int((inner * (occ - 1)).sum()) == 0  # no level pixel lies in another level's frame
