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
