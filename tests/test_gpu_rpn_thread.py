"""The RPN target / sampler chain issued by a helper thread beside the trunk's forward graph launch
(RegionProposalNetwork.start_targets, MX_RPN_TARGETS_THREAD=1, the default) against the same chain
issued after the trunk on the calling thread (=0): same launches, same RNG draws in the same order, so
over a capture step and two replay steps the losses and every trainable gradient are bitwise equal."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model(dev):
    from mx_det import frcnn
    torch.manual_seed(0)
    m = frcnn.fasterrcnn_resnet50_fpn_v2(weights=None)
    m.roi_heads.box_predictor = frcnn.FastRCNNPredictor(1024, 7)
    frcnn.set_trainable_layers(m.backbone.body, 3)
    return m.to(dev).train()


def _run(dev, monkeypatch, thread):
    from mx_det import frcnn
    from mx_det.data import synth_batch
    monkeypatch.setenv("MX_RPN_TARGETS_THREAD", thread)
    calls = []
    helper = frcnn._helper
    monkeypatch.setattr(frcnn, "_helper", lambda: (calls.append(1), helper())[1])
    m = _model(dev)
    imgs, tg = synth_batch(5, 6, H=448, W=640, device=dev)
    out = []
    for step in range(3):  # capture, then replays (the helper thread needs a replayed trunk)
        torch.cuda.manual_seed(100 + step)
        losses = m(imgs[2 * step:2 * step + 2], tg[2 * step:2 * step + 2])
        for p in m.parameters():
            p.grad = None
        sum(losses.values()).backward()
        out.append(([float(v) for v in losses.values()],
                    [p.grad.clone() for p in m.parameters() if p.requires_grad and p.grad is not None]))
    torch.cuda.synchronize()
    monkeypatch.setattr(frcnn, "_helper", helper)
    return out, len(calls)


def test_rpn_targets_helper_thread_matches_inline(dev, monkeypatch):
    a, na = _run(dev, monkeypatch, "1")
    b, nb = _run(dev, monkeypatch, "0")
    assert (na, nb) == (2, 0)  # the two replay steps issued the chain from the helper thread
    for step, ((la, ga), (lb, gb)) in enumerate(zip(a, b)):
        assert la == lb, (step, la, lb)
        assert len(ga) == len(gb)
        for x, y in zip(ga, gb):
            assert torch.equal(x, y), step
