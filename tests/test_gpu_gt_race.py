"""The padded GT batch race: the RPN's target / sampler chain builds the step's
padded GT batch (frcnn._gt_batch) on its side stream, and the RoI sampler reads that cached batch on
the main stream. FasterRCNN.forward makes the main stream wait for the batch's event right before the
RoI heads (frcnn.py, `_gt_ready`). Here the side stream is held back by a ~10 ms spin kernel issued
in front of the batch's construction: with the wait in place the RoI sample, the losses and every
trainable gradient stay bitwise equal to the undelayed step; without it the main stream would read
the batch before it is written (zero-filled or stale slots and counts)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SPIN_CYCLES = 25_000_000  # ~10 ms at gfx950 clocks: far longer than the proposal chain it races


def _model(dev):
    from mx_det import frcnn
    torch.manual_seed(0)
    m = frcnn.fasterrcnn_resnet50_fpn_v2(weights=None)
    m.roi_heads.box_predictor = frcnn.FastRCNNPredictor(1024, 7)
    frcnn.set_trainable_layers(m.backbone.body, 3)
    return m.to(dev).train()


def _run(dev, monkeypatch, delay):
    from mx_det import frcnn
    from mx_det.data import synth_batch
    orig = frcnn._gt_batch
    main = torch.cuda.current_stream(dev)
    delayed = []

    def slow_gt_batch(targets, d):
        if torch.cuda.current_stream(d) != main:  # the side stream's build, not the sampler's lookup
            torch.cuda._sleep(SPIN_CYCLES)
            delayed.append(1)
        return orig(targets, d)
    slow_gt_batch.cache = None

    if delay:
        monkeypatch.setattr(frcnn, "_gt_batch", slow_gt_batch)
    frcnn._gt_batch.cache = None
    orig.cache = None
    m = _model(dev)
    imgs, tg = synth_batch(17, 6, H=448, W=640, device=dev)
    out = []
    try:
        for step in range(3):  # capture, then graph replays
            torch.cuda.manual_seed(200 + step)
            losses = m(imgs[2 * step:2 * step + 2], tg[2 * step:2 * step + 2])
            for p in m.parameters():
                p.grad = None
            sum(losses.values()).backward()
            out.append(([float(v) for v in losses.values()],
                        [p.grad.clone() for p in m.parameters() if p.requires_grad and p.grad is not None]))
        torch.cuda.synchronize()
    finally:
        monkeypatch.setattr(frcnn, "_gt_batch", orig)
    return out, len(delayed)


@pytest.mark.timeout(300)
def test_gt_batch_side_stream_delay_is_waited_for(dev, monkeypatch):
    ref, n0 = _run(dev, monkeypatch, False)
    got, n1 = _run(dev, monkeypatch, True)
    assert n0 == 0 and n1 >= 3, (n0, n1)  # every step's batch was built behind the spin
    for step, ((la, ga), (lb, gb)) in enumerate(zip(got, ref)):
        assert la == lb, (step, la, lb)
        assert len(ga) == len(gb)
        for x, y in zip(ga, gb):
            assert torch.equal(x, y), step
