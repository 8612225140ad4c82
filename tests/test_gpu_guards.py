"""Guards on the product path that turn silent failures into errors.

* Stream identity. Round 4 found that torch's round-robin pool of 32 streams per device had aliased a
  new side stream onto another framework / capture stream, and a later backward capture crashed in
  hipStreamEndCapture (gpurun_out/r04t tests.log: segfault in capture_end <- frcnn._Graphs). The fix
  gave every framework side stream a HIP stream of its own (conv.dedicated_stream / mx_stream_create).
  This test exhausts the pool first (40 torch streams), then builds the model, captures and replays a
  train step, and checks that every dedicated stream is distinct from every other and from every pool
  stream handed out.
* Proposal NMS status. mx_batched_nms_grouped_sorted reports candidates outside its presorted layout as
  num_keep = -2 (its selection is then empty); the RPN now raises instead of training on zero
  proposals (RegionProposalNetwork.check_nms).
"""
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


def test_dedicated_streams_never_alias_pool_streams(dev):
    from mx_det import conv, frcnn
    from mx_det.data import synth_batch
    from mx_det.optim import SGD
    pool = [torch.cuda.Stream(device=dev) for _ in range(40)]  # more than the pool's 32 per priority
    m = _model(dev)
    opt = SGD([p for p in m.parameters() if p.requires_grad], lr=1e-3, momentum=0.9)
    imgs, tg = synth_batch(3, 4, H=384, W=512, device=dev)
    for step in range(2):  # capture, then replay
        loss = sum(m(imgs[2 * step:2 * step + 2], tg[2 * step:2 * step + 2]).values())
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    assert torch.isfinite(loss)
    assert any(isinstance(g, frcnn._Graphs) for g in m.__dict__.get("_mx_graphs", {}).values())
    conv.dedicated_stream(dev, "wgrad")  # every name the framework uses exists now
    conv.capture_stream(dev)
    ded = {k: s.cuda_stream for k, s in conv._dedicated.items() if k[0] == dev.index}
    for name in ("capture", "wgrad", "fpn", "rpn_head", "rpn_targets"):
        assert (dev.index, name) in ded, (name, sorted(ded))
    handles = list(ded.values())
    assert len(set(handles)) == len(handles), ded
    pool_handles = {s.cuda_stream for s in pool} | {torch.cuda.current_stream(dev).cuda_stream}
    assert not (set(handles) & pool_handles), (ded, pool_handles)
    assert conv.capture_stream(dev).cuda_stream == ded[(dev.index, "capture")]


def test_sorted_nms_layout_violation_raises(dev):
    """Candidates whose levels are interleaved (the presorted contract broken): the sorted NMS returns
    num_keep = -2 and an all-False selection; filter_proposals_padded's caller raises."""
    from mx_det import frcnn, ops
    from mx_det.backend import HipBackend
    be = HipBackend("f32")
    rpn = frcnn.fasterrcnn_resnet50_fpn_v2(weights=None).rpn.to(dev).train()
    N, pad = 2, (256, 320)
    grid = [(64, 80), (32, 40), (16, 20), (8, 10), (4, 5)]
    npl = [h * w * 3 for h, w in grid]
    A = sum(npl)
    anchors = rpn.anchor_generator(pad, grid, dev, be)
    g = torch.Generator(device=dev).manual_seed(3)
    obj = torch.randn(N, A, device=dev, generator=g)
    dl = torch.randn(N, A, 4, device=dev, generator=g) * 0.2
    props = be.box_decode(dl.reshape(-1, 4), anchors.repeat(N, 1), frcnn.RPN_WEIGHTS).view(N, A, 4)
    sizes = [(256, 320), (240, 320)]
    # the intact chain: no error
    pb, ps, valid = rpn.filter_proposals_padded(props, obj, sizes, npl, be)
    rpn.check_nms()
    assert int(valid.sum()) > 0
    # interleave the levels of the candidate list the NMS sees
    orig = HipBackend.proposal_nms_select

    def shuffled(self, boxes, scores, lvl, group, G, L, thr, max_seg, post):
        perm = torch.randperm(lvl.shape[0], generator=torch.Generator().manual_seed(0)).to(lvl.device)
        return orig(self, boxes, scores, lvl[perm], group, G, L, thr, max_seg, post)

    HipBackend.proposal_nms_select = shuffled
    try:
        _, _, valid = rpn.filter_proposals_padded(props, obj, sizes, npl, be)
        with pytest.raises(RuntimeError, match="presorted"):
            rpn.check_nms()
    finally:
        HipBackend.proposal_nms_select = orig
    # the op itself: interleaved levels -> num_keep == -2
    b = torch.rand(64, 2, device=dev) * 100
    boxes = torch.cat([b, b + 10], 1)
    scores = torch.linspace(1, 0, 64, device=dev)
    lvl = torch.arange(64, device=dev) % 2
    grp = torch.zeros(64, dtype=torch.int32, device=dev)
    _, nk, _, valid = ops.batched_nms_grouped_sorted(boxes, scores, lvl, grp, 1, 2, 0.7, 1000, 16)
    assert int(nk) == -2 and not bool(valid.any())


def test_capture_while_loader_threads_pin(dev):
    """the prefetch loader's producer (engine._pack_targets) and decode workers
    (jpeg.host_stage) allocate pinned host memory on their own threads while the training thread captures
    its graphs lazily (first step, new RoI-head shapes). Under the global capture mode a pinned allocation
    from another thread invalidates an open capture; both now take conv.capture_lock, which every capture
    holds. Here a thread pins fresh (growing, so cache-missing) buffers through both paths while the main
    thread captures and replays graphs under conv.capture_guard()."""
    import io
    import threading

    import numpy as np
    from PIL import Image

    from mx_det import conv, jpeg
    from mx_det.engine import _pack_targets

    buf = io.BytesIO()
    Image.fromarray((np.arange(64 * 96 * 3) % 251).astype(np.uint8).reshape(64, 96, 3)).save(buf, "JPEG", quality=90)
    data = np.frombuffer(buf.getvalue(), dtype=np.uint8)
    stop, errors, count = threading.Event(), [], [0]

    def pinner():
        k = 1
        try:
            while not stop.is_set():
                jpeg.host_stage(data)
                _pack_targets([{"boxes": torch.zeros(k * 1024, 4), "labels": torch.zeros(k, dtype=torch.int64)}])
                k += 1
                count[0] += 1
        except Exception as e:  # noqa: BLE001 -- reported by the main thread
            errors.append(repr(e))

    th = threading.Thread(target=pinner, daemon=True)
    th.start()
    try:
        side = conv.capture_stream(dev)
        x = torch.arange(1 << 16, device=dev, dtype=torch.float32)
        for i in range(20):
            side.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            with conv.capture_guard(), torch.cuda.graph(g, stream=side):
                y = x * (i + 1) + 1.0
            g.replay()
            torch.cuda.synchronize()
            assert torch.equal(y, x * (i + 1) + 1.0), i
    finally:
        stop.set()
        th.join(timeout=30)
    assert not errors, errors
    assert count[0] > 0
