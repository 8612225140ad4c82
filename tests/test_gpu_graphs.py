"""HIP-graph capture of the RPN proposal chain (box decode + filter_proposals_padded: per-level top-k,
clip, size/score filter, the grouped NMS over all images, post-NMS top-n) replayed against eager on
fresh inputs: bitwise-equal outputs on every replay. The chain has no host synchronisation (SURVEY.md
§8 row 2), so it is capturable as long as every op it issues is; this pins that property."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rpn(dev, training):
    from mx_det import frcnn
    m = frcnn.fasterrcnn_resnet50_fpn_v2(weights=None)
    rpn = m.rpn.to(dev)
    rpn.train(training)
    return rpn


@pytest.mark.parametrize("training", [True, False])
def test_rpn_proposal_chain_graph_replay_matches_eager(dev, training):
    from mx_det import frcnn
    from mx_det.backend import HipBackend
    be = HipBackend("f32")
    rpn = _rpn(dev, training)
    N, pad = 2, (800, 1344)
    grid = [(200, 336), (100, 168), (50, 84), (25, 42), (13, 21)]
    num_per_level = [h * w * 3 for h, w in grid]
    A = sum(num_per_level)
    anchors = rpn.anchor_generator(pad, grid, dev, be)
    sizes = [(800, 1333), (750, 1333)]
    g = torch.Generator(device=dev).manual_seed(5)

    def draw():
        return (torch.randn(N, A, device=dev, generator=g) * 2,
                torch.randn(N, A, 4, device=dev, generator=g) * 0.2)

    def chain(obj, dl):
        props = be.box_decode(dl.reshape(-1, 4), anchors.repeat(N, 1), frcnn.RPN_WEIGHTS).view(N, A, 4)
        return rpn.filter_proposals_padded(props, obj, sizes, num_per_level, be)

    s_obj, s_dl = draw()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # warm-up (allocator, per-shape caches) off the default stream
        for _ in range(2):
            chain(s_obj, s_dl)
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = chain(s_obj, s_dl)
    for _ in range(3):
        obj, dl = draw()
        s_obj.copy_(obj)
        s_dl.copy_(dl)
        graph.replay()
        ref = chain(obj, dl)
        torch.cuda.synchronize()
        for a, b in zip(out, ref):
            assert torch.equal(a, b)
        assert int(out[2].sum()) > 100  # survivors exist


def test_proposal_graph_survives_a_shape_change(dev):
    """A graph captured for one padded shape keeps replaying correctly after the anchor generator has
    served another shape (its anchors for the captured shape must stay allocated)."""
    from mx_det import frcnn
    from mx_det.backend import HipBackend
    be = HipBackend("f32")
    rpn = _rpn(dev, True)
    N = 2
    shapes = {(800, 1344): [(200, 336), (100, 168), (50, 84), (25, 42), (13, 21)],
              (832, 1344): [(208, 336), (104, 168), (52, 84), (26, 42), (13, 21)]}
    sizes = [(800, 1333), (790, 1333)]
    g = torch.Generator(device=dev).manual_seed(9)

    def chain(pad, obj, dl):
        grid = shapes[pad]
        npl = [h * w * 3 for h, w in grid]
        anchors = rpn.anchor_generator(pad, grid, dev, be)
        props = be.box_decode(dl.reshape(-1, 4), anchors.repeat(N, 1), frcnn.RPN_WEIGHTS).view(N, -1, 4)
        return rpn.filter_proposals_padded(props, obj, sizes, npl, be)

    pad0 = (800, 1344)
    A0 = sum(h * w * 3 for h, w in shapes[pad0])
    obj = torch.randn(N, A0, device=dev, generator=g)
    dl = torch.randn(N, A0, 4, device=dev, generator=g) * 0.2
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        chain(pad0, obj, dl)
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = chain(pad0, obj, dl)
    # another shape: its anchors are built (and, before the fix, replaced the captured shape's)
    pad1 = (832, 1344)
    A1 = sum(h * w * 3 for h, w in shapes[pad1])
    chain(pad1, torch.randn(N, A1, device=dev, generator=g), torch.randn(N, A1, 4, device=dev, generator=g) * 0.2)
    torch.cuda.empty_cache()
    for _ in range(2):
        obj.copy_(torch.randn(N, A0, device=dev, generator=g))
        graph.replay()
        ref = chain(pad0, obj, dl)
        torch.cuda.synchronize()
        for a, b in zip(out, ref):
            assert torch.equal(a, b)
