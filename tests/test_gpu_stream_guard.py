"""Cross-stream hand-offs of the captured backward: a GradChain's
running gradient sum and a GradSlot's absorbed gradient pass between backward nodes OUTSIDE autograd's
edges, so autograd inserts no cross-stream wait for them. A consumer moved to a side stream (the
round-3 downsample-branch attempt, which crashed the backward capture) must raise a clear error at
forward time; consumers on one stream still chain; an unclaimed GradSlot keeps its output a backward
root; the dense (1x1-GEMM) ConvAct branch adds a claimed slot's gradient."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _x(dev, shape=(2, 9, 11, 64)):
    return torch.randn(shape, device=dev).requires_grad_(True)


def _w(dev, K=64, C=64, k=3):
    return (0.05 * torch.randn(K, C, k, k, device=dev)).requires_grad_(True)


def test_chain_consumer_on_side_stream_raises(dev):
    from mx_det import conv as mc
    x, w1, w2 = _x(dev), _w(dev), _w(dev)
    side = torch.cuda.Stream(device=dev)
    with mc.absorb_mode():
        mc.chain_over(x)
        mc.ConvAct.apply(x, w1, None, (1, 1), (1, 1), 0, None)  # first consumer: main stream
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side), pytest.raises(RuntimeError, match="GradChain"):
            mc.ConvAct.apply(x, w2, None, (1, 1), (1, 1), 0, None)
    torch.cuda.synchronize()


def test_chain_consumers_on_one_stream_sum_gradients(dev):
    from mx_det import conv as mc
    x, w1, w2 = _x(dev), _w(dev), _w(dev)
    with mc.absorb_mode():
        mc.chain_over(x)
        y = mc.ConvAct.apply(x, w1, None, (1, 1), (1, 1), 0, None) + mc.ConvAct.apply(x, w2, None, (1, 1), (1, 1), 0, None)
    y.sum().backward()
    g_chain = x.grad.clone()
    x2 = x.detach().clone().requires_grad_(True)
    y2 = mc.ConvAct.apply(x2, w1, None, (1, 1), (1, 1), 0, None) + mc.ConvAct.apply(x2, w2, None, (1, 1), (1, 1), 0, None)
    y2.sum().backward()
    torch.testing.assert_close(g_chain, x2.grad, rtol=1e-4, atol=1e-4)


def test_slot_consumer_on_side_stream_raises(dev):
    from mx_det import conv as mc
    x, w = _x(dev), _w(dev)
    slot = mc.GradSlot()
    side = torch.cuda.Stream(device=dev)
    with mc.absorb_mode():
        mc.absorb_into(x, slot)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side), pytest.raises(RuntimeError, match="GradSlot"):
            mc.ConvAct.apply(x, w, None, (1, 1), (1, 1), 0, None)
    assert not slot.taken
    torch.cuda.synchronize()


def test_unclaimed_slot_stays_a_root(dev):
    from mx_det import conv as mc
    from mx_det.frcnn import _absorb_roots

    class Fn:
        def __init__(self, slots):
            self.slots = slots

        def absorbed(self):
            return self.slots

    a, b = torch.ones(3, device=dev), torch.ones(4, device=dev)
    ga, gb = torch.zeros(3, device=dev), torch.zeros(4, device=dev)
    claimed, unclaimed = mc.GradSlot().claim(), mc.GradSlot()
    roots, groots = _absorb_roots(Fn([claimed, unclaimed]), (a, b), (ga, gb))
    assert claimed.buf is ga and unclaimed.buf is None
    assert len(roots) == 1 and roots[0] is b and groots[0] is gb


def test_dense_branch_adds_claimed_slot(dev):
    """A valid 7x7 conv on a 7x7 map (FC6's dense GEMM branch): the claimed slot's gradient is added
    to dx, as the implicit-GEMM branch adds it in its epilogue."""
    from mx_det import conv as mc
    x = torch.randn(4, 7, 7, 64, device=dev).requires_grad_(True)
    w = (0.01 * torch.randn(64, 64, 7, 7, device=dev)).requires_grad_(True)
    slot = mc.GradSlot()
    with mc.absorb_mode():
        mc.absorb_into(x, slot)
        y = mc.ConvAct.apply(x, w, None, (1, 1), (0, 0), 0, None)
    assert slot.taken
    slot.buf = torch.randn_like(x)
    g = torch.randn_like(y)
    y.backward(g)
    x2 = x.detach().clone().requires_grad_(True)
    mc.ConvAct.apply(x2, w, None, (1, 1), (0, 0), 0, None).backward(g)
    torch.testing.assert_close(x.grad, x2.grad + slot.buf, rtol=1e-5, atol=1e-5)
