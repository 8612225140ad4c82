"""GPU numerics of the train-mode BatchNorm kernels (mx_bn.hip) against torch fp32 on the same
bf16-rounded tensors: forward statistics/finalize, backward reduce (partials + f64 column sums) and
the streaming backward apply, for every activation and the channel widths of the model."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,K,act", [(1000, 64, 1), (2100, 2048, 1), (777, 256, 0), (4099, 128, 2), (8, 8, 1)])
def test_bn_backward_matches_torch(dev, M, K, act):
    from mx_det import _lib
    from mx_det.conv import _p, _s
    g = torch.Generator().manual_seed(M + K + act)
    z = (torch.randn(M, K, generator=g) * 2 + 0.5).bfloat16()
    gamma = torch.rand(K, generator=g) + 0.5
    beta = torch.randn(K, generator=g) * 0.1
    dy = torch.randn(M, K, generator=g).bfloat16()
    # torch reference on the bf16 values
    zr = z.float().requires_grad_(True)
    gr, br = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    out = F.batch_norm(zr, None, None, gr, br, training=True, eps=1e-5)
    yr = F.relu(out) if act == 1 else F.leaky_relu(out, 0.2) if act == 2 else out
    yr.backward(dy.float())
    mean = z.float().mean(0)
    invstd = 1.0 / torch.sqrt(z.float().var(0, unbiased=False) + 1e-5)
    y = yr.detach().bfloat16()
    zd, yd, dyd = z.to(dev), y.to(dev), dy.to(dev)
    meand, invd, gd = mean.to(dev), invstd.to(dev), gamma.to(dev)
    wsb = _lib.load().mx_bn_bwd_workspace(M, K)
    ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)  # arrival counters start (and stay) zero
    sums = torch.empty(2, K, device=dev)
    coef = torch.empty(3, K, device=dev)
    _lib.call("mx_bn_bwd_reduce_ex", _p(dyd), _p(yd), _p(zd), 1, M, K, act, _p(meand), _p(invd), _p(gd), _p(ws), wsb,
              _p(sums), _p(coef), _s())
    # second launch on the same workspace: the counters were left zero, results identical
    sums_b, coef_b = torch.empty_like(sums), torch.empty_like(coef)
    _lib.call("mx_bn_bwd_reduce_ex", _p(dyd), _p(yd), _p(zd), 1, M, K, act, _p(meand), _p(invd), _p(gd), _p(ws), wsb,
              _p(sums_b), _p(coef_b), _s())
    torch.cuda.synchronize()
    assert torch.equal(sums, sums_b) and torch.equal(coef, coef_b)
    assert int(ws[:256].sum()) == 0
    dx = torch.empty_like(zd)
    dres = torch.empty_like(zd)
    _lib.call("mx_bn_bwd_apply_ex", _p(dyd), _p(yd), _p(zd), 1, M, K, act, _p(coef), _p(dx), _p(dres), _s())
    torch.cuda.synchronize()
    # the activation mask of the device path is the one of the bf16 y it was given
    mask = (y.float() > 0).float() if act == 1 else torch.where(y.float() > 0, 1.0, 0.2) if act == 2 else 1.0
    gmask = dy.float() * mask
    torch.testing.assert_close(dres.float().cpu(), gmask, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(sums[0].cpu(), gmask.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(sums[1].cpu(), gr.grad, rtol=2e-2, atol=5e-1)
    rel = ((dx.float().cpu() - zr.grad).norm() / zr.grad.norm()).item()
    assert rel < 2e-2, rel
    # legacy convenience entries agree with the hot path
    s2 = torch.full((2, K), 7.0, device=dev)
    _lib.call("mx_bn_bwd_reduce", _p(dyd), _p(yd), _p(zd), M, K, act, _p(meand), _p(invd), _p(s2), _s())
    dx2 = torch.empty_like(zd)
    _lib.call("mx_bn_bwd_apply", _p(dyd), _p(yd), _p(zd), M, K, act, _p(meand), _p(invd), _p(gd), _p(s2), _p(dx2),
              None, _s())
    torch.cuda.synchronize()
    assert torch.equal(s2, sums)
    torch.testing.assert_close(dx2.float(), dx.float(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("M,K", [(134400, 256), (2100, 2048), (100, 8)])
def test_bn_finalize_matches_torch(dev, M, K):
    """Stats partials [2][mblocks][K] -> mean/invstd/scale/shift and running-stat update."""
    from mx_det import _lib
    from mx_det.conv import _p, _s
    g = torch.Generator().manual_seed(K)
    z = torch.randn(M, K, generator=g) * 3 + 1
    mb = (M + 127) // 128
    zp = torch.nn.functional.pad(z, (0, 0, 0, mb * 128 - M)).view(mb, 128, K)
    stats = torch.stack([zp.sum(1), (zp * zp).sum(1)]).contiguous().to(dev)
    gamma, beta = torch.rand(K, generator=g) + 0.5, torch.randn(K, generator=g)
    rm, rv = torch.zeros(K, device=dev), torch.ones(K, device=dev)
    outs = [torch.empty(K, device=dev) for _ in range(4)]
    _lib.call("mx_bn_finalize", _p(stats), mb, K, M, _p(gamma.to(dev)), _p(beta.to(dev)), 1e-5, 0.1, _p(rm), _p(rv),
              *[_p(o) for o in outs], _s())
    torch.cuda.synchronize()
    zd = z.double()
    mean, var = zd.mean(0), zd.var(0, unbiased=False)
    torch.testing.assert_close(outs[0].cpu().double(), mean, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(outs[1].cpu().double(), 1 / torch.sqrt(var + 1e-5), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rm.cpu().double(), 0.1 * mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rv.cpu().double(), 0.9 + 0.1 * zd.var(0, unbiased=True), rtol=1e-5, atol=1e-6)
    # hot-path form (one launch, persistent zero-filled workspace), twice on the same workspace
    wsb = _lib.load().mx_bn_finalize_workspace(mb, K)
    ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
    for _ in range(2):
        o2 = [torch.empty(K, device=dev) for _ in range(4)]
        _lib.call("mx_bn_finalize_ex", _p(stats), mb, K, M, _p(gamma.to(dev)), _p(beta.to(dev)), 1e-5, 0.1, None,
                  None, *[_p(o) for o in o2], _p(ws), wsb, _s())
        torch.cuda.synchronize()
        for a, b in zip(outs, o2):
            assert torch.equal(a, b)
        assert int(ws[:256].sum()) == 0


@pytest.mark.parametrize("M,K,act,dt", [(134400, 15, 0, torch.float32), (8400, 256, 1, torch.bfloat16),
                                        (1024, 1024, 1, torch.bfloat16), (1024, 35, 0, torch.float32),
                                        (77, 24, 2, torch.bfloat16), (5, 3, 1, torch.float32)])
def test_act_bias_bwd_matches_torch(dev, M, K, act, dt):
    """ConvAct backward head: g = gy*act'(y) (bf16, zero-padded to K8) and db = sum of g."""
    from mx_det import conv as mc
    g = torch.Generator().manual_seed(M + K)
    gy = torch.randn(M, K, generator=g).to(dt)
    y = torch.randn(M, K, generator=g).to(dt)
    K8 = (K + 7) // 8 * 8
    for _ in range(2):  # second call reuses the persistent scratch (counters left zero)
        out, db = mc.act_bias_bwd(gy.to(dev), y.to(dev), act, K8, True)
        torch.cuda.synchronize()
    yf = y.float()
    mask = (yf > 0).float() if act == 1 else torch.where(yf > 0, 1.0, 0.2) if act == 2 else torch.ones_like(yf)
    ref = gy.float() * mask
    assert out.shape == (M, K8)
    assert torch.equal(out[:, :K].cpu(), ref.bfloat16())
    assert int((out[:, K:] != 0).sum()) == 0
    torch.testing.assert_close(db.cpu().double(), ref.double().sum(0), rtol=1e-5, atol=1e-3)


def test_sgd_matches_torch(dev):
    """mx_det.optim.SGD (one multi-tensor launch) == torch.optim.SGD over 6 steps (momentum, wd),
    including a parameter without grad, odd sizes (scalar tail path), the cached steady-state path
    and a load_state_dict in between."""
    from mx_det.optim import SGD
    g = torch.Generator().manual_seed(3)
    shapes = [(256, 256, 3, 3), (1000,), (7,), (12, 5), (3, 3)]
    ref = [torch.randn(s, generator=g) for s in shapes]
    a = [r.clone().to(dev).requires_grad_(True) for r in ref]
    b = [r.clone().to(dev).requires_grad_(True) for r in ref]
    oa = SGD(a, lr=0.005, momentum=0.9, weight_decay=5e-4)
    ob = torch.optim.SGD(b, lr=0.005, momentum=0.9, weight_decay=5e-4)
    for it in range(6):
        if it == 4:  # new momentum-buffer storage: the cached pointer arrays must be dropped
            oa.load_state_dict(oa.state_dict())
            ob.load_state_dict(ob.state_dict())
        for i, (x, y) in enumerate(zip(a, b)):
            if i == 4 and it == 1:  # no grad this step
                x.grad = y.grad = None
                continue
            gr = torch.randn(x.shape, generator=g).to(dev)
            x.grad, y.grad = gr.clone(), gr.clone()
        oa.step()
        ob.step()
        torch.cuda.synchronize()
        for x, y in zip(a, b):
            torch.testing.assert_close(x.detach(), y.detach(), rtol=1e-6, atol=1e-7)


def test_sgd_bumps_versions_for_the_packer(dev):
    """The fused SGD writes through raw pointers; it must bump _version like an in-place op so the
    conv WeightPacker repacks the bf16 operands after every step."""
    from mx_det.optim import SGD
    p = torch.randn(64, 32, 3, 3, device=dev, requires_grad=True)
    v0 = p._version
    opt = SGD([p], lr=0.1, momentum=0.9)
    p.grad = torch.ones_like(p)
    opt.step()
    assert p._version > v0
