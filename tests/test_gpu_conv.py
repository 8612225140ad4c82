"""GPU numerics of the MFMA implicit-GEMM conv and the BatchNorm kernels.

Reference: torch fp32 conv on the same bf16-rounded operands (the kernels multiply bf16 exactly and
accumulate in f32, so only the summation order differs): f32-output comparisons use rtol 2e-5 of
the |x|.|w| scale; bf16 outputs add one bf16 rounding (2^-8 relative).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CASES = [
    # N, H, W, C, K, k, stride, pad
    (2, 17, 23, 64, 128, 3, 1, 1),
    (2, 20, 34, 128, 128, 3, 2, 1),
    (1, 25, 42, 256, 512, 1, 2, 0),
    (2, 33, 41, 8, 64, 7, 2, 3),       # stem: 3 real channels padded to 8
    (4, 1, 1, 12544 // 16, 1024, 1, 1, 0),
    (3, 9, 11, 256, 15, 1, 1, 0),      # RPN cls+bbox head (odd K)
    (2, 7, 7, 256, 256, 3, 1, 1),      # box head conv on RoI tiles
    (2, 25, 42, 1024, 256, 1, 1, 0),   # small grid -> split-K (slab + reduce epilogue)
    (2, 13, 21, 512, 512, 3, 1, 1),    # split-K, 3x3
    (1, 15, 19, 64, 64, 3, 2, 1),      # stride 2, odd sizes: 4 parity classes of unequal shape
    (2, 16, 22, 64, 256, 1, 2, 0),     # 1x1 stride 2: three classes receive no taps (dx = 0)
]


@pytest.fixture(params=[(0, 0, 0), (1, 0, 2), (3, 0, 1), (4, 0, 1), (5, 0, 1), (6, 0, 1), (7, 0, 0), (8, 0, 1),
                        (7, 1, 3), (8, 1, 3), (9, 1, 3), (7, 1, 0)])
def variant(request):
    """Every fwd/dgrad staging variant of the implicit-GEMM kernel (mx_conv_set_variant), with the
    per-lane global loader (0) or the buffer-descriptor loader (1, the default), and the wgrad
    variants (mx_conv_set_wgrad_variant)."""
    from mx_det import _lib
    v, loader, wv = request.param
    import os
    tune = os.environ.get("MX_CONV_TUNE")
    os.environ["MX_CONV_TUNE"] = "0"  # exactly the forced variants, not the per-shape tuner's picks
    old = _lib.load().mx_conv_get_variant()
    oldw = _lib.load().mx_conv_get_wgrad_variant()
    _lib.call("mx_conv_set_variant", v)
    _lib.call("mx_conv_set_loader", loader)
    _lib.call("mx_conv_set_wgrad_variant", wv)
    yield v
    if tune is None:
        os.environ.pop("MX_CONV_TUNE", None)
    else:
        os.environ["MX_CONV_TUNE"] = tune
    _lib.call("mx_conv_set_variant", old)
    _lib.call("mx_conv_set_loader", 1)
    _lib.call("mx_conv_set_wgrad_variant", oldw)


def _scale(x, w, k):
    return (x.abs().amax() * w.abs().amax() * x.shape[-1] * k * k).item()


@pytest.mark.parametrize("N,H,W,C,K,k,st,pd", CASES)
def test_conv_fwd(dev, variant, N, H, W, C, K, k, st, pd):
    from mx_det import conv as mc
    g = torch.Generator().manual_seed(N * 1000 + C + K)
    x = torch.randn(N, H, W, C, generator=g).bfloat16()
    w = (torch.randn(K, C, k, k, generator=g) * 0.05).bfloat16()
    b = torch.randn(K, generator=g)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float(), b, st, pd).permute(0, 2, 3, 1)
    wk, _ = mc.pack_weight(w.float().to(dev), C, (st, st), (pd, pd))
    assert torch.equal(wk.cpu(), mc.weight_krsc(w.float()))  # fused cast+permute == torch's
    y, stats = mc.conv_fwd(x.to(dev), wk, (st, st), (pd, pd), bias=b.to(dev), out_dtype=torch.float32, stats=True)
    tol = 2e-5 * _scale(x.float(), w.float(), k)
    torch.testing.assert_close(y.cpu(), ref, rtol=0, atol=tol)
    # BN statistics partials are over the pre-bias accumulators
    z = (ref - b).reshape(-1, K).double()
    s = stats.cpu().double().sum(1)
    torch.testing.assert_close(s[0], z.sum(0), rtol=1e-4, atol=tol * 10)
    torch.testing.assert_close(s[1], (z * z).sum(0), rtol=1e-4, atol=tol * tol * 10 + 1e-3)
    yb = mc.conv_fwd(x.to(dev), wk, (st, st), (pd, pd), bias=b.to(dev), act=mc.ACT_RELU)
    torch.testing.assert_close(yb.float().cpu(), ref.clamp_min(0), rtol=1e-2, atol=tol + 1e-2)


def test_conv_fwd_residual_leaky(dev):
    from mx_det import conv as mc
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, 16, 16, 64, generator=g).bfloat16()
    w = (torch.randn(64, 64, 3, 3, generator=g) * 0.05).bfloat16()
    r = torch.randn(2, 16, 16, 64, generator=g).bfloat16()
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float(), None, 1, 1).permute(0, 2, 3, 1) + r.float()
    ref = F.leaky_relu(ref, 0.2)
    y = mc.conv_fwd(x.to(dev), mc.weight_krsc(w.float()).to(dev), (1, 1), (1, 1), residual=r.to(dev),
                    act=mc.ACT_LEAKY, out_dtype=torch.float32)
    torch.testing.assert_close(y.cpu(), ref, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("N,H,W,C,K,k,st,pd", [c for c in CASES if c[4] % 8 == 0])
def test_conv_dgrad_wgrad(dev, variant, N, H, W, C, K, k, st, pd):
    from mx_det import conv as mc
    g = torch.Generator().manual_seed(7 + C + K)
    x = torch.randn(N, H, W, C, generator=g).bfloat16()
    w = (torch.randn(K, C, k, k, generator=g) * 0.05).bfloat16()
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.float().requires_grad_(True)
    yr = F.conv2d(xr, wr, None, st, pd)
    dy = torch.randn(yr.shape, generator=g).bfloat16()
    yr.backward(dy.float())
    _, wt = mc.pack_weight(w.float().to(dev), C, (st, st), (pd, pd), krsc=False, dgrad=True)
    dyn = dy.permute(0, 2, 3, 1).contiguous().to(dev)
    dx = mc.conv_dgrad(dyn, wt, x.shape, k, k, (st, st), (pd, pd))
    ref_dx = xr.grad.permute(0, 2, 3, 1)
    tol = 2e-5 * (dy.abs().amax() * w.abs().amax() * K * k * k).item()
    torch.testing.assert_close(dx.float().cpu(), ref_dx, rtol=1e-2, atol=tol + 1e-2 * ref_dx.abs().amax().item())
    dw = mc.conv_wgrad(dyn, x.to(dev), K, k, k, (st, st), (pd, pd))
    ref_dw = wr.grad
    tolw = 2e-5 * (dy.abs().amax() * x.abs().amax()).item() * dy.numel() / K
    torch.testing.assert_close(dw.cpu(), ref_dw, rtol=0, atol=tolw)


@pytest.mark.parametrize("act", [0, 1])
def test_conv_bn_train_matches_torch(dev, act):
    """ConvBNAct (train-mode BN, residual) vs torch conv -> batch_norm(training) -> add -> relu."""
    from mx_det import conv as mc
    g = torch.Generator().manual_seed(3)
    N, H, W, C, K = 2, 20, 24, 64, 128
    x = torch.randn(N, H, W, C, generator=g).bfloat16()
    w = (torch.randn(K, C, 3, 3, generator=g) * 0.05).bfloat16().float()
    gamma = torch.rand(K, generator=g) + 0.5
    beta = torch.randn(K, generator=g) * 0.1
    res = torch.randn(N, H, W, K, generator=g).bfloat16()
    # torch reference
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr, gr, br = w.clone().requires_grad_(True), gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    rr = res.float().permute(0, 3, 1, 2).requires_grad_(True)
    rm, rv = torch.zeros(K), torch.ones(K)
    # mx
    xd = x.to(dev).requires_grad_(True)
    wd, gd, bd = w.to(dev).requires_grad_(True), gamma.to(dev).requires_grad_(True), beta.to(dev).requires_grad_(True)
    rd = res.to(dev).requires_grad_(True)
    rmd, rvd = torch.zeros(K, device=dev), torch.ones(K, device=dev)
    y = mc.ConvBNAct.apply(xd, wd, gd, bd, rd, rmd, rvd, (1, 1), (1, 1), act, 1e-5, 0.1)
    z = F.conv2d(xr, wr, None, 1, 1)
    yr = F.batch_norm(z, rm, rv, gr, br, training=True, momentum=0.1, eps=1e-5) + rr
    if act:
        # ReLU with the mask of the device output: elements within bf16 rounding of 0 may flip
        # sign between the two paths; the BN-backward math is what is compared here
        yr = yr * (y.detach().float().cpu().permute(0, 3, 1, 2) > 0)
    dy = torch.randn(yr.shape, generator=g).bfloat16().float()
    yr.backward(dy)
    y.backward(dy.permute(0, 2, 3, 1).bfloat16().to(dev))
    torch.testing.assert_close(y.float().cpu(), yr.detach().permute(0, 2, 3, 1), rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(rmd.cpu(), rm, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(rvd.cpu(), rv, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(gd.grad.cpu(), gr.grad, rtol=2e-2, atol=2e-1)
    torch.testing.assert_close(bd.grad.cpu(), br.grad, rtol=2e-2, atol=2e-1)
    torch.testing.assert_close(rd.grad.float().cpu(), rr.grad.permute(0, 2, 3, 1), rtol=2e-2, atol=2e-2)
    rel = lambda a, b: ((a - b).norm() / b.norm()).item()  # noqa: E731
    assert rel(xd.grad.float().cpu(), xr.grad.permute(0, 2, 3, 1)) < 2e-2
    assert rel(wd.grad.cpu(), wr.grad) < 2e-2


@pytest.mark.parametrize("st,k,pd", [(2, 3, 1), (1, 3, 1), (2, 1, 0)])
def test_dgrad_convenience_entry_matches_packed(dev, st, k, pd):
    """mx_conv2d_dgrad (KRSC weight, repacked inside) == the packed hot path, bit for bit."""
    import ctypes
    from mx_det import _lib, conv as mc
    g = torch.Generator().manual_seed(11)
    N, H, W, C, K = 2, 13, 17, 64, 128
    w = (torch.randn(K, C, k, k, generator=g) * 0.05).to(dev)
    Ho, Wo = mc.out_hw(H, W, k, k, (st, st), (pd, pd))
    dy = torch.randn(N, Ho, Wo, K, generator=g).bfloat16().to(dev)
    wk, wt = mc.pack_weight(w, C, (st, st), (pd, pd), dgrad=True)
    ref = mc.conv_dgrad(dy, wt, (N, H, W, C), k, k, (st, st), (pd, pd))
    dx = torch.empty_like(ref)
    sh = _lib.ConvShape(N, H, W, C, K, k, k, Ho, Wo, st, st, pd, pd)
    _lib.call("mx_conv2d_dgrad", ctypes.byref(sh), mc._p(dy), mc._p(wk), mc._p(dx), mc._s())
    torch.cuda.synchronize()
    assert torch.equal(dx, ref)


def test_wgrad_layouts_and_channel_padding(dev):
    """mx_conv2d_wgrad_ex writes KCRS (torch) and KRSC layouts and drops zero-padded channels; the
    convenience mx_conv2d_wgrad (KRSC, all channels) agrees with both."""
    import ctypes
    from mx_det import _lib, conv as mc
    g = torch.Generator().manual_seed(5)
    N, H, W, C, K, k = 2, 21, 19, 16, 40, 3
    x = torch.randn(N, H, W, C, generator=g).bfloat16()
    x[..., 11:] = 0          # channels 11.. are padding
    dy = torch.randn(N, H, W, K, generator=g).bfloat16()
    dy[..., 35:] = 0         # output channels 35.. are padding
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (K, C, k, k),
                                      dy.float().permute(0, 3, 1, 2), 1, 1)
    xd, dyd = x.to(dev), dy.to(dev)
    dw = mc.conv_wgrad(dyd, xd, K, k, k, (1, 1), (1, 1), kout=35, cin=11)
    tol = 2e-5 * (dy.abs().amax() * x.abs().amax()).item() * N * H * W
    torch.testing.assert_close(dw.cpu(), ref[:35, :11], rtol=0, atol=tol)
    sh = _lib.ConvShape(N, H, W, C, K, k, k, H, W, 1, 1, 1, 1)
    wsb = _lib.load().mx_conv_workspace(ctypes.byref(sh), 2)
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
    krsc = torch.empty(35, k, k, 11, device=dev)
    _lib.call("mx_conv2d_wgrad_ex", ctypes.byref(sh), mc._p(dyd), mc._p(xd), mc._p(krsc), 35, 11, 0, mc._p(ws),
              wsb, mc._s())
    full = torch.full((K, k, k, C), float("nan"), device=dev)
    _lib.call("mx_conv2d_wgrad", ctypes.byref(sh), mc._p(dyd), mc._p(xd), mc._p(full), mc._s())
    torch.cuda.synchronize()
    torch.testing.assert_close(krsc.permute(0, 3, 1, 2).cpu(), dw.cpu(), rtol=0, atol=0)
    torch.testing.assert_close(full.permute(0, 3, 1, 2).cpu(), ref, rtol=0, atol=tol)


@pytest.mark.parametrize("target", [64, 512, 4096])
def test_wgrad_split_counts_agree(dev, target):
    """Unsplit (direct store) and split (slab + reduce) wgrad give the same weights."""
    from mx_det import _lib, conv as mc
    g = torch.Generator().manual_seed(9)
    x = torch.randn(2, 30, 40, 64, generator=g).bfloat16().to(dev)
    dy = torch.randn(2, 30, 40, 128, generator=g).bfloat16().to(dev)
    _lib.call("mx_conv_set_wgrad_target", 1)
    ref = mc.conv_wgrad(dy, x, 128, 3, 3, (1, 1), (1, 1))
    _lib.call("mx_conv_set_wgrad_target", target)
    dw = mc.conv_wgrad(dy, x, 128, 3, 3, (1, 1), (1, 1))
    _lib.call("mx_conv_set_wgrad_target", 0)
    torch.testing.assert_close(dw, ref, rtol=1e-5, atol=1e-3)


def test_weight_packer_batched_matches_single_and_tracks_versions(dev):
    """WeightPacker: one batched launch == per-weight pack_weight for every registered conv (strides 1/2,
    padded stem channels, FC6 as a 7x7 view, narrow K); frozen weights are not repacked; an in-place
    update (optimizer step) is picked up by the next refresh."""
    from mx_det import conv as mc
    g = torch.Generator().manual_seed(2)
    specs = [((64, 3, 7, 7), (2, 2), (3, 3), True), ((256, 64, 1, 1), (1, 1), (0, 0), True),
             ((128, 128, 3, 3), (2, 2), (1, 1), True), ((512, 256, 1, 1), (2, 2), (0, 0), False),
             ((15, 256, 1, 1), (1, 1), (0, 0), True)]
    ws = [(torch.randn(*shp, generator=g) * 0.1).to(dev) for shp, _, _, _ in specs]
    fc = (torch.randn(1024, 256 * 49, generator=g) * 0.01).to(dev)
    pk = mc.WeightPacker()
    for w, (_, st, pd, dg) in zip(ws, specs):
        pk.register(w, st, pd, dg)
    fcv = fc.view(1024, 256, 7, 7)
    pk.register(fcv, (1, 1), (0, 0), True, dense=True)
    pk.refresh()
    wk, wt = pk.lookup(fcv, 256, 1024, (1, 1), (0, 0), True, dense=True)
    assert torch.equal(wk, mc.weight_krsc(fcv))
    assert torch.equal(wt.view(-1, 1024), wk.reshape(1024, -1).t())  # [R*S*C][K]: the 1x1-GEMM dgrad operand
    for w, (_, st, pd, dg) in zip(ws, specs):
        K, C = w.shape[:2]
        got = pk.lookup(w, mc._ceil8(C), mc._ceil8(K), st, pd, dg)
        assert got is not None
        ref = mc.pack_weight(w, mc._ceil8(C), st, pd, kpad=mc._ceil8(K), dgrad=dg)
        assert torch.equal(got[0], ref[0])
        if dg:
            assert torch.equal(got[1], ref[1])
    # in-place update of one weight -> stale until refresh, then repacked
    ws[1].add_(1.0)
    assert pk.lookup(ws[1], 64, 256, (1, 1), (0, 0), True) is None
    pk.refresh()
    got = pk.lookup(ws[1], 64, 256, (1, 1), (0, 0), True)
    ref = mc.pack_weight(ws[1], 64, (1, 1), (0, 0), dgrad=True)
    assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])


def test_fc6_dense_conv_matches_linear(dev):
    """FC6 as a valid 7x7 conv over the NHWC RoI tile == torch flatten(NCHW) + Linear + ReLU, forward
    and backward (the dense dgrad runs as a 1x1 GEMM)."""
    from mx_det import conv as mc
    g = torch.Generator().manual_seed(4)
    R, C, K = 96, 256, 1024
    x = torch.randn(R, 7, 7, C, generator=g).bfloat16()
    w = (torch.randn(K, C * 49, generator=g) * 0.01).bfloat16().float()
    b = torch.randn(K, generator=g) * 0.1
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = torch.relu(torch.nn.functional.linear(xr.flatten(1), wr, br))
    dy = torch.randn(yr.shape, generator=g).bfloat16().float()
    yr.backward(dy)
    xd = x.to(dev).requires_grad_(True)
    wd, bd = w.to(dev).requires_grad_(True), b.to(dev).requires_grad_(True)
    y = mc.ConvAct.apply(xd, wd.view(K, C, 7, 7), bd, (1, 1), (0, 0), mc.ACT_RELU, torch.float32)
    y.backward(dy.view(R, 1, 1, K).to(dev))
    torch.testing.assert_close(y.view(R, K).cpu(), yr.detach(), rtol=1e-2, atol=2e-2)
    rel = lambda a, c: ((a - c).norm() / c.norm()).item()  # noqa: E731
    assert rel(xd.grad.float().cpu().permute(0, 3, 1, 2), xr.grad) < 1e-2
    assert rel(wd.grad.cpu(), wr.grad) < 1e-2
    assert rel(bd.grad.cpu(), br.grad) < 1e-3


def test_side_stream_wgrad_matches_in_order(dev, monkeypatch):
    """Weight gradients on the side stream (conv.side_wgrad_enabled) equal the in-order ones bit for
    bit: a chain of single-use convs, a weight shared by two calls (its gradients are summed by
    autograd on the main stream, so it must stay in order), and a second backward that accumulates
    into existing .grad (also in order)."""
    from mx_det import conv as mc
    g = torch.Generator().manual_seed(11)
    N, H, W, C = 2, 40, 48, 64
    x0 = torch.randn(N, H, W, C, generator=g).bfloat16().to(dev)
    ws = [(torch.randn(C, C, 3, 3, generator=g) * 0.05).to(dev) for _ in range(3)]
    shared = (torch.randn(C, C, 3, 3, generator=g) * 0.05).to(dev)
    gam = torch.ones(C, device=dev)
    bet = torch.zeros(C, device=dev)

    def run():
        ps = [w.clone().requires_grad_(True) for w in ws] + [shared.clone().requires_grad_(True)]
        out = []
        for rep in range(2):  # the second pass accumulates into .grad
            y = x0
            for w in ps[:3]:
                y = mc.ConvBNAct.apply(y, w, gam, bet, None, torch.zeros(C, device=dev), torch.ones(C, device=dev),
                                       (1, 1), (1, 1), mc.ACT_RELU, 1e-5, 0.1)
            a = mc.ConvAct.apply(y, ps[3], None, (1, 1), (1, 1), mc.ACT_RELU, torch.bfloat16)
            b = mc.ConvAct.apply(y[:, ::2, ::2].contiguous(), ps[3], None, (1, 1), (1, 1), mc.ACT_RELU, torch.bfloat16)
            (a.float().square().mean() + b.float().mean()).backward()
            out.append([p.grad.clone() for p in ps])
        return out

    monkeypatch.setenv("MX_SIDE_WGRAD", "0")
    ref = run()
    monkeypatch.setenv("MX_SIDE_WGRAD", "1")
    got = run()
    torch.cuda.synchronize()
    for r, o in zip(ref, got):
        for a, b in zip(r, o):
            assert torch.isfinite(b).all()
            assert torch.equal(a, b)


@pytest.mark.parametrize("K,C,k,cp,kp", [(64, 3, 7, 8, 64), (1024, 256, 7, 256, 1024), (35, 256, 1, 256, 40),
                                         (96, 4096, 3, 4096, 96), (16, 24, 5, 24, 16), (130, 66, 3, 72, 136)])
def test_pack_weight_layouts(dev, K, C, k, cp, kp):
    """mx_conv_pack_weight: wk = bf16(w) as [K][R][S][Cpad] (zero channels past C) bit-exact, for
    every tile kind (single-row transposes, channel-split rows when C*R*S exceeds the LDS tile, 7x7
    and 5x5 taps, odd K), and the dense dgrad layout [R][S][Cpad][Kpad] (zero rows past K)."""
    from mx_det import conv as mc
    g = torch.Generator().manual_seed(K + C)
    w = torch.randn(K, C, k, k, generator=g).to(dev)
    wk, _ = mc.pack_weight(w, cin_pad=cp, kpad=kp)
    ref = torch.zeros(K, k, k, cp, dtype=torch.bfloat16, device=dev)
    ref[..., :C] = w.permute(0, 2, 3, 1).bfloat16()
    assert torch.equal(wk, ref)
    if k > 1:
        return
    _, wt = mc.pack_weight(w, cin_pad=cp, kpad=kp, krsc=False, dgrad=True)
    reft = torch.zeros(k, k, cp, kp, dtype=torch.bfloat16, device=dev)
    reft[:, :, :C, :K] = w.permute(2, 3, 1, 0).bfloat16()
    assert torch.equal(wt.view(k, k, cp, kp), reft)


def test_bn_backward_partials_from_dgrad_epilogue(dev, monkeypatch):
    """A bottleneck (no downsample and stride-2 downsample variants) trained one step with the BN
    backward partials produced in the next conv's dgrad epilogue (BNBLink: mx_conv2d_dgrad_bnb +
    mx_bn_bwd_finalize) and with the separate bn_bwd_reduce pass: same gradients up to f32
    summation order (and the bf16 roundings that order can flip)."""
    from mx_det import frcnn
    from mx_det.backend import default_backend
    be = default_backend()
    for inplanes, planes, stride in ((256, 64, 1), (256, 128, 2)):
        torch.manual_seed(0)
        ds = None
        if stride != 1 or inplanes != planes * 4:
            from mx_det.conv import BatchNorm2d, Conv2d
            ds = torch.nn.Sequential(Conv2d(inplanes, planes * 4, 1, stride, bias=False), BatchNorm2d(planes * 4))
        blk = frcnn.Bottleneck(inplanes, planes, stride, ds).to(dev).train()
        x0 = torch.randn(2, 40, 56, inplanes, device=dev).bfloat16()
        gy = None
        res = {}
        for mode in ("0", "1"):
            monkeypatch.setenv("MX_BNB", mode)
            from mx_det import conv as mc
            pk = mc.WeightPacker()
            for m in blk.modules():
                if isinstance(m, mc.Conv2d):
                    pk.register(m.weight, m.stride, m.padding, True)
            mc.set_packer(pk)
            pk.refresh()
            for p in blk.parameters():
                p.grad = None
            x = x0.clone().requires_grad_(True)
            y = blk(x, be)
            if gy is None:
                gy = torch.randn_like(y.float()).bfloat16()
            y.backward(gy)
            res[mode] = (x.grad.float(), {n: p.grad.clone() for n, p in blk.named_parameters()})
            mc.set_packer(None)
        rel = lambda a, b: ((a - b).norm() / b.norm().clamp_min(1e-12)).item()  # noqa: E731
        assert rel(res["1"][0], res["0"][0]) < 2e-3
        for n in res["0"][1]:
            assert rel(res["1"][1][n], res["0"][1][n]) < 2e-3, n


@pytest.mark.parametrize("ci", range(9))
@pytest.mark.parametrize("N,H,W,C,K,k,st,pd", [c for c in CASES if c[4] % 8 == 0])
def test_conv_tuner_candidates(dev, monkeypatch, ci, N, H, W, C, K, k, st, pd):
    """Every launch configuration the per-shape tuner may pick (block tile x split cap for fwd /
    dgrad, kernel variant x block target for wgrad) gives the torch results on every test shape."""
    from mx_det import conv as mc
    monkeypatch.setenv("MX_CONV_TUNE", "1")
    monkeypatch.setattr(mc, "_tune_cache", {})  # single candidates: the tuner must pick exactly them
    monkeypatch.setattr(mc, "_FD_CANDS", (mc._FD_CANDS[ci],))
    monkeypatch.setattr(mc, "_WG_CANDS", (mc._WG_CANDS[ci % len(mc._WG_CANDS)],))
    test_conv_fwd(dev, 7, N, H, W, C, K, k, st, pd)
    test_conv_dgrad_wgrad(dev, 7, N, H, W, C, K, k, st, pd)


@pytest.mark.parametrize("split", [False, True])
def test_sgd_fused_pack_equals_sgd_then_refresh(dev, split, monkeypatch):
    """mx_sgd_pack_step (update + wk/wt written in one pass) == sgd_kernel followed by the packer's
    batched repack, bit for bit: parameters, momentum buffers and every packed layout over 3 steps
    (1x1, 3x3 s1/s2, a 1x1 s2 without dgrad layout, narrow K, odd C, FC6 as a dense 7x7 view, FC7, and
    plain parameters sharing the launch); frozen / unregistered weights untouched."""
    from mx_det import conv as mc, optim
    g = torch.Generator().manual_seed(11)
    specs = [((256, 64, 1, 1), (1, 1), (0, 0), True), ((128, 128, 3, 3), (2, 2), (1, 1), True),
             ((64, 64, 3, 3), (1, 1), (1, 1), True), ((512, 256, 1, 1), (2, 2), (0, 0), False),
             ((15, 256, 1, 1), (1, 1), (0, 0), True), ((32, 3, 3, 3), (1, 1), (1, 1), True)]

    def build():
        gg = torch.Generator().manual_seed(5)
        ws = [torch.nn.Parameter((torch.randn(*shp, generator=gg) * 0.1).to(dev)) for shp, _, _, _ in specs]
        fc6 = torch.nn.Parameter((torch.randn(1024, 256 * 49, generator=gg) * 0.01).to(dev))
        fc7 = torch.nn.Parameter((torch.randn(1024, 1024, generator=gg) * 0.01).to(dev))
        extra = [torch.nn.Parameter(torch.randn(n, generator=gg).to(dev)) for n in (1024, 77, 5)]
        pk = mc.WeightPacker()
        for w, (_, st, pd, dg) in zip(ws, specs):
            pk.register(w, st, pd, dg, split=split)
        pk.register(fc6.view(1024, 256, 7, 7), (1, 1), (0, 0), True, dense=True, split=split)
        pk.register(fc7.view(1024, 1024, 1, 1), (1, 1), (0, 0), True, split=split)
        params = ws + [fc6, fc7] + extra
        return pk, params

    grads = None
    out = []
    for fused in (1, 0):
        monkeypatch.setattr(optim, "_SGD_PACK", fused)
        pk, params = build()
        mc.set_packer(pk)
        pk.refresh()
        opt = optim.SGD(params, lr=0.02, momentum=0.9, weight_decay=5e-4)
        if grads is None:
            grads = [[torch.randn(p.shape, generator=g).to(dev) * 0.1 for p in params] for _ in range(3)]
        for step in range(3):
            for p, gr in zip(params, grads[step]):
                p.grad = gr.clone()
            opt.step()
            if fused:
                assert all(pk.entries[k].version == pk.entries[k].w._version for k in pk.order)
            pk.refresh()  # fused: nothing dirty, no launch
        torch.cuda.synchronize()
        packed = [(pk.entries[k].wk.clone(), None if pk.entries[k].wt is None else pk.entries[k].wt.clone())
                  for k in pk.order]
        out.append(([p.detach().clone() for p in params],
                    [opt.state[p]["momentum_buffer"].clone() for p in params], packed))
        mc.set_packer(None)
    (pa, ba, ka), (pb, bb, kb) = out
    for x, y in zip(pa, pb):
        assert torch.equal(x, y)
    for x, y in zip(ba, bb):
        assert torch.equal(x, y)
    for (wk1, wt1), (wk2, wt2) in zip(ka, kb):
        assert torch.equal(wk1, wk2)
        assert (wt1 is None) == (wt2 is None) and (wt1 is None or torch.equal(wt1, wt2))
