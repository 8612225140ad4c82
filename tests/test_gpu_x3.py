"""GPU numerics of the precision-faithful (f32 activations, bf16x3 MFMA products) path against float64
torch on the same f32 operands, and against TF32-rounded operands as the reference's own precision
(its convs ran TF32 on Ampere: cudnn.allow_tf32 default, train_frcnn_baseline.py:139-176).

Bar: every conv output's error vs f64 is at least 10x below the error of the same conv computed
from TF32-rounded operands (10-bit mantissa, round-to-nearest-even), and below 1e-4 relative L2.
Elementwise kernels (BN, pool, upsample, act/bias backward) on f32 storage are checked at f32
rounding level (1e-5) or exactly.
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
    (2, 64, 80, 256, 256, 3, 1, 1),    # 128x128 tiles, no split
]

# configs[1]'s exact shapes (1333x800 padded to 1344x800, bs=2): the P2-level 3x3 (FPN output block
# and RPN head convs, 2x200x336x256), layer3 / layer4 3x3 and 1x1 convs, the layer4 downsample and the
# P5 lateral -- the launches the tuner maps to the 128x128 / 64x128 tiles and split-K in the bench
HEADLINE = [
    (2, 200, 336, 256, 256, 3, 1, 1),
    (2, 50, 84, 256, 256, 3, 1, 1),
    (2, 25, 42, 512, 512, 3, 1, 1),
    (2, 50, 84, 1024, 256, 1, 1, 0),
    (2, 50, 84, 1024, 2048, 1, 2, 0),
    (2, 25, 42, 2048, 256, 1, 1, 0),
]


def tf32(t):
    """Round f32 to TF32 (10 explicit mantissa bits, RNE): the operand precision of the reference's
    Ampere convs."""
    i = t.float().contiguous().view(torch.int32).to(torch.int64)
    r = ((i + 0xFFF + ((i >> 13) & 1)) >> 13) << 13
    return (((r + 2 ** 31) % 2 ** 32) - 2 ** 31).to(torch.int32).view(torch.float32)


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def _check(got, ref64, tf32_ref):
    e = rel(got, ref64)
    et = rel(tf32_ref, ref64)
    assert e < 1e-4, e
    assert e * 10 < et or e < 1e-6, (e, et)
    return e, et


def test_tf32_rounding_helper():
    x = torch.tensor([1.0, 1.0 + 2 ** -10, 1.0 + 2 ** -11, 1.0 + 3 * 2 ** -11, -3.3, 0.0])
    t = tf32(x)
    assert t[0] == 1.0 and t[1] == 1.0 + 2 ** -10 and t[2] == 1.0 and t[3] == 1.0 + 2 ** -9
    assert abs(t[4] + 3.3) < 3.3 * 2 ** -11 and t[5] == 0


def test_split_pack_planes(dev):
    """mx_conv_pack_weight split mode: plane 0 = bf16(w) (RNE), plane 1 = bf16(w - hi); hi + lo
    reconstructs w to 2^-16 relative; the KRSC / dgrad layouts match the unsplit pack plane by plane."""
    from mx_det import conv as mc
    g = torch.Generator().manual_seed(0)
    w = torch.randn(96, 40, 3, 3, generator=g)
    wk, wt = mc.pack_weight(w.to(dev), 40, (2, 2), (1, 1), kpad=96, dgrad=True, split=True)
    wk1, wt1 = mc.pack_weight(w.to(dev), 40, (2, 2), (1, 1), kpad=96, dgrad=True)
    assert torch.equal(wk[0], wk1) and torch.equal(wt[:wt1.numel()], wt1)
    hi = wk[0].float().cpu()
    lo = wk[1].float().cpu()
    ref = w.permute(0, 2, 3, 1)
    assert torch.equal(hi, ref.bfloat16().float())
    assert torch.equal(lo, (ref - hi).bfloat16().float())
    assert ((hi + lo - ref).abs() <= ref.abs() * 2 ** -16).all()


@pytest.mark.parametrize("N,H,W,C,K,k,st,pd", CASES + HEADLINE)
def test_x3_fwd(dev, N, H, W, C, K, k, st, pd):
    from mx_det import conv as mc
    g = torch.Generator().manual_seed(N * 1000 + C + K)
    x = torch.randn(N, H, W, C, generator=g)
    w = torch.randn(K, C, k, k, generator=g) * 0.05
    b = torch.randn(K, generator=g)
    xn = x.permute(0, 3, 1, 2)
    ref = F.conv2d(xn.double(), w.double(), b.double(), st, pd).permute(0, 2, 3, 1)
    reft = F.conv2d(tf32(xn).double(), tf32(w).double(), b.double(), st, pd).permute(0, 2, 3, 1)
    wk, _ = mc.pack_weight(w.to(dev), C, (st, st), (pd, pd), split=True)
    y, stats = mc.conv_fwd(x.to(dev), wk, (st, st), (pd, pd), bias=b.to(dev), stats=True)
    assert y.dtype == torch.float32
    _check(y, ref, reft)
    # BN statistics partials are over the pre-bias accumulators
    z = (ref - b.double()).reshape(-1, K)
    s = stats.cpu().double().sum(1)
    # (each z carries ~1e-5 relative error: the sums are held to 1e-5 of the sum of magnitudes)
    torch.testing.assert_close(s[0], z.sum(0), rtol=0, atol=1e-5 * z.abs().sum(0).max().item())
    torch.testing.assert_close(s[1], (z * z).sum(0), rtol=0, atol=1e-5 * (z * z).sum(0).max().item())


@pytest.mark.parametrize("N,H,W,cin,st,pd,act", [
    (2, 33, 41, 3, 2, 3, 1),     # odd sizes: a pixel tail below one 64-pixel statistics row
    (1, 64, 96, 3, 2, 3, 0),
    (2, 120, 200, 3, 2, 3, 1),   # several tiles per block
    (1, 23, 19, 4, 1, 2, 1),     # 4 real channels, stride 1, pad 2
    (2, 64, 128, 3, 2, 3, 1),    # Ho % 4 == 0, Wo % 16 == 0: 4 x 16 patch tiles
    (2, 800, 1344, 3, 2, 3, 1),  # the headline stem: configs[1]'s padded 2 x 800 x 1344 batch -> 400 x 672
])
def test_x3_stem_kernel(dev, N, H, W, cin, st, pd, act, monkeypatch):
    """mx_conv2d_stem_x3 (the 7x7 -> 64 ResNet stem, one MFMA K-step per filter row) against float64
    torch with the x3 bar, its BN statistics partials against the f64 sums, and against the generic
    x3 kernels (MX_STEM_KERNEL=0) on the same packed operands."""
    from mx_det import conv as mc
    g = torch.Generator().manual_seed(N * 100 + H)
    x = torch.zeros(N, H, W, 8)
    x[..., :cin] = torch.randn(N, H, W, cin, generator=g)
    w = torch.randn(64, cin, 7, 7, generator=g) * 0.05
    b = torch.randn(64, generator=g)
    xn = x[..., :cin].permute(0, 3, 1, 2)
    ref = F.conv2d(xn.double(), w.double(), b.double(), st, pd).permute(0, 2, 3, 1)
    reft = F.conv2d(tf32(xn).double(), tf32(w).double(), b.double(), st, pd).permute(0, 2, 3, 1)
    z = (ref - b.double()).reshape(-1, 64)
    if act:
        ref, reft = ref.clamp_min(0), reft.clamp_min(0)
    wk, _ = mc.pack_weight(w.to(dev), 8, (st, st), (pd, pd), split=True)
    xd = x.to(dev)
    monkeypatch.setenv("MX_STEM_KERNEL", "1")
    y, stats = mc.conv_fwd(xd, wk, (st, st), (pd, pd), bias=b.to(dev), act=act, stats=True, cin=cin)
    _check(y, ref, reft)
    s = stats.cpu().double().sum(1)
    torch.testing.assert_close(s[0], z.sum(0), rtol=0, atol=1e-5 * z.abs().sum(0).max().item())
    torch.testing.assert_close(s[1], (z * z).sum(0), rtol=0, atol=1e-5 * (z * z).sum(0).max().item())
    monkeypatch.setenv("MX_STEM_KERNEL", "0")
    y0 = mc.conv_fwd(xd, wk, (st, st), (pd, pd), bias=b.to(dev), act=act, cin=cin)
    assert rel(y, y0) < 1e-6


def test_stem_fused_bn_pool_matches_unfused(dev):
    """The frozen stem's conv -> train BN -> relu -> maxpool with the BN apply inside the pool
    (conv_bn_act_maxpool) returns bit-identically what conv_bn + maxpool return, and updates the
    running statistics identically."""
    import copy
    from mx_det import conv as mc
    from mx_det.backend import _MaxPool
    torch.manual_seed(3)
    conv = mc.Conv2d(3, 64, 7, 2, 3, bias=False).to(dev)
    bn = mc.BatchNorm2d(64).to(dev)
    with torch.no_grad():
        conv.weight.normal_(0, 0.05)
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    for p in list(conv.parameters()) + list(bn.parameters()):
        p.requires_grad_(False)
    bn2 = copy.deepcopy(bn)
    x = torch.zeros(2, 70, 90, 8, device=dev)
    x[..., :3] = torch.randn(2, 70, 90, 3, device=dev)
    y1 = mc.conv_bn_act_maxpool(x, conv, bn, mc.ACT_RELU, 3, 2, 1)
    y2 = _MaxPool.apply(mc.conv_bn(x, conv, bn2, mc.ACT_RELU), 3, 2, 1)
    assert y1.shape == y2.shape == (2, 18, 23, 64)
    assert torch.equal(y1, y2)
    assert torch.equal(bn.running_mean, bn2.running_mean) and torch.equal(bn.running_var, bn2.running_var)
    assert int(bn.num_batches_tracked) == int(bn2.num_batches_tracked) == 1


def test_x3_fwd_residual_leaky(dev):
    from mx_det import conv as mc
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, 16, 16, 64, generator=g)
    w = torch.randn(64, 64, 3, 3, generator=g) * 0.05
    r = torch.randn(2, 16, 16, 64, generator=g)
    ref = F.leaky_relu(F.conv2d(x.double().permute(0, 3, 1, 2), w.double(), None, 1, 1).permute(0, 2, 3, 1)
                       + r.double(), 0.2)
    wk, _ = mc.pack_weight(w.to(dev), 64, (1, 1), (1, 1), split=True)
    y = mc.conv_fwd(x.to(dev), wk, (1, 1), (1, 1), residual=r.to(dev), act=mc.ACT_LEAKY)
    assert rel(y, ref) < 1e-5


@pytest.mark.timeout(300)
@pytest.mark.parametrize("N,H,W,C,K,k,st,pd", [c for c in CASES + HEADLINE if c[4] % 8 == 0])
def test_x3_dgrad_wgrad(dev, N, H, W, C, K, k, st, pd):
    from mx_det import conv as mc
    g = torch.Generator().manual_seed(7 + C + K)
    x = torch.randn(N, H, W, C, generator=g)
    w = torch.randn(K, C, k, k, generator=g) * 0.05
    xr = x.double().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.double().requires_grad_(True)
    yr = F.conv2d(xr, wr, None, st, pd)
    dy = torch.randn(yr.shape, generator=g)
    yr.backward(dy.double())
    xt = tf32(x.permute(0, 3, 1, 2)).double().requires_grad_(True)
    wt_ = tf32(w).double().requires_grad_(True)
    F.conv2d(xt, wt_, None, st, pd).backward(tf32(dy).double())
    _, wt = mc.pack_weight(w.to(dev), C, (st, st), (pd, pd), krsc=False, dgrad=True, split=True)
    dyn = dy.permute(0, 2, 3, 1).contiguous().to(dev)
    dx = mc.conv_dgrad(dyn, wt, x.shape, k, k, (st, st), (pd, pd))
    assert dx.dtype == torch.float32
    _check(dx, xr.grad.permute(0, 2, 3, 1), xt.grad.permute(0, 2, 3, 1))
    dw = mc.conv_wgrad(dyn, x.to(dev), K, k, k, (st, st), (pd, pd))
    _check(dw, wr.grad, wt_.grad)


@pytest.mark.parametrize("tile", [(0, 0), (256, 128), (64, 64)])
def test_x3_dgrad_residual_and_bn_partials(dev, tile, monkeypatch):
    """dgrad epilogue extras on f32: + residual (bottleneck identity gradient) and the BN-backward
    column partials of g = dx * act'(y), g * (z - mean) * invstd per 64-row block; auto and forced
    block tiles (the 256-row tile stages its 8-wave epilogue one wave-row at a time)."""
    from mx_det._lib import call
    monkeypatch.setenv("MX_CONV_TUNE", "0")  # the forced tile, not the tuner's pick
    call("mx_conv_set_tile", *tile)
    try:
        _dgrad_residual_and_bn_partials(dev)
    finally:
        call("mx_conv_set_tile", 0, 0)


def _dgrad_residual_and_bn_partials(dev):
    from mx_det import conv as mc
    g = torch.Generator().manual_seed(3)
    N, H, W, C, K = 2, 20, 24, 64, 128
    w = torch.randn(K, C, 3, 3, generator=g) * 0.05
    dy = torch.randn(N, H, W, K, generator=g)
    res = torch.randn(N, H, W, C, generator=g)
    z = torch.randn(N, H, W, C, generator=g) * 2 + 0.3
    mean = z.reshape(-1, C).mean(0)
    invstd = 1.0 / torch.sqrt(z.reshape(-1, C).var(0, unbiased=False) + 1e-5)
    y = F.relu(z * 0.7 + 0.1)
    _, wt = mc.pack_weight(w.to(dev), C, (1, 1), (1, 1), krsc=False, dgrad=True, split=True)
    link = mc.BNBLink()
    link.y, link.z, link.mean, link.invstd, link.act = y.to(dev), z.to(dev), mean.to(dev), invstd.to(dev), 1
    dx = mc.conv_dgrad(dy.to(dev), wt, (N, H, W, C), 3, 3, (1, 1), (1, 1), residual=res.to(dev), bnb=link)
    ref = F.conv_transpose2d(dy.double().permute(0, 3, 1, 2), w.double(), None, 1, 1).permute(0, 2, 3, 1) + res.double()
    assert rel(dx, ref) < 1e-5
    gg = dx.double().cpu().reshape(-1, C) * (y.reshape(-1, C) > 0).double()
    xh = (z.reshape(-1, C).double() - mean.double()) * invstd.double()
    part = link.part.double().cpu()
    mb = part.shape[1]
    rows = torch.arange(gg.shape[0]) // 64
    s0 = torch.zeros(mb, C, dtype=torch.float64).index_add_(0, rows, gg)
    s1 = torch.zeros(mb, C, dtype=torch.float64).index_add_(0, rows, gg * xh)
    torch.testing.assert_close(part[0], s0, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(part[1], s1, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("act,res", [(0, False), (1, True), (1, False)])
def test_x3_conv_bn_train_matches_torch(dev, act, res):
    """ConvBNAct on f32 (train-mode BN, residual): forward and input/weight/affine gradients vs torch
    f64 conv -> batch_norm(training) -> add -> relu."""
    from mx_det import conv as mc
    g = torch.Generator().manual_seed(11 + act)
    N, H, W, C, K = 2, 18, 26, 64, 128
    x = torch.randn(N, H, W, C, generator=g)
    r = torch.randn(N, H, W, K, generator=g) if res else None
    conv = mc.Conv2d(C, K, 3, 1, 1, bias=False)
    bn = mc.BatchNorm2d(K)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(K, C, 3, 3, generator=g) * 0.05)
        bn.weight.copy_(torch.rand(K, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(K, generator=g) * 0.1)
    xr = x.double().permute(0, 3, 1, 2).requires_grad_(True)
    wr = conv.weight.detach().double().requires_grad_(True)
    gr = bn.weight.detach().double().requires_grad_(True)
    br = bn.bias.detach().double().requires_grad_(True)
    zr = F.batch_norm(F.conv2d(xr, wr, None, 1, 1), None, None, gr, br, training=True, eps=1e-5)
    if res:
        zr = zr + r.double().permute(0, 3, 1, 2)
    conv, bn = conv.to(dev), bn.to(dev).train()
    xd = x.to(dev).requires_grad_(True)
    y = mc.ConvBNAct.apply(xd, conv.weight, bn.weight, bn.bias, r.to(dev) if res else None, bn.running_mean,
                           bn.running_var, (1, 1), (1, 1), act, 1e-5, 0.1)
    assert rel(y, F.relu(zr).permute(0, 2, 3, 1) if act else zr.permute(0, 2, 3, 1)) < 1e-5
    # the backward's activation mask is the one of the device output (a pre-activation within float
    # noise of 0 may fall on either side: one flipped element moves dx by ~1e-3 relative)
    yr = zr * (y.detach().cpu() > 0).double().permute(0, 3, 1, 2) if act else zr
    dy = torch.randn(yr.shape, generator=g)
    yr.backward(dy.double())
    y.backward(dy.permute(0, 2, 3, 1).contiguous().to(dev))
    assert rel(xd.grad, xr.grad.permute(0, 2, 3, 1)) < 1e-4
    assert rel(conv.weight.grad, wr.grad) < 1e-4
    assert rel(bn.weight.grad, gr.grad) < 1e-4
    assert rel(bn.bias.grad, br.grad) < 1e-5


def test_x3_pool_upsample_exact(dev):
    from mx_det.backend import HipBackend
    be = HipBackend("f32")
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 33, 41, 16, generator=g)
    xd = x.to(dev).requires_grad_(True)
    y = be.maxpool(xd, 3, 2, 1)
    xr = x.permute(0, 3, 1, 2).clone().requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    assert torch.equal(y.cpu(), yr.permute(0, 2, 3, 1))
    gy = torch.randn(yr.shape, generator=g)
    yr.backward(gy)
    y.backward(gy.permute(0, 2, 3, 1).contiguous().to(dev))
    torch.testing.assert_close(xd.grad.cpu(), xr.grad.permute(0, 2, 3, 1), rtol=1e-6, atol=1e-6)
    a = torch.randn(2, 25, 42, 16, generator=g)
    s = torch.randn(2, 13, 21, 16, generator=g)
    sd = s.to(dev).requires_grad_(True)
    u = be.upsample_add(sd, a.to(dev), (25, 42))
    ur = F.interpolate(s.permute(0, 3, 1, 2).clone().requires_grad_(True), size=(25, 42), mode="nearest")
    assert torch.equal(u.cpu(), ur.permute(0, 2, 3, 1) + a)
    gu = torch.randn(2, 25, 42, 16, generator=g)
    u.backward(gu.to(dev))
    sr = s.permute(0, 3, 1, 2).clone().requires_grad_(True)
    F.interpolate(sr, size=(25, 42), mode="nearest").backward(gu.permute(0, 3, 1, 2))
    torch.testing.assert_close(sd.grad.cpu(), sr.grad.permute(0, 2, 3, 1), rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("M,K,act", [(134400, 15, 0), (1024, 1024, 1), (77, 24, 2)])
def test_x3_act_bias_bwd_f32(dev, M, K, act):
    from mx_det import conv as mc
    g = torch.Generator().manual_seed(M + K)
    gy = torch.randn(M, K, generator=g)
    y = torch.randn(M, K, generator=g)
    K8 = (K + 7) // 8 * 8
    out, db = mc.act_bias_bwd(gy.to(dev), y.to(dev), act, K8, True, g_dtype=torch.float32)
    mask = (y > 0).float() if act == 1 else torch.where(y > 0, 1.0, 0.2) if act == 2 else torch.ones_like(y)
    ref = gy * mask
    assert out.dtype == torch.float32 and torch.equal(out[:, :K].cpu(), ref)
    assert (out[:, K:] == 0).all()
    torch.testing.assert_close(db.cpu(), ref.double().sum(0).float(), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("ci", range(13))  # every entry of conv._FD_CANDS_X3
@pytest.mark.parametrize("case", [CASES[i] for i in (0, 1, 3, 7, 8, 9)])
def test_x3_tuner_candidates(dev, monkeypatch, ci, case):
    """Every launch configuration the per-shape tuner may pick for the bf16x3 kernels (block tile x
    split cap for fwd / dgrad, block target for wgrad) meets the same bar."""
    from mx_det import conv as mc
    monkeypatch.setenv("MX_CONV_TUNE", "1")
    monkeypatch.setattr(mc, "_tune_cache", {})
    monkeypatch.setattr(mc, "_FD_CANDS_X3", (mc._FD_CANDS_X3[ci],))
    monkeypatch.setattr(mc, "_WG_CANDS_X3", (mc._WG_CANDS_X3[ci % len(mc._WG_CANDS_X3)],))
    test_x3_fwd(dev, *case)
    if case[4] % 8 == 0:
        test_x3_dgrad_wgrad(dev, *case)


def test_x3_bottleneck_bn_partials_from_dgrad_epilogue(dev, monkeypatch):
    """f32 bottleneck blocks (identity and stride-2 downsample) trained one step with the BN-backward
    partials from the next conv's dgrad epilogue (BNBLink) and with the separate reduce pass: the same
    gradients up to f32 summation order."""
    from mx_det import conv as mc
    from mx_det import frcnn
    from mx_det.backend import HipBackend
    be = HipBackend("f32")
    for inplanes, planes, stride in ((256, 64, 1), (256, 128, 2)):
        torch.manual_seed(0)
        ds = None
        if stride != 1 or inplanes != planes * 4:
            ds = torch.nn.Sequential(mc.Conv2d(inplanes, planes * 4, 1, stride, bias=False), mc.BatchNorm2d(planes * 4))
        blk = frcnn.Bottleneck(inplanes, planes, stride, ds).to(dev).train()
        x0 = torch.randn(2, 40, 56, inplanes, device=dev)
        gy = None
        res = {}
        for mode in ("0", "1"):
            monkeypatch.setenv("MX_BNB", mode)
            pk = mc.WeightPacker()
            for m in blk.modules():
                if isinstance(m, mc.Conv2d):
                    pk.register(m.weight, m.stride, m.padding, True, split=True)
            mc.set_packer(pk)
            pk.refresh()
            for p in blk.parameters():
                p.grad = None
            x = x0.clone().requires_grad_(True)
            y = blk(x, be)
            if gy is None:
                gy = torch.randn_like(y)
            y.backward(gy)
            res[mode] = (x.grad.clone(), {n: p.grad.clone() for n, p in blk.named_parameters()})
            mc.set_packer(None)
        assert rel(res["1"][0], res["0"][0]) < 1e-5
        for n in res["0"][1]:
            assert rel(res["1"][1][n], res["0"][1][n]) < 1e-4, n


@pytest.mark.parametrize("variant", [4, 5, 6, 7])
@pytest.mark.parametrize("case", [CASES[i] for i in (0, 2, 4, 7, 8, 9, 11)])
def test_x3_wgrad_wide_tiles(dev, monkeypatch, variant, case):
    """The wgrad kernel variants forced for every shape (4: 128 x 256 at 8 waves; 5: 256 x 256 at one
    wave per SIMD, accumulators in AGPRs; 6: the 128 x 128 kernel with the interleaved schedule and
    unconditional loads / stores; 7: the 128 x 128 kernel fed by LDS-DMA from pre-split hi / lo
    planes): K / column counts below or not a multiple of the tile, split and
    unsplit pixel axes, strided gathers -- the same bar as the default kernel."""
    from mx_det._lib import call
    monkeypatch.setenv("MX_CONV_TUNE", "0")
    call("mx_conv_set_wgrad_variant", variant)
    try:
        test_x3_dgrad_wgrad(dev, *case)
    finally:
        call("mx_conv_set_wgrad_variant", 3)


@pytest.mark.parametrize("k,st,pd,tile", [(1, 2, 0, (0, 0)), (3, 2, 1, (0, 0)), (3, 2, 1, (64, 64)), (1, 2, 0, (64, 64))])
def test_x3_dgrad_residual_stride2(dev, k, st, pd, tile, monkeypatch):
    """Stride-2 dgrad with a residual (conv.GradChain: a stage output's gradient accumulated through
    the next stage's downsample): every parity class adds the residual at the pixels it writes, the
    tap-less classes of a 1x1 stride-2 conv write it alone -- equal to dgrad + residual."""
    from mx_det._lib import call
    from mx_det import conv as mc
    monkeypatch.setenv("MX_CONV_TUNE", "0")
    call("mx_conv_set_tile", *tile)
    try:
        g = torch.Generator().manual_seed(11 + k)
        N, H, W, C, K = 2, 21, 26, 64, 128
        w = torch.randn(K, C, k, k, generator=g) * 0.05
        Ho, Wo = (H + 2 * pd - k) // st + 1, (W + 2 * pd - k) // st + 1
        dy = torch.randn(N, Ho, Wo, K, generator=g).to(dev)
        res = torch.randn(N, H, W, C, generator=g).to(dev)
        _, wt = mc.pack_weight(w.to(dev), C, (st, st), (pd, pd), krsc=False, dgrad=True, split=True)
        a = mc.conv_dgrad(dy, wt, (N, H, W, C), k, k, (st, st), (pd, pd), residual=res)
        b = mc.conv_dgrad(dy, wt, (N, H, W, C), k, k, (st, st), (pd, pd)) + res
        torch.testing.assert_close(a, b, rtol=0, atol=0)
    finally:
        call("mx_conv_set_tile", 0, 0)


@pytest.mark.parametrize("case", [CASES[i] for i in (0, 1, 2, 4, 7, 8, 9, 11)] + [HEADLINE[0], HEADLINE[1]])
def test_x3_wgrad_presplit_is_bitwise_default(dev, monkeypatch, case):
    """The LDS-DMA wgrad on pre-split operand planes (variant 7) makes the same hi / lo values
    (split_planes_kernel = the staging kernel's split8), the same fragments and the same MFMA order as
    the register-staged kernel (3): dW is bitwise equal, split pixel axes and strided gathers included."""
    from mx_det import conv as mc
    from mx_det._lib import call
    monkeypatch.setenv("MX_CONV_TUNE", "0")
    N, H, W, C, K, k, st, pd = case
    g = torch.Generator().manual_seed(3 + C + K)
    x = torch.randn(N, H, W, C, generator=g).to(dev)
    Ho, Wo = mc.out_hw(H, W, k, k, (st, st), (pd, pd))
    dy = torch.randn(N, Ho, Wo, K, generator=g).to(dev)
    out = {}
    for v in (3, 7):
        call("mx_conv_set_wgrad_variant", v)
        try:
            out[v] = mc.conv_wgrad(dy, x, K, k, k, (st, st), (pd, pd))
            torch.cuda.synchronize()
        finally:
            call("mx_conv_set_wgrad_variant", 3)
    assert torch.equal(out[3], out[7])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape,with_add", [((2, 100, 168, 256, 200, 336), False), ((2, 13, 21, 256, 25, 42), True),
                                            ((1, 7, 5, 64, 100, 77), True)])
def test_upsample_rows_kernel_matches_torch(dev, dtype, shape, with_add):
    """The row-grid upsample kernel (FPN top-down, configs[1]'s P3 -> P2 shape): F.interpolate(nearest)
    (+ add) bit for bit, any scale."""
    from mx_det.backend import HipBackend
    be = HipBackend("f32" if dtype == torch.float32 else "bf16")
    N, H, W, C, Ho, Wo = shape
    g = torch.Generator().manual_seed(H + Wo)
    s = torch.randn(N, H, W, C, generator=g).to(dtype)
    a = torch.randn(N, Ho, Wo, C, generator=g).to(dtype) if with_add else None
    u = be.upsample_add(s.to(dev), a.to(dev) if a is not None else None, (Ho, Wo))
    ur = F.interpolate(s.float().permute(0, 3, 1, 2), size=(Ho, Wo), mode="nearest").permute(0, 2, 3, 1)
    if a is not None:
        ur = ur + a.float()
    assert torch.equal(u.cpu(), ur.to(dtype))
