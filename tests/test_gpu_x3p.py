"""Pre-split operands (x3p): an f32 conv operand split once into bf16 hi / lo planes (mx_split_planes,
the split the bf16x3 kernels otherwise make in registers) and read by LDS-DMA. The fwd / dgrad / wgrad
x3p entries must be bitwise equal to their x3 forms (same hi / lo values, same fragments, same MFMA
order, same epilogues), on the headline P2 shape, strided and split-K shapes and the forced tile
variants; a whole train step with planes on is bitwise equal to the step with planes off."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [  # N, H, W, C, K, k, stride, pad (test_gpu_x3.py's shapes with C, K % 32 == 0)
    (2, 17, 23, 64, 128, 3, 1, 1), (2, 20, 34, 128, 128, 3, 2, 1), (1, 25, 42, 256, 512, 1, 2, 0),
    (2, 7, 7, 256, 256, 3, 1, 1), (2, 25, 42, 1024, 256, 1, 1, 0), (2, 13, 21, 512, 512, 3, 1, 1),
    (1, 15, 19, 64, 64, 3, 2, 1), (2, 16, 22, 64, 256, 1, 2, 0), (2, 64, 80, 256, 256, 3, 1, 1),
    # configs[1]'s P2 3x3, layer3 / layer4 3x3, layer3 1x1, layer4 downsample, P5 lateral
    (2, 200, 336, 256, 256, 3, 1, 1), (2, 50, 84, 256, 256, 3, 1, 1), (2, 25, 42, 512, 512, 3, 1, 1),
    (2, 50, 84, 1024, 256, 1, 1, 0), (2, 50, 84, 1024, 2048, 1, 2, 0), (2, 25, 42, 2048, 256, 1, 1, 0),
]


def test_split_planes_is_the_register_split(dev):
    from mx_det import conv as mc
    x = torch.randn(3, 5, 7, 64, device=dev) * torch.logspace(-30, 30, 64, device=dev)
    x[0, 0, 0, :4] = torch.tensor([0.0, -0.0, 1.5, -3.0e38])
    pl = mc.split_planes(x)
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    assert torch.equal(pl[0].view(torch.int16), hi.view(torch.int16))
    assert torch.equal(pl[1].view(torch.int16), lo.view(torch.int16))


@pytest.mark.parametrize("tile", [(0, 0), (64, 64), (256, 128)])
@pytest.mark.parametrize("case", SHAPES)
def test_x3p_fwd_dgrad_wgrad_bitwise(dev, monkeypatch, case, tile):
    from mx_det import conv as mc
    from mx_det._lib import call
    monkeypatch.setenv("MX_CONV_TUNE", "0")
    N, H, W, C, K, k, st, pd = case
    g = torch.Generator().manual_seed(5 + C + K + k)
    x = torch.randn(N, H, W, C, generator=g).to(dev)
    w = (torch.randn(K, C, k, k, generator=g) * 0.05).to(dev)
    b = torch.randn(K, generator=g).to(dev)
    Ho, Wo = mc.out_hw(H, W, k, k, (st, st), (pd, pd))
    dy = torch.randn(N, Ho, Wo, K, generator=g).to(dev)
    res = torch.randn(N, H, W, C, generator=g).to(dev)
    wk, wt = mc.pack_weight(w, C, (st, st), (pd, pd), dgrad=True, split=True)
    xp, dyp = mc.split_planes(x), mc.split_planes(dy)
    call("mx_conv_set_tile", *tile)
    try:
        y0, s0 = mc.conv_fwd(x, wk, (st, st), (pd, pd), bias=b, act=1, stats=True)
        y1, s1 = mc.conv_fwd(x, wk, (st, st), (pd, pd), bias=b, act=1, stats=True, xp=xp)
        d0 = mc.conv_dgrad(dy, wt, x.shape, k, k, (st, st), (pd, pd), residual=res)
        d1 = mc.conv_dgrad(dy, wt, x.shape, k, k, (st, st), (pd, pd), residual=res, dyp=dyp)
    finally:
        call("mx_conv_set_tile", 0, 0)
    w0 = mc.conv_wgrad(dy, x, K, k, k, (st, st), (pd, pd))
    w1 = mc.wgrad_launch(mc.wgrad_prepare(dy, x, K, k, k, (st, st), (pd, pd), dyp=dyp, xp=xp))
    torch.cuda.synchronize()
    assert torch.equal(y0, y1) and torch.equal(s0, s1)
    assert torch.equal(d0, d1)
    assert torch.equal(w0, w1)


def test_x3p_dgrad_bn_partials_bitwise(dev, monkeypatch):
    """The dgrad epilogue's BN-backward partials (BNBLink) with dy as planes."""
    from mx_det import conv as mc
    monkeypatch.setenv("MX_CONV_TUNE", "0")
    N, H, W, C, K = 2, 40, 56, 128, 128
    g = torch.Generator().manual_seed(9)
    w = (torch.randn(K, C, 3, 3, generator=g) * 0.05).to(dev)
    dy = torch.randn(N, H, W, K, generator=g).to(dev)
    z = (torch.randn(N, H, W, C, generator=g) * 2 + 0.3).to(dev)
    mean = z.reshape(-1, C).mean(0)
    invstd = 1.0 / torch.sqrt(z.reshape(-1, C).var(0, unbiased=False) + 1e-5)
    y = torch.relu(z * 0.7 + 0.1)
    _, wt = mc.pack_weight(w, C, (1, 1), (1, 1), dgrad=True, split=True)
    out = []
    for dyp in (None, mc.split_planes(dy)):
        link = mc.BNBLink()
        link.y, link.z, link.mean, link.invstd, link.act = y, z, mean, invstd, 1
        dx = mc.conv_dgrad(dy, wt, (N, H, W, C), 3, 3, (1, 1), (1, 1), bnb=link, dyp=dyp)
        out.append((dx, link.part))
    torch.cuda.synchronize()
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])


@pytest.mark.timeout(300)
def test_train_step_with_planes_is_bitwise(dev, monkeypatch):
    """Three eager f32 train steps (MX_GRAPHS=0, tuner off: the same launch settings both ways) with
    the pre-split planes on (thresholds lowered so most convs use them) and off: equal losses and
    gradients, bit for bit."""
    from mx_det import frcnn
    from mx_det.data import synth_batch
    monkeypatch.setenv("MX_GRAPHS", "0")
    monkeypatch.setenv("MX_CONV_TUNE", "0")
    imgs, tg = synth_batch(23, 6, H=448, W=640, device=dev)
    res = {}
    for planes in ("0", "1"):
        monkeypatch.setenv("MX_X3_PLANES", planes)
        monkeypatch.setenv("MX_X3_PLANES_MIN", "0")
        monkeypatch.setenv("MX_X3_PLANES_KRS", "0")
        torch.manual_seed(0)
        m = frcnn.fasterrcnn_resnet50_fpn_v2(weights=None)
        m.roi_heads.box_predictor = frcnn.FastRCNNPredictor(1024, 7)
        frcnn.set_trainable_layers(m.backbone.body, 3)
        m = m.to(dev).train()
        out = []
        for step in range(3):
            torch.cuda.manual_seed(300 + step)
            losses = m(imgs[2 * step:2 * step + 2], tg[2 * step:2 * step + 2])
            for p in m.parameters():
                p.grad = None
            sum(losses.values()).backward()
            out.append(([float(v) for v in losses.values()],
                        [p.grad.clone() for p in m.parameters() if p.requires_grad and p.grad is not None]))
        torch.cuda.synchronize()
        res[planes] = out
    for (la, ga), (lb, gb) in zip(res["0"], res["1"]):
        assert la == lb, (la, lb)
        assert len(ga) == len(gb) and all(torch.equal(a, b) for a, b in zip(ga, gb))


@pytest.mark.parametrize("act", [0, 1])
def test_bn_apply_and_bwd_apply_planes(dev, act):
    """mx_bn_apply_p / mx_bn_bwd_apply_p: the same y / dx as the plain entries, and planes equal to
    split_planes of them."""
    from mx_det import conv as mc
    from mx_det._lib import call
    M, K = 3000, 96
    g = torch.Generator().manual_seed(1)
    z, res, gy = (torch.randn(M, K, generator=g).to(dev) for _ in range(3))
    scale, shift = (torch.randn(K, generator=g).to(dev) for _ in range(2))
    coef = torch.randn(3, K, generator=g).to(dev)
    y0, y1 = torch.empty_like(z), torch.empty_like(z)
    yp = torch.empty((2, M, K), dtype=torch.bfloat16, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    call("mx_bn_apply", z.data_ptr(), 0, M, K, scale.data_ptr(), shift.data_ptr(), res.data_ptr(), act, y0.data_ptr(), 0, s)
    call("mx_bn_apply_p", z.data_ptr(), M, K, scale.data_ptr(), shift.data_ptr(), res.data_ptr(), act, y1.data_ptr(),
         yp.data_ptr(), s)
    d0, d1, r0, r1 = (torch.empty_like(z) for _ in range(4))
    dp = torch.empty((2, M, K), dtype=torch.bfloat16, device=dev)
    call("mx_bn_bwd_apply_ex", gy.data_ptr(), y0.data_ptr(), z.data_ptr(), 0, M, K, act, coef.data_ptr(), d0.data_ptr(),
         r0.data_ptr(), s)
    call("mx_bn_bwd_apply_p", gy.data_ptr(), y0.data_ptr(), z.data_ptr(), M, K, act, coef.data_ptr(), d1.data_ptr(),
         r1.data_ptr(), dp.data_ptr(), s)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1) and torch.equal(yp.view(torch.int16), mc.split_planes(y0).view(torch.int16))
    assert torch.equal(d0, d1) and torch.equal(r0, r1)
    assert torch.equal(dp.view(torch.int16), mc.split_planes(d0).view(torch.int16))


@pytest.mark.parametrize("act,K,K8", [(1, 256, 256), (0, 15, 16), (1, 96, 96)])
def test_act_bias_bwd_planes(dev, act, K, K8):
    """mx_act_bias_bwd_p (the ConvAct backward head with the gradient's planes): the same g and bias
    gradient as mx_act_bias_bwd, and planes equal to split_planes(g)."""
    from mx_det import conv as mc
    g = torch.Generator().manual_seed(K)
    gy = torch.randn(2, 37, 41, K, generator=g).to(dev)
    y = torch.relu(torch.randn(2, 37, 41, K, generator=g)).to(dev)
    g0, db0 = mc.act_bias_bwd(gy, y, act, K8, True, g_dtype=torch.float32)
    g1, db1, gp = mc.act_bias_bwd(gy, y, act, K8, True, g_dtype=torch.float32, planes=True)
    torch.cuda.synchronize()
    assert torch.equal(g0, g1) and torch.equal(db0, db1)
    assert torch.equal(gp.view(torch.int16), mc.split_planes(g0).view(torch.int16))
