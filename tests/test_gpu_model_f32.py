"""End-to-end parity of the precision-faithful path (HipBackend("f32"): f32 activations, bf16x3 conv
products) with the CPU restatement backend (oracle/cpu_backend.py: torch-CPU fp32 conv / BN / pool
+ the C restatement of torchvision's detection ops) on the same seeded weights and inputs.

north_star bar: "within 1e-3 box/score tolerance" (eval_all.py:111 model(images)) and losses within
1e-3 relative for the training step (train_frcnn_baseline.py:171 model(images, targets)). Inputs:
2 synthetic VisDrone-shaped images of 512 x 672 (GeneralizedRCNNTransform resizes them to 800 x 1050).
The weights are seeded random init with the objectness and class logits scaled so that the RPN
top-k / NMS and the detection ranking are decided by real score gaps (an untrained head puts ~6,000
near-identical 1/7 class scores in the final top-100, where any 1e-7 perturbation reorders them).
The samplers draw the same key stream on both backends (BalancedPositiveNegativeSampler.rand)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model(dev):
    from mx_det import frcnn
    m = frcnn.fasterrcnn_resnet50_fpn_v2(weights=None)
    m.roi_heads.box_predictor = frcnn.FastRCNNPredictor(m.roi_heads.box_predictor.cls_score.in_features, 7)
    frcnn.set_trainable_layers(m.backbone.body, 3)
    return m.to(dev)


def _pair(dev, seed, damp=1.0, rpn_scale=40.0):
    from mx_det.backend import HipBackend
    from oracle.cpu_backend import CpuBackend
    torch.manual_seed(seed)
    m = _model("cpu")
    with torch.no_grad():
        m.rpn.head.cls_logits.weight.mul_(rpn_scale)
        m.roi_heads.box_predictor.cls_score.weight.mul_(40.0)
        for name, mod in m.backbone.body.named_modules():
            if name.endswith("bn3"):  # residual-branch gain (torchvision zero_init_residual at 0)
                mod.weight.mul_(damp)
    mc = _model("cpu").set_backend(CpuBackend())
    mc.load_state_dict(m.state_dict())
    return m.to(dev).set_backend(HipBackend("f32")), mc


def _keys(seed):
    g = torch.Generator().manual_seed(seed)
    return lambda shape, device: torch.rand(shape, generator=g).to(device)


def _eval_pair(dev):
    from mx_det.data import synth_batch
    m, mc = _pair(dev, 0)
    m.eval()
    mc.eval()
    imgs, _ = synth_batch(20, 2, H=512, W=672)
    with torch.no_grad():
        ref = mc(list(imgs))
        out = m(list(imgs.to(dev)))
    return out, ref


def test_f32_eval_detections_match_cpu_backend(dev, monkeypatch):
    """eval_all.py:111 model(images) with the RoI head fed the fp32 CPU model's proposals (see
    _pin_proposals: the RPN's 0.7-IoU NMS over a random-init anchor-grid-like proposal set flips on
    float noise): identical labels, boxes and scores within 1e-3."""
    from mx_det import frcnn
    monkeypatch.setattr(frcnn.RegionProposalNetwork, "filter_proposals_padded", _pin_proposals())
    out, ref = _eval_pair(dev)
    for o, r in zip(out, ref):
        n = r["labels"].numel()
        assert n > 10, n
        assert o["labels"].numel() == n
        assert torch.equal(o["labels"].cpu(), r["labels"])
        torch.testing.assert_close(o["scores"].cpu(), r["scores"], rtol=1e-3, atol=1e-3)
        torch.testing.assert_close(o["boxes"].cpu(), r["boxes"], rtol=1e-3, atol=1e-3)


def test_f32_eval_detections_unpinned(dev):
    """The same call end to end with each backend running its own RPN: at least 99 % of the CPU
    detections have a HIP detection with the same label, score and box within 1e-3 (a flipped
    proposal-NMS decision moves the odd detection by a few pixels: measured 1 of 200 on one box)."""
    out, ref = _eval_pair(dev)
    for o, r in zip(out, ref):
        n = r["labels"].numel()
        assert n > 10 and abs(o["labels"].numel() - n) <= max(2, n // 50), (o["labels"].numel(), n)
        ob, os_, ol = o["boxes"].cpu(), o["scores"].cpu(), o["labels"].cpu()
        hit = 0
        for b, s, lab in zip(r["boxes"], r["scores"], r["labels"]):
            ok = (ol == lab) & ((os_ - s).abs() <= 1e-3 + 1e-3 * s.abs()) & \
                 ((ob - b).abs() <= 1e-3 + 1e-3 * b.abs()).all(1)
            hit += bool(ok.any())
        assert hit >= 0.99 * n, (hit, n)


def _tf32(t):
    i = t.float().contiguous().view(torch.int32).to(torch.int64)
    r = ((i + 0xFFF + ((i >> 13) & 1)) >> 13) << 13
    return (((r + 2 ** 31) % 2 ** 32) - 2 ** 31).to(torch.int32).view(torch.float32)


def _tf32_backend():
    """The CPU restatement with every conv's operands rounded to TF32: the reference's own arithmetic
    on its Ampere GPU (cudnn.allow_tf32 default; train_frcnn_baseline.py:139-176)."""
    import torch.nn.functional as F
    from oracle.cpu_backend import CpuBackend, _act, _nchw, _nhwc

    class Tf32CpuBackend(CpuBackend):
        def conv_bn(self, x, conv, bn, act, residual=None, link=None, bnb_own=None, bnb_feed=None):
            xn, w = _nchw(x), conv.weight
            # rounded operands in the forward, gradients straight through to the f32 tensors (the
            # conv's own backward then also multiplies by the rounded saved operands)
            xt = xn + (_tf32(xn) - xn).detach()
            wt = w + (_tf32(w) - w).detach()
            z = F.conv2d(xt, wt, None, conv.stride, conv.padding)
            z = F.batch_norm(z, bn.running_mean, bn.running_var, bn.weight, bn.bias, bn.training, bn.momentum, bn.eps)
            if residual is not None:
                z = z + _nchw(residual)
            return _nhwc(_act(z, act))
    return Tf32CpuBackend()


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("damp", [1.0, 0.25])
def test_f32_trunk_closer_than_tf32(dev, damp):
    """Backbone + FPN in train mode (batch-statistics BN) end to end: the HIP f32 features' distance
    to the CPU fp32 restatement is at least 10x smaller than the reference's own TF32 arithmetic's
    distance (the same CPU model with TF32-rounded conv operands). A random-init ResNet with bs-2
    batch statistics amplifies any per-layer perturbation ~1.25x per block (~1.1x with the residual
    gain damped), so this, not an absolute bound, is the faithful-arithmetic check of the trunk."""
    from mx_det.data import synth_batch
    m, mc = _pair(dev, 1, damp)
    m.train()
    mc.train()
    import copy
    mt = copy.deepcopy(mc).set_backend(_tf32_backend())
    imgs, _ = synth_batch(30, 2, H=512, W=672)
    with torch.no_grad():
        fh = m.backbone(m.transform(list(imgs.to(dev)), None, m.be)[0].tensors, m.be)
        il, _ = mc.transform(list(imgs), None, mc.be)
        fc = mc.backbone(il.tensors, mc.be)
        ft = mt.backbone(il.tensors, mt.be)
    for k in fc:
        e, et = _rel(fh[k], fc[k]), _rel(ft[k], fc[k])
        assert e * 10 < et, (k, e, et)


def _pin_proposals():
    """Hand the fp32 CPU model's RPN proposals (padded boxes, scores, valid) to every later model's RoI
    head: the order of near-equal proposal scores is not defined at f32 level (adjacent top-2000
    objectness gaps ~3e-4 of its spread), and the RoI sampler draws its keys by proposal slot.
    The first call made on a CPU tensor is the one captured (the CPU models run first)."""
    from mx_det import frcnn
    orig = frcnn.RegionProposalNetwork.filter_proposals_padded
    cap = {}

    def fp(self, proposals, objectness, image_sizes, num_per_level, be, **kw):
        if "p" not in cap and proposals.device.type == "cpu":
            cap["p"] = orig(self, proposals, objectness, image_sizes, num_per_level, be, **kw)
            return cap["p"]
        if "p" not in cap:
            return orig(self, proposals, objectness, image_sizes, num_per_level, be, **kw)
        return tuple(t.to(proposals.device) if t is not None else None for t in cap["p"])
    return fp


@pytest.mark.timeout(400)
@pytest.mark.parametrize("hw", [(512, 672), (800, 1333)])
def test_f32_train_losses_and_grads_match_cpu_backend(dev, monkeypatch, hw):
    """One train forward + backward: all four losses within 1e-3 relative of the CPU fp32 path, and
    every trainable gradient closer to it than the reference's own arithmetic is (the CPU path with
    TF32-rounded conv operands, its Ampere GPU run), >= 5x closer on average over the parameters
    (measured: 7.5 % vs 56 % mean; the random-init network with bs-2 batch-statistics BN magnifies
    a 1e-3 feature perturbation ~50x in its gradients, for both). The RPN runs on each backend; the RoI head
    then consumes the fp32 CPU proposals on all three (see _pin_proposals). The proposal sets
    themselves are not compared: with a random-init RPN the proposals are the anchor grid plus ~1 %
    offsets, and the greedy 0.7-IoU NMS over that dense grid propagates any single flipped decision
    (one pair within float noise of IoU 0.7, or two near-equal scores in swapped order) through its
    neighbourhood -- measured (tools/debug_f32_parity.py) ~70 % of the sets agree whether the trunk
    features differ by 1e-3 or 5e-5, i.e. the divergence is the NMS cascade, not the size of the
    perturbation. Sizes: 512 x 672 frames (resized to 800 x 1050) and configs[1]'s own 1333 x 800
    (padded 1344 x 800, no resize)."""
    import copy
    from mx_det import frcnn
    from mx_det.data import synth_batch
    m, mc = _pair(dev, 1)
    mt = copy.deepcopy(mc).set_backend(_tf32_backend())
    for mod in (m, mc, mt):
        mod.train()
        mod.rpn.fg_bg_sampler.rand = _keys(7)
        mod.roi_heads.fg_bg_sampler.rand = _keys(8)
    monkeypatch.setattr(frcnn.RegionProposalNetwork, "filter_proposals_padded", _pin_proposals())
    imgs, tg = synth_batch(30, 2, H=hw[0], W=hw[1])
    ldc = mc(list(imgs), tg)
    ldt = mt(list(imgs), tg)
    ld = m(list(imgs.to(dev)), [{k: v.to(dev) for k, v in t.items()} for t in tg])
    assert list(ld) == list(ldc)
    for k in ld:
        a, b = float(ld[k].detach()), float(ldc[k].detach())
        assert abs(a - b) <= 1e-3 * abs(b), (k, a, b, float(ldt[k].detach()))
    for mod, d in ((m, ld), (mc, ldc), (mt, ldt)):
        sum(d.values()).backward()
    pc, pt = dict(mc.named_parameters()), dict(mt.named_parameters())
    eh, et, names = [], [], []
    for name, p in m.named_parameters():
        if not p.requires_grad:
            continue
        assert p.grad is not None and pc[name].grad is not None, name
        eh.append(_rel(p.grad, pc[name].grad))
        et.append(_rel(pt[name].grad, pc[name].grad))
        names.append(name)
    import os
    if os.environ.get("MX_DUMP_GRADS"):
        for n, a, b in zip(names, eh, et):
            print(f"GRAD {n:60s} hip {a:.3e} tf32 {b:.3e}")
    mh, mt_ = sum(eh) / len(eh), sum(et) / len(et)
    assert mh * 5 < mt_, (mh, mt_)
    bad = [(n, a, b) for n, a, b in zip(names, eh, et) if a > b]
    assert not bad, bad[:5]


def test_f32_rpn_proposal_drift_bounded(dev):
    """The HIP RPN's own proposal set vs the fp32 CPU restatement's on the scaled-logit RPN (eval,
    post_nms_top_n = 1000 per image): both backends run filter_proposals on their own objectness and
    decoded boxes. Float noise can flip a 0.7-IoU NMS decision between near-equal proposals, so the
    sets are compared as sets: per image the proposal counts agree within 1 %, and at least 99 % of
    the CPU proposals have a HIP proposal with the same box (1e-3) and score (1e-3) -- the bound the
    unpinned end-to-end test inherits."""
    from mx_det import frcnn
    orig = frcnn.RegionProposalNetwork.filter_proposals_padded
    cap = {}

    def fp(self, proposals, objectness, image_sizes, num_per_level, be, **kw):
        out = orig(self, proposals, objectness, image_sizes, num_per_level, be, **kw)
        cap.setdefault(proposals.device.type, out)
        return out
    frcnn.RegionProposalNetwork.filter_proposals_padded = fp
    try:
        _eval_pair(dev)
    finally:
        frcnn.RegionProposalNetwork.filter_proposals_padded = orig
    (hb, hs, hv), (cb, cs, cv) = [tuple(t.cpu() for t in cap[k][:3]) for k in ("cuda", "cpu")]
    for i in range(cb.shape[0]):
        rb, rs = cb[i][cv[i].bool()], cs[i][cv[i].bool()]
        ob, os_ = hb[i][hv[i].bool()], hs[i][hv[i].bool()]
        n = rs.numel()
        assert n > 500 and abs(os_.numel() - n) <= max(2, n // 100), (os_.numel(), n)
        d = (rb[:, None, :] - ob[None, :, :]).abs() <= 1e-3 + 1e-3 * rb[:, None, :].abs()
        ok = d.all(-1) & ((rs[:, None] - os_[None, :]).abs() <= 1e-3 + 1e-3 * rs[:, None].abs())
        hit = int(ok.any(1).sum())
        assert hit >= 0.99 * n, (hit, n)
