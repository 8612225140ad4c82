"""Faster R-CNN ResNet-50-FPN v2 on the libmx_det HIP backend (NHWC activations: f32 with bf16x3 conv
products by default, or bf16; mx_det.backend).

Drop-in for what the reference builds at scripts/train_frcnn_baseline.py:139-143 and
scripts/eval_all.py:79-87:
    model = fasterrcnn_resnet50_fpn_v2(weights=None)
    model.roi_heads.box_predictor = FastRCNNPredictor(model.roi_heads.box_predictor.cls_score.in_features, 7)
    loss_dict = model(images, targets)      # train: loss_classifier, loss_box_reg, loss_objectness, loss_rpn_box_reg
    detections = model(images)              # eval: [{"boxes", "labels", "scores"}], <= 100 per image
The module tree, parameter shapes and state_dict keys follow torchvision 0.20.1's
fasterrcnn_resnet50_fpn_v2 (detr_env_requirements.txt:31), so reference checkpoints
(best.pth {"model": state_dict}) load unchanged. Semantics restated from torchvision (SURVEY.md §8
notes): GeneralizedRCNNTransform, AnchorGenerator, RPNHead(conv_depth=2), RegionProposalNetwork,
RoIHeads with MultiScaleRoIAlign(['0'..'3'], 7, 2), FastRCNNConvFCHead (4 conv+BN, FC 1024),
BoxCoder weights (1,1,1,1) / (10,10,5,5), Matcher / BalancedPositiveNegativeSampler settings.
"""
import math
import os
from collections import OrderedDict

import torch
import torch.nn.functional as F
from torch import nn

from . import ops
from .backend import default_backend
from . import conv as mc
from .conv import ACT_NONE, ACT_RELU, BatchNorm2d, Conv2d, ConvNormAct

RPN_WEIGHTS = (1.0, 1.0, 1.0, 1.0)
ROI_WEIGHTS = (10.0, 10.0, 5.0, 5.0)


def _be(mod):
    return getattr(mod, "_be", None) or default_backend()


# ------------------------------------------------------------------------------------------ body
class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = BatchNorm2d(planes)
        self.conv2 = Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = BatchNorm2d(planes)
        self.conv3 = Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = BatchNorm2d(planes * 4)
        self.downsample = downsample
        # bn1's output is conv2's (3x3, planes -> planes) input: written as pre-split planes beside it
        # when conv2 reads them (conv.planes_for)
        self.conv1.planes_krs = planes * 9

    def forward(self, x, be, feed=None, own_out=False):
        """feed: the previous block's bn3 BNBLink (this block's conv1 dgrad, identity gradient included,
        is that BN's whole incoming gradient); own_out: also return this block's bn3 link (or None)."""
        # no downsample: the identity gradient is added inside conv1's dgrad (HIP backend, training)
        link = be.res_link() if (self.downsample is None and self.training and x.requires_grad
                                 and hasattr(be, "res_link")) else None
        # bn1 / bn2 backward partials from conv2's / conv3's dgrad epilogue (HIP backend, training)
        b1 = b2 = b3 = None
        if self.training and hasattr(be, "bnb_link") and torch.is_grad_enabled() and _bnb_enabled():
            b1, b2 = be.bnb_link(), be.bnb_link()
            b3 = be.bnb_link() if own_out else None
        if self.downsample is not None:
            feed = None  # x also feeds the downsample conv: conv1's dgrad is not its whole gradient
        out = be.conv_bn(x, self.conv1, self.bn1, ACT_RELU, link=link and link.bind("src"), bnb_own=b1,
                         bnb_feed=feed)
        out = be.conv_bn(out, self.conv2, self.bn2, ACT_RELU, bnb_own=b2, bnb_feed=b1)
        identity = x
        if self.downsample is not None:
            identity = be.conv_bn(x, self.downsample[0], self.downsample[1], ACT_NONE)
        y = be.conv_bn(out, self.conv3, self.bn3, ACT_RELU, residual=identity, link=link and link.bind("sink"),
                       bnb_feed=b2, bnb_own=b3)
        return (y, b3) if own_out else y


class ResNet50Body(nn.Module):
    """torchvision resnet50 minus avgpool/fc (IntermediateLayerGetter), nn.BatchNorm2d norm layer."""

    def __init__(self):
        super().__init__()
        self.conv1 = Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = BatchNorm2d(64)
        self.inplanes = 64
        self.layer1 = self._make(64, 3, 1)
        self.layer2 = self._make(128, 4, 2)
        self.layer3 = self._make(256, 6, 2)
        self.layer4 = self._make(512, 3, 2)
        for m in self.modules():
            if isinstance(m, Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")

    def _make(self, planes, blocks, stride):
        ds = None
        if stride != 1 or self.inplanes != planes * 4:
            ds = nn.Sequential(Conv2d(self.inplanes, planes * 4, 1, stride, bias=False), BatchNorm2d(planes * 4))
        layers = [Bottleneck(self.inplanes, planes, stride, ds)]
        self.inplanes = planes * 4
        layers += [Bottleneck(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    LAYERS = ("layer1", "layer2", "layer3", "layer4")

    def stem(self, x, be):
        if (getattr(be, "name", "") == "hip" and x.is_cuda and x.dtype == torch.float32 and self.bn1.training
                and os.environ.get("MX_STEM_FUSED", "1") != "0" and not (torch.is_grad_enabled() and (
                    x.requires_grad or any(p.requires_grad for p in self.conv1.parameters())
                    or any(p.requires_grad for p in self.bn1.parameters())))):
            # frozen stem (torchvision trainable_layers <= 4): no gradient flows through conv1 / bn1 /
            # relu / maxpool, so the BN apply runs inside the pool (mc.conv_bn_act_maxpool)
            return mc.conv_bn_act_maxpool(x, self.conv1, self.bn1, ACT_RELU, 3, 2, 1)
        x = be.conv_bn(x, self.conv1, self.bn1, ACT_RELU)
        return be.maxpool(x, 3, 2, 1)

    def run_layer(self, name, x, be):
        blocks = list(getattr(self, name))
        feed = None
        for j, blk in enumerate(blocks):
            # a block's output feeds only the next block of its layer (conv1 + identity); the
            # layer output also feeds the next layer's downsample and the FPN -> no hand-off
            own = j + 1 < len(blocks)
            r = blk(x, be, feed=feed, own_out=own)
            x, feed = r if own else (r, None)
        return x

    def forward(self, x, be):
        x = self.stem(x, be)
        out = OrderedDict()
        for i, name in enumerate(self.LAYERS):
            x = self.run_layer(name, x, be)
            if mc.absorbing() and 0 < i < len(self.LAYERS) - 1:
                mc.chain_over(x)  # C3 / C4: next stage's conv1 + downsample and the FPN lateral conv
            out[str(i)] = x
        return out


def _aux_stream(device):
    """The RPN loss chain's side stream, one per device."""
    return mc.dedicated_stream(device, "rpn_targets")


def _side_streams(knob):
    """Concurrent small levels (the FPN's P3..P6 output blocks, the RPN head's canvas chain) on side
    streams: on by default (knob "0" turns it off) and off while mc's per-launch timer is installed
    (bench.py's roofline step), so every timed conv runs alone and its event-timed duration is the
    kernel's own (the side-stream wgrad follows the same rule, conv.side_wgrad_enabled)."""
    return os.environ.get(knob, "1") != "0" and mc._timer is None


class FeaturePyramidNetwork(nn.Module):
    """torchvision.ops.FeaturePyramidNetwork(norm_layer=BatchNorm2d) + LastLevelMaxPool."""

    def __init__(self, in_channels_list=(256, 512, 1024, 2048), out_channels=256):
        super().__init__()
        self.inner_blocks = nn.ModuleList([ConvNormAct(c, out_channels, 1, padding=0, act=ACT_NONE)
                                           for c in in_channels_list])
        self.layer_blocks = nn.ModuleList([ConvNormAct(out_channels, out_channels, 3, act=ACT_NONE)
                                           for _ in in_channels_list])
        # producers of 3x3-conv inputs (pre-split planes written beside the output when the consumer
        # reads them): each inner block feeds its level's 3x3 output block, and the P2 output block
        # feeds the level-0 RPN head conv (P3..P6 go through the RPN canvas)
        for blk in self.inner_blocks:
            blk[0].planes_krs = out_channels * 9
        self.layer_blocks[0][0].planes_krs = out_channels * 9
        for m in self.modules():
            if isinstance(m, Conv2d):
                nn.init.kaiming_uniform_(m.weight, a=1)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)

    def forward(self, x, be):
        names = list(x.keys())
        feats = list(x.values())
        side = None
        if feats[0].is_cuda and getattr(be, "name", "") == "hip" and _side_streams("MX_FPN_STREAMS"):
            # the small levels' 3x3 output blocks (and P6) on a side stream beside the top-down chain
            main = torch.cuda.current_stream()
            side = mc.dedicated_stream(feats[0].device, "fpn")

        def block(idx, t):
            if side is None or idx == 0:
                return self.layer_blocks[idx](t, be)
            side.wait_stream(main)
            t.record_stream(side)
            pl = getattr(t, "_mx_planes", None)  # its pre-split planes, read there too
            if pl is not None:
                pl.record_stream(side)
            with torch.cuda.stream(side):
                return self.layer_blocks[idx](t, be)
        last_inner = self.inner_blocks[-1](feats[-1], be)
        results = [block(len(feats) - 1, last_inner)]
        if side is not None:
            with torch.cuda.stream(side):
                pool = be.maxpool(results[-1], 1, 2, 0)
        for idx in range(len(feats) - 2, -1, -1):
            lat = feats[idx]
            top_down = be.upsample_add(last_inner, None, (lat.shape[1], lat.shape[2]))
            # inner_lateral + top_down fused into the lateral conv's BN epilogue
            last_inner = self.inner_blocks[idx](lat, be, residual=top_down)
            results.insert(0, block(idx, last_inner))
        if side is None:
            pool = be.maxpool(results[-1], 1, 2, 0)  # LastLevelMaxPool: max_pool2d(x, 1, 2, 0)
        else:
            main.wait_stream(side)
            for t in results[1:] + [pool]:
                t.record_stream(main)
        results.append(pool)
        return OrderedDict(zip(names + ["pool"], results))


class BackboneWithFPN(nn.Module):
    def __init__(self, trainable_layers=3):
        super().__init__()
        self.body = ResNet50Body()
        self.fpn = FeaturePyramidNetwork()
        self.out_channels = 256
        set_trainable_layers(self.body, trainable_layers)

    def forward(self, x, be):
        return self.fpn(self.body(x, be), be)


def set_trainable_layers(body, trainable_layers):
    """torchvision _resnet_fpn_extractor: freeze every parameter outside the last `trainable_layers`."""
    layers = ["layer4", "layer3", "layer2", "layer1", "conv1"][:trainable_layers]
    if trainable_layers == 5:
        layers.append("bn1")
    for name, p in body.named_parameters():
        if all(not name.startswith(layer) for layer in layers):
            p.requires_grad_(False)


# ------------------------------------------------------------------------------------------ RPN
class RPNHead(nn.Module):
    def __init__(self, in_channels=256, num_anchors=3, conv_depth=2):
        super().__init__()
        self.conv = nn.Sequential(*[ConvNormAct(in_channels, in_channels, 3, norm=False, act=ACT_RELU)
                                    for _ in range(conv_depth)])
        self.cls_logits = Conv2d(in_channels, num_anchors, 1)
        self.bbox_pred = Conv2d(in_channels, num_anchors * 4, 1)
        for m in self.modules():
            if isinstance(m, Conv2d):
                nn.init.normal_(m.weight, std=0.01)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)

    @staticmethod
    def canvas_layout(hws):
        """Top-left corners of the levels hws[0..] on one zero canvas: the first at (0, 0), the rest in
        rows below it, every level framed by at least one zero row / column (the 3x3 convs' padding)."""
        H0, W0 = hws[0]
        pos, y, x, rowh, Wc = [(0, 0)], H0 + 1, 0, 0, W0
        for h, w in hws[1:]:
            if x > 0 and x + w > W0:
                y, x, rowh = y + rowh + 1, 0, 0
            pos.append((y, x))
            Wc = max(Wc, x + w)
            x, rowh = x + w + 1, max(rowh, h)
        return pos, y + rowh, Wc

    def _run(self, t, be, w, b, mask=None):
        for ci, c in enumerate(self.conv):
            t = c(t, be)
            if mask is not None and ci + 1 < len(self.conv):
                # zero frame between levels: the next 3x3 conv reads it as padding
                if t.is_cuda and getattr(be, "name", "") == "hip" and t.shape[3] % 8 == 0:
                    # one launch each way, with the next conv's operand planes (mx_mask_pixels)
                    wn = self.conv[ci + 1][0].weight  # [K, C, R, S] of the next conv
                    t = ops.mask_pixels(t, self._maskf(mask), planes_krs=wn.shape[0] * wn.shape[2] * wn.shape[3])
                else:
                    t = t * mask
        return be.conv(t, w, b, (1, 1), (0, 0), ACT_NONE, out_dtype=torch.float32)  # [N,H,W,A*5]

    def _maskf(self, mask):
        """The canvas mask as f32 [Hc * Wc] (mx_mask_pixels' operand), built once per mask."""
        cache = self.__dict__.setdefault("_maskf_cache", {})
        m = cache.get(id(mask))
        if m is None or m[0] is not mask:
            m = cache[id(mask)] = (mask, mask.reshape(-1).float().contiguous())
        return m[1]

    def layout(self, feats):
        """Static per input shape: (canvas?, level (h, w)s, canvas rectangles (y, x, h, w) of levels 1..,
        canvas (Hc, Wc)). MX_RPN_CANVAS=0 runs every level separately."""
        hws = [tuple(f.shape[1:3]) for f in feats]
        canvas = len(feats) >= 3 and os.environ.get("MX_RPN_CANVAS", "1") != "0"
        if not canvas:
            return False, hws, [], (0, 0)
        pos, Hc, Wc = self.canvas_layout(hws[1:])
        return True, hws, [(y, x, h, w) for (y, x), (h, w) in zip(pos, hws[1:])], (Hc, Wc)

    def raw(self, feats, be):
        """The head's conv outputs [N, H, W, 5A] (A logits, A x 4 deltas per pixel): level 0 alone and, on
        the canvas path, ONE map for the small levels (P3..P6) -- each framed by zero rows / columns on
        a zero canvas, so a 3x3 conv with padding 1 sees exactly each level's own neighbourhood and the
        ReLU outputs on the frame are zeroed before the next 3x3 conv: the same arithmetic per output
        element as per-level convs, in 2 launches per conv instead of 5 (the P4..P6 maps are too small
        to fill the GPU alone). The shared weights' gradients then sum the canvas pixels in one wgrad
        (frame pixels add exact zeros). Without the canvas: one map per level."""
        w, b = _head_cat(self, (self.cls_logits, self.bbox_pred), 4)
        canvas, hws, rects, (Hc, Wc) = self.layout(feats)
        hip = feats[0].is_cuda and getattr(be, "name", "") == "hip"
        # inside a trunk-graph capture (HIP): the levels' root gradients (RoIAlign's) are taken by the
        # level-0 conv's dgrad epilogue and the canvas unpack instead of separate autograd adds
        slots = [mc.GradSlot() for _ in feats] if hip and canvas and mc.absorbing() else None
        self._slots = slots
        if not canvas:
            return [self._run(f, be, w, b) for f in feats]
        if slots is not None:
            mc.absorb_into(feats[0], slots[0])
        f0 = feats[1]
        N, C = f0.shape[0], f0.shape[3]
        key = (Hc, Wc, tuple(rects), f0.dtype, str(f0.device))
        mask = self.__dict__.setdefault("_masks", {}).get(key)
        if mask is None:  # shape constant, built once (outside any capture: the first call is eager)
            mask = f0.new_zeros((1, Hc, Wc, 1))
            for (y, x, h, wd) in rects:
                mask[:, y:y + h, x:x + wd] = 1
            self._masks[key] = mask
        if hip and C % 8 == 0:
            cv = ops.canvas_pack(feats[1:], rects, Hc, Wc, slots[1:] if slots is not None else None)
        else:
            cv = f0.new_zeros((N, Hc, Wc, C))
            for f, (y, x, h, wd) in zip(feats[1:], rects):
                cv[:, y:y + h, x:x + wd] = f
        if hip and _side_streams("MX_RPN_STREAMS"):
            # the canvas chain (P3..P6) on a side stream beside level 0's: independent convs that fill
            # each other's tail rounds; autograd runs each backward on its forward's stream
            main = torch.cuda.current_stream()
            side = mc.dedicated_stream(cv.device, "rpn_head")
            side.wait_stream(main)
            cv.record_stream(side)
            with torch.cuda.stream(side):
                r1 = self._run(cv, be, w, b, mask)
            r0 = self._run(feats[0], be, w, b)
            main.wait_stream(side)
            r1.record_stream(main)
            return [r0, r1]
        return [self._run(feats[0], be, w, b), self._run(cv, be, w, b, mask)]

    def absorbed(self):
        """GradSlots of the last raw() (per feature level), or None."""
        return self.__dict__.get("_slots")

    def split(self, raws, feats_layout, be):
        """raw() outputs -> (objectness [N, Atot], pred_deltas [N, Atot, 4], anchors per level) in
        torchvision's concat_box_prediction_layers order (per image: level, then (h, w, a))."""
        A = self.cls_logits.weight.shape[0]
        canvas, hws, rects, _ = feats_layout
        num_per_level = [h * w * A for h, w in hws]
        if canvas and raws[0].is_cuda and getattr(be, "name", "") == "hip" and raws[0].dtype == torch.float32:
            obj, dl = ops.rpn_head_split(raws[0].contiguous(), raws[1].contiguous(), rects, A)
            return obj, dl, num_per_level
        outs = [raws[0]] + ([raws[1][:, y:y + h, x:x + wd] for (y, x, h, wd) in rects] if canvas else raws[1:])
        logits = [o[..., :A].reshape(o.shape[0], -1) for o in outs]      # (h, w, a) = torchvision permute
        deltas = [o[..., A:].reshape(o.shape[0], -1, 4) for o in outs]
        return torch.cat(logits, 1), torch.cat(deltas, 1), num_per_level

    def forward(self, feats, be):
        """torchvision RPNHead.forward + concat_box_prediction_layers: (objectness, pred_deltas,
        anchors per level)."""
        return self.split(self.raw(feats, be), self.layout(feats), be)


class AnchorGenerator(nn.Module):
    def __init__(self, sizes=((32,), (64,), (128,), (256,), (512,)), aspect_ratios=((0.5, 1.0, 2.0),) * 5):
        super().__init__()
        self.sizes, self.aspect_ratios = sizes, aspect_ratios
        self._cache = {}

    def num_anchors_per_location(self):
        return [len(s) * len(a) for s, a in zip(self.sizes, self.aspect_ratios)]

    def forward(self, padded_hw, grid_sizes, device, be):
        key = (tuple(padded_hw), tuple(grid_sizes), str(device))
        if key not in self._cache:
            out = []
            for (gh, gw), size, ratios in zip(grid_sizes, self.sizes, self.aspect_ratios):
                sh, sw = padded_hw[0] // gh, padded_hw[1] // gw  # torch integer division as torchvision
                out.append(be.anchors_level(float(size[0]), list(ratios), gh, gw, sh, sw, device))
            # every shape's anchors stay alive (a few MB each): a HIP graph captured for one input
            # shape holds their device address, and replacing the cache on a shape change freed that
            # memory under it (the replay read freed memory -- the round-1 "illegal address on replay"
            # of the proposal-chain graph, tests/test_gpu_graphs.py)
            self._cache[key] = torch.cat(out)
        return self._cache[key]


def _gt_batch(targets, dev):
    """(boxes [N, G, 4], labels [N, G], counts int32 [N]) of the step's targets, zero-padded to a
    multiple of 32 GT slots (ops.pad_gt); built once per step and shared by the RPN and RoI heads."""
    key = tuple((id(t["boxes"]), t["boxes"]._version, id(t["labels"]), t["labels"]._version) for t in targets)
    c = _gt_batch.cache
    if c is None or c[0] != key or c[1] != str(dev):
        c = _gt_batch.cache = (key, str(dev), ops.pad_gt(targets, dev), targets)
    return c[2]


_gt_batch.cache = None


def _gt_event(stream):
    """An event on `stream` after the step's padded GT batch (_gt_batch, built there when not cached):
    the RoI sampler reads the cached batch on the main stream."""
    ev = torch.cuda.Event()
    ev.record(stream)
    return ev


def _compact(mask, total):
    """Indices of the True entries of a flat bool mask, ascending, when their number is already
    known on the host (torch.nonzero without its device->host sync)."""
    slot = torch.where(mask, torch.cumsum(mask, 0) - 1, total)
    idx = torch.empty(total + 1, dtype=torch.int64, device=mask.device)
    idx.scatter_(0, slot, torch.arange(mask.numel(), device=mask.device))  # unselected -> spare slot
    return idx[:total]


def _fused_sampler():
    """MX_FUSED_SAMPLER (default on): both samplers draw with mx_sample_draw; off, the RPN's rows go
    to torch.topk and the RoI rows to mx_level_topk (the pre-fusion paths, same keys, same picks)."""
    return os.environ.get("MX_FUSED_SAMPLER", "1") != "0"


class BalancedPositiveNegativeSampler:
    """torchvision det_utils.BalancedPositiveNegativeSampler(batch_size_per_image, positive_fraction):
    per image min(#pos, B*frac) positives (label >= 1) and min(#neg, B - num_pos) negatives (label 0),
    each drawn uniformly without replacement. The draw takes the k smallest of i.i.d. uniform keys (a
    uniform random subset, as randperm(n)[:k] is) and keeps the counts on the device, so sampling
    never waits for the GPU. labels: [N, L] (padding -1) -> boolean masks (pos, neg) of that shape.
    `rand(shape, device)` draws the keys (default torch.rand on the device generator); a parity test
    injects the same key stream into two backends, as SURVEY.md §7 prescribes for the randperm."""

    def __init__(self, batch_size_per_image, positive_fraction):
        self.batch, self.frac = batch_size_per_image, positive_fraction
        self.rand = None
        self.last = None   # (union mask, per-row counts int32 [N, 2]) of the last fused draw

    def __call__(self, lab, be=None, counts=None, valid=None):
        """be: a backend with level_topk draws the k smallest keys with it (used for the RoI sampler's
        ~2k-wide rows; the RPN's 268k-anchor rows stay on torch.topk, which splits a row over many
        workgroups). counts: per-row (#label >= 1, #label == 0) when the matcher already produced them
        (int [N, 2]), sparing two reductions over the rows. valid: bool [N, L], entries where False are
        neither class (the fused draw reads it; the other paths mask the labels first)."""
        L = lab.shape[1]
        if valid is not None and not (be is not None and hasattr(be, "sample_draw") and lab.is_cuda and _fused_sampler()):
            lab = torch.where(valid, lab, -1)  # padding slots belong to neither class
            valid = None
        if be is not None and hasattr(be, "sample_draw") and lab.is_cuda and _fused_sampler():
            # the whole draw in one launch (mx_sample_draw: counts, per-class radix select, marks);
            # the union and the per-row counts stay available for the RoI sampler (self.last)
            r = self.rand(lab.shape, lab.device) if self.rand is not None else torch.rand(lab.shape, device=lab.device)
            pos, neg, un, nums = be.sample_draw(lab, r, self.batch, self.frac, with_union=True, valid=valid)
            self.last = (un, nums)
            return pos, neg
        pos, neg = lab >= 1, lab == 0
        P = int(self.batch * self.frac)
        if counts is not None:
            c = counts.to(torch.int64)
            num_pos = c[:, 0].clamp(max=P)
            num_neg = torch.minimum(c[:, 1], self.batch - num_pos)
        else:
            num_pos = pos.sum(1).clamp(max=P)
            num_neg = torch.minimum(neg.sum(1), self.batch - num_pos)
        r = self.rand(lab.shape, lab.device) if self.rand is not None else torch.rand(lab.shape, device=lab.device)
        kp, kn = min(P, L), min(self.batch, L)
        if (be is None or not hasattr(be, "level_topk")) and kp > 0 and kn > 0:
            # both draws in ONE torch.topk over the stacked [pos; neg] key rows (the RPN's 268k-anchor
            # rows: one multi-kernel top-k sequence instead of two); the sorted ascending prefix of
            # length kp is exactly topk(kp)'s answer
            N = lab.shape[0]
            keys = torch.cat([torch.where(pos, r, 2.0), torch.where(neg, r, 2.0)], 0)
            _, idx = keys.topk(max(kp, kn), dim=1, largest=False)
            return (self._mark(pos, idx[:N, :kp], num_pos), self._mark(neg, idx[N:, :kn], num_neg))
        if kp > 0 and kn > 0 and os.environ.get("MX_SAMPLER_ONE_TOPK", "1") != "0":
            # the same stacking with mx_level_topk: both draws in one launch (value order, ties by
            # index: the top-kp prefix of the top-max(kp, kn) rows is exactly the separate top-kp)
            N = lab.shape[0]
            keys = torch.cat([torch.where(pos, -r, -2.0), torch.where(neg, -r, -2.0)], 0)
            idx = be.level_topk(keys, [L], max(kp, kn))
            return (self._mark(pos, idx[:N, :kp], num_pos), self._mark(neg, idx[N:, :kn], num_neg))
        return self._pick(pos, r, kp, num_pos, be), self._pick(neg, r, kn, num_neg, be)

    @staticmethod
    def _mark(cand, idx, num):
        m = torch.zeros_like(cand)
        m.scatter_(1, idx, torch.arange(idx.shape[1], device=cand.device)[None, :] < num[:, None])
        return m

    @staticmethod
    def _pick(cand, r, k, num, be=None):
        m = torch.zeros_like(cand)
        if k > 0:
            if be is not None and hasattr(be, "level_topk"):
                # the k largest of -key = the k smallest keys, value order (one mx_level_topk launch)
                idx = be.level_topk(torch.where(cand, -r, -2.0), [cand.shape[1]], k)
            else:
                _, idx = torch.where(cand, r, 2.0).topk(k, dim=1, largest=False)  # ascending keys
            m.scatter_(1, idx, torch.arange(k, device=cand.device)[None, :] < num[:, None])
        return m


class RegionProposalNetwork(nn.Module):
    def __init__(self, anchor_generator, head, fg_iou_thresh=0.7, bg_iou_thresh=0.3, batch_size_per_image=256,
                 positive_fraction=0.5, pre_nms_top_n=None, post_nms_top_n=None, nms_thresh=0.7,
                 score_thresh=0.0, min_size=1e-3):
        super().__init__()
        self.anchor_generator = anchor_generator
        self.head = head
        self.fg, self.bg = fg_iou_thresh, bg_iou_thresh
        self.fg_bg_sampler = BalancedPositiveNegativeSampler(batch_size_per_image, positive_fraction)
        self._pre = pre_nms_top_n or dict(training=2000, testing=1000)
        self._post = post_nms_top_n or dict(training=2000, testing=1000)
        self.nms_thresh, self.score_thresh, self.min_size = nms_thresh, score_thresh, min_size
        self._hw = {}

    def pre_nms_top_n(self):
        return self._pre["training" if self.training else "testing"]

    def post_nms_top_n(self):
        return self._post["training" if self.training else "testing"]

    def filter_proposals_padded(self, proposals, objectness, image_sizes, num_per_level, be, with_scores=True):
        """torchvision's filter_proposals with padded outputs: boxes [N, post, 4], scores [N, post] and
        a validity mask (each image's survivors in score order form a prefix of its row). with_scores=False
        (the training forward: the RoI head reads boxes and validity only) returns None for the scores."""
        N = proposals.shape[0]
        dev = proposals.device
        ob = objectness.detach()
        pre = self.pre_nms_top_n()
        top = be.level_topk(ob, num_per_level, pre)  # [N, sum_l min(pre, n_l)], level offsets added
        ckey = ("lvl", tuple(num_per_level), pre, N, dev)
        cached = self._hw.get(ckey)
        if cached is None:  # level id per top-k slot and image index column: shape constants
            lv = torch.cat([torch.full((min(pre, n),), i, dtype=torch.int64, device=dev)
                            for i, n in enumerate(num_per_level)])
            cached = self._hw[ckey] = (lv.unsqueeze(0).expand(N, -1), torch.arange(N, device=dev)[:, None],
                                       lv.repeat(N))
        _, bi, lvl_flat = cached
        prob = torch.sigmoid(ob[bi, top])
        key = (tuple(map(tuple, image_sizes)), dev)
        hw = self._hw.get(key)
        if hw is None:  # (h, w) per image; built once per size set (a host->device copy waits for the GPU)
            hw = self._hw[key] = torch.tensor(image_sizes, dtype=torch.float32, device=dev)
        if hasattr(be, "proposal_clip_filter") and os.environ.get("MX_FUSED_PROPOSALS", "1") != "0":
            # gather + clip + small-box / score filter, one launch
            boxes, grp = be.proposal_clip_filter(proposals, top, prob, hw, self.min_size, self.score_thresh)
        else:
            boxes = proposals[bi, top]
            x = torch.minimum(boxes[..., 0::2].clamp(min=0), hw[:, 1, None, None])
            y = torch.minimum(boxes[..., 1::2].clamp(min=0), hw[:, 0, None, None])
            boxes = torch.stack((x[..., 0], y[..., 0], x[..., 1], y[..., 1]), dim=-1)
            ws, hs = boxes[..., 2] - boxes[..., 0], boxes[..., 3] - boxes[..., 1]
            keep = (ws >= self.min_size) & (hs >= self.min_size) & (prob >= self.score_thresh)
            grp = torch.where(keep, bi, N).reshape(-1)
        # one NMS for all images, torchvision's per-image CPU dispatch rule evaluated on the device;
        # filtered-out candidates are dead entries (group N): nothing here waits for the GPU
        T = top.shape[1]
        n = N * T
        post = self.post_nms_top_n()
        if hasattr(be, "proposal_nms_select") and os.environ.get("MX_SORTED_NMS", "1") != "0":
            # the candidates are presorted (image, level, score desc: the per-level top-k order): the
            # sort-free NMS also emits the padded per-image selection
            sel, valid, nk = be.proposal_nms_select(boxes.reshape(-1, 4), prob.reshape(-1), lvl_flat, grp, N,
                                                    len(num_per_level), self.nms_thresh, max(pre, 1000), post)
            self._watch_nms(nk)
            return boxes.reshape(-1, 4)[sel], (prob.reshape(-1)[sel] if with_scores else None), valid
        kk, nk = be.proposal_nms(boxes.reshape(-1, 4), prob.reshape(-1), lvl_flat, grp, N,
                                 len(num_per_level), self.nms_thresh, max(pre, 1000))
        kk, nk = kk.to(dev), nk.to(dev)
        self._watch_nms(nk)
        live = torch.arange(n, device=dev) < nk
        cnt = torch.zeros(N + 1, dtype=torch.int64, device=dev)
        cnt.scatter_add_(0, torch.where(live, grp[kk].to(torch.int64), N), live.to(torch.int64))
        cnt = cnt[:N]
        r = torch.arange(post, device=dev)
        sel = kk[((torch.cumsum(cnt, 0) - cnt)[:, None] + r[None, :]).clamp(max=n - 1)]  # [N, post]
        valid = r[None, :] < cnt[:, None]                 # survivors are a prefix of each row
        return boxes.reshape(-1, 4)[sel], prob.reshape(-1)[sel], valid

    def _watch_nms(self, nk):
        """The proposal NMS reports what its selection cannot show as num_keep < 0 (-2: candidates not in
        the presorted (image, level) layout, mx_batched_nms_grouped_sorted; -1: an (image, level) segment
        over max_seg): copied to pinned memory without waiting, checked by check_nms() once a later host
        sync has passed -- the step never trains on a silently empty selection."""
        if nk.is_cuda and torch.cuda.is_current_stream_capturing():
            return  # a captured proposal chain (tests/test_gpu_graphs.py) has no host sync to check at
        if not nk.is_cuda:
            if int(nk.reshape(-1)[0]) < 0:
                self._nk_pending = (nk.reshape(()).clone(), None)
            return
        host = self.__dict__.get("_nk_host")
        if host is None:
            with mc.capture_lock:  # pinned allocation: never beside an open graph capture
                host = self.__dict__["_nk_host"] = torch.empty((), dtype=torch.int64, pin_memory=True)
        host.copy_(nk.reshape(-1)[0], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._nk_pending = (host, ev)

    def check_nms(self):
        """Raise if the last proposal NMS reported a failure (see _watch_nms). Called after the RoI head,
        whose host sync has already waited for the NMS, so the event wait is free."""
        pend = self.__dict__.pop("_nk_pending", None)
        if pend is None:
            return
        host, ev = pend
        if ev is not None:
            ev.synchronize()
        v = int(host)
        if v < 0 and self.__dict__.get("_mx_defer_nms_error"):
            # mx_det.dp.DataParallel: recorded, raised on every rank by sync_gradients (a lone raise here
            # would leave the other ranks blocked in the next all-reduce)
            self._nms_error = f"proposal NMS num_keep = {v}"
            return
        if v == -2:
            raise RuntimeError("proposal NMS: candidates are not in the presorted (image, level, score) layout "
                               "mx_batched_nms_grouped_sorted requires (num_keep = -2); MX_SORTED_NMS=0 selects "
                               "the general grouped NMS")
        if v < 0:
            raise RuntimeError(f"proposal NMS: an (image, level) segment exceeds max_seg (num_keep = {v})")

    def filter_proposals(self, proposals, objectness, image_sizes, num_per_level, be):
        """torchvision's filter_proposals: per image, the kept proposal boxes and scores (lists; one
        host sync for the per-image counts)."""
        pb, ps, valid = self.filter_proposals_padded(proposals, objectness, image_sizes, num_per_level, be)
        counts = valid.sum(1).tolist()
        return [pb[i, :c] for i, c in enumerate(counts)], [ps[i, :c] for i, c in enumerate(counts)]

    def forward(self, images, features, targets=None, be=None, head=None, defer_losses=False):
        """torchvision RegionProposalNetwork.forward -> (proposals, losses). defer_losses=True returns a
        callable in place of the losses dict: the caller issues the shape-independent target / sampler
        / loss launches later (FasterRCNN.forward: right after the RoI sampler's host sync, so the GPU
        works on them while the host issues the RoI head instead of idling)."""
        feats = list(features.values())
        # objectness [N, A], pred_deltas [N, A, 4], anchors per level
        objectness, pred_deltas, num_per_level = head if head is not None else self.head(feats, be)
        grid = [(f.shape[1], f.shape[2]) for f in feats]
        anchors = self.anchor_generator(images.tensors.shape[1:3], grid, feats[0].device, be)
        N = feats[0].shape[0]
        A = anchors.shape[0]

        def compute_targets():
            # targets and sampling never wait for the GPU (no autograd: labels, targets, masks)
            if hasattr(be, "match_assign_batched"):  # every image in one launch pair, zero-padded GT
                return self.targets_of(anchors, _gt_batch(targets, anchors.device), be)
            else:
                lcnt = None
                labels, reg_targets = [], []
                for t in targets:
                    _, lab, tg = be.match_assign(t["boxes"], anchors, self.fg, self.bg, True, mode=1,
                                                 weights=RPN_WEIGHTS)
                    labels.append(lab)
                    reg_targets.append(tg)
                lab = torch.stack(labels)                 # [N, A] 1 / 0 / -1
                rt = torch.stack(reg_targets)             # [N, A, 4]
            pm, nm = self.fg_bg_sampler(lab, be if _fused_sampler() else None, counts=lcnt)
            return lab, rt, pm, nm

        def loss_of(tgt):
            # torchvision: BCE mean over the sampled anchors; smooth-L1 (beta 1/9) sum over the sampled
            # positives / number sampled
            lab, rt, pm, nm = tgt
            if hasattr(be, "rpn_loss"):  # HIP: one fused launch each way
                lo, lb = be.rpn_loss(objectness, pred_deltas, lab, rt, pm, nm, 1.0 / 9)
                return {"loss_objectness": lo, "loss_rpn_box_reg": lb}
            sm = pm | nm
            cnt = sm.sum()
            obj = F.binary_cross_entropy_with_logits(objectness, lab.clamp(min=0), reduction="none")
            bl = F.smooth_l1_loss(pred_deltas, rt, beta=1.0 / 9, reduction="none").sum(-1)
            return {"loss_objectness": torch.where(sm, obj, 0.0).sum() / cnt,
                    "loss_rpn_box_reg": torch.where(pm, bl, 0.0).sum() / cnt}

        def compute_losses():
            return loss_of(compute_targets()) if self.training else {}

        side = None
        if (self.training and not defer_losses and objectness.is_cuda and getattr(be, "name", "") == "hip"
                and _side_streams("MX_RPN_LOSS_STREAM")):
            # the target / sampler chain (~25 small launches: anchor matching, the sampler's top-k) on a
            # side stream beside the proposal chain (decode, per-level top-k, NMS, selection): two
            # latency-bound chains of small kernels overlap. Same launches, same RNG draws in the same
            # host order. The chain holds no autograd op: the fused loss (and so its backward) runs on
            # the main stream once FasterRCNN.forward has joined the side stream after the RoI head.
            # Its outputs, allocated on the side stream, need no record_stream: the side stream's next
            # work (and so any reuse of their blocks) is ordered after the main stream by the
            # wait_stream below, at the next step's start of this chain.
            main = torch.cuda.current_stream()
            side = _aux_stream(objectness.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                gt_ready = None
                if hasattr(be, "match_assign_batched"):
                    _gt_batch(targets, objectness.device)  # built (or found cached) first
                    gt_ready = _gt_event(side)
                tgt = compute_targets()
            # _gt_batch's cached batch, built on the side stream, is read by the RoI sampler on the main
            # stream: FasterRCNN.forward waits for this event right before the RoI heads (not here, where
            # the proposal chain, which does not read it, would wait too)
            self._gt_ready = gt_ready
            # recorded right away: if the proposal chain below raises, FasterRCNN.forward's finally
            # still joins the side stream (join_losses)
            self._loss_side = side
            losses = lambda: loss_of(tgt)  # noqa: E731 (deferred: called after join_losses)
        else:
            losses = compute_losses if defer_losses else compute_losses()
        proposals = be.box_decode(pred_deltas.detach().reshape(-1, 4), anchors.repeat(N, 1), RPN_WEIGHTS)
        proposals = proposals.view(N, A, 4)
        if self.training:  # padded (boxes, scores, valid): the RoI sampler works on the device
            boxes = self.filter_proposals_padded(proposals, objectness, images.image_sizes, num_per_level, be,
                                                 with_scores=False)
        else:
            boxes, _ = self.filter_proposals(proposals, objectness, images.image_sizes, num_per_level, be)
        return boxes, losses  # the side stream is joined by join_losses(): after the RoI head

    def targets_of(self, anchors, gt, be):
        """assign_targets_to_anchors + fg_bg_sampler on the device: (labels [N, A], regression targets
        [N, A, 4], positive mask, negative mask) from the zero-padded GT batch gt = (boxes, labels,
        counts) (_gt_batch). Never waits for the GPU."""
        gtp, _, gcnt = gt
        _, lab, rt, lcnt = be.match_assign_batched(gtp, gcnt, anchors, self.fg, self.bg, True, 1,
                                                   weights=RPN_WEIGHTS, with_counts=True)
        pm, nm = self.fg_bg_sampler(lab, be if _fused_sampler() else None, counts=lcnt)
        return lab, rt, pm, nm

    def join_losses(self):
        """Make the current stream wait for the side-stream loss chain (a no-op without one)."""
        side = self.__dict__.pop("_loss_side", None)
        if side is not None:
            torch.cuda.current_stream(side.device).wait_stream(side)


# ------------------------------------------------------------------------------------------ RoI heads
class Linear(nn.Module):
    """nn.Linear-compatible parameters (weight [out, in], bias); runs as a 1x1 MFMA conv."""

    def __init__(self, in_features, out_features, bias=True):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_features))
        self.bias = nn.Parameter(torch.empty(out_features)) if bias else None
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            bound = 1 / math.sqrt(in_features)
            nn.init.uniform_(self.bias, -bound, bound)


def _head_cat(owner, mods, wdim):
    """The fused cls + box GEMM operands: (cat of the modules' weights as a [K, C, 1, 1] conv weight, cat
    of their biases). Without autograd (eval) the same tensors are returned while the parameters are
    unchanged (mc.cached_operand), so conv.operands keeps their packed form too; with autograd (training,
    graph captures) they are recomputed every call."""
    def make():
        w = torch.cat([m.weight for m in mods])
        return (w if wdim == 4 else w[:, :, None, None]), torch.cat([m.bias for m in mods])
    if torch.is_grad_enabled() or (mods[0].weight.is_cuda and torch.cuda.is_current_stream_capturing()):
        return make()
    ts = [m.weight for m in mods] + [m.bias for m in mods]
    return mc.cached_operand(owner, ("head_cat",), ts, make)


class FastRCNNPredictor(nn.Module):
    """torchvision FastRCNNPredictor(in_channels, num_classes): cls_score + bbox_pred, fused in one
    MFMA GEMM (N = num_classes*5) with f32 output."""

    def __init__(self, in_channels, num_classes):
        super().__init__()
        self.cls_score = Linear(in_channels, num_classes)
        self.bbox_pred = Linear(in_channels, num_classes * 4)

    def forward(self, x, be):
        nc = self.cls_score.out_features
        w, b = _head_cat(self, (self.cls_score, self.bbox_pred), 2)
        o = be.conv(x, w, b, (1, 1), (0, 0), ACT_NONE, out_dtype=torch.float32).reshape(x.shape[0], -1)
        return o[:, :nc], o[:, nc:]


class FastRCNNConvFCHead(nn.Sequential):
    """FastRCNNConvFCHead((256,7,7), [256]*4, [1024], norm_layer=BatchNorm2d). FC6 runs as a valid 7x7
    conv over the NHWC RoI tile: torch's NCHW flatten + Linear is exactly a conv whose KCRS weight is
    the Linear weight viewed [1024, 256, 7, 7] (no permute copy, forward or backward); FC7 as 1x1."""

    def __init__(self, in_channels=256, conv_layers=(256, 256, 256, 256), fc_layers=(1024,), hw=7):
        blocks, prev = [], in_channels
        for c in conv_layers:
            if blocks:  # the previous conv's output is this 3x3 conv's input (pre-split planes)
                blocks[-1][0].planes_krs = c * 9
            blocks.append(ConvNormAct(prev, c, 3, act=ACT_RELU))
            prev = c
        blocks.append(nn.Flatten())
        prev = prev * hw * hw
        for c in fc_layers:
            blocks.append(Linear(prev, c))
            blocks.append(nn.ReLU(inplace=True))
            prev = c
        super().__init__(*blocks)
        self.hw = hw
        for m in self.modules():
            if isinstance(m, Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
                if m.bias is not None:
                    nn.init.zeros_(m.bias)

    def fc_weight_views(self):
        """(Linear, its conv-shaped weight view) for FC6 (valid hw x hw conv) and the following FCs (1x1)."""
        out, first = [], True
        for m in self:
            if isinstance(m, Linear):
                w = m.weight
                if first:
                    c = m.in_features // (self.hw * self.hw)
                    out.append((m, w.view(m.out_features, c, self.hw, self.hw)))
                    first = False
                else:
                    out.append((m, w[:, :, None, None]))
        return out

    def forward(self, x, be):
        fcs = iter(self.fc_weight_views())
        convs = [m for m in self if isinstance(m, ConvNormAct)]
        # conv i's BN gets its backward partials from conv i+1's dgrad (3x3 stride 1 chain)
        links = [None] * len(convs)
        if self.training and hasattr(be, "bnb_link") and torch.is_grad_enabled() and _bnb_enabled():
            links = [be.bnb_link() for _ in convs[:-1]] + [None]
        ci = 0
        for m in self:
            if isinstance(m, ConvNormAct):
                x = m(x, be, bnb_own=links[ci], bnb_feed=links[ci - 1] if ci else None)
                ci += 1
            elif isinstance(m, Linear):
                _, w = next(fcs)
                x = be.conv(x, w, m.bias, (1, 1), (0, 0), ACT_RELU)  # Linear + ReLU; [R,7,7,C] -> [R,1,1,1024]
        return x  # [R, 1, 1, 1024]


class RoIHeads(nn.Module):
    def __init__(self, box_head, box_predictor, fg_iou_thresh=0.5, bg_iou_thresh=0.5, batch_size_per_image=512,
                 positive_fraction=0.25, score_thresh=0.05, nms_thresh=0.5, detections_per_img=100):
        super().__init__()
        self.box_head = box_head
        self.box_predictor = box_predictor
        self.fg, self.bg = fg_iou_thresh, bg_iou_thresh
        self.fg_bg_sampler = BalancedPositiveNegativeSampler(batch_size_per_image, positive_fraction)
        self.score_thresh, self.nms_thresh, self.detections_per_img = score_thresh, nms_thresh, detections_per_img
        self.featmap_names = ["0", "1", "2", "3"]

    def _head_graph(self, x, be):
        """Box head + predictor forward/backward as two HIP graphs per RoI count (training, HIP
        backend): the ~90 launches of 4 conv+BN+ReLU, FC6, FC7 and the predictor (and their
        backward, including the RoI-feature gradient for RoIAlign's backward) replay from two graph
        launches. Training samples a fixed 512 RoIs per image whenever enough candidates exist, so
        one shape recurs; at most 4 shapes are captured, others run eagerly (as do MX_GRAPHS=0,
        eval and non-HIP backends)."""
        import os
        if not (x.is_cuda and getattr(be, "name", "") == "hip" and _graphs_enabled(self)
                and os.environ.get("MX_HEAD_GRAPHS", "1") != "0"):
            return None
        key = (tuple(x.shape), x.dtype)
        cache = self.__dict__.setdefault("_mx_graphs", {})
        g = cache.get(key)
        if g is None:
            if len(cache) >= 4:
                return None
            head = _Head(self, be)
            g = cache[key] = _Graphs(head, head.parameters(), self, x, input_grad=True)
        g.on_ready = self.__dict__.get("_mx_grads_ready")
        return g

    def _scales(self, feats, image_sizes):
        # MultiScaleRoIAlign._setup_scales / _infer_scale (height-based), LevelMapper k_min/k_max
        max_h = max(s[0] for s in image_sizes)
        scales = [2.0 ** round(math.log2(float(f.shape[1]) / float(max_h))) for f in feats]
        return scales, int(-math.log2(scales[0]))

    def forward(self, features, proposals, image_sizes, targets=None, be=None):
        feats = [features[k] for k in self.featmap_names]
        dev = feats[0].device
        if self.training:
            # candidates per image = its kept proposals (a valid prefix of `post` slots, score order)
            # then its GT boxes (torchvision: cat([proposals, gt])), padded to [N, post + Gmax] with
            # label -1 on padding, matched and sampled on the device; the one host sync of this stage
            # reads the number of sampled RoIs
            pb, _, pvalid = proposals
            N, post = pvalid.shape
            # GT slots padded to _gt_batch's width (a multiple of 32) on every backend, so the sampler
            # draws keys over the same [N, post + gm] rows whichever path builds them
            gtp, glp, gcnt = _gt_batch(targets, dev)
            gm = gtp.shape[1]
            fused = hasattr(be, "roi_candidates") and _fused_sampler()
            if fused:  # candidate boxes and validity in one launch; the sampler reads the validity
                box_p, valid = be.roi_candidates(pb, pvalid, gtp, gcnt)
            else:
                gslot = torch.arange(gm, device=dev)
                box_p = torch.cat([pb, gtp], 1)           # [N, post + gm, 4]
                valid = torch.cat([pvalid, gslot[None, :] < gcnt[:, None]], 1)
            if hasattr(be, "match_assign_batched"):       # both images in one launch pair
                _, lab_b, tg_p = be.match_assign_batched(gtp, gcnt, box_p, self.fg, self.bg, False, 2,
                                                         gt_labels=glp, weights=ROI_WEIGHTS)
            else:
                lab_l, tg_l = [], []
                for i, t in enumerate(targets):
                    g = int(t["boxes"].shape[0])
                    _, lab, tg = be.match_assign(gtp[i, :g], box_p[i], self.fg, self.bg, False, mode=2,
                                                 gt_labels=glp[i, :g], weights=ROI_WEIGHTS)
                    lab_l.append(lab.to(dev))
                    tg_l.append(tg.to(dev))
                lab_b, tg_p = torch.stack(lab_l), torch.stack(tg_l)
            # the sampled entries are valid ones, so the compaction below reads lab_b as it is; the
            # unfused path masks the padding to -1 first (torchvision's rows hold no padding)
            lab_p = lab_b if fused else torch.where(valid, lab_b, -1)
            self.fg_bg_sampler.last = None
            pos_m, neg_m = self.fg_bg_sampler(lab_p, be, valid=valid if fused else None)
            if self.fg_bg_sampler.last is not None:       # the fused draw's union and per-row counts
                un, nums = self.fg_bg_sampler.last
                sm = un.flatten()
                total = int(nums.sum())                   # the stage's one host sync (sizes the RoI head)
            else:
                sm = (pos_m | neg_m).flatten()
                total = int(sm.sum())                     # the stage's one host sync (sizes the RoI head)
            cm = lab_p.shape[1]
            if hasattr(be, "roi_compact") and os.environ.get("MX_FUSED_ROI_COMPACT", "1") != "0":
                # per image ascending, as torch.where per image: one launch after the sync
                rois, lab_k, tg_k = be.roi_compact(sm, total, cm, box_p.reshape(-1, 4), lab_p.reshape(-1),
                                                   tg_p.reshape(-1, 4))
                labels, tgts = [lab_k], [tg_k]
            else:
                idx = _compact(sm, total)
                rois = torch.cat([(idx // cm).to(torch.float32)[:, None], box_p.reshape(-1, 4)[idx]], 1)
                labels, tgts = [lab_p.reshape(-1)[idx]], [tg_p.reshape(-1, 4)[idx]]
        else:
            rois = torch.cat([torch.cat([torch.full((p.shape[0], 1), float(i), device=dev), p], 1)
                              for i, p in enumerate(proposals)])
        scales, k_min = self._scales(feats, image_sizes)
        x = be.multiscale_roi_align(feats, rois, scales, k_min)
        head = self._head_graph(x, be) if self.training else None
        if head is not None:  # HIP-graph replay of box head + predictor (static RoI count)
            class_logits, box_regression = head(x)
        else:
            class_logits, box_regression = self.box_predictor(self.box_head(x, be), be)
        if self.training:
            lab = labels[0] if len(labels) == 1 else torch.cat(labels)  # (one-entry lists: no copy launch)
            rt = tgts[0] if len(tgts) == 1 else torch.cat(tgts)
            if hasattr(be, "roi_loss"):  # HIP: one fused launch each way
                loss_cls, loss_box = be.roi_loss(class_logits, box_regression, lab, rt, 1.0 / 9)
            else:
                loss_cls = F.cross_entropy(class_logits, lab)
                R = class_logits.shape[0]
                reg = box_regression.reshape(R, -1, 4)[torch.arange(R, device=dev), lab]
                # torchvision: smooth-L1 (beta 1/9) summed over the positive RoIs / number of sampled RoIs
                bl = F.smooth_l1_loss(reg, rt, beta=1.0 / 9, reduction="none").sum(-1)
                loss_box = torch.where(lab > 0, bl, 0.0).sum() / lab.numel()
            return [], {"loss_classifier": loss_cls, "loss_box_reg": loss_box}
        return self.postprocess_detections(class_logits, box_regression, proposals, image_sizes, be), {}

    def postprocess_detections(self, class_logits, box_regression, proposals, image_sizes, be):
        dev = class_logits.device
        nc = class_logits.shape[-1]
        per = [p.shape[0] for p in proposals]
        pred = be.box_decode(box_regression, torch.cat(proposals), ROI_WEIGHTS).reshape(-1, nc, 4)
        scores = F.softmax(class_logits, -1)
        out = []
        for boxes, sc, hw in zip(pred.split(per), scores.split(per), image_sizes):
            h, w = float(hw[0]), float(hw[1])
            boxes = torch.stack((boxes[..., 0].clamp(0, w), boxes[..., 1].clamp(0, h),
                                 boxes[..., 2].clamp(0, w), boxes[..., 3].clamp(0, h)), -1)
            labels = torch.arange(nc, device=dev).view(1, -1).expand_as(sc)
            boxes, sc, labels = boxes[:, 1:].reshape(-1, 4), sc[:, 1:].reshape(-1), labels[:, 1:].reshape(-1)
            # torchvision's score threshold, then remove_small_boxes(1e-2) on the survivors: the same set in
            # the same order as one mask over both conditions (one nonzero -- one host sync -- not two)
            ws, hs = boxes[:, 2] - boxes[:, 0], boxes[:, 3] - boxes[:, 1]
            k = torch.where((sc > self.score_thresh) & (ws >= 1e-2) & (hs >= 1e-2))[0]
            boxes, sc, labels = boxes[k], sc[k], labels[k]
            k = be.batched_nms(boxes, sc, labels, self.nms_thresh, max_seg=max(per) if per else None)
            k = k[: self.detections_per_img]
            out.append({"boxes": boxes[k], "labels": labels[k], "scores": sc[k]})
        return out


# ------------------------------------------------------------------------------------------ transform
class ImageList:
    def __init__(self, tensors, image_sizes):
        self.tensors, self.image_sizes = tensors, image_sizes


class GeneralizedRCNNTransform(nn.Module):
    """normalize -> resize (min 800 / max 1333, bilinear) -> zero-pad to /32, NHWC output with the stem's
    8 channels. On the HIP backend every device input takes a fused kernel: uint8 [B,H,W,3] batches
    that need no resize mx_normalize_pad, uint8 HWC frames of any size and the reference loader's
    float32 CHW tensors mx_resize_normalize_pad(_f32). The torch ops below serve the CPU backend."""

    def __init__(self, min_size=800, max_size=1333, image_mean=(0.485, 0.456, 0.406),
                 image_std=(0.229, 0.224, 0.225), size_divisible=32):
        super().__init__()
        self.min_size, self.max_size = min_size, max_size
        self.image_mean, self.image_std = image_mean, image_std
        self.size_divisible = size_divisible

    def _scale(self, h, w):
        return min(self.min_size / min(h, w), self.max_size / max(h, w))

    def _padded(self, sizes):
        sd = self.size_divisible
        H = max(s[0] for s in sizes)
        W = max(s[1] for s in sizes)
        return int(math.ceil(H / sd) * sd), int(math.ceil(W / sd) * sd)

    def forward(self, images, targets, be):
        if isinstance(images, (list, tuple)) and len(images) and images[0].dtype == torch.uint8:
            same = all(im.shape == images[0].shape for im in images)
            images = torch.stack(list(images)) if same else images
        if isinstance(images, torch.Tensor) and images.dtype == torch.uint8 and images.dim() == 4:
            B, H, W, _ = images.shape
            if self._scale(H, W) == 1.0:
                sizes = [(H, W)] * B
                return ImageList(be.normalize_pad_u8(images, self._padded(sizes)), sizes), targets
        u8 = isinstance(images, torch.Tensor) and images.dtype == torch.uint8 and images.dim() == 4 or \
            isinstance(images, (list, tuple)) and len(images) and images[0].dtype == torch.uint8 and \
            all(im.dim() == 3 and im.shape[2] == 3 for im in images)
        if u8 and hasattr(be, "resize_normalize_pad_u8") and images[0].is_cuda == (getattr(be, "name", "") == "hip"):
            # uint8 HWC frames of any size (VisDrone): one fused resize + normalize + pad launch
            sizes, orig = [], []
            for im in images:
                h, w = int(im.shape[0]), int(im.shape[1])
                s = self._scale(h, w)
                # F.interpolate(recompute_scale_factor=True): out = floor(in * s) in double precision
                sizes.append((h, w) if s == 1.0 else (int(math.floor(h * s)), int(math.floor(w * s))))
                orig.append((h, w))
            batch = be.resize_normalize_pad_u8(list(images), sizes, self._padded(sizes))
            if targets is not None:
                targets = [self._resize_boxes(dict(t), o, n) for t, o, n in zip(targets, orig, sizes)]
            return ImageList(batch, sizes), targets
        f32chw = isinstance(images, (list, tuple)) and len(images) and all(
            isinstance(im, torch.Tensor) and im.dtype == torch.float32 and im.dim() == 3 and im.shape[0] == 3
            for im in images)
        if f32chw and hasattr(be, "resize_normalize_pad_u8") and getattr(be, "name", "") == "hip" and \
                all(im.is_cuda for im in images):
            # the reference loader's ToDtype(float32, scale=True) CHW tensors (train_frcnn_baseline.py:50-54):
            # the same fused resize + normalize + pad launch as uint8 frames (bit-identical batch)
            sizes, orig = [], []
            for im in images:
                h, w = int(im.shape[1]), int(im.shape[2])
                s = self._scale(h, w)
                sizes.append((h, w) if s == 1.0 else (int(math.floor(h * s)), int(math.floor(w * s))))
                orig.append((h, w))
            batch = be.resize_normalize_pad_u8(list(images), sizes, self._padded(sizes))
            if targets is not None:
                targets = [self._resize_boxes(dict(t), o, n) for t, o, n in zip(targets, orig, sizes)]
            return ImageList(batch, sizes), targets
        if len(images) and images[0].dtype == torch.uint8:  # HWC uint8 -> ToDtype(float32, scale=True)
            images = [im.permute(2, 0, 1).float().mul_(1.0 / 255) for im in images]
        dev = images[0].device
        mean = torch.tensor(self.image_mean, dtype=torch.float32, device=dev)[:, None, None]
        std = torch.tensor(self.image_std, dtype=torch.float32, device=dev)[:, None, None]
        out, sizes, new_targets = [], [], []
        for i, im in enumerate(images):
            im = (im - mean) / std
            h, w = im.shape[-2:]
            s = self._scale(h, w)
            if s != 1.0:
                im = F.interpolate(im[None], size=None, scale_factor=s, mode="bilinear",
                                   recompute_scale_factor=True, align_corners=False)[0]
            nh, nw = im.shape[-2:]
            if targets is not None:
                new_targets.append(self._resize_boxes(dict(targets[i]), (h, w), (nh, nw)))
            out.append(im)
            sizes.append((int(nh), int(nw)))
        Hp, Wp = self._padded(sizes)
        batch = torch.zeros((len(out), Hp, Wp, be.stem_channels), dtype=be.act_dtype, device=dev)
        for i, im in enumerate(out):
            batch[i, : im.shape[1], : im.shape[2], :3] = im.permute(1, 2, 0).to(be.act_dtype)
        return ImageList(batch, sizes), (new_targets if targets is not None else None)

    @staticmethod
    def _resize_boxes(t, orig, new):
        """torchvision transform.py resize_boxes: ratios as float32 tensors new / orig per axis."""
        (h, w), (nh, nw) = orig, new
        if (nh, nw) != (h, w):
            rh = torch.tensor(nh, dtype=torch.float32) / torch.tensor(h, dtype=torch.float32)
            rw = torch.tensor(nw, dtype=torch.float32) / torch.tensor(w, dtype=torch.float32)
            b = t["boxes"]
            t["boxes"] = torch.stack((b[:, 0] * rw.to(b.device), b[:, 1] * rh.to(b.device),
                                      b[:, 2] * rw.to(b.device), b[:, 3] * rh.to(b.device)), 1)
        return t

    def postprocess(self, result, image_sizes, original_sizes):
        for i, (pred, s, o) in enumerate(zip(result, image_sizes, original_sizes)):
            if tuple(s) == tuple(o):
                continue
            rh = torch.tensor(o[0], dtype=torch.float32) / torch.tensor(s[0], dtype=torch.float32)
            rw = torch.tensor(o[1], dtype=torch.float32) / torch.tensor(s[1], dtype=torch.float32)
            b = pred["boxes"]
            pred["boxes"] = torch.stack((b[:, 0] * rw.to(b.device), b[:, 1] * rh.to(b.device),
                                         b[:, 2] * rw.to(b.device), b[:, 3] * rh.to(b.device)), 1)
        return result


# ------------------------------------------------------------------------------------------ model
class FasterRCNN(nn.Module):
    def __init__(self, backbone, num_classes=91, rpn_head=None, box_head=None, **kw):
        super().__init__()
        self.transform = GeneralizedRCNNTransform()
        self.backbone = backbone
        ag = AnchorGenerator()
        self.rpn = RegionProposalNetwork(ag, rpn_head or RPNHead(backbone.out_channels,
                                                                 ag.num_anchors_per_location()[0]))
        box_head = box_head or FastRCNNConvFCHead()
        self.roi_heads = RoIHeads(box_head, FastRCNNPredictor(1024, num_classes))
        self._be = kw.get("backend")

    @property
    def be(self):
        return _be(self)

    def set_backend(self, be):
        self._be = be
        return self

    def _trunk(self, x, be):
        """Backbone + FPN + RPN-head convs as one captured HIP graph per input shape (training, HIP
        backend): their ~400 kernels per step replay from one forward and one backward graph launch
        instead of being issued op by op from Python (_Graphs; the op kernels are the same
        libmx_det launches, recorded on the capture stream). At most 8 input shapes are captured;
        further shapes, eval, MX_GRAPHS=0 and non-HIP backends run eagerly."""
        if not (self.training and x.is_cuda and getattr(be, "name", "") == "hip" and _graphs_enabled(self)):
            return None
        key = (tuple(x.shape), x.dtype)
        cache = self.__dict__.setdefault("_mx_graphs", {})
        g = cache.get(key)
        if g is None:
            if len(cache) >= 8:  # many distinct padded sizes (real datasets): the rest run eagerly
                return None
            g = cache[key] = _capture_trunk(self, be, x)
        outs = g(x)
        nf = len(self.backbone.fpn.inner_blocks) + 1
        feats = OrderedDict(zip([str(i) for i in range(nf - 1)] + ["pool"], outs[:nf]))
        head = self.rpn.head
        return feats, head.split(list(outs[nf:]), head.layout(outs[:nf]), be)

    def _flag_async(self, flags):
        """(pinned host bool, event) of any(flags) copied without waiting, or None."""
        if not flags:
            return None
        f = torch.stack(flags).any() if len(flags) > 1 else flags[0]
        host = self.__dict__.get("_degenerate_host")
        if host is None:
            host = self.__dict__["_degenerate_host"] = torch.empty((), dtype=torch.bool, pin_memory=True)
        host.copy_(f, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return host, ev

    def forward(self, images, targets=None):
        be = self.be
        if hasattr(be, "prepare"):
            be.prepare(self)  # per-step operand preparation (HIP: every conv weight packed in one launch)
        degenerate = None
        if self.training:
            if targets is None:
                raise ValueError("In training mode, targets should be passed")
            dev_boxes = []
            for t in targets:
                b = t["boxes"]
                if not (isinstance(b, torch.Tensor) and b.dim() == 2 and b.shape[-1] == 4):
                    raise ValueError(f"Expected target boxes to be a tensor of shape [N, 4], got {b.shape}.")
                if b.numel():
                    if b.is_cuda:
                        dev_boxes.append(b)
                    elif bool(((b[:, 2:] <= b[:, :2]).any())):
                        raise ValueError("All bounding boxes should have positive height and width.")
            # GeneralizedRCNN.forward's degenerate-box check without its per-image host round trips:
            # the device flag is copied to pinned memory asynchronously and read after the RPN's own
            # host sync (filter_proposals' per-image counts), where it is already complete.
            # Divergence: torchvision raises BEFORE any forward; here the backbone / FPN / RPN forward of
            # the rejected batch has already run, so its BatchNorm running statistics (v2 has BN in the
            # FPN and box head too) and the graphs' static buffers are updated by it. A loop that catches
            # the error and skips the batch should set MX_STRICT_TARGETS=1 (one host sync per step,
            # torchvision's order and state).
            if dev_boxes and os.environ.get("MX_STRICT_TARGETS", "0") == "1":
                if bool(torch.stack([(b[:, 2:] <= b[:, :2]).any() for b in dev_boxes]).any()):
                    raise ValueError("All bounding boxes should have positive height and width.")
                dev_boxes = []
        if isinstance(images, torch.Tensor) and images.dim() == 4 and images.dtype == torch.uint8:
            original = [(images.shape[1], images.shape[2])] * images.shape[0]
        else:  # float CHW (reference ToDtype output) or uint8 HWC tensors
            original = [(int(im.shape[0]), int(im.shape[1])) if im.dtype == torch.uint8 else
                        (int(im.shape[-2]), int(im.shape[-1])) for im in images]
        if self.training and dev_boxes:
            # one check launch + the pinned copy on the HIP backend (else the torch compares), issued
            # ahead of the trunk: two launches of host time before the step's first kernels, and the
            # event is complete long before the check below reads it
            flags = ([be.boxes_degenerate(dev_boxes)] if hasattr(be, "boxes_degenerate") else
                     [(b[:, 2:] <= b[:, :2]).any() for b in dev_boxes])
            degenerate = self._flag_async(flags)
        il, targets = self.transform(images, targets, be)
        # MX_RPN_DEFER_LOSSES=1 issues the RPN target / loss launches after the RoI sampler's host sync;
        # measured 0.5 % slower than issuing them while the trunk runs (A/B on one box), so off
        defer = os.environ.get("MX_RPN_DEFER_LOSSES", "0") != "0"
        try:
            trunk = self._trunk(il.tensors, be)
            if trunk is not None:  # HIP-graph replay of backbone + FPN + RPN head (static shapes)
                features, head = trunk
            else:
                features, head = self.backbone(il.tensors, be), None
            proposals, rpn_losses = self.rpn(il, features, targets, be, head=head, defer_losses=defer)
            if degenerate is not None:
                host, ev = degenerate
                ev.synchronize()
                if bool(host):
                    raise ValueError("All bounding boxes should have positive height and width.")
            gt_ready = self.rpn.__dict__.pop("_gt_ready", None)
            if gt_ready is not None:  # the RoI sampler reads the GT batch the RPN's side stream built
                torch.cuda.current_stream().wait_event(gt_ready)
            detections, det_losses = self.roi_heads(features, proposals, il.image_sizes, targets, be)
            self.rpn.check_nms()
        finally:  # also when the step raises: no side-stream work is left unjoined behind it
            self.rpn.join_losses()
        if self.training:
            losses = {}
            losses.update(det_losses)
            # deferred: issued after the RoI sampler's host sync, overlapping the host's RoI-head work
            losses.update(rpn_losses() if callable(rpn_losses) else rpn_losses)
            return losses
        return self.transform.postprocess(detections, il.image_sizes, original)


def _bnb_enabled():
    import os
    return os.environ.get("MX_BNB", "1") != "0"


def _graphs_enabled(mod=None):
    import os
    if os.environ.get("MX_GRAPHS", "1") == "0":
        return False
    if mod is not None and mod.__dict__.get("_mx_dp"):
        return True  # mx_det.dp.DataParallel: gradients averaged after the backward
    import torch.distributed as dist
    # under torch DDP the gradient all-reduce hooks live on the parameters' AccumulateGrad nodes,
    # which the replayed backward graph bypasses: such runs keep the trunk eager
    return not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1)


class _Trunk(nn.Module):
    """backbone + FPN + RPN head as one tensor -> tuple(tensors) callable (the graphed unit)."""

    def __init__(self, model, be):
        super().__init__()
        self.backbone, self.head = model.backbone, model.rpn.head
        self.be = be

    def forward(self, x):
        feats = self.backbone(x, self.be)
        return tuple(feats.values()) + tuple(self.head.raw(list(feats.values()), self.be))

    def absorbed(self):
        return self.head.absorbed()


class _Graphs:
    """Forward and backward HIP graphs of a static-shape sub-network fn(x) -> tuple(tensors). The
    backward graph writes the parameters' gradients (and, with input_grad, x's) into graph-owned
    buffers that become their .grad after each replay (added when a .grad already exists), so no
    per-parameter autograd work runs in the step. Capture follows torch.cuda.graph: eager warmup on
    a side stream, then one forward and one backward capture in a shared private pool; the BatchNorm
    running statistics of `stats_module` are restored afterwards."""

    def __init__(self, fn, params, stats_module, x, input_grad=False):
        self.params = [p for p in params if p.requires_grad]
        saved = {k: v.clone() for k, v in stats_module.state_dict().items()
                 if k.endswith(("running_mean", "running_var", "num_batches_tracked"))}
        grads = [p.grad for p in self.params]
        self.input_grad = input_grad
        self.static_x = x.detach().clone().requires_grad_(input_grad)
        side = mc.capture_stream(x.device)  # warm-up and capture share it (bn_scratch)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):
                outs = fn(self.static_x)
                torch.autograd.backward(outs, [torch.ones_like(o) for o in outs])
                del outs
                for p in self.params:
                    p.grad = None
                self.static_x.grad = None
        torch.cuda.current_stream().wait_stream(side)
        pool = torch.cuda.graph_pool_handle()
        self.fwd = torch.cuda.CUDAGraph()
        with mc.capture_guard(), torch.cuda.graph(self.fwd, pool=pool, stream=side), mc.absorb_mode():
            self.static_out = fn(self.static_x)
        self.static_gout = [torch.zeros_like(o) for o in self.static_out]
        roots, groots = _absorb_roots(fn, self.static_out, self.static_gout)
        self.bwd = torch.cuda.CUDAGraph()
        with mc.capture_guard(), torch.cuda.graph(self.bwd, pool=pool, stream=side):
            torch.autograd.backward(roots, groots)
        self.static_grads = [p.grad for p in self.params]
        self.static_xgrad = self.static_x.grad
        self.static_out = tuple(o.detach() for o in self.static_out)
        for p, g in zip(self.params, grads):
            p.grad = g
        with torch.no_grad():
            sd = stats_module.state_dict()
            for k, v in saved.items():
                sd[k].copy_(v)
        self.anchor = torch.zeros((), device=x.device, requires_grad=True)
        self.on_ready = None

    def __call__(self, x):
        return _GraphFn.apply(x, self.anchor, self)


def _absorb_roots(fn, outs, gouts):
    """Backward roots of a captured trunk: the outputs whose gradient an in-graph consumer takes from
    its static buffer (fn.absorbed(): conv.GradSlot per leading output) are left out; their slots get
    the buffers."""
    slots = fn.absorbed() if hasattr(fn, "absorbed") else None
    if not slots:
        return list(outs), list(gouts)
    roots, groots = [], []
    for i, (o, g) in enumerate(zip(outs, gouts)):
        # only a slot whose consumer claimed it at forward time replaces the root (an unclaimed one --
        # e.g. a copy in front of the consumer broke the tensor identity -- stays an ordinary root)
        if i < len(slots) and slots[i] is not None and slots[i].taken:
            slots[i].buf = g
        else:
            roots.append(o)
            groots.append(g)
    return roots, groots


def _tag_outputs(tg):
    """Fresh tensor objects over a graph's static outputs, each tagged with the static buffer its
    gradient is copied into before the backward replay (ops.grad_buffer: the RoIAlign and RPN-head
    backward kernels write there directly, and the copy is skipped)."""
    outs = tuple(o.detach() for o in tg.static_out)
    for o, b in zip(outs, tg.static_gout):
        o._mx_gbuf = b
    return outs


def _load_gouts(tg, gouts):
    for s, g in zip(tg.static_gout, gouts):
        if g is None:
            s.zero_()
        elif not (g.data_ptr() == s.data_ptr() and g.shape == s.shape and g.stride() == s.stride()
                  and g.dtype == s.dtype):
            s.copy_(g)


class _GraphFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, tg):
        tg.static_x.copy_(x)
        tg.fwd.replay()
        ctx.tg = tg
        # fresh tensor objects over the graph's static outputs (overwritten by the next replay)
        return _tag_outputs(tg)

    @staticmethod
    def backward(ctx, *gouts):
        tg = ctx.tg
        _load_gouts(tg, gouts)
        # A .grad still aliasing the graph's static buffer (adopted by the previous replay, kept by
        # zero_grad(set_to_none=False) or gradient accumulation) gets its own storage first: the
        # replay below overwrites the static buffer.
        for p, g in zip(tg.params, tg.static_grads):
            if g is not None and p.grad is g:
                p.grad = g.clone()
        tg.bwd.replay()
        for p, g in zip(tg.params, tg.static_grads):
            if g is None:
                continue
            if p.grad is None:
                p.grad = g  # adopted without a copy (the usual zero_grad(set_to_none=True) step)
            else:
                p.grad.add_(g)
        if tg.on_ready is not None:  # e.g. mx_det.dp.DataParallel starts this unit's all-reduce
            tg.on_ready()
        # the input gradient is the graph's static buffer: consumed by the producer's backward in
        # this same backward pass, before the next replay overwrites it
        return (tg.static_xgrad if tg.input_grad else None), None, None


def _capture_trunk(model, be, x):
    if model.__dict__.get("_mx_seg_ready") is not None:  # data-parallel: per-segment gradient hand-off
        return _SegGraphs(model, be, x)
    if os.environ.get("MX_SEG_GRAPHS", "0") == "1":
        # one backward graph per segment on one GPU too: the HIP graph executor submits a graph's node
        # lists one after another, so a segment's side-stream wgrads start before the next segment's
        # dgrad chain is submitted instead of after the whole trunk's (MX_WGRAD_FORK=early)
        return _SegGraphs(model, be, x)
    trunk = _Trunk(model, be)
    return _Graphs(trunk, trunk.parameters(), model, x)


class _SegGraphs:
    """The trunk (backbone + FPN + RPN head) as ONE forward graph and a chain of backward graphs, one
    per segment in backward order, so that when a segment's graph has been issued its parameters'
    gradients are final and `model._mx_seg_ready(key, params)` can start their all-reduce on RCCL's
    stream while the remaining segments' backward graphs run (mx_det.dp.DataParallel; SURVEY.md §8e:
    bucketed all-reduce overlapped with the backward).

    Segment boundaries sit at stage outputs C2..Cb (MX_DP_BOUNDS "2", "23", "234" or "2345"; default
    "23"): at a boundary the forward detaches the stage output into a leaf that the next stage and the
    FPN lateral both consume, and the segment below it back-propagates from that leaf's gradient
    (written by the graphs replayed before it). Without a boundary the next stage and the FPN consume
    the output itself and the backward flows through in one autograd pass -- the FPN's, so the
    boundaries are a prefix C2..Cb. "2345" gives five segments (FPN + RPN head, layer4, layer3, layer2,
    stem + layer1); "23" gives FPN + RPN head + layer4 + layer3 (106 MB of gradients, all-reduced while
    layer2's backward runs), layer2, stem + layer1. Every boundary
    costs a join: a segment's graph completes with its side-stream weight gradients, and the next
    segment's dgrad chain waits for them (one-GPU A/B: profiles/r06_ab.txt). Same kernels as the
    one-graph trunk; at a boundary the gradient reaching the stage output is summed over its consumers
    in a different order. Buffers and captures follow _Graphs (shared private pool, replays in
    capture order)."""

    LAYER_KEYS = ("stem+layer1", "layer2", "layer3", "layer4")  # producers of C2, C3, C4, C5

    def __init__(self, model, be, x):
        self.model, self.be = model, be
        body = model.backbone.body
        self.seg_params = {"stem+layer1": list(body.conv1.parameters()) + list(body.bn1.parameters()) +
                           list(body.layer1.parameters()),
                           "layer2": list(body.layer2.parameters()), "layer3": list(body.layer3.parameters()),
                           "layer4": list(body.layer4.parameters()),
                           "fpn+rpn_head": list(model.backbone.fpn.parameters()) + list(model.rpn.head.parameters())}
        self.seg_params = {k: [p for p in v if p.requires_grad] for k, v in self.seg_params.items()}
        spec = os.environ.get("MX_DP_BOUNDS", "23")
        self.bounds = {int(c) - 2 for c in spec if c in "2345"}  # leaf index k <-> C(k+2)
        # the FPN lateral reads every stage output that is not a boundary, so the first (FPN) segment's
        # pass reaches it: boundaries must be C2..Cb, a prefix ("2", "23", "234", "2345")
        if not self.bounds or len(spec) != len(self.bounds) or self.bounds != set(range(len(self.bounds))):
            raise ValueError(f"MX_DP_BOUNDS={spec!r}: one of 2, 23, 234, 2345 (the stage outputs C2..Cb that end a "
                             "backward segment)")
        # C(k+2) needs a gradient iff some stage below it trains
        up = list(self.LAYER_KEYS)
        self.need = [any(self.seg_params[u] for u in up[:k + 1]) for k in range(4)]
        self.params = [p for k in ("fpn+rpn_head",) + self.LAYER_KEYS for p in self.seg_params[k]]
        saved = {k: v.clone() for k, v in model.state_dict().items()
                 if k.endswith(("running_mean", "running_var", "num_batches_tracked"))}
        grads = [p.grad for p in self.params]
        self.static_x = x.detach().clone()
        side = mc.capture_stream(x.device)  # warm-up and capture share it (bn_scratch)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):
                outs, ins, cs = self._fwd(self.static_x)
                self._bwd_all(outs, [torch.ones_like(o) for o in outs], ins, cs)
                del outs, ins, cs
                for p in self.params:
                    p.grad = None
        torch.cuda.current_stream().wait_stream(side)
        pool = torch.cuda.graph_pool_handle()
        self.fwd = torch.cuda.CUDAGraph()
        with mc.capture_guard(), torch.cuda.graph(self.fwd, pool=pool, stream=side), mc.absorb_mode():
            outs, self.ins, self.cs = self._fwd(self.static_x)
        self.static_gout = [torch.zeros_like(o) for o in outs]
        r0, g0 = _absorb_roots(self.model.rpn.head, outs, self.static_gout)
        self.bwd = []  # (segment keys, graph)
        for keys, roots, groots in self._bwd_plan(outs, self.static_gout, self.ins, self.cs, (r0, g0)):
            g = torch.cuda.CUDAGraph()
            with mc.capture_guard(), torch.cuda.graph(g, pool=pool, stream=side):
                torch.autograd.backward(roots, groots())
            self.bwd.append((keys, g))
        self.static_out = tuple(o.detach() for o in outs)
        self.static_grads = {k: [p.grad for p in v] for k, v in self.seg_params.items()}
        # the boundary-leaf gradients pass between the backward graphs: keep them referenced
        self.keep = [self.ins[k].grad for k in sorted(self.bounds)] + [o for o in outs]
        self.ins, self.cs = None, None
        for p, g in zip(self.params, grads):
            p.grad = g
        with torch.no_grad():
            sd = model.state_dict()
            for k, v in saved.items():
                sd[k].copy_(v)
        self.anchor = torch.zeros((), device=x.device, requires_grad=True)
        self.on_ready = None

    def _fwd(self, x):
        """-> (trunk outputs, ins, cs): cs[k] = C(k+2) as produced, ins[k] = what the next stage and the
        FPN lateral consume (a detached leaf at a boundary, else cs[k] itself)."""
        body, be = self.model.backbone.body, self.be
        c = body.run_layer("layer1", body.stem(x, be), be)
        ins, cs = [], [c]
        for k, name in enumerate(("layer2", "layer3", "layer4", None)):
            t = c.detach().requires_grad_(self.need[k]) if k in self.bounds else c
            if k in (1, 2) and self.need[k] and mc.absorbing():
                mc.chain_over(t)  # C3 / C4: next stage's conv1 + downsample and the FPN lateral
            ins.append(t)
            if name is not None:
                c = body.run_layer(name, t, be)
                cs.append(c)
        feats = self.model.backbone.fpn(OrderedDict((str(i), l) for i, l in enumerate(ins)), be)
        return tuple(feats.values()) + tuple(self.model.rpn.head.raw(list(feats.values()), be)), ins, cs

    def _bwd_plan(self, outs, gouts, ins, cs, first=None):
        """[(segment keys, roots, () -> root gradients)] in backward order. The first segment starts at
        the trunk outputs (FPN + RPN head) and takes every stage above the highest boundary; each
        boundary C(k+2) starts a segment at cs[k] with its leaf's gradient (read lazily: the leaf's
        .grad exists once the segments above have run), down to the next boundary. A segment that
        would hold no gradient (frozen stages) is left out. first: the FPN + RPN-head roots after
        gradient absorption."""
        r0, g0 = first if first is not None else (outs, gouts)
        plan = [(["fpn+rpn_head"], r0, lambda: g0)]
        for k in (3, 2, 1, 0):  # C5 .. C2 and their producers layer4 .. stem+layer1
            key = self.LAYER_KEYS[k]
            if k in self.bounds:
                if not self.need[k]:
                    break  # nothing below trains
                plan.append(([key], [cs[k]], (lambda lf: (lambda: [lf.grad]))(ins[k])))
            else:
                plan[-1][0].append(key)
        return [(tuple(keys), roots, groots) for keys, roots, groots in plan]

    def _bwd_all(self, outs, gouts, ins, cs):
        for _, roots, groots in self._bwd_plan(outs, gouts, ins, cs):
            torch.autograd.backward(roots, groots())

    def __call__(self, x):
        return _SegGraphFn.apply(x, self.anchor, self)


class _SegGraphFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, tg):
        tg.static_x.copy_(x)
        tg.fwd.replay()
        ctx.tg = tg
        return _tag_outputs(tg)

    @staticmethod
    def backward(ctx, *gouts):
        tg = ctx.tg
        _load_gouts(tg, gouts)
        for keys, _ in tg.bwd:  # see _GraphFn.backward
            for key in keys:
                for p, g in zip(tg.seg_params[key], tg.static_grads[key]):
                    if g is not None and p.grad is g:
                        p.grad = g.clone()
        hook = tg.model.__dict__.get("_mx_seg_ready")
        # the .grad bookkeeping of every segment runs before the first replay: between two replays the
        # host only fires the hand-off hook (issuing a collective), so the segment graphs queue back
        # to back; a gradient accumulated onto an existing .grad (add_) must follow its graph
        plan = []
        for keys, graph in tg.bwd:
            ps, acc = [], []
            for key in keys:
                for p, g in zip(tg.seg_params[key], tg.static_grads[key]):
                    if g is None:
                        continue
                    ps.append(p)
                    if p.grad is None:
                        p.grad = g
                    else:
                        acc.append((p.grad, g))
            plan.append((keys, graph, ps, acc))
        for keys, graph, ps, acc in plan:
            graph.replay()
            for pg, g in acc:
                pg.add_(g)
            if hook is not None and ps:  # every group up to the segment's last trained key is final
                hook([k for k in keys if tg.seg_params[k]][-1], ps)
        return None, None, None


class _Head(nn.Module):
    """box head + predictor as one tensor -> (class_logits, box_regression) callable."""

    def __init__(self, roi_heads, be):
        super().__init__()
        self.box_head, self.box_predictor = roi_heads.box_head, roi_heads.box_predictor
        self.be = be

    def forward(self, x):
        return self.box_predictor(self.box_head(x, self.be), self.be)


def fasterrcnn_resnet50_fpn_v2(weights=None, progress=True, num_classes=None, weights_backbone=None,
                               trainable_backbone_layers=None, **kwargs):
    """torchvision.models.detection.fasterrcnn_resnet50_fpn_v2 signature.

    weights: None, or a path / state_dict of a reference checkpoint (there is no network: the
    reference's weights="DEFAULT" download is replaced by a local file). Trainable layers follow
    torchvision's rule (5 without weights, else 3 by default)."""
    is_trained = weights is not None or weights_backbone is not None
    if not is_trained:
        trainable = 5
    else:
        trainable = 3 if trainable_backbone_layers is None else trainable_backbone_layers
    if kwargs.pop("force_trainable_layers", None) is not None:
        trainable = trainable_backbone_layers
    nc = num_classes if num_classes is not None else 91
    model = FasterRCNN(BackboneWithFPN(trainable), num_classes=nc, **kwargs)
    if weights is not None:
        sd = weights if isinstance(weights, dict) else torch.load(weights, map_location="cpu", weights_only=True)
        sd = sd.get("model", sd)
        model.load_state_dict(sd)
    return model
