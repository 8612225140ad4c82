"""Op backend the detection model is written against.

`HipBackend` (this file) is the product path: every hot op is a libmx_det HIP kernel on NHWC
activations. The model never calls torch conv/pool/RoI ops itself; it calls `self.be.*`. (A CPU
restatement of the same interface lives in oracle/cpu_backend.py for parity tests and the CPU
baseline; the product never imports it.)

Precision (`HipBackend(precision=...)`, default from MX_PRECISION, else "f32"):
  "f32"   the reference's arithmetic (fp32 model, TF32 convs on Ampere; train_frcnn_baseline.py:139-176,
          no autocast): f32 activations / gradients / BN / RoIAlign, convs as bf16x3 MFMA products
          (~2^-16 relative, finer than TF32's 2^-11)
  "bf16"  bf16 activations and conv operands with f32 accumulation (faster, 2^-8 per rounding)
"""
import ctypes
import os

import torch

from . import conv as mc
from . import ops
from . import _lib
from ._lib import call


def _s():
    return _lib.stream()


def _p(t):
    return t.data_ptr() if t is not None else None


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, st, pd):
        x = x.contiguous()
        N, H, W, C = x.shape
        Ho, Wo = (H + 2 * pd - k) // st + 1, (W + 2 * pd - k) // st + 1
        y = torch.empty((N, Ho, Wo, C), dtype=x.dtype, device=x.device)
        arg = torch.empty((N, Ho, Wo, C), dtype=torch.int32, device=x.device) if x.requires_grad else None
        call("mx_maxpool_fwd", _p(x), mc.dcode(x), N, H, W, C, k, st, pd, _p(y), _p(arg), _s())
        ctx.save_for_backward(arg)
        ctx.cfg = (x.shape, k, st, pd)
        return y

    @staticmethod
    def backward(ctx, gy):
        (arg,) = ctx.saved_tensors
        (N, H, W, C), k, st, pd = ctx.cfg
        gy = gy.contiguous()
        gx = torch.empty((N, H, W, C), dtype=gy.dtype, device=gy.device)
        call("mx_maxpool_bwd", _p(gy), mc.dcode(gy), _p(arg), N, H, W, C, k, st, pd, _p(gx), _s())
        return gx, None, None, None


class _UpsampleAdd(torch.autograd.Function):
    """y = nearest_upsample(x, size) + add (FPN top-down)."""

    @staticmethod
    def forward(ctx, x, add, Ho, Wo):
        x = x.contiguous()
        N, H, W, C = x.shape
        y = torch.empty((N, Ho, Wo, C), dtype=x.dtype, device=x.device)
        a = add.contiguous() if add is not None else None
        if a is not None:
            assert a.dtype == x.dtype
        call("mx_upsample_nearest_fwd", _p(x), mc.dcode(x), N, H, W, C, Ho, Wo, _p(a), _p(y), _s())
        ctx.cfg = (x.shape, Ho, Wo, add is not None)
        return y

    @staticmethod
    def backward(ctx, gy):
        (N, H, W, C), Ho, Wo, has_add = ctx.cfg
        g = gy.contiguous()
        gx = torch.empty((N, H, W, C), dtype=g.dtype, device=gy.device)
        call("mx_upsample_nearest_bwd", _p(g), mc.dcode(g), N, H, W, C, Ho, Wo, _p(gx), _s())
        return gx, (g if has_add else None), None, None


def default_precision():
    p = os.environ.get("MX_PRECISION", "f32").lower()
    if p not in ("f32", "bf16"):
        raise ValueError(f"MX_PRECISION must be f32 or bf16, got {p!r}")
    return p


class HipBackend:
    name = "hip"
    stem_channels = 8  # RGB padded to 8 channels for the 8-channel gather of the stem conv

    def __init__(self, precision=None):
        self.precision = precision or default_precision()
        if self.precision not in ("f32", "bf16"):
            raise ValueError(f"precision must be 'f32' or 'bf16', got {self.precision!r}")
        self.act_dtype = torch.float32 if self.precision == "f32" else torch.bfloat16

    def prepare(self, model):
        """Register every conv weight of the model with one WeightPacker (first call) and repack the
        changed ones in a single launch; the conv autograd functions then read the packed operands."""
        key = "_mx_packer_" + self.precision
        pk = model.__dict__.get(key)
        if pk is None:
            from .frcnn import FastRCNNConvFCHead
            split = self.precision == "f32"
            pk = mc.WeightPacker()
            for m in model.modules():
                if isinstance(m, mc.Conv2d):
                    pk.register(m.weight, m.stride, m.padding, m.weight.requires_grad, split=split)
                elif isinstance(m, FastRCNNConvFCHead):
                    for i, (lin, w) in enumerate(m.fc_weight_views()):
                        pk.register(w, (1, 1), (0, 0), lin.weight.requires_grad, dense=i == 0, split=split)
            model.__dict__[key] = pk
        mc.set_packer(pk)
        pk.refresh()
        bns = model.__dict__.get("_mx_bns")
        if bns is None:
            bns = model.__dict__["_mx_bns"] = [m for m in model.modules() if isinstance(m, mc.BatchNorm2d)]
        mc.count_batches([b for b in bns if b.training] if model.training else [])

    # ---- dense ---------------------------------------------------------------------------
    def conv_bn(self, x, conv, bn, act, residual=None, link=None, bnb_own=None, bnb_feed=None):
        return mc.conv_bn(x, conv, bn, act, residual, link, bnb_own, bnb_feed)

    @staticmethod
    def res_link():
        return mc.ResLink()

    @staticmethod
    def bnb_link():
        return mc.BNBLink()

    def conv(self, x, weight, bias, stride, pad, act, out_dtype=None):
        if not torch.is_grad_enabled():  # eval: no autograd bookkeeping, no planes for an unused wgrad
            return mc.conv_act_nograd(x, weight, bias, stride, pad, act, out_dtype)
        return mc.ConvAct.apply(x, weight, bias, stride, pad, act, out_dtype)

    def maxpool(self, x, k, stride, pad):
        return _MaxPool.apply(x, k, stride, pad)

    def upsample_add(self, x, add, size):
        return _UpsampleAdd.apply(x, add, size[0], size[1])

    # ---- detection ops ---------------------------------------------------------------------
    def multiscale_roi_align(self, feats, rois, scales, k_min, output_size=(7, 7), sampling_ratio=2):
        return ops.multiscale_roi_align(feats, rois, scales, k_min, output_size, sampling_ratio)

    def match_assign(self, gt, boxes, high, low, allow_lq, mode, gt_labels=None, weights=None):
        return ops.match_assign(gt, boxes, high, low, allow_lq, mode, gt_labels, weights)

    def match_assign_batched(self, gt_pad, gcount, boxes, high, low, allow_lq, mode, gt_labels=None, weights=None,
                             with_counts=False):
        return ops.match_assign_batched(gt_pad, gcount, boxes, high, low, allow_lq, mode, gt_labels, weights,
                                        with_counts)

    def batched_nms(self, boxes, scores, idxs, thr, group=None, max_seg=None, mode=0):
        return ops.batched_nms(boxes, scores, idxs, thr, group=group, max_seg=max_seg, mode=mode)

    def roi_loss(self, class_logits, box_regression, labels, targets, beta):
        return ops.roi_loss(class_logits, box_regression, labels, targets, beta)

    def rpn_loss(self, objectness, deltas, labels, targets, pos, neg, beta):
        return ops.rpn_loss(objectness, deltas, labels, targets, pos, neg, beta)

    def level_topk(self, scores, num_per_level, k):
        return ops.level_topk(scores, num_per_level, k)

    def sample_draw(self, labels, keys, batch, positive_fraction, with_union=False, valid=None):
        return ops.sample_draw(labels, keys, batch, positive_fraction, with_union, valid=valid)

    def roi_candidates(self, pb, pvalid, gtp, gcnt):
        return ops.roi_candidates(pb, pvalid, gtp, gcnt)

    def proposal_nms(self, boxes, scores, lvl, group, G, L, thr, max_seg):
        return ops.batched_nms_grouped(boxes, scores, lvl, group, G, L, thr, max_seg)

    def proposal_nms_select(self, boxes, scores, lvl, group, G, L, thr, max_seg, post):
        """filter_proposals' NMS on its presorted candidates plus the padded per-image selection:
        (sel [G, post], valid [G, post], num_keep [1] int64) (mx_batched_nms_grouped_sorted). num_keep < 0
        flags a failure the selection cannot show (-2: candidates not in the presorted layout, -1: a
        segment over max_seg): the caller checks it (frcnn RegionProposalNetwork.check_nms)."""
        _, nk, sel, valid = ops.batched_nms_grouped_sorted(boxes, scores, lvl, group, G, L, thr, max_seg, post)
        return sel, valid, nk

    def box_decode(self, rel, boxes, weights):
        return ops.box_decode(rel, boxes, weights)

    def boxes_degenerate(self, boxes_list):
        return ops.boxes_degenerate(boxes_list)

    def roi_compact(self, mask, total, cm, box, lab, tg):
        return ops.roi_compact(mask, total, cm, box, lab, tg)

    def proposal_clip_filter(self, proposals, top, prob, hw, min_size, score_thresh):
        return ops.proposal_clip_filter(proposals, top, prob, hw, min_size, score_thresh)

    def anchors_level(self, size, ratios, gh, gw, sh, sw, device):
        return ops.anchors_level(size, ratios, gh, gw, sh, sw, device)

    def normalize_pad_u8(self, images_u8, padded_hw):
        return ops.normalize_pad(images_u8, padded_hw, channels=self.stem_channels, dtype=self.act_dtype)

    def resize_normalize_pad_u8(self, images_u8, out_sizes, padded_hw):
        return ops.resize_normalize_pad(images_u8, out_sizes, padded_hw, channels=self.stem_channels,
                                        dtype=self.act_dtype)


_default = {}


def default_backend():
    """The process's HipBackend for the current MX_PRECISION (one instance per precision)."""
    p = default_precision()
    if p not in _default:
        _default[p] = HipBackend(p)
    return _default[p]
