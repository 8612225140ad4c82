"""torch-facing wrappers of libmx_det (the HIP hot path).

Mirrors the torchvision operator surface the reference reaches:
  nms(boxes, scores, iou_threshold) / batched_nms(boxes, scores, idxs, iou_threshold)
      torchvision/ops/boxes.py (RPN filter_proposals, RoIHeads.postprocess_detections)
  roi_align(input, boxes, output_size, spatial_scale, sampling_ratio, aligned)
      torchvision/ops/roi_align.py (here on NHWC features)
  box_iou(boxes1, boxes2)                      torchvision/ops/boxes.py
plus fused ops the build adds (match_assign, multiscale_roi_align, anchors_level, box_decode,
corrupt_u8, normalize_pad). Errors follow torchvision's TORCH_CHECK style: RuntimeError on bad
rank/shape/device; empty inputs give empty outputs.
"""
import ctypes
import math
import os

import torch

from . import _lib
from ._lib import call

MX_F32, MX_BF16 = 0, 1
BBOX_CLIP = math.log(1000.0 / 16)


def _stream():
    return _lib.stream()


def _p(t):
    return t.data_ptr() if t is not None else None


def _check(cond, msg):
    if not cond:
        raise RuntimeError(msg)


def _dev(*ts):
    for t in ts:
        _check(t.is_cuda, "mx_det ops take CUDA (HIP) tensors")


def _dtype_code(t):
    if t.dtype == torch.float32:
        return MX_F32
    if t.dtype == torch.bfloat16:
        return MX_BF16
    raise RuntimeError(f"unsupported dtype {t.dtype}")


def _ws(nbytes, device):
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


# ---------------------------------------------------------------------------------------------
def box_iou(boxes1, boxes2):
    _dev(boxes1, boxes2)
    b1 = boxes1.float().contiguous().view(-1, 4)
    b2 = boxes2.float().contiguous().view(-1, 4)
    out = torch.empty((b1.shape[0], b2.shape[0]), dtype=torch.float32, device=b1.device)
    if out.numel():
        call("mx_box_iou", _p(b1), b1.shape[0], _p(b2), b2.shape[0], _p(out), _stream())
    return out


def match_assign(gt_boxes, boxes, high, low, allow_low_quality, mode=0, gt_labels=None, weights=None):
    """Fused box_iou + Matcher (+ labels / encoded regression targets).

    mode 0 -> matches; mode 1 (RPN) -> (matches, labels f32 1/0/-1, targets);
    mode 2 (RoI) -> (matches, labels i64, targets). See include/mx_det.h mx_match_assign.
    """
    _dev(gt_boxes, boxes)
    gt = gt_boxes.float().contiguous().view(-1, 4)
    bx = boxes.float().contiguous().view(-1, 4)
    G, A = gt.shape[0], bx.shape[0]
    dev = bx.device
    matches = torch.empty(A, dtype=torch.int64, device=dev)
    labels = None
    if mode == 1:
        labels = torch.empty(A, dtype=torch.float32, device=dev)
    elif mode == 2:
        labels = torch.empty(A, dtype=torch.int64, device=dev)
        _check(gt_labels is not None, "mode 2 needs gt_labels")
        gt_labels = gt_labels.to(torch.int64).contiguous()
    targets = torch.empty((A, 4), dtype=torch.float32, device=dev) if weights is not None else None
    w = (_lib.F4)(*weights) if weights is not None else None
    ws = _ws(_lib.load().mx_match_workspace(G, A), dev)
    call("mx_match_assign", _p(gt), _p(gt_labels) if mode == 2 else None, G, _p(bx), A, float(high), float(low),
         int(bool(allow_low_quality)), int(mode), w, _p(matches), _p(labels), _p(targets), _p(ws), ws.numel(),
         _stream())
    if mode == 0:
        return matches
    return matches, labels, targets


def match_assign_batched(gt_pad, gcount, boxes, high, low, allow_low_quality, mode, gt_labels=None, weights=None,
                         with_counts=False):
    """match_assign for B images in one launch pair: gt_pad [B, G, 4] (rows >= gcount[b] are padding),
    gcount int32 [B] on the device, boxes [A, 4] shared by every image or [B, A, 4]. Returns
    (matches [B, A], labels [B, A], targets [B, A, 4]) as match_assign's modes 1 / 2, plus with_counts
    the per-image (matched, background) counts int32 [B, 2]."""
    _dev(gt_pad, boxes, gcount)
    _check(gt_pad.dim() == 3 and gt_pad.shape[2] == 4, "gt_pad must be [B, G, 4]")
    B, G = gt_pad.shape[0], gt_pad.shape[1]
    gt = gt_pad.float().contiguous()
    bx = boxes.float().contiguous()
    shared = bx.dim() == 2
    _check(shared or (bx.dim() == 3 and bx.shape[0] == B), "boxes must be [A, 4] or [B, A, 4]")
    A = bx.shape[-2]
    dev = bx.device
    gc = gcount.to(torch.int32).contiguous()
    matches = torch.empty((B, A), dtype=torch.int64, device=dev)
    labels = torch.empty((B, A), dtype=torch.float32 if mode == 1 else torch.int64, device=dev) if mode else None
    if mode == 2:
        _check(gt_labels is not None and gt_labels.shape[:2] == (B, G), "mode 2 needs gt_labels [B, G]")
        gt_labels = gt_labels.to(torch.int64).contiguous()
    targets = torch.empty((B, A, 4), dtype=torch.float32, device=dev) if weights is not None else None
    w = (_lib.F4)(*weights) if weights is not None else None
    ws = _ws(_lib.load().mx_match_batched_workspace(B, G, A), dev)
    counts = torch.empty((B, 2), dtype=torch.int32, device=dev) if with_counts else None
    call("mx_match_assign_batched", _p(gt), _p(gt_labels) if mode == 2 else None, _p(gc), B, G, _p(bx),
         0 if shared else A, A, float(high), float(low), int(bool(allow_low_quality)), int(mode), w, _p(matches),
         _p(labels), _p(targets), _p(counts) if counts is not None else None, _p(ws), ws.numel(), _stream())
    return (matches, labels, targets, counts) if with_counts else (matches, labels, targets)


def pad_gt(targets, dev, multiple=32):
    """Per-image target boxes / labels -> zero-padded [B, G, 4] / [B, G] batches (G = the largest count
    rounded up to `multiple`, so a few static shapes recur) + the real counts (int32 [B], device)."""
    B = len(targets)
    counts = [int(t["boxes"].shape[0]) for t in targets]
    G = max(multiple, -(-max(counts) // multiple) * multiple) if B else multiple
    boxes = torch.zeros((B, G, 4), dtype=torch.float32, device=dev)
    labels = torch.zeros((B, G), dtype=torch.int64, device=dev)
    for i, t in enumerate(targets):
        if counts[i]:
            boxes[i, :counts[i]] = t["boxes"]
            labels[i, :counts[i]] = t["labels"]
    return boxes, labels, torch.tensor(counts, dtype=torch.int32).to(dev, non_blocking=True)


# ---------------------------------------------------------------------------------------------
def batched_nms(boxes, scores, idxs, iou_threshold, group=None, max_seg=None, mode=0):
    """torchvision.ops.batched_nms (CPU dispatch semantics). idxs=None -> plain nms.

    group: optional int tensor; output ordered by (group, score desc).
    Returns int64 indices of kept boxes.
    """
    _dev(boxes, scores)
    _check(boxes.dim() == 2 and boxes.shape[-1] == 4, f"boxes should be [N,4], got {tuple(boxes.shape)}")
    _check(scores.dim() == 1 and scores.shape[0] == boxes.shape[0], "scores should be [N]")
    n = boxes.shape[0]
    dev = boxes.device
    if n == 0:
        return torch.empty(0, dtype=torch.int64, device=dev)
    b = boxes.float().contiguous()
    s = scores.float().contiguous()
    ix = idxs.to(torch.int64).contiguous() if idxs is not None else None
    g = group.to(torch.int32).contiguous() if group is not None else None
    ms = int(max_seg) if max_seg else n
    keep = torch.empty(n, dtype=torch.int64, device=dev)
    nk = torch.empty(1, dtype=torch.int64, device=dev)
    ws = _ws(_lib.load().mx_nms_workspace(n, ms), dev)
    call("mx_batched_nms", _p(b), _p(s), _p(ix), _p(g), n, ms, float(iou_threshold), int(mode), _p(keep), _p(nk),
         _p(ws), ws.numel(), _stream())
    k = int(nk.item())
    _check(k >= 0, "batched_nms: a class segment exceeded max_seg")
    return keep[:k]


def batched_nms_grouped(boxes, scores, lvl, group, G, L, iou_threshold, max_seg):
    """All images of RegionProposalNetwork.filter_proposals in one NMS (mx_batched_nms_grouped):
    box i is in image group[i] (>= G: dead) and level lvl[i]; torchvision's per-image CPU dispatch
    rule (4n > 4000 -> per level, else coordinate trick) is applied per image on the device.
    Returns (keep [n] int64, num_keep [1] int64) on the device: keep[:num_keep] ordered by
    (image, score desc, index). No host synchronisation."""
    _dev(boxes, scores)
    n = boxes.shape[0]
    dev = boxes.device
    keep = torch.empty(n, dtype=torch.int64, device=dev)
    nk = torch.zeros(1, dtype=torch.int64, device=dev)
    if n == 0:
        return keep, nk
    b = boxes.float().contiguous()
    s = scores.float().contiguous()
    lv = lvl.to(torch.int64).contiguous()
    g = group.to(torch.int32).contiguous()
    ws = _ws(_lib.load().mx_nms_grouped_workspace(n, G, max_seg), dev)
    call("mx_batched_nms_grouped", _p(b), _p(s), _p(lv), _p(g), n, G, L, int(max_seg), float(iou_threshold),
         _p(keep), _p(nk), _p(ws), ws.numel(), _stream())
    return keep, nk


SORTED_NMS_MAX = (24576, 64, 8)  # n, G, L bounds of mx_batched_nms_grouped_sorted


def batched_nms_grouped_sorted(boxes, scores, lvl, group, G, L, iou_threshold, max_seg, post=0):
    """batched_nms_grouped for presorted candidates (mx_batched_nms_grouped_sorted: live entries
    image-major, level-major, score-descending per (image, level) run -- filter_proposals' per-level
    top-k layout; a run out of order is still ranked exactly). Same (keep, num_keep); with post > 0
    also (sel [G, post] int64, valid [G, post] bool): per image its first `post` survivors (score
    order), 0 / False past its count. Falls back to batched_nms_grouped outside the size bounds."""
    _dev(boxes, scores)
    n = boxes.shape[0]
    dev = boxes.device
    if n > SORTED_NMS_MAX[0] or G > SORTED_NMS_MAX[1] or L > SORTED_NMS_MAX[2]:
        keep, nk = batched_nms_grouped(boxes, scores, lvl, group, G, L, iou_threshold, max_seg)
        if not post:
            return keep, nk
        cnt = torch.zeros(G + 1, dtype=torch.int64, device=dev)
        live = torch.arange(n, device=dev) < nk
        cnt.scatter_add_(0, torch.where(live, group.to(torch.int64)[keep], G), live.to(torch.int64))
        cnt = cnt[:G]
        r = torch.arange(post, device=dev)
        valid = r[None, :] < cnt[:, None]
        sel = torch.where(valid, keep[((torch.cumsum(cnt, 0) - cnt)[:, None] + r[None, :]).clamp(max=max(n - 1, 0))], 0)
        return keep, nk, sel, valid
    keep = torch.empty(n, dtype=torch.int64, device=dev)
    nk = torch.zeros(1, dtype=torch.int64, device=dev)
    sel = torch.empty((G, post), dtype=torch.int64, device=dev) if post else None
    valid = torch.empty((G, post), dtype=torch.bool, device=dev) if post else None
    b = boxes.float().contiguous()
    s = scores.float().contiguous()
    lv = lvl.to(torch.int64).contiguous()
    g = group.to(torch.int32).contiguous()
    ws = _ws(_lib.load().mx_nms_grouped_workspace(max(n, 1), G, max_seg), dev)
    call("mx_batched_nms_grouped_sorted", _p(b), _p(s), _p(lv), _p(g), n, G, L, int(max_seg), float(iou_threshold),
         _p(keep), _p(nk), int(post), _p(sel) if post else None, _p(valid) if post else None, _p(ws), ws.numel(),
         _stream())
    return (keep, nk) if not post else (keep, nk, sel, valid)


def proposal_clip_filter(proposals, top, prob, hw, min_size, score_thresh):
    """filter_proposals' clip + small-box + score filter after the per-level top-k (one launch):
    proposals [N, A, 4] f32, top [N, T] int64, prob [N, T] f32, hw [N, 2] (h, w) f32 ->
    (boxes [N, T, 4] clipped, grp [N*T] int32: the image index, or N for a dropped candidate)."""
    _dev(proposals, top, prob, hw)
    N, A = proposals.shape[0], proposals.shape[1]
    T = top.shape[1]
    _check(top.dtype == torch.int64 and top.shape[0] == N and prob.shape == top.shape and hw.shape == (N, 2),
           "proposal_clip_filter: shapes")
    p = proposals.float().contiguous()
    boxes = torch.empty((N, T, 4), dtype=torch.float32, device=p.device)
    grp = torch.empty(N * T, dtype=torch.int32, device=p.device)
    call("mx_proposal_clip_filter", _p(p), _p(top.contiguous()), _p(prob.float().contiguous()),
         _p(hw.float().contiguous()), N, A, T, float(min_size), float(score_thresh), _p(boxes), _p(grp), _stream())
    return boxes, grp


def boxes_degenerate(boxes_list, out=None):
    """One device bool flag: any box (x1, y1, x2, y2) of the list's tensors with x2 <= x1 or y2 <= y1
    (mx_boxes_degenerate, up to 8 tensors per launch)."""
    _dev(*boxes_list)
    dev = boxes_list[0].device
    flags = []
    for c in range(0, len(boxes_list), 8):
        chunk = [b.float().contiguous() for b in boxes_list[c:c + 8]]
        f = out if (out is not None and len(boxes_list) <= 8) else torch.empty(1, dtype=torch.bool, device=dev)
        ptrs = (ctypes.c_void_p * len(chunk))(*[b.data_ptr() for b in chunk])
        cnts = (ctypes.c_int64 * len(chunk))(*[b.shape[0] for b in chunk])
        call("mx_boxes_degenerate", ptrs, cnts, len(chunk), _p(f), _stream())
        flags.append(f)
    return (flags[0] if len(flags) == 1 else torch.cat(flags).any()).reshape(())


def roi_compact(mask, total, cm, box, lab, tg):
    """select_training_samples' gather after the sampler: the `total` True entries of the flat mask
    (ascending) -> (rois [total, 5] = (entry // cm, box), labels [total] int64, targets [total, 4])."""
    _dev(mask, box, lab, tg)
    M = mask.numel()
    _check(mask.dtype == torch.bool and box.shape == (M, 4) and lab.shape == (M,) and tg.shape == (M, 4),
           "roi_compact: shapes")
    dev = mask.device
    rois = torch.empty((total, 5), dtype=torch.float32, device=dev)
    lo = torch.empty(total, dtype=torch.int64, device=dev)
    to = torch.empty((total, 4), dtype=torch.float32, device=dev)
    call("mx_roi_compact", _p(mask.contiguous()), M, int(total), int(cm), _p(box.float().contiguous()),
         _p(lab.to(torch.int64).contiguous()), _p(tg.float().contiguous()), _p(rois), _p(lo), _p(to), _stream())
    return rois, lo, to


SAMPLE_SLICED_MIN = 16384  # mx_sample_draw_ws's threshold (rows at most this long: one workgroup per row)


def roi_candidates(pb, pvalid, gtp, gcnt):
    """select_training_samples' candidate rows in one launch (mx_roi_candidates): per image the padded
    proposals pb [N, post, 4] (valid where pvalid) then the padded GT gtp [N, gm, 4] (valid below gcnt,
    int32 [N]) -> (boxes [N, post + gm, 4], valid bool [N, post + gm])."""
    _dev(pb, pvalid, gtp, gcnt)
    N, post = pvalid.shape
    gm = gtp.shape[1]
    _check(pb.shape == (N, post, 4) and gtp.shape == (N, gm, 4) and gcnt.shape == (N,), "roi_candidates: shapes")
    _check(pb.dtype == torch.float32 and gtp.dtype == torch.float32 and pvalid.dtype == torch.bool
           and gcnt.dtype == torch.int32, "roi_candidates: dtypes")
    box = torch.empty((N, post + gm, 4), dtype=torch.float32, device=pb.device)
    valid = torch.empty((N, post + gm), dtype=torch.uint8, device=pb.device)
    call("mx_roi_candidates", _p(pb.contiguous()), _p(pvalid.contiguous()), _p(gtp.contiguous()), _p(gcnt.contiguous()),
         N, post, gm, _p(box), _p(valid), _stream())
    return box, valid.view(torch.bool)


def sample_draw(labels, keys, batch, positive_fraction, with_union=False, sliced=True, valid=None):
    """BalancedPositiveNegativeSampler's draw in one launch (mx_sample_draw): labels [N, L] (float32: the
    RPN's 1 / 0 / -1, or int64: the RoI head's class / 0 / -1), keys [N, L] uniform -> (pos, neg bool
    [N, L], union bool [N, L] or None, nums int32 [N, 2] = (num_pos, num_neg)); per row the num smallest
    keys of each class's candidates, ties by lowest index. valid (bool [N, L], optional): entries where it
    is False belong to neither class (the RoI head's padding slots)."""
    _dev(labels, keys)
    _check(labels.dim() == 2 and keys.shape == labels.shape and keys.dtype == torch.float32, "sample_draw: shapes")
    _check(labels.dtype in (torch.float32, torch.int64), "sample_draw: labels must be float32 or int64")
    N, L = labels.shape
    dev = labels.device
    pos = torch.empty((N, L), dtype=torch.uint8, device=dev)
    neg = torch.empty_like(pos)
    un = torch.empty_like(pos) if with_union else None
    nums = torch.empty((N, 2), dtype=torch.int32, device=dev)
    lab, ky, ld = labels.contiguous(), keys.contiguous(), 0 if labels.dtype == torch.float32 else 2
    if valid is not None:
        _check(valid.shape == labels.shape and valid.dtype == torch.bool and valid.device == dev, "sample_draw: valid")
        valid = valid.contiguous()
    vp = _p(valid)
    if L > SAMPLE_SLICED_MIN and sliced:  # the RPN's long rows: split over many workgroups
        nb = _lib.load().mx_sample_draw_workspace(N, L)
        ws = torch.empty(nb, dtype=torch.uint8, device=dev)
        call("mx_sample_draw_ws", _p(lab), ld, vp, _p(ky), N, L, int(batch), float(positive_fraction), _p(pos),
             _p(neg), _p(un), _p(nums), _p(ws), nb, _stream())
    else:
        call("mx_sample_draw", _p(lab), ld, vp, _p(ky), N, L, int(batch), float(positive_fraction), _p(pos), _p(neg),
             _p(un), _p(nums), _stream())
    return pos.view(torch.bool), neg.view(torch.bool), (un.view(torch.bool) if un is not None else None), nums


def level_topk(scores, num_per_level, k):
    """RegionProposalNetwork._get_top_n_idx (torchvision rpn.py): per image row of scores [N, A] and
    per level, the indices of the min(k, n_l) largest scores (value descending, ties by index) plus
    the level offset, levels concatenated -> [N, sum_l min(k, n_l)] int64 (mx_level_topk; one launch)."""
    _dev(scores)
    _check(scores.dim() == 2, f"scores should be [N, A], got {tuple(scores.shape)}")
    s = scores.float().contiguous()
    N, A = s.shape
    L = len(num_per_level)
    offs = [0]
    for n in num_per_level[:-1]:
        offs.append(offs[-1] + int(n))
    _check(offs[-1] + int(num_per_level[-1]) <= A, "level_topk: levels exceed the row")
    tot = sum(min(int(k), int(n)) for n in num_per_level)
    out = torch.empty((N, tot), dtype=torch.int64, device=s.device)
    ln = (ctypes.c_int64 * L)(*[int(n) for n in num_per_level])
    # long levels are sliced over many workgroups and merged (MX_TOPK_SLICED=0: one workgroup per level)
    nb = _lib.load().mx_level_topk_workspace(N, L, ln) if os.environ.get("MX_TOPK_SLICED", "1") != "0" else 0
    ws = _ws(nb, s.device) if nb else None
    call("mx_level_topk_ws", _p(s), N, A, L, (ctypes.c_int64 * L)(*offs), ln, int(k), _p(out),
         _p(ws) if ws is not None else None, int(nb), _stream())
    return out


def nms(boxes, scores, iou_threshold):
    """torchvision.ops.nms: kept indices sorted by decreasing score."""
    return batched_nms(boxes, scores, None, iou_threshold)


# ---------------------------------------------------------------------------------------------
def roi_align_deterministic(C, ph=7, pw=7, sampling=2):
    """The RoIAlign backward runs the atomic-free gather (bitwise reproducible, writes every element
    of the gradient maps) unless MX_ROI_DETERMINISTIC=0 or the shape is outside its supported set
    (C % 4 == 0, C <= 256, ph * pw <= 64, 1 <= sampling <= 4)."""
    import os
    return (os.environ.get("MX_ROI_DETERMINISTIC", "1") != "0" and 4 <= C <= 256 and C % 4 == 0 and ph * pw <= 64
            and 1 <= sampling <= 4)


def roi_align_fwd_nhwc(feat, rois, scale, ph, pw, sampling, aligned):
    """mx_roi_align_fwd on NHWC features: rois [K,5] f32 -> [K, ph, pw, C] in the feature dtype."""
    _dev(feat, rois)
    _check(feat.dim() == 4, "roi_align input must be NHWC [N,H,W,C]")
    _check(rois.dim() == 2 and rois.shape[1] == 5, f"rois must be [K,5], got {tuple(rois.shape)}")
    f = feat.contiguous()
    r = rois.float().contiguous()
    N, H, W, C = f.shape
    out = torch.empty((r.shape[0], ph, pw, C), dtype=f.dtype, device=f.device)
    if r.shape[0]:
        call("mx_roi_align_fwd", _p(f), _dtype_code(f), N, H, W, C, _p(r), r.shape[0], float(scale), ph, pw,
             sampling, int(aligned), _p(out), _stream())
    return out


def roi_align_bwd_nhwc(gout, rois, N, H, W, C, scale, ph, pw, sampling, aligned):
    """mx_roi_align_bwd: gout [K, ph, pw, C] -> f32 grad_feat [N, H, W, C] (deterministic gather when
    supported, see roi_align_deterministic; else atomics into a zero-filled map)."""
    g = gout.contiguous()
    r = rois.float().contiguous()
    K = r.shape[0]
    det = roi_align_deterministic(C, ph, pw, sampling)
    gf = (torch.empty if det else torch.zeros)((N, H, W, C), dtype=torch.float32, device=g.device)
    ws = _ws(_lib.load().mx_roi_align_bwd_workspace(K, ph, pw, sampling) if det else 0, g.device)
    call("mx_roi_align_bwd", _p(g), _dtype_code(g), N, H, W, C, _p(r), K, float(scale), ph, pw, sampling,
         int(aligned), _p(gf), int(det), _p(ws), ws.numel(), _stream())
    return gf


class _RoIAlign(torch.autograd.Function):
    @staticmethod
    def forward(ctx, feat, rois, scale, ph, pw, sampling, aligned):
        out = roi_align_fwd_nhwc(feat, rois, scale, ph, pw, sampling, aligned)
        ctx.save_for_backward(rois.float().contiguous())
        N, H, W, C = feat.shape
        ctx.cfg = (N, H, W, C, float(scale), ph, pw, sampling, int(aligned), feat.dtype)
        return out

    @staticmethod
    def backward(ctx, gout):
        (r,) = ctx.saved_tensors
        N, H, W, C, scale, ph, pw, sampling, aligned, dt = ctx.cfg
        gf = roi_align_bwd_nhwc(gout, r, N, H, W, C, scale, ph, pw, sampling, aligned)
        return gf.to(dt), None, None, None, None, None, None


def roi_align(input, boxes, output_size, spatial_scale=1.0, sampling_ratio=2, aligned=False):
    """torchvision.ops.roi_align on NHWC input; boxes = Tensor[K,5] (batch, x1, y1, x2, y2).
    Returns [K, PH, PW, C]."""
    if isinstance(output_size, int):
        output_size = (output_size, output_size)
    return _RoIAlign.apply(input, boxes, spatial_scale, output_size[0], output_size[1], sampling_ratio, aligned)


def grad_buffer(t, dtype=torch.float32):
    """The buffer a HIP-graph replay will copy `t`'s gradient into (frcnn._GraphFn tags the tensors it
    returns with it): a backward that writes the gradient there directly saves that copy."""
    b = getattr(t, "_mx_gbuf", None)
    if b is not None and b.shape == t.shape and b.dtype == dtype and b.device == t.device and b.is_contiguous():
        return b
    return None


class _CanvasPack(torch.autograd.Function):
    @staticmethod
    def forward(ctx, rects, Hc, Wc, slots, *maps):
        _dev(*maps)
        N, C, dt = maps[0].shape[0], maps[0].shape[3], maps[0].dtype
        for m in maps:
            _check(m.dim() == 4 and m.shape[0] == N and m.shape[3] == C and m.dtype == dt and m.is_contiguous(),
                   "canvas: maps must be contiguous NHWC of one N, C and dtype")
        n = len(maps)
        r = (ctypes.c_int32 * (4 * n))(*[v for rc in rects for v in rc])
        cv = torch.empty((N, Hc, Wc, C), dtype=dt, device=maps[0].device)
        call("mx_canvas_pack", (ctypes.c_void_p * n)(*[m.data_ptr() for m in maps]), r, n, N, Hc, Wc, C,
             _dtype_code(maps[0]), _p(cv), _stream())
        ctx.cfg = (r, n, N, Hc, Wc, C, [tuple(m.shape) for m in maps], slots)
        return cv

    @staticmethod
    def backward(ctx, gcv):
        r, n, N, Hc, Wc, C, shapes, slots = ctx.cfg
        g = gcv.contiguous()
        grads = [torch.empty(s, dtype=g.dtype, device=g.device) for s in shapes]
        adds = [s.buf if s is not None and s.buf is not None else None for s in (slots or [None] * n)]
        for a, s in zip(adds, shapes):
            _check(a is None or (tuple(a.shape) == s and a.dtype == g.dtype and a.is_contiguous()),
                   "canvas: absorbed gradient must match its map")
        addp = (ctypes.c_void_p * n)(*[a.data_ptr() if a is not None else None for a in adds])
        call("mx_canvas_unpack", _p(g), r, n, N, Hc, Wc, C, _dtype_code(g), addp,
             (ctypes.c_void_p * n)(*[x.data_ptr() for x in grads]), _stream())
        return (None, None, None, None) + tuple(grads)


def canvas_pack(maps, rects, Hc, Wc, slots=None):
    """Zero canvas [N, Hc, Wc, C] holding maps[l] at rects[l] = (y, x, h, w) (one launch each way);
    slots[l].buf, when set, is added to map l's gradient in the backward (conv.GradSlot; the slots are
    claimed here, on the stream the backward's unpack will run on)."""
    if slots is not None and maps and maps[0].is_cuda:
        st = torch.cuda.current_stream(maps[0].device).cuda_stream
        for sl in slots:
            if sl is not None:
                sl.stream = st
                sl.claim()
    return _CanvasPack.apply([tuple(int(v) for v in rc) for rc in rects], int(Hc), int(Wc), slots,
                             *[m.contiguous() for m in maps])


class _MaskPixels(torch.autograd.Function):
    """t * mask for a per-pixel 0 / 1 mask (mx_mask_pixels both ways); planes_krs > 0: the output's bf16x3
    planes for the next conv (f32, policy conv.planes_for), attached as y._mx_planes."""

    @staticmethod
    def forward(ctx, x, maskf, planes_krs):
        from . import conv as mc
        x = x.contiguous()
        N, H, W, C = x.shape
        y = torch.empty_like(x)
        pl = None
        if planes_krs and x.dtype == torch.float32 and mc.planes_for(x.numel(), C, planes_krs):
            pl = torch.empty((2,) + tuple(x.shape), dtype=torch.bfloat16, device=x.device)
        call("mx_mask_pixels", _p(x), _dtype_code(x), _p(maskf), N, H * W, C, _p(y), _p(pl), _stream())
        if pl is not None:
            y._mx_planes = pl
        ctx.save_for_backward(maskf)
        return y

    @staticmethod
    def backward(ctx, g):
        (maskf,) = ctx.saved_tensors
        g = g.contiguous()
        N, H, W, C = g.shape
        gx = torch.empty_like(g)
        call("mx_mask_pixels", _p(g), _dtype_code(g), _p(maskf), N, H * W, C, _p(gx), None, _stream())
        return gx, None, None


def mask_pixels(x, maskf, planes_krs=0):
    """RPNHead's canvas frame mask: x [N, H, W, C] * maskf [H, W] (f32 0 / 1), one launch each way."""
    _dev(x, maskf)
    _check(x.dim() == 4 and x.shape[3] % 8 == 0 and maskf.numel() == x.shape[1] * x.shape[2]
           and maskf.dtype == torch.float32 and x.dtype in (torch.float32, torch.bfloat16), "mask_pixels: shapes")
    return _MaskPixels.apply(x, maskf.contiguous(), int(planes_krs))


class _RPNHeadSplit(torch.autograd.Function):
    @staticmethod
    def forward(ctx, o0, ocv, rects, A):
        _dev(o0, *([ocv] if ocv is not None else []))
        N, H0, W0, C = o0.shape
        _check(C == 5 * A and o0.dtype == torch.float32 and o0.is_contiguous(), "rpn head split: o0 must be f32 [N,H,W,5A]")
        ncv = len(rects)
        Hc = Wc = 0
        if ncv:
            _check(ocv is not None and ocv.shape[0] == N and ocv.shape[3] == C and ocv.dtype == torch.float32
                   and ocv.is_contiguous(), "rpn head split: bad canvas")
            Hc, Wc = ocv.shape[1], ocv.shape[2]
        r = (ctypes.c_int32 * max(1, 4 * ncv))(*[v for rc in rects for v in rc])
        atot = H0 * W0 * A + sum(h * w * A for _, _, h, w in rects)
        obj = torch.empty((N, atot), dtype=torch.float32, device=o0.device)
        dl = torch.empty((N, atot, 4), dtype=torch.float32, device=o0.device)
        call("mx_rpn_head_split", _p(o0), H0, W0, _p(ocv) if ncv else None, Hc, Wc, r, ncv, N, A, _p(obj), _p(dl),
             _stream())
        ctx.cfg = (N, H0, W0, Hc, Wc, r, ncv, A)
        ctx.gbufs = (grad_buffer(o0), grad_buffer(ocv) if ncv else None)
        ctx.shapes = (o0.shape, ocv.shape if ncv else None)
        return obj, dl

    @staticmethod
    def backward(ctx, gobj, gdl):
        N, H0, W0, Hc, Wc, r, ncv, A = ctx.cfg
        s0, scv = ctx.shapes
        b0, bcv = ctx.gbufs
        dev = (gobj if gobj is not None else gdl).device
        g0 = b0 if b0 is not None else torch.empty(s0, dtype=torch.float32, device=dev)
        gcv = (bcv if bcv is not None else torch.empty(scv, dtype=torch.float32, device=dev)) if ncv else None
        gobj = gobj.contiguous() if gobj is not None else None
        gdl = gdl.contiguous() if gdl is not None else None
        call("mx_rpn_head_merge", _p(gobj) if gobj is not None else None, _p(gdl) if gdl is not None else None,
             H0, W0, Hc, Wc, r, ncv, N, A, _p(g0), _p(gcv) if ncv else None, _stream())
        return g0, gcv, None, None


def rpn_head_split(o0, ocv, rects, A):
    """RPN head outputs (level 0 map, zero-framed canvas of the other levels at rects (y, x, h, w)) ->
    (objectness [N, Atot], pred_deltas [N, Atot, 4]) in torchvision's concat_box_prediction_layers order;
    autograd-aware (one launch each way)."""
    return _RPNHeadSplit.apply(o0, ocv, [tuple(int(v) for v in rc) for rc in rects], int(A))


class _MultiScaleRoIAlign(torch.autograd.Function):
    @staticmethod
    def forward(ctx, rois, scales, k_min, ph, pw, sampling, *feats):
        _dev(rois, *feats)
        r = rois.float().contiguous()
        fs = [f.contiguous() for f in feats]
        C = fs[0].shape[3]
        dt = fs[0].dtype
        for f in fs:
            _check(f.dim() == 4 and f.shape[3] == C and f.dtype == dt, "features must share C and dtype")
        n = len(fs)
        K = r.shape[0]
        out = torch.empty((K, ph, pw, C), dtype=dt, device=r.device)
        levels = torch.empty(K, dtype=torch.int32, device=r.device)
        ptrs = (ctypes.c_void_p * n)(*[f.data_ptr() for f in fs])
        Hs = (ctypes.c_int64 * n)(*[f.shape[1] for f in fs])
        Ws = (ctypes.c_int64 * n)(*[f.shape[2] for f in fs])
        sc = (ctypes.c_float * n)(*scales)
        if K:
            call("mx_multiscale_roi_align_fwd", ptrs, Hs, Ws, sc, n, int(k_min), _dtype_code(fs[0]), C, _p(r), K, ph,
                 pw, sampling, _p(out), _p(levels), _stream())
        ctx.save_for_backward(r, levels)
        ctx.cfg = ([tuple(f.shape) for f in fs], list(scales), ph, pw, sampling, dt)
        ctx.gbufs = [grad_buffer(f) for f in feats] if dt == torch.float32 else None
        return out

    @staticmethod
    def backward(ctx, gout):
        r, levels = ctx.saved_tensors
        shapes, scales, ph, pw, sampling, dt = ctx.cfg
        gfs = multiscale_roi_align_backward(gout, r, levels, shapes, scales, ph, pw, sampling, out=ctx.gbufs)
        return (None, None, None, None, None, None) + tuple(x.to(dt) for x in gfs)


def multiscale_roi_align_backward(gout, rois, levels, shapes, scales, ph=7, pw=7, sampling=2, out=None):
    """torchvision _roi_align_backward over the pyramid: grad_out [K,ph,pw,C] -> f32 NHWC gradients of
    the level maps `shapes` (deterministic gather when the shape allows it, else atomics). out: optional
    per-level f32 buffers to write into (None entries allocated)."""
    g = gout.contiguous()
    C, K = shapes[0][3], rois.shape[0]
    det = roi_align_deterministic(C, ph, pw, sampling)
    gfs = []
    for i, s in enumerate(shapes):
        b = out[i] if out is not None and i < len(out) else None
        if b is None or tuple(b.shape) != tuple(s):
            b = (torch.empty if det else torch.zeros)(s, dtype=torch.float32, device=g.device)
        elif not det:
            b.zero_()
        gfs.append(b)
    n = len(gfs)
    ws = _ws(_lib.load().mx_roi_align_bwd_workspace(K, ph, pw, sampling) if det else 0, g.device)
    ptrs = (ctypes.c_void_p * n)(*[f.data_ptr() for f in gfs])
    Hs = (ctypes.c_int64 * n)(*[s[1] for s in shapes])
    Ws = (ctypes.c_int64 * n)(*[s[2] for s in shapes])
    sc = (ctypes.c_float * n)(*scales)
    call("mx_multiscale_roi_align_bwd", _p(g), _dtype_code(g), ptrs, shapes[0][0], Hs, Ws, sc, n, C, _p(rois),
         _p(levels), K, ph, pw, sampling, int(det), _p(ws), ws.numel(), _stream())
    return gfs


def multiscale_roi_align(feats, rois, scales, k_min, output_size=(7, 7), sampling_ratio=2):
    """MultiScaleRoIAlign over NHWC feature maps with the fused LevelMapper. rois [K,5]."""
    return _MultiScaleRoIAlign.apply(rois, list(scales), int(k_min), output_size[0], output_size[1],
                                     sampling_ratio, *feats)


# ---------------------------------------------------------------------------------------------
def anchors_level(size, ratios, grid_h, grid_w, stride_h, stride_w, device):
    nr = len(ratios)
    out = torch.empty((grid_h * grid_w * nr, 4), dtype=torch.float32, device=device)
    if out.numel():
        rr = (ctypes.c_float * nr)(*ratios)
        call("mx_anchors_level", float(size), rr, nr, grid_h, grid_w, int(stride_h), int(stride_w), _p(out),
             _stream())
    return out


def box_decode(rel_codes, boxes, weights, clip=BBOX_CLIP):
    """BoxCoder.decode_single: rel [n, ncls*4] against boxes [n,4] -> [n, ncls*4]."""
    _dev(rel_codes, boxes)
    b = boxes.float().contiguous().view(-1, 4)
    n = b.shape[0]
    r = rel_codes.float().contiguous().view(n, -1)
    out = torch.empty_like(r)
    if n:
        call("mx_box_decode", _p(r), _p(b), n, r.shape[1] // 4, (_lib.F4)(*weights), float(clip), _p(out),
             _stream())
    return out


# ---------------------------------------------------------------------------------------------
CORRUPT_NONE, CORRUPT_NOISE, CORRUPT_BLUR, CORRUPT_LOWRES = 0, 1, 2, 3


def corrupt_u8(images, ops, sigma=15.0, seed=0, noise=None, factor=0.5):
    """augmentations.py corruption ops on uint8 [B,H,W,C] (one op code per image)."""
    _dev(images)
    _check(images.dtype == torch.uint8 and images.dim() == 4, "images must be uint8 [B,H,W,C]")
    x = images.contiguous()
    B, H, W, C = x.shape
    out = torch.empty_like(x)
    nw, nh = max(1, int(W * factor)), max(1, int(H * factor))
    tmp = torch.empty((B, nh, nw, C), dtype=torch.uint8, device=x.device) if 3 in list(ops) else None
    if noise is not None:
        noise = noise.float().contiguous()
        _check(noise.numel() == x.numel(), "noise field must match images")
    arr = (ctypes.c_int32 * B)(*[int(o) for o in ops])
    call("mx_corrupt_u8", _p(x), B, H, W, C, arr, float(sigma), ctypes.c_uint64(int(seed) & (2 ** 64 - 1)),
         _p(noise), float(factor), _p(tmp), _p(out), _stream())
    return out


def filter2d_u8(images, taps):
    """cv2.filter2D(img, -1, kernel) on uint8 [B,H,W,C] device images; taps = the kernel's non-zero
    coefficients as (dy, dx, coef) rows relative to the centre anchor, row-major (mx_filter2d_u8)."""
    _dev(images)
    _check(images.dtype == torch.uint8 and images.dim() == 4, "images must be uint8 [B,H,W,C]")
    x = images.contiguous()
    B, H, W, C = x.shape
    t = [float(v) for row in taps for v in row]
    _check(len(t) % 3 == 0 and len(t) // 3 <= 128, "filter2d_u8: at most 128 (dy, dx, coef) taps")
    out = torch.empty_like(x)
    call("mx_filter2d_u8", _p(x), B, H, W, C, (ctypes.c_float * max(len(t), 1))(*t), len(t) // 3, _p(out), _stream())
    return out


IMAGE_MEAN = (0.485, 0.456, 0.406)
IMAGE_STD = (0.229, 0.224, 0.225)


def normalize_pad(images, padded_hw, channels=3, dtype=torch.float32, mean=IMAGE_MEAN, std=IMAGE_STD):
    """uint8 [B,H,W,3] -> NHWC [B,Hp,Wp,channels] normalized, zero-padded (GeneralizedRCNNTransform)."""
    _dev(images)
    x = images.contiguous()
    B, H, W, _ = x.shape
    Hp, Wp = padded_hw
    out = torch.empty((B, Hp, Wp, channels), dtype=dtype, device=x.device)
    call("mx_normalize_pad", _p(x), B, H, W, (ctypes.c_float * 3)(*mean), (ctypes.c_float * 3)(*std), Hp, Wp,
         channels, _dtype_code(out), _p(out), _stream())
    return out


def resize_normalize_pad(images, out_sizes, padded_hw, channels=3, dtype=torch.float32, mean=IMAGE_MEAN,
                         std=IMAGE_STD):
    """GeneralizedRCNNTransform with a resize (torchvision transform.py _resize_image_and_masks: bilinear,
    align_corners=False, recompute_scale_factor=True) fused with ToDtype(scale=True), normalize and the
    zero-padded batch: uint8 HWC device images (or the reference loader's float32 CHW [3,H,W] tensors in
    [0, 1]) of any sizes -> NHWC [B,Hp,Wp,channels]; image b fills its out_sizes[b] = (nh, nw) corner."""
    B = len(images)
    _check(B == len(out_sizes), "resize_normalize_pad: one output size per image")
    xs = [im.contiguous() for im in images]
    f32 = B > 0 and xs[0].dtype == torch.float32
    for x in xs:
        _dev(x)
        if f32:  # the reference loader's ToDtype(float32, scale=True) output: f32 CHW [3, H, W]
            _check(x.dtype == torch.float32 and x.dim() == 3 and x.shape[0] == 3, "images must be float32 [3,H,W]")
        else:
            _check(x.dtype == torch.uint8 and x.dim() == 3 and x.shape[2] == 3, "images must be uint8 [H,W,3]")
    hw = [(x.shape[1], x.shape[2]) if f32 else (x.shape[0], x.shape[1]) for x in xs]
    Hp, Wp = padded_hw
    dev = xs[0].device if B else torch.device("cuda")
    out = torch.empty((B, Hp, Wp, channels), dtype=dtype, device=dev)
    if B:
        arr = lambda t, v: (t * B)(*v)  # noqa: E731
        call("mx_resize_normalize_pad_f32" if f32 else "mx_resize_normalize_pad",
             arr(ctypes.c_void_p, [x.data_ptr() for x in xs]),
             arr(ctypes.c_int64, [h for h, _ in hw]), arr(ctypes.c_int64, [w for _, w in hw]),
             arr(ctypes.c_int64, [int(s[0]) for s in out_sizes]), arr(ctypes.c_int64, [int(s[1]) for s in out_sizes]),
             B, (ctypes.c_float * 3)(*mean), (ctypes.c_float * 3)(*std), Hp, Wp, channels, _dtype_code(out), _p(out),
             _stream())
    return out


# ---------------------------------------------------------------------------------------------
class _RPNLoss(torch.autograd.Function):
    """RegionProposalNetwork.compute_loss fused (mx_rpn_loss_fwd / _bwd): two launches instead of the
    ~25 elementwise / reduction ops (and their autograd nodes) of the torch formulation."""

    @staticmethod
    def forward(ctx, objectness, deltas, labels, targets, pos, neg, beta):
        from .conv import bn_scratch
        x = objectness.detach().float().contiguous()
        d = deltas.detach().float().contiguous()
        y = labels.float().contiguous()
        t = targets.float().contiguous()
        pm = pos.to(torch.uint8).contiguous()
        nm = neg.to(torch.uint8).contiguous()
        n = x.numel()
        out = torch.empty(3, dtype=torch.float32, device=x.device)
        ws = bn_scratch(_lib.load().mx_rpn_loss_workspace(n), x.device)
        call("mx_rpn_loss_fwd", _p(x), _p(d), _p(y), _p(t), _p(pm), _p(nm), n, float(beta), _p(out), _p(ws),
             ws.numel(), _stream())
        ctx.save_for_backward(x, d, y, t, pm, nm, out)
        ctx.beta = beta
        ctx.shapes = (objectness.shape, deltas.shape)
        return out[0], out[1]

    @staticmethod
    def backward(ctx, g0, g1):
        x, d, y, t, pm, nm, out = ctx.saved_tensors
        g0, g1 = _loss_grad(g0), _loss_grad(g1)  # read by the kernel in place: no stack / zeros launches
        gx = torch.empty_like(x)
        gd = torch.empty_like(d)
        call("mx_rpn_loss_bwd", _p(x), _p(d), _p(y), _p(t), _p(pm), _p(nm), x.numel(), float(ctx.beta), _p(out),
             _p(g0), _p(g1), _p(gx), _p(gd), _stream())
        return gx.view(ctx.shapes[0]), gd.view(ctx.shapes[1]), None, None, None, None, None


def rpn_loss(objectness, deltas, labels, targets, pos, neg, beta=1.0 / 9):
    """(loss_objectness, loss_rpn_box_reg) of torchvision's RegionProposalNetwork.compute_loss given
    the sampler's masks; objectness [N, A], deltas / targets [N, A, 4], labels [N, A] (1/0/-1)."""
    _dev(objectness, deltas)
    return _RPNLoss.apply(objectness, deltas, labels, targets, pos, neg, beta)


def _loss_grad(g):
    """A loss's upstream gradient as the f32 device scalar the fused loss backward reads (None: that
    loss is unused, the kernel takes 0)."""
    if g is None:
        return None
    return g if g.dtype == torch.float32 and g.is_contiguous() else g.float().contiguous()


class _RoILoss(torch.autograd.Function):
    """fastrcnn_loss fused (mx_roi_loss_fwd / _bwd): cross-entropy + class-indexed smooth-L1."""

    @staticmethod
    def forward(ctx, logits, reg, labels, targets, beta):
        from .conv import bn_scratch
        lg = logits.detach().float()
        rg = reg.detach().float()
        if lg.stride(1) != 1:
            lg = lg.contiguous()
        if rg.stride(1) != 1:
            rg = rg.contiguous()
        lab = labels.to(torch.int64).contiguous()
        t = targets.float().contiguous()
        R, C = lg.shape
        out = torch.empty(2, dtype=torch.float32, device=lg.device)
        ws = bn_scratch(_lib.load().mx_rpn_loss_workspace(R), lg.device)
        call("mx_roi_loss_fwd", _p(lg), lg.stride(0), C, _p(rg), rg.stride(0), _p(lab), _p(t), R, float(beta),
             _p(out), _p(ws), ws.numel(), _stream())
        ctx.save_for_backward(lg, rg, lab, t)
        ctx.beta = beta
        return out[0], out[1]

    @staticmethod
    def backward(ctx, g0, g1):
        lg, rg, lab, t = ctx.saved_tensors
        R, C = lg.shape
        g0, g1 = _loss_grad(g0), _loss_grad(g1)
        gl = torch.empty((R, C), dtype=torch.float32, device=lg.device)
        gr = torch.empty((R, 4 * C), dtype=torch.float32, device=lg.device)
        call("mx_roi_loss_bwd", _p(lg), lg.stride(0), C, _p(rg), rg.stride(0), _p(lab), _p(t), R, float(ctx.beta),
             _p(g0), _p(g1), _p(gl), _p(gr), _stream())
        return gl, gr, None, None, None


def roi_loss(class_logits, box_regression, labels, regression_targets, beta=1.0 / 9):
    """(loss_classifier, loss_box_reg) of torchvision's fastrcnn_loss for the sampled RoIs."""
    _dev(class_logits, box_regression)
    return _RoILoss.apply(class_logits, box_regression, labels, regression_targets, beta)


SSIM_C1, SSIM_C2 = 0.01 ** 2, 0.03 ** 2  # train_restoration.py ssim() stabilisers (K1 = 0.01, K2 = 0.03, L = 1)


class _SSIML1(torch.autograd.Function):
    """Fused SSIM / L1 + w(1 - SSIM) loss (mx_ssim_l1_fwd / _bwd) on NCHW f32 images; the kernels read
    NHWC memory, so channels-last tensors (the HIP U-Net's output) pass without a copy. combined=True
    returns the L1 + weight * (1 - SSIM) loss, else the mean SSIM. Gradient w.r.t. `pred` only."""

    @staticmethod
    def forward(ctx, pred, target, weight, window, sigma, combined):
        x = pred.detach().permute(0, 2, 3, 1).float().contiguous()
        y = target.detach().permute(0, 2, 3, 1).float().contiguous()
        N, H, W, C = x.shape
        out = torch.empty(3, dtype=torch.float32, device=x.device)
        maps = torch.empty((3,) + tuple(x.shape), dtype=torch.float64, device=x.device) if pred.requires_grad else None
        ws = torch.empty(_lib.load().mx_ssim_workspace(N, H, W, C), dtype=torch.uint8, device=x.device)
        call("mx_ssim_l1_fwd", _p(x), _p(y), N, H, W, C, int(window), float(sigma), SSIM_C1, SSIM_C2, float(weight),
             _p(out), _p(maps), _p(ws), ws.numel(), _stream())
        ctx.save_for_backward(x, y, maps)
        ctx.cfg = (float(weight), int(window), float(sigma), bool(combined))
        return out[2] if combined else out[0]

    @staticmethod
    def backward(ctx, g):
        x, y, maps = ctx.saved_tensors
        weight, window, sigma, combined = ctx.cfg
        N, H, W, C = x.shape
        n = x.numel()
        cs, cl = (-weight / n, 1.0 / n) if combined else (1.0 / n, 0.0)
        gx = torch.empty_like(x)
        g = g.detach().float().reshape(1).contiguous()
        call("mx_ssim_l1_bwd", _p(x), _p(y), _p(maps), N, H, W, C, window, sigma, _p(g), cs, cl, _p(gx), _stream())
        return gx.permute(0, 3, 1, 2), None, None, None, None, None


def _ssim_args(pred, target, window):
    _dev(pred, target)
    _check(pred.dim() == 4 and pred.shape == target.shape, "ssim: pred and target must be [N, C, H, W] of one shape")
    _check(pred.dtype == torch.float32 and target.dtype == torch.float32, "ssim: float32 images")
    _check(not target.requires_grad, "ssim: no gradient w.r.t. target (the reference's clean image)")
    _check(window % 2 == 1 and 1 <= window <= 15, "ssim: odd window size <= 15")


def ssim(pred, target, window_size=11, sigma=1.5):
    """Mean SSIM of [N,C,H,W] images in [0, 1]: Gaussian window (σ 1.5), zero 'same' padding, no
    clipping -- the train_restoration.py:142-164 definition; differentiable in `pred`."""
    _ssim_args(pred, target, window_size)
    return _SSIML1.apply(pred, target, 0.0, window_size, sigma, False)


def ssim_l1_loss(pred, target, ssim_weight=0.3, window_size=11, sigma=1.5):
    """mean|pred - target| + ssim_weight * (1 - SSIM(pred, target)) in one forward and one backward launch
    pair (train_restoration.py:167-178 CombinedLoss)."""
    _ssim_args(pred, target, window_size)
    return _SSIML1.apply(pred, target, ssim_weight, window_size, sigma, True)
