"""CPU restatement of the detection backend interface (mx_det/backend.py HipBackend).

TEST INFRASTRUCTURE ONLY: used by tests/ (model-level parity) and bench.py's cpu_baseline leg.
The product never imports it. It is the reference's CPU path restated: torch-CPU fp32 conv / BN /
pool / interpolate (the ops torchvision's model calls) and the C restatement of the
torchvision detection ops (oracle/mx_oracle.c: box_iou + Matcher, nms / batched_nms with the CPU
dispatch rule, roi_align forward/backward, anchors, BoxCoder). Activations stay NHWC (as channels-last
views) so the same model code runs on both backends.
"""
import numpy as np
import torch
import torch.nn.functional as F

from oracle import oracle as orc

ACT_NONE, ACT_RELU, ACT_LEAKY = 0, 1, 2


def _act(y, act):
    if act == ACT_RELU:
        return F.relu(y)
    if act == ACT_LEAKY:
        return F.leaky_relu(y, 0.2)
    return y


def _nchw(x):
    return x.permute(0, 3, 1, 2)


def _nhwc(x):
    return x.permute(0, 2, 3, 1)


class _RoIAlignCPU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, rois, scales, k_min, lv, *feats):
        r = rois.detach().numpy()
        K = r.shape[0]
        C = feats[0].shape[3]
        out = np.zeros((K, C, 7, 7), np.float32)
        for l, f in enumerate(feats):
            sel = np.where(lv == l)[0]
            if len(sel):
                out[sel] = orc.roi_align(_nchw(f.detach()).contiguous().numpy(), r[sel], scales[l], (7, 7), 2, False)
        ctx.cfg = (r, scales, lv, [tuple(f.shape) for f in feats])
        return torch.from_numpy(out).permute(0, 2, 3, 1)

    @staticmethod
    def backward(ctx, g):
        r, scales, lv, shapes = ctx.cfg
        gn = _nchw(g).contiguous().numpy()
        grads = []
        for l, (N, H, W, C) in enumerate(shapes):
            sel = np.where(lv == l)[0]
            gi = orc.roi_align_backward(gn[sel], r[sel], scales[l], (N, C, H, W)) if len(sel) else \
                np.zeros((N, C, H, W), np.float32)
            grads.append(torch.from_numpy(gi).permute(0, 2, 3, 1))
        return (None, None, None, None) + tuple(grads)


def level_mapper(boxes, k_min, k_max):
    s = torch.sqrt((boxes[:, 2] - boxes[:, 0]) * (boxes[:, 3] - boxes[:, 1]))
    t = torch.floor(4 + torch.log2(s / 224) + torch.tensor(1e-6, dtype=s.dtype))
    t = torch.clamp(t, min=k_min, max=k_max)
    return (t.to(torch.int64) - k_min).numpy()


class CpuBackend:
    name = "cpu-oracle"
    act_dtype = torch.float32
    stem_channels = 3

    def conv_bn(self, x, conv, bn, act, residual=None, link=None, bnb_own=None, bnb_feed=None):
        z = F.conv2d(_nchw(x), conv.weight, None, conv.stride, conv.padding)
        if bn.training and bn.num_batches_tracked is not None:
            bn.num_batches_tracked.add_(1)
        z = F.batch_norm(z, bn.running_mean, bn.running_var, bn.weight, bn.bias, bn.training, bn.momentum, bn.eps)
        if residual is not None:
            z = z + _nchw(residual)
        return _nhwc(_act(z, act))

    def conv(self, x, weight, bias, stride, pad, act, out_dtype=torch.float32):
        return _nhwc(_act(F.conv2d(_nchw(x), weight, bias, stride, pad), act))

    def maxpool(self, x, k, stride, pad):
        return _nhwc(F.max_pool2d(_nchw(x), k, stride, pad))

    def upsample_add(self, x, add, size):
        y = _nhwc(F.interpolate(_nchw(x), size=tuple(size), mode="nearest"))
        return y + add if add is not None else y

    def multiscale_roi_align(self, feats, rois, scales, k_min, output_size=(7, 7), sampling_ratio=2):
        lv = level_mapper(rois[:, 1:].detach(), k_min, k_min + len(feats) - 1)
        return _RoIAlignCPU.apply(rois, list(scales), k_min, lv, *feats)

    def match_assign(self, gt, boxes, high, low, allow_lq, mode, gt_labels=None, weights=None):
        g = gt.detach().float().numpy().reshape(-1, 4)
        b = boxes.detach().float().numpy().reshape(-1, 4)
        A = b.shape[0]
        if g.shape[0] == 0:
            m = np.full(A, -1, np.int64)
        else:
            m = orc.matcher(orc.box_iou(g, b), high, low, allow_lq)
        matches = torch.from_numpy(m)
        if mode == 0:
            return matches
        gi = np.clip(m, 0, None)
        if mode == 1:
            lab = torch.from_numpy(np.where(m >= 0, 1.0, np.where(m == -1, 0.0, -1.0)).astype(np.float32))
        else:
            gl = gt_labels.numpy() if g.shape[0] else np.zeros(1, np.int64)
            lab = torch.from_numpy(np.where(m >= 0, gl[gi] if g.shape[0] else 0, np.where(m == -1, 0, -1)).astype(np.int64))
        tg = None
        if weights is not None:
            tg = torch.zeros((A, 4)) if g.shape[0] == 0 else torch.from_numpy(orc.box_encode(g[gi], b, weights))
        return matches, lab, tg

    def batched_nms(self, boxes, scores, idxs, thr, group=None, max_seg=None, mode=0):
        b = boxes.detach().float().numpy()
        s = scores.detach().float().numpy()
        if idxs is None:
            return torch.from_numpy(orc.nms(b, s, thr))
        ix = idxs.numpy()
        if group is None:
            return torch.from_numpy(orc.batched_nms(b, s, ix, thr))
        out = []
        gr = group.numpy()
        for gv in np.unique(gr):
            sel = np.where(gr == gv)[0]
            k = orc.batched_nms(b[sel], s[sel], ix[sel], thr) if mode != 1 else _vanilla(b[sel], s[sel], ix[sel], thr)
            out.append(sel[k])
        return torch.from_numpy(np.concatenate(out) if out else np.zeros(0, np.int64))

    def level_topk(self, scores, num_per_level, k):
        """RegionProposalNetwork._get_top_n_idx (torchvision rpn.py): per level topk(min(k, n)) on the
        CPU, level offset added, levels concatenated."""
        tops, off = [], 0
        for n in num_per_level:
            _, ti = scores[:, off:off + n].topk(min(k, n), dim=1)
            tops.append(ti + off)
            off += n
        return torch.cat(tops, 1)

    def proposal_nms(self, boxes, scores, lvl, group, G, L, thr, max_seg):
        """Per image (group g < G), torchvision's batched_nms with its CPU dispatch rule; output padded
        to n with num_keep as a 1-element tensor (the HIP entry's contract)."""
        b = boxes.detach().float().numpy()
        s = scores.detach().float().numpy()
        lv = lvl.numpy()
        gr = group.numpy()
        out = []
        for g in range(G):
            sel = np.where(gr == g)[0]
            if sel.size == 0:
                continue
            k = orc.batched_nms(b[sel], s[sel], lv[sel], thr)
            out.append(sel[k])
        keep = np.concatenate(out) if out else np.zeros(0, np.int64)
        n = b.shape[0]
        full = np.zeros(n, np.int64)
        full[:keep.size] = keep
        return torch.from_numpy(full), torch.tensor([keep.size], dtype=torch.int64)

    def box_decode(self, rel, boxes, weights):
        return torch.from_numpy(orc.box_decode(rel.detach().numpy(), boxes.detach().numpy(), weights))

    def anchors_level(self, size, ratios, gh, gw, sh, sw, device):
        return torch.from_numpy(orc.anchors_level(size, ratios, gh, gw, sh, sw))

    def resize_normalize_pad_u8(self, images_u8, out_sizes, padded_hw):
        out = torch.zeros((len(images_u8), padded_hw[0], padded_hw[1], 3))
        for i, (im, (nh, nw)) in enumerate(zip(images_u8, out_sizes)):
            out[i, :nh, :nw] = torch.from_numpy(orc.resize_normalize(im.cpu().numpy(), nh, nw))
        return out

    def normalize_pad_u8(self, images_u8, padded_hw):
        x = images_u8.float().mul_(1.0 / 255)
        mean = torch.tensor((0.485, 0.456, 0.406))
        std = torch.tensor((0.229, 0.224, 0.225))
        x = (x - mean) / std
        B, H, W, _ = x.shape
        out = torch.zeros((B, padded_hw[0], padded_hw[1], 3))
        out[:, :H, :W] = x
        return out


def _vanilla(b, s, ix, thr):
    """per-class path forced (batched_nms_vanilla)."""
    keep = np.zeros(len(s), bool)
    for c in np.unique(ix):
        sel = np.where(ix == c)[0]
        keep[sel[orc.nms(b[sel], s[sel], thr)]] = True
    ki = np.where(keep)[0]
    order = np.argsort(-s[ki], kind="stable")
    return ki[order]
