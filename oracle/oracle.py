"""numpy front-end for the CPU restatement in mx_oracle.c.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, as the checker. The product package (robust-object-detection_amd/mx_det) never imports it.
Each wrapper names the reference call site the restated algorithm serves (see mx_oracle.h).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

F32 = ctypes.POINTER(ctypes.c_float)
I64 = ctypes.POINTER(ctypes.c_int64)
U8 = ctypes.POINTER(ctypes.c_uint8)
i64 = ctypes.c_int64


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        _lib = ctypes.CDLL(_SO)
        _lib.orc_nms.restype = ctypes.c_int64
        _lib.orc_batched_nms.restype = ctypes.c_int64
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def box_iou(b1, b2):
    b1, b2 = _f32(b1).reshape(-1, 4), _f32(b2).reshape(-1, 4)
    out = np.empty((len(b1), len(b2)), np.float32)
    lib().orc_box_iou(_p(b1, F32), i64(len(b1)), _p(b2, F32), i64(len(b2)), _p(out, F32))
    return out


def matcher(q, high, low, allow_low_quality):
    """rpn.py / roi_heads.py Matcher (train_frcnn_baseline.py:171 reaches it)."""
    q = _f32(q)
    G, A = q.shape
    out = np.empty(A, np.int64)
    lib().orc_matcher(_p(q, F32), i64(G), i64(A), ctypes.c_float(high), ctypes.c_float(low),
                      ctypes.c_int(int(allow_low_quality)), _p(out, I64))
    return out


def nms(boxes, scores, thr):
    boxes, scores = _f32(boxes).reshape(-1, 4), _f32(scores)
    keep = np.empty(len(scores), np.int64)
    n = lib().orc_nms(_p(boxes, F32), _p(scores, F32), i64(len(scores)), ctypes.c_double(thr), _p(keep, I64))
    return keep[:n]


def batched_nms(boxes, scores, idxs, thr):
    boxes, scores = _f32(boxes).reshape(-1, 4), _f32(scores)
    idxs = np.ascontiguousarray(idxs, dtype=np.int64)
    keep = np.empty(len(scores), np.int64)
    n = lib().orc_batched_nms(_p(boxes, F32), _p(scores, F32), _p(idxs, I64), i64(len(scores)),
                              ctypes.c_double(thr), _p(keep, I64))
    return keep[:n]


def roi_align(feat_nchw, rois, scale, out_hw=(7, 7), sampling=2, aligned=False):
    f = _f32(feat_nchw)
    r = _f32(rois).reshape(-1, 5)
    N, C, H, W = f.shape
    out = np.empty((len(r), C, out_hw[0], out_hw[1]), np.float32)
    lib().orc_roi_align_fwd(_p(f, F32), i64(N), i64(C), i64(H), i64(W), _p(r, F32), i64(len(r)),
                            ctypes.c_float(scale), out_hw[0], out_hw[1], sampling, int(aligned), _p(out, F32))
    return out


def roi_align_backward(grad_out, rois, scale, nchw, sampling=2, aligned=False):
    g = _f32(grad_out)
    r = _f32(rois).reshape(-1, 5)
    N, C, H, W = nchw
    gi = np.zeros((N, C, H, W), np.float32)
    lib().orc_roi_align_bwd(_p(g, F32), i64(N), i64(C), i64(H), i64(W), _p(r, F32), i64(len(r)),
                            ctypes.c_float(scale), g.shape[2], g.shape[3], sampling, int(aligned), _p(gi, F32))
    return gi


def anchors_level(size, ratios, gh, gw, stride_h, stride_w):
    ratios = _f32(ratios)
    out = np.empty((gh * gw * len(ratios), 4), np.float32)
    lib().orc_anchors_level(ctypes.c_float(size), _p(ratios, F32), len(ratios), i64(gh), i64(gw),
                            i64(stride_h), i64(stride_w), _p(out, F32))
    return out


def box_decode(rel, boxes, weights, clip=float(np.log(1000.0 / 16))):
    boxes = _f32(boxes).reshape(-1, 4)
    rel = _f32(rel).reshape(len(boxes), -1)
    ncls = rel.shape[1] // 4
    w = _f32(weights)
    out = np.empty_like(rel)
    lib().orc_box_decode(_p(rel, F32), _p(boxes, F32), i64(len(boxes)), i64(ncls), _p(w, F32),
                         ctypes.c_float(clip), _p(out, F32))
    return out


def box_encode(gt, prop, weights):
    gt, prop = _f32(gt).reshape(-1, 4), _f32(prop).reshape(-1, 4)
    w = _f32(weights)
    out = np.empty_like(gt)
    lib().orc_box_encode(_p(gt, F32), _p(prop, F32), i64(len(gt)), _p(w, F32), _p(out, F32))
    return out


def noise_u8(img, noise):
    img = np.ascontiguousarray(img, np.uint8)
    noise = _f32(noise)
    out = np.empty_like(img)
    lib().orc_noise_u8(_p(img, U8), _p(noise, F32), i64(img.size), _p(out, U8))
    return out


def blur_u8(img):
    img = np.ascontiguousarray(img, np.uint8)
    H, W, C = img.shape
    out = np.empty_like(img)
    lib().orc_blur_h9_u8(_p(img, U8), i64(H), i64(W), i64(C), _p(out, U8))
    return out


def lowres_u8(img, factor=0.5):
    img = np.ascontiguousarray(img, np.uint8)
    H, W, C = img.shape
    nw, nh = max(1, int(W * factor)), max(1, int(H * factor))
    tmp = np.empty((nh, nw, C), np.uint8)
    out = np.empty_like(img)
    lib().orc_lowres_u8(_p(img, U8), i64(H), i64(W), i64(C), ctypes.c_double(factor), _p(tmp, U8), _p(out, U8))
    return out


def resize_area_u8(img, dh, dw):
    img = np.ascontiguousarray(img, np.uint8)
    H, W, C = img.shape
    out = np.empty((dh, dw, C), np.uint8)
    lib().orc_resize_area_u8(_p(img, U8), i64(H), i64(W), i64(C), _p(out, U8), i64(dh), i64(dw))
    return out


def resize_linear_u8(img, dh, dw):
    img = np.ascontiguousarray(img, np.uint8)
    H, W, C = img.shape
    out = np.empty((dh, dw, C), np.uint8)
    lib().orc_resize_linear_u8(_p(img, U8), i64(H), i64(W), i64(C), _p(out, U8), i64(dh), i64(dw))
    return out


def resize_normalize(img, nh, nw, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225)):
    """GeneralizedRCNNTransform normalize + bilinear resize (torch CUDA upsample_bilinear2d arithmetic,
    mx_oracle.c orc_resize_normalize): u8 HWC [H,W,3] -> f32 [nh,nw,3]."""
    img = np.ascontiguousarray(img, np.uint8)
    H, W, _ = img.shape
    out = np.empty((nh, nw, 3), np.float32)
    m = np.asarray(mean, np.float32)
    s = np.asarray(std, np.float32)
    lib().orc_resize_normalize(_p(img, U8), i64(H), i64(W), i64(nh), i64(nw), _p(m, F32), _p(s, F32), _p(out, F32))
    return out


def reflect_pad_u8(img, ph, pw):
    img = np.ascontiguousarray(img, np.uint8)
    H, W, C = img.shape
    out = np.empty((H + ph, W + pw, C), np.uint8)
    lib().orc_reflect_pad_u8(_p(img, U8), i64(H), i64(W), i64(C), i64(ph), i64(pw), _p(out, U8))
    return out


def motion_blur_kernel(k, angle_deg):
    """augmentations.py:21-27 restated in C (orc_motion_blur_kernel)."""
    out = np.empty((k, k), np.float32)
    lib().orc_motion_blur_kernel(int(k), ctypes.c_double(angle_deg), _p(out, F32))
    return out


def kernel_taps(kernel):
    """Non-zero taps of a k x k kernel, row-major, as (dy, dx, coef) relative to the centre anchor."""
    k = kernel.shape[0]
    ys, xs = np.nonzero(kernel)
    return np.stack([ys - k // 2, xs - k // 2, kernel[ys, xs]], 1).astype(np.float32)


def filter2d_u8(img, kernel):
    """cv2.filter2D(img, -1, kernel) on HxWxC uint8 (direct path, BORDER_REFLECT_101)."""
    img = np.ascontiguousarray(img, np.uint8)
    H, W, C = img.shape
    taps = np.ascontiguousarray(kernel_taps(np.asarray(kernel, np.float32)))
    out = np.empty_like(img)
    lib().orc_filter2d_u8(_p(img, U8), i64(H), i64(W), i64(C), _p(taps, F32), ctypes.c_int(len(taps)), _p(out, U8))
    return out


def motion_blur_u8(img, k=9, angle_deg=0.0):
    """apply_motion_blur (augmentations.py:36-38)."""
    return filter2d_u8(img, motion_blur_kernel(k, angle_deg))


def resize_area_fast2_u8(img):
    img = np.ascontiguousarray(img, np.uint8)
    H, W, C = img.shape
    out = np.empty((H // 2, W // 2, C), np.uint8)
    lib().orc_resize_area_fast2_u8(_p(img, U8), i64(H), i64(W), i64(C), _p(out, U8), i64(H // 2), i64(W // 2))
    return out


def jpeg_reconstruct(coefs, info, bgr=False):
    """libjpeg-turbo pixel reconstruction (islow IDCT, fancy upsampling, ycc->rgb) of the quantised
    coefficients `coefs` (int16, mx_jpeg_decode_coefs layout) described by `info` (an mx_jpeg_info
    ctypes structure) -> uint8 [H, W, 3]."""
    coefs = np.ascontiguousarray(coefs, np.int16)
    out = np.empty((info.height, info.width, 3), np.uint8)
    rc = lib().orc_jpeg_reconstruct(coefs.ctypes.data_as(ctypes.c_void_p), ctypes.byref(info),
                                    out.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(int(bool(bgr))))
    if rc != 0:
        raise MemoryError("orc_jpeg_reconstruct")
    return out


def balanced_sample(labels, keys, batch, positive_fraction):
    """torchvision det_utils.BalancedPositiveNegativeSampler.__call__ (RegionProposalNetwork /
    RoIHeads.select_training_samples, reached from train_frcnn_baseline.py:171) with the uniform
    permutation restated as keys: per row num_pos = min(#(label >= 1), int(batch * frac)) and num_neg =
    min(#(label == 0), batch - num_pos), each class's num smallest keys drawn, ties by lowest index (a
    stable sort). labels [N, L], keys [N, L] -> (pos, neg bool [N, L], nums int [N, 2])."""
    labels, keys = np.asarray(labels), np.asarray(keys, np.float32)
    N, L = labels.shape
    pos, neg = np.zeros((N, L), bool), np.zeros((N, L), bool)
    nums = np.zeros((N, 2), np.int64)
    P = int(batch * positive_fraction)
    for r in range(N):
        cp, cn = np.nonzero(labels[r] >= 1)[0], np.nonzero(labels[r] == 0)[0]
        kp = min(len(cp), P)
        kn = min(len(cn), batch - kp)
        for cand, k, out in ((cp, kp, pos), (cn, kn, neg)):
            order = np.argsort(keys[r, cand], kind="stable")
            out[r, cand[order[:k]]] = True
        nums[r] = (kp, kn)
    return pos, neg, nums
