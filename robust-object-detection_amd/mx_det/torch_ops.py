"""torch.library registrations of the HIP ops under torchvision's own operator schemas.

The reference reaches these through torchvision (pinned 0.20.1, not vendored in the reference):
  torchvision::nms(Tensor dets, Tensor scores, float iou_threshold) -> Tensor
      torchvision/ops/boxes.py nms / batched_nms <- rpn.py filter_proposals, roi_heads.py
      postprocess_detections (train_frcnn_baseline.py:171, eval_all.py:111)
  torchvision::roi_align(Tensor input, Tensor rois, float spatial_scale, SymInt pooled_height,
                         SymInt pooled_width, int sampling_ratio, bool aligned) -> Tensor
      torchvision/ops/roi_align.py <- poolers.py MultiScaleRoIAlign (RoIHeads.box_roi_pool)
  torchvision::_roi_align_backward(Tensor grad, Tensor rois, float spatial_scale,
                                   SymInt pooled_height, SymInt pooled_width, SymInt batch_size,
                                   SymInt channels, SymInt height, SymInt width, int sampling_ratio,
                                   bool aligned) -> Tensor
      torchvision/csrc/ops/autograd/roi_align_kernel.cpp (the autograd node of roi_align)
Here they are mx_det::nms, mx_det::roi_align and mx_det::_roi_align_backward with the same schemas,
NCHW tensors and argument meaning, so code written against torch.ops.torchvision.* switches by
namespace. CUDA (= HIP on ROCm) implementations call libmx_det; roi_align's autograd formula is
_roi_align_backward (the deterministic gather: bit-exact with torchvision's CPU kernel, see
ops.roi_align_deterministic); fake (meta) implementations give shapes for tracing. There is no CPU
implementation: a CPU tensor raises NotImplementedError from the dispatcher, as the product path
has no fallback. sampling_ratio <= 0 is torchvision's adaptive grid (ceil(roi_h / PH) x ceil(roi_w / PW)
samples per bin): forward bit-exact like the fixed grid, backward by float atomics (torchvision's CUDA
scheme; the deterministic gather needs a fixed grid).
"""
import torch

from . import ops

SCHEMAS = {
    "nms": "nms(Tensor dets, Tensor scores, float iou_threshold) -> Tensor",
    "roi_align": ("roi_align(Tensor input, Tensor rois, float spatial_scale, SymInt pooled_height, "
                  "SymInt pooled_width, int sampling_ratio, bool aligned) -> Tensor"),
    "_roi_align_backward": ("_roi_align_backward(Tensor grad, Tensor rois, float spatial_scale, "
                            "SymInt pooled_height, SymInt pooled_width, SymInt batch_size, SymInt channels, "
                            "SymInt height, SymInt width, int sampling_ratio, bool aligned) -> Tensor"),
}

_lib = torch.library.Library("mx_det", "DEF")
for _s in SCHEMAS.values():
    _lib.define(_s)


def _check(cond, msg):
    if not cond:
        raise RuntimeError(msg)


# ---- nms -----------------------------------------------------------------------------------------
@torch.library.impl(_lib, "nms", "CUDA")
def _nms_cuda(dets, scores, iou_threshold):
    _check(dets.dim() == 2 and dets.shape[-1] == 4, f"boxes should be a 2d tensor of shape [N, 4], got {tuple(dets.shape)}")
    _check(scores.dim() == 1 and scores.shape[0] == dets.shape[0], "scores should be a 1d tensor of the boxes' length")
    return ops.nms(dets, scores, iou_threshold)


@torch.library.register_fake("mx_det::nms")
def _nms_fake(dets, scores, iou_threshold):
    n = torch.library.get_ctx().new_dynamic_size()
    return dets.new_empty((n,), dtype=torch.int64)


# ---- roi_align -----------------------------------------------------------------------------------
@torch.library.impl(_lib, "roi_align", "CUDA")
def _roi_align_cuda(input, rois, spatial_scale, pooled_height, pooled_width, sampling_ratio, aligned):
    _check(input.dim() == 4, "input must be NCHW [N, C, H, W]")
    out = ops.roi_align_fwd_nhwc(input.permute(0, 2, 3, 1), rois, spatial_scale, int(pooled_height),
                                 int(pooled_width), int(sampling_ratio), bool(aligned))
    return out.permute(0, 3, 1, 2).contiguous()


@torch.library.register_fake("mx_det::roi_align")
def _roi_align_fake(input, rois, spatial_scale, pooled_height, pooled_width, sampling_ratio, aligned):
    return input.new_empty((rois.shape[0], input.shape[1], pooled_height, pooled_width))


@torch.library.impl(_lib, "_roi_align_backward", "CUDA")
def _roi_align_backward_cuda(grad, rois, spatial_scale, pooled_height, pooled_width, batch_size, channels, height,
                             width, sampling_ratio, aligned):
    _check(grad.dim() == 4, "grad must be [K, C, pooled_height, pooled_width]")
    gf = ops.roi_align_bwd_nhwc(grad.permute(0, 2, 3, 1), rois, int(batch_size), int(height), int(width),
                                int(channels), spatial_scale, int(pooled_height), int(pooled_width),
                                int(sampling_ratio), bool(aligned))
    return gf.permute(0, 3, 1, 2).contiguous().to(grad.dtype)


@torch.library.register_fake("mx_det::_roi_align_backward")
def _roi_align_backward_fake(grad, rois, spatial_scale, pooled_height, pooled_width, batch_size, channels, height,
                             width, sampling_ratio, aligned):
    return grad.new_empty((batch_size, channels, height, width))


def _roi_align_setup(ctx, inputs, output):
    input, rois, spatial_scale, pooled_height, pooled_width, sampling_ratio, aligned = inputs
    ctx.save_for_backward(rois)
    ctx.cfg = (tuple(input.shape), spatial_scale, pooled_height, pooled_width, sampling_ratio, aligned)


def _roi_align_grad(ctx, grad):
    (rois,) = ctx.saved_tensors
    (N, C, H, W), scale, ph, pw, sampling, aligned = ctx.cfg
    gi = torch.ops.mx_det._roi_align_backward(grad, rois, scale, ph, pw, N, C, H, W, sampling, aligned)
    return gi, None, None, None, None, None, None


torch.library.register_autograd("mx_det::roi_align", _roi_align_grad, setup_context=_roi_align_setup)


# ---- torchvision.ops-style wrappers (NCHW) -------------------------------------------------------------
def nms(boxes, scores, iou_threshold):
    """torchvision.ops.nms through the registered op."""
    return torch.ops.mx_det.nms(boxes, scores, float(iou_threshold))


def _rois(boxes, like):
    """torchvision.ops._utils.convert_boxes_to_roi_format: Tensor[K, 5] as is, or a list of per-image
    Tensor[L_i, 4] -> Tensor[sum L_i, 5] with the image index in column 0."""
    if isinstance(boxes, torch.Tensor):
        _check(boxes.dim() == 2 and boxes.shape[1] == 5, "boxes must be Tensor[K, 5] or a list of Tensor[L, 4]")
        return boxes
    _check(isinstance(boxes, (list, tuple)) and all(isinstance(b, torch.Tensor) and b.dim() == 2 and b.shape[1] == 4
                                                     for b in boxes), "boxes must be Tensor[K, 5] or a list of Tensor[L, 4]")
    if not boxes:
        return like.new_empty((0, 5))
    cat = torch.cat(list(boxes), 0)
    idx = torch.cat([torch.full_like(b[:, :1], i) for i, b in enumerate(boxes)], 0)
    return torch.cat([idx, cat], 1)


def roi_align(input, boxes, output_size, spatial_scale=1.0, sampling_ratio=-1, aligned=False):
    """torchvision.ops.roi_align (NCHW input; boxes Tensor[K, 5] or list of Tensor[L, 4]) through the
    registered op; sampling_ratio <= 0 is torchvision's adaptive grid (its default)."""
    if isinstance(output_size, int):
        output_size = (output_size, output_size)
    boxes = _rois(boxes, input)
    return torch.ops.mx_det.roi_align(input, boxes, float(spatial_scale), int(output_size[0]), int(output_size[1]),
                                      int(sampling_ratio), bool(aligned))
