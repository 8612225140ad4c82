"""ctypes binding of libmx_det.so (include/mx_det.h).

The library is the product path: if it is missing or fails to load, every op raises. There is no
CPU or eager-PyTorch fallback for the hot ops.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MX_DET_LIB: an alternative build of the same ABI (A/B timing of kernel changes); default in-tree
LIB_PATH = os.environ.get("MX_DET_LIB") or os.path.join(_HERE, "libmx_det.so")

c_i64 = ctypes.c_int64
c_int = ctypes.c_int
c_f = ctypes.c_float
c_d = ctypes.c_double
c_vp = ctypes.c_void_p
c_sz = ctypes.c_size_t
c_u64 = ctypes.c_uint64
F4 = ctypes.c_float * 4


class ConvShape(ctypes.Structure):
    _fields_ = [("N", c_i64), ("H", c_i64), ("W", c_i64), ("C", c_i64), ("K", c_i64), ("R", c_i64), ("S", c_i64),
                ("Ho", c_i64), ("Wo", c_i64), ("stride_h", ctypes.c_int32), ("stride_w", ctypes.c_int32),
                ("pad_h", ctypes.c_int32), ("pad_w", ctypes.c_int32)]


class JpegInfo(ctypes.Structure):
    """mx_jpeg_info (include/mx_det.h)."""
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("ncomp", ctypes.c_int32),
                ("h", ctypes.c_int32 * 3), ("v", ctypes.c_int32 * 3), ("tq", ctypes.c_int32 * 3),
                ("hmax", ctypes.c_int32), ("vmax", ctypes.c_int32), ("mcux", ctypes.c_int32), ("mcuy", ctypes.c_int32),
                ("bw", ctypes.c_int32 * 3), ("bh", ctypes.c_int32 * 3), ("dw", ctypes.c_int32 * 3),
                ("dh", ctypes.c_int32 * 3), ("coef_off", c_i64 * 3), ("coef_total", c_i64),
                ("restart_interval", ctypes.c_int32), ("scan_off", ctypes.c_int32),
                ("qt", (ctypes.c_uint16 * 64) * 4), ("cid", ctypes.c_uint8 * 3), ("td", ctypes.c_uint8 * 3),
                ("ta", ctypes.c_uint8 * 3), ("hbits", (ctypes.c_uint8 * 17) * 8), ("hval", (ctypes.c_uint8 * 256) * 8),
                ("hdef", ctypes.c_uint8 * 8)]


_SIGS = {
    "mx_version": (c_int, []),
    "mx_last_error": (ctypes.c_char_p, []),
    "mx_trace_marker": (c_int, [c_int, c_vp]),
    "mx_stream_create": (c_int, [c_int, c_vp]),
    "mx_stream_create_high_priority": (c_int, [c_int, c_vp]),
    "mx_match_workspace": (c_sz, [c_i64, c_i64]),
    "mx_match_assign": (c_int, [c_vp, c_vp, c_i64, c_vp, c_i64, c_f, c_f, c_int, c_int, c_vp, c_vp, c_vp, c_vp,
                                c_vp, c_sz, c_vp]),
    "mx_match_batched_workspace": (c_sz, [c_i64, c_i64, c_i64]),
    "mx_match_assign_batched": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_f, c_f, c_int, c_int, c_vp,
                                        c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "mx_box_iou": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp]),
    "mx_sample_draw": (c_int, [c_vp, c_int, c_vp, c_vp, c_i64, c_i64, c_int, c_d, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mx_sample_draw_workspace": (c_sz, [c_i64, c_i64]),
    "mx_sample_draw_ws": (c_int, [c_vp, c_int, c_vp, c_vp, c_i64, c_i64, c_int, c_d, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz,
                                  c_vp]),
    "mx_roi_candidates": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "mx_nms_workspace": (c_sz, [c_i64, c_i64]),
    "mx_nms_grouped_workspace": (c_sz, [c_i64, c_i64, c_i64]),
    "mx_batched_nms_grouped_sorted": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_d, c_vp, c_vp, c_i64,
                                              c_vp, c_vp, c_vp, c_sz, c_vp]),
    "mx_batched_nms_grouped": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_d, c_vp, c_vp, c_vp, c_sz,
                                       c_vp]),
    "mx_level_topk": (c_int, [c_vp, c_i64, c_i64, c_int, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "mx_level_topk_workspace": (c_sz, [c_i64, c_int, c_vp]),
    "mx_level_topk_ws": (c_int, [c_vp, c_i64, c_i64, c_int, c_vp, c_vp, c_i64, c_vp, c_vp, c_sz, c_vp]),
    "mx_batched_nms": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_d, c_int, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "mx_roi_align_fwd": (c_int, [c_vp, c_int, c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_f, c_int, c_int, c_int,
                                 c_int, c_vp, c_vp]),
    "mx_roi_align_bwd": (c_int, [c_vp, c_int, c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_f, c_int, c_int, c_int,
                                 c_int, c_vp, c_int, c_vp, c_sz, c_vp]),
    "mx_roi_align_bwd_workspace": (c_sz, [c_i64, c_int, c_int, c_int]),
    "mx_roi_bwd_set_strip": (c_int, [c_int]),
    "mx_roi_fwd_set_split": (c_int, [c_int]),
    "mx_multiscale_roi_align_fwd": (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_i64, c_vp, c_i64, c_int,
                                            c_int, c_int, c_vp, c_vp, c_vp]),
    "mx_multiscale_roi_align_bwd": (c_int, [c_vp, c_int, c_vp, c_i64, c_vp, c_vp, c_vp, c_int, c_i64, c_vp, c_vp,
                                            c_i64, c_int, c_int, c_int, c_int, c_vp, c_sz, c_vp]),
    "mx_anchors_level": (c_int, [c_f, c_vp, c_int, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "mx_proposal_clip_filter": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_f, c_f, c_vp, c_vp, c_vp]),
    "mx_boxes_degenerate": (c_int, [c_vp, c_vp, c_int, c_vp, c_vp]),
    "mx_roi_compact": (c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mx_box_decode": (c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_f, c_vp, c_vp]),
    "mx_corrupt_u8": (c_int, [c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_f, c_u64, c_vp, c_d, c_vp, c_vp, c_vp]),
    "mx_filter2d_u8": (c_int, [c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_int, c_vp, c_vp]),
    "mx_normalize_pad": (c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64, c_i64, c_i64, c_int, c_vp, c_vp]),
    "mx_resize_normalize_pad": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_i64, c_i64, c_int,
                                        c_vp, c_vp]),
    "mx_canvas_pack": (c_int, [c_vp, c_vp, c_int, c_i64, c_i64, c_i64, c_i64, c_int, c_vp, c_vp]),
    "mx_mask_pixels": (c_int, [c_vp, c_int, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "mx_canvas_unpack": (c_int, [c_vp, c_vp, c_int, c_i64, c_i64, c_i64, c_i64, c_int, c_vp, c_vp, c_vp]),
    "mx_rpn_head_split": (c_int, [c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_int, c_i64, c_int, c_vp, c_vp, c_vp]),
    "mx_rpn_head_merge": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_int, c_i64, c_int, c_vp, c_vp, c_vp]),
    "mx_resize_normalize_pad_f32": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_i64, c_i64, c_int,
                                        c_vp, c_vp]),
    "mx_conv_mblocks": (c_i64, [ctypes.POINTER(ConvShape)]),
    "mx_conv2d_fwd": (c_int, [ctypes.POINTER(ConvShape), c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp]),
    "mx_conv2d_dgrad": (c_int, [ctypes.POINTER(ConvShape), c_vp, c_vp, c_vp, c_vp]),
    "mx_conv2d_wgrad": (c_int, [ctypes.POINTER(ConvShape), c_vp, c_vp, c_vp, c_vp]),
    "mx_conv2d_fwd_ex": (c_int, [ctypes.POINTER(ConvShape), c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_vp, c_vp,
                                 c_sz, c_vp]),
    "mx_conv_workspace": (c_sz, [ctypes.POINTER(ConvShape), c_int]),
    "mx_conv_set_variant": (c_int, [c_int]),
    "mx_conv_get_variant": (c_int, []),
    "mx_conv_set_loader": (c_int, [c_int]),
    "mx_conv_set_tile": (c_int, [c_int, c_int]),
    "mx_conv_set_max_splits": (c_int, [c_int]),
    "mx_conv_set_stages": (c_int, [c_int]),
    "mx_conv_set_korder": (c_int, [c_int]),
    "mx_conv_set_debug": (c_int, [c_int]),
    "mx_jpeg_parse": (c_int, [c_vp, c_i64, c_vp]),
    "mx_jpeg_decode_coefs": (c_int, [c_vp, c_i64, c_vp, c_vp]),
    "mx_jpeg_workspace": (c_sz, [c_vp]),
    "mx_jpeg_reconstruct": (c_int, [c_vp, c_vp, c_vp, c_sz, c_vp, c_int, c_vp]),
    "mx_conv_set_wgrad_variant": (c_int, [c_int]),
    "mx_conv_get_wgrad_variant": (c_int, []),
    "mx_conv_set_wgrad_target": (c_int, [c_i64]),
    "mx_conv2d_wgrad_ex": (c_int, [ctypes.POINTER(ConvShape), c_vp, c_vp, c_vp, c_i64, c_i64, c_int, c_vp,
                                   ctypes.c_size_t, c_vp]),
    "mx_conv_transpose_weight": (c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "mx_conv_pack_weight": (c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_int, c_vp]),
    "mx_conv_dgrad_weight_elems": (ctypes.c_size_t, [c_vp, c_i64, c_i64]),
    "mx_conv_pack_plan_bytes": (ctypes.c_size_t, [c_i64]),
    "mx_conv_pack_batched": (c_int, [c_vp, c_i64, c_vp, ctypes.c_size_t, c_int, c_vp]),
    "mx_conv2d_dgrad_bnb": (c_int, [ctypes.POINTER(ConvShape), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int,
                                    c_vp, c_i64, c_vp, c_sz, c_vp]),
    "mx_rpn_loss_workspace": (c_sz, [c_i64]),
    "mx_rpn_loss_fwd": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_f, c_vp, c_vp, c_sz, c_vp]),
    "mx_rpn_loss_bwd": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_f, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mx_roi_loss_fwd": (c_int, [c_vp, c_i64, c_int, c_vp, c_i64, c_vp, c_vp, c_i64, c_f, c_vp, c_vp, c_sz, c_vp]),
    "mx_roi_loss_bwd": (c_int, [c_vp, c_i64, c_int, c_vp, c_i64, c_vp, c_vp, c_i64, c_f, c_vp, c_vp, c_vp, c_vp,
                                c_vp]),
    "mx_bn_bwd_finalize": (c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "mx_conv2d_dgrad_ex": (c_int, [ctypes.POINTER(ConvShape), c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "mx_conv2d_dgrad_t": (c_int, [ctypes.POINTER(ConvShape), c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "mx_maxpool_fwd": (c_int, [c_vp, c_int, c_i64, c_i64, c_i64, c_i64, c_int, c_int, c_int, c_vp, c_vp, c_vp]),
    "mx_maxpool_bwd": (c_int, [c_vp, c_int, c_vp, c_i64, c_i64, c_i64, c_i64, c_int, c_int, c_int, c_vp, c_vp]),
    "mx_upsample_nearest_fwd": (c_int, [c_vp, c_int, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "mx_upsample_nearest_bwd": (c_int, [c_vp, c_int, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "mx_reflect_pad_u8": (c_int, [c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "mx_up_concat": (c_int, [c_vp, c_vp, c_int, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "mx_up_concat_bwd": (c_int, [c_vp, c_int, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "mx_restore_finish": (c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp]),
    "mx_ssim_workspace": (c_sz, [c_i64, c_i64, c_i64, c_i64]),
    "mx_ssim_l1_fwd": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_int, c_f, c_f, c_f, c_f, c_vp, c_vp, c_vp,
                               c_sz, c_vp]),
    "mx_ssim_l1_bwd": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_int, c_f, c_vp, c_f, c_f, c_vp, c_vp]),
    "mx_bn_finalize": (c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_f, c_f, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                               c_vp]),
    "mx_bn_finalize_workspace": (ctypes.c_size_t, [c_i64, c_i64]),
    "mx_bn_finalize_ex": (c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_f, c_f, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                  c_vp, ctypes.c_size_t, c_vp]),
    "mx_act_bias_bwd_workspace": (ctypes.c_size_t, [c_i64, c_i64]),
    "mx_act_bias_bwd_p": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_int, c_vp, c_vp, c_vp, c_sz, c_vp, c_vp]),
    "mx_act_bias_bwd": (c_int, [c_vp, c_vp, c_int, c_i64, c_i64, c_i64, c_int, c_vp, c_int, c_vp, c_vp,
                                ctypes.c_size_t, c_vp]),
    "mx_sgd_step": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_f, c_f, c_f, c_f, c_int, c_vp]),
    "mx_sgd_pack_plan_bytes": (ctypes.c_size_t, [c_i64]),
    "mx_sgd_pack_build": (c_int, [c_vp, c_i64, c_vp, c_vp, ctypes.c_size_t, c_vp, c_vp]),
    "mx_sgd_pack_step": (c_int, [c_vp, c_vp, c_i64, c_i64, ctypes.c_size_t, c_f, c_f, c_f, c_f, c_int, c_vp]),
    "mx_bn_apply": (c_int, [c_vp, c_int, c_i64, c_i64, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_vp]),
    "mx_bn_act_maxpool": (c_int, [c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp,
                                  c_vp]),
    "mx_bn_bwd_reduce": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i64, c_int, c_vp, c_vp, c_vp, c_vp]),
    "mx_bn_bwd_apply": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i64, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mx_bn_bwd_workspace": (ctypes.c_size_t, [c_i64, c_i64]),
    "mx_bn_bwd_reduce_ex": (c_int, [c_vp, c_vp, c_vp, c_int, c_i64, c_i64, c_int, c_vp, c_vp, c_vp, c_vp,
                                    ctypes.c_size_t, c_vp, c_vp, c_vp]),
    "mx_bn_bwd_apply_ex": (c_int, [c_vp, c_vp, c_vp, c_int, c_i64, c_i64, c_int, c_vp, c_vp, c_vp, c_vp]),
    "mx_conv_workspace_x3": (c_sz, [ctypes.POINTER(ConvShape), c_int]),
    "mx_conv2d_stem_x3": (c_int, [ctypes.POINTER(ConvShape), c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp]),
    "mx_conv2d_fwd_x3": (c_int, [ctypes.POINTER(ConvShape), c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_sz,
                                 c_vp]),
    "mx_conv2d_dgrad_x3": (c_int, [ctypes.POINTER(ConvShape), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int,
                                   c_vp, c_i64, c_vp, c_sz, c_vp]),
    "mx_conv2d_wgrad_x3": (c_int, [ctypes.POINTER(ConvShape), c_vp, c_vp, c_vp, c_i64, c_i64, c_int, c_vp, c_sz,
                                   c_vp]),
    "mx_split_planes": (c_int, [c_vp, c_i64, c_vp, c_vp]),
    "mx_bn_apply_p": (c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp]),
    "mx_bn_bwd_apply_p": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i64, c_int, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mx_conv_workspace_x3p": (c_sz, [ctypes.POINTER(ConvShape), c_int]),
    "mx_conv2d_fwd_x3p": (c_int, [ctypes.POINTER(ConvShape), c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_sz,
                                  c_vp]),
    "mx_conv2d_dgrad_x3p": (c_int, [ctypes.POINTER(ConvShape), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int,
                                    c_vp, c_i64, c_vp, c_sz, c_vp]),
    "mx_conv2d_wgrad_x3p": (c_int, [ctypes.POINTER(ConvShape), c_vp, c_vp, c_vp, c_i64, c_i64, c_int, c_vp, c_sz,
                                    c_vp]),
}

_lib = None


class MxError(RuntimeError):
    pass


def load():
    """Load libmx_det.so (raises if absent: there is no fallback)."""
    global _lib
    if _lib is None:
        # torch first: its bundled libamdhip64 (soname libamdhip64.so.7) must be the one HIP runtime
        # in the process; libmx_det's NEEDED entry then binds to it.
        import torch  # noqa: F401
        if not os.path.exists(LIB_PATH):
            raise MxError(f"libmx_det.so not built at {LIB_PATH}; run `python -c 'import __graft_entry__ as g; g.build()'`")
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in _SIGS.items():
            if not hasattr(lib, name):
                continue  # reported by call() and by tests/test_abi.py
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def declared_symbols():
    return list(_SIGS)


_fns = {}


def call(name, *args):
    """Call an entry point; a non-zero return raises MxError with mx_last_error(). Pointer arguments
    may be plain ints (argtypes are bound), so the hot path passes data_ptr() values directly."""
    fn = _fns.get(name)
    if fn is None:
        lib = load()
        if not hasattr(lib, name):
            raise MxError(f"libmx_det.so does not export {name}")
        fn = _fns[name] = getattr(lib, name)
    rc = fn(*args)
    if rc != 0:
        msg = load().mx_last_error().decode(errors="replace")
        raise MxError(f"{name} failed ({rc}): {msg}")
    return rc


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return t.data_ptr() if t is not None else None


def stream():
    """The current HIP stream of the current device as a raw pointer (the C entry points enqueue on it)."""
    import torch
    return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())


def trace_marker(marker_id):
    """Enqueue the empty marker kernel (mx_trace_marker) on the current stream."""
    call("mx_trace_marker", int(marker_id), stream())
