/* mx_det.h — C ABI of libmx_det.so, the MI355X (gfx950) hot path of the Faster R-CNN
 * R50-FPN v2 train/eval step, corruption augmentation and U-Net restoration pre-pass of
 * ysbbin/Robust-Object-Detection.
 *
 * The reference has no plugin API of its own: its hot path is reached through
 * torchvision / OpenCV calls made from its scripts. Each entry point below names the reference call
 * site and the third-party operator it replaces, so a maintainer can bind it (ctypes stub in
 * INTEGRATION.md; the package robust-object-detection_amd/mx_det is that binding).
 *
 * Conventions
 *  - Every pointer argument is a device pointer owned by the caller; the library never allocates
 *    or frees on these paths. Scratch comes from a caller workspace sized by *_workspace().
 *  - Work is enqueued on `stream` (a hipStream_t) and is stream-ordered; nothing synchronises.
 *  - Exceptions, off the hot path and marked at their declarations: the convenience forms
 *    (mx_conv2d_fwd / _dgrad / _wgrad, mx_bn_finalize, mx_bn_bwd_reduce / _apply) allocate their
 *    temporaries with hipMallocAsync / hipFreeAsync on `stream` (the _ex forms take a workspace);
 *    mx_conv_pack_batched with upload = 1 synchronises `stream` once to copy a NEW job plan to the
 *    device (the steady state passes upload = 0 and only launches).
 *  - Return 0 on success, negative MX_E* on error; mx_last_error() gives the message (thread-local).
 *  - Activations are NHWC; conv weights are KRSC (Cout, kh, kw, Cin); dtype codes below.
 */
#ifndef MX_DET_H
#define MX_DET_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define MX_OK 0
#define MX_EINVAL -1
#define MX_EUNSUPPORTED -2
#define MX_EHIP -3

#define MX_F32 0
#define MX_BF16 1

typedef void* mx_stream_t; /* hipStream_t */

int mx_version(void);
const char* mx_last_error(void);
/* Launches an empty kernel (trace_marker_kernel) on `stream`: a marker in rocprofv3 kernel traces. */
int mx_trace_marker(int id, mx_stream_t stream);
/* A dedicated non-blocking HIP stream on `device` (never destroyed: the process's side streams). The
 * framework's own streams come from here, not from torch's round-robin pool of 32 streams per device:
 * a process creating more pool streams than that (a model per test, a loader per epoch) would alias
 * two of them -- e.g. a side stream with a graph's capture stream. */
int mx_stream_create(int device, mx_stream_t* out);
/* mx_stream_create at the device's highest stream priority (hipDeviceGetStreamPriorityRange's greatest):
 * the DataParallel NMS-flag read, a 4-B copy that must not wait behind the step's kernels. */
int mx_stream_create_high_priority(int device, mx_stream_t* out);

/* ---------------------------------------------------------------------------------------------
 * Anchor assignment: torchvision box_iou + Matcher (+ label/target construction), fused.
 * Replaces RegionProposalNetwork.assign_targets_to_anchors / RoIHeads.assign_targets_to_proposals
 * (reached from train_frcnn_baseline.py:171, model(images, targets)).
 *   gt[G,4], boxes[A,4] xyxy f32. matches[A] int64: gt index, -1 below low, -2 between.
 *   mode 0: matches only.
 *   mode 1 (RPN):  labels_f32[A] = 1 / 0 / -1 ; targets[A,4] = encode(gt[max(m,0)], boxes, w)
 *   mode 2 (RoI):  labels_i64[A] = gt_labels[max(m,0)] / 0 (below) / -1 (between); targets as mode 1
 *   G == 0 is allowed (all background, matches = -1, zero targets), as the empty-target path of
 *   coco_detection_dataset.py:44-48 requires.
 * ------------------------------------------------------------------------------------------- */
size_t mx_match_workspace(int64_t G, int64_t A);
int mx_match_assign(const float* gt, const int64_t* gt_labels, int64_t G, const float* boxes, int64_t A,
                    float high, float low, int allow_low_quality, int mode, const float* enc_weights4_host,
                    int64_t* matches, void* labels, float* targets, void* ws, size_t ws_bytes, mx_stream_t stream);

/* The same for B images in one launch (grid.y = image): gt [B][G][4] of which gcount[b] (device int32,
 * nullable = all G) rows are real -- a zero-padded, static-shape GT batch -- gt_labels [B][G]; boxes
 * [B][box_stride rows] (box_stride 0: one [A,4] set shared by every image, the RPN anchors);
 * matches / labels [B][A], targets [B][A][4]; counts (nullable) [B][2] int32 = per image the number of
 * boxes matched (label >= 1) and background (label 0) -- BalancedPositiveNegativeSampler's pos / neg
 * counts without a reduction pass. Workspace mx_match_batched_workspace(B, G, A). */
size_t mx_match_batched_workspace(int64_t B, int64_t G, int64_t A);
int mx_match_assign_batched(const float* gt, const int64_t* gt_labels, const int32_t* gcount, int64_t B, int64_t G,
                            const float* boxes, int64_t box_stride, int64_t A, float high, float low,
                            int allow_low_quality, int mode, const float* enc_weights4_host, int64_t* matches,
                            void* labels, float* targets, int32_t* counts, void* ws, size_t ws_bytes,
                            mx_stream_t stream);

/* det_utils.BalancedPositiveNegativeSampler in one launch (RegionProposalNetwork.fg_bg_sampler and
 * RoIHeads.select_training_samples, reached from train_frcnn_baseline.py:171): per row n of labels [N][L]
 * (ldtype MX_F32: the RPN's float 1 / 0 / -1; 2: int64, the RoI head's class >= 1 / 0 / -1), num_pos =
 * min(#(label >= 1), int(batch * positive_fraction)) positives and num_neg = min(#(label == 0), batch -
 * num_pos) negatives, each the num smallest keys [N][L] among its candidates (ties by lowest index: a
 * uniform draw without replacement for i.i.d. uniform keys). valid (nullable) uint8 [N][L]: entries with
 * valid == 0 are neither class (the RoI head's padding). pos / neg uint8 [N][L] masks, sm (nullable)
 * their union, nums int32 [N][2] = (num_pos, num_neg). One 1024-thread workgroup per row. */
int mx_sample_draw(const void* labels, int ldtype, const uint8_t* valid, const float* keys, int64_t N, int64_t L,
                   int batch, double positive_fraction, uint8_t* pos, uint8_t* neg, uint8_t* sm, int32_t* nums,
                   mx_stream_t stream);

/* The same draw for long rows (the RPN's anchors) split over many workgroups: a histogram launch, a
 * split launch (candidates below each class's boundary bin drawn, the boundary bin's appended to a
 * per-(row, class) list) and a finishing launch per row (radix select of the (key, index) pairs in the
 * lists), after a memset of the workspace's counters. ws: mx_sample_draw_workspace(N, L) bytes; rows of
 * at most 16,384 elements, or ws == NULL, take mx_sample_draw. Results identical to mx_sample_draw. */
size_t mx_sample_draw_workspace(int64_t N, int64_t L);
int mx_sample_draw_ws(const void* labels, int ldtype, const uint8_t* valid, const float* keys, int64_t N, int64_t L,
                      int batch, double positive_fraction, uint8_t* pos, uint8_t* neg, uint8_t* sm, int32_t* nums, void* ws,
                      size_t ws_bytes, mx_stream_t stream);

/* RoIHeads.select_training_samples' candidate rows (torchvision: cat([proposals, gt]) per image): boxes
 * [N][post + gm][4] = each image's post padded proposal boxes pb [N][post][4] then its gm padded GT boxes
 * gtp [N][gm][4], and validity bytes valid [N][post + gm] (pvalid [N][post] for the proposals, slot < gcnt[n]
 * (int32) for the GT) -- the matcher's and the sampler's rows (mx_sample_draw's valid). One launch. */
int mx_roi_candidates(const float* pb, const uint8_t* pvalid, const float* gtp, const int32_t* gcnt, int64_t N,
                      int64_t post, int64_t gm, float* box, uint8_t* valid, mx_stream_t stream);

/* torchvision.ops.box_iou -> out[n,m] (test/diagnostic entry). */
int mx_box_iou(const float* b1, int64_t n, const float* b2, int64_t m, float* out, mx_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * NMS: torchvision.ops.nms / batched_nms (boxes.py), CPU semantics: stable score-descending order,
 * suppress when IoU > thr. Replaces RegionProposalNetwork.filter_proposals' batched_nms(level) and
 * RoIHeads.postprocess_detections' batched_nms(label) (eval_all.py:111).
 *   idxs == NULL -> plain nms. mode: 0 = CPU dispatch rule (4*n > 4000 -> per-class, else
 *   coordinate-offset trick), 1 = per-class, 2 = coordinate trick.
 *   group (nullable, int32[n]): output is ordered by (group asc, score desc) instead of score desc,
 *   so several images can share one call.
 *   keep[n] int64 receives kept indices; *num_keep (device int64) the count.
 *   max_seg: upper bound on the number of boxes that share one idx value (n is always safe).
 * ------------------------------------------------------------------------------------------- */
/* One call for all images of RegionProposalNetwork.filter_proposals (torchvision calls batched_nms
 * once per image, rpn.py filter_proposals): box i belongs to image group[i] (entries with
 * group >= G are dead and never kept) and level lvl[i] in [0, L). Per image, the CPU dispatch rule
 * of torchvision.ops.batched_nms is applied on the device: more than 1000 live boxes -> NMS per
 * level, else the coordinate trick with that image's max coordinate. keep[0:num_keep] = survivors
 * ordered by (image, score desc, index); num_keep is written on the device (-1: a segment exceeded
 * max_seg). Workspace from mx_nms_grouped_workspace(n, G, max_seg). */
size_t mx_nms_grouped_workspace(int64_t n, int64_t G, int64_t max_seg);
int mx_batched_nms_grouped(const float* boxes, const float* scores, const int64_t* lvl, const int32_t* group,
                           int64_t n, int64_t G, int64_t L, int64_t max_seg, double iou_threshold, int64_t* keep,
                           int64_t* num_keep, void* ws, size_t ws_bytes, mx_stream_t stream);
/* Presorted form of mx_batched_nms_grouped, same result (bit-identical keep[0:num_keep]) in 4
 * launches instead of ~20 (no radix sorts): meant for filter_proposals' candidates, whose live entries
 * come image-major, level-major, and score-descending within each (image, level) run (the per-level
 * top-k order; a run found out of order is still ranked exactly, by counting). n <= 24576, G <= 64,
 * L <= 8. keep[num_keep:n] is filled with 0. post > 0: also sel [G, post] int64 = per image the first
 * post survivors (0 past the image's count) and valid [G, post] uint8 -- filter_proposals' padded
 * selection. Workspace from mx_nms_grouped_workspace(n, G, max_seg). Replaces the per-image
 * batched_nms of torchvision rpn.py filter_proposals (train_frcnn_baseline.py:171). */
int mx_batched_nms_grouped_sorted(const float* boxes, const float* scores, const int64_t* lvl, const int32_t* group,
                                  int64_t n, int64_t G, int64_t L, int64_t max_seg, double iou_threshold,
                                  int64_t* keep, int64_t* num_keep, int64_t post, int64_t* sel, uint8_t* valid,
                                  void* ws, size_t ws_bytes, mx_stream_t stream);
/* RegionProposalNetwork._get_top_n_idx (torchvision rpn.py:221-233, reached from
 * train_frcnn_baseline.py:171): for each image row of scores [N, row_stride] and each level l
 * (columns level_off[l] .. +level_n[l]), the indices of the min(k, level_n[l]) largest scores,
 * value descending (ties: index ascending; the set at a tied threshold takes the lowest indices),
 * plus level_off[l]; levels concatenated: out_idx [N, sum_l min(k, level_n[l])] int64.
 * 1 <= nlev <= 8, min(k, level_n[l]) <= 4096. */
int mx_level_topk(const float* scores, int64_t N, int64_t row_stride, int nlev, const int64_t* level_off,
                  const int64_t* level_n, int64_t k, int64_t* out_idx, mx_stream_t stream);
/* mx_level_topk with a workspace of mx_level_topk_workspace(N, nlev, level_n) bytes (0: no level is
 * long enough to slice; ws may then be NULL): a level above 24,576 elements is cut into slices whose
 * own top-k lists (in ws) are merged by a second launch -- the same result, read by many CUs.
 * ws == NULL: every level is one workgroup (mx_level_topk). */
size_t mx_level_topk_workspace(int64_t N, int nlev, const int64_t* level_n);
int mx_level_topk_ws(const float* scores, int64_t N, int64_t row_stride, int nlev, const int64_t* level_off,
                     const int64_t* level_n, int64_t k, int64_t* out_idx, void* ws, size_t ws_bytes,
                     mx_stream_t stream);
size_t mx_nms_workspace(int64_t n, int64_t max_seg);
int mx_batched_nms(const float* boxes, const float* scores, const int64_t* idxs, const int32_t* group, int64_t n,
                   int64_t max_seg, double iou_threshold, int mode, int64_t* keep, int64_t* num_keep, void* ws,
                   size_t ws_bytes, mx_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * RoIAlign (torchvision::roi_align / _roi_align_backward, aligned flag honoured), NHWC features.
 * Multi-scale form = MultiScaleRoIAlign(['0'..'3'], 7, 2) with its LevelMapper
 * (floor(4 + log2(sqrt(area)/224) + 1e-6) clamped to [k_min, k_max]) — replaces
 * RoIHeads.box_roi_pool reached from train_frcnn_baseline.py:171 / eval_all.py:111.
 *   feats[l]: NHWC [N, H[l], W[l], C] of dtype; rois[K,5] f32 (batch, x1,y1,x2,y2).
 *   out: [K, PH, PW, C] dtype.  Backward (torchvision _roi_align_backward,
 *   roi_align_kernel.cpp roi_align_backward_kernel_impl): grad_feats[l] NHWC f32 over N images.
 *     deterministic = 1: atomic-free gather -- every element of every grad map is WRITTEN (no
 *       zero-fill needed) with one fixed summation order per element (RoI ascending, bin, corner):
 *       bitwise reproducible run to run. Needs C % 4 == 0 with C <= 256, pooled bins <= 64, sampling <= 4, level maps
 *       < 32768 px a side, and a workspace of mx_roi_align_bwd_workspace(K, PH, PW, sampling) bytes.
 *     deterministic = 0: float atomics ACCUMULATE into caller-zeroed maps (order-dependent in
 *       the last bits; no workspace).
 *   sampling <= 0: torchvision's adaptive grid (the roi_align default sampling_ratio=-1): per RoI,
 *     ceil(roi_h / PH) x ceil(roi_w / PW) samples per bin. Forward bit-exact like the fixed grid;
 *     backward with deterministic = 0 only (atomics, as torchvision's CUDA kernel).
 * ------------------------------------------------------------------------------------------- */
size_t mx_roi_align_bwd_workspace(int64_t K, int PH, int PW, int sampling);
/* deterministic-gather tile width (pixels per wave strip): 2 (default), 4 or 8. Results are identical;
 * 4-wide tiles shorten the tail of tiles that many RoIs overlap. Not thread-safe (a process setting). */
int mx_roi_bwd_set_strip(int sw);
/* forward: channel slices per RoI (1, 2, 4 (default) or 8 when C / 8 divides): more, shorter blocks.
 * A process setting, results identical. */
int mx_roi_fwd_set_split(int n);
int mx_roi_align_fwd(const void* feat, int dtype, int64_t N, int64_t H, int64_t W, int64_t C, const float* rois,
                     int64_t K, float spatial_scale, int PH, int PW, int sampling, int aligned, void* out,
                     mx_stream_t stream);
int mx_roi_align_bwd(const void* grad_out, int dtype, int64_t N, int64_t H, int64_t W, int64_t C, const float* rois,
                     int64_t K, float spatial_scale, int PH, int PW, int sampling, int aligned, float* grad_feat,
                     int deterministic, void* ws, size_t ws_bytes, mx_stream_t stream);
int mx_multiscale_roi_align_fwd(const void* const* feats_host, const int64_t* H_host, const int64_t* W_host,
                                const float* scales_host, int nlev, int k_min, int dtype, int64_t C,
                                const float* rois, int64_t K, int PH, int PW, int sampling, void* out,
                                int32_t* levels_out, mx_stream_t stream);
int mx_multiscale_roi_align_bwd(const void* grad_out, int dtype, float* const* grad_feats_host, int64_t N,
                                const int64_t* H_host, const int64_t* W_host, const float* scales_host, int nlev,
                                int64_t C, const float* rois, const int32_t* levels, int64_t K, int PH, int PW,
                                int sampling, int deterministic, void* ws, size_t ws_bytes, mx_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Anchors and box coder (torchvision AnchorGenerator / BoxCoder, anchor_utils.py, _utils.py).
 * ------------------------------------------------------------------------------------------- */
/* One FPN level: cell anchors round([-ws,-hs,ws,hs]/2) for `size` and ratios, shifted by
 * arange*stride; order (y, x, ratio). out[gh*gw*nr, 4]. */
/* filter_proposals after the per-level top-k (rpn.py): boxes [N*T, 4] = proposals[n][top[n][t]]
 * clipped to (h, w) = hw[n] (clamp(min=0) then minimum, NaN-propagating as torch), grp [N*T] int32 = n
 * when the box is at least min_size wide and high and prob >= score_thresh, else N. top [N, T] int64
 * indices into the A proposals of the image; prob [N, T]; hw [N, 2] (h, w) f32. */
int mx_proposal_clip_filter(const float* proposals, const int64_t* top, const float* prob, const float* hw,
                            int64_t N, int64_t A, int64_t T, float min_size, float score_thresh, float* boxes_out,
                            int32_t* grp_out, mx_stream_t stream);
/* GeneralizedRCNN's degenerate-box check: flag[0] = any box of the m (<= 8) sets (boxes_host[j]:
 * counts_host[j] x 4 f32 on the device, x1 y1 x2 y2) has x2 <= x1 or y2 <= y1; one launch, the flag
 * is always written. */
int mx_boxes_degenerate(const float* const* boxes_host, const int64_t* counts_host, int m, uint8_t* flag,
                        mx_stream_t stream);
/* RoIHeads' sampled-RoI compaction: the K selected entries of mask [M] (bool, M = N x cm
 * candidates, K = their count, known on the host) in ascending order -> rois [K, 5] (entry / cm as
 * f32, then box[entry]), lab_out [K] = lab[entry] (int64), tg_out [K, 4] = tg[entry]. */
int mx_roi_compact(const uint8_t* mask, int64_t M, int64_t K, int64_t cm, const float* box, const int64_t* lab,
                   const float* tg, float* rois, int64_t* lab_out, float* tg_out, mx_stream_t stream);
int mx_anchors_level(float size, const float* ratios_host, int nr, int64_t gh, int64_t gw, int64_t stride_h,
                     int64_t stride_w, float* out, mx_stream_t stream);
/* decode_single: rel[n, ncls*4] against boxes[n,4] -> out[n, ncls*4]; weights (wx,wy,ww,wh);
 * dw/dh clamped at `clip`. */
int mx_box_decode(const float* rel, const float* boxes, int64_t n, int64_t ncls, const float* weights4_host,
                  float clip, float* out, mx_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Corruption augmentation (scripts/augmentations.py:14-56, RandomCorruption :60-74), uint8 HWC.
 *   op: 0 identity, 1 noise (sigma, Philox seed; or `noise` field f32 if non-NULL), 2 motion blur
 *   (k=9, angle 0), 3 low-res (INTER_AREA x factor, INTER_LINEAR back). Batched form takes one op
 *   per image; images are [B, H, W, 3] contiguous. tmp: >= B*nh*nw*3 bytes for op 3.
 * ------------------------------------------------------------------------------------------- */
int mx_corrupt_u8(const uint8_t* img, int64_t B, int64_t H, int64_t W, int64_t C, const int32_t* ops_host,
                  float sigma, uint64_t seed, const float* noise, double factor, uint8_t* tmp, uint8_t* out,
                  mx_stream_t stream);
/* apply_motion_blur at any kernel size / angle (augmentations.py:21-38): cv2.filter2D(img, -1, kernel)
 * on uint8 [B,H,W,C] with the non-zero taps of the k x k float kernel given as ntaps (dy, dx, coef)
 * triples (row-major kernel order, offsets from the anchor = kernel centre), BORDER_REFLECT_101,
 * f32 sum, round half to even. The kernel itself (getRotationMatrix2D + warpAffine of the centre row,
 * normalised) is built on the host (mx_det.augment.motion_blur_kernel). ntaps <= 128; not in place.
 * Low-res (op 3) takes OpenCV's exact-x2 INTER_AREA fast path when W == 2*nw and H == 2*nh. */
int mx_filter2d_u8(const uint8_t* img, int64_t B, int64_t H, int64_t W, int64_t C, const float* taps_host, int ntaps,
                   uint8_t* out, mx_stream_t stream);
/* GeneralizedRCNNTransform (normalize, zero-pad to /32) fused with ToDtype(scale=True):
 * u8 HWC [B,H,W,3] -> NHWC [B, Hp, Wp, Cp] dtype, (x/255 - mean)/std, zero padding; Cp >= 3 (extra
 * channels zero, for the conv stem's 8-channel gather). */
int mx_normalize_pad(const uint8_t* img, int64_t B, int64_t H, int64_t W, const float* mean3_host,
                     const float* std3_host, int64_t Hp, int64_t Wp, int64_t Cp, int dtype, void* out,
                     mx_stream_t stream);

/* GeneralizedRCNNTransform for images that need a resize (torchvision 0.20.1 transform.py
 * _resize_image_and_masks -> F.interpolate(scale_factor, bilinear, align_corners=False,
 * recompute_scale_factor=True), reached via the model call at train_frcnn_baseline.py:171 and
 * eval_all.py:111 on VisDrone frames of any size), fused with ToDtype(scale=True), normalize and
 * batch_images' zero padding: B u8 HWC images imgs[b] [Hs[b], Ws[b], 3] (device pointers; sizes host
 * arrays) -> NHWC [B, Hp, Wp, Cp] dtype; image b fills its [nhs[b], nws[b]] corner (nh = floor(H*s),
 * computed by the caller as torch does), the rest is zero. Bilinear weights as torch's CUDA kernel:
 * scale = (float)H / nh, src = scale * (dst + 0.5) - 0.5 (clamped at 0). */
int mx_resize_normalize_pad(const uint8_t* const* imgs, const int64_t* Hs, const int64_t* Ws, const int64_t* nhs,
                            const int64_t* nws, int64_t B, const float* mean3_host, const float* std3_host,
                            int64_t Hp, int64_t Wp, int64_t Cp, int dtype, void* out, mx_stream_t stream);
/* RPN head outputs -> torchvision's concatenated (objectness [N, Atot], pred_deltas [N, Atot, 4]) in
 * one pass (concat_box_prediction_layers, rpn.py; the reference model's RPN via train_frcnn_baseline.py:171)
 * and the reverse for the backward. o0: level 0's [N, H0, W0, 5A] head output (A logits then A x 4
 * deltas per pixel); ocv: the [N, Hc, Wc, 5A] canvas holding levels 1..ncv at rects[l] = (y, x, h, w).
 * merge writes every element of g0 / gcv (frame pixels 0; gobj / gdel nullable = zero). */
int mx_rpn_head_split(const float* o0, int64_t H0, int64_t W0, const float* ocv, int64_t Hc, int64_t Wc,
                      const int32_t* rects, int ncv, int64_t N, int A, float* obj, float* del, mx_stream_t stream);
int mx_rpn_head_merge(const float* gobj, const float* gdel, int64_t H0, int64_t W0, int64_t Hc, int64_t Wc,
                      const int32_t* rects, int ncv, int64_t N, int A, float* g0, float* gcv, mx_stream_t stream);
/* Zero-framed canvas of n NHWC maps (frcnn.RPNHead: the small FPN levels as one conv input):
 * pack writes every element of cv [N, Hc, Wc, C] (map l at rects[l] = (y, x, h, w), 0 elsewhere);
 * unpack is its backward: grads[l] = the slice of gcv (+ add[l], nullable list / entries). C % 8 == 0;
 * dtype MX_F32 / MX_BF16 for every buffer. */
int mx_canvas_pack(const void* const* maps, const int32_t* rects, int n, int64_t N, int64_t Hc, int64_t Wc, int64_t C,
                   int dtype, void* cv, mx_stream_t stream);
int mx_canvas_unpack(const void* gcv, const int32_t* rects, int n, int64_t N, int64_t Hc, int64_t Wc, int64_t C,
                     int dtype, const void* const* add, void* const* grads, mx_stream_t stream);
/* RPNHead's canvas frame mask between its convs (t * mask): y [N][HW][C] = x * mask[pixel] (mask f32 [HW] of
 * 0 / 1; the same IEEE products as the broadcast multiply), dtype MX_F32 or MX_BF16, C % 8 == 0; planes
 * (nullable, f32 only): y's bf16x3 hi / lo planes [2][N*HW*C] for the next conv's x3p operand. */
int mx_mask_pixels(const void* x, int dtype, const float* mask, int64_t N, int64_t HW, int64_t C, void* y,
                   uint16_t* planes, mx_stream_t stream);
/* The same for the reference loader's own image tensors: ToDtype(float32, scale=True) output, f32 CHW
 * [3, Hs[b], Ws[b]] contiguous (train_frcnn_baseline.py:50-54 build_transforms, fed to the model at :171).
 * A float image equal to u8 * (float)(1/255) gives the bit-identical batch of mx_resize_normalize_pad;
 * no resize (nh = H, nw = W) reproduces normalize + pad exactly. */
int mx_resize_normalize_pad_f32(const float* const* imgs_chw, const int64_t* Hs, const int64_t* Ws, const int64_t* nhs,
                                const int64_t* nws, int64_t B, const float* mean3_host, const float* std3_host,
                                int64_t Hp, int64_t Wp, int64_t Cp, int dtype, void* out, mx_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Convolution (implicit GEMM on MFMA, bf16 in / f32 accumulate), NHWC x KRSC.
 * Replaces the cuDNN convs of ResNet-50 / FPN / RPN head / box head (torchvision model reached at
 * train_frcnn_baseline.py:171) and the U-Net convs (restoration_net.py:17-30, restore_testsets.py:68).
 *   fwd:   y[N,Ho,Wo,K] = conv(x[N,H,W,C], w[K,R,S,C]) (+bias[K] f32, nullable), output dtype
 *          ydtype; stats (nullable) receives per-block column partial sums for train-mode
 *          BatchNorm: stats[2][mblocks][K] f32 (sum, sum of squares) of the f32 accumulators.
 *   dgrad: dx[N,H,W,C] = conv_transpose(dy[N,Ho,Wo,K], w)   (bf16; strides 1 and 2)
 *   wgrad: dw[K,R,S,C] f32 = sum over N,Ho,Wo dy (x) x      (overwritten; the pixel axis is split
 *          into per-split partials in a workspace and summed by a reduce kernel — no atomics)
 *   C % 8 == 0 is required (the stem input is padded to 8 channels).
 * ------------------------------------------------------------------------------------------- */
typedef struct {
  int64_t N, H, W, C, K, R, S, Ho, Wo;
  int32_t stride_h, stride_w, pad_h, pad_w;
} mx_conv_shape;
int64_t mx_conv_mblocks(const mx_conv_shape* s);
int mx_conv2d_fwd(const mx_conv_shape* s, const uint16_t* x, const uint16_t* w, const float* bias, void* y,
                  int ydtype, float* stats, mx_stream_t stream);
int mx_conv2d_dgrad(const mx_conv_shape* s, const uint16_t* dy, const uint16_t* w, uint16_t* dx,
                    mx_stream_t stream);
/* Hot-path forms. fwd_ex adds a fused epilogue: + residual[M][K] (bf16, nullable), then activation
 * (0 none, 1 ReLU, 2 LeakyReLU(0.2)) — the eval-mode conv+folded-BN(+add)+act of the backbone and
 * the U-Net. dgrad_t takes the weight in the dgrad layout written by mx_conv_pack_weight (the
 * plain mx_conv2d_fwd / mx_conv2d_dgrad allocate their temporaries with hipMallocAsync; the _ex / _t
 * forms take caller workspaces and are the graph-capturable hot path). Small grids split K: their
 * f32 partials go to `ws` (mx_conv_workspace bytes) and a reduce kernel applies the epilogue.
 * dgrad runs one dense GEMM per stride-parity class of dx (strides 1 and 2): rows with
 * h % st == ph only receive taps r == (ph + pad) % st, so no MFMA work is spent on the zero taps
 * of a strided conv. */
int mx_conv2d_fwd_ex(const mx_conv_shape* s, const uint16_t* x, const uint16_t* w, const float* bias,
                     const uint16_t* residual, int act, void* y, int ydtype, float* stats, void* ws, size_t ws_bytes,
                     mx_stream_t stream);
/* Split workspace for pass 0 (fwd) / 1 (dgrad) / 2 (wgrad): 0 when the grid fills the chip unsplit. */
size_t mx_conv_workspace(const mx_conv_shape* s, int pass);
/* Kernel-variant knobs for A/B measurement (process-wide). fwd/dgrad: 0 register-staged,
 * 1/2 direct-to-LDS 2-stage, 3..6 multi-stage direct-to-LDS (BK32x3, BK64x2, BK32x4, BK64x3),
 * 7 (default) per-launch choice between 3 and 4. wgrad: 0 32-pixel K-tiles, 1 (default) 64-pixel,
 * 2 direct-to-LDS. */
int mx_conv_set_variant(int variant);
int mx_conv_get_variant(void);
int mx_conv_set_wgrad_variant(int variant);
int mx_conv_get_wgrad_variant(void);
/* Per-step weight preparation from the f32 master parameter w[Kout][Cin][R][S] (torch layout) in
 * one pass (split != 0: every layout as hi / lo bf16 planes, see mx_pack_desc.flags bit 1): wk = [Kout][R][S][s->C] bf16 (input channels zero-padded to s->C; nullable) and
 * wt = the dgrad operand (nullable): for each tap-parity class (r0, s0) = (r % st_h, s % st_w), in
 * order r0*st_w + s0, a contiguous block [s->C][Rc][Sc][s->K] (output channels zero-padded to s->K);
 * for stride 1 this is the plain [C][R][S][K] transpose. Uses s->C, K, R, S, strides, pads.
 * Replaces the per-step .to(bfloat16) weight casts of the reference's autocast-free fp32 model. */
int mx_conv_pack_weight(const mx_conv_shape* s, const float* w, int64_t Cin, int64_t Kout, uint16_t* wk, uint16_t* wt,
                        int split, mx_stream_t stream);
size_t mx_conv_dgrad_weight_elems(const mx_conv_shape* s, int64_t Cpad, int64_t Kpad);
/* The same packing for a list of weights in ONE launch (per-step operand preparation of a whole
 * model). A job: f32 w[Kout][Cin][R][S] -> wk [Kout][R][S][Cpad] (nullable) and wt, the dgrad layout
 * with Cpad / Kpad (nullable). `plan` is a caller-owned device buffer of mx_conv_pack_plan_bytes(njobs)
 * holding the job table; upload=1 (re)writes it from `jobs` (synchronizes the stream; do it when the
 * job list changes), upload=0 reuses it. */
typedef struct {
  const float* w;
  uint16_t* wk;
  uint16_t* wt;
  int64_t Cin, Kout, Cpad, Kpad;
  int32_t R, S, stride_h, stride_w, pad_h, pad_w;
  int32_t flags; /* bit 0: "dense" dgrad layout [R][S][Cpad][Kpad] for a conv whose output is 1x1 (FC6 as a
                    valid 7x7 conv): its dgrad runs as the 1x1 GEMM dX[N, R*S*C] = dY[N, K] * W;
                    bit 1: split -- each layout written as two bf16 planes, hi = bf16(w) then
                    lo = bf16(w - hi) (the bf16x3 operands of the *_x3 convolutions; buffers twice
                    the size) */
} mx_pack_desc;
size_t mx_conv_pack_plan_bytes(int64_t njobs);
int mx_conv_pack_batched(const mx_pack_desc* jobs, int64_t njobs, void* plan, size_t plan_bytes, int upload,
                         mx_stream_t stream);
/* SGD step (torch.optim.SGD semantics, see mx_sgd_step) fused with the per-step conv operand pack:
 * a parameter with `pack` >= 0 is the f32 weight packs[pack].w, and its update and its wk / wt layouts
 * (exactly what mx_sgd_step followed by mx_conv_pack_batched would write) come out of one pass; the
 * others take plain multi-tensor SGD blocks of the same launch (scripts/train_frcnn_baseline.py:149-153,
 * 174-176: optimizer.step() then the next forward's weights). Fused packs take R*S <= 49.
 * mx_sgd_pack_build fills a HOST buffer of mx_sgd_pack_plan_bytes(nparams) (no device calls) and
 * returns the grid size and dynamic LDS bytes; the caller copies it to device memory (stream-ordered)
 * and launches mx_sgd_pack_step with it and a device array of the nparams gradient pointers. */
typedef struct {
  float* p;
  float* buf;    /* momentum buffer */
  int64_t n;
  int32_t first; /* 1: the buffer starts from this step's d (torch's first momentum step) */
  int32_t pack;  /* index into packs[] or -1 */
} mx_sgd_param;
size_t mx_sgd_pack_plan_bytes(int64_t nparams);
int mx_sgd_pack_build(const mx_sgd_param* params, int64_t nparams, const mx_pack_desc* packs, void* host_plan,
                      size_t plan_bytes, int64_t* blocks, size_t* lds_bytes);
int mx_sgd_pack_step(const void* plan, const float* const* grads, int64_t nparams, int64_t blocks, size_t lds_bytes,
                     float lr, float momentum, float dampening, float weight_decay, int nesterov, mx_stream_t stream);
/* [K][RS][C] -> [C][RS][K] bf16 (the stride-1 dgrad layout). */
int mx_conv_transpose_weight(const uint16_t* w, int64_t K, int64_t RS, int64_t C, uint16_t* wt, mx_stream_t stream);
int mx_conv2d_dgrad_t(const mx_conv_shape* s, const uint16_t* dy, const uint16_t* wt, uint16_t* dx, void* ws,
                      size_t ws_bytes, mx_stream_t stream);
/* mx_conv2d_dgrad_t plus a bf16 [N][H][W][C] tensor added to dx in the epilogue before the single
 * bf16 rounding (strides 1 and 2: each parity class adds it at the pixels it writes): the gradient of
 * an input that also feeds another branch (ResNet bottleneck x -> conv1 and x -> + identity, a stage
 * output read by the next stage and the FPN) without a separate add pass. */
int mx_conv2d_dgrad_ex(const mx_conv_shape* s, const uint16_t* dy, const uint16_t* wt, const uint16_t* residual,
                       uint16_t* dx, void* ws, size_t ws_bytes, mx_stream_t stream);
/* mx_conv2d_dgrad_ex whose output dx is the incoming gradient of a train-mode BatchNorm (+act)
 * that produced z -> y with batch mean / invstd: the epilogue also writes, per 64-row block, the
 * column sums of g = bf16(dx) * act'(y) and g * (z - mean) * invstd into part [2][part_mb][C]
 * (part_mb = cdiv(N*H*W, 64)); mx_bn_bwd_finalize then replaces mx_bn_bwd_reduce_ex (no second
 * pass over dx, y, z). Stride 1. */
int mx_conv2d_dgrad_bnb(const mx_conv_shape* s, const uint16_t* dy, const uint16_t* wt, const uint16_t* residual,
                        uint16_t* dx, const uint16_t* y, const uint16_t* z, const float* mean, const float* invstd,
                        int act, float* part, int64_t part_mb, void* ws, size_t ws_bytes, mx_stream_t stream);
int mx_conv2d_wgrad(const mx_conv_shape* s, const uint16_t* dy, const uint16_t* x, float* dw, mx_stream_t stream);
/* Hot-path wgrad: dw written directly in layout 0 ([Kout][R][S][Cin]) or 1 ([Kout][Cin][R][S], the
 * torch parameter layout, so the result is the weight's .grad as is), dropping the zero-padded
 * channels (Kout <= s->K, Cin <= s->C); ws = mx_conv_workspace(s, 2) bytes. */
int mx_conv2d_wgrad_ex(const mx_conv_shape* s, const uint16_t* dy, const uint16_t* x, float* dw, int64_t Kout,
                       int64_t Cin, int layout, void* ws, size_t ws_bytes, mx_stream_t stream);
/* wgrad grid sizing knob: split the pixel axis until ~blocks workgroups (default 512). */
/* fwd/dgrad operand loader knob: 1 (default) buffer descriptors with wave-uniform tap offsets where
 * the shape allows (input channels % 32 == 0, R*S <= 64, operands < 2 GiB), 0 per-lane global loads. */
int mx_conv_set_loader(int loader);
/* fwd/dgrad block-tile override for tuning: (0, 0) automatic, else rows 64/128 x columns 64/128/256. */
int mx_conv_set_tile(int block_rows, int block_cols);
/* Upper bound on the split-K factor of fwd / dgrad launches (0 = automatic; tuning only). */
int mx_conv_set_max_splits(int max_splits);
/* LDS ring depth of the 64x128 / 128x128 buffer-descriptor kernels (0 = automatic; tuning only). */
int mx_conv_set_stages(int stages);
/* K-tile order of the buffer-descriptor conv kernels: 0 tap-major, 1 (default) channel-major (all taps
   of a 32-channel chunk before the next chunk: cross-tap re-reads of the gathered rows hit L2). */
int mx_conv_set_korder(int order);
/* Timing experiments only: 1 = the bf16x3 buffer kernels skip their epilogue (outputs undefined). */
int mx_conv_set_debug(int v);
int mx_conv_set_wgrad_target(int64_t blocks);

/* ---------------------------------------------------------------------------------------------
 * Precision-faithful convolution (bf16x3): the reference trains and evaluates its convs in fp32
 * (TF32 on Ampere; train_frcnn_baseline.py:139-176, no autocast; U-Net restore_testsets.py:64-68).
 * Activations, gradients and outputs are f32 NHWC; every product is computed as
 * hi*hi + hi*lo + lo*hi of the operands' bf16 hi/lo split (three v_mfma_f32_16x16x32_bf16 per
 * K-step, f32 accumulation; ~2^-16 relative per product against TF32's 2^-11). Weights are the
 * split planes written by mx_conv_pack_weight / mx_conv_pack_batched with split set: w [2][K][R][S][C]
 * (fwd), wt [2][dgrad layout] (dgrad). Same shapes, epilogues, BN statistics, split-K workspaces
 * (mx_conv_workspace_x3) and layouts as the bf16 entries above.
 *   dgrad_x3: part != NULL adds the mx_conv2d_dgrad_bnb BN-backward partials (y, z, mean, invstd, act
 *   of the BN whose output gradient dx is; stride 1), else those arguments are ignored.
 * ------------------------------------------------------------------------------------------- */
size_t mx_conv_workspace_x3(const mx_conv_shape* s, int pass);
int mx_conv2d_fwd_x3(const mx_conv_shape* s, const float* x, const uint16_t* w, const float* bias, const float* residual,
                     int act, float* y, float* stats, void* ws, size_t ws_bytes, mx_stream_t stream);
/* The ResNet stem as mx_conv2d_fwd_x3 (torchvision resnet50 conv1, reached from
 * train_frcnn_baseline.py:171 through the detector's backbone): R = S = 7, K = 64, the same packed w
 * [2][64][7][7][C] and outputs (y = act(conv + bias), optional BN statistics partials, no residual),
 * with only channels 0..3 of x and w read -- the caller's real input channels are <= 4 (RGB padded
 * to C = 8 with zeros). One MFMA K-step per filter row: 224 products per output instead of 416. */
int mx_conv2d_stem_x3(const mx_conv_shape* s, const float* x, const uint16_t* w, const float* bias, int act, float* y,
                      float* stats, mx_stream_t stream);
int mx_conv2d_dgrad_x3(const mx_conv_shape* s, const float* dy, const uint16_t* wt, const float* residual, float* dx,
                       const float* y, const float* z, const float* mean, const float* invstd, int act, float* part,
                       int64_t part_mb, void* ws, size_t ws_bytes, mx_stream_t stream);
int mx_conv2d_wgrad_x3(const mx_conv_shape* s, const float* dy, const float* x, float* dw, int64_t Kout, int64_t Cin,
                       int layout, void* ws, size_t ws_bytes, mx_stream_t stream);

/* Pre-split operands (x3p): an f32 tensor of n elements (n % 8 == 0) as its bf16x3 planes, planes[0..n) = hi,
 * planes[n..2n) = lo -- the same split the x3 kernels make in registers, so the x3p entries below are
 * bitwise equal to their x3 forms. A conv whose input (fwd) or output gradient (dgrad, wgrad) arrives as
 * planes reads it by LDS-DMA straight into the MFMA fragments' layout: no split VALU, no register
 * staging. fwd_x3p / dgrad_x3p need C % 32 == 0 (fwd) / K % 32 == 0 (dgrad) and R*S <= 64 (the buffer
 * kernel) and take the x3 workspaces; wgrad_x3p takes both dy and x as planes and the workspace of
 * mx_conv_workspace_x3p(s, 2) (its split slab only). Same arguments otherwise. */
int mx_split_planes(const float* src, int64_t n, uint16_t* planes, mx_stream_t stream);
/* mx_bn_apply / mx_bn_bwd_apply_ex (f32) that also write their output (y, resp. dx) as those planes
 * [2][M][K]: the producer of a conv operand hands it over pre-split for one extra 4-B write per element
 * instead of an mx_split_planes pass (a read and a write). */
int mx_bn_apply_p(const float* x, int64_t M, int64_t K, const float* scale, const float* shift, const float* residual,
                  int act, float* y, uint16_t* planes, mx_stream_t stream);
int mx_bn_bwd_apply_p(const float* dy, const float* y, const float* x, int64_t M, int64_t K, int act,
                      const float* coef, float* dx, float* dres, uint16_t* planes, mx_stream_t stream);
size_t mx_conv_workspace_x3p(const mx_conv_shape* s, int pass);
int mx_conv2d_fwd_x3p(const mx_conv_shape* s, const uint16_t* xp, const uint16_t* w, const float* bias,
                      const float* residual, int act, float* y, float* stats, void* ws, size_t ws_bytes,
                      mx_stream_t stream);
int mx_conv2d_dgrad_x3p(const mx_conv_shape* s, const uint16_t* dyp, const uint16_t* wt, const float* residual,
                        float* dx, const float* y, const float* z, const float* mean, const float* invstd, int act,
                        float* part, int64_t part_mb, void* ws, size_t ws_bytes, mx_stream_t stream);
int mx_conv2d_wgrad_x3p(const mx_conv_shape* s, const uint16_t* dyp, const uint16_t* xp, float* dw, int64_t Kout,
                        int64_t Cin, int layout, void* ws, size_t ws_bytes, mx_stream_t stream);

/* NHWC pooling / resampling (dtype MX_BF16 or MX_F32 storage, C % 8 == 0).
 * maxpool: F.max_pool2d (ResNet stem k3 s2 p1 — torchvision resnet50 reached at
 *   train_frcnn_baseline.py:139; U-Net MaxPool2d(2), restoration_net.py:39); argmax (nullable,
 *   int32 [N,Ho,Wo,C]) feeds the gather-form backward.
 * upsample_nearest: F.interpolate(mode="nearest", size=(Ho,Wo)) of the FPN top-down path, fused with
 *   the lateral add (y = up(x) + add, add nullable); backward sums each source's destinations. */
int mx_maxpool_fwd(const void* x, int dtype, int64_t N, int64_t H, int64_t W, int64_t C, int k, int stride, int pad,
                   void* y, int32_t* argmax, mx_stream_t stream);
int mx_maxpool_bwd(const void* gy, int dtype, const int32_t* argmax, int64_t N, int64_t H, int64_t W, int64_t C, int k,
                   int stride, int pad, void* gx, mx_stream_t stream);
int mx_upsample_nearest_fwd(const void* x, int dtype, int64_t N, int64_t H, int64_t W, int64_t C, int64_t Ho, int64_t Wo,
                            const void* add, void* y, mx_stream_t stream);
int mx_upsample_nearest_bwd(const void* gy, int dtype, int64_t N, int64_t H, int64_t W, int64_t C, int64_t Ho, int64_t Wo,
                            void* gx, mx_stream_t stream);

/* Train-mode BatchNorm2d around the conv (torch.nn.BatchNorm2d semantics, momentum 0.1,
 * unbiased running_var). finalize: reduce stats partials -> mean/invstd (f64 accumulation), fold
 * into scale/shift, update running stats. apply: y = act(x*scale + shift (+ residual)), act 0 none,
 * 1 relu, 2 leaky relu(0.2). bwd_reduce + bwd_apply: BN backward through the activation mask. */
int mx_bn_finalize(const float* stats, int64_t mblocks, int64_t K, int64_t count, const float* gamma,
                   const float* beta, float eps, float momentum, float* running_mean, float* running_var,
                   float* mean_out, float* invstd_out, float* scale_out, float* shift_out, mx_stream_t stream);
/* Hot-path finalize: one launch (row-slice partials + the last block per 64-channel chunk finishes).
 * ws = mx_bn_finalize_workspace(mblocks, K) bytes; its first 256 bytes are arrival counters that
 * must be zero before the first use and are left zero by every launch, so one zero-filled scratch
 * serves all launches on a stream (use one scratch per concurrent stream). */
/* BN backward from column partials [2][mb][K] (mx_conv2d_dgrad_bnb): sums (dbeta, dgamma) and coef
 * as mx_bn_bwd_reduce_ex produces them. Workspace: mx_bn_finalize_workspace(mb, K), counters
 * zero-kept. */
int mx_bn_bwd_finalize(const float* part, int64_t mb, int64_t K, int64_t M, const float* mean, const float* invstd,
                       const float* gamma, float* sums, float* coef, void* ws, size_t ws_bytes, mx_stream_t stream);
/* RegionProposalNetwork.compute_loss over N*A anchors (objectness [n], deltas / targets [n][4] f32,
 * labels [n] (1 fg / 0 bg / -1), pos / neg sampler masks [n] u8): out[0] = mean BCE-with-logits over
 * the sampled anchors, out[1] = smooth-L1(beta) summed over the positives / number sampled,
 * out[2] = number sampled. Deterministic (fixed-order f64 finish). Workspace counters zero-kept. */
size_t mx_rpn_loss_workspace(int64_t n);
int mx_rpn_loss_fwd(const float* objectness, const float* deltas, const float* labels, const float* targets,
                    const uint8_t* pos, const uint8_t* neg, int64_t n, float beta, float* out, void* ws,
                    size_t ws_bytes, mx_stream_t stream);
/* Gradients of (out[0], out[1]) scaled by the device scalars *grad0, *grad1 (autograd's upstream
 * gradients; null = 0, that loss unused) w.r.t. objectness and deltas. */
int mx_rpn_loss_bwd(const float* objectness, const float* deltas, const float* labels, const float* targets,
                    const uint8_t* pos, const uint8_t* neg, int64_t n, float beta, const float* out, const float* grad0,
                    const float* grad1, float* grad_objectness, float* grad_deltas, mx_stream_t stream);
/* fastrcnn_loss over R sampled RoIs: logits [R][ldl] (C classes), box regression [R][ldr] (4 per
 * class), labels [R] int64, targets [R][4]: out[0] = mean cross-entropy, out[1] = smooth-L1(beta) of
 * the labelled class's box over positive RoIs / R. Workspace: mx_rpn_loss_workspace(R). Backward:
 * grad_logits [R][C], grad_reg [R][4C] (dense) for the upstream device scalars *grad0, *grad1 (null = 0). */
int mx_roi_loss_fwd(const float* logits, int64_t ldl, int C, const float* reg, int64_t ldr, const int64_t* labels,
                    const float* targets, int64_t R, float beta, float* out, void* ws, size_t ws_bytes,
                    mx_stream_t stream);
int mx_roi_loss_bwd(const float* logits, int64_t ldl, int C, const float* reg, int64_t ldr, const int64_t* labels,
                    const float* targets, int64_t R, float beta, const float* grad0, const float* grad1,
                    float* grad_logits, float* grad_reg, mx_stream_t stream);
size_t mx_bn_finalize_workspace(int64_t mblocks, int64_t K);
int mx_bn_finalize_ex(const float* stats, int64_t mblocks, int64_t K, int64_t count, const float* gamma,
                      const float* beta, float eps, float momentum, float* running_mean, float* running_var,
                      float* mean_out, float* invstd_out, float* scale_out, float* shift_out, void* ws,
                      size_t ws_bytes, mx_stream_t stream);
/* apply: x of xdtype, residual and y of ydtype (bf16 -> bf16, f32 -> bf16, f32 -> f32). */
int mx_bn_apply(const void* x, int xdtype, int64_t M, int64_t K, const float* scale, const float* shift,
                const void* residual, int act, void* y, int ydtype, mx_stream_t stream);
/* mx_bn_apply (f32, no residual) followed by mx_maxpool_fwd (k, stride, pad; no argmax) in one pass,
 * bit-identical to the two: y [N, Ho, Wo, C] = maxpool(act(z * scale + shift)). The ResNet stem's
 * bn1 -> relu -> maxpool (torchvision resnet.py _forward_impl, reached from train_frcnn_baseline.py:171)
 * when no gradient flows through them (frozen stem). */
int mx_bn_act_maxpool(const float* z, int64_t N, int64_t H, int64_t W, int64_t C, const float* scale, const float* shift,
                      int act, int k, int stride, int pad, float* y, mx_stream_t stream);
/* Hot-path backward: reduce_ex = one launch of per-row-block partials (no float atomics) whose last
 * block per 64-channel chunk does the f64 column reduce, writing sums[2][K] = (sum g, sum g*xhat) =
 * (dbeta, dgamma) and coef[3][K], the per-channel affine form dx = coef0*g + coef1*x + coef2;
 * workspace mx_bn_bwd_workspace bytes whose first 256 bytes are arrival counters (zero before first
 * use, left zero: see mx_bn_finalize_ex). apply_ex streams dx (and dres = g, nullable).
 * g = dy * act'(y); y may be null when act == 0. */
size_t mx_bn_bwd_workspace(int64_t M, int64_t K);
int mx_bn_bwd_reduce_ex(const void* dy, const void* y, const void* x, int dtype, int64_t M, int64_t K, int act,
                        const float* mean, const float* invstd, const float* gamma, void* ws, size_t ws_bytes,
                        float* sums, float* coef, mx_stream_t stream);
int mx_bn_bwd_apply_ex(const void* dy, const void* y, const void* x, int dtype, int64_t M, int64_t K, int act,
                       const float* coef, void* dx, void* dres, mx_stream_t stream);
/* Backward head of conv (+bias) (+act) (the ConvAct layers: RPN head convs, cls/bbox heads, FC6/FC7,
 * predictor): g[M][K8] (gdtype: bf16, or f32 for the bf16x3 path) = gy * act'(y) (columns K..K8-1 zero), db[K] f32 = column sums of the
 * unrounded g (nullable). gy, y: [M][K] of dtype MX_BF16 / MX_F32 (y nullable when act == 0).
 * ws = mx_act_bias_bwd_workspace(M, K) bytes with the zero-kept counters of mx_bn_finalize_ex
 * (needed only when db is given). */
size_t mx_act_bias_bwd_workspace(int64_t M, int64_t K);
int mx_act_bias_bwd(const void* gy, const void* y, int dtype, int64_t M, int64_t K, int64_t K8, int act,
                    void* g, int gdtype, float* db, void* ws, size_t ws_bytes, mx_stream_t stream);
/* The f32 form with g's bf16x3 planes [2][M][K8] written beside g (the x3p dgrad / wgrad operand of the conv
 * this backward head belongs to; bitwise what mx_split_planes of g writes). */
int mx_act_bias_bwd_p(const float* gy, const float* y, int64_t M, int64_t K, int64_t K8, int act, float* g, float* db,
                      void* ws, size_t ws_bytes, uint16_t* planes, mx_stream_t stream);
/* Convenience forms (allocate per call): sums[2][K] is overwritten. */
int mx_bn_bwd_reduce(const uint16_t* dy, const uint16_t* y, const uint16_t* x, int64_t M, int64_t K, int act,
                     const float* mean, const float* invstd, float* sums, mx_stream_t stream);
int mx_bn_bwd_apply(const uint16_t* dy, const uint16_t* y, const uint16_t* x, int64_t M, int64_t K, int act,
                    const float* mean, const float* invstd, const float* gamma, const float* sums,
                    uint16_t* dx, uint16_t* dres /*nullable: grad of residual = masked dy*/,
                    mx_stream_t stream);

/* Multi-tensor SGD step (torch.optim.SGD semantics; the reference's SGD(lr 0.005, momentum 0.9,
 * weight_decay 5e-4), scripts/train_frcnn_baseline.py:149-153, step at :176): for each of `count`
 * f32 tensors (host arrays of device pointers / element counts), d = g + wd*p; buf = first[i] ? d :
 * momentum*buf + (1-dampening)*d; p -= lr * (nesterov ? d + momentum*buf : buf). One launch per 64
 * tensors. */
int mx_sgd_step(float* const* params, const float* const* grads, float* const* momentum_bufs,
                const int64_t* numels, const uint8_t* first, int64_t count, float lr, float momentum,
                float dampening, float weight_decay, int nesterov, mx_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Restoration pre-pass on device (scripts/restore_testsets.py:53-79, restoration_net.py:44-106).
 *   reflect_pad_u8: cv2.copyMakeBorder(0, Hp-H, 0, Wp-W, BORDER_REFLECT), uint8 [B,H,W,C] -> [B,Hp,Wp,C]
 *   up_concat: ConvTranspose2d(2, s2) output held as [N,H,W,4*Cu] (channel = (i, j, co)) scattered to
 *              [N,2H,2W,Cu] and concatenated with skip [N,2H,2W,Cs] along channels (torch.cat dim=1)
 *   restore_finish: clamp(u8/255 + residual, 0, 1) * 255 -> clip -> truncate to uint8, cropped to H x W
 * ------------------------------------------------------------------------------------------- */
int mx_reflect_pad_u8(const uint8_t* src, int64_t B, int64_t H, int64_t W, int64_t C, int64_t Hp, int64_t Wp,
                      uint8_t* dst, mx_stream_t stream);
int mx_up_concat(const void* up, const void* skip, int dtype, int64_t N, int64_t H, int64_t W, int64_t Cu, int64_t Cs,
                 void* out, mx_stream_t stream);
/* Backward of mx_up_concat (U-Net training, train_restoration.py:199-205): gcat [N,2H,2W,Cu+Cs] ->
 * gup [N,H,W,4*Cu] and gskip [N,2H,2W,Cs] (NULL: skipped). */
int mx_up_concat_bwd(const void* gcat, int dtype, int64_t N, int64_t H, int64_t W, int64_t Cu, int64_t Cs, void* gup,
                     void* gskip, mx_stream_t stream);
int mx_restore_finish(const uint8_t* img_padded, int64_t B, int64_t Hp, int64_t Wp, const float* residual, int64_t H,
                      int64_t W, uint8_t* out, mx_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * U-Net training loss L1 + weight * (1 - SSIM) (train_restoration.py:142-178: ssim() with an 11x11
 * Gaussian window, sigma 1.5, zero 'same' padding, C1 = 0.01^2, C2 = 0.03^2; CombinedLoss). Images
 * pred / target NHWC f32 [N,H,W,C] (the NCHW tensors of the reference in channels-last memory).
 *   mx_ssim_l1_fwd: out3[0] = mean SSIM, out3[1] = mean |pred - target|, out3[2] = out3[1] +
 *                   weight * (1 - out3[0]) (device floats). dmaps (nullable, 3 * N*H*W*C f64) receives
 *                   the per-pixel derivatives of the SSIM map the backward needs. Deterministic
 *                   (fixed-order f64 reduction); window sums in f64. Workspace mx_ssim_workspace().
 *   mx_ssim_l1_bwd: grad = gout[0] * (cs * d(sum SSIM)/d pred + cl * sign(pred - target)); for the
 *                   combined loss cs = -weight / numel, cl = 1 / numel; for mean SSIM cs = 1/numel, cl = 0.
 *   window odd <= 15, sigma > 0.
 * ------------------------------------------------------------------------------------------- */
size_t mx_ssim_workspace(int64_t N, int64_t H, int64_t W, int64_t C);
int mx_ssim_l1_fwd(const float* pred, const float* target, int64_t N, int64_t H, int64_t W, int64_t C, int window,
                   float sigma, float c1, float c2, float weight, float* out3, double* dmaps, void* ws, size_t ws_bytes,
                   mx_stream_t stream);
int mx_ssim_l1_bwd(const float* pred, const float* target, const double* dmaps, int64_t N, int64_t H, int64_t W,
                   int64_t C, int window, float sigma, const float* gout, float cs, float cl, float* grad,
                   mx_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Baseline JPEG decode, hybrid (replaces the PIL / cv2.imread JPEG decode of
 * coco_detection_dataset.py:23 (Image.open(...).convert("RGB")), restore_testsets.py:99 and
 * build_corrupted_testsets.py:139, all libjpeg(-turbo) ISLOW + fancy upsampling):
 *   mx_jpeg_parse         host: markers of a baseline (SOF0/SOF1) Huffman JPEG -> mx_jpeg_info
 *                         (MX_EUNSUPPORTED for progressive / arithmetic / lossless / CMYK / 4:4:0,
 *                         RGB-coded frames (libjpeg default_decompress_parms: no JFIF and Adobe
 *                         transform 0, or component ids 'R','G','B') and frames over 2^28 pixels;
 *                         MX_EINVAL for malformed headers: over-subscribed Huffman counts, undefined
 *                         quantisation tables, short segments).
 *   mx_jpeg_decode_coefs  host: entropy decoding (sequential bitstream; restart markers honoured)
 *                         into quantised coefficients, natural order, int16 [comp][by][bx][64].
 *   mx_jpeg_reconstruct   device: dequantisation + jpeg_idct_islow (jidctint.c integer IDCT) per
 *                         8x8 block into component planes (ws, mx_jpeg_workspace() bytes), then
 *                         h2v1 / h2v2 fancy upsampling (jdsample.c) and the YCbCr -> RGB tables of
 *                         jdcolor.c into out[height][width][3] uint8 (RGB, or BGR with bgr = 1 like
 *                         cv2.imread). Bit-exact with libjpeg-turbo's default decode.
 * ------------------------------------------------------------------------------------------- */
typedef struct {
  int32_t width, height, ncomp;       /* ncomp 1 (grey) or 3 (YCbCr) */
  int32_t h[3], v[3], tq[3];          /* sampling factors, quantisation table per component */
  int32_t hmax, vmax, mcux, mcuy;     /* MCUs across / down */
  int32_t bw[3], bh[3];               /* blocks per row / block rows of each component (MCU padded) */
  int32_t dw[3], dh[3];               /* downsampled_width / height (jdmaster.c) */
  int64_t coef_off[3], coef_total;    /* int16 offsets of each component's blocks; total int16s */
  int32_t restart_interval;
  int32_t scan_off;                   /* byte offset of the entropy-coded data */
  uint16_t qt[4][64];                 /* quantisation tables, natural order */
  uint8_t cid[3], td[3], ta[3];       /* component ids, DC / AC Huffman table of each component */
  uint8_t hbits[8][17], hval[8][256]; /* Huffman tables: 0-3 DC, 4-7 AC (BITS, HUFFVAL) */
  uint8_t hdef[8];
} mx_jpeg_info;
int mx_jpeg_parse(const uint8_t* data, int64_t n, mx_jpeg_info* info);
int mx_jpeg_decode_coefs(const uint8_t* data, int64_t n, const mx_jpeg_info* info, int16_t* coefs_host);
size_t mx_jpeg_workspace(const mx_jpeg_info* info);
int mx_jpeg_reconstruct(const int16_t* coefs, const mx_jpeg_info* info, void* ws, size_t ws_bytes, uint8_t* out,
                        int bgr, mx_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif
