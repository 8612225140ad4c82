// mx_match.hip — fused box_iou + Matcher + label/target construction (gfx950).
//
// Restates torchvision 0.20.1 (oracle/mx_oracle.c orc_box_iou/orc_matcher):
//   box_iou:  inter/((area1 + area2) - inter) in f32, one rounding per op (built -ffp-contract=off)
//   Matcher:  max over gt (first index on ties); < low -> -1; [low, high) -> -2;
//             allow_low_quality: anchors whose IoU equals some gt's max over anchors take their argmax.
// Reached from RegionProposalNetwork.assign_targets_to_anchors and RoIHeads.assign_targets_to_proposals
// (model(images, targets) at reference scripts/train_frcnn_baseline.py:171).
//
// Never materialises the G x A matrix: pass 1 streams gt tiles from LDS per anchor (argmax) and keeps a
// per-block running max per gt that is published with one global atomicMax per gt per block (IoU >= 0,
// so the f32 bit pattern orders like uint32); pass 2 recomputes the identical IoU to apply the
// low-quality rule and writes matches/labels/targets in one sweep.
#include "mx_common.h"

namespace mx {

static constexpr int kTile = 1024;  // gt boxes staged per LDS tile

__device__ __forceinline__ float iou_tv(float4 a, float area_a, float4 b, float area_b) {
  float ltx = fmaxf(a.x, b.x), lty = fmaxf(a.y, b.y);
  float rbx = fminf(a.z, b.z), rby = fminf(a.w, b.w);
  float w = rbx - ltx, h = rby - lty;
  w = w < 0.f ? 0.f : w;
  h = h < 0.f ? 0.f : h;
  float inter = w * h;
  return inter / ((area_a + area_b) - inter);
}

__device__ __forceinline__ float area_tv(float4 b) { return (b.z - b.x) * (b.w - b.y); }

// Batched form: image b = blockIdx.y has gt rows gt[b * G ..] of which gcount[b] (nullable: all G) are
// real -- a padded, static-shape batch (graph capture) -- and its boxes at boxes + b * bstride
// (bstride 0: the same anchors for every image); per-image outputs are [B][A].
__device__ __forceinline__ int64_t match_g(int64_t G, const int32_t* gcount) {
  if (!gcount) return G;
  const int64_t c = gcount[blockIdx.y];
  return c < G ? (c < 0 ? 0 : c) : G;
}

__global__ void __launch_bounds__(256) match_pass1(const float4* __restrict__ gt, int64_t G, const int32_t* __restrict__ gcount,
                                                   const float4* __restrict__ boxes, int64_t bstride, int64_t A,
                                                   float* __restrict__ best_val, int32_t* __restrict__ best_idx,
                                                   uint32_t* __restrict__ gmax) {
  __shared__ float4 sg[kTile];
  __shared__ float sga[kTile];
  __shared__ uint32_t smax[kTile];
  const int64_t b = blockIdx.y;
  gt += b * G;
  gmax += b * G;
  boxes += b * bstride;
  best_val += b * A;
  best_idx += b * A;
  G = match_g(G, gcount);
  int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool valid = a < A;
  float4 bx = valid ? boxes[a] : make_float4(0.f, 0.f, 0.f, 0.f);
  float ba = area_tv(bx);
  float best = -1.f;
  int32_t bi = 0;
  for (int64_t g0 = 0; g0 < G; g0 += kTile) {
    int tn = (int)min<int64_t>(kTile, G - g0);
    __syncthreads();
    for (int i = threadIdx.x; i < tn; i += blockDim.x) {
      float4 g = gt[g0 + i];
      sg[i] = g;
      sga[i] = area_tv(g);
      smax[i] = 0u;
    }
    __syncthreads();
    for (int i = 0; i < tn; ++i) {
      float v = valid ? iou_tv(sg[i], sga[i], bx, ba) : 0.f;
      if (v > best) { best = v; bi = (int32_t)(g0 + i); }
      uint32_t u = __float_as_uint(v);
      // running block max per gt; only lanes that beat it touch LDS (rare after the first hits)
      if (__any(u > smax[i])) {
        if (u > smax[i]) atomicMax(&smax[i], u);
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < tn; i += blockDim.x)
      if (smax[i]) atomicMax(&gmax[g0 + i], smax[i]);
  }
  if (valid) {
    best_val[a] = best;
    best_idx[a] = bi;
  }
}

__global__ void __launch_bounds__(256) match_pass2(const float4* __restrict__ gt, const int64_t* __restrict__ gt_labels,
                                                   int64_t G, const int32_t* __restrict__ gcount,
                                                   const float4* __restrict__ boxes, int64_t bstride, int64_t A, float high,
                                                   float low, int allow_lq, int mode, float4 wts,
                                                   const float* __restrict__ best_val, const int32_t* __restrict__ best_idx,
                                                   const uint32_t* __restrict__ gmax, int64_t* __restrict__ matches,
                                                   void* __restrict__ labels, float4* __restrict__ targets,
                                                   int32_t* __restrict__ counts) {
  __shared__ float4 sg[kTile];
  __shared__ float sga[kTile];
  __shared__ uint32_t sm[kTile];
  const int64_t b = blockIdx.y;
  gt += b * G;
  if (gt_labels) gt_labels += b * G;
  gmax += b * G;
  boxes += b * bstride;
  best_val += b * A;
  best_idx += b * A;
  matches += b * A;
  if (labels) labels = (char*)labels + b * A * (mode == 1 ? 4 : 8);
  if (targets) targets += b * A;
  G = match_g(G, gcount);
  int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool valid = a < A;
  float4 bx = valid ? boxes[a] : make_float4(0.f, 0.f, 0.f, 0.f);
  float ba = area_tv(bx);
  int64_t m = -1;
  bool lq = false;
  int32_t bi = 0;
  if (G > 0 && valid) {
    float bv = best_val[a];
    bi = best_idx[a];
    m = bi;
    if (bv < low) m = -1;
    else if (bv < high) m = -2;
  }
  if (allow_lq && G > 0) {
    for (int64_t g0 = 0; g0 < G; g0 += kTile) {
      int tn = (int)min<int64_t>(kTile, G - g0);
      __syncthreads();
      for (int i = threadIdx.x; i < tn; i += blockDim.x) {
        float4 g = gt[g0 + i];
        sg[i] = g;
        sga[i] = area_tv(g);
        sm[i] = gmax[g0 + i];
      }
      __syncthreads();
      if (valid)
        for (int i = 0; i < tn; ++i) {
          float v = iou_tv(sg[i], sga[i], bx, ba);
          lq |= (__float_as_uint(v) == sm[i]);
        }
    }
    if (lq) m = bi;
  }
  if (counts) {  // per image: anchors labelled positive (m >= 0) / negative (m == -1), one atomic per wave
    const uint64_t bp = __ballot(valid && m >= 0), bn = __ballot(valid && m == -1);
    if ((threadIdx.x & 63) == 0) {
      if (bp) atomicAdd(&counts[2 * b], (int32_t)__popcll(bp));
      if (bn) atomicAdd(&counts[2 * b + 1], (int32_t)__popcll(bn));
    }
  }
  if (!valid) return;
  matches[a] = m;
  if (mode == 0) return;
  int64_t gi = m < 0 ? 0 : m;
  if (mode == 1) {
    ((float*)labels)[a] = m >= 0 ? 1.f : (m == -1 ? 0.f : -1.f);
  } else {
    int64_t l = G > 0 ? gt_labels[gi] : 0;
    ((int64_t*)labels)[a] = m >= 0 ? l : (m == -1 ? 0 : -1);
  }
  if (targets) {
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
    if (G > 0) {
      float4 g = gt[gi];
      // det_utils.encode_boxes(reference_boxes=g, proposals=bx)
      float ew = bx.z - bx.x, eh = bx.w - bx.y;
      float ecx = bx.x + 0.5f * ew, ecy = bx.y + 0.5f * eh;
      float gw = g.z - g.x, gh = g.w - g.y;
      float gcx = g.x + 0.5f * gw, gcy = g.y + 0.5f * gh;
      t.x = wts.x * (gcx - ecx) / ew;
      t.y = wts.y * (gcy - ecy) / eh;
      t.z = wts.z * logf(gw / ew);
      t.w = wts.w * logf(gh / eh);
    }
    targets[a] = t;
  }
}

__global__ void box_iou_kernel(const float4* b1, int64_t n, const float4* b2, int64_t m, float* out) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t i = blockIdx.y;
  if (j >= m) return;
  float4 a = b1[i], b = b2[j];
  out[i * m + j] = iou_tv(a, area_tv(a), b, area_tv(b));
}

}  // namespace mx

using namespace mx;

extern "C" size_t mx_match_workspace(int64_t G, int64_t A) {
  Carver c(nullptr, 0);
  c.take<float>(A);
  c.take<int32_t>(A);
  c.take<uint32_t>(G > 0 ? G : 1);
  return c.off;
}

extern "C" size_t mx_match_batched_workspace(int64_t B, int64_t G, int64_t A) {
  Carver c(nullptr, 0);
  c.take<float>(B * A);
  c.take<int32_t>(B * A);
  c.take<uint32_t>(B * G > 0 ? B * G : 1);
  return c.off;
}

static int match_launch(const float* gt, const int64_t* gt_labels, const int32_t* gcount, int64_t B, int64_t G,
                        const float* boxes, int64_t bstride, int64_t A, float high, float low, int allow_lq, int mode,
                        const float* enc_w, int64_t* matches, void* labels, float* targets, void* ws, size_t ws_bytes,
                        hipStream_t s, int32_t* counts = nullptr) {
  MX_CHECK_ARG(G >= 0 && A >= 0 && B >= 1 && B <= 65535, "mx_match_assign: bad sizes");
  MX_CHECK_ARG(mode >= 0 && mode <= 2, "mx_match_assign: bad mode %d", mode);
  MX_CHECK_ARG(mode == 0 || labels, "mx_match_assign: labels required for mode %d", mode);
  MX_CHECK_ARG(mode != 2 || G == 0 || gt_labels, "mx_match_assign: gt_labels required for mode 2");
  MX_CHECK_ARG(!targets || enc_w, "mx_match_assign: enc weights required with targets");
  if (counts) MX_HIP(hipMemsetAsync(counts, 0, sizeof(int32_t) * 2 * B, s));
  if (A == 0) return MX_OK;
  Carver c(ws, ws_bytes);
  float* bv = c.take<float>(B * A);
  int32_t* bi = c.take<int32_t>(B * A);
  uint32_t* gm = c.take<uint32_t>(B * G > 0 ? B * G : 1);
  MX_CHECK_ARG(c.ok(), "mx_match_assign: workspace too small (%zu < %zu)", ws_bytes, c.off);
  const dim3 grid((unsigned)cdiv(A, 256), (unsigned)B);
  if (G > 0) {
    MX_HIP(hipMemsetAsync(gm, 0, sizeof(uint32_t) * B * G, s));
    match_pass1<<<grid, 256, 0, s>>>((const float4*)gt, G, gcount, (const float4*)boxes, bstride, A, bv, bi, gm);
    MX_LAUNCH_CHECK();
  }
  float4 w = enc_w ? make_float4(enc_w[0], enc_w[1], enc_w[2], enc_w[3]) : make_float4(1.f, 1.f, 1.f, 1.f);
  match_pass2<<<grid, 256, 0, s>>>((const float4*)gt, gt_labels, G, gcount, (const float4*)boxes, bstride, A, high, low,
                                   allow_lq, mode, w, bv, bi, gm, matches, labels, (float4*)targets, counts);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_match_assign(const float* gt, const int64_t* gt_labels, int64_t G, const float* boxes, int64_t A,
                               float high, float low, int allow_lq, int mode, const float* enc_w, int64_t* matches,
                               void* labels, float* targets, void* ws, size_t ws_bytes, mx_stream_t stream) {
  return match_launch(gt, gt_labels, nullptr, 1, G, boxes, 0, A, high, low, allow_lq, mode, enc_w, matches, labels,
                      targets, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int mx_match_assign_batched(const float* gt, const int64_t* gt_labels, const int32_t* gcount, int64_t B,
                                       int64_t G, const float* boxes, int64_t box_stride, int64_t A, float high, float low,
                                       int allow_lq, int mode, const float* enc_w, int64_t* matches, void* labels,
                                       float* targets, int32_t* counts, void* ws, size_t ws_bytes,
                                       mx_stream_t stream) {
  MX_CHECK_ARG(box_stride == 0 || box_stride >= A, "mx_match_assign_batched: box_stride must be 0 or >= A");
  return match_launch(gt, gt_labels, gcount, B, G, boxes, box_stride, A, high, low, allow_lq, mode, enc_w, matches,
                      labels, targets, ws, ws_bytes, (hipStream_t)stream, counts);
}

extern "C" int mx_box_iou(const float* b1, int64_t n, const float* b2, int64_t m, float* out, mx_stream_t stream) {
  MX_CHECK_ARG(n >= 0 && m >= 0 && n < 65536, "mx_box_iou: bad sizes n=%lld m=%lld", (long long)n, (long long)m);
  if (n == 0 || m == 0) return MX_OK;
  dim3 grid((unsigned)cdiv(m, 256), (unsigned)n);
  box_iou_kernel<<<grid, 256, 0, (hipStream_t)stream>>>((const float4*)b1, n, (const float4*)b2, m, out);
  MX_LAUNCH_CHECK();
  return MX_OK;
}
