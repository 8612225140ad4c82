// mx_elementwise.hip — anchors, box decode, corruption augmentation, normalize+pad (gfx950).
// Built -ffp-contract=off: every f32 op rounds once, as the restated torch / OpenCV code does.
#include "mx_common.h"

namespace mx {

// ---- AnchorGenerator (torchvision anchor_utils.py; oracle orc_anchors_level) -------------------
__global__ void anchors_kernel(float4 b0, float4 b1, float4 b2, int nr, int64_t gh, int64_t gw, int64_t sh, int64_t sw,
                               float4* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = gh * gw * nr;
  if (i >= total) return;
  int r = (int)(i % nr);
  int64_t loc = i / nr;
  int64_t y = loc / gw, x = loc % gw;
  float4 b = r == 0 ? b0 : (r == 1 ? b1 : b2);
  float sx = (float)(x * sw), sy = (float)(y * sh);
  out[i] = make_float4(sx + b.x, sy + b.y, sx + b.z, sy + b.w);
}

// ---- BoxCoder.decode_single (torchvision _utils.py; oracle orc_box_decode) ------------------------
__global__ void decode_kernel(const float4* __restrict__ rel, const float4* __restrict__ boxes, int64_t n, int64_t ncls,
                              float4 w, float clip, float4* __restrict__ out) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * ncls) return;
  int64_t i = t / ncls;
  float4 b = boxes[i];
  float widths = b.z - b.x, heights = b.w - b.y;
  float cx = b.x + 0.5f * widths, cy = b.y + 0.5f * heights;
  float4 r = rel[t];
  float dx = r.x / w.x, dy = r.y / w.y, dw = r.z / w.z, dh = r.w / w.w;
  dw = dw > clip ? clip : dw;
  dh = dh > clip ? clip : dh;
  float pcx = dx * widths + cx, pcy = dy * heights + cy;
  float pw = expf(dw) * widths, ph = expf(dh) * heights;
  float hw = 0.5f * pw, hh = 0.5f * ph;
  out[t] = make_float4(pcx - hw, pcy - hh, pcx + hw, pcy + hh);
}

// ---- corruption (scripts/augmentations.py:30-45) --------------------------------------------
// Philox4x32-10 counter RNG + Box-Muller: N(0, sigma) per element (the on-device replacement of
// np.random.normal, which cannot be matched bit for bit; parity tests pass the field explicitly).
__device__ __forceinline__ uint4 philox(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

__device__ __forceinline__ float gauss(uint64_t seed, uint64_t idx) {
  uint4 r = philox(make_uint4((uint32_t)idx, (uint32_t)(idx >> 32), 0x5eedu, 0u), make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
  float u1 = ((float)(r.x >> 8) + 1.0f) * (1.0f / 16777217.0f);
  float u2 = (float)(r.y >> 8) * (1.0f / 16777216.0f);
  return sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
}

// apply_noise: clip(f32(img) + f32(noise), 0, 255).astype(uint8) (truncation)
__global__ void noise_kernel(const uint8_t* __restrict__ img, const float* __restrict__ noise, float sigma, uint64_t seed,
                             int64_t n, uint8_t* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float nz = noise ? noise[i] : sigma * gauss(seed, (uint64_t)i);
  float v = (float)img[i] + nz;
  v = v < 0.f ? 0.f : (v > 255.f ? 255.f : v);
  out[i] = (uint8_t)v;
}

__device__ __forceinline__ int64_t refl101(int64_t i, int64_t n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) {
    if (i < 0) i = -i;
    if (i >= n) i = 2 * n - 2 - i;
  }
  return i;
}

// filter2D with the angle-0 9x9 motion kernel: only row 4 is non-zero (float(1/9) each), so the
// filter is a 1x9 horizontal box over BORDER_REFLECT_101, summed in f32, rounded half-to-even.
__global__ void blur_kernel(const uint8_t* __restrict__ img, int64_t H, int64_t W, int64_t C, uint8_t* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= H * W * C) return;
  int64_t c = i % C, x = (i / C) % W, y = i / (C * W);
  const float k = 1.0f / 9.0f;
  float s = 0.f;
#pragma unroll
  for (int t = -4; t <= 4; ++t) s += k * (float)img[(y * W + refl101(x + t, W)) * C + c];
  float r = rintf(s);
  r = r < 0.f ? 0.f : (r > 255.f ? 255.f : r);
  out[i] = (uint8_t)r;
}

// filter2D(src, -1, kernel) for a general k x k float kernel (apply_motion_blur at any angle,
// augmentations.py:21-38): the non-zero taps in row-major kernel order (OpenCV preprocess2DKernel),
// sum = sum_t coef_t * src in f32 from 0 (delta), BORDER_REFLECT_101, saturate_cast<uchar> (round half
// to even). This file is built -ffp-contract=off: one rounding per multiply and per add, like the
// scalar / SSE path (an AVX2 build of OpenCV fuses them; results can differ only at exact .5 ties).
struct FilterTaps {
  int n;
  int dy[128], dx[128];
  float c[128];
};

__global__ void filter2d_kernel(const uint8_t* __restrict__ img, int64_t H, int64_t W, int64_t C, FilterTaps t,
                                uint8_t* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= H * W * C) return;
  int64_t c = i % C, x = (i / C) % W, y = i / (C * W);
  float s = 0.f;
  for (int k = 0; k < t.n; ++k) s += t.c[k] * (float)img[(refl101(y + t.dy[k], H) * W + refl101(x + t.dx[k], W)) * C + c];
  float r = rintf(s);
  r = r < 0.f ? 0.f : (r > 255.f ? 255.f : r);
  out[i] = (uint8_t)r;
}

// INTER_AREA with an exact integer scale of 2 in both axes (OpenCV resize's is_area_fast branch,
// resizeAreaFast_): the vectorised part (ResizeAreaFastVec_SIMD_8u, 3 channels: 48 output elements per
// 128-bit iteration, the x86-64 baseline) computes (a + b + c + d + 2) >> 2; the scalar tail of each
// row (the last dw*C mod 48 elements) computes saturate_cast<uchar>((a + b + c + d) * 0.25f), which
// rounds exact halves to even. vec_elems = elements per row taken by the vector loop.
__global__ void area_fast2_kernel(const uint8_t* __restrict__ src, int64_t sw, int64_t C, uint8_t* __restrict__ dst,
                                  int64_t dh, int64_t dw, int64_t vec_elems) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= dh * dw * C) return;
  const int64_t e = i % (dw * C), dy = i / (dw * C);
  const int64_t c = e % C, dx = e / C;
  const uint8_t* s0 = src + ((2 * dy) * sw + 2 * dx) * C + c;
  const uint8_t* s1 = s0 + sw * C;
  const int sum = (int)s0[0] + (int)s0[C] + (int)s1[0] + (int)s1[C];
  if (e < vec_elems) {
    dst[i] = (uint8_t)((sum + 2) >> 2);
  } else {
    const float r = rintf((float)sum * 0.25f);
    dst[i] = (uint8_t)(r > 255.f ? 255.f : r);
  }
}

// OpenCV computeResizeAreaTab for one destination index: up to 3 (src, alpha) entries
__device__ int area_entries(int64_t ssize, int64_t d, double scale, int64_t* si, float* al) {
  int k = 0;
  double fs1 = d * scale, fs2 = fs1 + scale;
  double cell = scale < (ssize - fs1) ? scale : (ssize - fs1);
  int64_t s1 = (int64_t)ceil(fs1), s2 = (int64_t)floor(fs2);
  if (s2 > ssize - 1) s2 = ssize - 1;
  if (s1 > s2) s1 = s2;
  if (s1 - fs1 > 1e-3) { si[k] = s1 - 1; al[k++] = (float)((s1 - fs1) / cell); }
  for (int64_t s = s1; s < s2 && k < 7; ++s) { si[k] = s; al[k++] = (float)(1.0 / cell); }
  if (fs2 - s2 > 1e-3 && k < 8) {
    double dd = fs2 - s2;
    if (dd > 1.) dd = 1.;
    if (dd > cell) dd = cell;
    si[k] = s2; al[k++] = (float)(dd / cell);
  }
  return k;
}

// INTER_AREA general path: out = sat(sum_y beta_y * (sum_x alpha_x * S)) in f32, same order as OpenCV
__global__ void area_kernel(const uint8_t* __restrict__ src, int64_t sh, int64_t sw, int64_t C, uint8_t* __restrict__ dst,
                            int64_t dh, int64_t dw) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= dh * dw * C) return;
  int64_t c = i % C, dx = (i / C) % dw, dy = i / (C * dw);
  int64_t xs[8], ys[8];
  float xa[8], ya[8];
  int nx = area_entries(sw, dx, (double)sw / dw, xs, xa);
  int ny = area_entries(sh, dy, (double)sh / dh, ys, ya);
  float sum = 0.f;
  for (int j = 0; j < ny; ++j) {
    const uint8_t* S = src + ys[j] * sw * C;
    float buf = 0.f;
    for (int k = 0; k < nx; ++k) buf = buf + (float)S[xs[k] * C + c] * xa[k];
    sum = j == 0 ? ya[j] * buf : sum + ya[j] * buf;
  }
  float r = rintf(sum);
  dst[i] = (uint8_t)(r < 0.f ? 0.f : (r > 255.f ? 255.f : r));
}

__device__ __forceinline__ void lin_coef(int64_t ssize, int64_t dsize, int64_t d, int64_t* s_out, int* a0, int* a1) {
  double scale = 1.0 / ((double)dsize / ssize);
  float f = (float)((d + 0.5) * scale - 0.5);
  int64_t s = (int64_t)floorf(f);
  f -= (float)s;
  if (s < 0) { f = 0.f; s = 0; }
  if (s >= ssize - 1) { f = 0.f; s = ssize - 1; }
  *s_out = s;
  *a0 = (int)rintf((1.f - f) * 2048.f);
  *a1 = (int)rintf(f * 2048.f);
}

// INTER_LINEAR 8U, 11-bit fixed point; vertical combine as OpenCV's SIMD path (see oracle)
__global__ void linear_kernel(const uint8_t* __restrict__ src, int64_t sh, int64_t sw, int64_t C, uint8_t* __restrict__ dst,
                              int64_t dh, int64_t dw) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= dh * dw * C) return;
  int64_t c = i % C, x = (i / C) % dw, y = i / (C * dw);
  int64_t r0, c0;
  int b0, b1, a0, a1;
  lin_coef(sh, dh, y, &r0, &b0, &b1);
  lin_coef(sw, dw, x, &c0, &a0, &a1);
  int64_t r1 = r0 + 1 < sh ? r0 + 1 : sh - 1, c1 = c0 + 1 < sw ? c0 + 1 : sw - 1;
  int S0 = src[(r0 * sw + c0) * C + c] * a0 + src[(r0 * sw + c1) * C + c] * a1;
  int S1 = src[(r1 * sw + c0) * C + c] * a0 + src[(r1 * sw + c1) * C + c] * a1;
  int v = ((((S0 >> 4) * b0) >> 16) + (((S1 >> 4) * b1) >> 16) + 2) >> 2;
  dst[i] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// ToDtype(float32, scale=True) -> x * float(1/255); GeneralizedRCNNTransform.normalize (x-mean)/std;
// batch_images zero padding; NHWC with Cp channels (channels >= 3 zero).
template <typename T>
__global__ void normalize_pad_kernel(const uint8_t* __restrict__ img, int64_t B, int64_t H, int64_t W, float3 mean, float3 stdv,
                                     int64_t Hp, int64_t Wp, int64_t Cp, T* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * Hp * Wp) return;
  int64_t x = i % Wp, y = (i / Wp) % Hp, b = i / (Wp * Hp);
  float v[3] = {0.f, 0.f, 0.f};
  if (y < H && x < W) {
    const uint8_t* p = img + ((b * H + y) * W + x) * 3;
    const float inv = (float)(1.0 / 255.0);
    v[0] = ((float)p[0] * inv - mean.x) / stdv.x;
    v[1] = ((float)p[1] * inv - mean.y) / stdv.y;
    v[2] = ((float)p[2] * inv - mean.z) / stdv.z;
  }
  T* o = out + i * Cp;
  for (int64_t c = 0; c < Cp; ++c) io<T>::st(o + c, c < 3 ? v[c] : 0.f);
}


// GeneralizedRCNNTransform for images that need a resize (torchvision 0.20.1 transform.py
// _resize_image_and_masks: F.interpolate(scale_factor=s, mode="bilinear", align_corners=False,
// recompute_scale_factor=True)), fused with ToDtype(scale=True), normalize and batch_images' zero
// padding. The interpolation restates torch's upsample_bilinear2d_out_frame (CUDA: the reference
// trains on the GPU) in float: scale = (float)in / out, src = scale * (dst + 0.5) - 0.5 clamped at 0,
// i0 = (int)src, i1 = i0 + (i0 < in - 1), l1 = src - i0, l0 = 1 - l1,
// v = h0 * (w0 * v00 + w1 * v01) + h1 * (w0 * v10 + w1 * v11) over the normalised source values.
// Built -ffp-contract=off: every product and sum rounds once, in this order.
struct RzImg {
  const void* src;     // u8 [H][W][3] (HWC) or f32 [3][H][W] (CHW, the ToDtype(float32, scale=True) output)
  int H, W, nh, nw;
  float sh, sw;        // (float)H / nh, (float)W / nw
};
static constexpr int RZ_MAX = 16;
struct RzBatch {
  RzImg im[RZ_MAX];
};

__device__ __forceinline__ float rz_src(float scale, int dst) {
  const float s = scale * ((float)dst + 0.5f) - 0.5f;
  return s < 0.f ? 0.f : s;
}

// source pixel (h, w), channel c, as the f32 value ToDtype(float32, scale=True) yields: u8 * (float)(1/255)
// for uint8 HWC frames, the stored value for float CHW tensors (already that product when the reference
// loader made them) -- so both inputs give bit-identical batches.
template <bool F32CHW>
__device__ __forceinline__ float rz_px(const RzImg& m, int h, int w, int c) {
  if constexpr (F32CHW) {
    return ((const float*)m.src)[((int64_t)c * m.H + h) * m.W + w];
  } else {
    return (float)((const uint8_t*)m.src)[((int64_t)h * m.W + w) * 3 + c] * (float)(1.0 / 255.0);
  }
}

template <typename T, bool F32CHW>
__global__ void resize_normalize_pad_kernel(RzBatch bt, int64_t B, float3 mean, float3 stdv, int64_t Hp, int64_t Wp,
                                            int64_t Cp, T* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * Hp * Wp) return;
  const int x = (int)(i % Wp), y = (int)((i / Wp) % Hp), b = (int)(i / (Wp * Hp));
  const RzImg& m = bt.im[b];
  float v[3] = {0.f, 0.f, 0.f};
  if (y < m.nh && x < m.nw) {
    const float hr = rz_src(m.sh, y), wr = rz_src(m.sw, x);
    const int h0 = (int)hr, w0 = (int)wr;
    const int h1 = h0 + (h0 < m.H - 1 ? 1 : 0), w1 = w0 + (w0 < m.W - 1 ? 1 : 0);
    const float hl1 = hr - (float)h0, wl1 = wr - (float)w0;
    const float hl0 = 1.f - hl1, wl0 = 1.f - wl1;
    const float mu[3] = {mean.x, mean.y, mean.z}, sd[3] = {stdv.x, stdv.y, stdv.z};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float a = (rz_px<F32CHW>(m, h0, w0, c) - mu[c]) / sd[c];
      const float bb = (rz_px<F32CHW>(m, h0, w1, c) - mu[c]) / sd[c];
      const float cc = (rz_px<F32CHW>(m, h1, w0, c) - mu[c]) / sd[c];
      const float d = (rz_px<F32CHW>(m, h1, w1, c) - mu[c]) / sd[c];
      v[c] = hl0 * (wl0 * a + wl1 * bb) + hl1 * (wl0 * cc + wl1 * d);
    }
  }
  T* o = out + i * Cp;
  for (int64_t c = 0; c < Cp; ++c) io<T>::st(o + c, c < 3 ? v[c] : 0.f);
}
}  // namespace mx

using namespace mx;

extern "C" int mx_anchors_level(float size, const float* ratios, int nr, int64_t gh, int64_t gw, int64_t sh, int64_t sw,
                                float* out, mx_stream_t stream) {
  MX_CHECK_ARG(nr >= 1 && nr <= 3, "mx_anchors_level: 1..3 ratios supported");
  float4 b[3];
  for (int r = 0; r < nr; ++r) {
    // generate_anchors on the host, same f32 ops (it is a 3-element table)
    float hr = sqrtf(ratios[r]);
    float wr = 1.f / hr;
    float ws = wr * size, hs = hr * size;
    b[r] = make_float4(rintf(-ws / 2.f), rintf(-hs / 2.f), rintf(ws / 2.f), rintf(hs / 2.f));
  }
  for (int r = nr; r < 3; ++r) b[r] = b[0];
  int64_t total = gh * gw * nr;
  if (total == 0) return MX_OK;
  anchors_kernel<<<(unsigned)cdiv(total, 256), 256, 0, (hipStream_t)stream>>>(b[0], b[1], b[2], nr, gh, gw, sh, sw,
                                                                               (float4*)out);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_box_decode(const float* rel, const float* boxes, int64_t n, int64_t ncls, const float* w, float clip,
                             float* out, mx_stream_t stream) {
  MX_CHECK_ARG(n >= 0 && ncls >= 1, "mx_box_decode: bad sizes");
  if (n == 0) return MX_OK;
  decode_kernel<<<(unsigned)cdiv(n * ncls, 256), 256, 0, (hipStream_t)stream>>>(
      (const float4*)rel, (const float4*)boxes, n, ncls, make_float4(w[0], w[1], w[2], w[3]), clip, (float4*)out);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

// filter_proposals' candidate clean-up after the per-level top-k (torchvision rpn.py filter_proposals:
// box_ops.clip_boxes_to_image, remove_small_boxes, the score threshold), one thread per candidate:
// box = proposals[n][top[n][t]]; x = minimum(clamp(x, min=0), w), y likewise with h (torch's NaN
// propagation kept: a NaN coordinate stays NaN); keep = (x2-x1 >= min_size) & (y2-y1 >= min_size) &
// (prob >= score_thresh); grp = keep ? n : N (the dead group). Replaces ~15 torch launches.
__device__ __forceinline__ float clip_coord(float v, float hi) {
  const float c = v < 0.f ? 0.f : v;                        // clamp(min=0): NaN stays NaN
  return c != c ? c : (hi != hi ? hi : (hi < c ? hi : c));  // torch.minimum
}

__global__ void proposal_clip_filter_kernel(const float4* __restrict__ props, const int64_t* __restrict__ top,
                                            const float* __restrict__ prob, const float* __restrict__ hw, int64_t N,
                                            int64_t A, int64_t T, float min_size, float score_thresh,
                                            float4* __restrict__ out, int32_t* __restrict__ grp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * T) return;
  const int64_t n = i / T;
  const float4 p = props[n * A + top[i]];
  const float h = hw[2 * n], w = hw[2 * n + 1];
  const float4 b = make_float4(clip_coord(p.x, w), clip_coord(p.y, h), clip_coord(p.z, w), clip_coord(p.w, h));
  out[i] = b;
  const bool keep = (b.z - b.x >= min_size) && (b.w - b.y >= min_size) && (prob[i] >= score_thresh);
  grp[i] = keep ? (int32_t)n : (int32_t)N;
}

extern "C" int mx_proposal_clip_filter(const float* proposals, const int64_t* top, const float* prob, const float* hw,
                                       int64_t N, int64_t A, int64_t T, float min_size, float score_thresh,
                                       float* boxes_out, int32_t* grp_out, mx_stream_t stream) {
  MX_CHECK_ARG(N >= 0 && A >= 0 && T >= 0 && N < (1ll << 31), "mx_proposal_clip_filter: bad sizes");
  if (N * T == 0) return MX_OK;
  proposal_clip_filter_kernel<<<(unsigned)cdiv(N * T, 256), 256, 0, (hipStream_t)stream>>>(
      (const float4*)proposals, top, prob, hw, N, A, T, min_size, score_thresh, (float4*)boxes_out, grp_out);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

// GeneralizedRCNN.forward's degenerate-box check (generalized_rcnn.py: any box with x2 <= x1 or
// y2 <= y1) over up to 8 images' target boxes in one single-workgroup launch: flag = 1 / 0 (always
// written, so the flag needs no clearing launch). NaN coordinates compare false, as in torch.
struct BoxSets {
  const float4* p[8];
  int64_t n[8];
  int m;
};
__global__ void __launch_bounds__(1024) boxes_degenerate_kernel(BoxSets s, uint8_t* __restrict__ flag) {
  int bad = 0;
  for (int j = 0; j < s.m; ++j)
    for (int64_t i = threadIdx.x; i < s.n[j]; i += blockDim.x) {
      const float4 b = s.p[j][i];
      bad |= (b.z <= b.x) || (b.w <= b.y);
    }
  bad = __syncthreads_or(bad);
  if (threadIdx.x == 0) flag[0] = bad ? 1 : 0;
}

extern "C" int mx_boxes_degenerate(const float* const* boxes_host, const int64_t* counts_host, int m, uint8_t* flag,
                                   mx_stream_t stream) {
  MX_CHECK_ARG(m >= 1 && m <= 8 && flag, "mx_boxes_degenerate: 1..8 box sets");
  BoxSets s{};
  for (int j = 0; j < m; ++j) {
    MX_CHECK_ARG(counts_host[j] >= 0 && (counts_host[j] == 0 || boxes_host[j]), "mx_boxes_degenerate: bad set %d", j);
    s.p[j] = (const float4*)boxes_host[j];
    s.n[j] = counts_host[j];
  }
  s.m = m;
  boxes_degenerate_kernel<<<1, 1024, 0, (hipStream_t)stream>>>(s, flag);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

// RoIHeads' sampled-RoI compaction (torchvision roi_heads.py select_training_samples: per image
// torch.where(pos | neg), proposals / labels / regression targets gathered, RoI format [img, box]):
// the selected entries of a flat mask over N x cm candidates, in ascending order, written to
// rois [K, 5] (image index = entry / cm as f32, then the box), labels [K] and targets [K, 4]. One
// 1024-thread workgroup: per-thread contiguous chunks, one block scan. Replaces ~12 torch launches.
static constexpr int RC_T = 1024;
__global__ void __launch_bounds__(RC_T) roi_compact_kernel(const uint8_t* __restrict__ mask, int64_t M, int64_t K,
                                                           int64_t cm, const float4* __restrict__ box,
                                                           const int64_t* __restrict__ lab, const float4* __restrict__ tg,
                                                           float* __restrict__ rois, int64_t* __restrict__ lab_out,
                                                           float4* __restrict__ tg_out) {
  __shared__ int64_t wsum[RC_T / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t per = (M + RC_T - 1) / RC_T, b0 = tid * per, b1 = min<int64_t>(M, b0 + per);
  int64_t c = 0;
  for (int64_t i = b0; i < b1; ++i) c += mask[i] ? 1 : 0;
  int64_t x = c;  // inclusive wave scan
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  int64_t base = 0;
  for (int w = 0; w < wave; ++w) base += wsum[w];
  int64_t k = base + x - c;  // exclusive prefix: this thread's first output slot
  for (int64_t i = b0; i < b1 && k < K; ++i) {
    if (!mask[i]) continue;
    const float4 b = box[i];
    float* r = rois + 5 * k;
    r[0] = (float)(i / cm);
    r[1] = b.x; r[2] = b.y; r[3] = b.z; r[4] = b.w;
    lab_out[k] = lab[i];
    tg_out[k] = tg[i];
    ++k;
  }
}

extern "C" int mx_roi_compact(const uint8_t* mask, int64_t M, int64_t K, int64_t cm, const float* box, const int64_t* lab,
                              const float* tg, float* rois, int64_t* lab_out, float* tg_out, mx_stream_t stream) {
  MX_CHECK_ARG(M >= 0 && K >= 0 && K <= M && cm >= 1, "mx_roi_compact: bad sizes M=%lld K=%lld cm=%lld",
               (long long)M, (long long)K, (long long)cm);
  if (K == 0) return MX_OK;
  roi_compact_kernel<<<1, RC_T, 0, (hipStream_t)stream>>>(mask, M, K, cm, (const float4*)box, lab, (const float4*)tg,
                                                        rois, lab_out, (float4*)tg_out);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

// elements per destination row that ResizeAreaFastVec_SIMD_8u (scale 2, 128-bit vectors) handles:
// cn 1: 8 per step, cn 3: 48 per step, cn 4: 16 per step; other channel counts: none (scalar)
static int64_t area_fast2_vec_elems(int64_t dw, int64_t C) {
  const int64_t w = dw * C;
  const int64_t step = C == 1 ? 8 : (C == 3 ? 48 : (C == 4 ? 16 : 0));
  return step ? (w / step) * step : 0;
}

extern "C" int mx_filter2d_u8(const uint8_t* img, int64_t B, int64_t H, int64_t W, int64_t C, const float* taps_host,
                              int ntaps, uint8_t* out, mx_stream_t stream) {
  MX_CHECK_ARG(B >= 0 && H > 0 && W > 0 && C > 0 && img != out, "mx_filter2d_u8: bad shape or in-place call");
  MX_CHECK_ARG(ntaps >= 0 && ntaps <= 128, "mx_filter2d_u8: at most 128 non-zero taps");
  FilterTaps t{};
  t.n = ntaps;
  for (int k = 0; k < ntaps; ++k) {
    t.dy[k] = (int)taps_host[3 * k];
    t.dx[k] = (int)taps_host[3 * k + 1];
    t.c[k] = taps_host[3 * k + 2];
  }
  const int64_t per = H * W * C;
  for (int64_t b = 0; b < B; ++b) {
    filter2d_kernel<<<(unsigned)cdiv(per, 256), 256, 0, (hipStream_t)stream>>>(img + b * per, H, W, C, t, out + b * per);
    MX_LAUNCH_CHECK();
  }
  return MX_OK;
}

extern "C" int mx_corrupt_u8(const uint8_t* img, int64_t B, int64_t H, int64_t W, int64_t C, const int32_t* ops, float sigma,
                             uint64_t seed, const float* noise, double factor, uint8_t* tmp, uint8_t* out,
                             mx_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  MX_CHECK_ARG(B >= 0 && H > 0 && W > 0 && C > 0, "mx_corrupt_u8: bad shape");
  int64_t nw = (int64_t)(W * factor), nh = (int64_t)(H * factor);
  if (nw < 1) nw = 1;
  if (nh < 1) nh = 1;
  const int64_t per = H * W * C;
  for (int64_t b = 0; b < B; ++b) {
    const uint8_t* src = img + b * per;
    uint8_t* dst = out + b * per;
    switch (ops[b]) {
      case 0:
        if (src != dst) MX_HIP(hipMemcpyAsync(dst, src, per, hipMemcpyDeviceToDevice, s));
        break;
      case 1:
        noise_kernel<<<(unsigned)cdiv(per, 256), 256, 0, s>>>(src, noise ? noise + b * per : nullptr, sigma,
                                                             seed + 0x9E3779B97F4A7C15ull * (uint64_t)b, per, dst);
        break;
      case 2:
        MX_CHECK_ARG(src != dst, "mx_corrupt_u8: blur cannot run in place");
        blur_kernel<<<(unsigned)cdiv(per, 256), 256, 0, s>>>(src, H, W, C, dst);
        break;
      case 3: {
        MX_CHECK_ARG(tmp != nullptr, "mx_corrupt_u8: low-res needs tmp");
        uint8_t* t = tmp + b * nh * nw * C;
        if (W == 2 * nw && H == 2 * nh) {  // exact x2: OpenCV's fast INTER_AREA path
          area_fast2_kernel<<<(unsigned)cdiv(nh * nw * C, 256), 256, 0, s>>>(src, W, C, t, nh, nw,
                                                                             area_fast2_vec_elems(nw, C));
        } else {
          area_kernel<<<(unsigned)cdiv(nh * nw * C, 256), 256, 0, s>>>(src, H, W, C, t, nh, nw);
        }
        linear_kernel<<<(unsigned)cdiv(per, 256), 256, 0, s>>>(t, nh, nw, C, dst, H, W);
        break;
      }
      default:
        MX_CHECK_ARG(false, "mx_corrupt_u8: bad op %d", ops[b]);
    }
    MX_LAUNCH_CHECK();
  }
  return MX_OK;
}

extern "C" int mx_normalize_pad(const uint8_t* img, int64_t B, int64_t H, int64_t W, const float* mean, const float* stdv,
                                int64_t Hp, int64_t Wp, int64_t Cp, int dtype, void* out, mx_stream_t stream) {
  MX_CHECK_ARG(Hp >= H && Wp >= W && Cp >= 3, "mx_normalize_pad: bad padded shape");
  int64_t n = B * Hp * Wp;
  if (n == 0) return MX_OK;
  float3 m = make_float3(mean[0], mean[1], mean[2]), sd = make_float3(stdv[0], stdv[1], stdv[2]);
  if (dtype == MX_F32)
    normalize_pad_kernel<float><<<(unsigned)cdiv(n, 256), 256, 0, (hipStream_t)stream>>>(img, B, H, W, m, sd, Hp, Wp, Cp,
                                                                                          (float*)out);
  else
    normalize_pad_kernel<uint16_t><<<(unsigned)cdiv(n, 256), 256, 0, (hipStream_t)stream>>>(img, B, H, W, m, sd, Hp, Wp,
                                                                                             Cp, (uint16_t*)out);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

static int resize_normalize_pad(const void* const* imgs, bool f32chw, const int64_t* Hs, const int64_t* Ws,
                                const int64_t* nhs, const int64_t* nws, int64_t B, const float* mean, const float* stdv,
                                int64_t Hp, int64_t Wp, int64_t Cp, int dtype, void* out, hipStream_t stream) {
  MX_CHECK_ARG(B >= 0 && Cp >= 3 && Hp >= 0 && Wp >= 0, "mx_resize_normalize_pad: bad batch / padded shape");
  MX_CHECK_ARG(dtype == MX_F32 || dtype == MX_BF16, "mx_resize_normalize_pad: bad dtype %d", dtype);
  const float3 m = make_float3(mean[0], mean[1], mean[2]), sd = make_float3(stdv[0], stdv[1], stdv[2]);
  for (int64_t b0 = 0; b0 < B; b0 += RZ_MAX) {
    const int64_t nb = std::min<int64_t>(RZ_MAX, B - b0);
    RzBatch bt{};
    for (int64_t j = 0; j < nb; ++j) {
      const int64_t b = b0 + j;
      MX_CHECK_ARG(imgs[b] != nullptr && Hs[b] >= 1 && Ws[b] >= 1 && nhs[b] >= 1 && nws[b] >= 1,
                   "mx_resize_normalize_pad: image %lld: bad source / output size", (long long)b);
      MX_CHECK_ARG(nhs[b] <= Hp && nws[b] <= Wp, "mx_resize_normalize_pad: image %lld larger than the padded batch",
                   (long long)b);
      MX_CHECK_ARG(Hs[b] < (1 << 24) && Ws[b] < (1 << 24) && nhs[b] < (1 << 24) && nws[b] < (1 << 24),
                   "mx_resize_normalize_pad: image too large");
      RzImg& r = bt.im[j];
      r.src = imgs[b];
      r.H = (int)Hs[b]; r.W = (int)Ws[b]; r.nh = (int)nhs[b]; r.nw = (int)nws[b];
      r.sh = (float)r.H / (float)r.nh;  // area_pixel_compute_scale: static_cast<float>(in) / out
      r.sw = (float)r.W / (float)r.nw;
    }
    const int64_t n = nb * Hp * Wp;
    if (n == 0) continue;
    const size_t es = dtype == MX_F32 ? 4 : 2;
    char* o = (char*)out + (size_t)b0 * Hp * Wp * Cp * es;
    const unsigned g = (unsigned)cdiv(n, 256);
    if (dtype == MX_F32 && f32chw)
      resize_normalize_pad_kernel<float, true><<<g, 256, 0, stream>>>(bt, nb, m, sd, Hp, Wp, Cp, (float*)o);
    else if (dtype == MX_F32)
      resize_normalize_pad_kernel<float, false><<<g, 256, 0, stream>>>(bt, nb, m, sd, Hp, Wp, Cp, (float*)o);
    else if (f32chw)
      resize_normalize_pad_kernel<uint16_t, true><<<g, 256, 0, stream>>>(bt, nb, m, sd, Hp, Wp, Cp, (uint16_t*)o);
    else
      resize_normalize_pad_kernel<uint16_t, false><<<g, 256, 0, stream>>>(bt, nb, m, sd, Hp, Wp, Cp, (uint16_t*)o);
    MX_LAUNCH_CHECK();
  }
  return MX_OK;
}

extern "C" int mx_resize_normalize_pad(const uint8_t* const* imgs, const int64_t* Hs, const int64_t* Ws,
                                       const int64_t* nhs, const int64_t* nws, int64_t B, const float* mean,
                                       const float* stdv, int64_t Hp, int64_t Wp, int64_t Cp, int dtype, void* out,
                                       mx_stream_t stream) {
  return resize_normalize_pad((const void* const*)imgs, false, Hs, Ws, nhs, nws, B, mean, stdv, Hp, Wp, Cp, dtype, out,
                              (hipStream_t)stream);
}

extern "C" int mx_resize_normalize_pad_f32(const float* const* imgs_chw, const int64_t* Hs, const int64_t* Ws,
                                           const int64_t* nhs, const int64_t* nws, int64_t B, const float* mean,
                                           const float* stdv, int64_t Hp, int64_t Wp, int64_t Cp, int dtype, void* out,
                                           mx_stream_t stream) {
  return resize_normalize_pad((const void* const*)imgs_chw, true, Hs, Ws, nhs, nws, B, mean, stdv, Hp, Wp, Cp, dtype,
                              out, (hipStream_t)stream);
}

// ---- RPN head outputs <-> (objectness, pred_deltas) ----------------------------------------------
// The RPN head's 1x1 cls/bbox conv writes [N, H, W, 5A] per pixel (A logits, then A x 4 deltas): level 0
// as its own map o0, levels 1.. side by side on one zero-framed canvas (frcnn.RPNHead.canvas_layout).
// torchvision's concat_box_prediction_layers order is per image: level, then (h, w, a). Forward gathers
// both outputs in one pass; backward writes every element of both gradient maps (frame pixels 0).
struct RpnLayout {
  int y[8], x[8], h[8], w[8];  // canvas rectangles of levels 1..ncv (index 0 unused)
  int64_t base[9];             // first anchor of each level (level 0 = o0) within an image
  int ncv;                     // canvas levels
};

__device__ __forceinline__ int rpn_level(const RpnLayout& L, int64_t a) {
  int l = 0;
  while (l < L.ncv && a >= L.base[l + 1]) ++l;
  return l;
}

__global__ void rpn_head_split_kernel(const float* __restrict__ o0, int64_t H0, int64_t W0, const float* __restrict__ ocv,
                                      int64_t Hc, int64_t Wc, RpnLayout L, int64_t N, int A, int64_t Atot,
                                      float* __restrict__ obj, float* __restrict__ del) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * Atot) return;
  const int64_t n = i / Atot, ag = i - n * Atot;
  const int l = rpn_level(L, ag);
  const int64_t r = ag - L.base[l], p = r / A;
  const int a = (int)(r - p * A), C = 5 * A;
  const float* src;
  if (l == 0) {
    src = o0 + (n * H0 * W0 + p) * C;
  } else {
    const int64_t yy = p / L.w[l], xx = p - yy * L.w[l];
    src = ocv + ((n * Hc + L.y[l] + yy) * Wc + L.x[l] + xx) * C;
  }
  obj[i] = src[a];
  const float* d = src + A + 4 * a;
  *(float4*)(del + 4 * i) = make_float4(d[0], d[1], d[2], d[3]);
}

__global__ void rpn_head_merge_kernel(const float* __restrict__ gobj, const float* __restrict__ gdel, int64_t H0,
                                      int64_t W0, int64_t Hc, int64_t Wc, RpnLayout L, int64_t N, int A, int64_t Atot,
                                      float* __restrict__ g0, float* __restrict__ gcv) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int C = 5 * A;
  const int64_t n0 = N * H0 * W0 * C, ncv = gcv ? N * Hc * Wc * C : 0;
  if (i >= n0 + ncv) return;
  const int64_t e = i < n0 ? i : i - n0;
  const int64_t pix = e / C;
  const int ch = (int)(e - pix * C);
  int64_t ag = -1, n;
  if (i < n0) {
    n = pix / (H0 * W0);
    ag = (pix - n * H0 * W0) * A;
  } else {
    n = pix / (Hc * Wc);
    const int64_t yx = pix - n * Hc * Wc, yy = yx / Wc, xx = yx - yy * Wc;
    for (int l = 1; l <= L.ncv; ++l)
      if (yy >= L.y[l] && yy < L.y[l] + L.h[l] && xx >= L.x[l] && xx < L.x[l] + L.w[l]) {
        ag = L.base[l] + ((yy - L.y[l]) * L.w[l] + (xx - L.x[l])) * A;
        break;
      }
  }
  float v = 0.f;
  if (ag >= 0) {
    if (ch < A) {
      if (gobj) v = gobj[n * Atot + ag + ch];
    } else {
      const int a = (ch - A) >> 2, c = (ch - A) & 3;
      if (gdel) v = gdel[(n * Atot + ag + a) * 4 + c];
    }
  }
  (i < n0 ? g0 : gcv)[e] = v;
}

static int rpn_layout(const int32_t* rects, int ncv, int64_t H0, int64_t W0, int A, RpnLayout& L, int64_t& Atot) {
  MX_CHECK_ARG(ncv >= 0 && ncv <= 7 && A > 0 && H0 > 0 && W0 > 0 && (ncv == 0 || rects), "rpn head: bad layout");
  L = RpnLayout{};
  L.ncv = ncv;
  L.base[0] = 0;
  L.base[1] = H0 * W0 * A;
  for (int l = 1; l <= ncv; ++l) {
    L.y[l] = rects[4 * (l - 1)]; L.x[l] = rects[4 * (l - 1) + 1];
    L.h[l] = rects[4 * (l - 1) + 2]; L.w[l] = rects[4 * (l - 1) + 3];
    MX_CHECK_ARG(L.h[l] > 0 && L.w[l] > 0 && L.y[l] >= 0 && L.x[l] >= 0, "rpn head: bad level rectangle");
    L.base[l + 1] = L.base[l] + (int64_t)L.h[l] * L.w[l] * A;
  }
  Atot = L.base[ncv + 1];
  return MX_OK;
}

extern "C" int mx_rpn_head_split(const float* o0, int64_t H0, int64_t W0, const float* ocv, int64_t Hc, int64_t Wc,
                                 const int32_t* rects, int ncv, int64_t N, int A, float* obj, float* del,
                                 mx_stream_t stream) {
  RpnLayout L;
  int64_t Atot = 0;
  int rc = rpn_layout(rects, ncv, H0, W0, A, L, Atot);
  if (rc) return rc;
  MX_CHECK_ARG(o0 && obj && del && N > 0 && (ncv == 0 || ocv), "rpn head split: null buffer");
  for (int l = 1; l <= ncv; ++l)
    MX_CHECK_ARG(L.y[l] + L.h[l] <= Hc && L.x[l] + L.w[l] <= Wc, "rpn head split: level %d outside the canvas", l);
  const int64_t n = N * Atot;
  rpn_head_split_kernel<<<(unsigned)cdiv(n, 256), 256, 0, (hipStream_t)stream>>>(o0, H0, W0, ocv, Hc, Wc, L, N, A, Atot,
                                                                                 obj, del);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_rpn_head_merge(const float* gobj, const float* gdel, int64_t H0, int64_t W0, int64_t Hc, int64_t Wc,
                                 const int32_t* rects, int ncv, int64_t N, int A, float* g0, float* gcv,
                                 mx_stream_t stream) {
  RpnLayout L;
  int64_t Atot = 0;
  int rc = rpn_layout(rects, ncv, H0, W0, A, L, Atot);
  if (rc) return rc;
  MX_CHECK_ARG(g0 && N > 0 && (ncv == 0 || gcv), "rpn head merge: null buffer");
  for (int l = 1; l <= ncv; ++l)
    MX_CHECK_ARG(L.y[l] + L.h[l] <= Hc && L.x[l] + L.w[l] <= Wc, "rpn head merge: level %d outside the canvas", l);
  const int64_t n = N * H0 * W0 * 5 * A + (ncv ? N * Hc * Wc * 5 * A : 0);
  rpn_head_merge_kernel<<<(unsigned)cdiv(n, 256), 256, 0, (hipStream_t)stream>>>(gobj, gdel, H0, W0, Hc, Wc, L, N, A,
                                                                                 Atot, g0, ncv ? gcv : nullptr);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

// ---- zero-framed canvas of several NHWC maps (frcnn.RPNHead: P3..P6 as one conv input) ----------
struct CanvasRects {
  const void* f[8];  // pack: level maps [N, h, w, C]; unpack: optional maps added to the slices
  void* g[8];        // unpack: level gradients [N, h, w, C]
  int y[8], x[8], h[8], w[8];
  int n;
};

__device__ __forceinline__ int canvas_level(const CanvasRects& R, int64_t yy, int64_t xx) {
  for (int l = 0; l < R.n; ++l)
    if (yy >= R.y[l] && yy < R.y[l] + R.h[l] && xx >= R.x[l] && xx < R.x[l] + R.w[l]) return l;
  return -1;
}

// cv[n, y, x, :] = level l's pixel when (y, x) lies in rect l, else 0; 8 channels per thread
template <typename T>
__global__ void canvas_pack_kernel(CanvasRects R, int64_t N, int64_t Hc, int64_t Wc, int64_t C, T* __restrict__ cv) {
  const int64_t C8 = C / 8, i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * Hc * Wc * C8) return;
  const int64_t c0 = (i % C8) * 8, pix = i / C8, n = pix / (Hc * Wc), yx = pix - n * Hc * Wc;
  const int64_t yy = yx / Wc, xx = yx - yy * Wc;
  const int l = canvas_level(R, yy, xx);
  float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (l >= 0)
    ld8((const T*)R.f[l] + ((n * R.h[l] + (yy - R.y[l])) * R.w[l] + (xx - R.x[l])) * C + c0, v);
  st8(cv + pix * C + c0, v);
}

// g_l[n, y, x, :] = gcv at the level's slice (+ add_l[n, y, x, :] when given); one thread per 8
// channels of every level pixel
template <typename T>
__global__ void canvas_unpack_kernel(CanvasRects R, int64_t N, int64_t Hc, int64_t Wc, int64_t C, const T* __restrict__ gcv,
                                     int64_t total8) {
  const int64_t C8 = C / 8;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total8) return;
  int l = 0;
  for (; l < R.n; ++l) {
    const int64_t nl = N * R.h[l] * R.w[l] * C8;
    if (i < nl) break;
    i -= nl;
  }
  const int64_t c0 = (i % C8) * 8, pix = i / C8, hw = (int64_t)R.h[l] * R.w[l];
  const int64_t n = pix / hw, yx = pix - n * hw, yy = yx / R.w[l], xx = yx - yy * R.w[l];
  float v[8];
  ld8(gcv + ((n * Hc + R.y[l] + yy) * Wc + R.x[l] + xx) * C + c0, v);
  if (R.f[l]) {
    float a[8];
    ld8((const T*)R.f[l] + pix * C + c0, a);
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] += a[t];
  }
  st8((T*)R.g[l] + pix * C + c0, v);
}

static int canvas_rects(const int32_t* rects, int n, int64_t Hc, int64_t Wc, int64_t C, CanvasRects& R) {
  MX_CHECK_ARG(n >= 1 && n <= 8 && rects && C > 0 && C % 8 == 0 && Hc > 0 && Wc > 0, "canvas: bad layout (C %% 8 == 0)");
  R = CanvasRects{};
  R.n = n;
  for (int l = 0; l < n; ++l) {
    R.y[l] = rects[4 * l]; R.x[l] = rects[4 * l + 1]; R.h[l] = rects[4 * l + 2]; R.w[l] = rects[4 * l + 3];
    MX_CHECK_ARG(R.h[l] > 0 && R.w[l] > 0 && R.y[l] >= 0 && R.x[l] >= 0 && R.y[l] + R.h[l] <= Hc &&
                 R.x[l] + R.w[l] <= Wc, "canvas: rect %d outside the canvas", l);
  }
  return MX_OK;
}

extern "C" int mx_canvas_pack(const void* const* maps, const int32_t* rects, int n, int64_t N, int64_t Hc, int64_t Wc,
                              int64_t C, int dtype, void* cv, mx_stream_t stream) {
  CanvasRects R;
  int rc = canvas_rects(rects, n, Hc, Wc, C, R);
  if (rc) return rc;
  MX_CHECK_ARG(maps && cv && N > 0, "canvas pack: null buffer");
  for (int l = 0; l < n; ++l) {
    MX_CHECK_ARG(maps[l], "canvas pack: map %d null", l);
    R.f[l] = maps[l];
  }
  const int64_t tot = N * Hc * Wc * (C / 8);
  hipStream_t st = (hipStream_t)stream;
  MX_CHECK_ARG(dtype == MX_F32 || dtype == MX_BF16, "canvas pack: bad dtype %d", dtype);
  if (dtype == MX_F32)
    canvas_pack_kernel<float><<<(unsigned)cdiv(tot, 256), 256, 0, st>>>(R, N, Hc, Wc, C, (float*)cv);
  else
    canvas_pack_kernel<uint16_t><<<(unsigned)cdiv(tot, 256), 256, 0, st>>>(R, N, Hc, Wc, C, (uint16_t*)cv);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_canvas_unpack(const void* gcv, const int32_t* rects, int n, int64_t N, int64_t Hc, int64_t Wc,
                                int64_t C, int dtype, const void* const* add, void* const* grads, mx_stream_t stream) {
  CanvasRects R;
  int rc = canvas_rects(rects, n, Hc, Wc, C, R);
  if (rc) return rc;
  MX_CHECK_ARG(gcv && grads && N > 0, "canvas unpack: null buffer");
  int64_t tot = 0;
  for (int l = 0; l < n; ++l) {
    MX_CHECK_ARG(grads[l], "canvas unpack: gradient %d null", l);
    R.g[l] = grads[l];
    R.f[l] = add ? add[l] : nullptr;
    tot += N * R.h[l] * R.w[l] * (C / 8);
  }
  hipStream_t st = (hipStream_t)stream;
  MX_CHECK_ARG(dtype == MX_F32 || dtype == MX_BF16, "canvas unpack: bad dtype %d", dtype);
  if (dtype == MX_F32)
    canvas_unpack_kernel<float><<<(unsigned)cdiv(tot, 256), 256, 0, st>>>(R, N, Hc, Wc, C, (const float*)gcv, tot);
  else
    canvas_unpack_kernel<uint16_t><<<(unsigned)cdiv(tot, 256), 256, 0, st>>>(R, N, Hc, Wc, C, (const uint16_t*)gcv,
                                                                            tot);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

// RPN canvas frame mask between the head's convs (frcnn RPNHead.raw: t * mask, mask [Hc][Wc] of 0 / 1 per
// pixel): y = x * mask[pixel] in f32 (the same IEEE products as torch's broadcast multiply: x * 1 = x,
// x * 0 = +-0 or NaN), 8 channels per thread with 16-B accesses; planes (f32 only, nullable): y's bf16x3
// hi / lo planes [2][N*HW*C] for the next conv's x3p operand. Used both ways (the backward is g * mask).
template <typename T>
__global__ void mask_pixels_kernel(const T* __restrict__ x, const float* __restrict__ mask, int64_t HW, int64_t C8,
                                   int64_t n8, T* __restrict__ y, uint16_t* __restrict__ planes) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n8) return;
  const float m = mask[(e / C8) % HW];
  float v[8];
  ld8(x + e * 8, v);
#pragma unroll
  for (int t = 0; t < 8; ++t) v[t] *= m;
  st8(y + e * 8, v);
  if (planes) {
    uint4 h, l;
    split8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), h, l);
    *(uint4*)(planes + e * 8) = h;
    *(uint4*)(planes + n8 * 8 + e * 8) = l;
  }
}

extern "C" int mx_mask_pixels(const void* x, int dtype, const float* mask, int64_t N, int64_t HW, int64_t C, void* y,
                              uint16_t* planes, mx_stream_t stream) {
  MX_CHECK_ARG(N >= 0 && HW >= 0 && C > 0 && C % 8 == 0, "mask_pixels: C must be a positive multiple of 8");
  MX_CHECK_ARG(dtype == MX_F32 || (dtype == MX_BF16 && !planes), "mask_pixels: f32, or bf16 without planes");
  const int64_t n8 = N * HW * (C / 8);
  if (n8 == 0) return MX_OK;
  MX_CHECK_ARG(x && mask && y, "mask_pixels: null operand");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == MX_F32)
    mask_pixels_kernel<float><<<(unsigned)cdiv(n8, 256), 256, 0, st>>>((const float*)x, mask, HW, C / 8, n8, (float*)y,
                                                                      planes);
  else
    mask_pixels_kernel<uint16_t><<<(unsigned)cdiv(n8, 256), 256, 0, st>>>((const uint16_t*)x, mask, HW, C / 8, n8,
                                                                         (uint16_t*)y, nullptr);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

// Empty kernel that marks a point in a rocprofv3 kernel trace (bench.py brackets its timed steps with
// ids 1 and 2, tools/prof_steps.py keeps only the dispatches between them).
__global__ void trace_marker_kernel(int id) { (void)id; }

extern "C" int mx_trace_marker(int id, mx_stream_t stream) {
  trace_marker_kernel<<<1, 64, 0, (hipStream_t)stream>>>(id);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

// the same with the device's highest stream priority (hipStreamCreateWithPriority): a small hand-off that must
// not queue behind the step's kernels on a shared hardware queue (DataParallel's NMS-flag read)
extern "C" int mx_stream_create_high_priority(int device, mx_stream_t* out) {
  MX_CHECK_ARG(out != nullptr, "mx_stream_create_high_priority: null output");
  int prev = 0;
  MX_HIP(hipGetDevice(&prev));
  MX_HIP(hipSetDevice(device));
  int least = 0, greatest = 0;
  hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
  hipStream_t s = nullptr;
  if (e == hipSuccess) e = hipStreamCreateWithPriority(&s, hipStreamNonBlocking, greatest);
  MX_HIP(hipSetDevice(prev));
  MX_HIP(e);
  *out = (mx_stream_t)s;
  return MX_OK;
}

extern "C" int mx_stream_create(int device, mx_stream_t* out) {
  MX_CHECK_ARG(out != nullptr, "mx_stream_create: null output");
  int prev = 0;
  MX_HIP(hipGetDevice(&prev));
  MX_HIP(hipSetDevice(device));
  hipStream_t s = nullptr;
  const hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  MX_HIP(hipSetDevice(prev));
  MX_HIP(e);
  *out = (mx_stream_t)s;
  return MX_OK;
}
