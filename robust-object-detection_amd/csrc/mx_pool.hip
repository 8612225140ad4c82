// mx_pool.hip — NHWC max-pool and nearest upsample (fwd + adjoint) for the ResNet stem, FPN
// top-down path and the U-Net encoder (gfx950). bf16 or f32 storage (dtype argument), 8 channels per
// lane.
//
//  maxpool: torch.nn.functional.max_pool2d semantics (-inf padding, first max in window order on
//           ties for the backward; ResNet stem k3 s2 p1, U-Net MaxPool2d(2), P6 = max_pool(P5,1,2)).
//  upsample_nearest: F.interpolate(mode="nearest", size=...): src = min(floor(dst*in/out), in-1)
//           with the scale computed in f32 (FPN top-down, torchvision ops/feature_pyramid_network.py).
//           Backward = per-source-pixel sum over the destinations that read it (gather, no atomics).
#include "mx_common.h"

namespace mx {

__device__ __forceinline__ int near_src(int d, int in, int out) {
  float sc = (float)in / (float)out;
  int s = (int)floorf((float)d * sc);
  return s < in - 1 ? s : in - 1;
}

template <typename T>
__global__ void maxpool_fwd_kernel(const T* __restrict__ x, int64_t N, int64_t H, int64_t W, int64_t C, int64_t Ho,
                                   int64_t Wo, int k, int st, int pd, T* __restrict__ y, int32_t* __restrict__ arg) {
  const int64_t C8 = C / 8;
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N * Ho * Wo * C8) return;
  int64_t c8 = e % C8, t = e / C8;
  int64_t ow = t % Wo, oh = (t / Wo) % Ho, n = t / (Wo * Ho);
  float best[8];
  int32_t bi[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) { best[q] = -INFINITY; bi[q] = -1; }
  for (int r = 0; r < k; ++r) {
    int64_t ih = oh * st - pd + r;
    if (ih < 0 || ih >= H) continue;
    for (int s = 0; s < k; ++s) {
      int64_t iw = ow * st - pd + s;
      if (iw < 0 || iw >= W) continue;
      float vv[8];
      ld8(x + ((n * H + ih) * W + iw) * C + c8 * 8, vv);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float v = vv[q];
        if (v > best[q] || bi[q] < 0 || v != v) { best[q] = v; bi[q] = (int32_t)(ih * W + iw); }
      }
    }
  }
  st8(y + t * C + c8 * 8, best);
  if (arg) {
#pragma unroll
    for (int q = 0; q < 8; ++q) arg[t * C + c8 * 8 + q] = bi[q];
  }
}

// gather form: input pixel (h,w) sums grads of the output windows whose argmax is (h,w)
template <typename T>
__global__ void maxpool_bwd_kernel(const T* __restrict__ gy, const int32_t* __restrict__ arg, int64_t N, int64_t H,
                                   int64_t W, int64_t C, int64_t Ho, int64_t Wo, int k, int st, int pd,
                                   T* __restrict__ gx) {
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N * H * W * C) return;
  int64_t c = e % C, t = e / C;
  int64_t w = t % W, h = (t / W) % H, n = t / (W * H);
  int32_t me = (int32_t)(h * W + w);
  // output rows oh with oh*st - pd <= h <= oh*st - pd + k - 1
  int64_t oh0 = (h + pd - k + st) / st; if (h + pd - k + 1 < 0) oh0 = 0;
  int64_t oh1 = (h + pd) / st;
  int64_t ow0 = (w + pd - k + st) / st; if (w + pd - k + 1 < 0) ow0 = 0;
  int64_t ow1 = (w + pd) / st;
  float acc = 0.f;
  for (int64_t oh = max<int64_t>(oh0, 0); oh <= min<int64_t>(oh1, Ho - 1); ++oh)
    for (int64_t ow = max<int64_t>(ow0, 0); ow <= min<int64_t>(ow1, Wo - 1); ++ow) {
      int64_t o = ((n * Ho + oh) * Wo + ow) * C + c;
      if (arg[o] == me) acc += ld1(gy + o);
    }
  st1(gx + e, acc);
}

// y = up(x) (+ add), NHWC
template <typename T>
__global__ void upsample_fwd_kernel(const T* __restrict__ x, int64_t N, int64_t H, int64_t W, int64_t C, int64_t Ho,
                                    int64_t Wo, const T* __restrict__ add, T* __restrict__ y) {
  const int64_t C8 = C / 8;
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N * Ho * Wo * C8) return;
  int64_t c8 = e % C8, t = e / C8;
  int64_t ow = t % Wo, oh = (t / Wo) % Ho, n = t / (Wo * Ho);
  int64_t ih = near_src((int)oh, (int)H, (int)Ho), iw = near_src((int)ow, (int)W, (int)Wo);
  float v[8];
  ld8(x + ((n * H + ih) * W + iw) * C + c8 * 8, v);
  if (add) {
    float a[8];
    ld8(add + t * C + c8 * 8, a);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] += a[q];
  }
  st8(y + t * C + c8 * 8, v);
}

// The same with one grid row per output image row (blockIdx.y = n * Ho + oh) and 32-bit index math: the
// generic form's five 64-bit divisions per thread made the FPN top-down P2 upsample run at ~2 TB/s
template <typename T>
__global__ void upsample_fwd_rows_kernel(const T* __restrict__ x, int H, int W, int C8, int Ho, int Wo,
                                         const T* __restrict__ add, T* __restrict__ y) {
  const int row = blockIdx.y, oh = row % Ho, n = row / Ho;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= Wo * C8) return;
  const int ow = idx / C8, c8 = idx - ow * C8;
  const int ih = near_src(oh, H, Ho), iw = near_src(ow, W, Wo);
  const int64_t src = (((int64_t)n * H + ih) * W + iw) * C8 + c8;  // in 8-element chunks
  const int64_t dst = (int64_t)row * Wo * C8 + idx;
  float v[8];
  ld8(x + src * 8, v);
  if (add) {
    float a[8];
    ld8(add + dst * 8, a);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] += a[q];
  }
  st8(y + dst * 8, v);
}

// gx[src] = sum over dst with near_src(dst) == src of gy[dst]
template <typename T>
__global__ void upsample_bwd_kernel(const T* __restrict__ gy, int64_t N, int64_t H, int64_t W, int64_t C, int64_t Ho,
                                    int64_t Wo, T* __restrict__ gx) {
  const int64_t C8 = C / 8;
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N * H * W * C8) return;
  int64_t c8 = e % C8, t = e / C8;
  int64_t iw = t % W, ih = (t / W) % H, n = t / (W * H);
  // destinations mapping to ih: dst in [lo, hi) ; scan a small window around ih*Ho/H
  int64_t oh_lo = (ih * Ho) / H - 1, ow_lo = (iw * Wo) / W - 1;
  int64_t oh_hi = ((ih + 1) * Ho + H - 1) / H + 1, ow_hi = ((iw + 1) * Wo + W - 1) / W + 1;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t oh = max<int64_t>(oh_lo, 0); oh < min<int64_t>(oh_hi, Ho); ++oh) {
    if (near_src((int)oh, (int)H, (int)Ho) != ih) continue;
    for (int64_t ow = max<int64_t>(ow_lo, 0); ow < min<int64_t>(ow_hi, Wo); ++ow) {
      if (near_src((int)ow, (int)W, (int)Wo) != iw) continue;
      float v[8];
      ld8(gy + ((n * Ho + oh) * Wo + ow) * C + c8 * 8, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += v[q];
    }
  }
  st8(gx + t * C + c8 * 8, acc);
}

}  // namespace mx

using namespace mx;


template <typename T>
static void maxpool_fwd_launch(const void* x, int64_t N, int64_t H, int64_t W, int64_t C, int64_t Ho, int64_t Wo, int k,
                               int st, int pd, void* y, int32_t* arg, int64_t n, hipStream_t s) {
  maxpool_fwd_kernel<T><<<(unsigned)cdiv(n, 256), 256, 0, s>>>((const T*)x, N, H, W, C, Ho, Wo, k, st, pd, (T*)y, arg);
}
template <typename T>
static void maxpool_bwd_launch(const void* gy, const int32_t* arg, int64_t N, int64_t H, int64_t W, int64_t C, int64_t Ho,
                               int64_t Wo, int k, int st, int pd, void* gx, int64_t n, hipStream_t s) {
  maxpool_bwd_kernel<T><<<(unsigned)cdiv(n, 256), 256, 0, s>>>((const T*)gy, arg, N, H, W, C, Ho, Wo, k, st, pd, (T*)gx);
}
template <typename T>
static void upsample_fwd_launch(const void* x, int64_t N, int64_t H, int64_t W, int64_t C, int64_t Ho, int64_t Wo,
                                const void* add, void* y, int64_t n, hipStream_t s) {
  if (N * Ho <= 65535 && Wo * (C / 8) < (1 << 30) && H * W < (1 << 30)) {
    const dim3 grid((unsigned)cdiv(Wo * (C / 8), 256), (unsigned)(N * Ho));
    upsample_fwd_rows_kernel<T><<<grid, 256, 0, s>>>((const T*)x, (int)H, (int)W, (int)(C / 8), (int)Ho, (int)Wo,
                                                     (const T*)add, (T*)y);
    return;
  }
  upsample_fwd_kernel<T><<<(unsigned)cdiv(n, 256), 256, 0, s>>>((const T*)x, N, H, W, C, Ho, Wo, (const T*)add, (T*)y);
}
template <typename T>
static void upsample_bwd_launch(const void* gy, int64_t N, int64_t H, int64_t W, int64_t C, int64_t Ho, int64_t Wo,
                                void* gx, int64_t n, hipStream_t s) {
  upsample_bwd_kernel<T><<<(unsigned)cdiv(n, 256), 256, 0, s>>>((const T*)gy, N, H, W, C, Ho, Wo, (T*)gx);
}

extern "C" int mx_maxpool_fwd(const void* x, int dtype, int64_t N, int64_t H, int64_t W, int64_t C, int k, int stride,
                              int pad, void* y, int32_t* argmax, mx_stream_t stream) {
  MX_CHECK_ARG(C % 8 == 0 && k > 0 && stride > 0 && pad >= 0 && pad * 2 <= k, "maxpool: bad args");
  int64_t Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  int64_t n = N * Ho * Wo * (C / 8);
  if (n == 0) return MX_OK;
  MX_DT_DISPATCH(dtype, maxpool_fwd_launch, x, N, H, W, C, Ho, Wo, k, stride, pad, y, argmax, n, (hipStream_t)stream);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_maxpool_bwd(const void* gy, int dtype, const int32_t* argmax, int64_t N, int64_t H, int64_t W, int64_t C,
                              int k, int stride, int pad, void* gx, mx_stream_t stream) {
  MX_CHECK_ARG(argmax != nullptr, "maxpool_bwd: argmax from the forward required");
  int64_t Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  int64_t n = N * H * W * C;
  if (n == 0) return MX_OK;
  MX_DT_DISPATCH(dtype, maxpool_bwd_launch, gy, argmax, N, H, W, C, Ho, Wo, k, stride, pad, gx, n, (hipStream_t)stream);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_upsample_nearest_fwd(const void* x, int dtype, int64_t N, int64_t H, int64_t W, int64_t C, int64_t Ho,
                                       int64_t Wo, const void* add, void* y, mx_stream_t stream) {
  MX_CHECK_ARG(C % 8 == 0, "upsample: C %% 8 != 0");
  int64_t n = N * Ho * Wo * (C / 8);
  if (n == 0) return MX_OK;
  MX_DT_DISPATCH(dtype, upsample_fwd_launch, x, N, H, W, C, Ho, Wo, add, y, n, (hipStream_t)stream);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_upsample_nearest_bwd(const void* gy, int dtype, int64_t N, int64_t H, int64_t W, int64_t C, int64_t Ho,
                                       int64_t Wo, void* gx, mx_stream_t stream) {
  MX_CHECK_ARG(C % 8 == 0, "upsample: C %% 8 != 0");
  int64_t n = N * H * W * (C / 8);
  if (n == 0) return MX_OK;
  MX_DT_DISPATCH(dtype, upsample_bwd_launch, gy, N, H, W, C, Ho, Wo, gx, n, (hipStream_t)stream);
  MX_LAUNCH_CHECK();
  return MX_OK;
}
