// mx_pool.hip — NHWC max-pool and nearest upsample (fwd + adjoint) for the ResNet stem, FPN
// top-down path and the U-Net encoder (gfx950). bf16 storage, 8 channels (16 B) per lane.
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

__global__ void maxpool_fwd_kernel(const uint16_t* __restrict__ x, int64_t N, int64_t H, int64_t W, int64_t C, int64_t Ho,
                                   int64_t Wo, int k, int st, int pd, uint16_t* __restrict__ y, int32_t* __restrict__ arg) {
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
      uint4 u = *(const uint4*)(x + ((n * H + ih) * W + iw) * C + c8 * 8);
      const uint16_t* h = (const uint16_t*)&u;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float v = bf2f(h[q]);
        if (v > best[q] || bi[q] < 0 || v != v) { best[q] = v; bi[q] = (int32_t)(ih * W + iw); }
      }
    }
  }
  uint4 o;
  uint16_t* oh16 = (uint16_t*)&o;
#pragma unroll
  for (int q = 0; q < 8; ++q) oh16[q] = f2bf(best[q]);
  *(uint4*)(y + t * C + c8 * 8) = o;
  if (arg) {
#pragma unroll
    for (int q = 0; q < 8; ++q) arg[t * C + c8 * 8 + q] = bi[q];
  }
}

// gather form: input pixel (h,w) sums grads of the output windows whose argmax is (h,w)
__global__ void maxpool_bwd_kernel(const uint16_t* __restrict__ gy, const int32_t* __restrict__ arg, int64_t N, int64_t H,
                                   int64_t W, int64_t C, int64_t Ho, int64_t Wo, int k, int st, int pd,
                                   uint16_t* __restrict__ gx) {
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
      if (arg[o] == me) acc += bf2f(gy[o]);
    }
  gx[e] = f2bf(acc);
}

// y = up(x) (+ add), NHWC
__global__ void upsample_fwd_kernel(const uint16_t* __restrict__ x, int64_t N, int64_t H, int64_t W, int64_t C, int64_t Ho,
                                    int64_t Wo, const uint16_t* __restrict__ add, uint16_t* __restrict__ y) {
  const int64_t C8 = C / 8;
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N * Ho * Wo * C8) return;
  int64_t c8 = e % C8, t = e / C8;
  int64_t ow = t % Wo, oh = (t / Wo) % Ho, n = t / (Wo * Ho);
  int64_t ih = near_src((int)oh, (int)H, (int)Ho), iw = near_src((int)ow, (int)W, (int)Wo);
  uint4 u = *(const uint4*)(x + ((n * H + ih) * W + iw) * C + c8 * 8);
  if (add) {
    uint4 a = *(const uint4*)(add + t * C + c8 * 8);
    uint16_t* uh = (uint16_t*)&u;
    const uint16_t* ah = (const uint16_t*)&a;
#pragma unroll
    for (int q = 0; q < 8; ++q) uh[q] = f2bf(bf2f(uh[q]) + bf2f(ah[q]));
  }
  *(uint4*)(y + t * C + c8 * 8) = u;
}

// gx[src] = sum over dst with near_src(dst) == src of gy[dst]
__global__ void upsample_bwd_kernel(const uint16_t* __restrict__ gy, int64_t N, int64_t H, int64_t W, int64_t C, int64_t Ho,
                                    int64_t Wo, uint16_t* __restrict__ gx) {
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
      uint4 u = *(const uint4*)(gy + ((n * Ho + oh) * Wo + ow) * C + c8 * 8);
      const uint16_t* h = (const uint16_t*)&u;
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += bf2f(h[q]);
    }
  }
  uint4 o;
  uint16_t* oh16 = (uint16_t*)&o;
#pragma unroll
  for (int q = 0; q < 8; ++q) oh16[q] = f2bf(acc[q]);
  *(uint4*)(gx + t * C + c8 * 8) = o;
}

}  // namespace mx

using namespace mx;

extern "C" int mx_maxpool_fwd(const uint16_t* x, int64_t N, int64_t H, int64_t W, int64_t C, int k, int stride, int pad,
                              uint16_t* y, int32_t* argmax, mx_stream_t stream) {
  MX_CHECK_ARG(C % 8 == 0 && k > 0 && stride > 0 && pad >= 0 && pad * 2 <= k, "maxpool: bad args");
  int64_t Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  int64_t n = N * Ho * Wo * (C / 8);
  if (n == 0) return MX_OK;
  maxpool_fwd_kernel<<<(unsigned)cdiv(n, 256), 256, 0, (hipStream_t)stream>>>(x, N, H, W, C, Ho, Wo, k, stride, pad, y, argmax);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_maxpool_bwd(const uint16_t* gy, const int32_t* argmax, int64_t N, int64_t H, int64_t W, int64_t C, int k,
                              int stride, int pad, uint16_t* gx, mx_stream_t stream) {
  MX_CHECK_ARG(argmax != nullptr, "maxpool_bwd: argmax from the forward required");
  int64_t Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  int64_t n = N * H * W * C;
  if (n == 0) return MX_OK;
  maxpool_bwd_kernel<<<(unsigned)cdiv(n, 256), 256, 0, (hipStream_t)stream>>>(gy, argmax, N, H, W, C, Ho, Wo, k, stride, pad,
                                                                               gx);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_upsample_nearest_fwd(const uint16_t* x, int64_t N, int64_t H, int64_t W, int64_t C, int64_t Ho, int64_t Wo,
                                       const uint16_t* add, uint16_t* y, mx_stream_t stream) {
  MX_CHECK_ARG(C % 8 == 0, "upsample: C %% 8 != 0");
  int64_t n = N * Ho * Wo * (C / 8);
  if (n == 0) return MX_OK;
  upsample_fwd_kernel<<<(unsigned)cdiv(n, 256), 256, 0, (hipStream_t)stream>>>(x, N, H, W, C, Ho, Wo, add, y);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_upsample_nearest_bwd(const uint16_t* gy, int64_t N, int64_t H, int64_t W, int64_t C, int64_t Ho, int64_t Wo,
                                       uint16_t* gx, mx_stream_t stream) {
  MX_CHECK_ARG(C % 8 == 0, "upsample: C %% 8 != 0");
  int64_t n = N * H * W * (C / 8);
  if (n == 0) return MX_OK;
  upsample_bwd_kernel<<<(unsigned)cdiv(n, 256), 256, 0, (hipStream_t)stream>>>(gy, N, H, W, C, Ho, Wo, gx);
  MX_LAUNCH_CHECK();
  return MX_OK;
}
