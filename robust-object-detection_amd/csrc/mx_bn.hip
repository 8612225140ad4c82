// mx_bn.hip — train-mode BatchNorm2d around the conv stack, NHWC rows x channels (gfx950).
//
// torch.nn.BatchNorm2d semantics (the reference model keeps nn.BatchNorm2d in train mode in the
// backbone, FPN and box head: torchvision fasterrcnn_resnet50_fpn_v2, model.train() at
// train_frcnn_baseline.py:164): normalise with the biased batch variance, update running stats with
// momentum 0.1 and the unbiased variance; backward
//   dx = gamma*invstd*(g - mean(g) - xhat*mean(g*xhat)),  g = dy * act'(y).
// Statistics arrive as per-block column partials from the conv epilogue (mx_conv.hip) and are
// reduced here in f64.
#include "mx_common.h"

namespace mx {

__device__ __forceinline__ float actf(float v, int act) {
  if (act == 1) return v > 0.f ? v : 0.f;
  if (act == 2) return v > 0.f ? v : 0.2f * v;
  return v;
}
__device__ __forceinline__ float actd(float y, int act) {
  if (act == 1) return y > 0.f ? 1.f : 0.f;
  if (act == 2) return y > 0.f ? 1.f : 0.2f;
  return 1.f;
}

// block = 16 channels x 16 row-slices of the per-block partials; f64 sums; LDS tree over slices
__global__ void __launch_bounds__(256) bn_finalize_kernel(const float* __restrict__ stats, int64_t mb, int64_t K, int64_t count,
                                   const float* __restrict__ gamma, const float* __restrict__ beta, float eps, float mom,
                                   float* __restrict__ rmean, float* __restrict__ rvar, float* __restrict__ mean_o,
                                   float* __restrict__ invstd_o, float* __restrict__ scale_o, float* __restrict__ shift_o) {
  __shared__ double ps[16][17], pq[16][17];
  const int cl = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int64_t k = (int64_t)blockIdx.x * 16 + cl;
  double s = 0.0, q = 0.0;
  if (k < K)
    for (int64_t b = sl; b < mb; b += 16) {
      s += (double)stats[b * K + k];
      q += (double)stats[(mb + b) * K + k];
    }
  ps[sl][cl] = s;
  pq[sl][cl] = q;
  __syncthreads();
  if (sl == 0 && k < K) {
    s = 0.0; q = 0.0;
#pragma unroll
    for (int t = 0; t < 16; ++t) { s += ps[t][cl]; q += pq[t][cl]; }
    double mean = s / (double)count;
    double var = q / (double)count - mean * mean;
    if (var < 0.0) var = 0.0;
    float invstd = (float)(1.0 / sqrt(var + (double)eps));
    float g = gamma ? gamma[k] : 1.f, bb = beta ? beta[k] : 0.f;
    mean_o[k] = (float)mean;
    invstd_o[k] = invstd;
    scale_o[k] = g * invstd;
    shift_o[k] = bb - (float)mean * (g * invstd);
    if (rmean) {
      double unb = count > 1 ? var * (double)count / (double)(count - 1) : var;
      rmean[k] = (float)((1.0 - mom) * rmean[k] + mom * mean);
      rvar[k] = (float)((1.0 - mom) * rvar[k] + mom * unb);
    }
  }
}

// Thread t owns channel chunk c8 = t % K8 for its whole life (per-channel constants stay in
// registers) and walks rows r = t / K8 + i * (T / K8): 16-B vector loads/stores, coalesced per row.
template <typename T>
__global__ void __launch_bounds__(256) bn_apply_kernel(const T* __restrict__ x, int64_t M, int64_t K, const float* __restrict__ scale,
                                const float* __restrict__ shift, const uint16_t* __restrict__ res, int act,
                                uint16_t* __restrict__ y) {
  const int64_t K8 = K / 8;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t rstride = ((int64_t)gridDim.x * blockDim.x) / K8;
  if (t >= rstride * K8) return;
  const int64_t c8 = t % K8, c0 = c8 * 8;
  float sc[8], sh[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) { sc[q] = scale[c0 + q]; sh[q] = shift[c0 + q]; }
  for (int64_t r = t / K8; r < M; r += rstride) {
    const int64_t e = r * K8 + c8;
    float v[8];
    if constexpr (sizeof(T) == 2) {
      uint4 u = *(const uint4*)(x + e * 8);
      const uint16_t* h = (const uint16_t*)&u;
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = bf2f(h[q]);
    } else {
      *(float4*)&v[0] = *(const float4*)(x + e * 8);
      *(float4*)&v[4] = *(const float4*)(x + e * 8 + 4);
    }
    float rv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (res) {
      uint4 u = *(const uint4*)(res + e * 8);
      const uint16_t* h = (const uint16_t*)&u;
#pragma unroll
      for (int q = 0; q < 8; ++q) rv[q] = bf2f(h[q]);
    }
    uint4 o;
    uint16_t* oh = (uint16_t*)&o;
#pragma unroll
    for (int q = 0; q < 8; ++q) oh[q] = f2bf(actf(v[q] * sc[q] + sh[q] + rv[q], act));
    *(uint4*)(y + e * 8) = o;
  }
}

// rows split over blocks; thread = (8-channel chunk, row lane); partials reduced in LDS, then atomics
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ y,
                                                            const uint16_t* __restrict__ x, int64_t M, int64_t K, int act,
                                                            const float* __restrict__ mean, const float* __restrict__ invstd,
                                                            int64_t rows_per_block, float* __restrict__ sums) {
  extern __shared__ float red[];  // [2][K]
  const int64_t K8 = K / 8;
  for (int64_t i = threadIdx.x; i < 2 * K; i += blockDim.x) red[i] = 0.f;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min<int64_t>(M, r0 + rows_per_block);
  const int lanes_per_row = (int)min<int64_t>(K8, blockDim.x);
  const int rows_par = blockDim.x / lanes_per_row;
  const int cl = threadIdx.x % lanes_per_row, rl = threadIdx.x / lanes_per_row;
  if (rl < rows_par)
    for (int64_t c8 = cl; c8 < K8; c8 += lanes_per_row) {
      float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      float mu[8], is[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) { mu[t] = mean[c8 * 8 + t]; is[t] = invstd[c8 * 8 + t]; }
      for (int64_t r = r0 + rl; r < r1; r += rows_par) {
        uint4 ud = *(const uint4*)(dy + r * K + c8 * 8);
        uint4 uy = *(const uint4*)(y + r * K + c8 * 8);
        uint4 ux = *(const uint4*)(x + r * K + c8 * 8);
        const uint16_t *hd = (const uint16_t*)&ud, *hy = (const uint16_t*)&uy, *hx = (const uint16_t*)&ux;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          float g = bf2f(hd[t]) * actd(bf2f(hy[t]), act);
          float xh = (bf2f(hx[t]) - mu[t]) * is[t];
          s[t] += g;
          q[t] += g * xh;
        }
      }
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        atomicAdd(&red[c8 * 8 + t], s[t]);
        atomicAdd(&red[K + c8 * 8 + t], q[t]);
      }
    }
  __syncthreads();
  for (int64_t i = threadIdx.x; i < 2 * K; i += blockDim.x) atomicAdd(&sums[i], red[i]);
}

__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ y,
                                    const uint16_t* __restrict__ x, int64_t M, int64_t K, int act,
                                    const float* __restrict__ mean, const float* __restrict__ invstd,
                                    const float* __restrict__ gamma, const float* __restrict__ sums,
                                    uint16_t* __restrict__ dx, uint16_t* __restrict__ dres) {
  const int64_t K8 = K / 8;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t rstride = ((int64_t)gridDim.x * blockDim.x) / K8;
  if (t >= rstride * K8) return;
  const int64_t c8 = t % K8, c0 = c8 * 8;
  const float invM = 1.0f / (float)M;
  // dx = a*g + b*x + c  with a = gamma*invstd, b = -a*invstd*mean(g*xhat), c = -a*(mean(g) - mean*invstd*mean(g*xhat))
  float A[8], Bc[8], Cc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int64_t c = c0 + q;
    float is = invstd[c], a = (gamma ? gamma[c] : 1.f) * is;
    float mg = sums[c] * invM, mgx = sums[K + c] * invM;
    A[q] = a;
    Bc[q] = -a * is * mgx;
    Cc[q] = -a * (mg - mean[c] * is * mgx);
  }
  for (int64_t r = t / K8; r < M; r += rstride) {
    const int64_t e = r * K8 + c8;
    uint4 ud = *(const uint4*)(dy + e * 8), uy = *(const uint4*)(y + e * 8), ux = *(const uint4*)(x + e * 8);
    const uint16_t *hd = (const uint16_t*)&ud, *hy = (const uint16_t*)&uy, *hx = (const uint16_t*)&ux;
    uint4 o, orr;
    uint16_t* oh = (uint16_t*)&o;
    uint16_t* orh = (uint16_t*)&orr;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float g = bf2f(hd[q]) * actd(bf2f(hy[q]), act);
      oh[q] = f2bf(A[q] * g + Bc[q] * bf2f(hx[q]) + Cc[q]);
      orh[q] = f2bf(g);
    }
    *(uint4*)(dx + e * 8) = o;
    if (dres) *(uint4*)(dres + e * 8) = orr;
  }
}

// grid for the fixed-channel-chunk kernels: ~2048 blocks of 256 threads, multiple of K8 threads
static unsigned grid_rows(int64_t M, int64_t K8) {
  int64_t want = std::min<int64_t>(cdiv(M * K8, 256), 2048);
  return (unsigned)std::max<int64_t>(want, cdiv(K8, 256));
}


}  // namespace mx

using namespace mx;

extern "C" int mx_bn_finalize(const float* stats, int64_t mb, int64_t K, int64_t count, const float* gamma,
                              const float* beta, float eps, float momentum, float* rm, float* rv, float* mean,
                              float* invstd, float* scale, float* shift, mx_stream_t stream) {
  MX_CHECK_ARG(mb > 0 && K > 0 && count > 0, "bn_finalize: bad sizes");
  MX_CHECK_ARG((rm == nullptr) == (rv == nullptr), "bn_finalize: running mean/var must both be given or both null");
  bn_finalize_kernel<<<(unsigned)cdiv(K, 16), 256, 0, (hipStream_t)stream>>>(stats, mb, K, count, gamma, beta, eps, momentum,
                                                                              rm, rv, mean, invstd, scale, shift);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_bn_apply(const void* x, int xdtype, int64_t M, int64_t K, const float* scale, const float* shift,
                           const uint16_t* residual, int act, uint16_t* y, mx_stream_t stream) {
  MX_CHECK_ARG(K % 8 == 0, "bn_apply: K %% 8 != 0");
  if (M == 0) return MX_OK;
  if (xdtype == MX_BF16)
    bn_apply_kernel<uint16_t><<<grid_rows(M, K / 8), 256, 0, (hipStream_t)stream>>>((const uint16_t*)x, M, K, scale, shift,
                                                                                     residual, act, y);
  else
    bn_apply_kernel<float><<<grid_rows(M, K / 8), 256, 0, (hipStream_t)stream>>>((const float*)x, M, K, scale, shift,
                                                                                  residual, act, y);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_bn_bwd_reduce(const uint16_t* dy, const uint16_t* y, const uint16_t* x, int64_t M, int64_t K, int act,
                                const float* mean, const float* invstd, float* sums, mx_stream_t stream) {
  MX_CHECK_ARG(K % 8 == 0 && K <= 4096, "bn_bwd_reduce: K must be a multiple of 8 and <= 4096");
  if (M == 0) return MX_OK;
  int64_t rpb = std::max<int64_t>(64, cdiv(M, 1024));
  unsigned blocks = (unsigned)cdiv(M, rpb);
  bn_bwd_reduce_kernel<<<blocks, 256, sizeof(float) * 2 * K, (hipStream_t)stream>>>(dy, y, x, M, K, act, mean, invstd, rpb,
                                                                                    sums);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_bn_bwd_apply(const uint16_t* dy, const uint16_t* y, const uint16_t* x, int64_t M, int64_t K, int act,
                               const float* mean, const float* invstd, const float* gamma, const float* sums,
                               uint16_t* dx, uint16_t* dres, mx_stream_t stream) {
  MX_CHECK_ARG(K % 8 == 0, "bn_bwd_apply: K %% 8 != 0");
  if (M == 0) return MX_OK;
  bn_bwd_apply_kernel<<<grid_rows(M, K / 8), 256, 0, (hipStream_t)stream>>>(dy, y, x, M, K, act, mean, invstd, gamma, sums,
                                                                           dx, dres);
  MX_LAUNCH_CHECK();
  return MX_OK;
}
