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

// Column sums of partials[2][R][K] f32 in f64: block = CPB (4) channels x 64 row-slices, 2
// independent accumulator pairs per thread (loads in flight), LDS tree over the slices. Result in
// ps/pq[0][cl].
static constexpr int CPB = 4, SLICES = 64;
__device__ __forceinline__ void col_sums(const float* __restrict__ part, int64_t R, int64_t K, int64_t k, int cl, int sl,
                                         double (*ps)[CPB + 1], double (*pq)[CPB + 1]) {
  double s0 = 0.0, s1 = 0.0, q0 = 0.0, q1 = 0.0;
  if (k < K) {
    int64_t b = sl;
    for (; b + SLICES < R; b += 2 * SLICES) {
      s0 += (double)part[b * K + k];
      q0 += (double)part[(R + b) * K + k];
      s1 += (double)part[(b + SLICES) * K + k];
      q1 += (double)part[(R + b + SLICES) * K + k];
    }
    if (b < R) {
      s0 += (double)part[b * K + k];
      q0 += (double)part[(R + b) * K + k];
    }
  }
  ps[sl][cl] = s0 + s1;
  pq[sl][cl] = q0 + q1;
  __syncthreads();
  for (int w = SLICES / 2; w > 0; w >>= 1) {
    if (sl < w) {
      ps[sl][cl] += ps[sl + w][cl];
      pq[sl][cl] += pq[sl + w][cl];
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256) bn_finalize_kernel(const float* __restrict__ stats, int64_t mb, int64_t K, int64_t count,
                                   const float* __restrict__ gamma, const float* __restrict__ beta, float eps, float mom,
                                   float* __restrict__ rmean, float* __restrict__ rvar, float* __restrict__ mean_o,
                                   float* __restrict__ invstd_o, float* __restrict__ scale_o, float* __restrict__ shift_o) {
  __shared__ double ps[SLICES][CPB + 1], pq[SLICES][CPB + 1];
  const int cl = threadIdx.x % CPB, sl = threadIdx.x / CPB;
  const int64_t k = (int64_t)blockIdx.x * CPB + cl;
  col_sums(stats, mb, K, k, cl, sl, ps, pq);
  if (sl == 0 && k < K) {
    const double s = ps[0][cl], q = pq[0][cl];
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

// ---- backward --------------------------------------------------------------------------------
// g = dy * act'(y), xhat = (x - mean) * invstd. Pass 1 (bwd_partials): per row-block column sums of g
// and g*xhat -> part[2][RB][K] (no atomics). Pass 2 (bwd_coef): f64 column sums -> sums[2][K]
// (= dbeta, dgamma) and the per-channel affine form of the backward, dx = A*g + B*x + C.
// Pass 3 (bwd_apply): dx (and dres = g) in one streaming pass.
template <int ACT>
__device__ __forceinline__ float act_grad(float y) {
  if (ACT == 1) return y > 0.f ? 1.f : 0.f;
  if (ACT == 2) return y > 0.f ? 1.f : 0.2f;
  return 1.f;
}

// block = CL channel-chunk lanes x (256/CL) row lanes over a row range; grid (RB, K8/CL)
template <int ACT>
__global__ void __launch_bounds__(256) bn_bwd_partials_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ y,
                                                              const uint16_t* __restrict__ x, int64_t M, int64_t K, int CL,
                                                              int64_t rows_per_block, const float* __restrict__ mean,
                                                              const float* __restrict__ invstd, float* __restrict__ part) {
  extern __shared__ float red[];  // [2][256/CL][CL*8]
  const int RL = 256 / CL;
  const int cl = threadIdx.x % CL, rl = threadIdx.x / CL;
  const int64_t c0 = ((int64_t)blockIdx.y * CL + cl) * 8;
  const bool cok = c0 < K;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (cok) {
    float mu[8], is[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) { mu[t] = mean[c0 + t]; is[t] = invstd[c0 + t]; }
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = min<int64_t>(M, r0 + rows_per_block);
    for (int64_t r = r0 + rl; r < r1; r += RL) {
      const uint4 ud = *(const uint4*)(dy + r * K + c0);
      const uint4 ux = *(const uint4*)(x + r * K + c0);
      uint4 uy = make_uint4(0, 0, 0, 0);
      if (ACT) uy = *(const uint4*)(y + r * K + c0);
      const uint16_t *hd = (const uint16_t*)&ud, *hy = (const uint16_t*)&uy, *hx = (const uint16_t*)&ux;
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const float g = bf2f(hd[t]) * act_grad<ACT>(bf2f(hy[t]));
        const float xh = (bf2f(hx[t]) - mu[t]) * is[t];
        s[t] += g;
        q[t] += g * xh;
      }
    }
  }
  const int W = CL * 8;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    red[rl * W + cl * 8 + t] = s[t];
    red[(RL + rl) * W + cl * 8 + t] = q[t];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 2 * W; e += 256) {
    const int which = e / W, col = e - which * W;
    float a = 0.f;
    for (int r = 0; r < RL; ++r) a += red[(which * RL + r) * W + col];
    const int64_t k = (int64_t)blockIdx.y * W + col;
    if (k < K) part[((int64_t)which * gridDim.x + blockIdx.x) * K + k] = a;
  }
}

__global__ void __launch_bounds__(256) bn_bwd_coef_kernel(const float* __restrict__ part, int64_t RB, int64_t K, int64_t M,
                                                          const float* __restrict__ mean, const float* __restrict__ invstd,
                                                          const float* __restrict__ gamma, float* __restrict__ sums,
                                                          float* __restrict__ coef) {
  __shared__ double ps[SLICES][CPB + 1], pq[SLICES][CPB + 1];
  const int cl = threadIdx.x % CPB, sl = threadIdx.x / CPB;
  const int64_t k = (int64_t)blockIdx.x * CPB + cl;
  col_sums(part, RB, K, k, cl, sl, ps, pq);
  if (sl == 0 && k < K) {
    const double sg = ps[0][cl], sgx = pq[0][cl];
    sums[k] = (float)sg;
    sums[K + k] = (float)sgx;
    // dx = a*g + b*x + c,  a = gamma*invstd, b = -a*invstd*mean(g*xhat),
    // c = -a*(mean(g) - mean*invstd*mean(g*xhat))
    const float is = invstd[k], a = (gamma ? gamma[k] : 1.f) * is;
    const float mg = (float)(sg / (double)M), mgx = (float)(sgx / (double)M);
    coef[k] = a;
    coef[K + k] = -a * is * mgx;
    coef[2 * K + k] = -a * (mg - mean[k] * is * mgx);
  }
}

// one 8-channel chunk of one row per thread
template <int ACT>
__global__ void __launch_bounds__(256) bn_bwd_apply2_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ y,
                                                            const uint16_t* __restrict__ x, int64_t n8, int K8,
                                                            const float* __restrict__ coef, uint16_t* __restrict__ dx,
                                                            uint16_t* __restrict__ dres) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n8) return;
  const int K = K8 * 8;
  const int c0 = (int)(e % K8) * 8;
  const uint4 ud = *(const uint4*)(dy + e * 8), ux = *(const uint4*)(x + e * 8);
  uint4 uy = make_uint4(0, 0, 0, 0);
  if (ACT) uy = *(const uint4*)(y + e * 8);
  const float4 a0 = *(const float4*)(coef + c0), a1 = *(const float4*)(coef + c0 + 4);
  const float4 b0 = *(const float4*)(coef + K + c0), b1 = *(const float4*)(coef + K + c0 + 4);
  const float4 d0 = *(const float4*)(coef + 2 * K + c0), d1 = *(const float4*)(coef + 2 * K + c0 + 4);
  const float A[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
  const float B[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
  const float C[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
  const uint16_t *hd = (const uint16_t*)&ud, *hy = (const uint16_t*)&uy, *hx = (const uint16_t*)&ux;
  uint4 o, orr;
  uint16_t* oh = (uint16_t*)&o;
  uint16_t* orh = (uint16_t*)&orr;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float g = bf2f(hd[q]) * act_grad<ACT>(bf2f(hy[q]));
    oh[q] = f2bf(A[q] * g + B[q] * bf2f(hx[q]) + C[q]);
    orh[q] = f2bf(g);
  }
  *(uint4*)(dx + e * 8) = o;
  if (dres) *(uint4*)(dres + e * 8) = orr;
}

// sums -> coef for the legacy mx_bn_bwd_apply entry
__global__ void bn_coef_from_sums_kernel(const float* __restrict__ sums, int64_t K, int64_t M, const float* __restrict__ mean,
                                         const float* __restrict__ invstd, const float* __restrict__ gamma,
                                         float* __restrict__ coef) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  const float is = invstd[k], a = (gamma ? gamma[k] : 1.f) * is;
  const float invM = 1.0f / (float)M;
  const float mg = sums[k] * invM, mgx = sums[K + k] * invM;
  coef[k] = a;
  coef[K + k] = -a * is * mgx;
  coef[2 * K + k] = -a * (mg - mean[k] * is * mgx);
}

// grid for the fixed-channel-chunk kernels: ~2048 blocks of 256 threads, multiple of K8 threads
static unsigned grid_rows(int64_t M, int64_t K8) {
  int64_t want = std::min<int64_t>(cdiv(M * K8, 256), 2048);
  return (unsigned)std::max<int64_t>(want, cdiv(K8, 256));
}

struct BwdGeo {
  int CL;
  int64_t RB, rows_per_block, gy;
};
static BwdGeo bwd_geo(int64_t M, int64_t K) {
  BwdGeo g;
  const int64_t K8 = K / 8;
  g.CL = (int)std::min<int64_t>(K8, 64);
  while (256 % g.CL) --g.CL;  // CL divides the block
  const int64_t RL = 256 / g.CL;
  g.gy = cdiv(K8, g.CL);
  // enough row blocks to fill the chip, >= 16 rows per thread, <= 512 partial rows for the reduce
  const int64_t rb_max = std::max<int64_t>(1, std::min<int64_t>(2048 / g.gy, 512));
  g.RB = std::max<int64_t>(1, std::min(cdiv(M, RL * 16), rb_max));
  g.rows_per_block = cdiv(M, g.RB);
  g.RB = cdiv(M, g.rows_per_block);
  return g;
}

}  // namespace mx

using namespace mx;

extern "C" int mx_bn_finalize(const float* stats, int64_t mb, int64_t K, int64_t count, const float* gamma,
                              const float* beta, float eps, float momentum, float* rm, float* rv, float* mean,
                              float* invstd, float* scale, float* shift, mx_stream_t stream) {
  MX_CHECK_ARG(mb > 0 && K > 0 && count > 0, "bn_finalize: bad sizes");
  MX_CHECK_ARG((rm == nullptr) == (rv == nullptr), "bn_finalize: running mean/var must both be given or both null");
  bn_finalize_kernel<<<(unsigned)cdiv(K, CPB), 256, 0, (hipStream_t)stream>>>(stats, mb, K, count, gamma, beta, eps, momentum,
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

extern "C" size_t mx_bn_bwd_workspace(int64_t M, int64_t K) {
  if (M <= 0 || K <= 0 || K % 8) return 0;
  BwdGeo g = bwd_geo(M, K);
  return sizeof(float) * 2 * (size_t)g.RB * K;
}

template <int ACT>
static void launch_partials(const uint16_t* dy, const uint16_t* y, const uint16_t* x, int64_t M, int64_t K,
                            const BwdGeo& g, const float* mean, const float* invstd, float* part, hipStream_t st) {
  dim3 grid((unsigned)g.RB, (unsigned)g.gy);
  bn_bwd_partials_kernel<ACT><<<grid, 256, sizeof(float) * 2 * 256 * 8, st>>>(dy, y, x, M, K, g.CL, g.rows_per_block,
                                                                               mean, invstd, part);
}

extern "C" int mx_bn_bwd_reduce_ex(const uint16_t* dy, const uint16_t* y, const uint16_t* x, int64_t M, int64_t K, int act,
                                   const float* mean, const float* invstd, const float* gamma, void* ws, size_t ws_bytes,
                                   float* sums, float* coef, mx_stream_t stream) {
  MX_CHECK_ARG(K % 8 == 0 && K > 0 && M > 0, "bn_bwd_reduce: K must be a positive multiple of 8, M > 0");
  MX_CHECK_ARG(act >= 0 && act <= 2, "bn_bwd_reduce: act 0/1/2");
  MX_CHECK_ARG(act == 0 || y, "bn_bwd_reduce: y required for an activation");
  BwdGeo g = bwd_geo(M, K);
  const size_t need = sizeof(float) * 2 * (size_t)g.RB * K;
  MX_CHECK_ARG(ws && ws_bytes >= need, "bn_bwd_reduce: workspace of %zu bytes required (mx_bn_bwd_workspace)", need);
  MX_CHECK_ARG(g.RB < 65536 && g.gy < 65536, "bn_bwd_reduce: grid too large");
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)ws;
  if (act == 1) launch_partials<1>(dy, y, x, M, K, g, mean, invstd, part, st);
  else if (act == 2) launch_partials<2>(dy, y, x, M, K, g, mean, invstd, part, st);
  else launch_partials<0>(dy, y, x, M, K, g, mean, invstd, part, st);
  MX_LAUNCH_CHECK();
  bn_bwd_coef_kernel<<<(unsigned)cdiv(K, CPB), 256, 0, st>>>(part, g.RB, K, M, mean, invstd, gamma, sums, coef);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_bn_bwd_apply_ex(const uint16_t* dy, const uint16_t* y, const uint16_t* x, int64_t M, int64_t K, int act,
                                  const float* coef, uint16_t* dx, uint16_t* dres, mx_stream_t stream) {
  MX_CHECK_ARG(K % 8 == 0 && K > 0 && K < (1 << 24), "bn_bwd_apply: K must be a positive multiple of 8");
  MX_CHECK_ARG(act >= 0 && act <= 2, "bn_bwd_apply: act 0/1/2");
  MX_CHECK_ARG(act == 0 || y, "bn_bwd_apply: y required for an activation");
  if (M == 0) return MX_OK;
  const int64_t n8 = M * (K / 8);
  const unsigned blocks = (unsigned)cdiv(n8, 256);
  hipStream_t st = (hipStream_t)stream;
  if (act == 1) bn_bwd_apply2_kernel<1><<<blocks, 256, 0, st>>>(dy, y, x, n8, (int)(K / 8), coef, dx, dres);
  else if (act == 2) bn_bwd_apply2_kernel<2><<<blocks, 256, 0, st>>>(dy, y, x, n8, (int)(K / 8), coef, dx, dres);
  else bn_bwd_apply2_kernel<0><<<blocks, 256, 0, st>>>(dy, y, x, n8, (int)(K / 8), coef, dx, dres);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

// Convenience forms (temporaries allocated per call): sums[2][K] is overwritten with (sum g, sum g*xhat).
extern "C" int mx_bn_bwd_reduce(const uint16_t* dy, const uint16_t* y, const uint16_t* x, int64_t M, int64_t K, int act,
                                const float* mean, const float* invstd, float* sums, mx_stream_t stream) {
  MX_CHECK_ARG(K % 8 == 0 && K > 0, "bn_bwd_reduce: K must be a positive multiple of 8");
  if (M == 0) return MX_OK;
  hipStream_t st = (hipStream_t)stream;
  const size_t wsb = mx_bn_bwd_workspace(M, K);
  void* ws = nullptr;
  float* coef = nullptr;
  MX_HIP(hipMallocAsync(&ws, wsb, st));
  MX_HIP(hipMallocAsync((void**)&coef, sizeof(float) * 3 * K, st));
  int rc = mx_bn_bwd_reduce_ex(dy, y, x, M, K, act, mean, invstd, nullptr, ws, wsb, sums, coef, stream);
  MX_HIP(hipFreeAsync(ws, st));
  MX_HIP(hipFreeAsync(coef, st));
  return rc;
}

extern "C" int mx_bn_bwd_apply(const uint16_t* dy, const uint16_t* y, const uint16_t* x, int64_t M, int64_t K, int act,
                               const float* mean, const float* invstd, const float* gamma, const float* sums,
                               uint16_t* dx, uint16_t* dres, mx_stream_t stream) {
  MX_CHECK_ARG(K % 8 == 0 && K > 0, "bn_bwd_apply: K %% 8 != 0");
  if (M == 0) return MX_OK;
  hipStream_t st = (hipStream_t)stream;
  float* coef = nullptr;
  MX_HIP(hipMallocAsync((void**)&coef, sizeof(float) * 3 * K, st));
  bn_coef_from_sums_kernel<<<(unsigned)cdiv(K, 256), 256, 0, st>>>(sums, K, M, mean, invstd, gamma, coef);
  int rc = MX_OK;
  if (hipGetLastError() != hipSuccess) rc = MX_EHIP;
  if (!rc) rc = mx_bn_bwd_apply_ex(dy, y, x, M, K, act, coef, dx, dres, stream);
  MX_HIP(hipFreeAsync(coef, st));
  return rc;
}
