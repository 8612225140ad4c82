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

// ---- one-launch column reductions ----------------------------------------------------------
// Every block writes its partial column sums to the workspace; the last block to arrive for a
// channel chunk sums the partials in a fixed order and finishes. Hand-off without L2 write-back
// fences (MI355X_MICROARCH.md, inter-workgroup visibility, valid form "ONE lane of each storing
// workgroup ... the workgroup whose add came last"): partials are stored sc1 (relaxed agent-scope
// atomic stores, write-through), every wave drains vmcnt before the block barrier, one lane adds to
// the chunk's counter, and the last block reads the partials with sc1 loads. The last block resets
// its counter, so a workspace zero-filled once stays valid for every later launch on one stream.
static constexpr int CTR_BYTES = 256, MAX_CHUNKS = CTR_BYTES / 4;

template <typename T>
__device__ __forceinline__ void st_sc1(T* p, T v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <typename T>
__device__ __forceinline__ T ld_sc1(const T* p) { return __hip_atomic_load((T*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

__device__ __forceinline__ bool arrive_last(unsigned* ctr, unsigned nblocks) {
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 partial stores have landed
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = prev == nblocks - 1;
    if (last) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return last;
}

// Last-block column sums: out[w][col] = sum_{b < R} part[(w * R + b) * K + k0 + col] in f64, for
// NW x 64 outputs, by all 256 threads (256 / (64 NW) threads per output, 8 sc1 loads in flight per
// thread, combined in a fixed order: deterministic).
template <int NW, typename T>
__device__ __forceinline__ void last_sums(const T* __restrict__ part, int64_t R, int64_t K, int64_t k0, double (*out)[64],
                                          double* scratch /* [256] */) {
  constexpr int TPO = 256 / (64 * NW);  // threads per output
  const int o = threadIdx.x % (64 * NW), j = threadIdx.x / (64 * NW);
  const int w = o / 64, col = o % 64;
  const int64_t k = k0 + col;
  double a = 0.0;
  if (k < K) {
    const T* p = part + (int64_t)w * R * K + k;
    int64_t b = j;
    for (; b + 7 * TPO < R; b += 8 * TPO) {
      T v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = ld_sc1(p + (b + u * TPO) * K);
#pragma unroll
      for (int u = 0; u < 8; ++u) a += (double)v[u];
    }
    for (; b < R; b += TPO) a += (double)ld_sc1(p + b * K);
  }
  scratch[threadIdx.x] = a;
  __syncthreads();
  if (threadIdx.x < 64 * NW) {
    double t = 0.0;
#pragma unroll
    for (int q = 0; q < TPO; ++q) t += scratch[q * 64 * NW + threadIdx.x];
    out[w][col] = t;
  }
  __syncthreads();
}

// finalize: grid (channel chunks of 64, RS row slices); block = 64 channels x 4 row lanes (one wave
// per row: 256-B coalesced reads of the [2][mb][K] conv-epilogue partials), f64 accumulation.
__global__ void __launch_bounds__(256) bn_finalize_kernel(const float* __restrict__ stats, int64_t mb, int64_t K, int64_t count,
                                   const float* __restrict__ gamma, const float* __restrict__ beta, float eps, float mom,
                                   float* __restrict__ rmean, float* __restrict__ rvar, float* __restrict__ mean_o,
                                   float* __restrict__ invstd_o, float* __restrict__ scale_o, float* __restrict__ shift_o,
                                   unsigned* __restrict__ ctr, double* __restrict__ part) {
  __shared__ double red[2][4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int64_t k = (int64_t)blockIdx.x * 64 + cl;
  const int64_t RS = gridDim.y, per = (mb + RS - 1) / RS;
  const int64_t r0 = (int64_t)blockIdx.y * per, r1 = min<int64_t>(mb, r0 + per);
  double s0 = 0.0, s1 = 0.0, q0 = 0.0, q1 = 0.0;
  if (k < K) {
    int64_t r = r0 + rl;
    for (; r + 4 < r1; r += 8) {
      s0 += (double)stats[r * K + k];
      q0 += (double)stats[(mb + r) * K + k];
      s1 += (double)stats[(r + 4) * K + k];
      q1 += (double)stats[(mb + r + 4) * K + k];
    }
    if (r < r1) {
      s0 += (double)stats[r * K + k];
      q0 += (double)stats[(mb + r) * K + k];
    }
  }
  red[0][rl][cl] = s0 + s1;
  red[1][rl][cl] = q0 + q1;
  __syncthreads();
  if (rl < 2 && k < K) {
    const double v = (red[rl][0][cl] + red[rl][1][cl]) + (red[rl][2][cl] + red[rl][3][cl]);
    st_sc1(part + ((int64_t)rl * RS + blockIdx.y) * K + k, v);
  }
  if (!arrive_last(ctr + blockIdx.x, (unsigned)RS)) return;
  __shared__ double fin[2][64], scr[256];
  last_sums<2>(part, RS, K, (int64_t)blockIdx.x * 64, fin, scr);
  if (rl == 0 && k < K) {
    const double s = fin[0][cl], q = fin[1][cl];
    const double mean = s / (double)count;
    double var = q / (double)count - mean * mean;
    if (var < 0.0) var = 0.0;
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    const float g = gamma ? gamma[k] : 1.f, bb = beta ? beta[k] : 0.f;
    mean_o[k] = (float)mean;
    invstd_o[k] = invstd;
    scale_o[k] = g * invstd;
    shift_o[k] = bb - (float)mean * (g * invstd);
    if (rmean) {
      const double unb = count > 1 ? var * (double)count / (double)(count - 1) : var;
      rmean[k] = (float)((1.0 - mom) * rmean[k] + mom * mean);
      rvar[k] = (float)((1.0 - mom) * rvar[k] + mom * unb);
    }
  }
}

// BN backward from column partials produced elsewhere (the dgrad epilogue, mx_conv2d_dgrad_bnb):
// part [2][mb][K] = per 64-row block sums of g and g*xhat -> sums (dbeta, dgamma) and the affine
// coefficients of dx = a*g + b*x + c, exactly as bn_bwd_reduce_kernel's last block (f64 finish).
__global__ void __launch_bounds__(256) bn_bwd_finalize_kernel(const float* __restrict__ stats, int64_t mb, int64_t K,
                                                              int64_t M, const float* __restrict__ mean,
                                                              const float* __restrict__ invstd,
                                                              const float* __restrict__ gamma, float* __restrict__ sums,
                                                              float* __restrict__ coef, unsigned* __restrict__ ctr,
                                                              double* __restrict__ part) {
  __shared__ double red[2][4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int64_t k = (int64_t)blockIdx.x * 64 + cl;
  const int64_t RS = gridDim.y, per = (mb + RS - 1) / RS;
  const int64_t r0 = (int64_t)blockIdx.y * per, r1 = min<int64_t>(mb, r0 + per);
  double s0 = 0.0, s1 = 0.0, q0 = 0.0, q1 = 0.0;
  if (k < K) {
    int64_t r = r0 + rl;
    for (; r + 4 < r1; r += 8) {
      s0 += (double)stats[r * K + k];
      q0 += (double)stats[(mb + r) * K + k];
      s1 += (double)stats[(r + 4) * K + k];
      q1 += (double)stats[(mb + r + 4) * K + k];
    }
    if (r < r1) {
      s0 += (double)stats[r * K + k];
      q0 += (double)stats[(mb + r) * K + k];
    }
  }
  red[0][rl][cl] = s0 + s1;
  red[1][rl][cl] = q0 + q1;
  __syncthreads();
  if (rl < 2 && k < K) {
    const double v = (red[rl][0][cl] + red[rl][1][cl]) + (red[rl][2][cl] + red[rl][3][cl]);
    st_sc1(part + ((int64_t)rl * RS + blockIdx.y) * K + k, v);
  }
  if (!arrive_last(ctr + blockIdx.x, (unsigned)RS)) return;
  __shared__ double fin[2][64], scr[256];
  last_sums<2>(part, RS, K, (int64_t)blockIdx.x * 64, fin, scr);
  if (rl == 0 && k < K) {
    const double sg = fin[0][cl], sgx = fin[1][cl];
    sums[k] = (float)sg;
    sums[K + k] = (float)sgx;
    const float is = invstd[k], a = (gamma ? gamma[k] : 1.f) * is;
    const float mg = (float)(sg / (double)M), mgx = (float)(sgx / (double)M);
    coef[k] = a;
    coef[K + k] = -a * is * mgx;
    coef[2 * K + k] = -a * (mg - mean[k] * is * mgx);
  }
}

// 8 f32 values (element chunk e of an n-element tensor) -> their split8 hi / lo at planes[e*8] / planes[n + e*8]
__device__ __forceinline__ void store_planes8(uint16_t* __restrict__ planes, int64_t n, int64_t e, const float (&o)[8]) {
  uint4 h, l;
  split8(make_float4(o[0], o[1], o[2], o[3]), make_float4(o[4], o[5], o[6], o[7]), h, l);
  *(uint4*)(planes + e * 8) = h;
  *(uint4*)(planes + n + e * 8) = l;
}

// Thread t owns channel chunk c8 = t % K8 for its whole life (per-channel constants stay in
// registers) and walks rows r = t / K8 + i * (T / K8): 16-B vector loads/stores, coalesced per row.
// planes (f32 only, nullable): y also as its bf16x3 planes [2][M][K] (split8: mx_split_planes' values) for
// a consumer conv that reads pre-split operands -- one 4-B write per element instead of a split pass
template <typename T, typename TY>
__global__ void __launch_bounds__(256) bn_apply_kernel(const T* __restrict__ x, int64_t M, int64_t K, const float* __restrict__ scale,
                                const float* __restrict__ shift, const TY* __restrict__ res, int act,
                                TY* __restrict__ y, uint16_t* __restrict__ planes = nullptr) {
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
    ld8(x + e * 8, v);
    float rv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (res) ld8(res + e * 8, rv);
    float o[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = actf(v[q] * sc[q] + sh[q] + rv[q], act);
    st8(y + e * 8, o);
    if (planes) store_planes8(planes, M * K, e, o);
  }
}

// ---- backward --------------------------------------------------------------------------------
// g = dy * act'(y), xhat = (x - mean) * invstd. Launch 1 (bwd_reduce): per row-block column sums of g
// and g*xhat -> part[2][RB][K] (no float atomics), then in the last block per channel chunk the f64
// column sums -> sums[2][K] (= dbeta, dgamma) and the per-channel affine form of the backward,
// dx = A*g + B*x + C. Launch 2 (bwd_apply): dx (and dres = g) in one streaming pass.
template <int ACT>
__device__ __forceinline__ float act_grad(float y) {
  if (ACT == 1) return y > 0.f ? 1.f : 0.f;
  if (ACT == 2) return y > 0.f ? 1.f : 0.2f;
  return 1.f;
}

// block = 64 channels (8 chunk lanes x 8 channels) x 32 row lanes over a row range; grid (RB, gy).
// f32 per-thread sums over the block's rows, f32 partial per block, f64 across blocks in the last
// block of the channel chunk, which also writes sums[2][K] and the affine coefficients.
template <int ACT, typename T>
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(const T* __restrict__ dy, const T* __restrict__ y,
                                                            const T* __restrict__ x, int64_t M, int64_t K,
                                                            int64_t rows_per_block, const float* __restrict__ mean,
                                                            const float* __restrict__ invstd, const float* __restrict__ gamma,
                                                            unsigned* __restrict__ ctr, float* __restrict__ part,
                                                            float* __restrict__ sums, float* __restrict__ coef) {
  __shared__ float red[2][32][65];
  __shared__ double fin[2][64];
  const int cl = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int64_t c0 = (int64_t)blockIdx.y * 64 + cl * 8;
  const bool cok = c0 < K;
  const int64_t RB = gridDim.x;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (cok) {
    float mu[8], is[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) { mu[t] = mean[c0 + t]; is[t] = invstd[c0 + t]; }
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = min<int64_t>(M, r0 + rows_per_block);
    // U rows per thread per step: all 3*U 16-B loads issued before the arithmetic (one row per
    // step would leave a single load set in flight per thread); per-row summation order unchanged
    constexpr int U = 4;
    for (int64_t rb = r0 + rl; rb < r1; rb += 32 * U) {
      float vd[U][8], vx[U][8], vy[U][8];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t r = rb + 32 * u;
#pragma unroll
        for (int t = 0; t < 8; ++t) vd[u][t] = vx[u][t] = vy[u][t] = 0.f;
        if (r < r1) {
          ld8(dy + r * K + c0, vd[u]);
          ld8(x + r * K + c0, vx[u]);
          if (ACT) ld8(y + r * K + c0, vy[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (rb + 32 * u >= r1) break;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const float g = vd[u][t] * act_grad<ACT>(vy[u][t]);
          const float xh = (vx[u][t] - mu[t]) * is[t];
          s[t] += g;
          q[t] += g * xh;
        }
      }
    }
  }
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    red[0][rl][cl * 8 + t] = s[t];
    red[1][rl][cl * 8 + t] = q[t];
  }
  __syncthreads();
  const int which = threadIdx.x >> 6, col = threadIdx.x & 63;
  const int64_t k = (int64_t)blockIdx.y * 64 + col;
  if (which < 2) {
    float a = 0.f;
#pragma unroll 8
    for (int r = 0; r < 32; ++r) a += red[which][r][col];
    if (k < K) st_sc1(part + ((int64_t)which * RB + blockIdx.x) * K + k, a);
  }
  if (!arrive_last(ctr + blockIdx.y, (unsigned)RB)) return;
  __shared__ double scr[256];
  last_sums<2>((const float*)part, RB, K, (int64_t)blockIdx.y * 64, fin, scr);
  if (which == 0 && k < K) {
    const double sg = fin[0][col], sgx = fin[1][col];
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

// ---- conv (+bias) (+act) backward head -------------------------------------------------------
// g = gy * act'(y) rounded to bf16 into [M][K8] (columns K..K8 zero: the dgrad/wgrad operands of
// the narrow RPN / predictor heads are padded to 8), and db = column sums of the unrounded g
// (torch: bias grad = grad_out.sum over N,H,W). Block = 64 columns (8 lanes x 8) x 32 row lanes;
// grid (RB, cdiv(K8, 64)); the last block per column chunk sums the RB partials (f64) into db.
template <typename T, int ACT, typename TG>
__global__ void __launch_bounds__(256) act_bias_bwd_kernel(const T* __restrict__ gy, const T* __restrict__ y, int64_t M,
                                                           int K, int K8, int64_t rows_per_block, TG* __restrict__ g,
                                                           float* __restrict__ db, unsigned* __restrict__ ctr,
                                                           float* __restrict__ part, uint16_t* __restrict__ planes) {
  __shared__ float red[32][65];
  const int cl = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c0 = blockIdx.y * 64 + cl * 8;
  const int64_t RB = gridDim.x;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c0 < K8) {
    const bool vec = (K % 8) == 0;
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = min<int64_t>(M, r0 + rows_per_block);
    for (int64_t r = r0 + rl; r < r1; r += 32) {
      float v[8];
      if (vec) {
        float vg[8], vy[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        ld8(gy + r * K + c0, vg);
        if (ACT) ld8(y + r * K + c0, vy);
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] = vg[t] * act_grad<ACT>(vy[t]);
      } else {
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const int c = c0 + t;
          v[t] = c < K ? io<T>::ld(gy + r * K + c) * (ACT ? act_grad<ACT>(io<T>::ld(y + r * K + c)) : 1.f) : 0.f;
        }
      }
#pragma unroll
      for (int t = 0; t < 8; ++t) s[t] += v[t];
      st8(g + r * K8 + c0, v);
      if (planes) store_planes8(planes, M * (int64_t)K8, (r * K8 + c0) >> 3, v);  // f32 g's bf16x3 planes
    }
  }
  if (!db) return;
#pragma unroll
  for (int t = 0; t < 8; ++t) red[rl][cl * 8 + t] = s[t];
  __syncthreads();
  const int col = threadIdx.x & 63;
  const int k = blockIdx.y * 64 + col;
  if (threadIdx.x < 64) {
    float a = 0.f;
#pragma unroll 8
    for (int r = 0; r < 32; ++r) a += red[r][col];
    if (k < K) st_sc1(part + (int64_t)blockIdx.x * K + k, a);
  }
  if (!arrive_last(ctr + blockIdx.y, (unsigned)RB)) return;
  __shared__ double fin[1][64], scr[256];
  last_sums<1>((const float*)part, RB, (int64_t)K, (int64_t)blockIdx.y * 64, fin, scr);
  if (threadIdx.x < 64 && k < K) db[k] = (float)fin[0][col];
}

// one 8-channel chunk of one row per thread
template <int ACT, typename T>
__global__ void __launch_bounds__(256) bn_bwd_apply2_kernel(const T* __restrict__ dy, const T* __restrict__ y,
                                                            const T* __restrict__ x, int64_t n8, int K8,
                                                            const float* __restrict__ coef, T* __restrict__ dx,
                                                            T* __restrict__ dres, uint16_t* __restrict__ planes = nullptr) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n8) return;
  const int K = K8 * 8;
  const int c0 = (int)(e % K8) * 8;
  float vd[8], vx[8], vy[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  ld8(dy + e * 8, vd);
  ld8(x + e * 8, vx);
  if (ACT) ld8(y + e * 8, vy);
  const float4 a0 = *(const float4*)(coef + c0), a1 = *(const float4*)(coef + c0 + 4);
  const float4 b0 = *(const float4*)(coef + K + c0), b1 = *(const float4*)(coef + K + c0 + 4);
  const float4 d0 = *(const float4*)(coef + 2 * K + c0), d1 = *(const float4*)(coef + 2 * K + c0 + 4);
  const float A[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
  const float B[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
  const float C[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
  float o[8], og[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    og[q] = vd[q] * act_grad<ACT>(vy[q]);
    o[q] = A[q] * og[q] + B[q] * vx[q] + C[q];
  }
  st8(dx + e * 8, o);
  if (dres) st8(dres + e * 8, og);
  if (planes) store_planes8(planes, n8 * 8, e, o);  // dx as bf16x3 planes too (bn_apply_kernel)
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
  int64_t RB, rows_per_block, gy;
};
static BwdGeo bwd_geo(int64_t M, int64_t K) {
  BwdGeo g;
  g.gy = cdiv(K, 64);
  // ~1024 blocks, >= 64 rows per block, <= 128 partial rows for the last block's sum
  g.RB = std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(128, cdiv(M, 64)), std::max<int64_t>(1, 1024 / g.gy)));
  g.rows_per_block = cdiv(M, g.RB);
  g.RB = cdiv(M, g.rows_per_block);
  return g;
}

static int64_t fin_slices(int64_t mb) { return std::max<int64_t>(1, std::min<int64_t>(64, cdiv(mb, 32))); }

// ---- RPN losses (RegionProposalNetwork.compute_loss) -------------------------------------------
// Over all N*A anchors with the sampler's masks: sum_sampled BCE-with-logits(x, y) and
// sum_positive smooth-L1(beta)(d - t) (summed over the 4 coordinates), each / number sampled.
// Per-block f64 partials, last block finishes in a fixed order (deterministic); BCE restated as
// torch's binary_cross_entropy_with_logits: (1 - y) x + m + log(exp(-m) + exp(-x - m)), m = max(-x, 0).
__device__ __forceinline__ float smooth_l1(float u, float beta) {
  const float a = fabsf(u);
  return a < beta ? 0.5f * u * u / beta : a - 0.5f * beta;
}

__global__ void __launch_bounds__(256) rpn_loss_fwd_kernel(const float* __restrict__ x, const float4* __restrict__ d,
                                                           const float* __restrict__ y, const float4* __restrict__ t,
                                                           const uint8_t* __restrict__ pm, const uint8_t* __restrict__ nm,
                                                           int64_t n, float beta, unsigned* __restrict__ ctr,
                                                           double* __restrict__ part, float* __restrict__ out) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const bool p = pm[i], s = p || nm[i];
    if (!s) continue;
    const float xi = x[i], yi = y[i] > 0.f ? 1.f : 0.f;
    const float m = fmaxf(-xi, 0.f);
    a0 += (double)((1.f - yi) * xi + m + logf(expf(-m) + expf(-xi - m)));
    a2 += 1.0;
    if (p) {
      const float4 di = d[i], ti = t[i];
      a1 += (double)(smooth_l1(di.x - ti.x, beta) + smooth_l1(di.y - ti.y, beta) + smooth_l1(di.z - ti.z, beta) +
                     smooth_l1(di.w - ti.w, beta));
    }
  }
  __shared__ double red[3][256];
  red[0][threadIdx.x] = a0;
  red[1][threadIdx.x] = a1;
  red[2][threadIdx.x] = a2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o)
      for (int w = 0; w < 3; ++w) red[w][threadIdx.x] += red[w][threadIdx.x + o];
    __syncthreads();
  }
  const int64_t RB = gridDim.x;
  if (threadIdx.x < 3) st_sc1(part + threadIdx.x * RB + blockIdx.x, red[threadIdx.x][0]);
  if (!arrive_last(ctr, (unsigned)RB)) return;
  __shared__ double fin[3][64], scr[256];
  last_sums<3>(part, RB, 1, 0, fin, scr);
  if (threadIdx.x == 0) {
    const double cnt = fin[2][0];
    out[0] = (float)(fin[0][0] / cnt);  // loss_objectness
    out[1] = (float)(fin[1][0] / cnt);  // loss_rpn_box_reg
    out[2] = (float)cnt;
  }
}

// d loss / d x = (sigmoid(x) - y) / cnt * g0 on sampled anchors; d loss / d d = smooth-L1'(d - t) / cnt
// * g1 on positives; zero elsewhere.
__global__ void __launch_bounds__(256) rpn_loss_bwd_kernel(const float* __restrict__ x, const float4* __restrict__ d,
                                                           const float* __restrict__ y, const float4* __restrict__ t,
                                                           const uint8_t* __restrict__ pm, const uint8_t* __restrict__ nm,
                                                           int64_t n, float beta, const float* __restrict__ stats,
                                                           const float* __restrict__ g0p, const float* __restrict__ g1p,
                                                           float* __restrict__ gx, float4* __restrict__ gd) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float g[2] = {g0p ? *g0p : 0.f, g1p ? *g1p : 0.f};  // upstream grads (null: that loss unused)
  const float inv = 1.f / stats[2];
  const bool p = pm[i], s = p || nm[i];
  float gxi = 0.f;
  float4 gdi = make_float4(0.f, 0.f, 0.f, 0.f);
  if (s) {
    const float xi = x[i], yi = y[i] > 0.f ? 1.f : 0.f;
    gxi = (1.f / (1.f + expf(-xi)) - yi) * inv * g[0];
  }
  if (p) {
    const float4 di = d[i], ti = t[i];
    const float sc = inv * g[1];
    auto dl = [&](float u) { return (fabsf(u) < beta ? u / beta : (u > 0.f ? 1.f : (u < 0.f ? -1.f : 0.f))) * sc; };
    gdi = make_float4(dl(di.x - ti.x), dl(di.y - ti.y), dl(di.z - ti.z), dl(di.w - ti.w));
  }
  gx[i] = gxi;
  gd[i] = gdi;
}

// ---- Fast R-CNN losses (roi_heads.fastrcnn_loss) ---------------------------------------------------
// logits [R][ldl] (first C columns), reg [R][ldr] (4 per class), labels [R] int64, targets [R][4]:
// out[0] = mean cross-entropy, out[1] = sum over positive RoIs of smooth-L1(beta)(reg[r, 4*label:+4]
// - targets[r]) / R. One thread per RoI, fixed-order f64 finish in the last block.
__global__ void __launch_bounds__(256) roi_loss_fwd_kernel(const float* __restrict__ logits, int64_t ldl, int C,
                                                           const float* __restrict__ reg, int64_t ldr,
                                                           const int64_t* __restrict__ labels,
                                                           const float* __restrict__ targets, int64_t R, float beta,
                                                           unsigned* __restrict__ ctr, double* __restrict__ part,
                                                           float* __restrict__ out) {
  double a0 = 0.0, a1 = 0.0;
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r < R) {
    const float* l = logits + r * ldl;
    const int64_t lab = labels[r];
    float mx = l[0];
    for (int c = 1; c < C; ++c) mx = fmaxf(mx, l[c]);
    float se = 0.f;
    for (int c = 0; c < C; ++c) se += expf(l[c] - mx);
    a0 = (double)(logf(se) + mx - l[lab]);
    if (lab > 0) {
      const float* q = reg + r * ldr + 4 * lab;
      const float* tt = targets + r * 4;
      a1 = (double)(smooth_l1(q[0] - tt[0], beta) + smooth_l1(q[1] - tt[1], beta) + smooth_l1(q[2] - tt[2], beta) +
                    smooth_l1(q[3] - tt[3], beta));
    }
  }
  __shared__ double red[2][256];
  red[0][threadIdx.x] = a0;
  red[1][threadIdx.x] = a1;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      red[0][threadIdx.x] += red[0][threadIdx.x + o];
      red[1][threadIdx.x] += red[1][threadIdx.x + o];
    }
    __syncthreads();
  }
  const int64_t RB = gridDim.x;
  if (threadIdx.x < 2) st_sc1(part + threadIdx.x * RB + blockIdx.x, red[threadIdx.x][0]);
  if (!arrive_last(ctr, (unsigned)RB)) return;
  __shared__ double fin[2][64], scr[256];
  last_sums<2>(part, RB, 1, 0, fin, scr);
  if (threadIdx.x == 0) {
    out[0] = (float)(fin[0][0] / (double)R);
    out[1] = (float)(fin[1][0] / (double)R);
  }
}

__global__ void __launch_bounds__(256) roi_loss_bwd_kernel(const float* __restrict__ logits, int64_t ldl, int C,
                                                           const float* __restrict__ reg, int64_t ldr,
                                                           const int64_t* __restrict__ labels,
                                                           const float* __restrict__ targets, int64_t R, float beta,
                                                           const float* __restrict__ g0p, const float* __restrict__ g1p,
                                                           float* __restrict__ gl, float* __restrict__ gr) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= R) return;
  const float g[2] = {g0p ? *g0p : 0.f, g1p ? *g1p : 0.f};  // upstream grads (null: that loss unused)
  const float* l = logits + r * ldl;
  const int64_t lab = labels[r];
  const float s0 = g[0] / (float)R, s1 = g[1] / (float)R;
  float mx = l[0];
  for (int c = 1; c < C; ++c) mx = fmaxf(mx, l[c]);
  float se = 0.f;
  for (int c = 0; c < C; ++c) se += expf(l[c] - mx);
  for (int c = 0; c < C; ++c) gl[r * C + c] = (expf(l[c] - mx) / se - (c == lab ? 1.f : 0.f)) * s0;
  float* q = gr + r * (4 * C);
  for (int j = 0; j < 4 * C; ++j) q[j] = 0.f;
  if (lab > 0) {
    const float* p = reg + r * ldr + 4 * lab;
    const float* tt = targets + r * 4;
    for (int j = 0; j < 4; ++j) {
      const float u = p[j] - tt[j];
      q[4 * lab + j] = (fabsf(u) < beta ? u / beta : (u > 0.f ? 1.f : (u < 0.f ? -1.f : 0.f))) * s1;
    }
  }
}

// BatchNorm apply + activation + max pooling in one pass (the ResNet stem's bn1 -> relu -> maxpool when
// no gradient flows through them): every window element is transformed exactly as bn_apply_kernel
// does (no residual) and reduced exactly as maxpool_fwd_kernel does (first valid element, then
// greater or NaN), so the result is bit-identical to the two kernels -- without writing and
// re-reading the full-resolution activation. One thread per (output pixel, 8 channels).
__global__ void __launch_bounds__(256) bn_act_maxpool_kernel(const float* __restrict__ z, int64_t N, int64_t H,
                                                             int64_t W, int64_t C, int64_t Ho, int64_t Wo, int k,
                                                             int st, int pd, const float* __restrict__ scale,
                                                             const float* __restrict__ shift, int act,
                                                             float* __restrict__ y) {
  const int64_t C8 = C / 8;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N * Ho * Wo * C8) return;
  const int64_t c8 = e % C8, t = e / C8;
  const int64_t ow = t % Wo, oh = (t / Wo) % Ho, n = t / (Wo * Ho);
  float sc[8], sh[8], best[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    sc[q] = scale[c8 * 8 + q];
    sh[q] = shift[c8 * 8 + q];
    best[q] = -INFINITY;
  }
  const float zero = 0.f;
  bool have = false;
  for (int r = 0; r < k; ++r) {
    const int64_t ih = oh * st - pd + r;
    if (ih < 0 || ih >= H) continue;
    for (int s = 0; s < k; ++s) {
      const int64_t iw = ow * st - pd + s;
      if (iw < 0 || iw >= W) continue;
      float vv[8];
      ld8(z + ((n * H + ih) * W + iw) * C + c8 * 8, vv);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float v = actf(vv[q] * sc[q] + sh[q] + zero, act);
        if (v > best[q] || !have || v != v) best[q] = v;
      }
      have = true;
    }
  }
  st8(y + t * C + c8 * 8, best);
}

}  // namespace mx

using namespace mx;

extern "C" size_t mx_bn_finalize_workspace(int64_t mb, int64_t K) {
  if (mb <= 0 || K <= 0) return 0;
  return CTR_BYTES + sizeof(double) * 2 * (size_t)fin_slices(mb) * K;
}

extern "C" int mx_bn_finalize_ex(const float* stats, int64_t mb, int64_t K, int64_t count, const float* gamma,
                                 const float* beta, float eps, float momentum, float* rm, float* rv, float* mean,
                                 float* invstd, float* scale, float* shift, void* ws, size_t ws_bytes, mx_stream_t stream) {
  MX_CHECK_ARG(mb > 0 && K > 0 && count > 0, "bn_finalize: bad sizes");
  MX_CHECK_ARG((rm == nullptr) == (rv == nullptr), "bn_finalize: running mean/var must both be given or both null");
  MX_CHECK_ARG(cdiv(K, 64) <= MAX_CHUNKS, "bn_finalize: K > %d", MAX_CHUNKS * 64);
  const size_t need = mx_bn_finalize_workspace(mb, K);
  MX_CHECK_ARG(ws && ws_bytes >= need, "bn_finalize: workspace of %zu bytes required (mx_bn_finalize_workspace)", need);
  dim3 grid((unsigned)cdiv(K, 64), (unsigned)fin_slices(mb));
  bn_finalize_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(stats, mb, K, count, gamma, beta, eps, momentum, rm, rv, mean,
                                                            invstd, scale, shift, (unsigned*)ws,
                                                            (double*)((char*)ws + CTR_BYTES));
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_bn_bwd_finalize(const float* part, int64_t mb, int64_t K, int64_t M, const float* mean,
                                  const float* invstd, const float* gamma, float* sums, float* coef, void* ws,
                                  size_t ws_bytes, mx_stream_t stream) {
  MX_CHECK_ARG(mb > 0 && K > 0 && M > 0 && part && mean && invstd && sums && coef, "bn_bwd_finalize: bad arguments");
  MX_CHECK_ARG(cdiv(K, 64) <= MAX_CHUNKS, "bn_bwd_finalize: K > %d", MAX_CHUNKS * 64);
  const size_t need = mx_bn_finalize_workspace(mb, K);
  MX_CHECK_ARG(ws && ws_bytes >= need, "bn_bwd_finalize: workspace of %zu bytes required (mx_bn_finalize_workspace)",
               need);
  dim3 grid((unsigned)cdiv(K, 64), (unsigned)fin_slices(mb));
  bn_bwd_finalize_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(part, mb, K, M, mean, invstd, gamma, sums, coef,
                                                                (unsigned*)ws, (double*)((char*)ws + CTR_BYTES));
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_bn_finalize(const float* stats, int64_t mb, int64_t K, int64_t count, const float* gamma,
                              const float* beta, float eps, float momentum, float* rm, float* rv, float* mean,
                              float* invstd, float* scale, float* shift, mx_stream_t stream) {
  MX_CHECK_ARG(mb > 0 && K > 0 && count > 0, "bn_finalize: bad sizes");
  hipStream_t st = (hipStream_t)stream;
  const size_t wsb = mx_bn_finalize_workspace(mb, K);
  void* ws = nullptr;
  MX_HIP(hipMallocAsync(&ws, wsb, st));
  MX_HIP(hipMemsetAsync(ws, 0, CTR_BYTES, st));
  int rc = mx_bn_finalize_ex(stats, mb, K, count, gamma, beta, eps, momentum, rm, rv, mean, invstd, scale, shift, ws,
                             wsb, stream);
  MX_HIP(hipFreeAsync(ws, st));
  return rc;
}

extern "C" int mx_bn_apply(const void* x, int xdtype, int64_t M, int64_t K, const float* scale, const float* shift,
                           const void* residual, int act, void* y, int ydtype, mx_stream_t stream) {
  MX_CHECK_ARG(K % 8 == 0, "bn_apply: K %% 8 != 0");
  MX_CHECK_ARG((xdtype == MX_BF16 || xdtype == MX_F32) && (ydtype == MX_BF16 || ydtype == MX_F32), "bn_apply: bad dtype");
  if (M == 0) return MX_OK;
  const unsigned grid = grid_rows(M, K / 8);
  hipStream_t st = (hipStream_t)stream;
  if (xdtype == MX_BF16 && ydtype == MX_BF16)
    bn_apply_kernel<uint16_t, uint16_t><<<grid, 256, 0, st>>>((const uint16_t*)x, M, K, scale, shift,
                                                             (const uint16_t*)residual, act, (uint16_t*)y);
  else if (xdtype == MX_F32 && ydtype == MX_BF16)
    bn_apply_kernel<float, uint16_t><<<grid, 256, 0, st>>>((const float*)x, M, K, scale, shift, (const uint16_t*)residual,
                                                          act, (uint16_t*)y);
  else if (xdtype == MX_F32 && ydtype == MX_F32)
    bn_apply_kernel<float, float><<<grid, 256, 0, st>>>((const float*)x, M, K, scale, shift, (const float*)residual, act,
                                                       (float*)y);
  else
    MX_CHECK_ARG(false, "bn_apply: bf16 input with f32 output is not a supported combination");
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_bn_apply_p(const float* x, int64_t M, int64_t K, const float* scale, const float* shift,
                             const float* residual, int act, float* y, uint16_t* planes, mx_stream_t stream) {
  MX_CHECK_ARG(K % 8 == 0 && x && y && planes, "bn_apply_p: K %% 8 != 0 or a null operand");
  if (M == 0) return MX_OK;
  bn_apply_kernel<float, float><<<grid_rows(M, K / 8), 256, 0, (hipStream_t)stream>>>(x, M, K, scale, shift, residual,
                                                                                       act, y, planes);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" size_t mx_bn_bwd_workspace(int64_t M, int64_t K) {
  if (M <= 0 || K <= 0 || K % 8) return 0;
  BwdGeo g = bwd_geo(M, K);
  return CTR_BYTES + sizeof(float) * 2 * (size_t)g.RB * K;
}

template <typename T>
static void bn_bwd_reduce_launch(const void* dy, const void* y, const void* x, int64_t M, int64_t K, int act,
                                 const BwdGeo& g, const float* mean, const float* invstd, const float* gamma, unsigned* ctr,
                                 float* part, float* sums, float* coef, hipStream_t st) {
  dim3 grid((unsigned)g.RB, (unsigned)g.gy);
  const T *d = (const T*)dy, *yy = (const T*)y, *xx = (const T*)x;
  if (act == 1)
    bn_bwd_reduce_kernel<1, T><<<grid, 256, 0, st>>>(d, yy, xx, M, K, g.rows_per_block, mean, invstd, gamma, ctr, part, sums, coef);
  else if (act == 2)
    bn_bwd_reduce_kernel<2, T><<<grid, 256, 0, st>>>(d, yy, xx, M, K, g.rows_per_block, mean, invstd, gamma, ctr, part, sums, coef);
  else
    bn_bwd_reduce_kernel<0, T><<<grid, 256, 0, st>>>(d, yy, xx, M, K, g.rows_per_block, mean, invstd, gamma, ctr, part, sums, coef);
}

extern "C" int mx_bn_bwd_reduce_ex(const void* dy, const void* y, const void* x, int dtype, int64_t M, int64_t K, int act,
                                   const float* mean, const float* invstd, const float* gamma, void* ws, size_t ws_bytes,
                                   float* sums, float* coef, mx_stream_t stream) {
  MX_CHECK_ARG(K % 8 == 0 && K > 0 && M > 0, "bn_bwd_reduce: K must be a positive multiple of 8, M > 0");
  MX_CHECK_ARG(act >= 0 && act <= 2, "bn_bwd_reduce: act 0/1/2");
  MX_CHECK_ARG(act == 0 || y, "bn_bwd_reduce: y required for an activation");
  BwdGeo g = bwd_geo(M, K);
  const size_t need = mx_bn_bwd_workspace(M, K);
  MX_CHECK_ARG(ws && ws_bytes >= need, "bn_bwd_reduce: workspace of %zu bytes required (mx_bn_bwd_workspace)", need);
  MX_CHECK_ARG(g.gy <= MAX_CHUNKS && g.RB < 65536, "bn_bwd_reduce: K > %d", MAX_CHUNKS * 64);
  unsigned* ctr = (unsigned*)ws;
  float* part = (float*)((char*)ws + CTR_BYTES);
  MX_DT_DISPATCH(dtype, bn_bwd_reduce_launch, dy, y, x, M, K, act, g, mean, invstd, gamma, ctr, part, sums, coef,
                 (hipStream_t)stream);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

template <typename T>
static void bn_bwd_apply_launch(const void* dy, const void* y, const void* x, int64_t n8, int K8, int act, const float* coef,
                                void* dx, void* dres, hipStream_t st) {
  const unsigned blocks = (unsigned)cdiv(n8, 256);
  const T *d = (const T*)dy, *yy = (const T*)y, *xx = (const T*)x;
  if (act == 1) bn_bwd_apply2_kernel<1, T><<<blocks, 256, 0, st>>>(d, yy, xx, n8, K8, coef, (T*)dx, (T*)dres);
  else if (act == 2) bn_bwd_apply2_kernel<2, T><<<blocks, 256, 0, st>>>(d, yy, xx, n8, K8, coef, (T*)dx, (T*)dres);
  else bn_bwd_apply2_kernel<0, T><<<blocks, 256, 0, st>>>(d, yy, xx, n8, K8, coef, (T*)dx, (T*)dres);
}

extern "C" int mx_bn_bwd_apply_ex(const void* dy, const void* y, const void* x, int dtype, int64_t M, int64_t K, int act,
                                  const float* coef, void* dx, void* dres, mx_stream_t stream) {
  MX_CHECK_ARG(K % 8 == 0 && K > 0 && K < (1 << 24), "bn_bwd_apply: K must be a positive multiple of 8");
  MX_CHECK_ARG(act >= 0 && act <= 2, "bn_bwd_apply: act 0/1/2");
  MX_CHECK_ARG(act == 0 || y, "bn_bwd_apply: y required for an activation");
  if (M == 0) return MX_OK;
  const int64_t n8 = M * (K / 8);
  MX_DT_DISPATCH(dtype, bn_bwd_apply_launch, dy, y, x, n8, (int)(K / 8), act, coef, dx, dres, (hipStream_t)stream);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_bn_bwd_apply_p(const float* dy, const float* y, const float* x, int64_t M, int64_t K, int act,
                                 const float* coef, float* dx, float* dres, uint16_t* planes, mx_stream_t stream) {
  MX_CHECK_ARG(K % 8 == 0 && K > 0 && K < (1 << 24) && planes, "bn_bwd_apply_p: K %% 8 != 0 or no planes");
  MX_CHECK_ARG(act >= 0 && act <= 2 && (act == 0 || y), "bn_bwd_apply_p: act 0/1/2 (y required for 1, 2)");
  if (M == 0) return MX_OK;
  const int64_t n8 = M * (K / 8);
  const unsigned blocks = (unsigned)cdiv(n8, 256);
  hipStream_t st = (hipStream_t)stream;
  const int K8 = (int)(K / 8);
  if (act == 1) bn_bwd_apply2_kernel<1, float><<<blocks, 256, 0, st>>>(dy, y, x, n8, K8, coef, dx, dres, planes);
  else if (act == 2) bn_bwd_apply2_kernel<2, float><<<blocks, 256, 0, st>>>(dy, y, x, n8, K8, coef, dx, dres, planes);
  else bn_bwd_apply2_kernel<0, float><<<blocks, 256, 0, st>>>(dy, y, x, n8, K8, coef, dx, dres, planes);
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
  MX_HIP(hipMemsetAsync(ws, 0, CTR_BYTES, st));
  MX_HIP(hipMallocAsync((void**)&coef, sizeof(float) * 3 * K, st));
  int rc = mx_bn_bwd_reduce_ex(dy, y, x, MX_BF16, M, K, act, mean, invstd, nullptr, ws, wsb, sums, coef, stream);
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
  if (!rc) rc = mx_bn_bwd_apply_ex(dy, y, x, MX_BF16, M, K, act, coef, dx, dres, stream);
  MX_HIP(hipFreeAsync(coef, st));
  return rc;
}

static BwdGeo act_geo(int64_t M, int64_t K8) {
  BwdGeo g;
  g.gy = cdiv(K8, 64);
  g.RB = std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(128, cdiv(M, 64)), std::max<int64_t>(1, 1024 / g.gy)));
  g.rows_per_block = cdiv(M, g.RB);
  g.RB = cdiv(M, g.rows_per_block);
  return g;
}

extern "C" size_t mx_act_bias_bwd_workspace(int64_t M, int64_t K) {
  if (M <= 0 || K <= 0) return 0;
  BwdGeo g = act_geo(M, (K + 7) / 8 * 8);
  return CTR_BYTES + sizeof(float) * (size_t)g.RB * K;
}

template <typename T, typename TG>
static void launch_act_bias(const void* gy, const void* y, int64_t M, int K, int K8, int act, const BwdGeo& g,
                            void* out_, float* db, unsigned* ctr, float* part, hipStream_t st, uint16_t* planes = nullptr) {
  dim3 grid((unsigned)g.RB, (unsigned)g.gy);
  TG* out = (TG*)out_;
  if (act == 1)
    act_bias_bwd_kernel<T, 1, TG><<<grid, 256, 0, st>>>((const T*)gy, (const T*)y, M, K, K8, g.rows_per_block, out, db, ctr,
                                                        part, planes);
  else if (act == 2)
    act_bias_bwd_kernel<T, 2, TG><<<grid, 256, 0, st>>>((const T*)gy, (const T*)y, M, K, K8, g.rows_per_block, out, db, ctr,
                                                        part, planes);
  else
    act_bias_bwd_kernel<T, 0, TG><<<grid, 256, 0, st>>>((const T*)gy, (const T*)y, M, K, K8, g.rows_per_block, out, db, ctr,
                                                        part, planes);
}

extern "C" int mx_act_bias_bwd(const void* gy, const void* y, int dtype, int64_t M, int64_t K, int64_t K8, int act,
                               void* g, int gdtype, float* db, void* ws, size_t ws_bytes, mx_stream_t stream) {
  MX_CHECK_ARG(M >= 0 && K > 0 && K8 >= K && K8 % 8 == 0 && K8 < (1 << 24), "act_bias_bwd: need 0 < K <= K8, K8 %% 8 == 0");
  MX_CHECK_ARG(act >= 0 && act <= 2 && (act == 0 || y), "act_bias_bwd: act 0/1/2 (y required for 1/2)");
  MX_CHECK_ARG(dtype == MX_BF16 || dtype == MX_F32, "act_bias_bwd: dtype bf16 or f32");
  MX_CHECK_ARG(gdtype == MX_BF16 || gdtype == MX_F32, "act_bias_bwd: gdtype bf16 or f32");
  if (M == 0) {
    if (db) MX_HIP(hipMemsetAsync(db, 0, sizeof(float) * K, (hipStream_t)stream));
    return MX_OK;
  }
  BwdGeo g_ = act_geo(M, K8);
  MX_CHECK_ARG(g_.gy <= MAX_CHUNKS, "act_bias_bwd: K8 > %d", MAX_CHUNKS * 64);
  unsigned* ctr = nullptr;
  float* part = nullptr;
  if (db) {
    const size_t need = mx_act_bias_bwd_workspace(M, K);
    MX_CHECK_ARG(ws && ws_bytes >= need, "act_bias_bwd: workspace of %zu bytes required (mx_act_bias_bwd_workspace)", need);
    ctr = (unsigned*)ws;
    part = (float*)((char*)ws + CTR_BYTES);
  }
  hipStream_t st = (hipStream_t)stream;
  if (dtype == MX_BF16 && gdtype == MX_BF16)
    launch_act_bias<uint16_t, uint16_t>(gy, y, M, (int)K, (int)K8, act, g_, g, db, ctr, part, st);
  else if (dtype == MX_F32 && gdtype == MX_BF16)
    launch_act_bias<float, uint16_t>(gy, y, M, (int)K, (int)K8, act, g_, g, db, ctr, part, st);
  else if (dtype == MX_F32 && gdtype == MX_F32)
    launch_act_bias<float, float>(gy, y, M, (int)K, (int)K8, act, g_, g, db, ctr, part, st);
  else
    MX_CHECK_ARG(false, "act_bias_bwd: bf16 input with f32 gradient output is not a supported combination");
  MX_LAUNCH_CHECK();
  return MX_OK;
}

// mx_act_bias_bwd for f32 (the bf16x3 path) that also writes g's bf16x3 planes [2][M][K8] (split8: what
// mx_split_planes would write) for the convs' x3p dgrad / wgrad -- no separate split pass over g
extern "C" int mx_act_bias_bwd_p(const float* gy, const float* y, int64_t M, int64_t K, int64_t K8, int act, float* g,
                                 float* db, void* ws, size_t ws_bytes, uint16_t* planes, mx_stream_t stream) {
  MX_CHECK_ARG(planes != nullptr && M > 0, "act_bias_bwd_p: planes and M > 0 required");
  MX_CHECK_ARG(K > 0 && K8 >= K && K8 % 8 == 0 && K8 < (1 << 24), "act_bias_bwd: need 0 < K <= K8, K8 %% 8 == 0");
  MX_CHECK_ARG(act >= 0 && act <= 2 && (act == 0 || y), "act_bias_bwd: act 0/1/2 (y required for 1/2)");
  BwdGeo g_ = act_geo(M, K8);
  MX_CHECK_ARG(g_.gy <= MAX_CHUNKS, "act_bias_bwd: K8 > %d", MAX_CHUNKS * 64);
  unsigned* ctr = nullptr;
  float* part = nullptr;
  if (db) {
    const size_t need = mx_act_bias_bwd_workspace(M, K);
    MX_CHECK_ARG(ws && ws_bytes >= need, "act_bias_bwd: workspace of %zu bytes required (mx_act_bias_bwd_workspace)", need);
    ctr = (unsigned*)ws;
    part = (float*)((char*)ws + CTR_BYTES);
  }
  launch_act_bias<float, float>(gy, y, M, (int)K, (int)K8, act, g_, g, db, ctr, part, (hipStream_t)stream, planes);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" size_t mx_rpn_loss_workspace(int64_t n) {
  (void)n;
  return CTR_BYTES + sizeof(double) * 3 * 1024;
}

extern "C" int mx_rpn_loss_fwd(const float* objectness, const float* deltas, const float* labels, const float* targets,
                               const uint8_t* pos, const uint8_t* neg, int64_t n, float beta, float* out, void* ws,
                               size_t ws_bytes, mx_stream_t stream) {
  MX_CHECK_ARG(n > 0 && objectness && deltas && labels && targets && pos && neg && out, "rpn_loss: bad arguments");
  MX_CHECK_ARG(ws && ws_bytes >= mx_rpn_loss_workspace(n), "rpn_loss: workspace too small");
  const unsigned blocks = (unsigned)std::min<int64_t>(1024, cdiv(n, 256 * 4));
  rpn_loss_fwd_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(objectness, (const float4*)deltas, labels,
                                                               (const float4*)targets, pos, neg, n, beta,
                                                               (unsigned*)ws, (double*)((char*)ws + CTR_BYTES), out);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_rpn_loss_bwd(const float* objectness, const float* deltas, const float* labels, const float* targets,
                               const uint8_t* pos, const uint8_t* neg, int64_t n, float beta, const float* out,
                               const float* grad0, const float* grad1, float* grad_objectness, float* grad_deltas,
                               mx_stream_t stream) {
  MX_CHECK_ARG(n > 0 && out && grad_objectness && grad_deltas, "rpn_loss bwd: bad arguments");
  rpn_loss_bwd_kernel<<<(unsigned)cdiv(n, 256), 256, 0, (hipStream_t)stream>>>(
      objectness, (const float4*)deltas, labels, (const float4*)targets, pos, neg, n, beta, out, grad0, grad1,
      grad_objectness, (float4*)grad_deltas);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_roi_loss_fwd(const float* logits, int64_t ldl, int C, const float* reg, int64_t ldr,
                               const int64_t* labels, const float* targets, int64_t R, float beta, float* out, void* ws,
                               size_t ws_bytes, mx_stream_t stream) {
  MX_CHECK_ARG(R > 0 && C > 0 && ldl >= C && ldr >= 4 * C && logits && reg && labels && targets && out,
               "roi_loss: bad arguments");
  const int64_t blocks = cdiv(R, 256);
  MX_CHECK_ARG(blocks <= 1024 && ws && ws_bytes >= mx_rpn_loss_workspace(R), "roi_loss: workspace / size");
  roi_loss_fwd_kernel<<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(logits, ldl, C, reg, ldr, labels, targets, R,
                                                                         beta, (unsigned*)ws,
                                                                         (double*)((char*)ws + CTR_BYTES), out);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_roi_loss_bwd(const float* logits, int64_t ldl, int C, const float* reg, int64_t ldr,
                               const int64_t* labels, const float* targets, int64_t R, float beta, const float* grad0,
                               const float* grad1, float* grad_logits, float* grad_reg, mx_stream_t stream) {
  MX_CHECK_ARG(R > 0 && C > 0 && grad_logits && grad_reg, "roi_loss bwd: bad arguments");
  roi_loss_bwd_kernel<<<(unsigned)cdiv(R, 256), 256, 0, (hipStream_t)stream>>>(logits, ldl, C, reg, ldr, labels, targets,
                                                                               R, beta, grad0, grad1, grad_logits,
                                                                               grad_reg);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_bn_act_maxpool(const float* z, int64_t N, int64_t H, int64_t W, int64_t C, const float* scale,
                                 const float* shift, int act, int k, int stride, int pad, float* y, mx_stream_t stream) {
  MX_CHECK_ARG(z && scale && shift && y, "bn_act_maxpool: null operand");
  MX_CHECK_ARG(N >= 0 && H > 0 && W > 0 && C > 0 && C % 8 == 0, "bn_act_maxpool: bad shape (C %% 8 == 0)");
  MX_CHECK_ARG(k > 0 && stride > 0 && pad >= 0 && pad * 2 <= k, "bn_act_maxpool: bad pooling window");
  MX_CHECK_ARG(act >= 0 && act <= 2, "bn_act_maxpool: act %d", act);
  const int64_t Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  const int64_t n = N * Ho * Wo * (C / 8);
  if (n == 0) return MX_OK;
  bn_act_maxpool_kernel<<<(unsigned)cdiv(n, 256), 256, 0, (hipStream_t)stream>>>(z, N, H, W, C, Ho, Wo, k, stride, pad,
                                                                                   scale, shift, act, y);
  MX_LAUNCH_CHECK();
  return MX_OK;
}
