// mx_sample.hip — the BalancedPositiveNegativeSampler draw in one launch, gfx950.
//
// torchvision det_utils.BalancedPositiveNegativeSampler (reached through RegionProposalNetwork and
// RoIHeads.select_training_samples from train_frcnn_baseline.py:171): per image row of labels, positives
// (label >= 1) and negatives (label == 0); num_pos = min(#pos, int(B * frac)), num_neg = min(#neg, B -
// num_pos); each drawn uniformly without replacement. The framework draws them as the num smallest of
// i.i.d. uniform keys among the candidates (ties by lowest index) -- a uniform random subset, as
// randperm(n)[:num] is (mx_det.frcnn.BalancedPositiveNegativeSampler). One 1024-thread workgroup per
// row does, for both classes at once:
//   1. radix select of each class's num-th smallest key on order-preserving u32 keys: three digit passes
//      (11 / 11 / 10 bits, MSB first) into LDS histograms (four copies by wave group: uniform keys
//      cluster in the exponent bits), coalesced grid-stride reads of the row; the first pass also
//      counts the candidates, so no count input is needed;
//   2. one marking pass: a candidate is drawn when its key is below its class's threshold T, or equal
//      to T and among the first (num - #below) such keys by index (a block-wide ballot scan per tile of
//      1,024 consecutive elements, run only when the keys equal to T outnumber the ones still needed).
// Outputs pos / neg (uint8 [N][L]), optionally their union sm, and nums [N][2] = (num_pos, num_neg).
// Replaces ~30 small launches per sampler (compares, where, cat, the top-k, scatter marks, sums).
#include "mx_common.h"

namespace mx {

static constexpr int64_t SP_SLICED_MIN = 16384;  // rows longer than this take the sliced form
static constexpr int SP_THREADS = 1024, SP_BINS = 2048, SP_COPIES = 4, SP_WAVES = SP_THREADS / 64, SP_UNROLL = 8;

__device__ __forceinline__ uint32_t sp_ord(float f) {  // order-preserving; -0.0 and +0.0 tie
  uint32_t u = __float_as_uint(f);
  if (u == 0x80000000u) u = 0u;
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

template <typename LT>
__device__ __forceinline__ int sp_class(LT v, const uint8_t* __restrict__ valid = nullptr, int64_t i = 0) {
  // 0 positive, 1 negative, -1 neither (or masked out by the optional validity bytes)
  if (valid && !valid[i]) return -1;
  if constexpr (sizeof(LT) == 4) {
    const float f = (float)v;
    return f >= 1.f ? 0 : (f == 0.f ? 1 : -1);
  } else {
    return v >= 1 ? 0 : (v == 0 ? 1 : -1);
  }
}

template <typename LT>
__global__ void __launch_bounds__(SP_THREADS) sample_draw_kernel(const LT* __restrict__ lab, const uint8_t* __restrict__ valid,
                                                                const float* __restrict__ keys,
                                                                int64_t L, int P, int B, uint8_t* __restrict__ pos,
                                                                uint8_t* __restrict__ neg, uint8_t* __restrict__ sm,
                                                                int32_t* __restrict__ nums) {
  __shared__ uint32_t hist[2][SP_COPIES][SP_BINS];
  __shared__ uint32_t s_prefix[2], s_need[2], s_eq[2], s_k[2], s_cnt[2];
  __shared__ uint32_t s_wave[2][SP_WAVES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, copy = wave & (SP_COPIES - 1);
  const int64_t row = blockIdx.x;
  const LT* lr = lab + row * L;
  const uint8_t* vr = valid ? valid + row * L : nullptr;
  const float* kr = keys + row * L;
  // digit d covers bits [sh, sh + w) of the key; the bits above it must equal the prefix so far
  const int shs[3] = {21, 10, 0}, ws[3] = {11, 11, 10};
  uint32_t himask = 0;
  if (tid < 2) s_prefix[tid] = 0;
  for (int d = 0; d < 3; ++d) {
    for (int i = tid; i < 2 * SP_COPIES * SP_BINS; i += SP_THREADS) (&hist[0][0][0])[i] = 0;
    __syncthreads();
    const uint32_t p0 = s_prefix[0], p1 = s_prefix[1];
    const int sh = shs[d];
    const uint32_t dm = (1u << ws[d]) - 1u;
    // SP_UNROLL independent (label, key) loads in flight per thread, coalesced across the wave
    for (int64_t i0 = tid; i0 < L; i0 += (int64_t)SP_THREADS * SP_UNROLL) {
      int cl[SP_UNROLL];
      uint32_t kk[SP_UNROLL];
#pragma unroll
      for (int u = 0; u < SP_UNROLL; ++u) {
        const int64_t i = i0 + (int64_t)u * SP_THREADS;
        cl[u] = i < L ? sp_class<LT>(lr[i], vr, i) : -1;
        kk[u] = i < L ? sp_ord(kr[i]) : 0u;
      }
#pragma unroll
      for (int u = 0; u < SP_UNROLL; ++u) {
        const int c = cl[u];
        if (c >= 0 && (kk[u] & himask) == (c ? p1 : p0)) atomicAdd(&hist[c][copy][(kk[u] >> sh) & dm], 1u);
      }
    }
    __syncthreads();
    // sum the copies; the first pass also yields the candidate counts and the draw sizes
    for (int i = tid; i < 2 * SP_BINS; i += SP_THREADS) {
      const int c = i / SP_BINS, b = i % SP_BINS;
      hist[c][0][b] += hist[c][1][b] + hist[c][2][b] + hist[c][3][b];
    }
    __syncthreads();
    if (d == 0 && wave < 2) {  // wave c counts class c
      uint32_t s = 0;
      for (int b = lane; b < SP_BINS; b += 64) s += hist[wave][0][b];
      for (int o = 32; o; o >>= 1) s += __shfl_xor(s, o);
      if (lane == 0) s_cnt[wave] = s;
    }
    __syncthreads();
    if (d == 0 && tid == 0) {
      const uint32_t kp = min(s_cnt[0], (uint32_t)P);
      const uint32_t kn = min(s_cnt[1], (uint32_t)(B - (int)kp));
      s_k[0] = s_need[0] = kp;
      s_k[1] = s_need[1] = kn;
    }
    __syncthreads();
    // find the bin holding the need-th smallest key of each class: wave c scans class c's bins
    if (wave < 2) {
      const int c = wave;
      const uint32_t need = s_need[c];
      if (need > 0) {
        uint32_t base = 0;  // keys in the bins below this 64-bin chunk
        for (int b0 = 0; b0 < SP_BINS; b0 += 64) {
          const uint32_t h = hist[c][0][b0 + lane];
          uint32_t incl = h;  // inclusive prefix within the chunk
          for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(incl, o);
            if (lane >= o) incl += t;
          }
          const uint32_t tot = __shfl(incl, 63);
          if (base + tot >= need) {
            const uint64_t hit = __ballot(base + incl >= need);
            const int b = __ffsll((unsigned long long)hit) - 1;
            const uint32_t below = base + __shfl(incl - h, b);
            if (lane == 0) {
              s_prefix[c] |= (uint32_t)(b0 + b) << sh;
              s_need[c] = need - below;
              s_eq[c] = hist[c][0][b0 + b];
            }
            break;
          }
          base += tot;
        }
      }
    }
    __syncthreads();
    himask |= dm << sh;
  }
  // marking pass: thresholds T_c = s_prefix[c]; keys equal to T_c are drawn in index order while needed
  const uint32_t T0 = s_prefix[0], T1 = s_prefix[1];
  const uint32_t k0 = s_k[0], k1 = s_k[1];
  const bool rank0 = k0 > 0 && s_need[0] < s_eq[0], rank1 = k1 > 0 && s_need[1] < s_eq[1];
  const bool ranked = rank0 || rank1;
  if (!ranked) {  // the usual case: no rank needed, SP_UNROLL elements in flight per thread
    for (int64_t i0 = tid; i0 < L; i0 += (int64_t)SP_THREADS * SP_UNROLL) {
      int cl[SP_UNROLL];
      uint32_t kk[SP_UNROLL];
#pragma unroll
      for (int u = 0; u < SP_UNROLL; ++u) {
        const int64_t i = i0 + (int64_t)u * SP_THREADS;
        cl[u] = i < L ? sp_class<LT>(lr[i], vr, i) : -1;
        kk[u] = i < L ? sp_ord(kr[i]) : 0u;
      }
#pragma unroll
      for (int u = 0; u < SP_UNROLL; ++u) {
        const int64_t i = i0 + (int64_t)u * SP_THREADS;
        if (i >= L) break;
        const bool t0 = cl[u] == 0 && k0 > 0 && kk[u] <= T0, t1 = cl[u] == 1 && k1 > 0 && kk[u] <= T1;
        pos[row * L + i] = t0;
        neg[row * L + i] = t1;
        if (sm) sm[row * L + i] = t0 || t1;
      }
    }
    if (tid == 0) {
      nums[2 * row] = (int32_t)k0;
      nums[2 * row + 1] = (int32_t)k1;
    }
    return;
  }
  uint32_t taken0 = 0, taken1 = 0;  // equal keys drawn in earlier tiles (uniform)
  for (int64_t t0 = 0; t0 < L; t0 += SP_THREADS) {
    const int64_t i = t0 + tid;
    int c = -1;
    uint32_t k = 0;
    if (i < L) {
      c = sp_class<LT>(lr[i], vr, i);
      k = sp_ord(kr[i]);
    }
    const bool below0 = c == 0 && k0 > 0 && k < T0, below1 = c == 1 && k1 > 0 && k < T1;
    const bool eq0 = c == 0 && k0 > 0 && k == T0, eq1 = c == 1 && k1 > 0 && k == T1;
    bool take0 = below0 || (eq0 && !rank0), take1 = below1 || (eq1 && !rank1);
    if (ranked) {  // (block-uniform branch) rank of this equal key among the tile's, in index order
      const uint64_t m0 = __ballot(eq0), m1 = __ballot(eq1);
      if (lane == 0) {
        s_wave[0][wave] = (uint32_t)__popcll(m0);
        s_wave[1][wave] = (uint32_t)__popcll(m1);
      }
      __syncthreads();
      uint32_t pre0 = 0, pre1 = 0, tot0 = 0, tot1 = 0;
      for (int w = 0; w < SP_WAVES; ++w) {
        const uint32_t a = s_wave[0][w], b = s_wave[1][w];
        if (w < wave) { pre0 += a; pre1 += b; }
        tot0 += a;
        tot1 += b;
      }
      const uint64_t lm = lane ? ((1ull << lane) - 1) : 0ull;
      if (rank0 && eq0) take0 = taken0 + pre0 + (uint32_t)__popcll(m0 & lm) < s_need[0];
      if (rank1 && eq1) take1 = taken1 + pre1 + (uint32_t)__popcll(m1 & lm) < s_need[1];
      taken0 += tot0;
      taken1 += tot1;
      __syncthreads();  // s_wave is rewritten by the next tile
    }
    if (i < L) {
      pos[row * L + i] = take0;
      neg[row * L + i] = take1;
      if (sm) sm[row * L + i] = take0 || take1;
    }
  }
  if (tid == 0) {
    nums[2 * row] = (int32_t)k0;
    nums[2 * row + 1] = (int32_t)k1;
  }
}

// ---- long rows (the RPN's 268,569 anchors): the row split over many workgroups -------------------
// One workgroup reading a 2 MB row three times is bound by one CU's bandwidth (~370 us for two RPN rows).
// Long rows take three launches instead, each over (slices x rows) workgroups:
//   A. sample_hist_kernel: each class's histogram of the keys' top 11 bits (LDS, then global atomics);
//   B. sample_split_kernel: every workgroup finds, from the row's histogram, the boundary bin b_c
//      holding each class's num-th smallest key; candidates below b_c are drawn, above it not, and the
//      boundary bin's candidates are appended to a per-(row, class) list as 64-bit (key, index) pairs;
//   C. sample_finish_kernel: one workgroup per row selects, in each list, the (num - #below) smallest
//      pairs by a radix select on (the key's low 21 bits, index) -- pairs are unique, so "ties by lowest
//      index" is the pair order -- and marks them; it writes nums.
// Uniform keys put a few dozen candidates in a boundary bin; a list can hold the whole row (equal keys).

static constexpr int SH_THREADS = 256, SH_ITEMS = 16;  // elements per thread per slice
static constexpr uint32_t SP_NONE = 0xffffffffu;

__device__ __forceinline__ void sp_hist_zero(uint32_t* h, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) h[i] = 0;
}

template <typename LT>
__global__ void __launch_bounds__(SH_THREADS) sample_hist_kernel(const LT* __restrict__ lab, const uint8_t* __restrict__ valid,
                                                                const float* __restrict__ keys, int64_t L,
                                                                uint32_t* __restrict__ ghist) {
  __shared__ uint32_t h[2][SP_BINS];
  sp_hist_zero(&h[0][0], 2 * SP_BINS);
  __syncthreads();
  const int64_t row = blockIdx.y, base = (int64_t)blockIdx.x * SH_THREADS * SH_ITEMS;
  const LT* lr = lab + row * L;
  const uint8_t* vr = valid ? valid + row * L : nullptr;
  const float* kr = keys + row * L;
#pragma unroll 4
  for (int u = 0; u < SH_ITEMS; ++u) {
    const int64_t i = base + (int64_t)u * SH_THREADS + threadIdx.x;
    if (i < L) {
      const int c = sp_class<LT>(lr[i], vr, i);
      if (c >= 0) atomicAdd(&h[c][sp_ord(kr[i]) >> 21], 1u);
    }
  }
  __syncthreads();
  uint32_t* g = ghist + row * 2 * SP_BINS;
  for (int i = threadIdx.x; i < 2 * SP_BINS; i += SH_THREADS) {
    const uint32_t v = (&h[0][0])[i];
    if (v) atomicAdd(&g[i], v);
  }
}

// per class c of a row: draw size k_c, boundary bin b_c (SP_NONE: nothing drawn) and #candidates below
// it, from the row's global histogram; waves 0 / 1 of the calling workgroup, results in LDS
__device__ __forceinline__ void sp_boundaries(const uint32_t* __restrict__ g, int P, int B, uint32_t* s_cnt,
                                              uint32_t* s_k, uint32_t* s_bin, uint32_t* s_below) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (wave < 2) {
    uint32_t t = 0;
    for (int b = lane; b < SP_BINS; b += 64) t += g[wave * SP_BINS + b];
    for (int o = 32; o; o >>= 1) t += __shfl_xor(t, o);
    if (lane == 0) s_cnt[wave] = t;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    s_k[0] = min(s_cnt[0], (uint32_t)P);
    s_k[1] = min(s_cnt[1], (uint32_t)(B - (int)s_k[0]));
  }
  __syncthreads();
  if (wave < 2) {
    const uint32_t need = s_k[wave];
    const uint32_t* gc = g + wave * SP_BINS;
    uint32_t bin = SP_NONE, below = 0, base = 0;
    if (need > 0) {
      for (int b0 = 0; b0 < SP_BINS; b0 += 64) {
        const uint32_t hv = gc[b0 + lane];
        uint32_t incl = hv;
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t t = __shfl_up(incl, o);
          if (lane >= o) incl += t;
        }
        const uint32_t tot = __shfl(incl, 63);
        if (base + tot >= need) {
          const int b = __ffsll((unsigned long long)__ballot(base + incl >= need)) - 1;
          bin = (uint32_t)(b0 + b);
          below = base + __shfl(incl - hv, b);
          break;
        }
        base += tot;
      }
    }
    if (lane == 0) {
      s_bin[wave] = bin;
      s_below[wave] = below;
    }
  }
  __syncthreads();
}

template <typename LT>
__global__ void __launch_bounds__(SH_THREADS) sample_split_kernel(const LT* __restrict__ lab, const uint8_t* __restrict__ valid,
                                                                 const float* __restrict__ keys,
                                                                 int64_t L, int P, int B, const uint32_t* __restrict__ ghist,
                                                                 uint32_t* __restrict__ lcount, uint64_t* __restrict__ lists,
                                                                 uint8_t* __restrict__ pos, uint8_t* __restrict__ neg,
                                                                 uint8_t* __restrict__ sm) {
  __shared__ uint32_t s_cnt[2], s_k[2], s_bin[2], s_below[2];
  const int64_t row = blockIdx.y, base = (int64_t)blockIdx.x * SH_THREADS * SH_ITEMS;
  sp_boundaries(ghist + row * 2 * SP_BINS, P, B, s_cnt, s_k, s_bin, s_below);
  const uint32_t b0 = s_bin[0], b1 = s_bin[1];
  const LT* lr = lab + row * L;
  const uint8_t* vr = valid ? valid + row * L : nullptr;
  const float* kr = keys + row * L;
#pragma unroll 4
  for (int u = 0; u < SH_ITEMS; ++u) {
    const int64_t i = base + (int64_t)u * SH_THREADS + threadIdx.x;
    if (i < L) {
      const int c = sp_class<LT>(lr[i], vr, i);
      bool t0 = false, t1 = false;
      if (c >= 0) {
        const uint32_t k = sp_ord(kr[i]), b = k >> 21, bc = c ? b1 : b0;
        if (bc == SP_NONE) {
        } else if (b < bc) {
          t0 = c == 0;
          t1 = c == 1;
        } else if (b == bc) {  // boundary bin: decided by sample_finish_kernel
          const uint32_t at = atomicAdd(&lcount[row * 2 + c], 1u);
          lists[(row * 2 + c) * L + at] = ((uint64_t)(k & 0x1fffffu) << 32) | (uint64_t)i;
        }
      }
      pos[row * L + i] = t0;
      neg[row * L + i] = t1;
      if (sm) sm[row * L + i] = t0 || t1;
    }
  }
}

__global__ void __launch_bounds__(SP_THREADS) sample_finish_kernel(int64_t L, int P, int B, const uint32_t* __restrict__ ghist,
                                                                  const uint32_t* __restrict__ lcount,
                                                                  const uint64_t* __restrict__ lists, uint8_t* __restrict__ pos,
                                                                  uint8_t* __restrict__ neg, uint8_t* __restrict__ sm,
                                                                  int32_t* __restrict__ nums) {
  __shared__ uint32_t s_cnt[2], s_k[2], s_bin[2], s_below[2];
  __shared__ uint32_t hist[SP_BINS];
  __shared__ uint64_t s_prefix, s_pairs[SP_THREADS];
  __shared__ uint32_t s_need;
  const int64_t row = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  sp_boundaries(ghist + row * 2 * SP_BINS, P, B, s_cnt, s_k, s_bin, s_below);
  for (int c = 0; c < 2; ++c) {
    if (s_k[c] == 0) continue;  // block-uniform
    const uint64_t* lst = lists + (row * 2 + c) * L;
    const uint32_t m = lcount[row * 2 + c];
    const uint32_t need0 = s_k[c] - s_below[c];  // 1 <= need0 <= m
    uint8_t* mk = c ? neg : pos;
    uint64_t T = ~0ull;                          // take the pairs <= T
    if (need0 < m && m <= SP_THREADS) {
      // short list (the usual case: a few dozen uniform keys share the boundary bin): rank each pair by
      // counting the smaller ones (LDS broadcast reads); the pair of rank need0 - 1 is the threshold
      s_pairs[tid] = tid < (int)m ? lst[tid] : ~0ull;
      __syncthreads();
      if (tid < (int)m) {
        const uint64_t v = s_pairs[tid];
        uint32_t r = 0;
        for (uint32_t j = 0; j < m; ++j) r += s_pairs[j] < v;
        if (r == need0 - 1) s_prefix = v;
      }
      __syncthreads();
      T = s_prefix;
    } else if (need0 < m) {
      // radix select of the need0-th smallest 53-bit pair: digits of 11 / 10 (key) and 11 / 11 / 10 (index)
      const int shs[5] = {42, 32, 21, 10, 0}, ws[5] = {11, 10, 11, 11, 10};
      if (tid == 0) {
        s_prefix = 0;
        s_need = need0;
      }
      uint64_t himask = 0;
      for (int d = 0; d < 5; ++d) {
        sp_hist_zero(hist, SP_BINS);
        __syncthreads();
        const uint64_t pre = s_prefix;
        const uint32_t dm = (1u << ws[d]) - 1u;
        for (uint32_t j = tid; j < m; j += SP_THREADS) {
          const uint64_t v = lst[j];
          if ((v & himask) == pre) atomicAdd(&hist[(uint32_t)(v >> shs[d]) & dm], 1u);
        }
        __syncthreads();
        if (wave == 0) {
          const uint32_t need = s_need;
          uint32_t base = 0;
          for (int b0 = 0; b0 < SP_BINS; b0 += 64) {
            const uint32_t hv = hist[b0 + lane];
            uint32_t incl = hv;
            for (int o = 1; o < 64; o <<= 1) {
              const uint32_t t = __shfl_up(incl, o);
              if (lane >= o) incl += t;
            }
            const uint32_t tot = __shfl(incl, 63);
            if (base + tot >= need) {
              const int b = __ffsll((unsigned long long)__ballot(base + incl >= need)) - 1;
              const uint32_t below = base + __shfl(incl - hv, b);  // all lanes: a shuffle reads lane b
              if (lane == 0) {
                s_prefix = pre | ((uint64_t)(b0 + b) << shs[d]);
                s_need = need - below;
              }
              break;
            }
            base += tot;
          }
        }
        __syncthreads();
        himask |= (uint64_t)dm << shs[d];
      }
      T = s_prefix;  // the need0-th smallest pair itself (pairs are unique)
    }
    for (uint32_t j = tid; j < m; j += SP_THREADS) {
      const uint64_t v = lst[j];
      if (v <= T) {
        const int64_t i = (int64_t)(v & 0xffffffffu);
        mk[row * L + i] = 1;
        if (sm) sm[row * L + i] = 1;
      }
    }
    __syncthreads();  // hist / s_prefix are reused by the next class
  }
  if (tid == 0) {
    nums[2 * row] = (int32_t)s_k[0];
    nums[2 * row + 1] = (int32_t)s_k[1];
  }
}

// RoIHeads.select_training_samples' candidate rows: per image its post padded proposal slots (valid where
// pvalid) then its gm padded GT slots (valid below gcnt), torchvision's cat([proposals, gt]) -- boxes
// [N][post + gm][4] and validity bytes in one launch (replacing an arange, a compare and two cats)
__global__ void roi_candidates_kernel(const float4* __restrict__ pb, const uint8_t* __restrict__ pvalid,
                                      const float4* __restrict__ gtp, const int32_t* __restrict__ gcnt, int64_t N,
                                      int64_t post, int64_t gm, float4* __restrict__ box, uint8_t* __restrict__ valid) {
  const int64_t L = post + gm;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N * L) return;
  const int64_t n = e / L, j = e - n * L;
  if (j < post) {
    box[e] = pb[n * post + j];
    valid[e] = pvalid[n * post + j] ? 1 : 0;
  } else {
    box[e] = gtp[n * gm + (j - post)];
    valid[e] = (j - post) < (int64_t)gcnt[n] ? 1 : 0;
  }
}

}  // namespace mx

using namespace mx;

extern "C" int mx_roi_candidates(const float* pb, const uint8_t* pvalid, const float* gtp, const int32_t* gcnt, int64_t N,
                                 int64_t post, int64_t gm, float* box, uint8_t* valid, mx_stream_t stream) {
  MX_CHECK_ARG(N >= 0 && post >= 0 && gm >= 0, "roi_candidates: negative size");
  const int64_t n = N * (post + gm);
  if (n == 0) return MX_OK;
  MX_CHECK_ARG(box && valid && gcnt && (post == 0 || (pb && pvalid)) && (gm == 0 || gtp), "roi_candidates: null operand");
  mx::roi_candidates_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      (const float4*)pb, pvalid, (const float4*)gtp, gcnt, N, post, gm, (float4*)box, valid);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

// workspace of mx_sample_draw_ws for N rows of L: histograms, list counts, boundary lists
static size_t sample_ws_bytes(int64_t N, int64_t L) {
  return (size_t)N * (2 * SP_BINS + 2) * 4 + (size_t)N * 2 * L * 8 + 64;
}

extern "C" size_t mx_sample_draw_workspace(int64_t N, int64_t L) { return sample_ws_bytes(N, L); }

// the sliced three-launch form for rows longer than one workgroup's comfortable share (see above);
// shorter rows (and ws == NULL) take mx_sample_draw's one-workgroup-per-row kernel. Same results.
extern "C" int mx_sample_draw(const void* labels, int ldtype, const uint8_t* valid, const float* keys, int64_t N,
                              int64_t L, int batch, double positive_fraction, uint8_t* pos, uint8_t* neg, uint8_t* sm,
                              int32_t* nums, mx_stream_t stream);

extern "C" int mx_sample_draw_ws(const void* labels, int ldtype, const uint8_t* valid, const float* keys, int64_t N,
                                 int64_t L, int batch, double positive_fraction, uint8_t* pos, uint8_t* neg, uint8_t* sm,
                                 int32_t* nums, void* ws, size_t ws_bytes, mx_stream_t stream) {
  if (ws == nullptr || L <= SP_SLICED_MIN)
    return mx_sample_draw(labels, ldtype, valid, keys, N, L, batch, positive_fraction, pos, neg, sm, nums, stream);
  MX_CHECK_ARG(N >= 0 && batch >= 0 && labels && keys && pos && neg && nums, "sample_draw: null operand");
  MX_CHECK_ARG(ldtype == MX_F32 || ldtype == 2, "sample_draw: labels must be f32 (0) or int64 (2)");
  MX_CHECK_ARG(N < 65536 && L < (1ll << 31), "sample_draw: sliced rows must be < 2^31 long, < 65536 rows");
  MX_CHECK_ARG(ws_bytes >= sample_ws_bytes(N, L), "sample_draw: workspace too small (%zu < %zu)", ws_bytes,
               sample_ws_bytes(N, L));
  if (N == 0) return MX_OK;
  const int P = (int)(batch * positive_fraction);
  hipStream_t st = (hipStream_t)stream;
  uint32_t* ghist = (uint32_t*)ws;
  uint32_t* lcount = ghist + N * 2 * SP_BINS;
  uint64_t* lists = (uint64_t*)(((uintptr_t)(lcount + N * 2) + 63) & ~(uintptr_t)63);
  MX_HIP(hipMemsetAsync(ws, 0, (size_t)N * (2 * SP_BINS + 2) * 4, st));
  const dim3 grid((unsigned)((L + SH_THREADS * SH_ITEMS - 1) / (SH_THREADS * SH_ITEMS)), (unsigned)N);
  if (ldtype == MX_F32) {
    sample_hist_kernel<float><<<grid, SH_THREADS, 0, st>>>((const float*)labels, valid, keys, L, ghist);
    sample_split_kernel<float><<<grid, SH_THREADS, 0, st>>>((const float*)labels, valid, keys, L, P, batch, ghist, lcount,
                                                            lists, pos, neg, sm);
  } else {
    sample_hist_kernel<int64_t><<<grid, SH_THREADS, 0, st>>>((const int64_t*)labels, valid, keys, L, ghist);
    sample_split_kernel<int64_t><<<grid, SH_THREADS, 0, st>>>((const int64_t*)labels, valid, keys, L, P, batch, ghist,
                                                              lcount, lists, pos, neg, sm);
  }
  sample_finish_kernel<<<(unsigned)N, SP_THREADS, 0, st>>>(L, P, batch, ghist, lcount, lists, pos, neg, sm, nums);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

// labels: ldtype MX_F32 (float, the RPN's 1 / 0 / -1) or 2 (int64, the RoI head's class / 0 / -1)
extern "C" int mx_sample_draw(const void* labels, int ldtype, const uint8_t* valid, const float* keys, int64_t N,
                              int64_t L, int batch, double positive_fraction, uint8_t* pos, uint8_t* neg, uint8_t* sm,
                              int32_t* nums, mx_stream_t stream) {
  MX_CHECK_ARG(N >= 0 && L >= 0 && batch >= 0, "sample_draw: negative size");
  // empty rows (L == 0) come with null row operands; the launch then only writes nums = (0, 0)
  MX_CHECK_ARG((N == 0 || nums) && (N * L == 0 || (labels && keys && pos && neg)), "sample_draw: null operand");
  MX_CHECK_ARG(ldtype == MX_F32 || ldtype == 2, "sample_draw: labels must be f32 (0) or int64 (2)");
  MX_CHECK_ARG(N < (1 << 30) && L < (1ll << 40), "sample_draw: too many rows");
  if (N == 0) return MX_OK;
  const int P = (int)(batch * positive_fraction);  // torchvision: int(batch_size_per_image * positive_fraction)
  hipStream_t st = (hipStream_t)stream;
  if (ldtype == MX_F32)
    sample_draw_kernel<float><<<(unsigned)N, SP_THREADS, 0, st>>>((const float*)labels, valid, keys, L, P, batch, pos,
                                                                 neg, sm, nums);
  else
    sample_draw_kernel<int64_t><<<(unsigned)N, SP_THREADS, 0, st>>>((const int64_t*)labels, valid, keys, L, P, batch, pos,
                                                                   neg, sm, nums);
  MX_LAUNCH_CHECK();
  return MX_OK;
}
