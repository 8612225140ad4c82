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

static constexpr int SP_THREADS = 1024, SP_BINS = 2048, SP_COPIES = 4, SP_WAVES = SP_THREADS / 64, SP_UNROLL = 8;

__device__ __forceinline__ uint32_t sp_ord(float f) {  // order-preserving; -0.0 and +0.0 tie
  uint32_t u = __float_as_uint(f);
  if (u == 0x80000000u) u = 0u;
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

template <typename LT>
__device__ __forceinline__ int sp_class(LT v) {  // 0 positive, 1 negative, -1 neither
  if constexpr (sizeof(LT) == 4) {
    const float f = (float)v;
    return f >= 1.f ? 0 : (f == 0.f ? 1 : -1);
  } else {
    return v >= 1 ? 0 : (v == 0 ? 1 : -1);
  }
}

template <typename LT>
__global__ void __launch_bounds__(SP_THREADS) sample_draw_kernel(const LT* __restrict__ lab, const float* __restrict__ keys,
                                                                int64_t L, int P, int B, uint8_t* __restrict__ pos,
                                                                uint8_t* __restrict__ neg, uint8_t* __restrict__ sm,
                                                                int32_t* __restrict__ nums) {
  __shared__ uint32_t hist[2][SP_COPIES][SP_BINS];
  __shared__ uint32_t s_prefix[2], s_need[2], s_eq[2], s_k[2], s_cnt[2];
  __shared__ uint32_t s_wave[2][SP_WAVES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, copy = wave & (SP_COPIES - 1);
  const int64_t row = blockIdx.x;
  const LT* lr = lab + row * L;
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
        cl[u] = i < L ? sp_class<LT>(lr[i]) : -1;
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
        cl[u] = i < L ? sp_class<LT>(lr[i]) : -1;
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
      c = sp_class<LT>(lr[i]);
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

}  // namespace mx

using namespace mx;

// labels: ldtype MX_F32 (float, the RPN's 1 / 0 / -1) or 2 (int64, the RoI head's class / 0 / -1)
extern "C" int mx_sample_draw(const void* labels, int ldtype, const float* keys, int64_t N, int64_t L, int batch,
                              double positive_fraction, uint8_t* pos, uint8_t* neg, uint8_t* sm, int32_t* nums,
                              mx_stream_t stream) {
  MX_CHECK_ARG(N >= 0 && L >= 0 && batch >= 0, "sample_draw: negative size");
  // empty rows (L == 0) come with null row operands; the launch then only writes nums = (0, 0)
  MX_CHECK_ARG((N == 0 || nums) && (N * L == 0 || (labels && keys && pos && neg)), "sample_draw: null operand");
  MX_CHECK_ARG(ldtype == MX_F32 || ldtype == 2, "sample_draw: labels must be f32 (0) or int64 (2)");
  MX_CHECK_ARG(N < (1 << 30) && L < (1ll << 40), "sample_draw: too many rows");
  if (N == 0) return MX_OK;
  const int P = (int)(batch * positive_fraction);  // torchvision: int(batch_size_per_image * positive_fraction)
  hipStream_t st = (hipStream_t)stream;
  if (ldtype == MX_F32)
    sample_draw_kernel<float><<<(unsigned)N, SP_THREADS, 0, st>>>((const float*)labels, keys, L, P, batch, pos, neg, sm,
                                                                 nums);
  else
    sample_draw_kernel<int64_t><<<(unsigned)N, SP_THREADS, 0, st>>>((const int64_t*)labels, keys, L, P, batch, pos, neg,
                                                                   sm, nums);
  MX_LAUNCH_CHECK();
  return MX_OK;
}
