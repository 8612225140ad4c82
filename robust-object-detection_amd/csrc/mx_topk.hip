// mx_topk.hip — per-level objectness top-k of RegionProposalNetwork._get_top_n_idx, gfx950.
//
// torchvision 0.20.1 rpn.py _get_top_n_idx: for every feature level, ob[:, off:off+n].topk(min(pre, n))
// and the level offset added; the levels' index lists are concatenated. Here one launch covers every
// (level, image) pair: one 1024-thread workgroup each (grid = levels x images). Per workgroup:
//   1. radix select of the k-th largest value on order-preserving u32 keys, four 8-bit digit passes
//      (MSB first) with an LDS histogram; the first pass (sign + exponent bits, which cluster) counts
//      with wave-aggregated atomics (one LDS atomic per distinct digit per wave);
//   2. the k winners -- every key above the threshold T, then the keys equal to T in index order
//      (torch's gatherTopK tie rule) -- are gathered into LDS as (~key << 32 | index);
//   3. an LDS bitonic sort orders them by value descending, index ascending (sorted=True), and the
//      indices + level offset are written to out[image, level slot].
// Reads a level's scores 5 times (4 select passes + gather), the later passes from L2.
#include "mx_common.h"

namespace mx {

static constexpr int TK_THREADS = 1024, TK_MAXK = 4096, TK_MAXL = 8;

struct TopkLv {
  int64_t off[TK_MAXL], n[TK_MAXL], oofs[TK_MAXL];
  int k[TK_MAXL];
  int L;
  int64_t out_stride;
};

// order-preserving key; -0.0 and +0.0 share one key (they compare equal, so they tie)
__device__ __forceinline__ uint32_t ord_f32(float f) {
  uint32_t u = __float_as_uint(f);
  if (u == 0x80000000u) u = 0u;
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// wave-aggregated append: lanes with `take` get consecutive slots from *ctr; returns the slot
__device__ __forceinline__ int wave_append(bool take, uint32_t* ctr) {
  const uint64_t m = __ballot(take);
  if (!m) return -1;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((unsigned long long)m) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(ctr, (uint32_t)__popcll(m));
  base = __shfl(base, leader);
  const uint64_t below = lane ? (m & ((1ull << lane) - 1)) : 0ull;
  return take ? (int)(base + __popcll(below)) : -1;
}

__global__ void __launch_bounds__(TK_THREADS) level_topk_kernel(const float* __restrict__ sc, int64_t rs, TopkLv P,
                                                                int64_t* __restrict__ out) {
  __shared__ uint32_t hist[256];
  __shared__ uint64_t keys[TK_MAXK];
  __shared__ uint32_t s_digit, s_above, s_eq, s_cnt;
  __shared__ uint32_t wsum[TK_THREADS / 64];
  const int l = blockIdx.x, img = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t n = P.n[l];
  const int k = P.k[l];
  const float* x = sc + img * rs + P.off[l];
  int64_t* o = out + img * P.out_stride + P.oofs[l];
  if (k <= 0) return;

  // 1. radix select
  uint32_t prefix = 0, pmask = 0;
  uint32_t krem = (uint32_t)k;  // winners still to place at or below the current prefix
  uint32_t ceq = 0;
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    if (tid < 256) hist[tid] = 0;
    __syncthreads();
    for (int64_t i0 = 0; i0 < n; i0 += TK_THREADS) {
      const int64_t i = i0 + tid;
      const bool in = i < n;
      const uint32_t u = in ? ord_f32(x[i]) : 0u;
      const bool m = in && (u & pmask) == prefix;
      const uint32_t d = (u >> shift) & 255u;
      if (pass == 0) {
        bool pending = m;
        for (;;) {
          const uint64_t pm = __ballot(pending);
          if (!pm) break;
          const int leader = __ffsll((unsigned long long)pm) - 1;
          const uint32_t dl = (uint32_t)__shfl((int)d, leader);
          const uint64_t same = __ballot(pending && d == dl);
          if (lane == leader) atomicAdd(&hist[dl], (uint32_t)__popcll(same));
          if (pending && d == dl) pending = false;
        }
      } else if (m) {
        atomicAdd(&hist[d], 1u);
      }
    }
    __syncthreads();
    if (wid == 0) {
      // lane j owns bins 255-4j .. 252-4j (descending); inclusive scan of the lane sums
      uint32_t c[4], s = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) { c[q] = hist[255 - 4 * lane - q]; s += c[q]; }
      uint32_t inc = s;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t v = (uint32_t)__shfl_up((int)inc, off);
        if (lane >= off) inc += v;
      }
      const uint32_t exc = inc - s;
      const uint64_t hit = __ballot(inc >= krem);
      const int j = __ffsll((unsigned long long)hit) - 1;  // first lane crossing krem (exists: total >= krem)
      if (lane == j) {
        uint32_t acc = exc;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (acc + c[q] >= krem) {
            s_digit = 255 - 4 * lane - q;
            s_above = acc;
            s_eq = c[q];
            break;
          }
          acc += c[q];
        }
      }
    }
    __syncthreads();
    prefix |= s_digit << shift;
    pmask |= 255u << shift;
    krem -= s_above;
    ceq = s_eq;
    __syncthreads();
  }
  const uint32_t T = prefix;
  const uint32_t ngt = (uint32_t)k - krem;  // keys strictly above T
  const bool take_all_eq = ceq == krem;

  // 2. gather the winners
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  for (int64_t i0 = 0; i0 < n; i0 += TK_THREADS) {
    const int64_t i = i0 + tid;
    const uint32_t u = i < n ? ord_f32(x[i]) : 0u;
    const bool take = i < n && (u > T || (take_all_eq && u == T));
    const int pos = wave_append(take, &s_cnt);
    if (take) keys[pos] = ((uint64_t)(~u) << 32) | (uint64_t)(uint32_t)i;
  }
  if (!take_all_eq) {
    // ties at T: the first krem of them in index order, slots ngt.. (rare path)
    uint32_t taken = 0;
    for (int64_t i0 = 0; i0 < n && taken < krem; i0 += TK_THREADS) {
      const int64_t i = i0 + tid;
      const bool f = i < n && ord_f32(x[i]) == T;
      const uint64_t m = __ballot(f);
      if (lane == 0) wsum[wid] = (uint32_t)__popcll(m);
      __syncthreads();
      uint32_t before = 0, total = 0;
      for (int w = 0; w < TK_THREADS / 64; ++w) {
        before += w < wid ? wsum[w] : 0u;
        total += wsum[w];
      }
      const uint64_t below = lane ? (m & ((1ull << lane) - 1)) : 0ull;
      const uint32_t rank = taken + before + (uint32_t)__popcll(below);
      if (f && rank < krem) keys[ngt + rank] = ((uint64_t)(~T) << 32) | (uint64_t)(uint32_t)i;
      taken += total;
      __syncthreads();
    }
  }
  // 3. bitonic sort (ascending key = value descending, index ascending)
  int P2 = 1;
  while (P2 < k) P2 <<= 1;
  for (int i = k + tid; i < P2; i += TK_THREADS) keys[i] = ~0ull;
  for (int size = 2; size <= P2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int t = tid; t < (P2 >> 1); t += TK_THREADS) {
        const int i = 2 * t - (t & (stride - 1)), j = i + stride;
        const bool asc = (i & size) == 0;
        const uint64_t a = keys[i], b = keys[j];
        if ((a > b) == asc) { keys[i] = b; keys[j] = a; }
      }
    }
  }
  __syncthreads();
  for (int j = tid; j < k; j += TK_THREADS) o[j] = P.off[l] + (int64_t)(uint32_t)keys[j];
}

}  // namespace mx

using namespace mx;

extern "C" int mx_level_topk(const float* scores, int64_t N, int64_t row_stride, int nlev, const int64_t* level_off,
                             const int64_t* level_n, int64_t k, int64_t* out_idx, mx_stream_t stream) {
  MX_CHECK_ARG(nlev >= 1 && nlev <= TK_MAXL, "level_topk: 1..%d levels, got %d", TK_MAXL, nlev);
  MX_CHECK_ARG(k >= 0, "level_topk: k=%lld", (long long)k);
  MX_CHECK_ARG(N >= 0 && N <= 65535, "level_topk: N=%lld", (long long)N);
  TopkLv P{};
  int64_t tot = 0;
  for (int i = 0; i < nlev; ++i) {
    MX_CHECK_ARG(level_n[i] >= 0 && level_n[i] < (1ll << 31), "level_topk: level %d size %lld", i, (long long)level_n[i]);
    MX_CHECK_ARG(level_off[i] >= 0 && level_off[i] + level_n[i] <= row_stride, "level_topk: level %d out of the row", i);
    P.off[i] = level_off[i];
    P.n[i] = level_n[i];
    P.k[i] = (int)(k < level_n[i] ? k : level_n[i]);
    MX_CHECK_ARG(P.k[i] <= TK_MAXK, "level_topk: min(k, n)=%d above %d at level %d", P.k[i], TK_MAXK, i);
    P.oofs[i] = tot;
    tot += P.k[i];
  }
  P.L = nlev;
  P.out_stride = tot;
  if (N == 0 || tot == 0) return MX_OK;
  level_topk_kernel<<<dim3((unsigned)nlev, (unsigned)N), TK_THREADS, 0, (hipStream_t)stream>>>(scores, row_stride, P,
                                                                                               out_idx);
  MX_LAUNCH_CHECK();
  return MX_OK;
}
