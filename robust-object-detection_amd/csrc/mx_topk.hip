// mx_topk.hip — per-level objectness top-k of RegionProposalNetwork._get_top_n_idx, gfx950.
//
// torchvision 0.20.1 rpn.py _get_top_n_idx: for every feature level, ob[:, off:off+n].topk(min(pre, n))
// and the level offset added; the levels' index lists are concatenated. Here one launch covers every
// (level, image) pair: one 1024-thread workgroup each (grid = levels x images). Per workgroup:
//   1. radix select of the k-th largest value on order-preserving u32 keys, three digit passes of
//      11/11/10 bits (MSB first) into LDS histograms (4 copies by wave group, summed by the scan: the
//      first digit -- sign, exponent, 2 mantissa bits -- clusters); 8 float4 loads in flight per thread;
//      After the first pass the elements whose first digit reaches the threshold digit (at most
//      TK_CAND of them, else the passes stay on global memory) are compacted into LDS, and the
//      remaining passes and the gather read only them;
//   2. the k winners -- every key above the threshold T, then the keys equal to T by lowest index
//      (torch's gatherTopK tie rule) -- are gathered into LDS as (~key << 32 | index);
//   3. an LDS bitonic sort orders them by value descending, index ascending (sorted=True), and the
//      indices + level offset are written to out[image, level slot].
// Reads a level's scores twice from global memory (first pass + compaction) in the common case.
#include "mx_common.h"

namespace mx {

static constexpr int TK_THREADS = 1024, TK_MAXK = 4096, TK_MAXL = 8, TK_UNROLL4 = 8, TK_HCOPIES = 4, TK_BINS = 2048,
                     TK_CAND = 8192;

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
  __shared__ uint32_t hist[TK_HCOPIES * TK_BINS];  // per-wave-group copies: fewer same-address atomics
  __shared__ uint64_t keys[TK_MAXK];
  __shared__ uint2 cand[TK_CAND];                  // (key, index) of the first pass's survivors
  __shared__ uint32_t s_digit, s_above, s_eq, s_cnt, s_ncand;
  __shared__ uint32_t wsum[TK_THREADS / 64];
  const int l = blockIdx.x, img = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t n = P.n[l];
  const int k = P.k[l];
  const float* x = sc + img * rs + P.off[l];
  int64_t* o = out + img * P.out_stride + P.oofs[l];
  if (k <= 0) return;

  // visits every element (valid flag, key, index) of the level -- from global memory (8 float4
  // loads in flight per thread) or, once compacted, from the LDS candidate list; wave-uniform trip counts
  bool use_lds = false;
  uint32_t ncand = 0;
  auto visit = [&](auto&& f) {
    if (use_lds) {
      for (uint32_t j0 = 0; j0 < ncand; j0 += TK_THREADS) {
        const uint32_t j = j0 + tid;
        const bool in = j < ncand;
        const uint2 c = in ? cand[j] : make_uint2(0u, 0u);
        f(in, c.x, (int64_t)c.y);
      }
    } else {
      // scalar head up to the first 16-B boundary, float4 body (TK_UNROLL4 loads in flight per
      // thread), scalar tail
      const int64_t h = min<int64_t>((int64_t)((16 - ((uintptr_t)x & 15)) & 15) >> 2, n);
      f(tid < h, tid < h ? ord_f32(x[tid]) : 0u, (int64_t)tid);
      const int64_t nb4 = (n - h) >> 2;
      const float4* x4 = (const float4*)(x + h);
      for (int64_t q0 = 0; q0 < nb4; q0 += TK_THREADS * TK_UNROLL4) {
        float4 xv[TK_UNROLL4];
#pragma unroll
        for (int r = 0; r < TK_UNROLL4; ++r) {
          const int64_t q = q0 + r * TK_THREADS + tid;
          xv[r] = q < nb4 ? x4[q] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int r = 0; r < TK_UNROLL4; ++r) {
          const int64_t q = q0 + r * TK_THREADS + tid;
          const bool in = q < nb4;
          const int64_t i = h + 4 * q;
          f(in, ord_f32(xv[r].x), i);
          f(in, ord_f32(xv[r].y), i + 1);
          f(in, ord_f32(xv[r].z), i + 2);
          f(in, ord_f32(xv[r].w), i + 3);
        }
      }
      const int64_t t0 = h + 4 * nb4;
      f(t0 + tid < n, t0 + tid < n ? ord_f32(x[t0 + tid]) : 0u, t0 + tid);
    }
  };

  // 1. radix select: digits of 11, 11 and 10 bits, most significant first
  uint32_t prefix = 0, pmask = 0;
  uint32_t krem = (uint32_t)k;  // winners still to place at or below the current prefix
  uint32_t ceq = 0;
  for (int pass = 0; pass < 3; ++pass) {
    const int nbits = pass < 2 ? 11 : 10, shift = pass < 2 ? 21 - 11 * pass : 0;
    const int NB = 1 << nbits, per = NB / 64;
    const uint32_t dmask = (uint32_t)NB - 1;
    for (int i = tid; i < TK_HCOPIES * TK_BINS; i += TK_THREADS) hist[i] = 0;
    __syncthreads();
    uint32_t* hh = hist + (wid & (TK_HCOPIES - 1)) * TK_BINS;
    visit([&](bool in, uint32_t u, int64_t) {
      if (in && (u & pmask) == prefix) atomicAdd(&hh[(u >> shift) & dmask], 1u);
    });
    __syncthreads();
    if (wid == 0) {
      // lane j owns bins NB-1-per*j .. NB-per*(j+1) (descending); inclusive scan of the lane sums
      uint32_t sum = 0;
      for (int q = 0; q < per; ++q) {
        const int bin = NB - 1 - per * lane - q;
#pragma unroll
        for (int h = 0; h < TK_HCOPIES; ++h) sum += hist[h * TK_BINS + bin];
      }
      uint32_t inc = sum;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t v = (uint32_t)__shfl_up((int)inc, off);
        if (lane >= off) inc += v;
      }
      const uint64_t hit = __ballot(inc >= krem);
      const int j = __ffsll((unsigned long long)hit) - 1;  // first lane crossing krem (exists: total >= krem)
      if (lane == j) {
        uint32_t acc = inc - sum;
        for (int q = 0; q < per; ++q) {
          const int bin = NB - 1 - per * lane - q;
          uint32_t c = 0;
#pragma unroll
          for (int h = 0; h < TK_HCOPIES; ++h) c += hist[h * TK_BINS + bin];
          if (acc + c >= krem) {
            s_digit = (uint32_t)bin;
            s_above = acc;
            s_eq = c;
            break;
          }
          acc += c;
        }
      }
    }
    __syncthreads();
    prefix |= s_digit << shift;
    pmask |= dmask << shift;
    krem -= s_above;
    ceq = s_eq;
    __syncthreads();
    if (pass == 0 && (uint32_t)k - krem + ceq <= (uint32_t)TK_CAND) {
      // every later winner has a first digit >= the threshold digit: keep just those (key >= prefix)
      if (tid == 0) s_ncand = 0;
      __syncthreads();
      visit([&](bool in, uint32_t u, int64_t i) {
        const bool take = in && u >= prefix;
        const int pos = wave_append(take, &s_ncand);
        if (take) cand[pos] = make_uint2(u, (uint32_t)i);
      });
      __syncthreads();
      ncand = s_ncand;
      use_lds = true;
    }
  }
  const uint32_t T = prefix;
  const uint32_t ngt = (uint32_t)k - krem;  // keys strictly above T
  // every key tied at T fits the sort buffer: take them all and let the (value, index) sort keep
  // the lowest indices; otherwise place the first krem ties in index order (global, rare path)
  const bool all_ties = ngt + ceq <= (uint32_t)TK_MAXK;

  // 2. gather the winners
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  visit([&](bool in, uint32_t u, int64_t i) {
    const bool take = in && (u > T || (all_ties && u == T));
    const int pos = wave_append(take, &s_cnt);
    if (take) keys[pos] = ((uint64_t)(~u) << 32) | (uint64_t)(uint32_t)i;
  });
  if (!all_ties) {
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
  // 3. bitonic sort (ascending key = value descending, index ascending); the first k are the output
  const int nsort = all_ties ? (int)(ngt + ceq) : k;
  int P2 = 1;
  while (P2 < nsort) P2 <<= 1;
  for (int i = nsort + tid; i < P2; i += TK_THREADS) keys[i] = ~0ull;
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
