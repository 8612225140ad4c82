// mx_topk.hip — per-level objectness top-k of RegionProposalNetwork._get_top_n_idx, gfx950.
//
// torchvision 0.20.1 rpn.py _get_top_n_idx: for every feature level, ob[:, off:off+n].topk(min(pre, n))
// and the level offset added; the levels' index lists are concatenated. Every (level, image) pair is
// one or more 1024-thread workgroups:
//   * a level of at most `slice` elements (or any level when no workspace is given) is finished by one
//     workgroup of level_topk_kernel;
//   * a longer level (the P2 level's 201,600 anchors at 1344x800) is cut into slices, each slice's own
//     top-k (a superset of its share of the level's top-k under the total order value desc / index
//     asc) is written to the workspace by level_topk_kernel, and level_topk_merge_kernel selects and
//     sorts the level's top-k from the slices' lists: the level is read by ~9 CUs instead of one.
// Per workgroup:
//   1. radix select of the k-th largest value on order-preserving u32 keys, three digit passes of
//      11/11/10 bits (MSB first) into LDS histograms (4 copies by wave group, summed by the scan: the
//      first digit -- sign, exponent, 2 mantissa bits -- clusters); 8 float4 loads in flight per thread;
//      After the first pass the elements whose first digit reaches the threshold digit (at most
//      TK_CAND of them, else the passes stay on global memory) are compacted into LDS, and the
//      remaining passes and the gather read only them;
//   2. the k winners -- every key above the threshold T, then the keys equal to T by lowest index
//      (torch's gatherTopK tie rule) -- are gathered into LDS as (~key << 32 | index);
//   3. a bitonic sort orders them by value descending, index ascending (sorted=True): strides below a
//      wave's share of the keys run in registers (shuffles, no barrier), the longer ones in LDS; the
//      indices + level offset are written to out[image, level slot].
#include "mx_common.h"

namespace mx {

static constexpr int TK_THREADS = 1024, TK_MAXK = 4096, TK_MAXL = 8, TK_UNROLL4 = 8, TK_HCOPIES = 4, TK_BINS = 2048,
                     TK_CAND = 8192, TK_WAVES = TK_THREADS / 64;
static constexpr int64_t TK_SLICE = 24576;  // elements per slice of a long level

struct TopkLv {
  int64_t off[TK_MAXL], n[TK_MAXL], oofs[TK_MAXL];
  int k[TK_MAXL];
  int nsl[TK_MAXL];   // slices of the level (1: finished by level_topk_kernel)
  int sl0[TK_MAXL];   // first slice id of the level
  int mlev[TK_MAXL];  // merge launch: block x -> level
  int L, ts;          // levels, slices over all levels
  int64_t slice;      // elements per slice
  int64_t out_stride;
  uint2* ws;          // [N][ts][TK_MAXK] (key, index in level) lists of the sliced levels' slices
  uint32_t* cnt;      // [N][ts] list lengths
};

struct TopkSmem {
  uint32_t hist[TK_HCOPIES * TK_BINS];  // per-wave-group copies: fewer same-address atomics
  uint64_t keys[TK_MAXK];
  uint2 cand[TK_CAND];                  // (key, index) of the first pass's survivors
  uint32_t s_digit, s_above, s_eq, s_cnt, s_ncand;
  uint32_t wsum[TK_WAVES];
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

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int s) {
  const int lo = __shfl_xor((int)(uint32_t)v, s), hi = __shfl_xor((int)(uint32_t)(v >> 32), s);
  return ((uint64_t)(uint32_t)hi << 32) | (uint64_t)(uint32_t)lo;
}

// compare-exchange of register pairs (e, e + ES): stride 64 * ES of merge size `size`
template <int E, int ES>
__device__ __forceinline__ void bitonic_pairs(uint64_t (&r)[E], int size, int base) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    if ((e & ES) || e + ES >= E) continue;
    const int i = base + e * 64 + lane;
    const bool asc = (i & size) == 0;
    const uint64_t a = r[e], b = r[e + ES];
    if ((a > b) == asc) { r[e] = b; r[e + ES] = a; }
  }
}

// Register phase of the bitonic network: strides s0, s0/2, ..., 1 of merge size `size`, on the keys
// this wave holds (lane l, register e = element w*C + 64e + l, C = 64E).
template <int E>
__device__ __forceinline__ void bitonic_regs(uint64_t (&r)[E], int size, int s0, int base) {
  const int lane = threadIdx.x & 63;
  for (int s = s0; s >= 1; s >>= 1) {
    if (s >= 128) {
      bitonic_pairs<E, 2>(r, size, base);
    } else if (s == 64) {
      bitonic_pairs<E, 1>(r, size, base);
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const uint64_t o = shfl_xor64(r[e], s);
        const int i = base + e * 64 + lane;
        const bool asc = (i & size) == 0, lower = (lane & s) == 0;
        const uint64_t mn = r[e] < o ? r[e] : o, mx = r[e] < o ? o : r[e];
        r[e] = (lower == asc) ? mn : mx;
      }
    }
  }
}

// bitonic sort of keys[0, P2) ascending, P2 = 64 * E * TK_WAVES; every thread of the block calls it
template <int E>
__device__ void bitonic_sort_regs(uint64_t* keys) {
  constexpr int C = 64 * E, P2 = C * TK_WAVES;
  const int tid = threadIdx.x, lane = tid & 63, base = (tid >> 6) * C;
  uint64_t r[E];
  __syncthreads();
#pragma unroll
  for (int e = 0; e < E; ++e) r[e] = keys[base + e * 64 + lane];
  for (int size = 2; size <= C; size <<= 1) bitonic_regs<E>(r, size, size >> 1, base);
#pragma unroll
  for (int e = 0; e < E; ++e) keys[base + e * 64 + lane] = r[e];
  for (int size = 2 * C; size <= P2; size <<= 1) {
    for (int stride = size >> 1; stride >= C; stride >>= 1) {
      __syncthreads();
      for (int t = tid; t < (P2 >> 1); t += TK_THREADS) {
        const int i = 2 * t - (t & (stride - 1)), j = i + stride;
        const bool asc = (i & size) == 0;
        const uint64_t a = keys[i], b = keys[j];
        if ((a > b) == asc) { keys[i] = b; keys[j] = a; }
      }
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; ++e) r[e] = keys[base + e * 64 + lane];
    bitonic_regs<E>(r, size, C >> 1, base);
#pragma unroll
    for (int e = 0; e < E; ++e) keys[base + e * 64 + lane] = r[e];
  }
  __syncthreads();
}

// ascending sort of keys[0, nsort) (padded with ~0 up to a power of two); ends with a barrier
__device__ void sort_keys(uint64_t* keys, int nsort) {
  const int tid = threadIdx.x;
  int P2 = 1;
  while (P2 < nsort) P2 <<= 1;
  if (P2 >= 1024) {
    const int P = P2 < 1024 ? 1024 : P2;  // 1024, 2048 or 4096: 1, 2 or 4 keys per lane
    for (int i = nsort + tid; i < P; i += TK_THREADS) keys[i] = ~0ull;
    if (P == 1024) bitonic_sort_regs<1>(keys);
    else if (P == 2048) bitonic_sort_regs<2>(keys);
    else bitonic_sort_regs<4>(keys);
    return;
  }
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
}

// The top-k of one element set. `gvisit(f)` calls f(valid, key, index) on every element from global
// memory (wave-uniform trip counts); x / n: the level's scores in index order (the rare many-ties
// path). Final: the sorted indices + ioff to o[0, k). Otherwise the winners (unsorted; every tie at
// the threshold when they fit, else the lowest-index ones) go to list[] and their count to *cnt.
template <class GVisit>
__device__ void topk_block(TopkSmem& sm, GVisit&& gvisit, const float* x, int64_t n, int k, bool final,
                           int64_t* o, int64_t ioff, uint2* list, uint32_t* cnt) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  bool use_lds = false;
  uint32_t ncand = 0;
  auto visit = [&](auto&& f) {
    if (use_lds) {
      for (uint32_t j0 = 0; j0 < ncand; j0 += TK_THREADS) {
        const uint32_t j = j0 + tid;
        const bool in = j < ncand;
        const uint2 c = in ? sm.cand[j] : make_uint2(0u, 0u);
        f(in, c.x, (int64_t)c.y);
      }
    } else {
      gvisit(f);
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
    for (int i = tid; i < TK_HCOPIES * TK_BINS; i += TK_THREADS) sm.hist[i] = 0;
    __syncthreads();
    uint32_t* hh = sm.hist + (wid & (TK_HCOPIES - 1)) * TK_BINS;
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
        for (int h = 0; h < TK_HCOPIES; ++h) sum += sm.hist[h * TK_BINS + bin];
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
          for (int h = 0; h < TK_HCOPIES; ++h) c += sm.hist[h * TK_BINS + bin];
          if (acc + c >= krem) {
            sm.s_digit = (uint32_t)bin;
            sm.s_above = acc;
            sm.s_eq = c;
            break;
          }
          acc += c;
        }
      }
    }
    __syncthreads();
    prefix |= sm.s_digit << shift;
    pmask |= dmask << shift;
    krem -= sm.s_above;
    ceq = sm.s_eq;
    __syncthreads();
    if (pass == 0 && (uint32_t)k - krem + ceq <= (uint32_t)TK_CAND) {
      // every later winner has a first digit >= the threshold digit: keep just those (key >= prefix)
      if (tid == 0) sm.s_ncand = 0;
      __syncthreads();
      visit([&](bool in, uint32_t u, int64_t i) {
        const bool take = in && u >= prefix;
        const int pos = wave_append(take, &sm.s_ncand);
        if (take) sm.cand[pos] = make_uint2(u, (uint32_t)i);
      });
      __syncthreads();
      ncand = sm.s_ncand;
      use_lds = true;
    }
  }
  const uint32_t T = prefix;
  const uint32_t ngt = (uint32_t)k - krem;  // keys strictly above T
  // every key tied at T fits the sort buffer: take them all and let the (value, index) sort keep
  // the lowest indices; otherwise place the first krem ties in index order (global, rare path)
  const bool all_ties = ngt + ceq <= (uint32_t)TK_MAXK;

  // 2. gather the winners (to LDS, or straight to the slice's list)
  if (tid == 0) sm.s_cnt = 0;
  __syncthreads();
  visit([&](bool in, uint32_t u, int64_t i) {
    const bool take = in && (u > T || (all_ties && u == T));
    const int pos = wave_append(take, &sm.s_cnt);
    if (take) {
      if (final) sm.keys[pos] = ((uint64_t)(~u) << 32) | (uint64_t)(uint32_t)i;
      else list[pos] = make_uint2(u, (uint32_t)i);
    }
  });
  if (!all_ties) {
    uint32_t taken = 0;
    for (int64_t i0 = 0; i0 < n && taken < krem; i0 += TK_THREADS) {
      const int64_t i = i0 + tid;
      const bool f = i < n && ord_f32(x[i]) == T;
      const uint64_t m = __ballot(f);
      if (lane == 0) sm.wsum[wid] = (uint32_t)__popcll(m);
      __syncthreads();
      uint32_t before = 0, total = 0;
      for (int w = 0; w < TK_WAVES; ++w) {
        before += w < wid ? sm.wsum[w] : 0u;
        total += sm.wsum[w];
      }
      const uint64_t below = lane ? (m & ((1ull << lane) - 1)) : 0ull;
      const uint32_t rank = taken + before + (uint32_t)__popcll(below);
      if (f && rank < krem) {
        if (final) sm.keys[ngt + rank] = ((uint64_t)(~T) << 32) | (uint64_t)(uint32_t)i;
        else list[ngt + rank] = make_uint2(T, (uint32_t)(i + ioff));
      }
      taken += total;
      __syncthreads();
    }
  }
  const int nout = all_ties ? (int)(ngt + ceq) : k;
  if (!final) {
    if (tid == 0) *cnt = (uint32_t)nout;
    return;
  }
  // 3. sort (ascending key = value descending, index ascending); the first k are the output
  __syncthreads();
  sort_keys(sm.keys, nout);
  for (int j = tid; j < k; j += TK_THREADS) o[j] = ioff + (int64_t)(uint32_t)sm.keys[j];
}

// block (slice id, image): a whole level (its only slice) or one slice of a long level
__global__ void __launch_bounds__(TK_THREADS) level_topk_kernel(const float* __restrict__ sc, int64_t rs, TopkLv P,
                                                                int64_t* __restrict__ out) {
  __shared__ TopkSmem sm;
  const int sid = blockIdx.x, img = blockIdx.y, tid = threadIdx.x;
  int l = 0;
  while (l + 1 < P.L && sid >= P.sl0[l + 1]) ++l;
  const int j = sid - P.sl0[l];
  const int64_t s0 = (int64_t)j * P.slice;
  const int64_t n = P.nsl[l] == 1 ? P.n[l] : min<int64_t>(P.slice, P.n[l] - s0);
  const int k = P.k[l];
  const bool final = P.nsl[l] == 1;
  const float* x = sc + img * rs + P.off[l] + s0;
  int64_t* o = out + img * P.out_stride + P.oofs[l];
  uint2* list = final ? nullptr : P.ws + ((int64_t)img * P.ts + sid) * TK_MAXK;
  uint32_t* cnt = final ? nullptr : P.cnt + (int64_t)img * P.ts + sid;
  if (k <= 0 || n <= 0) return;
  if (!final && n <= k) {  // the whole slice is a candidate list
    for (int64_t i = tid; i < n; i += TK_THREADS) list[i] = make_uint2(ord_f32(x[i]), (uint32_t)(s0 + i));
    if (tid == 0) *cnt = (uint32_t)n;
    return;
  }
  // scalar head up to the first 16-B boundary, float4 body (TK_UNROLL4 loads in flight per thread),
  // scalar tail; indices are the level's (slice offset s0 added)
  auto gvisit = [&](auto&& f) {
    const int64_t h = min<int64_t>((int64_t)((16 - ((uintptr_t)x & 15)) & 15) >> 2, n);
    f(tid < h, tid < h ? ord_f32(x[tid]) : 0u, s0 + tid);
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
        const int64_t i = s0 + h + 4 * q;
        f(in, ord_f32(xv[r].x), i);
        f(in, ord_f32(xv[r].y), i + 1);
        f(in, ord_f32(xv[r].z), i + 2);
        f(in, ord_f32(xv[r].w), i + 3);
      }
    }
    const int64_t t0 = h + 4 * nb4;
    f(t0 + tid < n, t0 + tid < n ? ord_f32(x[t0 + tid]) : 0u, s0 + t0 + tid);
  };
  topk_block(sm, gvisit, x, n, k, final, o, final ? P.off[l] : s0, list, cnt);
}

// block (sliced level, image): the level's top-k from its slices' candidate lists
__global__ void __launch_bounds__(TK_THREADS) level_topk_merge_kernel(const float* __restrict__ sc, int64_t rs,
                                                                      TopkLv P, int64_t* __restrict__ out) {
  __shared__ TopkSmem sm;
  const int l = P.mlev[blockIdx.x], img = blockIdx.y, tid = threadIdx.x;
  const int k = P.k[l];
  const float* x = sc + img * rs + P.off[l];
  int64_t* o = out + img * P.out_stride + P.oofs[l];
  const uint2* lists = P.ws + ((int64_t)img * P.ts + P.sl0[l]) * TK_MAXK;
  const uint32_t* cnts = P.cnt + (int64_t)img * P.ts + P.sl0[l];
  const int nsl = P.nsl[l];
  auto gvisit = [&](auto&& f) {
    for (int s = 0; s < nsl; ++s) {
      const uint32_t c = cnts[s];
      const uint2* li = lists + (int64_t)s * TK_MAXK;
      for (uint32_t j0 = 0; j0 < c; j0 += TK_THREADS) {
        const uint32_t j = j0 + tid;
        const bool in = j < c;
        const uint2 v = in ? li[j] : make_uint2(0u, 0u);
        f(in, v.x, (int64_t)v.y);
      }
    }
  };
  topk_block(sm, gvisit, x, P.n[l], k, true, o, P.off[l], nullptr, nullptr);
}

static int topk_plan(TopkLv& P, int nlev, const int64_t* level_off, const int64_t* level_n, int64_t k, int64_t slice,
                     int64_t row_stride) {
  P = TopkLv{};
  int64_t tot = 0;
  int ts = 0, nm = 0;
  for (int i = 0; i < nlev; ++i) {
    MX_CHECK_ARG(level_n[i] >= 0 && level_n[i] < (1ll << 31), "level_topk: level %d size %lld", i, (long long)level_n[i]);
    MX_CHECK_ARG(level_off[i] >= 0 && level_off[i] + level_n[i] <= row_stride, "level_topk: level %d out of the row", i);
    P.off[i] = level_off[i];
    P.n[i] = level_n[i];
    P.k[i] = (int)(k < level_n[i] ? k : level_n[i]);
    MX_CHECK_ARG(P.k[i] <= TK_MAXK, "level_topk: min(k, n)=%d above %d at level %d", P.k[i], TK_MAXK, i);
    P.oofs[i] = tot;
    tot += P.k[i];
    const int64_t ns = slice > 0 && level_n[i] > slice ? (level_n[i] + slice - 1) / slice : 1;
    P.nsl[i] = (int)ns;
    P.sl0[i] = ts;
    ts += (int)ns;
    if (ns > 1) P.mlev[nm++] = i;
  }
  P.L = nlev;
  P.ts = ts;
  P.slice = slice;
  P.out_stride = tot;
  return nm;
}

}  // namespace mx

using namespace mx;

extern "C" size_t mx_level_topk_workspace(int64_t N, int nlev, const int64_t* level_n) {
  if (N <= 0 || nlev < 1 || nlev > TK_MAXL || !level_n) return 0;
  int64_t ts = 0;
  bool sliced = false;
  for (int i = 0; i < nlev; ++i) {
    const int64_t ns = level_n[i] > TK_SLICE ? (level_n[i] + TK_SLICE - 1) / TK_SLICE : 1;
    sliced |= ns > 1;
    ts += ns;
  }
  if (!sliced) return 0;
  return (size_t)N * ts * (TK_MAXK * sizeof(uint2) + sizeof(uint32_t));
}

extern "C" int mx_level_topk_ws(const float* scores, int64_t N, int64_t row_stride, int nlev, const int64_t* level_off,
                                const int64_t* level_n, int64_t k, int64_t* out_idx, void* ws, size_t ws_bytes,
                                mx_stream_t stream) {
  MX_CHECK_ARG(nlev >= 1 && nlev <= TK_MAXL, "level_topk: 1..%d levels, got %d", TK_MAXL, nlev);
  MX_CHECK_ARG(k >= 0, "level_topk: k=%lld", (long long)k);
  MX_CHECK_ARG(N >= 0 && N <= 65535, "level_topk: N=%lld", (long long)N);
  const size_t need = N > 0 ? mx_level_topk_workspace(N, nlev, level_n) : 0;
  const bool sliced = ws != nullptr && need > 0;
  MX_CHECK_ARG(!sliced || ws_bytes >= need, "level_topk: workspace of %zu bytes required (mx_level_topk_workspace)",
               need);
  TopkLv P;
  const int nm = topk_plan(P, nlev, level_off, level_n, k, sliced ? TK_SLICE : 0, row_stride);
  if (nm < 0) return MX_EINVAL;
  if (N == 0 || P.out_stride == 0) return MX_OK;
  if (sliced) {
    P.ws = (uint2*)ws;
    P.cnt = (uint32_t*)((char*)ws + (size_t)N * P.ts * TK_MAXK * sizeof(uint2));
  }
  hipStream_t st = (hipStream_t)stream;
  level_topk_kernel<<<dim3((unsigned)P.ts, (unsigned)N), TK_THREADS, 0, st>>>(scores, row_stride, P, out_idx);
  MX_LAUNCH_CHECK();
  if (nm > 0) {
    level_topk_merge_kernel<<<dim3((unsigned)nm, (unsigned)N), TK_THREADS, 0, st>>>(scores, row_stride, P, out_idx);
    MX_LAUNCH_CHECK();
  }
  return MX_OK;
}

extern "C" int mx_level_topk(const float* scores, int64_t N, int64_t row_stride, int nlev, const int64_t* level_off,
                             const int64_t* level_n, int64_t k, int64_t* out_idx, mx_stream_t stream) {
  return mx_level_topk_ws(scores, N, row_stride, nlev, level_off, level_n, k, out_idx, nullptr, 0, stream);
}
