// mx_nms.hip — torchvision nms / batched_nms with CPU semantics, segmented, on gfx950.
//
// Restates torchvision 0.20.1 (oracle/mx_oracle.c orc_nms / orc_batched_nms):
//   nms: stable score-descending order; keep i unless suppressed; suppress j (later) when
//        inter/((area_i + area_j) - inter) > thr (f32 IoU compared in double).
//   batched_nms: CPU rule 4n > 4000 -> per-class ("vanilla"), else coordinate trick
//        boxes + idx*(max(boxes) + 1); result ordered by score descending.
// Serves RegionProposalNetwork.filter_proposals (batched over levels) and
// RoIHeads.postprocess_detections (batched over labels), reached from train_frcnn_baseline.py:171
// and eval_all.py:111.
//
// Design: one radix sort by (class, score desc, index) makes every class a contiguous segment;
// a 64x64 bitmask tile kernel (one lane per row, 64 columns per tile) fills only tiles inside a
// segment; one wave per segment then resolves the suppression scan 64 rows at a time: the
// in-tile dependency chain runs on the diagonal word in registers (v_readlane per step), the
// survivors' rows are OR-ed into the LDS "removed" bitmap lane-parallel over words. A second
// stable radix sort orders survivors by (group, score desc, index).
#include <hipcub/hipcub.hpp>

#include "mx_common.h"
#include "mx_dma.h"

namespace mx {

__device__ __forceinline__ uint32_t ord_f32(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ uint32_t ord_i32(int64_t v) { return ((uint32_t)(int32_t)v) ^ 0x80000000u; }

__global__ void nms_max_kernel(const float* __restrict__ b, int64_t n4, uint32_t* __restrict__ out) {
  uint32_t m = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x)
    m = max(m, ord_f32(b[i]));
  for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
  if ((threadIdx.x & 63) == 0) atomicMax(out, m);
}

__device__ __forceinline__ float unord_f32(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// keys for the segment sort; offset boxes for the coordinate trick
__global__ void nms_keys_kernel(const float4* __restrict__ boxes, const float* __restrict__ scores,
                                const int64_t* __restrict__ idxs, int64_t n, int trick, const uint32_t* __restrict__ maxbits,
                                uint64_t* __restrict__ keys, int32_t* __restrict__ vals, float4* __restrict__ obox,
                                int32_t* __restrict__ flags, int32_t* __restrict__ nk) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  flags[i] = 0;  // keep flags / keep count for the scan (no separate memsets)
  if (i == 0) *nk = 0;
  float4 b = boxes[i];
  uint32_t hi = 0;
  if (trick) {
    float step = unord_f32(*maxbits) + 1.0f;
    float off = (float)idxs[i] * step;  // idxs.to(boxes) * (max_coordinate + 1)
    b.x = b.x + off; b.y = b.y + off; b.z = b.z + off; b.w = b.w + off;
  } else if (idxs) {
    hi = ord_i32(idxs[i]);
  }
  obox[i] = b;
  keys[i] = ((uint64_t)hi << 32) | (uint64_t)(~ord_f32(scores[i]));
  vals[i] = (int32_t)i;
}

// gather sorted boxes, areas and segment heads
__global__ void nms_gather_kernel(const uint64_t* __restrict__ skeys, const int32_t* __restrict__ svals,
                                  const float4* __restrict__ obox, int64_t n, float4* __restrict__ sbox,
                                  float* __restrict__ sarea, int32_t* __restrict__ head) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float4 b = obox[svals[i]];
  sbox[i] = b;
  sarea[i] = (b.z - b.x) * (b.w - b.y);
  head[i] = (i == 0 || (skeys[i] >> 32) != (skeys[i - 1] >> 32)) ? 1 : 0;
}

// seg_id = inclusive_sum(head) - 1 ; seg_start[seg] = i for heads; nseg = seg_id[n-1]+1
__global__ void nms_seg_kernel(const int32_t* __restrict__ head, const int32_t* __restrict__ incl, int64_t n,
                               int32_t* __restrict__ seg_start, int32_t* __restrict__ nseg) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (head[i]) seg_start[incl[i] - 1] = (int32_t)i;
  if (i == n - 1) {
    *nseg = incl[i];
    seg_start[incl[i]] = (int32_t)n;
  }
}

// one 64-thread block per (64-row block, 64-column tile relative to the row's segment start). The
// column tile of the block's first row's segment is staged in LDS once (one coalesced load per lane);
// rows of another segment (a block straddling a segment start) read their columns from global.
// colm (optional): for the row's own 64-box block of its segment, the column form of the diagonal
// tile -- bit j - c0 set when an EARLIER box j of the block overlaps box i (the same IoU value as
// row j's bit for i: fmaxf / fminf and the area sum are symmetric in the pair)
__global__ void __launch_bounds__(64) nms_mask_kernel(const float4* __restrict__ sbox, const float* __restrict__ sarea,
                                                      const int32_t* __restrict__ incl, const int32_t* __restrict__ seg_start,
                                                      int64_t n, int Wm, double thr, uint64_t* __restrict__ mask,
                                                      uint64_t* __restrict__ colm) {
  __shared__ float4 tbox[64];
  __shared__ float tarea[64];
  const int tid = threadIdx.x, cb = blockIdx.y;
  const int64_t i0 = (int64_t)blockIdx.x * 64, i = i0 + tid;
  if (i0 >= n) return;  // whole block
  const int sid0 = incl[i0] - 1;
  const int64_t t0 = seg_start[sid0] + (int64_t)cb * 64, t1 = min<int64_t>(t0 + 64, seg_start[sid0 + 1]);
  if (t0 + tid < t1) {
    tbox[tid] = sbox[t0 + tid];
    tarea[tid] = sarea[t0 + tid];
  }
  __syncthreads();
  if (i >= n) return;
  const int sid = incl[i] - 1;
  const int64_t s0 = seg_start[sid], s1 = seg_start[sid + 1];
  const int64_t c0 = s0 + (int64_t)cb * 64;
  if (c0 >= s1) return;
  const bool staged = sid == sid0;
  const bool diag = colm && cb == (int)((i - s0) >> 6);
  const float4 bi = sbox[i];
  const float ai = sarea[i];
  uint64_t bits = 0, lo = 0;
  const int jn = (int)(min<int64_t>(c0 + 64, s1) - c0);
  const int jstart = diag ? 0 : (int)min<int64_t>(64, max<int64_t>(0, i + 1 - c0));
  for (int jj = jstart; jj < jn; ++jj) {
    const int64_t j = c0 + jj;
    if (j == i) continue;
    const float4 bj = staged ? tbox[jj] : sbox[j];
    const float aj = staged ? tarea[jj] : sarea[j];
    float xx1 = fmaxf(bi.x, bj.x), yy1 = fmaxf(bi.y, bj.y);
    float xx2 = fminf(bi.z, bj.z), yy2 = fminf(bi.w, bj.w);
    float w = fmaxf(0.f, xx2 - xx1), h = fmaxf(0.f, yy2 - yy1);
    float inter = w * h;
    float ovr = inter / ((ai + aj) - inter);
    if ((double)ovr > thr) {
      if (j > i) bits |= 1ull << jj;
      else lo |= 1ull << jj;
    }
  }
  mask[i * Wm + cb] = bits;
  if (diag) colm[i] = lo;
}

// one wave per segment: greedy scan, 64 rows per step
__global__ void __launch_bounds__(64) nms_scan_kernel(const uint64_t* __restrict__ mask, const int32_t* __restrict__ seg_start,
                                                      const int32_t* __restrict__ nseg_p, const int32_t* __restrict__ svals,
                                                      int Wm, int32_t* __restrict__ flags, int32_t* __restrict__ nkeep) {
  extern __shared__ uint64_t removed[];
  const int lane = threadIdx.x;
  const int nseg = *nseg_p;
  for (int seg = blockIdx.x; seg < nseg; seg += gridDim.x) {
    const int64_t s0 = seg_start[seg], len = seg_start[seg + 1] - s0;
    const int W = (int)((len + 63) / 64);
    if (W > Wm) {  // caller's max_seg bound was violated: report, never read past the mask rows
      if (lane == 0) atomicExch(nkeep, (int32_t)0x80000000);
      continue;
    }
    for (int w = lane; w < W; w += 64) removed[w] = 0;
    __syncthreads();
    int kept_total = 0;
    for (int blk = 0; blk < W; ++blk) {
      const int64_t rbase = s0 + (int64_t)blk * 64;
      const int cnt = (int)min<int64_t>(64, len - (int64_t)blk * 64);
      const uint64_t diag = lane < cnt ? mask[(rbase + lane) * Wm + blk] : 0ull;
      uint64_t cur = removed[blk];
      uint64_t kept = 0;
      const uint32_t dlo = (uint32_t)diag, dhi = (uint32_t)(diag >> 32);
      for (int t = 0; t < cnt; ++t) {
        if (!((cur >> t) & 1ull)) {
          kept |= 1ull << t;
          uint64_t row = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)dhi, t) << 32) |
                         (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)dlo, t);
          cur |= row;
        }
      }
      if (lane < cnt && ((kept >> lane) & 1ull)) flags[svals[rbase + lane]] = 1;
      kept_total += __popcll(kept);
      __syncthreads();
      for (int w = blk + 1 + lane; w < W; w += 64) {
        uint64_t acc = removed[w];
        uint64_t k = kept;
        while (k) {
          int t = __ffsll((unsigned long long)k) - 1;
          k &= k - 1;
          acc |= mask[(rbase + t) * Wm + w];
        }
        removed[w] = acc;
      }
      __syncthreads();
    }
    if (lane == 0 && kept_total) atomicAdd(nkeep, kept_total);
    __syncthreads();
  }
}

// LDS-staged scan (segments of up to 64*SCAN_LDS_W boxes): one 256-thread block per segment. Per
// 64-row block, all threads stage the block's mask rows (words blk..W-1, coalesced) in LDS in one
// round trip; wave 0 resolves the in-tile chain on the diagonal word; then all threads OR the kept
// rows into the removed bitmap from LDS. Same result as nms_scan_kernel (kept = the greedy set).
static constexpr int SCAN_LDS_W = 112;  // (Wm + 64 Wm) * 8 B <= 64 KB of dynamic LDS
__global__ void __launch_bounds__(256) nms_scan_lds_kernel(const uint64_t* __restrict__ mask,
                                                           const int32_t* __restrict__ seg_start,
                                                           const int32_t* __restrict__ nseg_p,
                                                           const int32_t* __restrict__ svals, int Wm,
                                                           int32_t* __restrict__ flags, int32_t* __restrict__ nkeep) {
  extern __shared__ uint64_t sm[];
  uint64_t* removed = sm;             // [Wm]
  uint64_t* rows = sm + Wm;           // [64][Wm]: row t, word w at rows[t * Wm + w]
  __shared__ uint64_t kept_s;
  const int tid = threadIdx.x, lane = tid & 63;
  const int nseg = *nseg_p;
  for (int seg = blockIdx.x; seg < nseg; seg += gridDim.x) {
    const int64_t s0 = seg_start[seg], len = seg_start[seg + 1] - s0;
    const int W = (int)((len + 63) / 64);
    if (W > Wm) {
      if (tid == 0) atomicExch(nkeep, (int32_t)0x80000000);
      continue;
    }
    for (int w = tid; w < W; w += 256) removed[w] = 0;
    int kept_total = 0;
    // the next 64-row block's mask words are loaded into registers while this block is resolved
    // (when they fit: <= 8 words per thread), hiding the global-load latency of each step
    constexpr int PF = 8;
    uint64_t pre[PF];
    auto fetch = [&](int b) {
      const int64_t rb = s0 + (int64_t)b * 64;
      const int c = (int)min<int64_t>(64, len - (int64_t)b * 64), nw_ = W - b;
#pragma unroll
      for (int i = 0; i < PF; ++i) {
        const int e = tid + i * 256;
        if (e < c * nw_) {
          const int t = e / nw_, w = b + (e - t * nw_);
          pre[i] = mask[(rb + t) * Wm + w];
        }
      }
    };
    auto fits = [&](int b) { return b < W && (int)min<int64_t>(64, len - (int64_t)b * 64) * (W - b) <= PF * 256; };
    if (fits(0)) fetch(0);
    for (int blk = 0; blk < W; ++blk) {
      const int64_t rbase = s0 + (int64_t)blk * 64;
      const int cnt = (int)min<int64_t>(64, len - (int64_t)blk * 64);
      const int nw = W - blk;  // words blk..W-1
      if (fits(blk)) {
#pragma unroll
        for (int i = 0; i < PF; ++i) {
          const int e = tid + i * 256;
          if (e < cnt * nw) {
            const int t = e / nw, w = blk + (e - t * nw);
            rows[t * Wm + w] = pre[i];
          }
        }
      } else {
        for (int e = tid; e < cnt * nw; e += 256) {
          const int t = e / nw, w = blk + (e - t * nw);
          rows[t * Wm + w] = mask[(rbase + t) * Wm + w];
        }
      }
      __syncthreads();
      if (fits(blk + 1)) fetch(blk + 1);
      if (tid < 64) {
        const uint64_t diag = lane < cnt ? rows[lane * Wm + blk] : 0ull;
        const uint64_t rm = removed[blk];
        // wave-uniform scalar walk over the not-yet-suppressed boxes only (s_ff1 jumps to the next
        // survivor; suppressed ones cost nothing): same greedy result as testing all cnt bits
        const uint64_t valid = cnt >= 64 ? ~0ull : ((1ull << cnt) - 1);
        uint64_t cur = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(rm >> 32)) << 32) |
                       (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)rm);
        uint64_t kept = 0;
        const uint32_t dlo = (uint32_t)diag, dhi = (uint32_t)(diag >> 32);
        uint64_t avail = ~cur & valid;
        while (avail) {
          const int t = __builtin_ctzll(avail);
          kept |= 1ull << t;
          const uint64_t row = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)dhi, t) << 32) |
                               (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)dlo, t);
          cur |= row;
          avail = ~cur & valid & ~((2ull << t) - 1ull);  // bits above t (t = 63: none)
        }
        if (lane < cnt && ((kept >> lane) & 1ull)) flags[svals[rbase + lane]] = 1;
        if (lane == 0) kept_s = kept;
      }
      __syncthreads();
      const uint64_t kept = kept_s;
      if (tid == 0) kept_total += __popcll(kept);
      // OR the kept rows into `removed`: (word, 1/8 of the kept rows) per thread, combined with LDS
      // atomic ORs -- 8x shorter dependent LDS-read chains than one thread per word
      for (int e = tid; e < (W - blk - 1) * 8; e += 256) {
        const int w = blk + 1 + (e >> 3), part = e & 7;
        uint64_t k = kept & (0x0101010101010101ull << part);
        uint64_t acc = 0;
        while (k) {
          const int t = __ffsll((unsigned long long)k) - 1;
          k &= k - 1;
          acc |= rows[t * Wm + w];
        }
        if (acc) atomicOr((unsigned long long*)&removed[w], (unsigned long long)acc);
      }
      __syncthreads();
    }
    if (tid == 0 && kept_total) atomicAdd(nkeep, kept_total);
    __syncthreads();
  }
}

// Greedy NMS inside one 64 x 64 diagonal tile from its column form: lane t holds colm (bit s: earlier
// box s suppresses box t). Jacobi steps K -> live & ~{t : colm_t & K != 0} (one AND, one compare, one
// ballot each) fix at least one more leading position per step, so the greedy set -- the unique
// fixpoint -- is reached after at most 65 steps, usually a handful.
__device__ __forceinline__ uint64_t tile_greedy_col(uint64_t colm, uint64_t live) {
  uint64_t k = live;
  for (int it = 0; it <= 64; ++it) {
    const uint64_t nk = live & ~(uint64_t)__ballot((colm & k) != 0ull);
    if (nk == k) break;
    k = nk;
  }
  return k;
}

// Single-wave scan (segments of up to 64*SCAN_WAVE_W boxes): one 64-lane workgroup per segment and
// no workgroup barriers. A 64-row block's mask rows are one contiguous run of 64*Wm words; it is
// copied whole into an LDS ring slot by LDS-DMA (16 coalesced 1 KiB buffer_load_dwordx4 ... lds, plus
// one for the block's 64 box ids, one for its 64 column words), SCAN_RING - 1 blocks ahead of the one
// being resolved, so the dependent chain waits on L2/MALL latency once per segment instead of once per
// block. Lane w keeps the removed bits of word w in a register; the in-tile chain is resolved by
// tile_greedy_col (ballot Jacobi steps on the column words) and lanes w and w + 32 OR the kept rows'
// word w from LDS (half the rows each, eight reads in flight), combined with one cross-lane permute.
// Same greedy result as nms_scan_kernel. Every block issues exactly SCAN_DMA VMEM instructions
// (slots past the rows read out of range -> zero) and one flags store, so the counted waits are exact.
static constexpr int SCAN_WAVE_W = 32;
static constexpr int SCAN_RING = 5;
static constexpr int SCAN_COLM = 64 * SCAN_WAVE_W * 8 + 256;   // slot offset of the column words
static constexpr int SCAN_SLOT = SCAN_COLM + 1024;  // bytes: rows + box ids + column words (+ pad)
static constexpr int SCAN_DMA = 18;

__device__ __forceinline__ void scan_wait(int ahead) {  // DMA of the block `ahead` blocks before the newest done
  if (ahead >= 3) wait_vmcnt<3 * SCAN_DMA>();
  else if (ahead == 2) wait_vmcnt<2 * SCAN_DMA>();
  else if (ahead == 1) wait_vmcnt<SCAN_DMA>();
  else wait_vmcnt<0>();
}

__global__ void __launch_bounds__(64) nms_scan_wave_kernel(const uint64_t* __restrict__ mask,
                                                           const int32_t* __restrict__ seg_start,
                                                           const int32_t* __restrict__ nseg_p,
                                                           const int32_t* __restrict__ svals,
                                                           const uint64_t* __restrict__ colm, int Wm,
                                                           int32_t* __restrict__ flags, int32_t* __restrict__ nkeep) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smb[];  // [SCAN_RING][SCAN_SLOT]
  const int lane = threadIdx.x;
  const int nseg = *nseg_p;
  const int64_t ntot = seg_start[nseg];
  const i32x4 mrs = dma_rsrc(mask, (uint32_t)(ntot * Wm * 8)), vrs = dma_rsrc(svals, (uint32_t)(ntot * 4));
  const i32x4 crs = dma_rsrc(colm, (uint32_t)(ntot * 8));
  const uint32_t lds0 = lds_addr(smb);
  const int nrow_inst = (Wm + 1) >> 1;  // 1 KiB per instruction: 64 rows x Wm words = Wm / 2 KiB
  for (int seg = blockIdx.x; seg < nseg; seg += gridDim.x) {
    const int64_t s0 = seg_start[seg], len = seg_start[seg + 1] - s0;
    const int W = (int)((len + 63) / 64);
    if (W > Wm || W > SCAN_WAVE_W) {
      if (lane == 0) atomicExch(nkeep, (int32_t)0x80000000);
      continue;
    }
    auto issue = [&](int b) {
      const uint32_t dst = lds0 + (uint32_t)((b % SCAN_RING) * SCAN_SLOT);
      const uint32_t src = (uint32_t)((s0 + 64 * (int64_t)b) * Wm * 8);
#pragma unroll
      for (int i = 0; i < SCAN_DMA - 1; ++i)
        lds_dma16(mrs, dst + i * 1024, i < nrow_inst ? src + i * 1024 + lane * 16 : 0xfffffff0u, 0);
      lds_dma4(vrs, dst + 64 * SCAN_WAVE_W * 8, (uint32_t)((s0 + 64 * (int64_t)b) * 4) + lane * 4, 0);
      lds_dma16(crs, dst + SCAN_COLM, (uint32_t)((s0 + 64 * (int64_t)b) * 8) + lane * 16, 0);  // 128 words
    };
    for (int b = 0; b < SCAN_RING - 1 && b < W; ++b) issue(b);
    uint64_t rem = 0;  // removed bits of word `lane`
    int kept_total = 0;
    for (int blk = 0; blk < W; ++blk) {
      scan_wait(min(W - 1, blk + SCAN_RING - 2) - blk);
      const uint8_t* slot = smb + (blk % SCAN_RING) * SCAN_SLOT;
      const uint64_t* rows = (const uint64_t*)slot;
      const int32_t* ids = (const int32_t*)(slot + 64 * SCAN_WAVE_W * 8);
      const int cnt = (int)min<int64_t>(64, len - (int64_t)blk * 64);
      const uint64_t cm = ((const uint64_t*)(slot + SCAN_COLM))[lane];
      const uint64_t rm = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(rem >> 32), blk) << 32) |
                          (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)rem, blk);
      const uint64_t valid = cnt >= 64 ? ~0ull : ((1ull << cnt) - 1);
      const uint64_t kept = tile_greedy_col(cm, ~rm & valid);
      // flags were zeroed by the keys kernel: every lane < cnt (>= 1 of them) stores, so each block
      // issues exactly one store instruction
      if (lane < cnt) flags[ids[lane]] = (int32_t)((kept >> lane) & 1ull);
      kept_total += __popcll(kept);
      // word w = lane & 31 of the kept rows: lanes < 32 take rows 0..31, lanes >= 32 rows 32..63, all 32
      // reads independent and selected by the kept bit (most rows survive at RPN densities: a bit walk's
      // dependent ctz chain cost more than the unneeded reads), then the halves are combined across lanes
      uint64_t acc = 0;
      const int w = lane & 31;
      if (w > blk && w < W) {
        const uint32_t m = lane < 32 ? (uint32_t)kept : (uint32_t)(kept >> 32);
        const uint64_t* base = rows + (lane < 32 ? 0 : 32) * Wm + w;
#pragma unroll
        for (int t = 0; t < 32; ++t) {
          const uint64_t v = base[t * Wm];
          acc |= ((m >> t) & 1u) ? v : 0ull;
        }
      }
      {
        const int src = (lane ^ 32) << 2;
        const uint32_t olo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)acc);
        const uint32_t ohi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(acc >> 32));
        rem |= acc | ((uint64_t)ohi << 32) | olo;  // lanes < 32 hold the removed words
      }
      // the slot refilled next is the one resolved in the previous iteration: its ds_reads returned
      // (their results were consumed) before this point
      if (blk + SCAN_RING - 1 < W) {
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this block's LDS reads are done
        issue(blk + SCAN_RING - 1);
      }
    }
    if (lane == 0 && kept_total) atomicAdd(nkeep, kept_total);
    wait_vmcnt<0>();  // the next segment's DMA must not land while a straggling store is counted
  }
}

// final order: kept first by (group, score desc, index); the rest after
__global__ void nms_final_keys_kernel(const float* __restrict__ scores, const int32_t* __restrict__ group,
                                      const int32_t* __restrict__ flags, int64_t n, uint64_t* __restrict__ keys,
                                      int32_t* __restrict__ vals) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t k = ~0ull;
  if (flags[i]) {
    uint32_t hi = group ? ord_i32(group[i]) : 0u;
    k = ((uint64_t)hi << 32) | (uint64_t)(~ord_f32(scores[i]));
    if (k == ~0ull) k = ~0ull - 1;
  }
  keys[i] = k;
  vals[i] = (int32_t)i;
}

__global__ void nms_out_kernel(const int32_t* __restrict__ vals, int64_t n, const int32_t* __restrict__ nk32,
                               int64_t* __restrict__ keep, int64_t* __restrict__ num_keep) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) keep[i] = vals[i];
  if (i == 0) *num_keep = *nk32;
}

// ---- grouped dispatch (mx_batched_nms_grouped) -------------------------------------------------
// torchvision's filter_proposals calls batched_nms once per image; the CPU dispatch rule then picks
// per image: 4n > 4000 -> per-level ("vanilla") NMS, else the coordinate trick with that image's
// own max coordinate. Here all images go in one call and the rule is evaluated per group on the
// device (no host round trip for the counts): pass 1 counts each group's live boxes and takes its
// max coordinate; the keys then put a trick group in one segment with offset boxes and a vanilla
// group in one segment per level. Dead entries (group >= G) get singleton segments and are dropped
// from the output.
// Per wave: one global atomic pair per distinct group present (groups are contiguous runs of the
// image-major candidate list, so usually one or two per wave) instead of one per box -- thousands of
// same-address atomics serialise at L2.
__global__ void nms_group_stats_kernel(const float4* __restrict__ boxes, const int32_t* __restrict__ group, int64_t n,
                                       int G, int32_t* __restrict__ gcnt, uint32_t* __restrict__ gmax) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  int g = -1;
  uint32_t m = 0;
  if (i < n) {
    g = group[i];
    if (g >= 0 && g < G) {
      const float4 b = boxes[i];
      m = max(max(ord_f32(b.x), ord_f32(b.y)), max(ord_f32(b.z), ord_f32(b.w)));
    } else {
      g = -1;
    }
  }
  bool todo = g >= 0;
  while (__ballot(todo)) {
    const uint64_t act = __ballot(todo);
    const int leader = __ffsll((unsigned long long)act) - 1;
    const int gg = __shfl(g, leader);
    const bool mine = todo && g == gg;
    const uint64_t sel = __ballot(mine);
    uint32_t v = mine ? m : 0u;
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
    if (lane == leader) {
      atomicAdd(gcnt + gg, (int)__popcll(sel));
      atomicMax(gmax + gg, v);
    }
    todo = todo && !mine;
  }
}

__global__ void nms_group_keys_kernel(const float4* __restrict__ boxes, const float* __restrict__ scores,
                                      const int64_t* __restrict__ lvl, const int32_t* __restrict__ group, int64_t n, int G,
                                      int L, const int32_t* __restrict__ gcnt, const uint32_t* __restrict__ gmax,
                                      uint64_t* __restrict__ keys, int32_t* __restrict__ vals, float4* __restrict__ obox,
                                      int32_t* __restrict__ flags, int32_t* __restrict__ nk) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  flags[i] = 0;
  if (i == 0) *nk = 0;
  float4 b = boxes[i];
  const int g = group[i];
  uint32_t hi;
  if (g < 0 || g >= G) {
    hi = (uint32_t)G * (uint32_t)(L + 1) + (uint32_t)i;  // dead: a segment of its own
  } else if ((int64_t)gcnt[g] * 4 <= 4000) {               // coordinate trick over the whole image
    const float step = unord_f32(gmax[g]) + 1.0f;
    const float off = (float)lvl[i] * step;
    b.x = b.x + off; b.y = b.y + off; b.z = b.z + off; b.w = b.w + off;
    hi = (uint32_t)g * (uint32_t)(L + 1) + (uint32_t)L;
  } else {                                                 // per level
    hi = (uint32_t)g * (uint32_t)(L + 1) + (uint32_t)lvl[i];
  }
  obox[i] = b;
  keys[i] = ((uint64_t)hi << 32) | (uint64_t)(~ord_f32(scores[i]));
  vals[i] = (int32_t)i;
}

__global__ void nms_group_final_keys_kernel(const float* __restrict__ scores, const int32_t* __restrict__ group,
                                            const int32_t* __restrict__ flags, int64_t n, int G,
                                            uint64_t* __restrict__ keys, int32_t* __restrict__ vals) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // live: (group, score desc); removed / dead: the sentinel (G, max), above every live key, so the
  // sort only needs the low 32 + bit_length(G) bits
  uint64_t k = ((uint64_t)G << 32) | 0xffffffffull;
  const int g = group[i];
  if (flags[i] && g >= 0 && g < G) k = ((uint64_t)g << 32) | (uint64_t)(~ord_f32(scores[i]));
  keys[i] = k;
  vals[i] = (int32_t)i;
}

// keep = survivors by (group, score desc, index); num_keep = number of non-sentinel keys
__global__ void nms_group_out_kernel(const uint64_t* __restrict__ skeys, const int32_t* __restrict__ vals, int64_t n,
                                     uint64_t dead, const int32_t* __restrict__ nk32, int64_t* __restrict__ keep,
                                     int64_t* __restrict__ num_keep) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  keep[i] = vals[i];
  const bool live = skeys[i] != dead;
  // -1: a segment exceeded max_seg (the scan's overflow flag)
  if (live && (i == n - 1 || skeys[i + 1] == dead)) *num_keep = *nk32 < 0 ? -1 : i + 1;
  if (i == 0 && !live) *num_keep = *nk32 < 0 ? -1 : 0;
}

// ---- presorted grouped dispatch (mx_batched_nms_grouped_sorted) --------------------------------
// filter_proposals' candidates are already ordered: image-major, level-major, and within each
// (image, level) run by the per-level top-k's value order (score = sigmoid(logit) of a descending
// logit list). Then the segment sort of mx_batched_nms_grouped is a stable compaction plus, for a
// coordinate-trick image, a merge of its level runs -- and the final (image, score desc, index)
// order of the survivors is a merge of their level runs. One workgroup per image does each with a
// block scan in list order and merge ranks by binary search over the runs' score keys in LDS:
// 2 launches replace the two radix sorts, the scans and their helper kernels (4 launches in all with
// the mask and scan kernels). Exactness does not rest on the presorted order: every run's key order
// is checked in LDS, and a run found out of order (e.g. a non-monotone sigmoid at ulp level) is ranked
// by counting instead of binary search -- the result is always the stable (segment, score desc,
// index) order of mx_batched_nms_grouped.
static constexpr int PS_T = 1024, PS_NMAX = 24576, PS_GMAX = 64, PS_LMAX = 8, PS_CH = PS_NMAX / PS_T;
static constexpr int PS_SLICES = 8;  // workgroups per image in the compaction / ranking kernels

// wave-aggregated counters: cnt[key] += #lanes with that key, mx[key / L] = max(m) (key < 0: none);
// LDS or global (agent-scope atomics) alike
__device__ __forceinline__ void ps_wave_add(int key, uint32_t m, int lane, uint32_t* cnt, uint32_t* mx, int L) {
  bool todo = key >= 0;
  while (__ballot(todo)) {
    const uint64_t act = __ballot(todo);
    const int leader = __ffsll((unsigned long long)act) - 1;
    const int kk = __shfl(key, leader);
    const bool mine = todo && key == kk;
    const uint64_t sel = __ballot(mine);
    if (mx) {
      uint32_t v = mine ? m : 0u;
      for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
      if (lane == leader) atomicMax(mx + kk / L, v);
    }
    if (lane == leader) atomicAdd(cnt + kk, (uint32_t)__popcll(sel));
    todo = todo && !mine;
  }
}

// block-wide exclusive scan of one int per thread (16 waves); *total = the block's sum
__device__ __forceinline__ int ps_excl_scan(int v, int lane, int wave, int* wsum, int* total) {
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  int wb = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < PS_T / 64; ++w) {
    const int c = wsum[w];
    wb += w < wave ? c : 0;
    tot += c;
  }
  __syncthreads();
  *total = tot;
  return wb + x - v;
}

// entries of run [lo, hi) (keys non-increasing unless `bad`) ranked before key x at compacted index q:
// key greater, or equal and earlier in list order (index below q)
__device__ __forceinline__ int ps_before(const uint32_t* key, int lo, int hi, uint32_t x, int q, bool bad) {
  if (bad) {
    int c = 0;
    for (int j = lo; j < hi; ++j) {
      const uint32_t y = key[j];
      c += (y > x || (y == x && j < q)) ? 1 : 0;
    }
    return c;
  }
  if (q >= hi) {  // whole run earlier in list order: ties precede
    int a = lo, b = hi;
    while (a < b) {
      const int mid = (a + b) >> 1;
      if (key[mid] >= x) a = mid + 1; else b = mid;
    }
    return a - lo;
  }
  if (q < lo) {  // whole run later: ties follow
    int a = lo, b = hi;
    while (a < b) {
      const int mid = (a + b) >> 1;
      if (key[mid] > x) a = mid + 1; else b = mid;
    }
    return a - lo;
  }
  return q - lo;  // x's own sorted run
}

__device__ __forceinline__ int ps_run_of(const int* rs, int L, int q) {
  int l = 0;
  while (l + 1 < L && q >= rs[l + 1]) ++l;
  return l;
}

// pass over the list by many blocks: live entries per (image, level) and the max coordinate per image
// into tab (zeroed by a memset; tab[G*L .. G*L+G) = max bits), flags zeroed, keep count reset
__global__ void __launch_bounds__(256) nms_sorted_stats_kernel(const float4* __restrict__ boxes,
                                                               const int64_t* __restrict__ lvl,
                                                               const int32_t* __restrict__ group, int n, int G, int L,
                                                               uint32_t* __restrict__ tab, int32_t* __restrict__ flags,
                                                               int32_t* __restrict__ nk) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  int k = -1;
  uint32_t m = 0;
  if (i < n) {
    flags[i] = 0;
    const int gi = group[i];
    if (gi >= 0 && gi < G) {
      const float4 b = boxes[i];
      m = max(max(ord_f32(b.x), ord_f32(b.y)), max(ord_f32(b.z), ord_f32(b.w)));
      k = gi * L + (int)lvl[i];
    }
  }
  if (i == 0) *nk = 0;
  ps_wave_add(k, m, threadIdx.x & 63, tab, tab + G * L, L);
}

// survivors per (image, level) into tab2 (zeroed by nms_sorted_pre_kernel)
__global__ void __launch_bounds__(256) nms_sorted_post_stats_kernel(const int64_t* __restrict__ lvl,
                                                                    const int32_t* __restrict__ group,
                                                                    const int32_t* __restrict__ flags, int n, int G,
                                                                    int L, uint32_t* __restrict__ tab2) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  int k = -1;
  if (i < n && flags[i]) {
    const int gi = group[i];
    if (gi >= 0 && gi < G) k = gi * L + (int)lvl[i];
  }
  ps_wave_add(k, 0u, threadIdx.x & 63, tab2, nullptr, L);
}

// The block's image entries in list order: thread t owns [t*ch, t*ch + ch) (ch a multiple of 4, so
// its group / flag / score words come as 16-B loads, all in flight at once). Entries of group g (and,
// with flags, flagged) are compacted in list order: key[q] = ord_f32(score), idx[q] = list index.
// Returns the block's count.
__device__ __forceinline__ int ps_compact(const int32_t* __restrict__ group, const int32_t* __restrict__ flags,
                                          const float* __restrict__ scores, int n, int g, int ch, int tid, int lane,
                                          int wave, int* wsum, uint32_t* key, uint16_t* idx) {
  const int b0 = tid * ch;
  int gv[PS_CH], fv[PS_CH];
  float sv[PS_CH];
#pragma unroll
  for (int v = 0; v < PS_CH / 4; ++v) {
    const int i = b0 + 4 * v;
    if (4 * v < ch && i + 3 < n) {
      const int4 a = *(const int4*)(group + i);
      gv[4 * v] = a.x; gv[4 * v + 1] = a.y; gv[4 * v + 2] = a.z; gv[4 * v + 3] = a.w;
      const float4 b = *(const float4*)(scores + i);
      sv[4 * v] = b.x; sv[4 * v + 1] = b.y; sv[4 * v + 2] = b.z; sv[4 * v + 3] = b.w;
      if (flags) {
        const int4 c = *(const int4*)(flags + i);
        fv[4 * v] = c.x; fv[4 * v + 1] = c.y; fv[4 * v + 2] = c.z; fv[4 * v + 3] = c.w;
      } else {
        fv[4 * v] = fv[4 * v + 1] = fv[4 * v + 2] = fv[4 * v + 3] = 1;
      }
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bool in = 4 * v + t < ch && i + t < n;
        gv[4 * v + t] = in ? group[i + t] : -1;
        sv[4 * v + t] = in ? scores[i + t] : 0.f;
        fv[4 * v + t] = (in && flags) ? flags[i + t] : 1;
      }
    }
  }
  int own = 0;
#pragma unroll
  for (int u = 0; u < PS_CH; ++u) own += (gv[u] == g && fv[u] != 0) ? 1 : 0;
  int tot;
  int q = ps_excl_scan(own, lane, wave, wsum, &tot);
#pragma unroll
  for (int u = 0; u < PS_CH; ++u) {
    if (gv[u] == g && fv[u] != 0) {
      key[q] = ord_f32(sv[u]);
      idx[q] = (uint16_t)(b0 + u);
      ++q;
    }
  }
  return tot;
}

// run-order check of the compacted keys: bit l of the result = run l out of order (non-increasing
// expected); LDS only
__device__ __forceinline__ void ps_check_runs(const uint32_t* key, const int* rs, int L, int cnt, int tid, uint32_t* bad) {
  for (int q = tid + 1; q < cnt; q += PS_T) {
    const int l = ps_run_of(rs, L, q);
    if (q > rs[l] && key[q] > key[q - 1]) atomicOr(bad, 1u << l);
  }
}

// one workgroup per image g: segment layout (positions, segment ids, offset boxes) for the mask /
// scan kernels -- the outputs of nms_group_keys + sort + gather + scan + seg of the general path
__global__ void __launch_bounds__(PS_T) nms_sorted_pre_kernel(
    const float4* __restrict__ boxes, const float* __restrict__ scores, const int64_t* __restrict__ lvl,
    const int32_t* __restrict__ group, int n, int G, int L, const uint32_t* __restrict__ tab, uint32_t* __restrict__ tab2,
    float4* __restrict__ sbox, float* __restrict__ sarea, int32_t* __restrict__ v1, int32_t* __restrict__ incl,
    int32_t* __restrict__ seg_start, int32_t* __restrict__ nseg_out, int32_t* __restrict__ err) {
  extern __shared__ uint32_t key[];  // [n] score keys of this image's live entries, list order; then [n] u16 indices
  uint16_t* idx = (uint16_t*)(key + n);
  __shared__ uint32_t bad;
  __shared__ int wsum[PS_T / 64], rs[PS_LMAX + 1], runseg[PS_LMAX];
  __shared__ int s_gbase, s_segbase, s_gcnt, s_trick, s_nlive, s_nseg;
  // blockIdx.y = slice: every slice of an image compacts the image's entries (LDS), then ranks and
  // writes its own share -- the dependent binary-search chains run on S CUs per image, not one
  const int g = blockIdx.x, sl = blockIdx.y, S = gridDim.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (g == 0 && sl == 0)
    for (int k = tid; k < G * L; k += PS_T) tab2[k] = 0;  // the post pass's counters
  if (tid == 0) {
    bad = 0;
    int nl = 0, ns = 0;
    for (int gg = 0; gg < G; ++gg) {
      int gc = 0, nr = 0;
      for (int l = 0; l < L; ++l) {
        gc += (int)tab[gg * L + l];
        nr += tab[gg * L + l] ? 1 : 0;
      }
      const int tr = gc * 4 <= 4000;  // torchvision's CPU dispatch rule, per image
      if (gg == g) {
        s_gbase = nl;
        s_segbase = ns;
        s_gcnt = gc;
        s_trick = tr;
        int r = 0, sid = 0;
        for (int l = 0; l < L; ++l) {
          rs[l] = r;
          runseg[l] = tr ? 0 : sid;
          sid += tab[gg * L + l] ? 1 : 0;
          r += (int)tab[gg * L + l];
        }
        rs[L] = r;
      }
      nl += gc;
      ns += tr ? (gc > 0 ? 1 : 0) : nr;
    }
    s_nlive = nl;
    s_nseg = ns;
  }
  __syncthreads();
  const int gbase = s_gbase, gc = s_gcnt, trick = s_trick, nlive = s_nlive, nseg = s_nseg, segbase = s_segbase;
  // segment starts: one per non-empty level run, or one for a coordinate-trick image
  if (sl == 0) {
    if (trick) {
      if (tid == 0 && gc > 0) seg_start[segbase] = gbase;
    } else if (tid < L && tab[g * L + tid]) {
      seg_start[segbase + runseg[tid]] = gbase + rs[tid];
    }
  }
  if (g == G - 1 && sl == 0 && tid == 0) {
    *nseg_out = nseg;
    seg_start[nseg] = nlive;
    if (nlive < n) seg_start[nseg + 1] = nlive;  // the tail's empty pseudo-segment
  }
  const int ch = ((n + PS_T - 1) / PS_T + 3) & ~3;
  ps_compact(group, nullptr, scores, n, g, ch, tid, lane, wave, wsum, key, idx);
  __syncthreads();
  ps_check_runs(key, rs, L, gc, tid, &bad);
  __syncthreads();
  const uint32_t badm = bad;
  const float step = unord_f32(tab[G * L + g]) + 1.0f;
  // positions, 8 entries per thread per round: ranks from LDS, then all 8 gathers in flight
  for (int q0 = sl * 8 * PS_T; q0 < gc; q0 += S * 8 * PS_T) {
    int pos[8], ii[8], ll[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int q = q0 + e * PS_T + tid;
      pos[e] = -1;
      ii[e] = 0;
      ll[e] = 0;
      if (q < gc) {
        const int l = ps_run_of(rs, L, q);
        const uint32_t x = key[q];
        int rank;
        if (trick) {  // one segment: the merge of the level runs
          rank = 0;
          for (int l2 = 0; l2 < L; ++l2) rank += ps_before(key, rs[l2], rs[l2 + 1], x, q, (badm >> l2) & 1u);
        } else {
          rank = rs[l] + ps_before(key, rs[l], rs[l + 1], x, q, (badm >> l) & 1u);
        }
        pos[e] = gbase + rank;
        ii[e] = idx[q];
        ll[e] = l;
      }
    }
    float4 b[8];
    int lvv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      b[e] = boxes[ii[e]];
      lvv[e] = (int)lvl[ii[e]];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (pos[e] < 0) continue;
      if (lvv[e] != ll[e]) atomicExch(err, 1);  // layout contract: levels contiguous in list order
      float4 bb = b[e];
      if (trick) {  // boxes + idxs * (max_coordinate + 1), as nms_group_keys_kernel
        const float off = (float)lvv[e] * step;
        bb.x = bb.x + off; bb.y = bb.y + off; bb.z = bb.z + off; bb.w = bb.w + off;
      }
      sbox[pos[e]] = bb;
      sarea[pos[e]] = (bb.z - bb.x) * (bb.w - bb.y);
      v1[pos[e]] = ii[e];
      incl[pos[e]] = segbase + runseg[ll[e]] + 1;
    }
  }
  for (int p = nlive + (g * S + sl) * PS_T + tid; p < n; p += G * S * PS_T) incl[p] = nseg + 1;  // empty pseudo-segment
}

// one workgroup per image: survivors (flags) -> keep in (image, score desc, index) order, num_keep,
// and optionally the padded per-image selection sel [G, post] / valid [G, post] of filter_proposals
__global__ void __launch_bounds__(PS_T) nms_sorted_post_kernel(
    const float* __restrict__ scores, const int32_t* __restrict__ group, const int32_t* __restrict__ flags, int n, int G,
    int L, const uint32_t* __restrict__ tab2, const int32_t* __restrict__ nk32, const int32_t* __restrict__ err,
    int64_t* __restrict__ keep, int64_t* __restrict__ num_keep, int post, int64_t* __restrict__ sel,
    uint8_t* __restrict__ valid) {
  extern __shared__ uint32_t key[];
  uint16_t* idx = (uint16_t*)(key + n);
  __shared__ uint32_t bad;
  __shared__ int wsum[PS_T / 64], rs[PS_LMAX + 1];
  __shared__ int s_sbase, s_sc, s_total;
  const int g = blockIdx.x, sl = blockIdx.y, S = gridDim.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) {
    bad = 0;
    int tot = 0;
    for (int gg = 0; gg < G; ++gg) {
      int gc = 0;
      for (int l = 0; l < L; ++l) gc += (int)tab2[gg * L + l];
      if (gg == g) {
        s_sbase = tot;
        s_sc = gc;
        int r = 0;
        for (int l = 0; l < L; ++l) {
          rs[l] = r;
          r += (int)tab2[gg * L + l];
        }
        rs[L] = r;
      }
      tot += gc;
    }
    s_total = tot;
  }
  __syncthreads();
  const int sbase = s_sbase, sc = s_sc, total = s_total;
  const bool failed = *err != 0;
  const int ch = ((n + PS_T - 1) / PS_T + 3) & ~3;
  ps_compact(group, flags, scores, n, g, ch, tid, lane, wave, wsum, key, idx);
  __syncthreads();
  ps_check_runs(key, rs, L, sc, tid, &bad);
  __syncthreads();
  const uint32_t badm = bad;
  for (int q = sl * PS_T + tid; q < sc; q += S * PS_T) {
    const uint32_t x = key[q];
    int rank = 0;
    for (int l2 = 0; l2 < L; ++l2) rank += ps_before(key, rs[l2], rs[l2 + 1], x, q, (badm >> l2) & 1u);
    keep[sbase + rank] = idx[q];
    if (sel && rank < post && !failed) sel[(int64_t)g * post + rank] = idx[q];
  }
  // -1: a segment exceeded max_seg (the scan's overflow flag); -2: the presorted layout contract broken
  if (g == 0 && sl == 0 && tid == 0) *num_keep = failed ? -2 : (*nk32 < 0 ? -1 : total);
  for (int p = total + (g * S + sl) * PS_T + tid; p < n; p += G * S * PS_T) keep[p] = 0;
  if (sel) {  // ranks < min(post, count) were written above by the slice that ranked them
    for (int r = sl * PS_T + tid; r < post; r += S * PS_T) {
      const bool ok = r < sc && !failed;
      if (!ok) sel[(int64_t)g * post + r] = 0;
      valid[(int64_t)g * post + r] = ok ? 1 : 0;
    }
  }
}

struct NmsWs {
  uint64_t *k0, *k1, *mask;
  int32_t *v0, *v1, *head, *incl, *seg_start, *nseg, *flags, *nk;
  uint32_t* maxbits;
  uint32_t* tab;
  int32_t* gcnt;
  uint32_t* gmax;
  float4 *obox, *sbox;
  float* sarea;
  uint64_t* colm;  // column form of the diagonal mask tiles (wave scan)
  void* cub;
  size_t cub_bytes;
};

static size_t cub_bytes_needed(int64_t n) {
  size_t a = 0, b = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (uint64_t*)nullptr, (uint64_t*)nullptr, (int32_t*)nullptr,
                                           (int32_t*)nullptr, (int)n, 0, 64, (hipStream_t)0);
  (void)hipcub::DeviceScan::InclusiveSum(nullptr, b, (int32_t*)nullptr, (int32_t*)nullptr, (int)n, (hipStream_t)0);
  return a > b ? a : b;
}

static size_t carve(Carver& c, int64_t n, int Wm, NmsWs* w, int G = 0) {
  int64_t m = n > 0 ? n : 1;
  w->gcnt = G > 0 ? c.take<int32_t>(2 * (size_t)G) : nullptr;  // [G] counts then [G] max bits
  // the presorted path's tables: [G*L] live counts, [G] max bits, [G*L] survivor counts, error word
  w->tab = G > 0 ? c.take<uint32_t>(2 * (size_t)PS_GMAX * PS_LMAX + PS_GMAX + 1) : nullptr;
  w->gmax = G > 0 ? (uint32_t*)(w->gcnt + G) : nullptr;
  w->k0 = c.take<uint64_t>(m); w->k1 = c.take<uint64_t>(m);
  w->v0 = c.take<int32_t>(m); w->v1 = c.take<int32_t>(m);
  w->head = c.take<int32_t>(m); w->incl = c.take<int32_t>(m);
  w->seg_start = c.take<int32_t>(m + 1); w->nseg = c.take<int32_t>(1);
  w->flags = c.take<int32_t>(m); w->nk = c.take<int32_t>(1);
  w->maxbits = c.take<uint32_t>(1);
  w->obox = c.take<float4>(m); w->sbox = c.take<float4>(m); w->sarea = c.take<float>(m);
  w->mask = c.take<uint64_t>((size_t)m * Wm);
  w->colm = c.take<uint64_t>(m);
  w->cub_bytes = cub_bytes_needed(m);
  w->cub = c.take<char>(w->cub_bytes);
  return c.off;
}

}  // namespace mx

using namespace mx;

extern "C" size_t mx_nms_workspace(int64_t n, int64_t max_seg) {
  if (max_seg <= 0 || max_seg > n) max_seg = n;
  if (n * 4 <= 4000) max_seg = n;  // coordinate-trick path treats all boxes as one segment
  int Wm = (int)cdiv(max_seg > 0 ? max_seg : 1, 64);
  Carver c(nullptr, 0);
  NmsWs w;
  return carve(c, n, Wm, &w);
}

extern "C" int mx_batched_nms(const float* boxes, const float* scores, const int64_t* idxs, const int32_t* group,
                              int64_t n, int64_t max_seg, double thr, int mode, int64_t* keep, int64_t* num_keep,
                              void* ws, size_t ws_bytes, mx_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  MX_CHECK_ARG(n >= 0 && n < (1ll << 31), "mx_batched_nms: bad n %lld", (long long)n);
  MX_CHECK_ARG(mode >= 0 && mode <= 2, "mx_batched_nms: bad mode %d", mode);
  if (n == 0) {
    MX_HIP(hipMemsetAsync(num_keep, 0, sizeof(int64_t), s));
    return MX_OK;
  }
  int trick = 0;
  if (idxs) trick = (mode == 2) || (mode == 0 && n * 4 <= 4000);
  if (!idxs || trick) max_seg = n;
  if (max_seg <= 0 || max_seg > n) max_seg = n;
  int Wm = (int)cdiv(max_seg, 64);
  Carver c(ws, ws_bytes);
  NmsWs w;
  carve(c, n, Wm, &w);
  MX_CHECK_ARG(c.ok(), "mx_batched_nms: workspace too small (%zu < %zu); size it with max_seg=%lld", ws_bytes, c.off,
               (long long)max_seg);
  MX_CHECK_ARG(Wm * 8 <= 64 * 1024, "mx_batched_nms: segment bound %lld too large", (long long)max_seg);
  const int T = 256;
  const int nb = (int)cdiv(n, T);
  if (trick) {
    MX_HIP(hipMemsetAsync(w.maxbits, 0, sizeof(uint32_t), s));
    nms_max_kernel<<<(int)std::min<int64_t>(cdiv(4 * n, T), 1024), T, 0, s>>>(boxes, 4 * n, w.maxbits);
    MX_LAUNCH_CHECK();
  }
  nms_keys_kernel<<<nb, T, 0, s>>>((const float4*)boxes, scores, idxs, n, trick, w.maxbits, w.k0, w.v0, w.obox, w.flags,
                                   w.nk);
  MX_LAUNCH_CHECK();
  size_t cb = w.cub_bytes;
  int end_bit = (idxs && !trick) ? 64 : 32;
  MX_HIP(hipcub::DeviceRadixSort::SortPairs(w.cub, cb, w.k0, w.k1, w.v0, w.v1, (int)n, 0, end_bit, s));
  nms_gather_kernel<<<nb, T, 0, s>>>(w.k1, w.v1, w.obox, n, w.sbox, w.sarea, w.head);
  MX_LAUNCH_CHECK();
  cb = w.cub_bytes;
  MX_HIP(hipcub::DeviceScan::InclusiveSum(w.cub, cb, w.head, w.incl, (int)n, s));
  nms_seg_kernel<<<nb, T, 0, s>>>(w.head, w.incl, n, w.seg_start, w.nseg);
  MX_LAUNCH_CHECK();
  dim3 mg((unsigned)cdiv(n, 64), (unsigned)Wm);
  nms_mask_kernel<<<mg, 64, 0, s>>>(w.sbox, w.sarea, w.incl, w.seg_start, n, Wm, thr, w.mask,
                                    Wm <= SCAN_WAVE_W ? w.colm : nullptr);
  MX_LAUNCH_CHECK();
  int sgrid = (int)std::min<int64_t>(n, 1024);
  if (Wm <= SCAN_WAVE_W)
    nms_scan_wave_kernel<<<sgrid, 64, (size_t)SCAN_RING * SCAN_SLOT, s>>>(w.mask, w.seg_start, w.nseg, w.v1,
                                                                                   w.colm, Wm, w.flags, w.nk);
  else if (Wm <= SCAN_LDS_W)
    nms_scan_lds_kernel<<<sgrid, 256, sizeof(uint64_t) * (Wm + 64 * (size_t)Wm), s>>>(w.mask, w.seg_start, w.nseg, w.v1,
                                                                                       Wm, w.flags, w.nk);
  else
    nms_scan_kernel<<<sgrid, 64, sizeof(uint64_t) * Wm, s>>>(w.mask, w.seg_start, w.nseg, w.v1, Wm, w.flags, w.nk);
  MX_LAUNCH_CHECK();
  nms_final_keys_kernel<<<nb, T, 0, s>>>(scores, group, w.flags, n, w.k0, w.v0);
  MX_LAUNCH_CHECK();
  cb = w.cub_bytes;
  MX_HIP(hipcub::DeviceRadixSort::SortPairs(w.cub, cb, w.k0, w.k1, w.v0, w.v1, (int)n, 0, 64, s));
  nms_out_kernel<<<nb, T, 0, s>>>(w.v1, n, w.nk, keep, num_keep);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_batched_nms_grouped_sorted(const float* boxes, const float* scores, const int64_t* lvl,
                                             const int32_t* group, int64_t n, int64_t G, int64_t L, int64_t max_seg,
                                             double thr, int64_t* keep, int64_t* num_keep, int64_t post, int64_t* sel,
                                             uint8_t* valid, void* ws, size_t ws_bytes, mx_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  MX_CHECK_ARG(n >= 0 && n <= PS_NMAX && G > 0 && G <= PS_GMAX && L > 0 && L <= PS_LMAX,
               "mx_batched_nms_grouped_sorted: bad sizes n=%lld (<= %d) G=%lld (<= %d) L=%lld (<= %d)", (long long)n,
               PS_NMAX, (long long)G, PS_GMAX, (long long)L, PS_LMAX);
  MX_CHECK_ARG(num_keep && (n == 0 || (boxes && scores && lvl && group && keep)),
               "mx_batched_nms_grouped_sorted: null pointer");
  MX_CHECK_ARG(post >= 0 && (post == 0 || (sel && valid)), "mx_batched_nms_grouped_sorted: sel / valid needed for post > 0");
  if (n == 0) {
    MX_HIP(hipMemsetAsync(num_keep, 0, sizeof(int64_t), s));
    if (post > 0) {
      MX_HIP(hipMemsetAsync(sel, 0, sizeof(int64_t) * (size_t)(G * post), s));
      MX_HIP(hipMemsetAsync(valid, 0, (size_t)(G * post), s));
    }
    return MX_OK;
  }
  if (max_seg <= 0 || max_seg > n) max_seg = n;
  const int Wm = (int)cdiv(max_seg, 64);
  Carver c(ws, ws_bytes);
  NmsWs w;
  carve(c, n, Wm, &w, (int)G);
  // small tables in the (unused here) sort-key buffer: [G*L] counts + [G] max bits, [G*L] survivor
  // counts, one error word
  MX_CHECK_ARG(c.ok(), "mx_batched_nms_grouped_sorted: workspace too small (%zu < %zu)", ws_bytes, c.off);
  MX_CHECK_ARG(Wm * 8 <= 64 * 1024, "mx_batched_nms_grouped_sorted: segment bound %lld too large", (long long)max_seg);
  uint32_t* tab = w.tab;
  uint32_t* tab2 = tab + G * L + G;
  int32_t* err = (int32_t*)(tab2 + G * L);
  MX_HIP(hipMemsetAsync(tab, 0, sizeof(uint32_t) * (size_t)(G * L + G) + sizeof(uint32_t) * (size_t)(G * L) + 4, s));
  const int nb = (int)cdiv(n, 256);
  nms_sorted_stats_kernel<<<nb, 256, 0, s>>>((const float4*)boxes, lvl, group, (int)n, (int)G, (int)L, tab, w.flags, w.nk);
  MX_LAUNCH_CHECK();
  const size_t lds = (sizeof(uint32_t) + sizeof(uint16_t)) * (size_t)n + 16;
  const dim3 pg((unsigned)G, (unsigned)PS_SLICES);
  nms_sorted_pre_kernel<<<pg, PS_T, lds, s>>>((const float4*)boxes, scores, lvl, group, (int)n, (int)G, (int)L, tab,
                                                  tab2, w.sbox, w.sarea, w.v1, w.incl, w.seg_start, w.nseg, err);
  MX_LAUNCH_CHECK();
  dim3 mg((unsigned)cdiv(n, 64), (unsigned)Wm);
  nms_mask_kernel<<<mg, 64, 0, s>>>(w.sbox, w.sarea, w.incl, w.seg_start, n, Wm, thr, w.mask,
                                    Wm <= SCAN_WAVE_W ? w.colm : nullptr);
  MX_LAUNCH_CHECK();
  const int sgrid = (int)std::min<int64_t>(n, 1024);
  if (Wm <= SCAN_WAVE_W)
    nms_scan_wave_kernel<<<sgrid, 64, (size_t)SCAN_RING * SCAN_SLOT, s>>>(w.mask, w.seg_start, w.nseg, w.v1,
                                                                                   w.colm, Wm, w.flags, w.nk);
  else if (Wm <= SCAN_LDS_W)
    nms_scan_lds_kernel<<<sgrid, 256, sizeof(uint64_t) * (Wm + 64 * (size_t)Wm), s>>>(w.mask, w.seg_start, w.nseg, w.v1,
                                                                                       Wm, w.flags, w.nk);
  else
    nms_scan_kernel<<<sgrid, 64, sizeof(uint64_t) * Wm, s>>>(w.mask, w.seg_start, w.nseg, w.v1, Wm, w.flags, w.nk);
  MX_LAUNCH_CHECK();
  nms_sorted_post_stats_kernel<<<nb, 256, 0, s>>>(lvl, group, w.flags, (int)n, (int)G, (int)L, tab2);
  MX_LAUNCH_CHECK();
  nms_sorted_post_kernel<<<pg, PS_T, lds, s>>>(scores, group, w.flags, (int)n, (int)G, (int)L, tab2, w.nk, err,
                                                   keep, num_keep, (int)post, post > 0 ? sel : nullptr,
                                                   post > 0 ? valid : nullptr);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" size_t mx_nms_grouped_workspace(int64_t n, int64_t G, int64_t max_seg) {
  if (n <= 0 || G <= 0) return 0;
  if (max_seg <= 0 || max_seg > n) max_seg = n;
  Carver c(nullptr, 0);
  NmsWs w;
  return carve(c, n, (int)cdiv(max_seg, 64), &w, (int)G);
}

extern "C" int mx_batched_nms_grouped(const float* boxes, const float* scores, const int64_t* lvl, const int32_t* group,
                                      int64_t n, int64_t G, int64_t L, int64_t max_seg, double thr, int64_t* keep,
                                      int64_t* num_keep, void* ws, size_t ws_bytes, mx_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  MX_CHECK_ARG(n >= 0 && n < (1ll << 30) && G > 0 && L > 0 && G * (L + 1) + n < (1ll << 31),
               "mx_batched_nms_grouped: bad sizes n=%lld G=%lld L=%lld", (long long)n, (long long)G, (long long)L);
  MX_CHECK_ARG(boxes && scores && lvl && group && keep && num_keep, "mx_batched_nms_grouped: null pointer");
  if (n == 0) {
    MX_HIP(hipMemsetAsync(num_keep, 0, sizeof(int64_t), s));
    return MX_OK;
  }
  if (max_seg <= 0 || max_seg > n) max_seg = n;
  const int Wm = (int)cdiv(max_seg, 64);
  Carver c(ws, ws_bytes);
  NmsWs w;
  carve(c, n, Wm, &w, (int)G);
  MX_CHECK_ARG(c.ok(), "mx_batched_nms_grouped: workspace too small (%zu < %zu)", ws_bytes, c.off);
  MX_CHECK_ARG(Wm * 8 <= 64 * 1024, "mx_batched_nms_grouped: segment bound %lld too large", (long long)max_seg);
  const int T = 256;
  const int nb = (int)cdiv(n, T);
  MX_HIP(hipMemsetAsync(w.gcnt, 0, sizeof(int32_t) * 2 * (size_t)G, s));
  nms_group_stats_kernel<<<nb, T, 0, s>>>((const float4*)boxes, group, n, (int)G, w.gcnt, w.gmax);
  MX_LAUNCH_CHECK();
  nms_group_keys_kernel<<<nb, T, 0, s>>>((const float4*)boxes, scores, lvl, group, n, (int)G, (int)L, w.gcnt, w.gmax,
                                         w.k0, w.v0, w.obox, w.flags, w.nk);
  MX_LAUNCH_CHECK();
  // segment keys: hi < G*(L+1) + n, so only the low 32 + bit_length of that bound are sorted
  const int end1 = std::min(64, 32 + (64 - __builtin_clzll((unsigned long long)(G * (L + 1) + n))));
  size_t cb = w.cub_bytes;
  MX_HIP(hipcub::DeviceRadixSort::SortPairs(w.cub, cb, w.k0, w.k1, w.v0, w.v1, (int)n, 0, end1, s));
  nms_gather_kernel<<<nb, T, 0, s>>>(w.k1, w.v1, w.obox, n, w.sbox, w.sarea, w.head);
  MX_LAUNCH_CHECK();
  cb = w.cub_bytes;
  MX_HIP(hipcub::DeviceScan::InclusiveSum(w.cub, cb, w.head, w.incl, (int)n, s));
  nms_seg_kernel<<<nb, T, 0, s>>>(w.head, w.incl, n, w.seg_start, w.nseg);
  MX_LAUNCH_CHECK();
  dim3 mg((unsigned)cdiv(n, 64), (unsigned)Wm);
  nms_mask_kernel<<<mg, 64, 0, s>>>(w.sbox, w.sarea, w.incl, w.seg_start, n, Wm, thr, w.mask,
                                    Wm <= SCAN_WAVE_W ? w.colm : nullptr);
  MX_LAUNCH_CHECK();
  const int sgrid = (int)std::min<int64_t>(n, 1024);
  if (Wm <= SCAN_WAVE_W)
    nms_scan_wave_kernel<<<sgrid, 64, (size_t)SCAN_RING * SCAN_SLOT, s>>>(w.mask, w.seg_start, w.nseg, w.v1,
                                                                                   w.colm, Wm, w.flags, w.nk);
  else if (Wm <= SCAN_LDS_W)
    nms_scan_lds_kernel<<<sgrid, 256, sizeof(uint64_t) * (Wm + 64 * (size_t)Wm), s>>>(w.mask, w.seg_start, w.nseg, w.v1,
                                                                                       Wm, w.flags, w.nk);
  else
    nms_scan_kernel<<<sgrid, 64, sizeof(uint64_t) * Wm, s>>>(w.mask, w.seg_start, w.nseg, w.v1, Wm, w.flags, w.nk);
  MX_LAUNCH_CHECK();
  nms_group_final_keys_kernel<<<nb, T, 0, s>>>(scores, group, w.flags, n, (int)G, w.k0, w.v0);
  MX_LAUNCH_CHECK();
  const uint64_t dead = ((uint64_t)G << 32) | 0xffffffffull;
  const int end2 = 32 + (64 - __builtin_clzll((unsigned long long)G));
  cb = w.cub_bytes;
  MX_HIP(hipcub::DeviceRadixSort::SortPairs(w.cub, cb, w.k0, w.k1, w.v0, w.v1, (int)n, 0, end2, s));
  nms_group_out_kernel<<<nb, T, 0, s>>>(w.k1, w.v1, n, dead, w.nk, keep, num_keep);
  MX_LAUNCH_CHECK();
  return MX_OK;
}
