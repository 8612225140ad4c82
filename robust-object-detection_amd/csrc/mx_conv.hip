// mx_conv.hip — NHWC implicit-GEMM convolution on gfx950 MFMA (bf16 in, f32 accumulate).
//
// Replaces the cuDNN convolutions the reference reaches through torchvision's
// fasterrcnn_resnet50_fpn_v2 (ResNet-50 body, FPN lateral/output convs, RPN head, box head convs,
// FC6/FC7 as 1x1 convs) and the U-Net (scripts/restoration_net.py:17-57):
//   fwd   y[m = (n,oh,ow)][k]  = sum_{r,s,c} x[n, oh*st-pad+r, ow*st-pad+s, c] * w[k][r][s][c]
//   dgrad dx[m = (n,h,w)][c]   = sum_{r,s,k} dy[n, (h+pad-r)/st, (w+pad-s)/st, k] * wt[c][r][s][k]
//         (only taps where the division is exact; wt = w transposed to [C][R][S][K])
//   wgrad dw[k][(r,s,c)]       = sum_{p = (n,oh,ow)} dy[p][k] * x[n, oh*st-pad+r, ow*st-pad+s, c]
//
// fwd/dgrad: 128 x BN x 64 block tile, 4 waves (2x2), each wave 64 x BN/2 via
// v_mfma_f32_16x16x32_bf16; A rows are gathered 16 B (8 channels) per lane straight from NHWC
// with zero-fill for padding, double-buffered through XOR-swizzled LDS (one barrier per K-tile);
// the epilogue reduces BatchNorm batch statistics from the f32 accumulators (per-block column
// partials, no atomics) and stages the tile through LDS for 16-byte coalesced NHWC stores with
// fused bias / residual / activation.
// wgrad: the GEMM's K dimension is the pixel axis, which is the strided axis of both NHWC operands;
// tiles are staged pixel-major (coalesced) and read transposed with ds_read_b64_tr_b16, split-K
// over pixels with f32 atomic accumulation.
#include "mx_common.h"
#include "mx_dma.h"

#include <vector>

namespace mx {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

static constexpr int BM = 128, BK = 64, NT = 256;

struct ConvP {
  const uint16_t* src;  // A source (x for fwd/wgrad-B, dy for dgrad)
  const uint16_t* wt;   // B [Ncol][Kdim], k contiguous
  int64_t M, Ncol, Kdim;
  int64_t OH, OW;       // row grid (n, oh, ow) of the GEMM rows
  int64_t IH, IW, IC;   // gathered source grid
  int R, S, st_h, st_w, pad_h, pad_w;
  // epilogue (residual / bnb_y / bnb_z: activation storage, bf16 or f32 per the kernel's TA)
  const float* bias;
  const void* residual;
  int act;
  void* out;
  int out_f32;
  float* stats;  // [2][mblocks][Ncol]
  int64_t mblocks;
  // split-K: every split writes its f32 partial tile to slab[split][M][Ncol]; a reduce kernel applies
  // the epilogue (slab == nullptr -> single pass, epilogue fused)
  float* slab;
  int splits;
  int64_t kt_per_split;
  // dgrad parity class: GEMM row m = (n, hh, ww) of the class grid stores to dx row
  // (n, st_h*hh + ph, st_w*ww + pw) of the full [N][H][W] grid
  int remap, rst_h, rst_w, rph, rpw;
  int64_t rH, rW;
  // element counts of the A source and of the B operand (buffer-descriptor ranges)
  int64_t src_elems, wt_elems;
  // bf16x3 (f32 activation) kernels: the lo plane of the split weight operand starts wt_plane
  // elements after the hi plane (wt)
  int64_t wt_plane;
  // K-tile order of the buffer-descriptor kernels: 0 tap-major (all channel chunks of a tap, then
  // the next tap), 1 channel-major (all taps of a 32-channel chunk, then the next chunk): the rows a
  // block gathers between two visits of the same cache line shrink from BMT full pixel rows to the
  // tap window of one chunk, so the re-reads across taps stay in L2
  int korder;
  int dbg_skip_epi;  // timing experiments only (mx_conv_set_debug): skip the bf16x3 buffer kernel's epilogue
  int aplanes;       // bf16x3 buffer kernel: A arrives as bf16 hi / lo planes (src = hi, lo at src + src_elems)
  // dgrad feeding a train-mode BatchNorm backward (mx_conv2d_dgrad_bnb): per 64-row block column
  // sums of g = bf16(dx) * act'(y) and g * (z - mean) * invstd -> bnb_part [2][mblocks64][Ncol]
  const void* bnb_y;
  const void* bnb_z;
  const float* bnb_mean;
  const float* bnb_invstd;
  float* bnb_part;
  int64_t bnb_mb;
  int bnb_act;
};

__device__ __forceinline__ float bnb_act_grad(float y, int act) {
  if (act == 1) return y > 0.f ? 1.f : 0.f;
  if (act == 2) return y > 0.f ? 1.f : 0.2f;
  return 1.f;
}

__device__ __forceinline__ int64_t out_row(const ConvP& p, int64_t m) {
  if (!p.remap) return m;
  const int64_t ww = m % p.OW, t = m / p.OW, hh = t % p.OH, n = t / p.OH;
  return (n * p.rH + hh * p.rst_h + p.rph) * p.rW + ww * p.rst_w + p.rpw;
}

__device__ __forceinline__ float act_f(float v, int act) {
  if (act == 1) return v > 0.f ? v : 0.f;
  if (act == 2) return v > 0.f ? v : 0.2f * v;
  return v;
}

// MODE 0 fwd: x[n, oh*st - pad + r, ow*st - pad + s]; MODE 1 dgrad of one stride-parity class
// (rows = the class's (n, hh, ww) grid, taps = the class's (ri, si), pad = the class offset dh/dw):
// dy[n, hh + dh - ri, ww + dw - si] — a dense stride-1 correlation, no wasted taps.
template <int MODE>
__device__ __forceinline__ bool gather_pos(const ConvP& p, int oh, int ow, int r, int s, int& ih, int& iw) {
  if (MODE == 0) {
    ih = oh * p.st_h - p.pad_h + r;
    iw = ow * p.st_w - p.pad_w + s;
  } else {
    ih = oh + p.pad_h - r;
    iw = ow + p.pad_w - s;
  }
  return ih >= 0 && iw >= 0 && ih < p.IH && iw < p.IW;
}

// Epilogue shared by the fwd/dgrad kernels: BN statistics from the f32 accumulators, then the tile
// staged through LDS (after the last K-tile's barrier) for 16-B coalesced NHWC stores with fused
// bias / residual / activation.
// BMT = block tile rows (128 or 64; each wave-row wm covers BMT/2 rows, TI = BMT/32 MFMA row
// tiles). HALVES == 2 stages the f32 tile in two passes of BMT/2 rows (half the LDS: lets the
// multi-stage kernel keep 3 blocks per CU). BatchNorm statistics partials have 64-row
// granularity: stats[2][ceil(M/64)][Ncol] (row = m / 64).
static constexpr int SROWS = 64;

// WR = wave-rows of the block (2: 4 waves in 2x2, 4: 8 waves in 4x2; HALVES == WR then stages one
// wave-row per pass).
// WC = wave-columns (2: wave tiles of BN/2 columns; 1: each wave spans all BN columns).
template <int BN, int HALVES = 1, int BMT = BM, typename TA = uint16_t, int WR = 2, int WC = 2, bool GROUP = false>
__device__ __forceinline__ void conv_epilogue(const ConvP& p, f32x4 (&acc)[BMT / (16 * WR)][BN / (16 * WC)],
                                              char* smem, int64_t m0, int64_t n0, int64_t mt, int wm, int wn,
                                              int lane, int tid, int split) {
  constexpr int WN = BN / WC, TJ = WN / 16, WM = BMT / WR, TI = WM / 16, NT = 64 * WR * WC;
  constexpr int PR = BMT / HALVES;  // rows staged per pass
  static_assert(HALVES == 1 || HALVES == WR, "staging: the whole tile at once, or one wave-row per pass");
  static_assert(WM == SROWS || (SROWS % WM == 0 && WR * WM >= SROWS), "wave-rows of 64, 32 or 16 rows");
  (void)mt;
  if (p.slab) {  // split-K partial: f32 tile to the slab, epilogue deferred to the reduce kernel
    constexpr int LD = BN + 4;
    float* Ct = (float*)smem;
    float* dst = p.slab + (int64_t)split * p.M * p.Ncol;
    constexpr int CPR = BN / 4;
#pragma unroll
    for (int h = 0; h < HALVES; ++h) {
      if (HALVES == 1 || wm == h) {
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              Ct[((HALVES == 1 ? wm * WM : 0) + i * 16 + (lane >> 4) * 4 + r) * LD + wn * WN + j * 16 + (lane & 15)] =
                  acc[i][j][r];
      }
      __syncthreads();
      for (int e = tid; e < PR * CPR; e += NT) {
        int row = e / CPR, cc = (e % CPR) * 4;
        int64_t m = m0 + h * PR + row, col0 = n0 + cc;
        if (m < p.M && col0 < p.Ncol) *(float4*)(dst + m * p.Ncol + col0) = *(const float4*)&Ct[row * LD + cc];
      }
      if (HALVES > 1) __syncthreads();
    }
    return;
  }
  // ---- BatchNorm batch statistics from the f32 accumulators --------------------------------
  // C/D map (16x16): col = lane & 15, row = (lane >> 4) * 4 + reg
  if (p.stats) {
    float* red = (float*)smem;  // [WR wm][2 (sum,sq)][BN]
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int64_t m = m0 + wm * WM + i * 16 + (lane >> 4) * 4 + r;
          float v = m < p.M ? acc[i][j][r] : 0.f;
          s += v;
          q += v * v;
        }
      s += __shfl_xor(s, 16); q += __shfl_xor(q, 16);
      s += __shfl_xor(s, 32); q += __shfl_xor(q, 32);
      if (lane < 16) {
        int col = wn * WN + j * 16 + lane;
        red[(wm * 2 + 0) * BN + col] = s;
        red[(wm * 2 + 1) * BN + col] = q;
      }
    }
    __syncthreads();
    const int64_t srow = m0 / SROWS;
    constexpr int WPS = WM >= SROWS ? 1 : SROWS / WM;  // wave-rows per 64-row statistics row
    for (int c = tid; c < BN; c += NT) {
      int64_t col = n0 + c;
      if (col >= p.Ncol) continue;
#pragma unroll
      for (int g = 0; g < WR / WPS; ++g)
        if (m0 + g * SROWS < p.M) {
          float sg = red[(g * WPS * 2) * BN + c], qg = red[(g * WPS * 2 + 1) * BN + c];
#pragma unroll
          for (int w = g * WPS + 1; w < (g + 1) * WPS; ++w) {
            sg += red[(w * 2) * BN + c];
            qg += red[(w * 2 + 1) * BN + c];
          }
          p.stats[(srow + g) * p.Ncol + col] = sg;
          p.stats[(p.mblocks + srow + g) * p.Ncol + col] = qg;
        }
    }
    __syncthreads();
  }

  // ---- stage the f32 tile through LDS, then coalesced NHWC stores ---------------------------
  constexpr int LD = BN + 4;  // padded row (floats), keeps 16-B alignment
  float* Ct = (float*)smem;
  constexpr int CPR = BN / 8;  // 8-column chunks per row
  constexpr int RL = NT / CPR;  // row lanes: a thread's column chunk (tid % CPR) is fixed
  const bool vec = (p.Ncol % 8) == 0;
  // BN-backward partials (bnb): this thread's 8 columns, accumulated over its rows of a 64-row group
  constexpr int BG = BMT / SROWS;  // 64-row statistics groups per tile
  float bs[BG][8] = {}, bq[BG][8] = {}, bmu[8], bis[8];
  const int64_t bcol0 = n0 + (tid % CPR) * 8;
  if (p.bnb_part) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      bmu[t] = bcol0 + t < p.Ncol ? p.bnb_mean[bcol0 + t] : 0.f;
      bis[t] = bcol0 + t < p.Ncol ? p.bnb_invstd[bcol0 + t] : 0.f;
    }
  }
  auto bnb_flush = [&](int gi) {  // LDS reduce over the RL row lanes, one partial row per 64 rows
    float* red = (float*)smem;       // [2][RL][BN] (aliases the drained staging tile)
    __syncthreads();
    const int rl = tid / CPR, cc = (tid % CPR) * 8;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      red[(0 * RL + rl) * BN + cc + t] = bs[gi][t];
      red[(1 * RL + rl) * BN + cc + t] = bq[gi][t];
    }
    __syncthreads();
    for (int c = tid; c < 2 * BN; c += NT) {
      const int w = c / BN, col = c % BN;
      float a = 0.f;
      for (int r = 0; r < RL; ++r) a += red[(w * RL + r) * BN + col];
      const int64_t srow = m0 / SROWS + gi;
      if (n0 + col < p.Ncol && srow * SROWS < p.M) p.bnb_part[(w * p.bnb_mb + srow) * p.Ncol + n0 + col] = a;
    }
    __syncthreads();
  };
#pragma unroll
  for (int h = 0; h < HALVES; ++h) {
  if (HALVES == 1 || wm == h) {
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int row = (HALVES == 1 ? wm * WM : 0) + i * 16 + (lane >> 4) * 4 + r;
          int col = wn * WN + j * 16 + (lane & 15);
          Ct[row * LD + col] = acc[i][j][r];
        }
  }
  __syncthreads();
  if constexpr (GROUP) {  // f32 (bf16x3) dgrad kernels
  // rows of the staged tile in groups of EU: every global operand of the group (residual, the BN
  // backward's y / z) is loaded before any of its rows is finished, so a thread waits one memory
  // round trip per group instead of one per row (the memory-bound 1x1 dgrads with BN-backward
  // epilogues were latency-bound here). Per element the arithmetic and its order are unchanged.
  constexpr int ITER = (PR * CPR + NT - 1) / NT;
  constexpr int EU = ITER < 2 ? ITER : 2;
  for (int k0 = 0; k0 < ITER; k0 += EU) {
    float rr[EU][8], yy[EU][8], zz[EU][8];
    int64_t mm[EU], cc0[EU];
    int rw[EU];
    bool ok[EU];
#pragma unroll
    for (int u = 0; u < EU; ++u) {
      const int e = tid + (k0 + u) * NT;
      const int row = e / CPR, cc = (e % CPR) * 8;
      int64_t m = m0 + h * PR + row;
      const int64_t col0 = n0 + cc;
      ok[u] = k0 + u < ITER && e < PR * CPR && m < p.M && col0 < p.Ncol;
      rw[u] = row;
      cc0[u] = col0;
      mm[u] = ok[u] ? out_row(p, m) : 0;
      if (ok[u] && vec) {
        if (p.residual) ld8((const TA*)p.residual + mm[u] * p.Ncol + col0, rr[u]);
        if (sizeof(TA) == 4 && p.out_f32 && p.bnb_part) {
          ld8((const TA*)p.bnb_y + mm[u] * p.Ncol + col0, yy[u]);
          ld8((const TA*)p.bnb_z + mm[u] * p.Ncol + col0, zz[u]);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < EU; ++u) {
      if (!ok[u]) continue;
      const int row = rw[u];
      const int64_t m = mm[u], col0 = cc0[u];
      const int cc = (int)(col0 - n0);
      float v[8];
      *(float4*)&v[0] = *(const float4*)&Ct[row * LD + cc];
      *(float4*)&v[4] = *(const float4*)&Ct[row * LD + cc + 4];
      if (vec) {
        if (p.bias) {
#pragma unroll
          for (int t = 0; t < 8; ++t) v[t] += p.bias[col0 + t];
        }
        if (p.residual) {
#pragma unroll
          for (int t = 0; t < 8; ++t) v[t] += rr[u][t];
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] = act_f(v[t], p.act);
        if (p.out_f32) {
          float* o = (float*)p.out + m * p.Ncol + col0;
          *(float4*)o = *(float4*)&v[0];
          *(float4*)(o + 4) = *(float4*)&v[4];
          if (sizeof(TA) == 4 && p.bnb_part) {  // f32 activations: the stored gradient is v itself
            const int gi = BG == 1 ? 0 : (int)((h * PR + row) / SROWS);
#pragma unroll
            for (int t = 0; t < 8; ++t) {
              const float g = v[t] * bnb_act_grad(yy[u][t], p.bnb_act);
              bs[gi][t] += g;
              bq[gi][t] += g * ((zz[u][t] - bmu[t]) * bis[t]);
            }
          }
        } else {
          uint4 w;
          uint16_t* wh = (uint16_t*)&w;
#pragma unroll
          for (int t = 0; t < 8; ++t) wh[t] = f2bf(v[t]);
          *(uint4*)((uint16_t*)p.out + m * p.Ncol + col0) = w;
          if (p.bnb_part) {  // the stored (bf16-rounded) gradient, as a separate reduce would read it
            const uint4 yb = *(const uint4*)((const uint16_t*)p.bnb_y + m * p.Ncol + col0);
            const uint4 zb = *(const uint4*)((const uint16_t*)p.bnb_z + m * p.Ncol + col0);
            const uint16_t *yh = (const uint16_t*)&yb, *zh = (const uint16_t*)&zb;
            const int gi = BG == 1 ? 0 : (int)((h * PR + row) / SROWS);
#pragma unroll
            for (int t = 0; t < 8; ++t) {
              const float g = bf2f(wh[t]) * bnb_act_grad(bf2f(yh[t]), p.bnb_act);
              bs[gi][t] += g;
              bq[gi][t] += g * ((bf2f(zh[t]) - bmu[t]) * bis[t]);
            }
          }
        }
      } else {
        for (int t = 0; t < 8 && col0 + t < p.Ncol; ++t) {
          float x = v[t];
          if (p.bias) x += p.bias[col0 + t];
          if (p.residual) x += ld1((const TA*)p.residual + m * p.Ncol + col0 + t);
          x = act_f(x, p.act);
          if (p.out_f32) ((float*)p.out)[m * p.Ncol + col0 + t] = x;
          else ((uint16_t*)p.out)[m * p.Ncol + col0 + t] = f2bf(x);
        }
      }
    }
  }
  } else {  // one row at a time: the forward (no residual / BN-backward operands) and the bf16
           // kernels (whose 3-blocks-per-CU register budget has no room for a second row's), and
           // fewer registers beside the side-stream wgrad
  for (int e = tid; e < PR * CPR; e += NT) {
    int row = e / CPR, cc = (e % CPR) * 8;
    int64_t m = m0 + h * PR + row, col0 = n0 + cc;
    if (m >= p.M || col0 >= p.Ncol) continue;
    m = out_row(p, m);
    float v[8];
    *(float4*)&v[0] = *(const float4*)&Ct[row * LD + cc];
    *(float4*)&v[4] = *(const float4*)&Ct[row * LD + cc + 4];
    if (vec) {
      if (p.bias) {
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] += p.bias[col0 + t];
      }
      if (p.residual) {
        float rr[8];
        ld8((const TA*)p.residual + m * p.Ncol + col0, rr);
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] += rr[t];
      }
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = act_f(v[t], p.act);
      if (p.out_f32) {
        float* o = (float*)p.out + m * p.Ncol + col0;
        *(float4*)o = *(float4*)&v[0];
        *(float4*)(o + 4) = *(float4*)&v[4];
        if (sizeof(TA) == 4 && p.bnb_part) {  // f32 activations: the stored gradient is v itself
          float yy[8], zz[8];
          ld8((const TA*)p.bnb_y + m * p.Ncol + col0, yy);
          ld8((const TA*)p.bnb_z + m * p.Ncol + col0, zz);
          const int gi = BG == 1 ? 0 : (int)((h * PR + row) / SROWS);
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            const float g = v[t] * bnb_act_grad(yy[t], p.bnb_act);
            bs[gi][t] += g;
            bq[gi][t] += g * ((zz[t] - bmu[t]) * bis[t]);
          }
        }
      } else {
        uint4 w;
        uint16_t* wh = (uint16_t*)&w;
#pragma unroll
        for (int t = 0; t < 8; ++t) wh[t] = f2bf(v[t]);
        *(uint4*)((uint16_t*)p.out + m * p.Ncol + col0) = w;
        if (p.bnb_part) {  // the stored (bf16-rounded) gradient, as a separate reduce would read it
          const uint4 yy = *(const uint4*)((const uint16_t*)p.bnb_y + m * p.Ncol + col0);
          const uint4 zz = *(const uint4*)((const uint16_t*)p.bnb_z + m * p.Ncol + col0);
          const uint16_t *yh = (const uint16_t*)&yy, *zh = (const uint16_t*)&zz;
          const int gi = BG == 1 ? 0 : (int)((h * PR + row) / SROWS);
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            const float g = bf2f(wh[t]) * bnb_act_grad(bf2f(yh[t]), p.bnb_act);
            bs[gi][t] += g;
            bq[gi][t] += g * ((bf2f(zh[t]) - bmu[t]) * bis[t]);
          }
        }
      }
    } else {
      for (int t = 0; t < 8 && col0 + t < p.Ncol; ++t) {
        float x = v[t];
        if (p.bias) x += p.bias[col0 + t];
        if (p.residual) x += ld1((const TA*)p.residual + m * p.Ncol + col0 + t);
        x = act_f(x, p.act);
        if (p.out_f32) ((float*)p.out)[m * p.Ncol + col0 + t] = x;
        else ((uint16_t*)p.out)[m * p.Ncol + col0 + t] = f2bf(x);
      }
    }
  }
  }
  if (HALVES > 1) __syncthreads();
  }
  if (p.bnb_part) {
#pragma unroll
    for (int gi = 0; gi < BG; ++gi) bnb_flush(gi);
  }
}

template <int BN, int MODE>
__global__ void __launch_bounds__(NT, 2) conv_igemm_kernel(ConvP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int WN = BN / 2;          // columns per wave
  constexpr int TJ = WN / 16;         // 16-wide tiles per wave in N
  constexpr int BCH = BN * 8 / NT;    // B chunks per thread (4 or 2)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  const int64_t ntiles_n = (p.Ncol + BN - 1) / BN;
  const int64_t nwg = (int64_t)gridDim.x;
  const int64_t bid = xcd_remap(blockIdx.x, nwg);
  const int64_t mt = bid / ntiles_n, nt = bid % ntiles_n;
  const int64_t m0 = mt * BM, n0 = nt * BN;

  // per-thread A rows: row = (tid>>3) + 32*i, chunk kc = tid&7
  const int kc = tid & 7;
  int a_n[4], a_oh[4], a_ow[4];
  bool a_ok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int64_t m = m0 + (tid >> 3) + 32 * i;
    a_ok[i] = m < p.M;
    int64_t mm = a_ok[i] ? m : 0;
    a_ow[i] = (int)(mm % p.OW);
    int64_t t = mm / p.OW;
    a_oh[i] = (int)(t % p.OH);
    a_n[i] = (int)(t / p.OH);
  }
  const int64_t nk = (p.Kdim + BK - 1) / BK;

  uint4 ra[4], rb[BCH];
  auto load_tile = [&](int64_t kt) {
    const int64_t k = kt * BK + kc * 8;
    const bool kin = k < p.Kdim;
    const int tap = (int)(k / p.IC);
    const int c = (int)(k - (int64_t)tap * p.IC);
    const int r = tap / p.S, s = tap - (tap / p.S) * p.S;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int ih, iw;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (kin && a_ok[i] && gather_pos<MODE>(p, a_oh[i], a_ow[i], r, s, ih, iw))
        v = *(const uint4*)(p.src + (((int64_t)a_n[i] * p.IH + ih) * p.IW + iw) * p.IC + c);
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      int64_t n = n0 + (tid >> 3) + 32 * i;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (kin && n < p.Ncol) v = *(const uint4*)(p.wt + n * p.Kdim + k);
      rb[i] = v;
    }
  };
  auto store_tile = [&](int buf) {
    char* A = smem + buf * STAGE;
    char* B = A + A_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int row = (tid >> 3) + 32 * i;
      *(uint4*)(A + row * (BK * 2) + ((kc ^ (row & 7)) << 4)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      int row = (tid >> 3) + 32 * i;
      *(uint4*)(B + row * (BK * 2) + ((kc ^ (row & 7)) << 4)) = rb[i];
    }
  };

  f32x4 acc[4][TJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (int64_t kt = 0; kt < nk; ++kt) {
    const int buf = (int)(kt & 1);
    if (kt + 1 < nk) load_tile(kt + 1);
    const char* A = smem + buf * STAGE;
    const char* B = A + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = ks * 4 + (lane >> 4);
      bf16x8 af[4], bfr[TJ];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int row = wm * 64 + i * 16 + (lane & 15);
        af[i] = *(const bf16x8*)(A + row * (BK * 2) + ((ch ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        int row = wn * WN + j * 16 + (lane & 15);
        bfr[j] = *(const bf16x8*)(B + row * (BK * 2) + ((ch ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tile(buf ^ 1);
    __syncthreads();
  }

  conv_epilogue<BN>(p, acc, smem, m0, n0, mt, wm, wn, lane, tid, 0);
}

// ------------------------------------------------------------------------------------------------
// Same GEMM as conv_igemm_kernel, staged with direct-to-LDS loads (global_load_lds_dwordx4): each
// wave instruction lands 64 x 16 B = 8 tile rows x 128 B in LDS; the XOR swizzle moves to the
// per-lane SOURCE address (logical chunk = physical ^ (row & 7)); padding / out-of-range lanes read a
// zero page. No staging registers, no ds_write pass.
__device__ uint4 g_zero_page[4];

template <int BN, int MODE>
__global__ void __launch_bounds__(NT, 2) conv_igemm_glds_kernel(ConvP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int WN = BN / 2, TJ = WN / 16;
  constexpr int BI = BN / 32;  // B instructions per wave (BN/4 rows per wave, 8 rows each)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t ntiles_n = (p.Ncol + BN - 1) / BN;
  const int64_t gid = xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  const int split = (int)(gid % p.splits);
  const int64_t bid = gid / p.splits;  // the splits of one tile run on one XCD (shared A/B lines in L2)
  const int64_t mt = bid / ntiles_n, nt = bid % ntiles_n;
  const int64_t m0 = mt * BM, n0 = nt * BN;
  const int lrow = lane >> 3;
  const int lch = (lane & 7) ^ lrow;  // logical 16-B chunk this lane fetches (rows are 8-aligned)
  int a_n[4], a_oh[4], a_ow[4];
  bool a_ok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int64_t m = m0 + wave * 32 + i * 8 + lrow;
    a_ok[i] = m < p.M;
    int64_t mm = a_ok[i] ? m : 0;
    a_ow[i] = (int)(mm % p.OW);
    int64_t t = mm / p.OW;
    a_oh[i] = (int)(t % p.OH);
    a_n[i] = (int)(t / p.OH);
  }
  const uint16_t* zero = (const uint16_t*)g_zero_page;
  const int64_t nk = (p.Kdim + BK - 1) / BK;
  auto issue = [&](int64_t kt, int buf) {
    char* A = smem + buf * STAGE;
    char* B = A + A_BYTES;
    const int64_t k = kt * BK + lch * 8;
    const bool kin = k < p.Kdim;
    const int tap = (int)(k / p.IC);
    const int c = (int)(k - (int64_t)tap * p.IC);
    const int r = tap / p.S, s = tap - (tap / p.S) * p.S;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int ih, iw;
      const uint16_t* src = zero;
      if (kin && a_ok[i] && gather_pos<MODE>(p, a_oh[i], a_ow[i], r, s, ih, iw))
        src = p.src + (((int64_t)a_n[i] * p.IH + ih) * p.IW + iw) * p.IC + c;
      __builtin_amdgcn_global_load_lds((const void*)src, (LDS_AS void*)(A + (wave * 32 + i * 8) * (BK * 2)), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int row = wave * (BN / 4) + i * 8;
      const int64_t n = n0 + row + lrow;
      const uint16_t* src = (kin && n < p.Ncol) ? p.wt + n * p.Kdim + k : zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (LDS_AS void*)(B + row * (BK * 2)), 16, 0, 0);
    }
  };
  f32x4 acc[4][TJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int64_t kbeg = (int64_t)split * p.kt_per_split;
  const int64_t kend = min<int64_t>(nk, kbeg + p.kt_per_split);
  issue(kbeg, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int64_t kt = kbeg; kt < kend; ++kt) {
    const int buf = (int)((kt - kbeg) & 1);
    if (kt + 1 < kend) issue(kt + 1, buf ^ 1);
    const char* A = smem + buf * STAGE;
    const char* B = A + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = ks * 4 + (lane >> 4);
      bf16x8 af[4], bfr[TJ];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int row = wm * 64 + i * 16 + (lane & 15);
        af[i] = *(const bf16x8*)(A + row * (BK * 2) + ((ch ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        int row = wn * WN + j * 16 + (lane & 15);
        bfr[j] = *(const bf16x8*)(B + row * (BK * 2) + ((ch ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  conv_epilogue<BN>(p, acc, smem, m0, n0, mt, wm, wn, lane, tid, split);
}

// ------------------------------------------------------------------------------------------------
// Multi-stage direct-to-LDS variant: BKT-wide K-tiles (32 or 64), STAGES-deep LDS ring with
// STAGES-1 tiles in flight. One barrier per K-tile; the wait before it is a counted vmcnt that leaves
// the younger tiles' loads outstanding across the barrier, so HBM/L2 latency overlaps the MFMAs of
// STAGES-2 further tiles. With BKT = 32 a tile row is 64 B: an instruction lands 16 rows and the
// swizzle (phys chunk = logical ^ (row & 4 ? 2 : 0)) keeps the 16-lane ds_read_b128 groups
// conflict-free. The epilogue stages the tile in two 64-row halves (LDS = max(ring, 33.8 KB)).
template <int CPR>
__device__ __forceinline__ int tile_swz(int row) {
  if (CPR == 8) return row & 7;
  return (row >> 1) & 2;
}

__device__ __forceinline__ void block_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int BN, int MODE, int BKT, int STAGES, int OCC, int BMT = BM>
__global__ void __launch_bounds__(NT, OCC) conv_igemm_pipe_kernel(ConvP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int RB = BKT * 2;          // bytes per tile row
  constexpr int CPR = BKT / 8;         // 16-B chunks per row
  constexpr int RPI = 64 / CPR;        // rows landed per wave instruction (8 or 16)
  constexpr int AR = BMT / 4;          // A rows landed per wave
  constexpr int AI = AR / RPI;         // A instructions per wave
  constexpr int BI = (BN / 4) / RPI;   // B instructions per wave
  constexpr int LOADS = AI + BI;       // vmem instructions per K-tile per wave
  constexpr int A_BYTES = BMT * RB, STAGE = (BMT + BN) * RB;
  constexpr int WN = BN / 2, TJ = WN / 16, KS = BKT / 32, WM = BMT / 2, TI = WM / 16;
  static_assert(AI >= 1 && BI >= 1 && KS >= 1 && STAGES >= 2, "tile shape");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t ntiles_n = (p.Ncol + BN - 1) / BN;
  const int64_t gid = xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  const int split = (int)(gid % p.splits);
  const int64_t bid = gid / p.splits;
  const int64_t mt = bid / ntiles_n, nt = bid % ntiles_n;
  const int64_t m0 = mt * BMT, n0 = nt * BN;
  const int lrow = lane / CPR;
  const int lch = (lane % CPR) ^ tile_swz<CPR>(lrow);  // instruction row bases are RPI-aligned
  // per A row: gather origin (h0, w0) and its pixel index; tap (r, s) moves it by +-(r, s)
  // (MODE 0: ih = oh*st - pad + r; MODE 1: ih = hh + dh - r)
  const int IH = (int)p.IH, IW = (int)p.IW;
  int a_h0[AI], a_w0[AI];
  int64_t a_pix[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    int64_t m = m0 + wave * AR + i * RPI + lrow;
    const bool ok = m < p.M;
    int64_t mm = ok ? m : 0;
    const int ow = (int)(mm % p.OW);
    int64_t t = mm / p.OW;
    const int oh = (int)(t % p.OH);
    const int n = (int)(t / p.OH);
    a_h0[i] = MODE == 0 ? oh * p.st_h - p.pad_h : oh + p.pad_h;
    a_w0[i] = MODE == 0 ? ow * p.st_w - p.pad_w : ow + p.pad_w;
    if (!ok) a_h0[i] = -(1 << 28);  // never in range
    a_pix[i] = ((int64_t)n * IH + a_h0[i]) * IW + a_w0[i];
  }
  const uint16_t* zero = (const uint16_t*)g_zero_page;
  const int64_t nk = (p.Kdim + BKT - 1) / BKT;
  const int64_t kbeg = (int64_t)split * p.kt_per_split;
  const int64_t ntk = min<int64_t>(nk, kbeg + p.kt_per_split) - kbeg;
  // this lane's K position (k = kt*BKT + lch*8 -> tap (r, s), channel c), advanced incrementally:
  // tiles are issued strictly in order, so no per-tile division
  const int IC = (int)p.IC, Kd = (int)p.Kdim;
  int ik = (int)(kbeg * BKT) + lch * 8;
  int ic_c, ic_r, ic_s;
  {
    const int tap = ik / IC;
    ic_c = ik - tap * IC;
    ic_r = tap / p.S;
    ic_s = tap - ic_r * p.S;
  }
  auto issue = [&](int buf) {
    char* A = smem + buf * STAGE;
    char* B = A + A_BYTES;
    const int k = ik;
    const bool kin = k < Kd;
    const int c = ic_c, r = ic_r, s = ic_s;
    ik += BKT;
    ic_c += BKT;
    while (ic_c >= IC) {
      ic_c -= IC;
      if (++ic_s == p.S) { ic_s = 0; ++ic_r; }
    }
    const int dr = MODE == 0 ? r : -r, ds = MODE == 0 ? s : -s;
    const int64_t toff = (int64_t)dr * IW + ds;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int ih = a_h0[i] + dr, iw = a_w0[i] + ds;
      const uint16_t* src = zero;
      if (kin && (unsigned)ih < (unsigned)IH && (unsigned)iw < (unsigned)IW) src = p.src + (a_pix[i] + toff) * IC + c;
      __builtin_amdgcn_global_load_lds((const void*)src, (LDS_AS void*)(A + (wave * AR + i * RPI) * RB), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int row = wave * (BN / 4) + i * RPI;
      const int64_t n = n0 + row + lrow;
      const uint16_t* src = (kin && n < p.Ncol) ? p.wt + n * p.Kdim + k : zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (LDS_AS void*)(B + row * RB), 16, 0, 0);
    }
  };
  f32x4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int st = 0; st < STAGES - 1; ++st)
    if (st < ntk) issue(st);
  for (int64_t t = 0; t < ntk; ++t) {
    // tile t landed (this wave's part): the younger STAGES-2 tiles may stay in flight
    if (t + STAGES - 2 < ntk) wait_vmcnt<LOADS * (STAGES - 2)>();
    else wait_vmcnt<0>();
    block_barrier();  // ... and every wave's part; all waves are done reading tile t-1's buffer
    if (t + STAGES - 1 < ntk) issue((int)((t + STAGES - 1) % STAGES));
    const char* A = smem + (int)(t % STAGES) * STAGE;
    const char* B = A + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int ch = ks * 4 + (lane >> 4);
      bf16x8 af[TI], bfr[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        int row = wm * WM + i * 16 + (lane & 15);
        af[i] = *(const bf16x8*)(A + row * RB + ((ch ^ tile_swz<CPR>(row)) << 4));
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        int row = wn * WN + j * 16 + (lane & 15);
        bfr[j] = *(const bf16x8*)(B + row * RB + ((ch ^ tile_swz<CPR>(row)) << 4));
      }
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();  // last tile's buffer is reused by the epilogue staging
  conv_epilogue<BN, 2, BMT>(p, acc, smem, m0, n0, mt, wm, wn, lane, tid, split);
}

// ------------------------------------------------------------------------------------------------
// Buffer-descriptor variant of conv_igemm_pipe_kernel (BKT = 32, IC % 32 == 0, R*S <= 64): a 32-wide
// K-tile lies inside one tap, so the tap (r, s) and channel offset are wave-uniform and ride in the
// SGPR soffset of buffer_load_dwordx4 ... lds; every lane keeps a loop-invariant 32-bit voffset per
// A row / B row. Padding taps come from a per-row 64-bit validity mask (one bit per tap): an
// invalid row points its voffset past the descriptor's range, so the hardware range check returns
// zeros (no zero page, no per-tile 64-bit address arithmetic). Same LDS ring, MFMA loop and
// epilogue as the pipe kernel.
static constexpr uint32_t kOOB = 0x80000000u;

// Wave-uniform K position (tap row cr, tap column cq, channel chunk cc) of the buffer kernels' next
// K-tile, advanced in value form: both K-tile orders computed branch-free and selected. A branchy
// update (`if (++cq == S) ...` / `else if ((cc += BKT) == IC) ...`) let the compiler merge the two
// branches' stores into one store through a selected address, which kept the counters in scratch
// memory (a scratch load plus a vmcnt drain per K-tile, i.e. a wait for the ring's own LDS-DMA) and
// made the B operand's soffset look divergent (a readfirstlane waterfall loop around every load).
struct KPos {
  int cc, cr, cq;
  __device__ __forceinline__ void init(int korder, int kb, int R, int S, int IC, int bkt) {
    const int RS = R * S;
    const int ctap = korder ? kb % RS : kb * bkt / IC;
    cc = korder ? kb / RS * bkt : kb * bkt - ctap * IC;
    cr = ctap / S;
    cq = ctap - cr * S;
  }
  __device__ __forceinline__ void advance(int korder, int R, int S, int IC, int bkt) {
    // korder 1 (channel-major): q, then r, then the channel chunk
    const int q1 = cq + 1;
    const int wq = q1 == S ? 1 : 0;
    const int r1 = cr + wq;
    const int wr = (wq && r1 == R) ? 1 : 0;
    const int a_cq = wq ? 0 : q1, a_cr = wr ? 0 : r1, a_cc = cc + (wr ? bkt : 0);
    // korder 0 (tap-major): the channel chunk, then q, then r
    const int c1 = cc + bkt;
    const int wc = c1 == IC ? 1 : 0;
    const int q0 = cq + wc;
    const int wq0 = (wc && q0 == S) ? 1 : 0;
    const int b_cc = wc ? 0 : c1, b_cq = wq0 ? 0 : q0, b_cr = cr + wq0;
    cc = korder ? a_cc : b_cc;
    cr = korder ? a_cr : b_cr;
    cq = korder ? a_cq : b_cq;
  }
};

template <int BN, int MODE, int STAGES, int OCC, int BMT = BM>
__global__ void __launch_bounds__(NT, OCC) conv_igemm_buf_kernel(ConvP p) {
#if defined(__HIP_DEVICE_COMPILE__)  // buffer-resource builtins exist only in the device pass
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BKT = 32, RB = BKT * 2, CPR = BKT / 8, RPI = 64 / CPR;
  constexpr int AR = BMT / 4, AI = AR / RPI, BI = (BN / 4) / RPI, LOADS = AI + BI;
  constexpr int A_BYTES = BMT * RB, STAGE = (BMT + BN) * RB;
  constexpr int WN = BN / 2, TJ = WN / 16, WM = BMT / 2, TI = WM / 16;
  static_assert(AI >= 1 && BI >= 1 && STAGES >= 2, "tile shape");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t ntiles_n = (p.Ncol + BN - 1) / BN;
  const int64_t gid = xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  const int split = (int)(gid % p.splits);
  const int64_t bid = gid / p.splits;
  const int64_t mt = bid / ntiles_n, nt = bid % ntiles_n;
  const int64_t m0 = mt * BMT, n0 = nt * BN;
  const int lrow = lane / CPR;
  const int lch = (lane % CPR) ^ tile_swz<CPR>(lrow);
  const int IH = (int)p.IH, IW = (int)p.IW, IC = (int)p.IC, R = p.R, S = p.S;
  // A rows: origin pixel offset (elements) and tap validity mask
  uint32_t a_voff[AI];
  uint64_t a_mask[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int64_t m = m0 + wave * AR + i * RPI + lrow;
    uint64_t mask = 0;
    int32_t off = 0;
    if (m < p.M) {
      const int ow = (int)(m % p.OW);
      const int64_t t = m / p.OW;
      const int oh = (int)(t % p.OH);
      const int n = (int)(t / p.OH);
      // MODE 0: ih = oh*st - pad + r; MODE 1: ih = hh + dh - ri = (hh + dh - (R-1)) + (R-1-ri)
      const int h0 = MODE == 0 ? oh * p.st_h - p.pad_h : oh + p.pad_h - (R - 1);
      const int w0 = MODE == 0 ? ow * p.st_w - p.pad_w : ow + p.pad_w - (S - 1);
      off = ((n * IH + h0) * IW + w0) * IC + lch * 8;
      for (int r = 0; r < R; ++r)
        for (int q = 0; q < S; ++q) {
          // tap index in the B column order; its source row/col offset (rr, qq) from the origin
          const int rr = MODE == 0 ? r : R - 1 - r, qq = MODE == 0 ? q : S - 1 - q;
          if ((unsigned)(h0 + rr) < (unsigned)IH && (unsigned)(w0 + qq) < (unsigned)IW) mask |= 1ull << (r * S + q);
        }
    }
    a_voff[i] = (uint32_t)off * 2u;
    a_mask[i] = mask;
  }
  uint32_t b_voff[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int64_t n = n0 + wave * (BN / 4) + i * RPI + lrow;
    b_voff[i] = n < p.Ncol ? (uint32_t)((n * p.Kdim + lch * 8) * 2) : kOOB;
  }
  const i32x4 arsrc = dma_rsrc(p.src, (uint32_t)(p.src_elems * 2));
  const i32x4 brsrc = dma_rsrc(p.wt, (uint32_t)(p.wt_elems * 2));
  const uint32_t lds0 = lds_addr(smem);
  const int64_t nk = p.Kdim / BKT;
  const int64_t kbeg = (int64_t)split * p.kt_per_split;
  const int64_t ntk = min<int64_t>(nk, kbeg + p.kt_per_split) - kbeg;
  // wave-uniform K position of the next tile to issue: tap (r, q), channel c (p.korder: K-tile order)
  const int korder = __builtin_amdgcn_readfirstlane(p.korder);
  KPos kp;
  kp.init(korder, (int)kbeg, R, S, IC, BKT);
  auto issue = [&](int buf) {
    const uint32_t A = lds0 + buf * STAGE;
    const uint32_t B = A + A_BYTES;
    const int cr = kp.cr, cq = kp.cq, cc = kp.cc;
    const int rr = MODE == 0 ? cr : R - 1 - cr, qq = MODE == 0 ? cq : S - 1 - cq;
    const uint32_t a_soff = (uint32_t)(((rr * IW + qq) * IC + cc) * 2);
    const int tap = cr * S + cq;
    const uint32_t b_soff = (uint32_t)__builtin_amdgcn_readfirstlane((int)((tap * IC + cc) * 2));
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      // the whole offset in voffset (the origin may be negative; the tap offset brings it in range)
      const uint32_t v = ((a_mask[i] >> tap) & 1ull) ? a_voff[i] + a_soff : kOOB;
      lds_dma16(arsrc, A + (wave * AR + i * RPI) * RB, v, 0u);
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) lds_dma16(brsrc, B + (wave * (BN / 4) + i * RPI) * RB, b_voff[i], b_soff);
    kp.advance(korder, R, S, IC, BKT);
  };
  f32x4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int st = 0; st < STAGES - 1; ++st)
    if (st < ntk) issue(st);
  for (int64_t t = 0; t < ntk; ++t) {
    if (t + STAGES - 2 < ntk) wait_vmcnt<LOADS * (STAGES - 2)>();
    else wait_vmcnt<0>();
    block_barrier();
    if (t + STAGES - 1 < ntk) issue((int)((t + STAGES - 1) % STAGES));
    const char* A = smem + (int)(t % STAGES) * STAGE;
    const char* B = A + A_BYTES;
    const int ch = lane >> 4;
    bf16x8 af[TI], bfr[TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      int row = wm * WM + i * 16 + (lane & 15);
      af[i] = *(const bf16x8*)(A + row * RB + ((ch ^ tile_swz<CPR>(row)) << 4));
    }
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      int row = wn * WN + j * 16 + (lane & 15);
      bfr[j] = *(const bf16x8*)(B + row * RB + ((ch ^ tile_swz<CPR>(row)) << 4));
    }
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
  }
  __syncthreads();
  conv_epilogue<BN, 2, BMT>(p, acc, smem, m0, n0, mt, wm, wn, lane, tid, split);
#endif
}

// Split-K reduce + epilogue: block = 128 rows x (8*CG) columns; thread = 8 columns x 128/(256/CG)
// rows (CG 8: 64 columns, 4 rows per thread; CG 2: 16 columns, one row -- 4x the blocks for small
// maps, where 64-column blocks would leave most CUs idle). Sums the splits' f32 partials, then
// bias / residual / activation / store and the BN statistics partials of the 128-row block (same
// [2][mblocks][Ncol] layout as the fused epilogue).
template <int CG, typename TA = uint16_t>
__global__ void __launch_bounds__(256) conv_splitk_reduce_kernel(ConvP p) {
  constexpr int RL = 256 / CG, RPT = BM / RL, CW = 8 * CG;
  __shared__ float red[2][RL][CW + 1];
  const int tid = threadIdx.x, cl = tid % CG, rl = tid / CG;
  const int64_t mt = blockIdx.x, col0 = (int64_t)blockIdx.y * CW + cl * 8;
  const bool cok = col0 < p.Ncol;
  float s2[2][8] = {}, q2[2][8] = {};
  float b2[2][8] = {}, c2[2][8] = {}, bmu[8], bis[8];  // BN-backward partials (p.bnb_part)
  if (p.bnb_part && cok) {
#pragma unroll
    for (int t = 0; t < 8; ++t) { bmu[t] = p.bnb_mean[col0 + t]; bis[t] = p.bnb_invstd[col0 + t]; }
  }
  const int64_t stride = p.M * p.Ncol;
  // the rows' loads of one split plane are issued together (2*RPT x 16 B in flight per thread); the
  // per-element summation order over the splits is sequential
  float va[RPT][8] = {};
  for (int k = 0; k < p.splits; ++k) {
    float4 a[RPT], b[RPT];
#pragma unroll
    for (int rr = 0; rr < RPT; ++rr) {
      const int64_t m = mt * BM + rl + RL * rr;
      if (cok && m < p.M) {
        const float* src = p.slab + k * stride + m * p.Ncol + col0;
        a[rr] = *(const float4*)src;
        b[rr] = *(const float4*)(src + 4);
      } else {
        a[rr] = b[rr] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int rr = 0; rr < RPT; ++rr) {
      va[rr][0] += a[rr].x; va[rr][1] += a[rr].y; va[rr][2] += a[rr].z; va[rr][3] += a[rr].w;
      va[rr][4] += b[rr].x; va[rr][5] += b[rr].y; va[rr][6] += b[rr].z; va[rr][7] += b[rr].w;
    }
  }
#pragma unroll
  for (int rr = 0; rr < RPT; ++rr) {
    const int64_t m = mt * BM + rl + RL * rr;
    if (!cok || m >= p.M) continue;
    float* v = va[rr];
    const int h = (rl + RL * rr) >= 64;  // 64-row statistics half of this row
#pragma unroll
    for (int t = 0; t < 8; ++t) { s2[h][t] += v[t]; q2[h][t] += v[t] * v[t]; }
    if (p.bias) {
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] += p.bias[col0 + t];
    }
    const int64_t mo = out_row(p, m);
    if (p.residual) {
      float rr[8];
      ld8((const TA*)p.residual + mo * p.Ncol + col0, rr);
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] += rr[t];
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = act_f(v[t], p.act);
    if (p.out_f32) {
      float* o = (float*)p.out + mo * p.Ncol + col0;
      *(float4*)o = *(float4*)&v[0];
      *(float4*)(o + 4) = *(float4*)&v[4];
      if (sizeof(TA) == 4 && p.bnb_part) {
        float yy[8], zz[8];
        ld8((const TA*)p.bnb_y + mo * p.Ncol + col0, yy);
        ld8((const TA*)p.bnb_z + mo * p.Ncol + col0, zz);
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const float g = v[t] * bnb_act_grad(yy[t], p.bnb_act);
          b2[h][t] += g;
          c2[h][t] += g * ((zz[t] - bmu[t]) * bis[t]);
        }
      }
    } else {
      uint4 w;
      uint16_t* wh = (uint16_t*)&w;
#pragma unroll
      for (int t = 0; t < 8; ++t) wh[t] = f2bf(v[t]);
      *(uint4*)((uint16_t*)p.out + mo * p.Ncol + col0) = w;
      if (p.bnb_part) {
        const uint4 yy = *(const uint4*)((const uint16_t*)p.bnb_y + mo * p.Ncol + col0);
        const uint4 zz = *(const uint4*)((const uint16_t*)p.bnb_z + mo * p.Ncol + col0);
        const uint16_t *yh = (const uint16_t*)&yy, *zh = (const uint16_t*)&zz;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const float g = bf2f(wh[t]) * bnb_act_grad(bf2f(yh[t]), p.bnb_act);
          b2[h][t] += g;
          c2[h][t] += g * ((bf2f(zh[t]) - bmu[t]) * bis[t]);
        }
      }
    }
  }
  // 64-row statistics rows: half h = rows [64h, 64h+64) of this 128-row block
  for (int pass = 0; pass < 2; ++pass) {
    float* dst = pass == 0 ? p.stats : p.bnb_part;
    if (!dst) continue;
    const int64_t mbk = pass == 0 ? p.mblocks : p.bnb_mb;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        red[0][rl][cl * 8 + t] = pass == 0 ? s2[h][t] : b2[h][t];
        red[1][rl][cl * 8 + t] = pass == 0 ? q2[h][t] : c2[h][t];
      }
      __syncthreads();
      if (tid < 2 * CW) {
        const int w = tid / CW, c = tid % CW;
        float a = 0.f;
        for (int r = 0; r < RL; ++r) a += red[w][r][c];
        const int64_t col = (int64_t)blockIdx.y * CW + c;
        const int64_t srow = 2 * mt + h;
        if (col < p.Ncol && srow * SROWS < p.M) dst[(w * mbk + srow) * p.Ncol + col] = a;
      }
      __syncthreads();
    }
  }
}

// ------------------------------------------------------------------------------------------------
// wgrad: dw[k][(r,s,c)] += sum_p dy[p][k] * x[gather(p, r, s)][c]; tiles [BKW pixels][128]
struct WgP {
  const uint16_t* dy;  // [P][K]
  const uint16_t* x;   // [N][H][W][C]
  float* dw;           // layout 0: [Kout][R][S][Cin]; 1: [Kout][Cin][R][S] (torch's weight layout)
  int64_t P, K, Ncol;  // Ncol = R*S*C
  int64_t OH, OW, H, W, C, N;
  int R, S, st_h, st_w, pad_h, pad_w;
  int64_t kchunk;      // pixels per split
  float* slab;         // splits > 1: per-split partials [splits][K][Ncol], summed by wgrad_reduce_kernel
  int64_t Kout, Cin;   // real (unpadded) output / input channels written to dw
  int layout;
  int dC, dRS;         // dw's (channels per tap, taps): = (C, R*S) unless a dense conv runs as a 1x1 GEMM
};

// dw element (k, col = tap*C + c) -> its offset in the requested layout, or -1 for padding
__device__ __forceinline__ int64_t wgrad_dst(const WgP& p, int64_t k, int col) {
  const int C = p.dC;
  const int tap = col / C, c = col - tap * C;
  if (k >= p.Kout || c >= p.Cin) return -1;
  const int64_t RS = p.dRS;
  return p.layout == 0 ? (k * RS + tap) * p.Cin + c : (k * p.Cin + c) * RS + tap;
}

// Block epilogue: the split's partial tile to the slab (plain stores), or, unsplit, the final dw.
__device__ __forceinline__ void wgrad_store(const WgP& p, f32x4 (&acc)[4][4], int64_t k0, int64_t c0, int wm, int wn,
                                            int lane, int64_t split = -1) {
  float* slab = p.slab ? p.slab + (split < 0 ? (int64_t)blockIdx.y : split) * p.K * p.Ncol : nullptr;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int64_t k = k0 + wm * 64 + i * 16 + (lane >> 4) * 4 + rr;
        const int64_t cl = c0 + wn * 64 + j * 16 + (lane & 15);
        if (k >= p.K || cl >= p.Ncol) continue;
        if (slab) {
          slab[k * p.Ncol + cl] = acc[i][j][rr];
        } else {
          const int64_t o = wgrad_dst(p, k, (int)cl);
          if (o >= 0) p.dw[o] = acc[i][j][rr];
        }
      }
}

// Sum of the split partials, written in dw's layout. Block = one output channel k x 256 columns:
// wave w sums the split planes w, w+4, w+8, ... for its 64 float4 column groups (4 independent
// 1-KiB loads in flight per wave per step), then wave 0 adds the other three waves' sums from LDS
// in a fixed order (deterministic).
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(WgP p, int splits) {
  __shared__ float4 part[3][64];
  const int cg = threadIdx.x & 63, sg = threadIdx.x >> 6;
  const int64_t nc4 = p.Ncol >> 2;  // Ncol = R*S*C, C % 8 == 0
  const int64_t k = blockIdx.y, c4 = (int64_t)blockIdx.x * 64 + cg;
  const bool ok = c4 < nc4;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ok) {
    const int64_t plane = p.K * p.Ncol;
    const float* src = p.slab + k * p.Ncol + c4 * 4;
    int sp = sg;
    for (; sp + 12 < splits; sp += 16) {
      const float4 a = *(const float4*)(src + sp * plane), b = *(const float4*)(src + (sp + 4) * plane);
      const float4 c = *(const float4*)(src + (sp + 8) * plane), d = *(const float4*)(src + (sp + 12) * plane);
      v.x += (a.x + b.x) + (c.x + d.x);
      v.y += (a.y + b.y) + (c.y + d.y);
      v.z += (a.z + b.z) + (c.z + d.z);
      v.w += (a.w + b.w) + (c.w + d.w);
    }
    for (; sp < splits; sp += 4) {
      const float4 a = *(const float4*)(src + sp * plane);
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
  }
  if (sg) part[sg - 1][cg] = v;
  __syncthreads();
  if (sg || !ok) return;
#pragma unroll
  for (int w = 0; w < 3; ++w) {
    const float4 o = part[w][cg];
    v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
  }
  const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int64_t o = wgrad_dst(p, k, (int)(c4 * 4 + t));
    if (o >= 0) p.dw[o] = vv[t];
  }
}

static constexpr int BKW = 32;  // pixels per MFMA k-step

__device__ __forceinline__ int swz_w(int row, int chunk) {
  return chunk ^ (((row & 3) << 1) | (((row >> 3) & 1) << 3));
}

// PXT pixels per K-tile (32 or 64: one or two MFMA k-steps per barrier)
template <int PXT>
__global__ void __launch_bounds__(NT, 2) conv_wgrad_kernel(WgP p) {
  // LDS per stage: A [PXT px][128 k] + B [PXT px][128 col], 256-B rows, swizzled 16-B chunks
  constexpr int NR = PXT / 16;  // pixel rows per thread per operand
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * PXT * 256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t ntn = (p.Ncol + 127) / 128;
  const int64_t tile = blockIdx.x;
  const int64_t mt = tile / ntn, nt = tile % ntn;
  const int64_t k0 = mt * 128, c0 = nt * 128;
  const int64_t pbeg = (int64_t)blockIdx.y * p.kchunk;
  const int64_t pend = min<int64_t>(p.P, pbeg + p.kchunk);
  if (pbeg >= pend) return;

  // thread -> (pixel row pr = tid>>4 + 16*i, chunk ch = tid&15), 2 rows per thread per operand
  const int ch = tid & 15;
  // B column decomposition for this thread's chunk (fixed over the K loop)
  const int64_t col = c0 + ch * 8;
  const bool col_ok = col < p.Ncol;
  const int tap = col_ok ? (int)(col / p.C) : 0;
  const int cc = col_ok ? (int)(col - (int64_t)tap * p.C) : 0;
  const int r = tap / p.S, s = tap % p.S;
  const bool kk_ok = (k0 + ch * 8) < p.K;

  uint4 ra[NR], rb[NR];
  // this thread's pixel rows px = pb + (tid>>4) + 16*i as (n, oh, ow), advanced by PXT per
  // K-tile without divisions
  const int OW = (int)p.OW, OH = (int)p.OH, H = (int)p.H, W = (int)p.W;
  int px_n[NR], px_oh[NR], px_ow[NR];
  int64_t px_i[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    px_i[i] = pbeg + (tid >> 4) + 16 * i;
    const int64_t t = px_i[i] / OW;
    px_ow[i] = (int)(px_i[i] - t * OW);
    px_oh[i] = (int)(t % OH);
    px_n[i] = (int)(t / OH);
  }
  auto load = [&]() {
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int64_t px = px_i[i];
      uint4 va = make_uint4(0, 0, 0, 0), vb = make_uint4(0, 0, 0, 0);
      if (px < pend) {
        if (kk_ok) va = *(const uint4*)(p.dy + px * p.K + k0 + ch * 8);
        if (col_ok) {
          const int ih = px_oh[i] * p.st_h - p.pad_h + r, iw = px_ow[i] * p.st_w - p.pad_w + s;
          if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
            vb = *(const uint4*)(p.x + (((int64_t)px_n[i] * H + ih) * W + iw) * p.C + cc);
        }
      }
      ra[i] = va;
      rb[i] = vb;
      px_i[i] += PXT;
      px_ow[i] += PXT;
      if (px_ow[i] >= OW) {  // small maps (RoI 7x7, 1x1 FC) wrap several rows per tile
        const int q = px_ow[i] / OW;
        px_ow[i] -= q * OW;
        px_oh[i] += q;
        if (px_oh[i] >= OH) {
          const int q2 = px_oh[i] / OH;
          px_oh[i] -= q2 * OH;
          px_n[i] += q2;
        }
      }
    }
  };
  auto store = [&](int buf) {
    char* A = smem + buf * (2 * PXT * 256);
    char* B = A + PXT * 256;
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      int row = (tid >> 4) + 16 * i;
      *(uint4*)(A + row * 256 + (swz_w(row, ch) << 4)) = ra[i];
      *(uint4*)(B + row * 256 + (swz_w(row, ch) << 4)) = rb[i];
    }
  };
  // transposed fragment read: rows k0r..k0r+3 (pixels), column block cb (16 wide) of a [px][128] tile
  auto tr_read = [&](const char* T, int prow0, int colbase) -> s16x4 {
    const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    int row = prow0 + 8 * g + q;
    int colx = colbase + 4 * pp;  // element column
    int chunk = colx >> 3, within = (colx & 7) * 2;
    const char* addr = T + row * 256 + (swz_w(row, chunk) << 4) + within;
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(addr));
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int64_t nk = (pend - pbeg + PXT - 1) / PXT;
  load();
  store(0);
  __syncthreads();
  for (int64_t it = 0; it < nk; ++it) {
    const int buf = (int)(it & 1);
    if (it + 1 < nk) load();
    const char* A = smem + buf * (2 * PXT * 256);
    const char* B = A + PXT * 256;
#pragma unroll
    for (int ks = 0; ks < PXT / BKW; ++ks) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s16x4 lo = tr_read(A, ks * BKW + 0, wm * 64 + i * 16);
        s16x4 hi = tr_read(A, ks * BKW + 4, wm * 64 + i * 16);
        short tmp[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = *(bf16x8*)tmp;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s16x4 lo = tr_read(B, ks * BKW + 0, wn * 64 + j * 16);
        s16x4 hi = tr_read(B, ks * BKW + 4, wn * 64 + j * 16);
        short tmp[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfr[j] = *(bf16x8*)tmp;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (it + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }
  wgrad_store(p, acc, k0, c0, wm, wn, lane);
}

// wgrad, direct-to-LDS: 64-pixel K-tiles (two MFMA k-steps per barrier), both operands staged by
// global_load_lds (one wave instruction = 4 pixel rows x 256 B), the swz_w XOR applied on the source
// chunk; fragments read transposed with ds_read_b64_tr_b16 as in conv_wgrad_kernel.
static constexpr int BKG = 64;

__global__ void __launch_bounds__(NT, 2) conv_wgrad_glds_kernel(WgP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int OPB = BKG * 256, STAGE = 2 * OPB;  // per operand / per stage bytes
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t ntn = (p.Ncol + 127) / 128;
  const int64_t tile = blockIdx.x;
  const int64_t mt = tile / ntn, nt = tile % ntn;
  const int64_t k0 = mt * 128, c0 = nt * 128;
  const int64_t pbeg = (int64_t)blockIdx.y * p.kchunk;
  const int64_t pend = min<int64_t>(p.P, pbeg + p.kchunk);
  if (pbeg >= pend) return;
  const int lr = lane >> 4;                       // row within a 4-row instruction group
  const uint16_t* zero = (const uint16_t*)g_zero_page;
  // per instruction i (0..3): rows wave*16 + i*4 + lr; logical chunk depends on the row
  int lcs[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) lcs[i] = swz_w(wave * 16 + i * 4 + lr, lane & 15);
  auto issue = [&](int64_t pb, int buf) {
    char* A = smem + buf * STAGE;
    char* B = A + OPB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wave * 16 + i * 4;
      const int64_t px = pb + row + lr;
      const int lc = lcs[i];
      const uint16_t* sa = zero;
      const uint16_t* sb = zero;
      if (px < pend) {
        if (k0 + lc * 8 < p.K) sa = p.dy + px * p.K + k0 + lc * 8;
        const int64_t col = c0 + lc * 8;
        if (col < p.Ncol) {
          const int tap = (int)(col / p.C);
          const int cc = (int)(col - (int64_t)tap * p.C);
          const int r = tap / p.S, s2 = tap - (tap / p.S) * p.S;
          const int64_t ow = px % p.OW, t = px / p.OW;
          const int64_t oh = t % p.OH, n = t / p.OH;
          const int64_t ih = oh * p.st_h - p.pad_h + r, iw = ow * p.st_w - p.pad_w + s2;
          if (ih >= 0 && iw >= 0 && ih < p.H && iw < p.W) sb = p.x + ((n * p.H + ih) * p.W + iw) * p.C + cc;
        }
      }
      __builtin_amdgcn_global_load_lds((const void*)sa, (LDS_AS void*)(A + row * 256), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)sb, (LDS_AS void*)(B + row * 256), 16, 0, 0);
    }
  };
  auto tr_read = [&](const char* T, int prow0, int colbase) -> s16x4 {
    const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    int row = prow0 + 8 * g + q;
    int colx = colbase + 4 * pp;
    int chunk = colx >> 3, within = (colx & 7) * 2;
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(T + row * 256 + (swz_w(row, chunk) << 4) + within));
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int64_t nk = (pend - pbeg + BKG - 1) / BKG;
  issue(pbeg, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int64_t it = 0; it < nk; ++it) {
    const int buf = (int)(it & 1);
    if (it + 1 < nk) issue(pbeg + (it + 1) * BKG, buf ^ 1);
    const char* A = smem + buf * STAGE;
    const char* B = A + OPB;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s16x4 lo = tr_read(A, ks * 32, wm * 64 + i * 16), hi = tr_read(A, ks * 32 + 4, wm * 64 + i * 16);
        short t8[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = *(bf16x8*)t8;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s16x4 lo = tr_read(B, ks * 32, wn * 64 + j * 16), hi = tr_read(B, ks * 32 + 4, wn * 64 + j * 16);
        short t8[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfr[j] = *(bf16x8*)t8;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  wgrad_store(p, acc, k0, c0, wm, wn, lane);
}

// wgrad on buffer descriptors (the buf analogue of conv_wgrad_glds_kernel): 32-pixel K-tiles in a
// 3-deep LDS ring (48 KiB, 3 blocks per CU), both operands staged by buffer_load_dwordx4 ... lds (one
// wave instruction = 4 pixel rows x 256 B; the swz_w XOR applied on the source chunk). Every lane
// owns fixed rows of every tile and one fixed column chunk, so its gather position advances by a
// division-free (n, oh, ow) walk and its offsets stay 32-bit: dy rows through a descriptor whose
// range ends at this split's last pixel (later rows read zero), x rows through a validity select.
__global__ void __launch_bounds__(NT, 3) conv_wgrad_buf_kernel(WgP p) {
#if defined(__HIP_DEVICE_COMPILE__)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int PXT = 32, STAGES = 3, OPB = PXT * 256, STAGE = 2 * OPB, LOADS = 4;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t ntn = (p.Ncol + 127) / 128;
  // flat XCD-aware grid (as conv_wgrad_x3_kernel): one XCD runs all tiles of the same pixel splits
  const int64_t ntiles = ((p.K + 127) / 128) * ntn;
  const int64_t work = xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  const int64_t split = work / ntiles, tile = work % ntiles;
  const int64_t mt = tile / ntn, nt = tile % ntn;
  const int64_t k0 = mt * 128, c0 = nt * 128;
  const int64_t pbeg = split * p.kchunk;
  const int64_t pend = min<int64_t>(p.P, pbeg + p.kchunk);
  if (pbeg >= pend) return;
  const int lr = lane >> 4;
  const int K = (int)p.K, C = (int)p.C, H = (int)p.H, W = (int)p.W, OW = (int)p.OW, OH = (int)p.OH;
  // per instruction i (0, 1): tile row = wave * 8 + i * 4 + lr
  uint32_t a_off[2];
  int bn_[2], boh[2], bow[2], bpx[2];
  int lcs[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = wave * 8 + i * 4 + lr;
    lcs[i] = swz_w(row, lane & 15);
    const int64_t px = pbeg + row;
    a_off[i] = (k0 + lcs[i] * 8 < p.K) ? (uint32_t)((px * p.K + k0 + lcs[i] * 8) * 2) : kOOB;
    bpx[i] = (int)px;
    const int64_t t = px / OW;
    bow[i] = (int)(px - t * OW);
    boh[i] = (int)(t % OH);
    bn_[i] = (int)(t / OH);
  }
  // B column chunk of each instruction's lane (fixed over the pixel loop): tap (r, s), channel c
  int b_r[2], b_s[2], b_c[2];
  bool b_col[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int64_t col = c0 + lcs[i] * 8;
    b_col[i] = col < p.Ncol;
    const int tap = b_col[i] ? (int)(col / C) : 0;
    b_c[i] = b_col[i] ? (int)(col - (int64_t)tap * C) : 0;
    b_r[i] = tap / p.S;
    b_s[i] = tap - b_r[i] * p.S;
  }
  const i32x4 arsrc = dma_rsrc(p.dy, (uint32_t)(pend * p.K * 2));
  const i32x4 brsrc = dma_rsrc(p.x, (uint32_t)(p.N * p.H * p.W * p.C * 2));
  const uint32_t lds0 = lds_addr(smem);
  const uint32_t a_step = (uint32_t)(PXT * K * 2);
  auto issue = [&](int buf) {
    const uint32_t A = lds0 + buf * STAGE;
    const uint32_t B = A + OPB;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = wave * 8 + i * 4;
      lds_dma16(arsrc, A + row * 256, a_off[i], 0u);
      const int ih = boh[i] * p.st_h - p.pad_h + b_r[i], iw = bow[i] * p.st_w - p.pad_w + b_s[i];
      const bool ok = b_col[i] && bpx[i] < pend && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      const uint32_t bo = ok ? (uint32_t)((((bn_[i] * H + ih) * W + iw) * C + b_c[i]) * 2) : kOOB;
      lds_dma16(brsrc, B + row * 256, bo, 0u);
      // advance this lane's rows by one tile
      a_off[i] = a_off[i] == kOOB ? kOOB : a_off[i] + a_step;
      bpx[i] += PXT;
      if (OW == 1 && OH == 1) {  // 1x1 maps (a dense conv as a GEMM over images): pixel = image
        bn_[i] += PXT;
      } else {
        bow[i] += PXT;
        while (bow[i] >= OW) {
          bow[i] -= OW;
          if (++boh[i] == OH) { boh[i] = 0; ++bn_[i]; }
        }
      }
    }
  };
  auto tr_read = [&](const char* T, int prow0, int colbase) -> s16x4 {
    const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    int row = prow0 + 8 * g + q;
    int colx = colbase + 4 * pp;
    int chunk = colx >> 3, within = (colx & 7) * 2;
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(T + row * 256 + (swz_w(row, chunk) << 4) + within));
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int64_t nk = (pend - pbeg + PXT - 1) / PXT;
#pragma unroll
  for (int st = 0; st < STAGES - 1; ++st)
    if (st < nk) issue(st);
  for (int64_t it = 0; it < nk; ++it) {
    if (it + STAGES - 2 < nk) wait_vmcnt<LOADS * (STAGES - 2)>();
    else wait_vmcnt<0>();
    block_barrier();
    if (it + STAGES - 1 < nk) issue((int)((it + STAGES - 1) % STAGES));
    const char* A = smem + (int)(it % STAGES) * STAGE;
    const char* B = A + OPB;
    bf16x8 af[4], bfr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const s16x4 lo = tr_read(A, 0, wm * 64 + i * 16), hi = tr_read(A, 4, wm * 64 + i * 16);
      af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const s16x4 lo = tr_read(B, 0, wn * 64 + j * 16), hi = tr_read(B, 4, wn * 64 + j * 16);
      bfr[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
  }
  wgrad_store(p, acc, k0, c0, wm, wn, lane, split);
#endif
}

// ------------------------------------------------------------------------------------------------
// bf16x3 implicit GEMM (precision-faithful mode: f32 activations, f32 accumulate). The reference
// trains its convs in fp32 (TF32 on Ampere; train_frcnn_baseline.py:139-176, no autocast). gfx950
// has no xf32 MFMA and its f32 MFMA runs at 1/16 of the bf16 rate, so each f32 operand is split
// into bf16 hi + lo planes and a K-step issues hi*hi + hi*lo + lo*hi (three bf16 MFMAs, f32
// accumulation): ~2^-16 relative per product (TF32 rounds each operand to 2^-11) at 1/3 of the
// bf16 MFMA rate. Weights arrive pre-split (mx_conv_pack_* split mode, planes p.wt / p.wt +
// p.wt_plane); activations are read as f32 by register-staged loads and split once per block while
// they are written to LDS (each element is read by two waves, so splitting at staging halves the
// VALU work of splitting fragments). Tile BMT x BN x 32, 4 waves (2x2), double-buffered LDS of
// [A hi | A lo | B hi | B lo] bf16 tiles (64-B rows, tile_swz<4> chunk swizzle: conflict-free
// ds_read_b128 fragment reads and ds_write_b128 stores). Any C % 8 == 0 (a lane's 8-channel chunk
// stays inside one tap): the stem's 8-channel input included.
template <int BN, int MODE, int BMT>
__global__ void __launch_bounds__(NT, 2) conv_x3_kernel(ConvP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BKT = 32, RB = BKT * 2;
  constexpr int APL = BMT * RB, BPL = BN * RB, STAGE = 2 * (APL + BPL);
  constexpr int WN = BN / 2, TJ = WN / 16, WM = BMT / 2, TI = WM / 16;
  constexpr int ACH = BMT * 4 / NT, BCH = BN * 4 / NT, RPS = NT / 4;  // chunks per thread; rows per sweep
  static_assert(ACH >= 1 && BCH >= 1, "tile shape");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t ntiles_n = (p.Ncol + BN - 1) / BN;
  const int64_t gid = xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  const int split = (int)(gid % p.splits);
  const int64_t bid = gid / p.splits;
  const int64_t mt = bid / ntiles_n, nt = bid % ntiles_n;
  const int64_t m0 = mt * BMT, n0 = nt * BN;
  const float* __restrict__ src = (const float*)p.src;
  const uint16_t* __restrict__ whi = p.wt;
  const uint16_t* __restrict__ wlo = p.wt + p.wt_plane;
  const int IH = (int)p.IH, IW = (int)p.IW, IC = (int)p.IC, S = p.S, Kd = (int)p.Kdim;
  const int kc = tid & 3;  // this thread's 8-element K chunk of every A and B row it stages
  int a_h0[ACH], a_w0[ACH];
  int64_t a_pix[ACH];
#pragma unroll
  for (int i = 0; i < ACH; ++i) {
    const int64_t m = m0 + (tid >> 2) + RPS * i;
    const bool ok = m < p.M;
    const int64_t mm = ok ? m : 0;
    const int ow = (int)(mm % p.OW);
    const int64_t t = mm / p.OW;
    const int oh = (int)(t % p.OH);
    const int n = (int)(t / p.OH);
    // MODE 0: ih = oh*st - pad + r; MODE 1 (dgrad parity class): ih = hh + dh - ri
    a_h0[i] = MODE == 0 ? oh * p.st_h - p.pad_h : oh + p.pad_h;
    a_w0[i] = MODE == 0 ? ow * p.st_w - p.pad_w : ow + p.pad_w;
    if (!ok) a_h0[i] = -(1 << 28);
    a_pix[i] = ((int64_t)n * IH + a_h0[i]) * IW + a_w0[i];
  }
  int64_t b_row[BCH];
#pragma unroll
  for (int i = 0; i < BCH; ++i) b_row[i] = n0 + (tid >> 2) + RPS * i;
  const int64_t nk = (p.Kdim + BKT - 1) / BKT;
  const int64_t kbeg = (int64_t)split * p.kt_per_split;
  const int64_t ntk = min<int64_t>(nk, kbeg + p.kt_per_split) - kbeg;
  // K position of this thread's chunk (k -> tap (cr, cq), channel cc), walked incrementally
  int ik = (int)(kbeg * BKT) + kc * 8;
  int cc, cr, cq;
  {
    const int tap = ik / IC;
    cc = ik - tap * IC;
    cr = tap / S;
    cq = tap - cr * S;
  }
  float4 ra[ACH][2];
  uint4 rbh[BCH], rbl[BCH];
  auto load = [&]() {
    const int k = ik;
    const bool kin = k < Kd;
    const int dr = MODE == 0 ? cr : -cr, ds = MODE == 0 ? cq : -cq, c = cc;
    ik += BKT;
    cc += BKT;
    while (cc >= IC) {
      cc -= IC;
      if (++cq == S) { cq = 0; ++cr; }
    }
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int ih = a_h0[i] + dr, iw = a_w0[i] + ds;
      if (kin && (unsigned)ih < (unsigned)IH && (unsigned)iw < (unsigned)IW) {
        const float* sp = src + (a_pix[i] + (int64_t)dr * IW + ds) * IC + c;
        ra[i][0] = *(const float4*)sp;
        ra[i][1] = *(const float4*)(sp + 4);
      } else {
        ra[i][0] = ra[i][1] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      if (kin && b_row[i] < p.Ncol) {
        rbh[i] = *(const uint4*)(whi + b_row[i] * p.Kdim + k);
        rbl[i] = *(const uint4*)(wlo + b_row[i] * p.Kdim + k);
      } else {
        rbh[i] = rbl[i] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto store = [&](int buf) {
    char* Ah = smem + buf * STAGE;
    char* Al = Ah + APL;
    char* Bh = Al + APL;
    char* Bl = Bh + BPL;
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int row = (tid >> 2) + RPS * i;
      const int off = row * RB + ((kc ^ tile_swz<4>(row)) << 4);
      uint4 h, l;
      split8(ra[i][0], ra[i][1], h, l);
      *(uint4*)(Ah + off) = h;
      *(uint4*)(Al + off) = l;
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int row = (tid >> 2) + RPS * i;
      const int off = row * RB + ((kc ^ tile_swz<4>(row)) << 4);
      *(uint4*)(Bh + off) = rbh[i];
      *(uint4*)(Bl + off) = rbl[i];
    }
  };
  f32x4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (ntk > 0) {
    load();
    store(0);
  }
  __syncthreads();
  for (int64_t t = 0; t < ntk; ++t) {
    const int buf = (int)(t & 1);
    if (t + 1 < ntk) load();
    const char* Ah = smem + buf * STAGE;
    const char* Al = Ah + APL;
    const char* Bh = Al + APL;
    const char* Bl = Bh + BPL;
    const int ch = lane >> 4;
    bf16x8 ah[TI], al[TI], bh[TJ], bl[TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int row = wm * WM + i * 16 + (lane & 15);
      const int off = row * RB + ((ch ^ tile_swz<4>(row)) << 4);
      ah[i] = *(const bf16x8*)(Ah + off);
      al[i] = *(const bf16x8*)(Al + off);
    }
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int row = wn * WN + j * 16 + (lane & 15);
      const int off = row * RB + ((ch ^ tile_swz<4>(row)) << 4);
      bh[j] = *(const bf16x8*)(Bh + off);
      bl[j] = *(const bf16x8*)(Bl + off);
    }
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
      }
    if (t + 1 < ntk) store(buf ^ 1);
    __syncthreads();
  }
  conv_epilogue<BN, 2, BMT, float, 2, 2, MODE == 1>(p, acc, smem, m0, n0, mt, wm, wn, lane, tid, split);
}

// Chunk swizzle of the f32 A half-tiles of conv_x3_buf_kernel (64-B rows = 4 chunks of 4 f32): the
// Gray code of the row's quarter within its 16-row fragment. A 16x16x32 fragment lane reads chunks
// 2*(g&1) and 2*(g&1)+1 of half g>>1 (g = lane>>4), so each 16-lane ds_read_b128 group holds rows
// 0..15 once, a quarter of them on the other chunk pair; with phys = logical ^ gray(quarter) the 16
// lanes land on 16 distinct 4-bank groups (tile_swz<4> would collide rows 0-3 with 4-7).
__device__ __forceinline__ int x3_swz(int row) {
  const int g = (row >> 2) & 3;
  return g ^ (g >> 1);
}

// bf16x3 implicit GEMM with an LDS-DMA ring (IC % 32 == 0, R*S <= 64, operands < 2 GiB): the f32 A
// tile (BMT rows x 32 channels, one tap) lands as two 16-channel half-tiles of 64-B rows through
// buffer_load_dwordx4 ... lds with wave-uniform tap offsets and per-row validity masks (as in
// conv_igemm_buf_kernel); the pre-split weight planes land the same way. A fragments are split into
// hi / lo in registers at read time (6 VALU per pair, ~2 per MFMA, hidden in the MFMA issue gaps),
// so no register staging or ds_write sits on the critical path and STAGES-1 K-tiles stay in flight.
// WC = 1 (wide wave tiles: WR waves stacked along M, each spanning all BN columns): every A row is
// split by exactly one wave (WC = 2 splits each row in both wave-columns), half the split VALU per
// MFMA, at twice the B fragment reads per wave.
// AP (mx_conv2d_*_x3p): A arrives pre-split as bf16 hi / lo planes (mx_split_planes, the same split8 values)
// and lands like the weight planes -- a hi and a lo plane of 64-B rows (32 channels) -- so its fragments
// are read directly, without the split VALU; bitwise the same products.
template <int BN, int MODE, int STAGES, int OCC, int BMT, int WR = 2, int WC = 2, bool AP = false>
__global__ void __launch_bounds__(64 * WR * WC, OCC) conv_x3_buf_kernel(ConvP p) {
#if defined(__HIP_DEVICE_COMPILE__)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int RB = 64, RPI = 16;  // bytes per LDS row; rows landed per wave instruction
  constexpr int NW = WC * WR;  // waves: WR rows x WC columns of wave tiles
  constexpr int AR = BMT / NW, AI = AR / RPI, BR = BN / NW, BI = BR / RPI;
  constexpr int LOADS = 2 * AI + 2 * BI;  // vmem instructions per K-tile per wave
  constexpr int AH = BMT * RB, BP = BN * RB, STAGE = 2 * AH + 2 * BP;
  constexpr int WN = BN / WC, TJ = WN / 16, WM = BMT / WR, TI = WM / 16;
  static_assert(AI >= 1 && BI >= 1 && STAGES >= 2, "tile shape");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WC, wn = wave % WC;
  const int64_t ntiles_n = (p.Ncol + BN - 1) / BN;
  const int64_t gid = xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  const int split = (int)(gid % p.splits);
  const int64_t bid = gid / p.splits;
  const int64_t mt = bid / ntiles_n, nt = bid % ntiles_n;
  const int64_t m0 = mt * BMT, n0 = nt * BN;
  const int lrow = lane >> 2, pc = lane & 3;  // landing row within the instruction, physical chunk
  const int qa = AP ? (pc ^ tile_swz<4>(lrow)) : (pc ^ x3_swz(lrow)), qb = pc ^ tile_swz<4>(lrow);  // logical chunks
  const int IH = (int)p.IH, IW = (int)p.IW, IC = (int)p.IC, R = p.R, S = p.S;
  uint32_t a_voff[AI];
  uint64_t a_mask[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int64_t m = m0 + wave * AR + i * RPI + lrow;
    uint64_t mask = 0;
    int32_t off = 0;
    if (m < p.M) {
      const int ow = (int)(m % p.OW);
      const int64_t t = m / p.OW;
      const int oh = (int)(t % p.OH);
      const int n = (int)(t / p.OH);
      const int h0 = MODE == 0 ? oh * p.st_h - p.pad_h : oh + p.pad_h - (R - 1);
      const int w0 = MODE == 0 ? ow * p.st_w - p.pad_w : ow + p.pad_w - (S - 1);
      off = ((n * IH + h0) * IW + w0) * IC + qa * (AP ? 8 : 4);
      for (int r = 0; r < R; ++r)
        for (int q = 0; q < S; ++q) {
          const int rr = MODE == 0 ? r : R - 1 - r, qq = MODE == 0 ? q : S - 1 - q;
          if ((unsigned)(h0 + rr) < (unsigned)IH && (unsigned)(w0 + qq) < (unsigned)IW) mask |= 1ull << (r * S + q);
        }
    }
    a_voff[i] = (uint32_t)off * (AP ? 2u : 4u);
    a_mask[i] = mask;
  }
  uint32_t b_voff[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int64_t n = n0 + wave * BR + i * RPI + lrow;
    b_voff[i] = n < p.Ncol ? (uint32_t)((n * p.Kdim + qb * 8) * 2) : kOOB;
  }
  const i32x4 arsrc = dma_rsrc(p.src, (uint32_t)(p.src_elems * (AP ? 2 : 4)));
  const i32x4 alrsrc = AP ? dma_rsrc(p.src + p.src_elems, (uint32_t)(p.src_elems * 2)) : arsrc;
  const i32x4 bhrsrc = dma_rsrc(p.wt, (uint32_t)(p.wt_elems * 2));
  const i32x4 blrsrc = dma_rsrc(p.wt + p.wt_plane, (uint32_t)(p.wt_elems * 2));
  const uint32_t lds0 = lds_addr(smem);
  const int64_t nk = p.Kdim / 32;
  const int64_t kbeg = (int64_t)split * p.kt_per_split;
  const int64_t ntk = min<int64_t>(nk, kbeg + p.kt_per_split) - kbeg;
  // wave-uniform K position of the next tile to issue: tap (cr, cq), channel cc
  const int korder = __builtin_amdgcn_readfirstlane(p.korder);
  KPos kp;
  kp.init(korder, (int)kbeg, R, S, IC, 32);
  // timing-only diagnostics (round 2, mx_conv_set_debug bits 1 no epilogue, 2 no hi/lo split, 4 no B
  // LDS-DMA, 8 no A LDS-DMA) are compiled out: their run-time tests cost branches and register moves
  // in every K-tile
  constexpr int dbg = 0;
  auto issue = [&](int buf) {
    const uint32_t A = lds0 + buf * STAGE;
    const uint32_t B = A + 2 * AH;
    const int cr = kp.cr, cq = kp.cq, cc = kp.cc;
    const int rr = MODE == 0 ? cr : R - 1 - cr, qq = MODE == 0 ? cq : S - 1 - cq;
    const uint32_t a_soff = (uint32_t)(((rr * IW + qq) * IC + cc) * (AP ? 2 : 4));
    const int tap = cr * S + cq;
    const uint32_t b_soff = (uint32_t)__builtin_amdgcn_readfirstlane((int)((tap * IC + cc) * 2));
    if (!(dbg & 8)) {
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const bool ok = (a_mask[i] >> tap) & 1ull;
      const uint32_t v = a_voff[i] + a_soff;
      const uint32_t dst = A + (wave * AR + i * RPI) * RB;
      if constexpr (AP) {  // hi and lo planes: 64-B rows of 32 bf16 channels each
        lds_dma16(arsrc, dst, ok ? v : kOOB, 0u);
        lds_dma16(alrsrc, dst + AH, ok ? v : kOOB, 0u);
      } else {             // two 16-channel f32 half-tiles
        lds_dma16(arsrc, dst, ok ? v : kOOB, 0u);
        lds_dma16(arsrc, dst + AH, ok ? v + 64u : kOOB, 0u);
      }
    }
    }
    if (!(dbg & 4)) {
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const uint32_t dst = B + (wave * BR + i * RPI) * RB;
      lds_dma16(bhrsrc, dst, b_voff[i], b_soff);
      lds_dma16(blrsrc, dst + BP, b_voff[i], b_soff);
    }
    }
    kp.advance(korder, R, S, IC, 32);
  };
  f32x4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int st = 0; st < STAGES - 1; ++st)
    if (st < ntk) issue(st);
  const int g = lane >> 4, q0 = (g & 1) * 2;
  for (int64_t t = 0; t < ntk; ++t) {
    if (t + STAGES - 2 < ntk) wait_vmcnt<LOADS * (STAGES - 2)>();
    else wait_vmcnt<0>();
    block_barrier();
    if (t + STAGES - 1 < ntk) issue((int)((t + STAGES - 1) % STAGES));
    const char* A = smem + (int)(t % STAGES) * STAGE;
    const char* Ag = A + (g >> 1) * AH;
    const char* Bh = A + 2 * AH;
    const char* Bl = Bh + BP;
    constexpr int TJB = (TJ > 4 && WC == 2) ? 1 : TJ;  // B fragments held at once
    bf16x8 ah[TI], al[TI], bh[TJB], bl[TJB];
    auto loadb = [&](int j, int slot) {
      const int row = wn * WN + j * 16 + (lane & 15);
      const int off = row * RB + ((g ^ tile_swz<4>(row)) << 4);
      bh[slot] = *(const bf16x8*)(Bh + off);
      bl[slot] = *(const bf16x8*)(Bl + off);
    };
    if constexpr (TJB == TJ) {
#pragma unroll
      for (int j = 0; j < TJ; ++j) loadb(j, j);
    }
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int row = wm * WM + i * 16 + (lane & 15);
      if constexpr (AP) {  // pre-split: read like the weight planes
        const int off = row * RB + ((g ^ tile_swz<4>(row)) << 4);
        ah[i] = *(const bf16x8*)(A + off);
        al[i] = *(const bf16x8*)(A + AH + off);
        continue;
      }
      const int f = x3_swz(row);
      const float4 u = *(const float4*)(Ag + row * RB + ((q0 ^ f) << 4));
      const float4 w = *(const float4*)(Ag + row * RB + (((q0 + 1) ^ f) << 4));
      uint4 h, l;
      if (dbg & 2) {
        h = __builtin_bit_cast(uint4, u);
        l = __builtin_bit_cast(uint4, w);
      } else {
        split8(u, w, h, l);
      }
      ah[i] = __builtin_bit_cast(bf16x8, h);
      al[i] = __builtin_bit_cast(bf16x8, l);
    }
    if constexpr (TJB == TJ) {
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
    } else {
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        loadb(j, 0);
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[0], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[0], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[0], acc[i][j], 0, 0, 0);
        }
      }
    }
  }
  if (dbg & 1) {  // keep every accumulator live, store nothing
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) sum += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (sum == 1.2345e-30f) ((float*)p.out)[0] = sum;
    return;
  }
  __syncthreads();
  // wide tiles stage the whole f32 tile at once (one barrier, every wave storing); 8-wave 2x2 tiles
  // stage one wave-row per pass (their whole tile would not fit beside a second block)
  conv_epilogue<BN, (WC == 1 ? 1 : WR), BMT, float, WR, WC, MODE == 1>(p, acc, smem, m0, n0, mt, wm, wn, lane, tid,
                                                                       split);
#endif
}

// bf16x3 wgrad: dw[k][(r,s,c)] = sum_p dy[p][k] * x[gather(p, r, s)][c] on f32 dy / x, both split
// into hi / lo while staged (register loads, 32-pixel K-tiles, pixel-major bf16 LDS tiles with the
// swz_w swizzle), fragments read transposed with ds_read_b64_tr_b16 as in conv_wgrad_buf_kernel;
// 128 x 128 (k, col) block tiles, the pixel axis split into slab partials (wgrad_reduce_kernel).
// IL (mx_conv_set_wgrad_variant(6)): the next K-tile's hi / lo split and LDS stores are interleaved with
// the second half of this K-tile's MFMAs (sched_group_barrier) instead of following all of them; the
// loads and stores are unconditional (past the split they read zeros into the unused buffer), so the
// loop body is one basic block the scheduler can interleave.
template <bool IL>
__global__ void __launch_bounds__(NT, 2) conv_wgrad_x3_kernel(WgP p) {
#if defined(__HIP_DEVICE_COMPILE__)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int PXT = 32, OPB = PXT * 256, STAGE = 4 * OPB;  // planes: dy hi, dy lo, x hi, x lo
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t ntn = (p.Ncol + 127) / 128;
  // flat grid, XCD-aware: the blocks an XCD runs are consecutive work items, i.e. all (k, col) tiles of
  // the same pixel splits, so the dy / x rows they share stay in that XCD's L2
  const int64_t ntiles = ((p.K + 127) / 128) * ntn;
  const int64_t work = xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  const int64_t split = work / ntiles, tile = work % ntiles;
  const int64_t mt = tile / ntn, nt = tile % ntn;
  const int64_t k0 = mt * 128, c0 = nt * 128;
  const int64_t pbeg = split * p.kchunk;
  const int64_t pend = min<int64_t>(p.P, pbeg + p.kchunk);
  if (pbeg >= pend) return;
  const float* __restrict__ dy = (const float*)p.dy;
  const float* __restrict__ x = (const float*)p.x;
  const int ch = tid & 15;  // this thread's 8-wide chunk of the k columns (dy) and of the (r,s,c) columns (x)
  const int64_t col = c0 + ch * 8;
  const bool col_ok = col < p.Ncol;
  const int tap = col_ok ? (int)(col / p.C) : 0;
  const int cc = col_ok ? (int)(col - (int64_t)tap * p.C) : 0;
  const int r = tap / p.S, s = tap - (tap / p.S) * p.S;
  const bool k_ok = (k0 + ch * 8) < p.K;
  const int OW = (int)p.OW, OH = (int)p.OH, H = (int)p.H, W = (int)p.W, C = (int)p.C;
  // operands read through buffer descriptors with 32-bit byte offsets (mx_conv2d_wgrad_x3 checks
  // that both fit): an invalid row (past the split, a padding tap, a column / channel past the
  // matrix) gets an out-of-range offset and the hardware returns zeros -- no 64-bit address math,
  // no divergent branches around the loads
  const __amdgpu_buffer_rsrc_t dyr = __builtin_amdgcn_make_buffer_rsrc((void*)dy, (short)0, (int)(p.P * p.K * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, (int)(p.N * p.H * p.W * p.C * 4), 0x00020000);
  // per-tile pixel step PXT = dn images + dh rows + dw columns of the output grid (wave-uniform)
  const int dw = PXT % OW, dh = (PXT / OW) % OH, dn = PXT / (OW * OH);
  const int ihb = -p.pad_h + r, iwb = -p.pad_w + s;
  int px_n[2], px_oh[2], px_ow[2], px_i[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int64_t pi = pbeg + (tid >> 4) + 16 * i;
    px_i[i] = (int)pi;
    const int64_t t = pi / OW;
    px_ow[i] = (int)(pi - t * OW);
    px_oh[i] = (int)(t % OH);
    px_n[i] = (int)(t / OH);
  }
  const int pend32 = (int)pend;
  const uint32_t dy_col = (uint32_t)(k0 + ch * 8) * 4u;
  float4 rd[2][2], rx[2][2];
  auto load = [&]() {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bool pok = px_i[i] < pend32;
      const uint32_t od = (pok && k_ok) ? __umul24((uint32_t)px_i[i], (uint32_t)(p.K * 4)) + dy_col : kOOB;
      const int ih = __mul24(px_oh[i], p.st_h) + ihb, iw = __mul24(px_ow[i], p.st_w) + iwb;
      const bool xok = pok && col_ok && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      const uint32_t ox = xok ? (uint32_t)__mul24(__mul24(px_n[i], H) + ih, W) + (uint32_t)iw : 0u;
      const uint32_t oxb = xok ? __umul24(ox, (uint32_t)(C * 4)) + (uint32_t)cc * 4u : kOOB;
      rd[i][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(dyr, od, 0, 0));
      rd[i][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(dyr, od + 16u, 0, 0));
      rx[i][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, oxb, 0, 0));
      rx[i][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, oxb + 16u, 0, 0));
      // advance PXT pixels: branch-free carries (ow < OW, oh < OH stay invariant)
      px_i[i] += PXT;
      int ow = px_ow[i] + dw;
      const int c1 = ow >= OW ? 1 : 0;
      ow -= c1 * OW;
      int oh = px_oh[i] + dh + c1;
      const int c2 = oh >= OH ? 1 : 0;
      oh -= c2 * OH;
      px_ow[i] = ow;
      px_oh[i] = oh;
      px_n[i] += dn + c2;
    }
  };
  auto store = [&](int buf) {
    char* Dh = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = (tid >> 4) + 16 * i;
      const int off = row * 256 + (swz_w(row, ch) << 4);
      uint4 h, l;
      split8(rd[i][0], rd[i][1], h, l);
      *(uint4*)(Dh + off) = h;
      *(uint4*)(Dh + OPB + off) = l;
      split8(rx[i][0], rx[i][1], h, l);
      *(uint4*)(Dh + 2 * OPB + off) = h;
      *(uint4*)(Dh + 3 * OPB + off) = l;
    }
  };
  auto tr_read = [&](const char* T, int prow0, int colbase) -> s16x4 {
    const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    const int row = prow0 + 8 * g + q;
    const int colx = colbase + 4 * pp;
    const int chunk = colx >> 3, within = (colx & 7) * 2;
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(T + row * 256 + (swz_w(row, chunk) << 4) + within));
  };
  auto frag = [&](const char* T, int colbase) -> bf16x8 {
    const s16x4 lo = tr_read(T, 0, colbase), hi = tr_read(T, 4, colbase);
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int64_t nk = (pend - pbeg + PXT - 1) / PXT;
  load();
  store(0);
  __syncthreads();
  for (int64_t it = 0; it < nk; ++it) {
    const int buf = (int)(it & 1);
    if (IL || it + 1 < nk) load();
    const char* Dh = smem + buf * STAGE;
    bf16x8 ah[4], al[4], bh[4], bl[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ah[i] = frag(Dh, wm * 64 + i * 16);
      al[i] = frag(Dh + OPB, wm * 64 + i * 16);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bh[j] = frag(Dh + 2 * OPB, wn * 64 + j * 16);
      bl[j] = frag(Dh + 3 * OPB, wn * 64 + j * 16);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
      }
    if (IL) {
      store(buf ^ 1);
      // schedule of one K-tile: the next tile's 8 loads, the 32 fragment reads beside the first 12
      // MFMAs, then the remaining 36 MFMAs each with ~3 of the split VALU and every third with one of
      // the 8 LDS stores
      __builtin_amdgcn_sched_group_barrier(0x020, 8, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
      for (int q = 0; q < 12; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      }
#pragma unroll
      for (int q = 0; q < 36; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
        if (q % 3 == 2) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
      }
    } else if (it + 1 < nk) {
      store(buf ^ 1);
    }
    __syncthreads();
  }
  wgrad_store(p, acc, k0, c0, wm, wn, lane, split);
#endif
}

// Pre-split operand planes for conv_wgrad_x3d_kernel: f32 src[n] -> bf16 hi[n], lo[n] (split8, the same
// hi / lo values the register-staged kernels make). 8 elements per thread; n % 8 == 0.
__global__ void __launch_bounds__(256) split_planes_kernel(const float* __restrict__ src, int64_t n8,
                                                           uint16_t* __restrict__ hi, uint16_t* __restrict__ lo) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  const float4 a = ((const float4*)src)[2 * i], b = ((const float4*)src)[2 * i + 1];
  uint4 h, l;
  split8(a, b, h, l);
  ((uint4*)hi)[i] = h;
  ((uint4*)lo)[i] = l;
}

// bf16x3 wgrad on pre-split operands (mx_conv_set_wgrad_variant(7)): dy and x arrive as bf16 hi / lo
// planes (split_planes_kernel), so each K-tile's four LDS planes [32 px][128] (dy hi, dy lo, x hi, x
// lo; 256-B rows, swz_w swizzle) are filled by LDS-DMA (buffer_load_dwordx4 ... lds: no register
// staging, no split VALU, no ds_write) one K-tile ahead of the MFMAs; fragments, MFMA order and the
// epilogue are those of conv_wgrad_x3_kernel, so the result is bitwise the same. Wave w fills rows
// [8w, 8w + 8) of every plane, 4 rows per DMA instruction; the swizzle is applied on the source chunk.
// p.dy / p.x: the hi planes; the lo planes follow at +P*K / +N*H*W*C elements.
__global__ void __launch_bounds__(NT, 2) conv_wgrad_x3d_kernel(WgP p) {
#if defined(__HIP_DEVICE_COMPILE__)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int PXT = 32, OPB = PXT * 256, STAGE = 4 * OPB;  // planes: dy hi, dy lo, x hi, x lo
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t ntn = (p.Ncol + 127) / 128;
  const int64_t ntiles = ((p.K + 127) / 128) * ntn;
  const int64_t work = xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  const int64_t split = work / ntiles, tile = work % ntiles;
  const int64_t mt = tile / ntn, nt = tile % ntn;
  const int64_t k0 = mt * 128, c0 = nt * 128;
  const int64_t pbeg = split * p.kchunk;
  const int64_t pend = min<int64_t>(p.P, pbeg + p.kchunk);
  if (pbeg >= pend) return;
  const int64_t dyel = p.P * p.K, xel = p.N * p.H * p.W * p.C;
  const i32x4 dyh = dma_rsrc(p.dy, (uint32_t)(dyel * 2)), dyl = dma_rsrc(p.dy + dyel, (uint32_t)(dyel * 2));
  const i32x4 xh = dma_rsrc(p.x, (uint32_t)(xel * 2)), xl = dma_rsrc(p.x + xel, (uint32_t)(xel * 2));
  const int OW = (int)p.OW, OH = (int)p.OH, H = (int)p.H, W = (int)p.W, C = (int)p.C;
  // this lane's two landing rows (j = 0, 1) and the logical chunk its 16 B come from
  const int dw = PXT % OW, dh = (PXT / OW) % OH, dn = PXT / (OW * OH);
  int px_n[2], px_oh[2], px_ow[2], px_i[2], ihb[2], iwb[2], xcol[2];
  uint32_t dcol[2];
  bool kok[2], cok[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = wave * 8 + j * 4 + (lane >> 4);
    const int lc = swz_w(row, lane & 15);
    const int64_t pi = pbeg + row;
    px_i[j] = (int)pi;
    const int64_t t = pi / OW;
    px_ow[j] = (int)(pi - t * OW);
    px_oh[j] = (int)(t % OH);
    px_n[j] = (int)(t / OH);
    kok[j] = k0 + lc * 8 < p.K;
    dcol[j] = (uint32_t)(k0 + lc * 8) * 2u;
    const int64_t col = c0 + lc * 8;
    cok[j] = col < p.Ncol;
    const int tap = cok[j] ? (int)(col / C) : 0;
    xcol[j] = cok[j] ? (int)(col - (int64_t)tap * C) : 0;
    const int r = tap / p.S, sq = tap - (tap / p.S) * p.S;
    ihb[j] = -p.pad_h + r;
    iwb[j] = -p.pad_w + sq;
  }
  const int pend32 = (int)pend;
  const uint32_t lds0 = lds_addr(smem);
  auto issue = [&](int buf) {
    const uint32_t D = lds0 + buf * STAGE;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bool pok = px_i[j] < pend32;
      const uint32_t od = (pok && kok[j]) ? __umul24((uint32_t)px_i[j], (uint32_t)(p.K * 2)) + dcol[j] : kOOB;
      const int ih = __mul24(px_oh[j], p.st_h) + ihb[j], iw = __mul24(px_ow[j], p.st_w) + iwb[j];
      const bool xok = pok && cok[j] && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      const uint32_t ox = xok ? (uint32_t)__mul24(__mul24(px_n[j], H) + ih, W) + (uint32_t)iw : 0u;
      const uint32_t oxb = xok ? __umul24(ox, (uint32_t)(C * 2)) + (uint32_t)xcol[j] * 2u : kOOB;
      const uint32_t dst = D + (wave * 8 + j * 4) * 256;
      lds_dma16(dyh, dst, od, 0u);
      lds_dma16(dyl, dst + OPB, od, 0u);
      lds_dma16(xh, dst + 2 * OPB, oxb, 0u);
      lds_dma16(xl, dst + 3 * OPB, oxb, 0u);
      px_i[j] += PXT;
      int ow = px_ow[j] + dw;
      const int c1 = ow >= OW ? 1 : 0;
      ow -= c1 * OW;
      int oh = px_oh[j] + dh + c1;
      const int c2 = oh >= OH ? 1 : 0;
      oh -= c2 * OH;
      px_ow[j] = ow;
      px_oh[j] = oh;
      px_n[j] += dn + c2;
    }
  };
  auto tr_read = [&](const char* T, int prow0, int colbase) -> s16x4 {
    const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    const int row = prow0 + 8 * g + q;
    const int colx = colbase + 4 * pp;
    const int chunk = colx >> 3, within = (colx & 7) * 2;
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(T + row * 256 + (swz_w(row, chunk) << 4) + within));
  };
  auto frag = [&](const char* T, int colbase) -> bf16x8 {
    const s16x4 lo = tr_read(T, 0, colbase), hi = tr_read(T, 4, colbase);
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int64_t nk = (pend - pbeg + PXT - 1) / PXT;
  issue(0);
  wait_vmcnt<0>();
  __syncthreads();
  for (int64_t it = 0; it < nk; ++it) {
    const int buf = (int)(it & 1);
    issue(buf ^ 1);  // the next K-tile (rows past the split read zeros; the last one lands unused)
    const char* Dh = smem + buf * STAGE;
    bf16x8 ah[4], al[4], bh[4], bl[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ah[i] = frag(Dh, wm * 64 + i * 16);
      al[i] = frag(Dh + OPB, wm * 64 + i * 16);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bh[j] = frag(Dh + 2 * OPB, wn * 64 + j * 16);
      bl[j] = frag(Dh + 3 * OPB, wn * 64 + j * 16);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
      }
    wait_vmcnt<0>();  // this wave's DMA of the next K-tile has landed; the barrier publishes everyone's
    __syncthreads();
  }
  wgrad_store(p, acc, k0, c0, wm, wn, lane, split);
#endif
}

// bf16x3 wgrad, wide block tile: 128 output channels x 256 (r,s,c) columns, 8 waves (2 x 4 wave tiles
// of 64 x 64, the same MFMA inner loop). Per 32-pixel K-step a block stores 32 x (128 + 256) split
// elements for 384 MFMAs: 0.75x the LDS stores and split VALU per MFMA of the 128 x 128 tile (whose
// LDS store path prices ~25 % of the P2 wgrad), and dy is re-read for every 256 columns instead of
// every 128. LDS: dy hi / lo [32][128] and x hi / lo as two [32][128] halves each, 256-B rows with the
// swz_w swizzle -- 6 sub-planes of 8 KiB per stage, double-buffered (96 KiB, one block per CU).
__global__ void __launch_bounds__(512, 1) conv_wgrad_x3w_kernel(WgP p) {
#if defined(__HIP_DEVICE_COMPILE__)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int PXT = 32, OPB = PXT * 256, STAGE = 6 * OPB;  // dy hi, dy lo, x hi 0/1, x lo 0/1
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int64_t ntn = (p.Ncol + 255) / 256;
  const int64_t ntiles = ((p.K + 127) / 128) * ntn;
  const int64_t work = xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  const int64_t split = work / ntiles, tile = work % ntiles;
  const int64_t mt = tile / ntn, nt = tile % ntn;
  const int64_t k0 = mt * 128, c0 = nt * 256;
  const int64_t pbeg = split * p.kchunk;
  const int64_t pend = min<int64_t>(p.P, pbeg + p.kchunk);
  if (pbeg >= pend) return;
  const float* __restrict__ dy = (const float*)p.dy;
  const float* __restrict__ x = (const float*)p.x;
  // dy: one 8-channel chunk of one pixel row per thread; x: one 8-column chunk of two pixel rows
  const int chd = tid & 15, rowd = tid >> 4;
  const int chx = tid & 31, rowx = tid >> 5;
  const bool k_ok = (k0 + chd * 8) < p.K;
  const int64_t col = c0 + chx * 8;
  const bool col_ok = col < p.Ncol;
  const int tap = col_ok ? (int)(col / p.C) : 0;
  const int cc = col_ok ? (int)(col - (int64_t)tap * p.C) : 0;
  const int r = tap / p.S, s = tap - (tap / p.S) * p.S;
  const int OW = (int)p.OW, OH = (int)p.OH, H = (int)p.H, W = (int)p.W, C = (int)p.C;
  const __amdgpu_buffer_rsrc_t dyr = __builtin_amdgcn_make_buffer_rsrc((void*)dy, (short)0, (int)(p.P * p.K * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, (int)(p.N * p.H * p.W * p.C * 4), 0x00020000);
  const int dw = PXT % OW, dh = (PXT / OW) % OH, dn = PXT / (OW * OH);
  const int ihb = -p.pad_h + r, iwb = -p.pad_w + s;
  int pxd = (int)(pbeg + rowd);
  int px_n[2], px_oh[2], px_ow[2], px_i[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int64_t pi = pbeg + rowx + 16 * i;
    px_i[i] = (int)pi;
    const int64_t t = pi / OW;
    px_ow[i] = (int)(pi - t * OW);
    px_oh[i] = (int)(t % OH);
    px_n[i] = (int)(t / OH);
  }
  const int pend32 = (int)pend;
  const uint32_t dy_col = (uint32_t)(k0 + chd * 8) * 4u;
  float4 rd[2], rx[2][2];
  auto load = [&]() {
    {
      const uint32_t od = (pxd < pend32 && k_ok) ? __umul24((uint32_t)pxd, (uint32_t)(p.K * 4)) + dy_col : kOOB;
      rd[0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(dyr, od, 0, 0));
      rd[1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(dyr, od + 16u, 0, 0));
      pxd += PXT;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bool pok = px_i[i] < pend32;
      const int ih = __mul24(px_oh[i], p.st_h) + ihb, iw = __mul24(px_ow[i], p.st_w) + iwb;
      const bool xok = pok && col_ok && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      const uint32_t ox = xok ? (uint32_t)__mul24(__mul24(px_n[i], H) + ih, W) + (uint32_t)iw : 0u;
      const uint32_t oxb = xok ? __umul24(ox, (uint32_t)(C * 4)) + (uint32_t)cc * 4u : kOOB;
      rx[i][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, oxb, 0, 0));
      rx[i][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, oxb + 16u, 0, 0));
      px_i[i] += PXT;
      int ow = px_ow[i] + dw;
      const int c1 = ow >= OW ? 1 : 0;
      ow -= c1 * OW;
      int oh = px_oh[i] + dh + c1;
      const int c2 = oh >= OH ? 1 : 0;
      oh -= c2 * OH;
      px_ow[i] = ow;
      px_oh[i] = oh;
      px_n[i] += dn + c2;
    }
  };
  // x column chunk chx of 32: half chx >> 4 (sub-plane), chunk chx & 15 within the 256-B row
  const int xh = chx >> 4, xc = chx & 15;
  auto store = [&](int buf) {
    char* D = smem + buf * STAGE;
    uint4 h, l;
    {
      const int off = rowd * 256 + (swz_w(rowd, chd) << 4);
      split8(rd[0], rd[1], h, l);
      *(uint4*)(D + off) = h;
      *(uint4*)(D + OPB + off) = l;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = rowx + 16 * i;
      const int off = row * 256 + (swz_w(row, xc) << 4);
      split8(rx[i][0], rx[i][1], h, l);
      *(uint4*)(D + (2 + xh) * OPB + off) = h;
      *(uint4*)(D + (4 + xh) * OPB + off) = l;
    }
  };
  auto tr_read = [&](const char* T, int prow0, int colbase) -> s16x4 {
    const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    const int row = prow0 + 8 * g + q;
    const int colx = colbase + 4 * pp;
    const int chunk = colx >> 3, within = (colx & 7) * 2;
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(T + row * 256 + (swz_w(row, chunk) << 4) + within));
  };
  auto frag = [&](const char* T, int colbase) -> bf16x8 {
    const s16x4 lo = tr_read(T, 0, colbase), hi = tr_read(T, 4, colbase);
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int64_t nk = (pend - pbeg + PXT - 1) / PXT;
  load();
  store(0);
  __syncthreads();
  const int xplane = wn >> 1, xcol = (wn & 1) * 64;
  for (int64_t it = 0; it < nk; ++it) {
    const int buf = (int)(it & 1);
    if (it + 1 < nk) load();
    const char* D = smem + buf * STAGE;
    bf16x8 ah[4], al[4], bh[4], bl[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ah[i] = frag(D, wm * 64 + i * 16);
      al[i] = frag(D + OPB, wm * 64 + i * 16);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bh[j] = frag(D + (2 + xplane) * OPB, xcol + j * 16);
      bl[j] = frag(D + (4 + xplane) * OPB, xcol + j * 16);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
      }
    if (it + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }
  wgrad_store(p, acc, k0, c0, wm, wn, lane, split);
#endif
}

// bf16x3 wgrad, 256 x 256 block tile at one wave per SIMD (4 waves, 2 x 2 wave tiles of 128 x 128,
// accumulators in the AGPR half of the 512-entry register file). PMC of the 128 x 128 kernel on the
// P2 3x3 wgrad: 4.4 VALU per MFMA and 36 % of wave cycles stalled on instruction issue -- the split
// (2 VALU per MFMA) and the other per-K-tile work are paid per 48 MFMAs a wave. Here a wave runs 192
// MFMAs per 32-pixel K-tile for the same per-thread staging work pattern, so the split and the LDS
// stores cost 1 VALU / 0.08 stores per MFMA and the K-tile's issue fits beside its MFMA time; the
// global loads of the next K-tile are issued before the MFMAs and consumed after them (3072 MFMA
// cycles to cover them). LDS per stage: dy hi / lo and x hi / lo, each [32 px][256] as two [32][128]
// sub-planes of 256-B rows (swz_w swizzle), double-buffered: 128 KiB, one block per CU.
__device__ __forceinline__ void wgrad_store8(const WgP& p, f32x4 (&acc)[8][8], int64_t k0, int64_t c0, int wm, int wn,
                                             int lane, int64_t split) {
  float* slab = p.slab ? p.slab + split * p.K * p.Ncol : nullptr;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int64_t k = k0 + wm * 128 + i * 16 + (lane >> 4) * 4 + rr;
        const int64_t cl = c0 + wn * 128 + j * 16 + (lane & 15);
        if (k >= p.K || cl >= p.Ncol) continue;
        if (slab) {
          slab[k * p.Ncol + cl] = acc[i][j][rr];
        } else {
          const int64_t o = wgrad_dst(p, k, (int)cl);
          if (o >= 0) p.dw[o] = acc[i][j][rr];
        }
      }
}

__global__ void __launch_bounds__(256, 1) conv_wgrad_x3ww_kernel(WgP p) {
#if defined(__HIP_DEVICE_COMPILE__)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int PXT = 32, SUB = PXT * 256, STAGE = 8 * SUB;  // sub-planes: dy hi 0/1, dy lo 0/1, x hi 0/1, x lo 0/1
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t ntn = (p.Ncol + 255) / 256;
  const int64_t ntiles = ((p.K + 255) / 256) * ntn;
  const int64_t work = xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  const int64_t split = work / ntiles, tile = work % ntiles;
  const int64_t mt = tile / ntn, nt = tile % ntn;
  const int64_t k0 = mt * 256, c0 = nt * 256;
  const int64_t pbeg = split * p.kchunk;
  const int64_t pend = min<int64_t>(p.P, pbeg + p.kchunk);
  if (pbeg >= pend) return;
  const float* __restrict__ dy = (const float*)p.dy;
  const float* __restrict__ x = (const float*)p.x;
  // this thread's fixed 8-wide chunk (0..31) of the dy k columns and of the x (r,s,c) columns; its
  // pixel rows of every K-tile: row0 + 8 i, i < 4
  const int ch = tid & 31, row0 = tid >> 5;
  const bool k_ok = (k0 + ch * 8) < p.K;
  const int64_t col = c0 + ch * 8;
  const bool col_ok = col < p.Ncol;
  const int tap = col_ok ? (int)(col / p.C) : 0;
  const int cc = col_ok ? (int)(col - (int64_t)tap * p.C) : 0;
  const int r = tap / p.S, s = tap - (tap / p.S) * p.S;
  const int OW = (int)p.OW, OH = (int)p.OH, H = (int)p.H, W = (int)p.W, C = (int)p.C;
  const __amdgpu_buffer_rsrc_t dyr = __builtin_amdgcn_make_buffer_rsrc((void*)dy, (short)0, (int)(p.P * p.K * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, (int)(p.N * p.H * p.W * p.C * 4), 0x00020000);
  const int dw = PXT % OW, dh = (PXT / OW) % OH, dn = PXT / (OW * OH);
  const int ihb = -p.pad_h + r, iwb = -p.pad_w + s;
  int px_n[4], px_oh[4], px_ow[4], px_i[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t pi = pbeg + row0 + 8 * i;
    px_i[i] = (int)pi;
    const int64_t t = pi / OW;
    px_ow[i] = (int)(pi - t * OW);
    px_oh[i] = (int)(t % OH);
    px_n[i] = (int)(t / OH);
  }
  const int pend32 = (int)pend;
  const uint32_t dy_col = (uint32_t)(k0 + ch * 8) * 4u;
  float4 rd[4][2], rx[4][2];
  auto load = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool pok = px_i[i] < pend32;
      const uint32_t od = (pok && k_ok) ? __umul24((uint32_t)px_i[i], (uint32_t)(p.K * 4)) + dy_col : kOOB;
      const int ih = __mul24(px_oh[i], p.st_h) + ihb, iw = __mul24(px_ow[i], p.st_w) + iwb;
      const bool xok = pok && col_ok && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      const uint32_t ox = xok ? (uint32_t)__mul24(__mul24(px_n[i], H) + ih, W) + (uint32_t)iw : 0u;
      const uint32_t oxb = xok ? __umul24(ox, (uint32_t)(C * 4)) + (uint32_t)cc * 4u : kOOB;
      rd[i][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(dyr, od, 0, 0));
      rd[i][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(dyr, od + 16u, 0, 0));
      rx[i][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, oxb, 0, 0));
      rx[i][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, oxb + 16u, 0, 0));
      px_i[i] += PXT;
      int ow = px_ow[i] + dw;
      const int c1 = ow >= OW ? 1 : 0;
      ow -= c1 * OW;
      int oh = px_oh[i] + dh + c1;
      const int c2 = oh >= OH ? 1 : 0;
      oh -= c2 * OH;
      px_ow[i] = ow;
      px_oh[i] = oh;
      px_n[i] += dn + c2;
    }
  };
  const int sub = ch >> 4, c16 = ch & 15;
  auto store = [&](int buf) {
    char* D = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = row0 + 8 * i;
      const int off = row * 256 + (swz_w(row, c16) << 4);
      uint4 h, l;
      split8(rd[i][0], rd[i][1], h, l);
      *(uint4*)(D + (0 + sub) * SUB + off) = h;
      *(uint4*)(D + (2 + sub) * SUB + off) = l;
      split8(rx[i][0], rx[i][1], h, l);
      *(uint4*)(D + (4 + sub) * SUB + off) = h;
      *(uint4*)(D + (6 + sub) * SUB + off) = l;
    }
  };
  auto tr_read = [&](const char* T, int prow0, int colbase) -> s16x4 {
    const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    const int row = prow0 + 8 * g + q;
    const int colx = colbase + 4 * pp;
    const int chunk = colx >> 3, within = (colx & 7) * 2;
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(T + row * 256 + (swz_w(row, chunk) << 4) + within));
  };
  auto frag = [&](const char* T, int colbase) -> bf16x8 {
    const s16x4 lo = tr_read(T, 0, colbase), hi = tr_read(T, 4, colbase);
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int64_t nk = (pend - pbeg + PXT - 1) / PXT;
  load();
  store(0);
  __syncthreads();
  for (int64_t it = 0; it < nk; ++it) {
    const int buf = (int)(it & 1);
    if (it + 1 < nk) load();
    const char* D = smem + buf * STAGE;
    // this wave's k rows wm*128.. (dy sub-plane wm) and columns wn*128.. (x sub-plane wn)
    const char* Ah = D + (0 + wm) * SUB;
    const char* Al = D + (2 + wm) * SUB;
    const char* Bh = D + (4 + wn) * SUB;
    const char* Bl = D + (6 + wn) * SUB;
    bf16x8 ah[8], al[8], bh[8], bl[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      ah[i] = frag(Ah, i * 16);
      al[i] = frag(Al, i * 16);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bh[j] = frag(Bh, j * 16);
      bl[j] = frag(Bl, j * 16);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
      }
    if (it + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }
  wgrad_store8(p, acc, k0, c0, wm, wn, lane, split);
#endif
}

__global__ void transpose_w_kernel(const uint16_t* __restrict__ w, int64_t K, int64_t RS, int64_t C, uint16_t* __restrict__ wt) {
  // w[K][RS][C] -> wt[C][RS][K]
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= K * RS * C) return;
  int64_t c = i % C, rs = (i / C) % RS, k = i / (C * RS);
  wt[(c * RS + rs) * K + k] = w[i];
}

// Per-step weight preparation, one pass over the f32 master weight w[K][C][R][S] (torch layout):
//   wk [K][R][S][Cpad] bf16      — fwd / wgrad operand (input channels zero-padded to Cpad)
//   wt [class][Cpad][Rc][Sc][Kpad] bf16 — dgrad operand, taps grouped by stride-parity class
// Tiles go through LDS so the f32 reads and both bf16 writes run along their contiguous axes
// (pack_plan; R*S <= 196).
struct PackP {
  const float* w;
  uint16_t* wk;
  uint16_t* wt;
  int64_t K, C, Cpad, Kpad;
  int R, S, st_h, st_w;
  int64_t off[4];
  int Rc[4], Sc[4];
  int dense;  // wt as [R][S][Cpad][Kpad]: the 1x1-GEMM dgrad operand of a conv whose output is 1x1
  // split: bf16x3 operands -- every layout is written twice, plane 0 = bf16(w) (hi) and plane 1 =
  // bf16(w - hi) (lo), the lo plane wk_plane / wt_plane elements after the hi plane
  int split;
  int64_t wk_plane, wt_plane;
  // tiling (pack_plan): wk tiles = kr output rows x cw input channels x all taps (nwk of them, first),
  // then wt tiles = 64 output channels x tct input channels x all taps
  int kr, cw, tct;
  int64_t nwk, nwt;
};

// Two tile kinds, each with contiguous f32 reads and 128-B bf16 write runs (values staged in LDS as
// bf16, so the rounding is the one f2bf of the f32 master value):
//  * wk tile: kr whole output rows (cw input channels x all taps each; cw = Cpad unless one row
//    exceeds the LDS tile) -- a per-row [C][RS] -> [RS][Cpad] transpose, both sides contiguous;
//  * wt tile: 64 output channels x tct input channels x all taps -- read as 64 contiguous runs of
//    tct*RS floats, written along the innermost Kpad axis as output-channel pairs.
static constexpr int PACK_LDS = 25600;  // bf16 elements (50 KiB)
static constexpr int PK = 64;

__device__ __forceinline__ uint32_t fdiv(uint32_t a, uint32_t d, float inv) {  // a / d for a < 2^22
  uint32_t q = (uint32_t)((float)a * inv);
  if (q * d > a) --q;
  else if ((q + 1) * d <= a) ++q;
  return q;
}

__device__ __forceinline__ void st_bf2(uint16_t* d, uint16_t a, uint16_t b, bool two) {
  if (two && ((uintptr_t)d & 3) == 0) {
    *(uint32_t*)d = (uint32_t)a | ((uint32_t)b << 16);
  } else {
    d[0] = a;
    if (two) d[1] = b;
  }
}

// plane 0 (hi) / 1 (lo) of the bf16x3 split of an f32 weight
__device__ __forceinline__ uint16_t plane_bf(float v, int plane) {
  const uint16_t h = f2bf(v);
  return plane ? f2bf(v - bf2f(h)) : h;
}

// T[row * ldt + j] = bf16(w[(k0 + row) * C * RS + c0 * RS + j]) for j < n_valid (zero past the real
// input channels / output rows); ldt % 4 == 0. plane 1: the lo part bf16(w - bf16(w)).
__device__ __forceinline__ void pack_stage(const PackP& p, int64_t k0, int64_t c0, int rows, int width, int ldt,
                                           uint16_t* T, int plane) {
  const int RS = p.R * p.S;
  const int64_t cend = p.C < c0 + width / RS ? p.C : c0 + width / RS;
  const int nvalid = cend > c0 ? (int)((cend - c0) * RS) : 0;
  // U independent loads in flight per thread before the first LDS write (a load -> ds_write loop
  // would wait out the full memory latency once per element)
  constexpr int U = 8;
  if ((p.C & 3) == 0 && (c0 & 3) == 0 && (width & 3) == 0 && ((uintptr_t)p.w & 15) == 0) {
    // float4 path: every row run starts 16-B aligned and holds whole groups of 4
    const int w4 = width >> 2, total4 = rows * w4, nv4 = nvalid >> 2;
    const float inv4 = 1.f / (float)w4;
    for (int base = 0; base < total4; base += 256 * U) {
      float4 v[U];
      int dst[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = base + u * 256 + threadIdx.x;
        const int row = (int)fdiv((uint32_t)e, (uint32_t)w4, inv4), j4 = e - row * w4;
        const int64_t k = k0 + row;
        dst[u] = e < total4 ? row * ldt + 4 * j4 : -1;
        v[u] = (e < total4 && k < p.K && j4 < nv4) ? *(const float4*)(p.w + (k * p.C + c0) * RS + 4 * j4)
                                                   : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (dst[u] >= 0)
          *(uint2*)(T + dst[u]) =
              make_uint2((uint32_t)plane_bf(v[u].x, plane) | ((uint32_t)plane_bf(v[u].y, plane) << 16),
                         (uint32_t)plane_bf(v[u].z, plane) | ((uint32_t)plane_bf(v[u].w, plane) << 16));
    }
    __syncthreads();
    return;
  }
  const float inv = 1.f / (float)width;
  const int total = rows * width;
  for (int base = 0; base < total; base += 256 * U) {
    float v[U];
    int dst[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = base + u * 256 + threadIdx.x;
      const int row = (int)fdiv((uint32_t)e, (uint32_t)width, inv), j = e - row * width;
      const int64_t k = k0 + row;
      dst[u] = e < total ? row * ldt + j : -1;
      v[u] = (e < total && k < p.K && j < nvalid) ? p.w[(k * p.C + c0) * RS + j] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (dst[u] >= 0) T[dst[u]] = plane_bf(v[u], plane);
  }
  __syncthreads();
}

__device__ __forceinline__ void pack_wk_tile(const PackP& p, int64_t t, uint16_t* T, int plane) {
  const int RS = p.R * p.S;
  const int64_t nc = (p.Cpad + p.cw - 1) / p.cw;
  const int64_t k0 = (t / nc) * p.kr, c0 = (t % nc) * p.cw;
  const int cwv = (int)(p.Cpad - c0 < p.cw ? p.Cpad - c0 : p.cw);
  const int width = cwv * RS, ldt = width + 4;
  pack_stage(p, k0, c0, p.kr, width, ldt, T, plane);
  uint16_t* wk = p.wk + plane * p.wk_plane;
  const int h = (cwv + 1) >> 1, per = RS * h;  // channel pairs per (row, tap)
  const float inv_per = 1.f / (float)per, inv_h = 1.f / (float)h;
  for (int e = threadIdx.x; e < p.kr * per; e += 256) {
    const int row = (int)fdiv((uint32_t)e, (uint32_t)per, inv_per), rem = e - row * per;
    const int rs = (int)fdiv((uint32_t)rem, (uint32_t)h, inv_h), c2 = rem - rs * h;
    const int64_t k = k0 + row;
    if (k >= p.K) continue;
    const int cc = 2 * c2;
    const uint16_t* tt = T + row * ldt + cc * RS + rs;
    st_bf2(wk + (k * RS + rs) * p.Cpad + c0 + cc, tt[0], cc + 1 < cwv ? tt[RS] : (uint16_t)0, cc + 1 < cwv);
  }
}

__device__ __forceinline__ void pack_wt_tile(const PackP& p, int64_t t, uint16_t* T, int plane) {
  const int RS = p.R * p.S;
  const int64_t nc = (p.Cpad + p.tct - 1) / p.tct;
  const int64_t k0 = (t / nc) * PK, c0 = (t % nc) * p.tct;
  const int width = p.tct * RS, ldt = width + 4;
  pack_stage(p, k0, c0, PK, width, ldt, T, plane);
  uint16_t* wt = p.wt + plane * p.wt_plane;
  constexpr int PK2 = PK / 2;
  const int per = RS * PK2;
  const float inv_per = 1.f / (float)per;
  for (int e = threadIdx.x; e < p.tct * per; e += 256) {
    const int cc = (int)fdiv((uint32_t)e, (uint32_t)per, inv_per), rem = e - cc * per;
    const int rs = rem / PK2, k2 = rem % PK2;  // PK2 is a power of two
    const int64_t k = k0 + 2 * k2, c = c0 + cc;
    if (k >= p.Kpad || c >= p.Cpad) continue;
    const uint16_t* tt = T + 2 * k2 * ldt + cc * RS + rs;
    int64_t dst;
    if (p.dense) {  // [R][S][Cpad][Kpad]: the 1x1-GEMM dgrad operand of a conv whose output is 1x1
      dst = ((int64_t)rs * p.Cpad + c) * p.Kpad + k;
    } else {  // tap-parity class q (r % st_h, s % st_w): [c][r / st_h][s / st_w][Kpad]
      const int r = rs / p.S, sx = rs - r * p.S;
      const int q = (r % p.st_h) * p.st_w + (sx % p.st_w);
      dst = p.off[q] + ((c * p.Rc[q] + r / p.st_h) * p.Sc[q] + sx / p.st_w) * p.Kpad + k;
    }
    st_bf2(wt + dst, tt[0], tt[ldt], k + 1 < p.Kpad);
  }
}

// tiles: nwk wk tiles, then nwt wt tiles; a split job's block writes both planes of its tile, the
// second staging re-reading the f32 region it has just read (L2-hot) instead of another block
// fetching it from HBM again
__device__ __forceinline__ void pack_tile(const PackP& p, int64_t t) {
  __shared__ uint16_t T[PACK_LDS];
  const int np = p.split ? 2 : 1;
  for (int plane = 0; plane < np; ++plane) {
    if (plane) __syncthreads();  // the previous plane's writes have read T
    if (t < p.nwk) pack_wk_tile(p, t, T, plane);
    else pack_wt_tile(p, t - p.nwk, T, plane);
  }
}

__global__ void __launch_bounds__(256) pack_weight_kernel(PackP p) { pack_tile(p, blockIdx.x); }

// Every conv weight of a step in one launch: block -> (job, tile) through the tile prefix sums.
__global__ void __launch_bounds__(256) pack_batched_kernel(const PackP* __restrict__ jobs, const int64_t* __restrict__ prefix,
                                                           int njobs) {
  const int64_t b = blockIdx.x;
  int lo = 0, hi = njobs - 1;  // last job with prefix[j] <= b
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (prefix[mid] <= b) lo = mid; else hi = mid - 1;
  }
  const PackP p = jobs[lo];
  pack_tile(p, b - prefix[lo]);
}

// ---------------------------------------------------------------------------------------------
// SGD step fused with the operand pack: a conv weight's update and its bf16 operand layouts in ONE
// pass (mx_sgd_pack_step). The per-step order was sgd_kernel (p, g, buf -> p, buf) and then
// pack_batched_kernel re-reading every updated f32 weight twice (wk tile, wt tile); here a block owns
// a kr x tc x (all taps) tile of w[K][C][R][S]: it updates the tile in registers (p, buf written back),
// keeps the (hi, lo) bf16 pair of each new weight in LDS as one u32, and writes both the wk and the wt
// layout from there. Each weight element is read once and written once per layout, as sgd + pack
// would produce it (same sgd_update, same rounding). Non-conv parameters take the plain
// multi-tensor SGD blocks of the same launch.
struct SgdJob {
  float* p;
  float* b;
  int64_t n;
  int first, fused;
  int kr, tc;    // fused tile: kr output rows x tc input channels x all taps (powers of two)
  int64_t ncb;   // channel blocks (cdiv(Cpad, tc)) per row block
  PackP pk;      // fused: pk.w == p
};
struct SgdHyper {
  float lr, momentum, dampening, wd;
  int nesterov;
};
static constexpr int SGDP_PER_BLOCK = 2048;

__device__ __forceinline__ uint32_t hilo_word(float v) {  // bf16(v) | bf16(v - bf16(v)) << 16
  const uint16_t h = f2bf(v);
  return (uint32_t)h | ((uint32_t)f2bf(v - bf2f(h)) << 16);
}

__device__ __forceinline__ void sgd_plain_block(const SgdJob& J, const float* __restrict__ g, int64_t blk,
                                                const SgdHyper& h) {
  const int64_t e0 = blk * SGDP_PER_BLOCK, e1 = min<int64_t>(J.n, e0 + SGDP_PER_BLOCK);
  float* __restrict__ p = J.p;
  float* __restrict__ b = J.b;
  const bool first = J.first;
  if (((((uintptr_t)p) | ((uintptr_t)g) | ((uintptr_t)b)) & 15u) == 0) {
    for (int64_t e = e0 + threadIdx.x * 4; e + 3 < e1; e += 256 * 4) {
      float4 pv = *(float4*)(p + e), bv = *(float4*)(b + e);
      const float4 gv = *(const float4*)(g + e);
      sgd_update(pv.x, gv.x, bv.x, first, h.lr, h.momentum, h.dampening, h.wd, h.nesterov);
      sgd_update(pv.y, gv.y, bv.y, first, h.lr, h.momentum, h.dampening, h.wd, h.nesterov);
      sgd_update(pv.z, gv.z, bv.z, first, h.lr, h.momentum, h.dampening, h.wd, h.nesterov);
      sgd_update(pv.w, gv.w, bv.w, first, h.lr, h.momentum, h.dampening, h.wd, h.nesterov);
      *(float4*)(p + e) = pv;
      *(float4*)(b + e) = bv;
    }
    const int64_t tail = e0 + ((e1 - e0) & ~(int64_t)3);
    for (int64_t e = tail + threadIdx.x; e < e1; e += 256)
      sgd_update(p[e], g[e], b[e], first, h.lr, h.momentum, h.dampening, h.wd, h.nesterov);
  } else {
    for (int64_t e = e0 + threadIdx.x; e < e1; e += 256)
      sgd_update(p[e], g[e], b[e], first, h.lr, h.momentum, h.dampening, h.wd, h.nesterov);
  }
}

__device__ __forceinline__ void sgd_pack_tile(const SgdJob& J, const float* __restrict__ g, int64_t t,
                                              const SgdHyper& h, uint32_t* T) {
  const PackP& pk = J.pk;
  const int RS = pk.R * pk.S;
  const int kr = J.kr, tc = J.tc;
  const int64_t k0 = (t / J.ncb) * kr, c0 = (t % J.ncb) * tc;
  const int width = tc * RS, ldt = width + 1;  // odd row stride: column reads spread over the banks
  const int64_t cend = pk.C < c0 + tc ? pk.C : c0 + tc;
  const int nvalid = cend > c0 ? (int)((cend - c0) * RS) : 0;
  const bool first = J.first;
  float* __restrict__ p = J.p;
  float* __restrict__ b = J.b;
  // 1. update the tile: row k's run of nvalid weights starts at (k * C + c0) * RS
  if ((pk.C & 3) == 0 && ((((uintptr_t)p) | ((uintptr_t)g) | ((uintptr_t)b)) & 15u) == 0) {
    const int w4 = width >> 2, nv4 = nvalid >> 2;
    const float inv4 = 1.f / (float)w4;
    for (int e = threadIdx.x; e < kr * w4; e += 256) {
      const int row = (int)fdiv((uint32_t)e, (uint32_t)w4, inv4), j4 = e - row * w4;
      const int64_t k = k0 + row;
      uint32_t o0 = 0, o1 = 0, o2 = 0, o3 = 0;
      if (k < pk.K && j4 < nv4) {
        const int64_t i = (k * pk.C + c0) * RS + 4 * j4;
        float4 pv = *(float4*)(p + i), bv = *(float4*)(b + i);
        const float4 gv = *(const float4*)(g + i);
        sgd_update(pv.x, gv.x, bv.x, first, h.lr, h.momentum, h.dampening, h.wd, h.nesterov);
        sgd_update(pv.y, gv.y, bv.y, first, h.lr, h.momentum, h.dampening, h.wd, h.nesterov);
        sgd_update(pv.z, gv.z, bv.z, first, h.lr, h.momentum, h.dampening, h.wd, h.nesterov);
        sgd_update(pv.w, gv.w, bv.w, first, h.lr, h.momentum, h.dampening, h.wd, h.nesterov);
        *(float4*)(p + i) = pv;
        *(float4*)(b + i) = bv;
        o0 = hilo_word(pv.x); o1 = hilo_word(pv.y); o2 = hilo_word(pv.z); o3 = hilo_word(pv.w);
      }
      uint32_t* d = T + row * ldt + 4 * j4;
      d[0] = o0; d[1] = o1; d[2] = o2; d[3] = o3;
    }
  } else {
    const float inv = 1.f / (float)width;
    for (int e = threadIdx.x; e < kr * width; e += 256) {
      const int row = (int)fdiv((uint32_t)e, (uint32_t)width, inv), j = e - row * width;
      const int64_t k = k0 + row;
      uint32_t o = 0;
      if (k < pk.K && j < nvalid) {
        const int64_t i = (k * pk.C + c0) * RS + j;
        float pv = p[i], bv = b[i];
        sgd_update(pv, g[i], bv, first, h.lr, h.momentum, h.dampening, h.wd, h.nesterov);
        p[i] = pv;
        b[i] = bv;
        o = hilo_word(pv);
      }
      T[row * ldt + j] = o;
    }
  }
  __syncthreads();
  const int np = pk.split ? 2 : 1;
  // 2. wk [K][R][S][Cpad]: runs of tc channels per (row, tap), written as channel pairs
  if (pk.wk) {
    const int h2 = tc >> 1, per = RS * h2;
    const float inv_per = 1.f / (float)per, inv_h = 1.f / (float)h2;
    for (int e = threadIdx.x; e < kr * per; e += 256) {
      const int row = (int)fdiv((uint32_t)e, (uint32_t)per, inv_per), rem = e - row * per;
      const int rs = (int)fdiv((uint32_t)rem, (uint32_t)h2, inv_h), c2 = rem - rs * h2;
      const int64_t k = k0 + row, c = c0 + 2 * c2;
      if (k >= pk.K || c >= pk.Cpad) continue;
      const uint32_t* tt = T + row * ldt + 2 * c2 * RS + rs;
      const uint32_t a = tt[0], a2 = tt[RS];  // Cpad is even: c + 1 < Cpad
      const int64_t dst = (k * RS + rs) * pk.Cpad + c;
      for (int pl = 0; pl < np; ++pl)
        *(uint32_t*)(pk.wk + pl * pk.wk_plane + dst) =
            pl ? (a >> 16) | (a2 & 0xffff0000u) : (a & 0xffffu) | (a2 << 16);
    }
  }
  // 3. wt (dgrad layout): runs along the output channels, written as output-channel pairs
  if (pk.wt) {
    const int kr2 = kr >> 1, per = RS * kr2;
    const float inv_per = 1.f / (float)per, inv_k = 1.f / (float)kr2;
    for (int e = threadIdx.x; e < tc * per; e += 256) {
      const int cc = (int)fdiv((uint32_t)e, (uint32_t)per, inv_per), rem = e - cc * per;
      const int rs = (int)fdiv((uint32_t)rem, (uint32_t)kr2, inv_k), k2 = rem - rs * kr2;
      const int64_t k = k0 + 2 * k2, c = c0 + cc;
      if (k >= pk.Kpad || c >= pk.Cpad) continue;
      const uint32_t* tt = T + 2 * k2 * ldt + cc * RS + rs;
      const uint32_t a = tt[0], a2 = tt[ldt];  // Kpad is even: k + 1 < Kpad
      int64_t dst;
      if (pk.dense) {
        dst = ((int64_t)rs * pk.Cpad + c) * pk.Kpad + k;
      } else {
        const int r = rs / pk.S, sx = rs - r * pk.S;
        const int q = (r % pk.st_h) * pk.st_w + (sx % pk.st_w);
        dst = pk.off[q] + ((c * pk.Rc[q] + r / pk.st_h) * pk.Sc[q] + sx / pk.st_w) * pk.Kpad + k;
      }
      for (int pl = 0; pl < np; ++pl)
        *(uint32_t*)(pk.wt + pl * pk.wt_plane + dst) =
            pl ? (a >> 16) | (a2 & 0xffff0000u) : (a & 0xffffu) | (a2 << 16);
    }
  }
}

// block -> (job, tile or 2048-element chunk) through the prefix sums; grads by job index (their
// pointers change more often than the job table)
__global__ void __launch_bounds__(256) sgd_pack_kernel(const SgdJob* __restrict__ jobs, const int64_t* __restrict__ prefix,
                                                       const float* const* __restrict__ grads, int njobs, SgdHyper h) {
  extern __shared__ uint32_t Tsm[];
  const int64_t bidx = blockIdx.x;
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (prefix[mid] <= bidx) lo = mid; else hi = mid - 1;
  }
  const SgdJob J = jobs[lo];
  if (J.fused) sgd_pack_tile(J, grads[lo], bidx - prefix[lo], h, Tsm);
  else sgd_plain_block(J, grads[lo], bidx - prefix[lo], h);
}

// Host: tile sizes of one pack job (both tile kinds fit PACK_LDS, rows padded by 4 elements)
static int pack_plan(PackP& p) {
  const int RS = p.R * p.S;
  if (RS > 196) return MX_EINVAL;
  p.tct = RS == 1 ? 64 : (RS <= 9 ? 32 : ((392 / RS) & ~3));  // multiples of 4: float4 staging
  if (p.tct < 2) p.tct = 2;
  int64_t cw = p.Cpad;
  if (cw * RS + 4 > PACK_LDS) cw = ((PACK_LDS - 4) / RS) & ~3ll;
  p.cw = (int)cw;
  int64_t kr = 12288 / (cw * RS);
  if (kr > 64) kr = 64;
  while (kr > 1 && kr * (cw * RS + 4) > PACK_LDS) --kr;
  if (kr < 1) kr = 1;
  p.kr = (int)kr;
  p.nwk = p.wk ? cdiv(p.K, p.kr) * cdiv(p.Cpad, p.cw) : 0;
  p.nwt = p.wt ? cdiv(p.Kpad, (int64_t)PK) * cdiv(p.Cpad, (int64_t)p.tct) : 0;
  p.wk_plane = p.K * RS * p.Cpad;
  p.wt_plane = p.Cpad * RS * p.Kpad;
  return MX_OK;
}

// KRSC bf16 weight -> the dgrad parity-class layout of pack_weight_kernel (element-wise; used by
// the convenience mx_conv2d_dgrad only)
__global__ void krsc_to_dgrad_kernel(const uint16_t* __restrict__ w, PackP p) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.K * p.R * p.S * p.C) return;
  const int64_t c = i % p.C, t = i / p.C;
  const int sx = (int)(t % p.S), r = (int)((t / p.S) % p.R);
  const int64_t k = t / ((int64_t)p.S * p.R);
  const int q = (r % p.st_h) * p.st_w + sx % p.st_w;
  p.wt[p.off[q] + ((c * p.Rc[q] + r / p.st_h) * p.Sc[q] + sx / p.st_w) * p.Kpad + k] = w[i];
}


// ------------------------------------------------------------------------------------------------
// ResNet stem (torchvision resnet50 conv1 -> bn1 -> ReLU), bf16x3: a 7x7 conv of an NHWC f32 image whose
// first 4 channels (RGB + one zero pad) are read, to 64 channels. The generic x3 kernels walk
// K = 7*7*8 = 392 (two-thirds zero products, padded to 416); here one MFMA K-step of 32 is one filter
// row r: 8 taps (s = 0..6 and a zero s = 7) x 4 channels, so 7 K-steps (224) cover the 147 real
// products. The MFMA's A operand is the weights (rows = output channels; the packed hi / lo planes are
// rearranged into fragment-ready [plane][r][k][s*4 + c] rows in LDS once per block), B the pixels:
// lane (g, c16) of a 16-pixel tile loads taps 2g, 2g+1 of pixel c16 as two float4 (channels 0..3)
// and splits them into hi / lo in registers -- no LDS staging of the image. A wave owns 64 output
// pixels (STEM_T tiles of 16, one BatchNorm statistics row) for all 64 channels: per-channel
// (sum, sum of squares) partials of the train-mode BatchNorm, or bias + activation, in the epilogue;
// the accumulator layout (4 consecutive channels of one pixel per lane) gives float4 stores. Blocks
// loop over contiguous pixel ranges (XCD-aware), so the weight rearrangement is paid ~2 x CUs times.
static constexpr int STEM_T = 4, STEM_K = 64, STEM_R = 7;
struct StemP {
  const float* x;       // [N][H][W][C] f32, channels 0..3 read
  const uint16_t* w;    // [2][64][7][7][C] bf16 hi / lo planes (mx_conv2d_fwd_x3's packing)
  const float* bias;    // [64] or null
  float* y;             // [N][Ho][Wo][64]
  float* stats;         // null, or [2][mblocks][64] BatchNorm partials (sum; sum of squares)
  int64_t M, mblocks;   // M = N * Ho * Wo
  int64_t tiles_per_block;
  int H, W, C, Ho, Wo, st_h, st_w, pad_h, pad_w, act;
  int xbytes;           // bytes of x: the buffer loads' range (out-of-range offsets read zeros)
};

__global__ void __launch_bounds__(256, 2) conv_stem_x3_kernel(StemP p) {
#if defined(__HIP_DEVICE_COMPILE__)
  __shared__ __attribute__((aligned(16))) uint16_t wl[2 * STEM_R * STEM_K * 32];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = p.H, W = p.W, C = p.C;
  {
    // (plane, r, k, s) quads of 4 channels: 8-B loads of the packed planes, zeros at s = 7
    const int64_t plane = (int64_t)STEM_K * 49 * C;
    for (int i = tid; i < 2 * STEM_R * STEM_K * 8; i += 256) {
      const int sx = i & 7, k = (i >> 3) & 63, r = (i >> 9) % STEM_R, pl = i / (8 * 64 * STEM_R);
      uint2 v = make_uint2(0u, 0u);
      if (sx < 7) v = *(const uint2*)(p.w + pl * plane + ((int64_t)k * 49 + r * 7 + sx) * C);
      *(uint2*)(wl + ((pl * STEM_R + r) * STEM_K + k) * 32 + sx * 4) = v;
    }
  }
  __syncthreads();
  const int64_t blk = xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  const int g = lane >> 4, c16 = lane & 15;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.xbytes, 0x00020000);
  const int64_t ntiles = (p.M + 16 * STEM_T - 1) / (16 * STEM_T);
  const int64_t tbeg = blk * p.tiles_per_block, tend = min<int64_t>(ntiles, tbeg + p.tiles_per_block);
  float4 bias4[4];  // this lane's 4 channels of each 16-channel column tile (loaded once: no vmcnt wait
                    // between the epilogue's stores)
#pragma unroll
  for (int j = 0; j < 4; ++j)
    bias4[j] = p.bias ? *(const float4*)(p.bias + 16 * j + 4 * g) : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t tile = tbeg + wave; tile < tend; tile += 4) {
    const int64_t m0 = tile * (16 * STEM_T);
    int rowb[STEM_T], ih0[STEM_T], iw0[STEM_T];
#pragma unroll
    for (int t = 0; t < STEM_T; ++t) {
      const int64_t m = m0 + t * 16 + c16;
      if (m < p.M) {  // M < 2^31 (conv_check): 32-bit index math
        const int mi = (int)m, q = mi / p.Wo, ow = mi - q * p.Wo;
        const int n = q / p.Ho, oh = q - n * p.Ho;
        rowb[t] = n * H;
        ih0[t] = oh * p.st_h - p.pad_h;
        iw0[t] = ow * p.st_w - p.pad_w + 2 * g;
      } else {
        rowb[t] = 0;
        ih0[t] = -(1 << 20);  // every row invalid
        iw0[t] = 0;
      }
    }
    f32x4 acc[STEM_T][4];
#pragma unroll
    for (int t = 0; t < STEM_T; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[t][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // filter row r + 1's image loads are issued before row r's MFMAs (two register stages; the
    // scheduling barriers keep the compiler from sinking them next to their first use)
    float4 ra[2][STEM_T], rb[2][STEM_T];
    auto issue = [&](const int r, float4 (&xa)[STEM_T], float4 (&xb)[STEM_T]) {
#pragma unroll
      for (int t = 0; t < STEM_T; ++t) {
        const int ih = ih0[t] + r;
        const bool rok = (unsigned)ih < (unsigned)H;
        const uint32_t e0 = ((uint32_t)(rowb[t] + ih) * (uint32_t)W + (uint32_t)iw0[t]) * (uint32_t)C;
        const bool ok0 = rok && (unsigned)iw0[t] < (unsigned)W;
        const bool ok1 = rok && g < 3 && (unsigned)(iw0[t] + 1) < (unsigned)W;
        xa[t] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, ok0 ? e0 * 4u : kOOB, 0, 0));
        xb[t] = __builtin_bit_cast(float4,
                                   __builtin_amdgcn_raw_buffer_load_b128(xr, ok1 ? (e0 + (uint32_t)C) * 4u : kOOB, 0, 0));
      }
    };
    issue(0, ra[0], rb[0]);
#pragma unroll
    for (int r = 0; r < STEM_R; ++r) {
      const int b = r & 1;
      if (r + 1 < STEM_R) issue(r + 1, ra[b ^ 1], rb[b ^ 1]);
      __builtin_amdgcn_sched_barrier(0);
      bf16x8 ah[4], al[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = r * STEM_K + 16 * j + c16;
        ah[j] = *(const bf16x8*)(wl + row * 32 + g * 8);
        al[j] = *(const bf16x8*)(wl + (STEM_R * STEM_K + row) * 32 + g * 8);
      }
#pragma unroll
      for (int t = 0; t < STEM_T; ++t) {
        uint4 h, l;
        split8(ra[b][t], rb[b][t], h, l);
        const bf16x8 bh = __builtin_bit_cast(bf16x8, h), bl = __builtin_bit_cast(bf16x8, l);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[j], bh, acc[t][j], 0, 0, 0);
          acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[j], bl, acc[t][j], 0, 0, 0);
          acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[j], bh, acc[t][j], 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (p.stats) {  // this wave's 64 pixels are statistics row m0 / 64
      const int64_t srow = m0 / SROWS;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float s[4] = {0.f, 0.f, 0.f, 0.f}, q[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < STEM_T; ++t) {
          const bool ok = m0 + t * 16 + c16 < p.M;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float v = ok ? acc[t][j][i] : 0.f;
            s[i] += v;
            q[i] += v * v;
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) {
            s[i] += __shfl_xor(s[i], o);
            q[i] += __shfl_xor(q[i], o);
          }
        if (c16 == 0) {
          const int ch = 16 * j + 4 * g;
          *(float4*)(p.stats + srow * STEM_K + ch) = make_float4(s[0], s[1], s[2], s[3]);
          *(float4*)(p.stats + (p.mblocks + srow) * STEM_K + ch) = make_float4(q[0], q[1], q[2], q[3]);
        }
      }
    }
#pragma unroll
    for (int t = 0; t < STEM_T; ++t) {
      const int64_t m = m0 + t * 16 + c16;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ch = 16 * j + 4 * g;
        const float4 b = bias4[j];
        float4 v = make_float4(acc[t][j][0] + b.x, acc[t][j][1] + b.y, acc[t][j][2] + b.z, acc[t][j][3] + b.w);
        if (p.act == 1) {
          v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
        }
        *(float4*)(p.y + m * STEM_K + ch) = v;
      }
    }
  }
#endif
}

}  // namespace mx

using namespace mx;

static int conv_check(const mx_conv_shape* s) {
  MX_CHECK_ARG(s && s->N > 0 && s->H > 0 && s->W > 0 && s->C > 0 && s->K > 0 && s->R > 0 && s->S > 0,
               "conv: bad shape");
  MX_CHECK_ARG(s->stride_h > 0 && s->stride_w > 0 && s->pad_h >= 0 && s->pad_w >= 0, "conv: bad stride/pad");
  int64_t ho = (s->H + 2 * s->pad_h - s->R) / s->stride_h + 1, wo = (s->W + 2 * s->pad_w - s->S) / s->stride_w + 1;
  MX_CHECK_ARG(ho == s->Ho && wo == s->Wo, "conv: Ho/Wo (%lld,%lld) inconsistent, expected (%lld,%lld)",
               (long long)s->Ho, (long long)s->Wo, (long long)ho, (long long)wo);
  MX_CHECK_ARG(s->N * s->H * s->W < (1ll << 31) && s->N * s->Ho * s->Wo < (1ll << 31), "conv: too many pixels");
  return MX_OK;
}

// rows of the BatchNorm statistics partials (64 output pixels each)
extern "C" int64_t mx_conv_mblocks(const mx_conv_shape* s) { return cdiv(s->N * s->Ho * s->Wo, SROWS); }

// Kernel variant (mx_conv_set_variant): 0 register staging, 1/2 direct-to-LDS 2-stage (2 also
// direct-to-LDS wgrad), 3..6 multi-stage direct-to-LDS, 7 (default) per-launch choice of 3 / 4.
static int g_conv_variant = 7;

// GEMM geometry of one launch and its split-K factor: grids that would leave the chip under-filled
// (< ~1.25 blocks per CU) split the K loop, keeping >= 4 K-tiles (of 64) per split.
struct Geo {
  int64_t M, Ncol, Kdim, tiles, nk;
  int splits, bmt, bn;
  bool narrow;
};
static int num_cus();
static int g_force_bmt = 0, g_force_bn = 0;  // mx_conv_set_tile (0 = automatic)
extern "C" int mx_conv_set_tile(int bmt, int bn) {
  MX_CHECK_ARG((bmt == 0 && bn == 0) || ((bmt == 64 || bmt == 128 || bmt == 256) && (bn == 64 || bn == 128 || bn == 256)),
               "mx_conv_set_tile: (0,0) auto, or bmt 64/128/256 (256: bf16x3 kernels only) x bn 64/128/256");
  g_force_bmt = bmt;
  g_force_bn = bn;
  return MX_OK;
}

static int g_buf_stages = 0;  // mx_conv_set_stages: LDS ring depth of the 64x128 / 128x128 buffer kernels
extern "C" int mx_conv_set_stages(int n) {
  MX_CHECK_ARG(n == 0 || n == 3 || n == 4 || n == 5 || n == 6,
               "mx_conv_set_stages: 0 (auto), 3, 4, 5 or 6 (x3 kernels: 3 alternative ring, 4 2x2 wave tiles, "
               "5 alternative ring with wide wave tiles)");
  g_buf_stages = n;
  return MX_OK;
}
static int g_conv_debug = 0;  // mx_conv_set_debug: bf16x3 buffer kernel timing-only bits (see the kernel)
extern "C" int mx_conv_set_debug(int v) {
  MX_CHECK_ARG(v == 0, "mx_conv_set_debug: the timing-only kernel bits are compiled out (0 only)");
  g_conv_debug = v;
  return MX_OK;
}
static int g_conv_korder = 1;  // mx_conv_set_korder: K-tile order of the buffer kernels (ConvP::korder)
extern "C" int mx_conv_set_korder(int v) {
  MX_CHECK_ARG(v == 0 || v == 1, "mx_conv_set_korder: 0 tap-major, 1 channel-major");
  g_conv_korder = v;
  return MX_OK;
}
static int g_max_splits = 0;  // mx_conv_set_max_splits (0 = automatic, 1 = never split K)
extern "C" int mx_conv_set_max_splits(int n) {
  MX_CHECK_ARG(n >= 0 && n <= 16, "mx_conv_set_max_splits: 0 (auto) .. 16");
  g_max_splits = n;
  return MX_OK;
}

static Geo make_geo(int64_t M, int64_t Ncol, int64_t Kdim) {
  Geo g;
  g.M = M; g.Ncol = Ncol; g.Kdim = Kdim;
  g.narrow = g.Ncol <= 64;
  g.bn = g.narrow ? 64 : 128;
  g.bmt = BM;
  g.tiles = cdiv(g.M, BM) * cdiv(g.Ncol, g.bn);
  if (g_conv_variant == 9 && g.Ncol >= 256) {
    g.bn = 256;
    g.tiles = cdiv(g.M, BM) * cdiv(g.Ncol, 256);
  } else if (g_conv_variant == 7 && !g.narrow && g.tiles >= 320) {
    // big grids: pick the block tile by (relative per-round throughput) x (wave fill), where a
    // round is one resident block per slot (occupancy x CUs): 128x256 reads the gathered A operand
    // once per 256 output channels and issues 12 LDS reads per 32 MFMAs (fastest per full round),
    // but few, large tiles leave the last round mostly empty (measured, MI355X: P2 3x3 picks
    // 128x128, the box-head 3x3 on 1024 RoIs 128x256, layer2 3x3 64x128)
    struct Cand { int bmt, bn, occ; double thr; };
    const Cand cand[3] = {{128, 256, 2, 1.0}, {128, 128, 3, 0.78}, {64, 128, 4, 0.62}};
    const int64_t cus = num_cus();
    double best = -1.0;
    for (const Cand& c : cand) {
      if (c.bn > g.Ncol) continue;
      const int64_t tiles = cdiv(g.M, c.bmt) * cdiv(g.Ncol, c.bn), slots = c.occ * cus;
      const double fill = (double)tiles / (double)(cdiv(tiles, slots) * slots);
      if (c.thr * fill > best) {
        best = c.thr * fill;
        g.bmt = c.bmt; g.bn = c.bn; g.tiles = tiles;
      }
    }
  }
  const int64_t ntn = cdiv(g.Ncol, g.bn);
  // small grids: 64-row tiles first (twice the blocks, no partial-sum traffic), split-K only below that
  if (g.bn != 256 && g.bmt == BM && (g_conv_variant == 8 || (g_conv_variant == 7 && g.tiles < 320))) {
    g.bmt = 64;
    g.tiles = cdiv(g.M, 64) * ntn;
  }
  if (g_force_bmt) {
    g.bmt = std::min(g_force_bmt, 128);
    g.bn = g_force_bn;
    g.narrow = g.bn == 64;
    g.tiles = cdiv(g.M, g.bmt) * cdiv(g.Ncol, g.bn);
  }
  g.nk = cdiv(g.Kdim, BK);
  g.splits = 1;
  const int64_t split_below = 320;
  if (g_conv_variant >= 1 && g.Ncol % 8 == 0 && g.tiles < split_below && g.nk >= 8) {
    int64_t sp = std::min<int64_t>(std::min<int64_t>(cdiv(640, g.tiles), g.nk / 4), 16);
    g.splits = (int)std::max<int64_t>(1, sp);
  }
  if (g_max_splits && g.splits > g_max_splits) g.splits = g_max_splits;
  return g;
}

// The variant a launch runs: long K loops on big grids favour 64-wide K-tiles (fewer barriers),
// short loops and small / split grids the 3-deep 32-wide ring at 3 blocks per CU; 64-row tiles
// for grids under ~1.25 blocks per CU.
static int launch_kind(const Geo& g) {
  if (g.bn == 256 && g.bmt == 128) return 9;
  if (g.bmt == 64) return 8;
  if (g_conv_variant != 7) return g_conv_variant;
  if (g.splits > 1 || g.nk < 16) return 3;
  // wave quantisation: BK32x3 holds 3 blocks per CU, BK64x2 holds 2 (each then ~1.5x faster)
  const int64_t cus = num_cus();
  const double c3 = (double)cdiv(g.tiles, 3 * cus), c4 = (double)cdiv(g.tiles, 2 * cus) * (2.0 / 3.0);
  return c4 < c3 ? 4 : 3;
}

// dgrad stride-parity classes. dx(h) receives dy((h + pad - r) / st) only from taps with
// r = (h + pad) mod st, so the rows with h = st*hh + ph form an independent dense GEMM over the
// taps r = r0 + st*ri (r0 = (ph + pad) mod st): dx[n, st*hh+ph] = sum dy[n, hh + dh - ri] w_t[ri],
// dh = (ph + pad - r0) / st. The classes partition both dx and the taps; wt stores each tap-parity
// class's [C][Rc][Sc][K] block contiguously (block index = tap parity r0*st_w + s0).
struct DClass {
  int ph, pw, r0, s0, Rc, Sc, dh, dw;
  int64_t Hc, Wc, off;
};
static int tap_count(int R, int r0, int st) { return r0 < R ? (R - r0 + st - 1) / st : 0; }
static int dgrad_classes(const mx_conv_shape* s, int64_t Cpad, int64_t Kpad, DClass* out, int64_t* blk_off,
                         int* blk_R, int* blk_S) {
  const int sh = s->stride_h, sw = s->stride_w;
  // block offsets by tap parity
  int64_t off = 0;
  for (int a = 0; a < sh; ++a)
    for (int b = 0; b < sw; ++b) {
      const int q = a * sw + b;
      blk_R[q] = tap_count((int)s->R, a, sh);
      blk_S[q] = tap_count((int)s->S, b, sw);
      blk_off[q] = off;
      off += Cpad * blk_R[q] * blk_S[q] * Kpad;
    }
  int n = 0;
  for (int ph = 0; ph < sh; ++ph)
    for (int pw = 0; pw < sw; ++pw) {
      DClass c;
      c.ph = ph; c.pw = pw;
      c.r0 = (ph + s->pad_h) % sh; c.s0 = (pw + s->pad_w) % sw;
      const int q = c.r0 * sw + c.s0;
      c.Rc = blk_R[q]; c.Sc = blk_S[q]; c.off = blk_off[q];
      c.dh = (ph + s->pad_h - c.r0) / sh; c.dw = (pw + s->pad_w - c.s0) / sw;
      c.Hc = ph < s->H ? (s->H - ph + sh - 1) / sh : 0;
      c.Wc = pw < s->W ? (s->W - pw + sw - 1) / sw : 0;
      out[n++] = c;
    }
  return n;
}

static size_t wgrad_ws(const mx_conv_shape* s);

extern "C" size_t mx_conv_workspace(const mx_conv_shape* s, int pass) {
  if (!s || pass < 0 || pass > 2) return 0;
  if (pass == 2) return wgrad_ws(s);
  if (pass == 0) {
    Geo g = make_geo(s->N * s->Ho * s->Wo, s->K, s->R * s->S * s->C);
    return g.splits > 1 ? sizeof(float) * (size_t)g.splits * g.M * g.Ncol : 0;
  }
  if (s->stride_h < 1 || s->stride_h > 2 || s->stride_w < 1 || s->stride_w > 2) return 0;
  DClass cl[4];
  int64_t off[4];
  int br[4], bs[4];
  const int n = dgrad_classes(s, s->C, s->K, cl, off, br, bs);
  size_t mx = 0;
  for (int i = 0; i < n; ++i) {
    Geo g = make_geo(s->N * cl[i].Hc * cl[i].Wc, s->C, (int64_t)cl[i].Rc * cl[i].Sc * s->K);
    if (g.splits > 1) mx = std::max(mx, sizeof(float) * (size_t)g.splits * g.M * g.Ncol);
  }
  return mx;
}

template <int BN, int MODE, int BKT, int STAGES, int OCC, int BMT = BM>
static void launch_pipe(const ConvP& p, int64_t blocks, hipStream_t st) {
  size_t ring = (size_t)STAGES * (BMT + BN) * BKT * 2;
  size_t epi = (size_t)(BMT / 2) * (BN + 4) * 4;
  conv_igemm_pipe_kernel<BN, MODE, BKT, STAGES, OCC, BMT><<<(unsigned)blocks, NT, std::max(ring, epi), st>>>(p);
}

template <int BN, int MODE, int STAGES, int OCC, int BMT>
static void launch_buf(const ConvP& p, int64_t blocks, hipStream_t st) {
  size_t ring = (size_t)STAGES * (BMT + BN) * 32 * 2;
  size_t epi = (size_t)(BMT / 2) * (BN + 4) * 4;
  conv_igemm_buf_kernel<BN, MODE, STAGES, OCC, BMT><<<(unsigned)blocks, NT, std::max(ring, epi), st>>>(p);
}

// A/B loader: 1 (default) buffer descriptors with wave-uniform tap offsets where the shape allows
// (conv_igemm_buf_kernel), 0 the per-lane 64-bit global_load_lds kernels only
static int g_conv_loader = 1;
extern "C" int mx_conv_set_loader(int v) {
  // 2 / 3: timing-only diagnostics (wrong results): the A / B descriptor gets zero records, so the
  // range check drops that operand's loads (prices its memory traffic)
  MX_CHECK_ARG(v >= 0 && v <= 3, "mx_conv_set_loader: 0 global_load_lds, 1 buffer descriptors, 2/3 timing-only");
  g_conv_loader = v;
  return MX_OK;
}

template <int BN, int MODE>
static void launch_variant(int v, const ConvP& p, int64_t blocks, hipStream_t st) {
  switch (v) {
    case 0: {
      size_t lds = std::max<size_t>(2 * (BM + BN) * BK * 2, (size_t)BM * (BN + 4) * 4);
      conv_igemm_kernel<BN, MODE><<<(unsigned)blocks, NT, lds, st>>>(p);
      break;
    }
    case 1: case 2: {
      size_t lds = std::max<size_t>(2 * (BM + BN) * BK * 2, (size_t)BM * (BN + 4) * 4);
      conv_igemm_glds_kernel<BN, MODE><<<(unsigned)blocks, NT, lds, st>>>(p);
      break;
    }
    case 3: launch_pipe<BN, MODE, 32, 3, 3>(p, blocks, st); break;
    case 4: launch_pipe<BN, MODE, 64, 2, 2>(p, blocks, st); break;
    case 5: launch_pipe<BN, MODE, 32, 4, 2>(p, blocks, st); break;
    case 8: launch_pipe<BN, MODE, 32, 3, 3, 64>(p, blocks, st); break;
    default: launch_pipe<BN, MODE, 64, 3, 1>(p, blocks, st); break;
  }
}

template <int MODE>
static int launch_igemm(ConvP& p, const Geo& g, void* ws, size_t ws_bytes, hipStream_t st) {
  int64_t blocks = g.tiles;
  MX_CHECK_ARG(g.Kdim < (1ll << 30) && p.IH < (1ll << 26) && p.IW < (1ll << 26), "conv: GEMM K or spatial size too large");
  MX_CHECK_ARG(blocks * g.splits < (1ll << 31), "conv: grid too large");
  const bool buf = g_conv_loader >= 1 && p.IC % 32 == 0 && p.R * p.S <= 64 && p.Kdim % 32 == 0 && p.src_elems > 0 &&
                   p.src_elems * 2 < (1ll << 31) && p.wt_elems > 0 && p.wt_elems * 2 < (1ll << 31);
  MX_CHECK_ARG(buf || g.bn != 256 || g.bmt == BM, "conv: 64x256 tiles need the buffer loader");
  const int v = buf ? 3 : launch_kind(g);
  const int64_t bkt = (buf || v == 3 || v == 5 || v == 8 || v == 9) ? 32 : 64;
  const int64_t nk = cdiv(g.Kdim, bkt);  // K-tiles in the kernel's tile width
  p.splits = 1;
  p.kt_per_split = nk;
  p.slab = nullptr;
  if (g.splits > 1) {
    size_t need = sizeof(float) * (size_t)g.splits * g.M * g.Ncol;
    MX_CHECK_ARG(ws && ws_bytes >= need, "conv: split-K workspace of %zu bytes required (mx_conv_workspace)", need);
    p.kt_per_split = cdiv(nk, (int64_t)g.splits);
    p.splits = (int)cdiv(nk, p.kt_per_split);
    p.slab = (float*)ws;
    blocks *= p.splits;
  }
  if (buf) {
    p.korder = g_conv_korder;
    if (g_conv_loader == 2) p.src_elems = 0;
    if (g_conv_loader == 3) p.wt_elems = 0;
    if (g.bmt == 64) {
      if (g.bn == 256) launch_buf<256, MODE, 3, 2, 64>(p, blocks, st);
      else if (g.narrow) launch_buf<64, MODE, 3, 4, 64>(p, blocks, st);
      else if (g_buf_stages == 4) launch_buf<128, MODE, 4, 3, 64>(p, blocks, st);
      else if (g_buf_stages == 6) launch_buf<128, MODE, 6, 2, 64>(p, blocks, st);
      else launch_buf<128, MODE, 3, 4, 64>(p, blocks, st);
    } else if (g.bn == 256) launch_buf<256, MODE, 3, 2, 128>(p, blocks, st);
    else if (g.narrow) launch_buf<64, MODE, 3, 3, 128>(p, blocks, st);
    else if (g_buf_stages == 4) launch_buf<128, MODE, 4, 2, 128>(p, blocks, st);
    else if (g_buf_stages == 6) launch_buf<128, MODE, 6, 1, 128>(p, blocks, st);
    else launch_buf<128, MODE, 3, 3, 128>(p, blocks, st);
  } else if (g.bn == 256) launch_pipe<256, MODE, 32, 3, 2>(p, blocks, st);
  else if (g.narrow) launch_variant<64, MODE>(v, p, blocks, st);
  else launch_variant<128, MODE>(v, p, blocks, st);
  MX_LAUNCH_CHECK();
  if (p.slab) {
    // the reduce works in 128-row blocks; 16-column blocks when 64-column ones would not fill the chip
    if (cdiv(g.M, BM) * cdiv(g.Ncol, 64) >= 2 * (int64_t)num_cus()) {
      dim3 rg((unsigned)cdiv(g.M, BM), (unsigned)cdiv(g.Ncol, 64));
      conv_splitk_reduce_kernel<8><<<rg, 256, 0, st>>>(p);
    } else {
      dim3 rg((unsigned)cdiv(g.M, BM), (unsigned)cdiv(g.Ncol, 16));
      conv_splitk_reduce_kernel<2><<<rg, 256, 0, st>>>(p);
    }
    MX_LAUNCH_CHECK();
  }
  return MX_OK;
}

extern "C" int mx_conv_get_variant(void) { return g_conv_variant; }

// wgrad kernel variant: 0 register-staged 32-pixel K-tiles, 1 64-pixel K-tiles, 2 direct-to-LDS,
// 3 (default) buffer descriptors (conv_wgrad_buf_kernel; maps under 32 output pixels take 0)
static int g_wgrad_variant = 3;
extern "C" int mx_conv_set_wgrad_variant(int v) {
  MX_CHECK_ARG(v >= 0 && v <= 7, "mx_conv_set_wgrad_variant: 0 px32, 1 px64, 2 direct-to-LDS, 3 buffer descriptors, "
                                "4 = 3 for bf16 / the 128 x 256 wide block for bf16x3, 5 the 256 x 256 bf16x3 block, "
                                "6 = 3 for bf16 / the interleaved-schedule bf16x3 kernel, 7 = 3 for bf16 / the bf16x3 "
                                "kernel on pre-split operand planes (LDS-DMA)");
  g_wgrad_variant = v;
  return MX_OK;
}
extern "C" int mx_conv_get_wgrad_variant(void) { return g_wgrad_variant; }

extern "C" int mx_conv_set_variant(int v) {
  MX_CHECK_ARG(v >= 0 && v <= 9,
               "mx_conv_set_variant: 0 register staging, 1/2 direct-to-LDS fwd/dgrad, 3-6 multi-stage "
               "direct-to-LDS (3: BK32x3, 4: BK64x2, 5: BK32x4, 6: BK64x3), 7 auto, 8 64-row tiles BK32x3, "
               "9 as 7 with 128x256 tiles wherever Ncol >= 256");
  g_conv_variant = v;
  return MX_OK;
}

extern "C" int mx_conv2d_fwd_ex(const mx_conv_shape* s, const uint16_t* x, const uint16_t* w, const float* bias,
                                const uint16_t* residual, int act, void* y, int ydtype, float* stats, void* ws,
                                size_t ws_bytes, mx_stream_t stream) {
  int rc = conv_check(s);
  if (rc) return rc;
  MX_CHECK_ARG(s->C % 8 == 0, "conv fwd: C=%lld must be a multiple of 8 (pad the input channels)", (long long)s->C);
  MX_CHECK_ARG(ydtype == MX_BF16 || ydtype == MX_F32, "conv fwd: bad output dtype");
  MX_CHECK_ARG(!residual || s->K % 8 == 0, "conv fwd: residual needs K %% 8 == 0");
  ConvP p{};
  p.src = x; p.wt = w;
  p.M = s->N * s->Ho * s->Wo; p.Ncol = s->K; p.Kdim = s->R * s->S * s->C;
  p.OH = s->Ho; p.OW = s->Wo; p.IH = s->H; p.IW = s->W; p.IC = s->C;
  p.R = (int)s->R; p.S = (int)s->S; p.st_h = s->stride_h; p.st_w = s->stride_w; p.pad_h = s->pad_h; p.pad_w = s->pad_w;
  p.bias = bias; p.residual = residual; p.act = act; p.out = y; p.out_f32 = ydtype == MX_F32;
  p.stats = stats; p.mblocks = cdiv(p.M, SROWS);
  p.src_elems = s->N * s->H * s->W * s->C; p.wt_elems = p.Ncol * p.Kdim;
  return launch_igemm<0>(p, make_geo(p.M, p.Ncol, p.Kdim), ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int mx_conv2d_fwd(const mx_conv_shape* s, const uint16_t* x, const uint16_t* w, const float* bias, void* y,
                             int ydtype, float* stats, mx_stream_t stream) {
  size_t ws = mx_conv_workspace(s, 0);
  void* buf = nullptr;
  if (ws) MX_HIP(hipMallocAsync(&buf, ws, (hipStream_t)stream));
  int rc = mx_conv2d_fwd_ex(s, x, w, bias, nullptr, 0, y, ydtype, stats, buf, ws, stream);
  if (buf) MX_HIP(hipFreeAsync(buf, (hipStream_t)stream));
  return rc;
}

extern "C" int mx_conv_transpose_weight(const uint16_t* w, int64_t K, int64_t RS, int64_t C, uint16_t* wt, mx_stream_t stream) {
  int64_t n = K * RS * C;
  if (n == 0) return MX_OK;
  transpose_w_kernel<<<(unsigned)cdiv(n, 256), 256, 0, (hipStream_t)stream>>>(w, K, RS, C, wt);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" size_t mx_conv_dgrad_weight_elems(const mx_conv_shape* s, int64_t Cpad, int64_t Kpad) {
  if (!s) return 0;
  return (size_t)(Cpad ? Cpad : s->C) * s->R * s->S * (Kpad ? Kpad : s->K);
}

extern "C" int mx_conv_pack_weight(const mx_conv_shape* s, const float* w, int64_t Cin, int64_t Kout, uint16_t* wk,
                                   uint16_t* wt, int split, mx_stream_t stream) {
  // s->C / s->K are the padded channel counts the kernels see (Cin <= s->C real input channels,
  // Kout <= s->K real output channels of the f32 parameter w[Kout][Cin][R][S])
  MX_CHECK_ARG(s && w && s->R > 0 && s->S > 0 && Cin > 0 && Kout > 0 && Cin <= s->C && Kout <= s->K,
               "conv pack: bad shape");
  MX_CHECK_ARG(!wt || (s->stride_h >= 1 && s->stride_h <= 2 && s->stride_w >= 1 && s->stride_w <= 2),
               "conv pack: dgrad layout supports strides 1 and 2");
  if (!wk && !wt) return MX_OK;
  PackP p{};
  p.w = w; p.wk = wk; p.wt = wt;
  p.K = Kout; p.C = Cin; p.Cpad = s->C; p.Kpad = s->K;
  p.R = (int)s->R; p.S = (int)s->S; p.st_h = s->stride_h; p.st_w = s->stride_w;
  if (wt) {
    DClass cl[4];
    dgrad_classes(s, s->C, s->K, cl, p.off, p.Rc, p.Sc);
  } else {
    p.st_h = p.st_w = 1;
  }
  // wk covers Kout rows only; wt also covers the zero-padded output channels up to s->K
  MX_CHECK_ARG(pack_plan(p) == MX_OK, "conv pack: at most 196 taps");
  p.split = split ? 1 : 0;
  const int64_t tiles = p.nwk + p.nwt;
  MX_CHECK_ARG(tiles < (1ll << 31), "conv pack: too many tiles");
  pack_weight_kernel<<<(unsigned)tiles, 256, 0, (hipStream_t)stream>>>(p);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

static int make_pack(const mx_pack_desc& d, PackP& p, int64_t& tiles) {
  MX_CHECK_ARG(d.w && d.R > 0 && d.S > 0 && d.Cin > 0 && d.Kout > 0 && d.Cin <= d.Cpad && d.Kout <= d.Kpad,
               "conv pack: bad job");
  MX_CHECK_ARG(!d.wt || (d.stride_h >= 1 && d.stride_h <= 2 && d.stride_w >= 1 && d.stride_w <= 2),
               "conv pack: dgrad layout supports strides 1 and 2");
  p = PackP{};
  p.w = d.w; p.wk = d.wk; p.wt = d.wt;
  p.K = d.Kout; p.C = d.Cin; p.Cpad = d.Cpad; p.Kpad = d.Kpad;
  p.R = d.R; p.S = d.S; p.st_h = d.stride_h; p.st_w = d.stride_w;
  p.dense = d.flags & 1;
  p.split = (d.flags >> 1) & 1;
  if (d.wt && !p.dense) {
    mx_conv_shape s{};
    s.C = d.Cpad; s.K = d.Kpad; s.R = d.R; s.S = d.S; s.H = 1; s.W = 1;
    s.stride_h = d.stride_h; s.stride_w = d.stride_w; s.pad_h = d.pad_h; s.pad_w = d.pad_w;
    DClass cl[4];
    dgrad_classes(&s, d.Cpad, d.Kpad, cl, p.off, p.Rc, p.Sc);
  } else {
    p.st_h = p.st_w = 1;
  }
  MX_CHECK_ARG(pack_plan(p) == MX_OK, "conv pack: at most 196 taps");
  tiles = p.nwk + p.nwt;
  return MX_OK;
}

extern "C" size_t mx_conv_pack_plan_bytes(int64_t njobs) {
  return njobs > 0 ? sizeof(PackP) * (size_t)njobs + sizeof(int64_t) * (size_t)(njobs + 1) : 0;
}

extern "C" int mx_conv_pack_batched(const mx_pack_desc* jobs, int64_t njobs, void* plan, size_t plan_bytes, int upload,
                                    mx_stream_t stream) {
  MX_CHECK_ARG(jobs && njobs > 0 && njobs < (1 << 20), "conv pack batched: bad job list");
  MX_CHECK_ARG(plan && plan_bytes >= mx_conv_pack_plan_bytes(njobs), "conv pack batched: plan buffer too small");
  std::vector<PackP> host((size_t)njobs);
  std::vector<int64_t> prefix((size_t)njobs + 1, 0);
  for (int64_t j = 0; j < njobs; ++j) {
    int64_t t = 0;
    int rc = make_pack(jobs[j], host[(size_t)j], t);
    if (rc) return rc;
    if (!jobs[j].wk && !jobs[j].wt) t = 0;
    prefix[(size_t)j + 1] = prefix[(size_t)j] + t;
  }
  const int64_t total = prefix[(size_t)njobs];
  MX_CHECK_ARG(total < (1ll << 31), "conv pack batched: too many tiles");
  hipStream_t st = (hipStream_t)stream;
  PackP* dj = (PackP*)plan;
  int64_t* dp = (int64_t*)((char*)plan + sizeof(PackP) * (size_t)njobs);
  if (upload) {
    // the host vectors die with this call: synchronous copies (the plan changes rarely)
    MX_HIP(hipStreamSynchronize(st));
    MX_HIP(hipMemcpy(dj, host.data(), sizeof(PackP) * (size_t)njobs, hipMemcpyHostToDevice));
    MX_HIP(hipMemcpy(dp, prefix.data(), sizeof(int64_t) * (size_t)(njobs + 1), hipMemcpyHostToDevice));
  }
  if (total == 0) return MX_OK;
  pack_batched_kernel<<<(unsigned)total, 256, 0, st>>>(dj, dp, (int)njobs);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

// fused tile for R*S taps (sgd_pack_tile): 64x64 (1x1), 32x32 (<= 9 taps), 16x8 (<= 49 taps; FC6).
// One launch reserves the largest tile's LDS for every block: FC6's 16x16 (50 KiB) held the whole
// launch to 3 blocks per CU; 16x8 (25 KiB) leaves the 3x3 tile (37 KiB) as the bound (4 per CU).
static bool sgd_tile(int RS, int& kr, int& tc) {
  if (RS == 1) { kr = 64; tc = 64; return true; }
  if (RS <= 9) { kr = 32; tc = 32; return true; }
  if (RS <= 49) { kr = 16; tc = 8; return true; }
  return false;
}

extern "C" size_t mx_sgd_pack_plan_bytes(int64_t nparams) {
  return nparams > 0 ? sizeof(SgdJob) * (size_t)nparams + sizeof(int64_t) * (size_t)(nparams + 1) : 0;
}

extern "C" int mx_sgd_pack_build(const mx_sgd_param* params, int64_t nparams, const mx_pack_desc* packs,
                                 void* host_plan, size_t plan_bytes, int64_t* blocks, size_t* lds_bytes) {
  MX_CHECK_ARG(params && nparams > 0 && nparams < (1 << 20) && blocks && lds_bytes, "sgd pack build: bad lists");
  MX_CHECK_ARG(host_plan && plan_bytes >= mx_sgd_pack_plan_bytes(nparams), "sgd pack build: plan buffer too small");
  SgdJob* jobs = (SgdJob*)host_plan;
  int64_t* prefix = (int64_t*)((char*)host_plan + sizeof(SgdJob) * (size_t)nparams);
  prefix[0] = 0;
  size_t lds = 0;
  for (int64_t j = 0; j < nparams; ++j) {
    const mx_sgd_param& q = params[j];
    MX_CHECK_ARG(q.p && q.buf && q.n > 0, "sgd pack build: parameter %lld empty or null", (long long)j);
    SgdJob J{};
    J.p = q.p; J.b = q.buf; J.n = q.n; J.first = q.first ? 1 : 0;
    int64_t nb = cdiv(q.n, SGDP_PER_BLOCK);
    if (q.pack >= 0) {
      MX_CHECK_ARG(packs, "sgd pack build: pack index without pack list");
      const mx_pack_desc& d = packs[q.pack];
      int64_t tiles = 0;
      int rc = make_pack(d, J.pk, tiles);
      if (rc) return rc;
      const int RS = d.R * d.S;
      MX_CHECK_ARG(d.w == q.p && d.Kout * d.Cin * RS == q.n, "sgd pack build: pack %lld is not parameter %lld",
                   (long long)q.pack, (long long)j);
      MX_CHECK_ARG(sgd_tile(RS, J.kr, J.tc), "sgd pack build: %d taps (fused packing takes <= 49)", RS);
      MX_CHECK_ARG(d.wk || d.wt, "sgd pack build: pack %lld has no layout", (long long)q.pack);
      J.fused = 1;
      J.ncb = cdiv(J.pk.Cpad, J.tc);
      nb = cdiv(J.pk.Kpad, J.kr) * J.ncb;
      const size_t need = sizeof(uint32_t) * (size_t)J.kr * (size_t)(J.tc * RS + 1);
      if (need > lds) lds = need;
    }
    jobs[j] = J;
    prefix[j + 1] = prefix[j] + nb;
  }
  MX_CHECK_ARG(prefix[nparams] < (1ll << 31), "sgd pack build: too many blocks");
  *blocks = prefix[nparams];
  *lds_bytes = lds;
  return MX_OK;
}

extern "C" int mx_sgd_pack_step(const void* plan, const float* const* grads, int64_t nparams, int64_t blocks,
                                size_t lds_bytes, float lr, float momentum, float dampening, float weight_decay,
                                int nesterov, mx_stream_t stream) {
  MX_CHECK_ARG(plan && grads && nparams > 0 && blocks > 0 && blocks < (1ll << 31) && lds_bytes <= 65536,
               "sgd pack step: bad plan");
  const SgdJob* jobs = (const SgdJob*)plan;
  const int64_t* prefix = (const int64_t*)((const char*)plan + sizeof(SgdJob) * (size_t)nparams);
  SgdHyper h{lr, momentum, dampening, weight_decay, nesterov};
  sgd_pack_kernel<<<(unsigned)blocks, 256, lds_bytes, (hipStream_t)stream>>>(jobs, prefix, grads, (int)nparams, h);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

// dgrad with the weight packed by mx_conv_pack_weight (for stride 1 that layout is the plain
// [C][R][S][K] transpose of mx_conv_transpose_weight)
extern "C" int mx_conv2d_dgrad_t(const mx_conv_shape* s, const uint16_t* dy, const uint16_t* wt, uint16_t* dx,
                                 void* ws, size_t ws_bytes, mx_stream_t stream) {
  return mx_conv2d_dgrad_ex(s, dy, wt, nullptr, dx, ws, ws_bytes, stream);
}

struct BnbArgs {
  const uint16_t *y, *z;
  const float *mean, *invstd;
  int act;
  float* part;
  int64_t mb;
};

static int dgrad_impl(const mx_conv_shape* s, const uint16_t* dy, const uint16_t* wt, const uint16_t* residual,
                      uint16_t* dx, const BnbArgs* bnb, void* ws, size_t ws_bytes, mx_stream_t stream);

extern "C" int mx_conv2d_dgrad_ex(const mx_conv_shape* s, const uint16_t* dy, const uint16_t* wt,
                                  const uint16_t* residual, uint16_t* dx, void* ws, size_t ws_bytes,
                                  mx_stream_t stream) {
  return dgrad_impl(s, dy, wt, residual, dx, nullptr, ws, ws_bytes, stream);
}

extern "C" int mx_conv2d_dgrad_bnb(const mx_conv_shape* s, const uint16_t* dy, const uint16_t* wt,
                                   const uint16_t* residual, uint16_t* dx, const uint16_t* y, const uint16_t* z,
                                   const float* mean, const float* invstd, int act, float* part, int64_t part_mb,
                                   void* ws, size_t ws_bytes, mx_stream_t stream) {
  MX_CHECK_ARG(s && s->stride_h == 1 && s->stride_w == 1, "conv dgrad bnb: stride 1 only");
  MX_CHECK_ARG(y && z && mean && invstd && part && act >= 0 && act <= 2, "conv dgrad bnb: bad BN arguments");
  MX_CHECK_ARG(part_mb == cdiv(s->N * s->H * s->W, 64), "conv dgrad bnb: part rows must be cdiv(N*H*W, 64)");
  BnbArgs b{y, z, mean, invstd, act, part, part_mb};
  return dgrad_impl(s, dy, wt, residual, dx, &b, ws, ws_bytes, stream);
}

static int dgrad_impl(const mx_conv_shape* s, const uint16_t* dy, const uint16_t* wt, const uint16_t* residual,
                      uint16_t* dx, const BnbArgs* bnb, void* ws, size_t ws_bytes, mx_stream_t stream) {
  // residual: a gradient accumulated in the epilogue; under stride 2 each parity class adds it at the
  // pixels it writes (classes without taps write it alone), so every pixel gets it exactly once
  int rc = conv_check(s);
  if (rc) return rc;
  MX_CHECK_ARG(s->K % 8 == 0, "conv dgrad: K=%lld must be a multiple of 8", (long long)s->K);
  MX_CHECK_ARG(s->C % 8 == 0, "conv dgrad: C=%lld must be a multiple of 8", (long long)s->C);
  MX_CHECK_ARG(s->stride_h <= 2 && s->stride_w <= 2, "conv dgrad: strides 1 and 2 are supported");
  DClass cl[4];
  int64_t off[4];
  int br[4], bs[4];
  const int n = dgrad_classes(s, s->C, s->K, cl, off, br, bs);
  const bool remap = s->stride_h > 1 || s->stride_w > 1;
  for (int i = 0; i < n; ++i) {
    const DClass& c = cl[i];
    if (c.Hc * c.Wc == 0) continue;
    ConvP p{};
    p.src = dy; p.wt = wt + c.off;
    p.M = s->N * c.Hc * c.Wc; p.Ncol = s->C; p.Kdim = (int64_t)c.Rc * c.Sc * s->K;
    p.OH = c.Hc; p.OW = c.Wc; p.IH = s->Ho; p.IW = s->Wo; p.IC = s->K;
    p.R = std::max(c.Rc, 1); p.S = std::max(c.Sc, 1); p.st_h = 1; p.st_w = 1; p.pad_h = c.dh; p.pad_w = c.dw;
    p.out = dx; p.out_f32 = 0; p.act = 0; p.residual = residual;
    if (bnb) {
      p.bnb_y = bnb->y; p.bnb_z = bnb->z; p.bnb_mean = bnb->mean; p.bnb_invstd = bnb->invstd;
      p.bnb_act = bnb->act; p.bnb_part = bnb->part; p.bnb_mb = bnb->mb;
    }
    p.remap = remap; p.rst_h = s->stride_h; p.rst_w = s->stride_w; p.rph = c.ph; p.rpw = c.pw;
    p.rH = s->H; p.rW = s->W;
    p.src_elems = s->N * s->Ho * s->Wo * s->K; p.wt_elems = p.Ncol * p.Kdim;
    rc = launch_igemm<1>(p, make_geo(p.M, p.Ncol, p.Kdim), ws, ws_bytes, (hipStream_t)stream);
    if (rc) return rc;
  }
  return MX_OK;
}

extern "C" int mx_conv2d_dgrad(const mx_conv_shape* s, const uint16_t* dy, const uint16_t* w, uint16_t* dx,
                               mx_stream_t stream) {
  // Convenience form taking the KRSC bf16 weight: repacks it into a stream-ordered temporary
  // (allocates per call; the hot path uses mx_conv_pack_weight + mx_conv2d_dgrad_t).
  int rc = conv_check(s);
  if (rc) return rc;
  MX_CHECK_ARG(s->stride_h <= 2 && s->stride_w <= 2, "conv dgrad: strides 1 and 2 are supported");
  hipStream_t st = (hipStream_t)stream;
  const int64_t RS = s->R * s->S;
  uint16_t* wt = nullptr;
  size_t bytes = sizeof(uint16_t) * s->K * RS * s->C;
  size_t wsb = mx_conv_workspace(s, 1);
  void* ws = nullptr;
  MX_HIP(hipMallocAsync((void**)&wt, bytes, st));
  if (wsb) MX_HIP(hipMallocAsync(&ws, wsb, st));
  {
    DClass cl[4];
    PackP p{};
    dgrad_classes(s, s->C, s->K, cl, p.off, p.Rc, p.Sc);
    p.K = s->K; p.C = s->C; p.Cpad = s->C; p.Kpad = s->K;
    p.R = (int)s->R; p.S = (int)s->S; p.st_h = s->stride_h; p.st_w = s->stride_w;
    p.wt = wt;
    const int64_t n = s->K * RS * s->C;
    krsc_to_dgrad_kernel<<<(unsigned)cdiv(n, 256), 256, 0, st>>>(w, p);
    if (hipGetLastError() != hipSuccess) rc = MX_EHIP;
  }
  if (!rc) rc = mx_conv2d_dgrad_t(s, dy, wt, dx, ws, wsb, stream);
  MX_HIP(hipFreeAsync(wt, st));
  if (ws) MX_HIP(hipFreeAsync(ws, st));
  return rc;
}

// wgrad launch geometry: 128x128 (k, col) tiles; the pixel axis is split until the grid covers
// ~g_wgrad_target blocks (each split's partial goes to a slab, summed by wgrad_reduce_kernel).
static int64_t g_wgrad_target = 0;  // 0: one full wave of resident blocks (occupancy x CUs)
struct WGeo {
  int64_t tiles, splits, kchunk;
  int pxt;
};
static int g_num_cus = 0;
static int num_cus() {
  if (!g_num_cus) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      g_num_cus = n;
    else
      g_num_cus = 256;
  }
  return g_num_cus;
}
static WGeo wgrad_geo(const mx_conv_shape* s) {
  WGeo g;
  const int64_t P = s->N * s->Ho * s->Wo, Ncol = s->R * s->S * s->C;
  g.tiles = cdiv(s->K, 128) * cdiv(Ncol, 128);
  const int v = g_wgrad_variant >= 4 ? 3 : g_wgrad_variant;
  g.pxt = v == 2 ? BKG : (v == 1 ? 64 : BKW);
  // resident blocks per CU: px32 / buffer 3 (142 VGPRs), px64 / direct-to-LDS 2
  const int64_t slots = g_wgrad_target ? g_wgrad_target : (int64_t)num_cus() * ((v == 0 || v == 3) ? 3 : 2);
  int64_t splits = std::max<int64_t>(1, slots / g.tiles);  // never past one wave of blocks
  const int64_t max_splits = std::max<int64_t>(1, P / (g.pxt * 4));
  splits = std::min(splits, max_splits);
  g.kchunk = cdiv(cdiv(P, splits), g.pxt) * g.pxt;
  g.splits = cdiv(P, g.kchunk);
  return g;
}

extern "C" int mx_conv_set_wgrad_target(int64_t blocks) {
  MX_CHECK_ARG(blocks >= 0 && blocks <= (1 << 20), "mx_conv_set_wgrad_target: bad block count (0 = auto)");
  g_wgrad_target = blocks;
  return MX_OK;
}

// A dense conv (valid RxS on an RxS map: one output pixel per image, FC6 as a 7x7 conv) has the
// same weight gradient as a 1x1 conv over R*S*C channels (NHWC order = (r, s, c) column order):
// that form gives the pixel-tiled wgrad kernel one image per pixel row instead of wrapping 7x7 maps.
static mx_conv_shape wgrad_shape(const mx_conv_shape* s, bool* dense) {
  mx_conv_shape d = *s;
  *dense = s->Ho == 1 && s->Wo == 1 && s->H == s->R && s->W == s->S && s->pad_h == 0 && s->pad_w == 0 &&
           s->R * s->S > 1;
  if (*dense) {
    d.C = s->R * s->S * s->C;
    d.H = d.W = d.R = d.S = 1;
    d.stride_h = d.stride_w = 1;
  }
  return d;
}

static size_t wgrad_ws(const mx_conv_shape* s0) {
  bool dense;
  const mx_conv_shape sd = wgrad_shape(s0, &dense);
  const mx_conv_shape* s = &sd;
  WGeo g = wgrad_geo(s);
  return g.splits > 1 ? sizeof(float) * (size_t)g.splits * s->K * s->R * s->S * s->C : 0;
}

extern "C" int mx_conv2d_wgrad_ex(const mx_conv_shape* s, const uint16_t* dy, const uint16_t* x, float* dw,
                                  int64_t Kout, int64_t Cin, int layout, void* ws, size_t ws_bytes,
                                  mx_stream_t stream) {
  int rc = conv_check(s);
  if (rc) return rc;
  MX_CHECK_ARG(s->K % 8 == 0 && s->C % 8 == 0, "conv wgrad: K and C must be multiples of 8");
  MX_CHECK_ARG(Kout >= 1 && Kout <= s->K && Cin >= 1 && Cin <= s->C, "conv wgrad: Kout/Cin out of range");
  MX_CHECK_ARG(layout == 0 || layout == 1, "conv wgrad: layout 0 (KRSC) or 1 (KCRS)");
  MX_CHECK_ARG(s->K * s->R * s->S * s->C < (1ll << 31), "conv wgrad: weight too large");
  hipStream_t st = (hipStream_t)stream;
  const int dC = (int)s->C, dRS = (int)(s->R * s->S);
  bool dense;
  const mx_conv_shape sd = wgrad_shape(s, &dense);
  s = &sd;
  WgP p{};
  p.dy = dy; p.x = x; p.dw = dw;
  p.P = s->N * s->Ho * s->Wo; p.K = s->K; p.Ncol = s->R * s->S * s->C;
  p.OH = s->Ho; p.OW = s->Wo; p.H = s->H; p.W = s->W; p.C = s->C; p.N = s->N;
  p.R = (int)s->R; p.S = (int)s->S; p.st_h = s->stride_h; p.st_w = s->stride_w; p.pad_h = s->pad_h; p.pad_w = s->pad_w;
  p.Kout = Kout; p.Cin = Cin; p.layout = layout;
  p.dC = dC; p.dRS = dRS;
  WGeo g = wgrad_geo(s);
  p.kchunk = g.kchunk;
  if (g.splits > 1) {
    const size_t need = sizeof(float) * (size_t)g.splits * p.K * p.Ncol;
    MX_CHECK_ARG(ws && ws_bytes >= need, "conv wgrad: split workspace of %zu bytes required (mx_conv_workspace pass 2)",
                 need);
    p.slab = (float*)ws;
  }
  MX_CHECK_ARG(g.tiles < (1ll << 31) && g.splits < 65536, "conv wgrad: grid too large");
  dim3 grid((unsigned)g.tiles, (unsigned)g.splits);
  int v = g_wgrad_variant >= 4 ? 3 : g_wgrad_variant;
  // the buffer kernel walks each lane's pixels by (n, oh, ow) increments: maps of fewer than 32
  // output pixels (FC6 as a 7x7 conv on the RoI tile) would wrap many times per tile -> register kernel
  if (v == 3 && !(p.P * p.K * 2 < (1ll << 31) && s->N * s->H * s->W * s->C * 2 < (1ll << 31) &&
                 (p.OH * p.OW >= 32 || (p.OH == 1 && p.OW == 1))))
    v = 0;
  if (v == 3) conv_wgrad_buf_kernel<<<(unsigned)(g.tiles * g.splits), NT, 3 * 2 * 32 * 256, st>>>(p);
  else if (v == 2) conv_wgrad_glds_kernel<<<grid, NT, 2 * 2 * BKG * 256, st>>>(p);
  else if (v == 1) conv_wgrad_kernel<64><<<grid, NT, 0, st>>>(p);
  else conv_wgrad_kernel<32><<<grid, NT, 0, st>>>(p);
  MX_LAUNCH_CHECK();
  if (g.splits > 1) {
    MX_CHECK_ARG(Kout < 65536, "conv wgrad: too many output channels for the split reduce");
    wgrad_reduce_kernel<<<dim3((unsigned)cdiv(p.Ncol / 4, 64), (unsigned)Kout), 256, 0, st>>>(p, (int)g.splits);
    MX_LAUNCH_CHECK();
  }
  return MX_OK;
}

extern "C" int mx_conv2d_wgrad(const mx_conv_shape* s, const uint16_t* dy, const uint16_t* x, float* dw, mx_stream_t stream) {
  // convenience form: dw [K][R][S][C] f32 (overwritten), temporaries allocated per call
  int rc = conv_check(s);
  if (rc) return rc;
  size_t wsb = wgrad_ws(s);
  void* ws = nullptr;
  if (wsb) MX_HIP(hipMallocAsync(&ws, wsb, (hipStream_t)stream));
  rc = mx_conv2d_wgrad_ex(s, dy, x, dw, s->K, s->C, 0, ws, wsb, stream);
  if (ws) MX_HIP(hipFreeAsync(ws, (hipStream_t)stream));
  return rc;
}

// ================================================================================================
// bf16x3 (f32 activation) entry points: same GEMM decompositions as the bf16 path (fwd, dgrad per
// stride-parity class, wgrad split over pixels), f32 activations / gradients, split weights.
static Geo make_geo_x3(int64_t M, int64_t Ncol, int64_t Kdim) {
  Geo g;
  g.M = M; g.Ncol = Ncol; g.Kdim = Kdim;
  g.narrow = Ncol <= 64;
  g.bn = g.narrow ? 64 : 128;
  const int64_t cus = num_cus();
  // 2 blocks per CU: below two full rounds of 128-row tiles, 64-row tiles (twice the blocks)
  // 128 x 128 at 2 blocks per CU; below two full rounds, 64-row tiles. (256 x 128 tiles -- 8 waves,
  // one block per CU, 25 % fewer LDS-DMA pieces per MFMA -- measured 15 % slower on the P2 3x3; a
  // tuner candidate only. 256 x 256 with 8 waves of 64 x 128 -- 8 pieces per 96 MFMAs -- measured
  // no faster than 128 x 128 on the P2 3x3 (615 vs 592 us fwd) and slower everywhere else: removed.)
  g.bmt = 128;
  g.tiles = cdiv(M, 128) * cdiv(Ncol, g.bn);
  if (g.tiles < 2 * cus) {
    g.bmt = 64;
    g.tiles = cdiv(M, 64) * cdiv(Ncol, g.bn);
  }
  if (g_force_bmt) {
    g.bmt = g_force_bmt;
    g.bn = g.bmt == 256 ? 128 : std::min(g_force_bn, 128);
    g.narrow = g.bn == 64;
    g.tiles = cdiv(M, g.bmt) * cdiv(Ncol, g.bn);
  }
  g.nk = cdiv(Kdim, 32);
  g.splits = 1;
  if (Ncol % 8 == 0 && g.tiles < 320 && g.nk >= 8) {
    int64_t sp = std::min<int64_t>(std::min<int64_t>(cdiv(640, g.tiles), g.nk / 4), 16);
    g.splits = (int)std::max<int64_t>(1, sp);
  }
  if (g_max_splits && g.splits > g_max_splits) g.splits = g_max_splits;
  return g;
}

template <int BN, int MODE, int BMT>
static void launch_x3(const ConvP& p, int64_t blocks, hipStream_t st) {
  const size_t ring = (size_t)2 * 2 * (BMT + BN) * 64;
  const size_t epi = (size_t)(BMT / 2) * (BN + 4) * 4;
  conv_x3_kernel<BN, MODE, BMT><<<(unsigned)blocks, NT, std::max(ring, epi), st>>>(p);
}

template <int BN, int MODE, int STAGES, int OCC, int BMT, int WR = 2, int WC = 2>
static void launch_x3_buf(const ConvP& p, int64_t blocks, hipStream_t st) {
  const size_t ring = (size_t)STAGES * 2 * (BMT + BN) * 64;
  const size_t epi = (size_t)(WC == 1 ? BMT : BMT / WR) * (BN + 4) * 4;
  if (p.aplanes)
    conv_x3_buf_kernel<BN, MODE, STAGES, OCC, BMT, WR, WC, true>
        <<<(unsigned)blocks, 64 * WR * WC, std::max(ring, epi), st>>>(p);
  else
    conv_x3_buf_kernel<BN, MODE, STAGES, OCC, BMT, WR, WC, false>
        <<<(unsigned)blocks, 64 * WR * WC, std::max(ring, epi), st>>>(p);
}

template <int MODE>
static int launch_igemm_x3(ConvP& p, const Geo& g0, void* ws, size_t ws_bytes, hipStream_t st) {
  const bool buf = g_conv_loader >= 1 && p.IC % 32 == 0 && p.R * p.S <= 64 && p.Kdim % 32 == 0 && p.src_elems > 0 &&
                   p.src_elems * 4 < (1ll << 31) && p.wt_elems > 0 && p.wt_plane + p.wt_elems < (1ll << 30);
  // (a tap-less stride-parity class of a strided dgrad, Kdim = 0, reads no A: the plain kernel writes its epilogue)
  MX_CHECK_ARG(buf || !p.aplanes || p.Kdim == 0,
               "conv x3p: pre-split A planes need the buffer kernel (channels %% 32 == 0, R*S <= 64)");
  Geo g = g0;
  if (g.bmt == 256 && !buf) {  // 256-row tiles exist only as the buffer kernel
    g.bmt = 128;
    g.tiles = cdiv(g.M, 128) * cdiv(g.Ncol, g.bn);
  }
  int64_t blocks = g.tiles;
  MX_CHECK_ARG(g.Kdim < (1ll << 30) && p.IH < (1ll << 26) && p.IW < (1ll << 26) && p.IC < (1ll << 30),
               "conv: GEMM K or spatial size too large");
  MX_CHECK_ARG(p.IC % 8 == 0 && p.Kdim % 8 == 0, "conv x3: channel counts must be multiples of 8");
  const int64_t nk = cdiv(g.Kdim, 32);
  p.splits = 1;
  p.kt_per_split = nk;
  p.slab = nullptr;
  if (g.splits > 1) {
    const size_t need = sizeof(float) * (size_t)g.splits * g.M * g.Ncol;
    MX_CHECK_ARG(ws && ws_bytes >= need, "conv: split-K workspace of %zu bytes required (mx_conv_workspace_x3)", need);
    p.kt_per_split = cdiv(nk, (int64_t)g.splits);
    p.splits = (int)cdiv(nk, p.kt_per_split);
    p.slab = (float*)ws;
    blocks *= p.splits;
  }
  MX_CHECK_ARG(blocks < (1ll << 31), "conv: grid too large");
  if (buf) {
    // ring depth x blocks per CU; mx_conv_set_stages(3) picks the alternative of each tile shape
    const bool alt = g_buf_stages == 3;
    // 128 x 128 / 64 x 128 tiles as 4 wide wave tiles (32 x 128 / 16 x 128: each A row split by one
    // wave) unless mx_conv_set_stages(4) asks for the 2 x 2 layout of 64 x 64 / 32 x 64 wave tiles
    const bool wide = g_buf_stages == 0, wide64 = wide;
    const bool altw = g_buf_stages == 5;  // the alternative ring depth with wide wave tiles
    p.korder = g_conv_korder;
    p.dbg_skip_epi = g_conv_debug;
    if (g_conv_loader == 2) p.src_elems = 0;  // timing-only diagnostics (mx_conv_set_loader)
    if (g_conv_loader == 3) p.wt_elems = 0;
    if (g.bmt == 256) {
      alt ? launch_x3_buf<128, MODE, 2, 1, 256, 4>(p, blocks, st) : launch_x3_buf<128, MODE, 3, 1, 256, 4>(p, blocks, st);
    } else if (g.bmt == 64) {
      if (g.bn == 64) {
        if (altw) launch_x3_buf<64, MODE, 3, 3, 64, 4, 1>(p, blocks, st);  // 4 wide wave tiles of 16 x 64
        else alt ? launch_x3_buf<64, MODE, 4, 2, 64>(p, blocks, st) : launch_x3_buf<64, MODE, 3, 3, 64>(p, blocks, st);
      } else if (altw) launch_x3_buf<128, MODE, 2, 3, 64, 4, 1>(p, blocks, st);
      else if (wide64) launch_x3_buf<128, MODE, 3, 2, 64, 4, 1>(p, blocks, st);
      else alt ? launch_x3_buf<128, MODE, 2, 3, 64>(p, blocks, st) : launch_x3_buf<128, MODE, 3, 2, 64>(p, blocks, st);
    } else {
      if (g.bn == 64) alt ? launch_x3_buf<64, MODE, 2, 3, 128>(p, blocks, st) : launch_x3_buf<64, MODE, 3, 2, 128>(p, blocks, st);
      else if (altw) launch_x3_buf<128, MODE, 3, 1, 128, 4, 1>(p, blocks, st);
      else if (wide) launch_x3_buf<128, MODE, 2, 2, 128, 4, 1>(p, blocks, st);
      else alt ? launch_x3_buf<128, MODE, 3, 1, 128>(p, blocks, st) : launch_x3_buf<128, MODE, 2, 2, 128>(p, blocks, st);
    }
  } else if (g.bmt == 64) {
    if (g.bn == 64) launch_x3<64, MODE, 64>(p, blocks, st);
    else launch_x3<128, MODE, 64>(p, blocks, st);
  } else {
    if (g.bn == 64) launch_x3<64, MODE, 128>(p, blocks, st);
    else launch_x3<128, MODE, 128>(p, blocks, st);
  }
  MX_LAUNCH_CHECK();
  if (p.slab) {
    if (cdiv(g.M, BM) * cdiv(g.Ncol, 64) >= 2 * (int64_t)num_cus()) {
      dim3 rg((unsigned)cdiv(g.M, BM), (unsigned)cdiv(g.Ncol, 64));
      conv_splitk_reduce_kernel<8, float><<<rg, 256, 0, st>>>(p);
    } else {
      dim3 rg((unsigned)cdiv(g.M, BM), (unsigned)cdiv(g.Ncol, 16));
      conv_splitk_reduce_kernel<2, float><<<rg, 256, 0, st>>>(p);
    }
    MX_LAUNCH_CHECK();
  }
  return MX_OK;
}

// wgrad x3 block shape: 0 = 128 x 128 (4 waves, 2 blocks per CU), 1 = 128 x 256 (8 waves, one block
// per CU; mx_conv_set_wgrad_variant(4) -- a tuner candidate)
static int wgrad_x3_wide() { return g_wgrad_variant == 4; }
// 5: 256 x 256 tile, one wave per SIMD (conv_wgrad_x3ww_kernel; a tuner candidate)
static int wgrad_x3_ww() { return g_wgrad_variant == 5; }
// std128: the 128 x 128 geometry whatever the variant (the pre-split x3p entry, one kernel)
static WGeo wgrad_geo_x3(const mx_conv_shape* s, bool std128 = false) {
  WGeo g;
  const int64_t P = s->N * s->Ho * s->Wo, Ncol = s->R * s->S * s->C;
  const bool wide = !std128 && wgrad_x3_wide(), ww = !std128 && wgrad_x3_ww();
  g.tiles = ww ? cdiv(s->K, 256) * cdiv(Ncol, 256) : cdiv(s->K, 128) * cdiv(Ncol, wide ? 256 : 128);
  g.pxt = 32;
  const int64_t slots = g_wgrad_target ? g_wgrad_target : (int64_t)num_cus() * ((wide || ww) ? 1 : 2);
  int64_t splits = std::max<int64_t>(1, slots / g.tiles);
  const int64_t max_splits = std::max<int64_t>(1, P / (g.pxt * 4));
  splits = std::min(splits, max_splits);
  g.kchunk = cdiv(cdiv(P, splits), g.pxt) * g.pxt;
  g.splits = cdiv(P, g.kchunk);
  return g;
}

// variant 7 (conv_wgrad_x3d_kernel): bf16 hi / lo planes of dy and x after the split slab
static int wgrad_x3_dma() { return g_wgrad_variant == 7; }
static size_t wgrad_x3_slab(const mx_conv_shape* sd, const WGeo& g) {
  return g.splits > 1 ? (sizeof(float) * (size_t)g.splits * sd->K * sd->R * sd->S * sd->C + 255) / 256 * 256 : 0;
}
static size_t wgrad_x3_planes(const mx_conv_shape* sd) {
  return 2 * sizeof(uint16_t) * (size_t)(sd->N * sd->Ho * sd->Wo * sd->K + sd->N * sd->H * sd->W * sd->C);
}

// pre-split (x3p) entry points: the wgrad needs only its split slab
extern "C" size_t mx_conv_workspace_x3p(const mx_conv_shape* s, int pass) {
  if (!s || pass < 0 || pass > 2) return 0;
  if (pass < 2) return mx_conv_workspace_x3(s, pass);
  bool dense;
  const mx_conv_shape sd = wgrad_shape(s, &dense);
  return wgrad_x3_slab(&sd, wgrad_geo_x3(&sd, true));
}

extern "C" size_t mx_conv_workspace_x3(const mx_conv_shape* s, int pass) {
  if (!s || pass < 0 || pass > 2) return 0;
  if (pass == 2) {
    bool dense;
    const mx_conv_shape sd = wgrad_shape(s, &dense);
    const WGeo g = wgrad_geo_x3(&sd);
    return wgrad_x3_slab(&sd, g) + (wgrad_x3_dma() ? wgrad_x3_planes(&sd) : 0);
  }
  if (pass == 0) {
    const Geo g = make_geo_x3(s->N * s->Ho * s->Wo, s->K, s->R * s->S * s->C);
    return g.splits > 1 ? sizeof(float) * (size_t)g.splits * g.M * g.Ncol : 0;
  }
  if (s->stride_h < 1 || s->stride_h > 2 || s->stride_w < 1 || s->stride_w > 2) return 0;
  DClass cl[4];
  int64_t off[4];
  int br[4], bs[4];
  const int n = dgrad_classes(s, s->C, s->K, cl, off, br, bs);
  size_t mx = 0;
  for (int i = 0; i < n; ++i) {
    const Geo g = make_geo_x3(s->N * cl[i].Hc * cl[i].Wc, s->C, (int64_t)cl[i].Rc * cl[i].Sc * s->K);
    if (g.splits > 1) mx = std::max(mx, sizeof(float) * (size_t)g.splits * g.M * g.Ncol);
  }
  return mx;
}

static int conv_fwd_x3(const mx_conv_shape* s, const void* x, int aplanes, const uint16_t* w, const float* bias,
                       const float* residual, int act, float* y, float* stats, void* ws, size_t ws_bytes,
                       mx_stream_t stream) {
  int rc = conv_check(s);
  if (rc) return rc;
  MX_CHECK_ARG(s->C % 8 == 0, "conv fwd x3: C=%lld must be a multiple of 8 (pad the input channels)", (long long)s->C);
  MX_CHECK_ARG(s->K % 8 == 0 || !residual, "conv fwd x3: residual needs K %% 8 == 0");
  MX_CHECK_ARG(x && w && y, "conv fwd x3: null operand");
  ConvP p{};
  p.src = (const uint16_t*)x; p.wt = w; p.aplanes = aplanes;
  p.M = s->N * s->Ho * s->Wo; p.Ncol = s->K; p.Kdim = s->R * s->S * s->C;
  p.OH = s->Ho; p.OW = s->Wo; p.IH = s->H; p.IW = s->W; p.IC = s->C;
  p.R = (int)s->R; p.S = (int)s->S; p.st_h = s->stride_h; p.st_w = s->stride_w; p.pad_h = s->pad_h; p.pad_w = s->pad_w;
  p.bias = bias; p.residual = residual; p.act = act; p.out = y; p.out_f32 = 1;
  p.stats = stats; p.mblocks = cdiv(p.M, SROWS);
  p.src_elems = s->N * s->H * s->W * s->C; p.wt_elems = p.Ncol * p.Kdim; p.wt_plane = p.Ncol * p.Kdim;
  return launch_igemm_x3<0>(p, make_geo_x3(p.M, p.Ncol, p.Kdim), ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int mx_conv2d_fwd_x3(const mx_conv_shape* s, const float* x, const uint16_t* w, const float* bias,
                                const float* residual, int act, float* y, float* stats, void* ws, size_t ws_bytes,
                                mx_stream_t stream) {
  return conv_fwd_x3(s, x, 0, w, bias, residual, act, y, stats, ws, ws_bytes, stream);
}

extern "C" int mx_conv2d_fwd_x3p(const mx_conv_shape* s, const uint16_t* xp, const uint16_t* w, const float* bias,
                                 const float* residual, int act, float* y, float* stats, void* ws, size_t ws_bytes,
                                 mx_stream_t stream) {
  return conv_fwd_x3(s, xp, 1, w, bias, residual, act, y, stats, ws, ws_bytes, stream);
}

static int conv_dgrad_x3(const mx_conv_shape* s, const void* dy, int aplanes, const uint16_t* wt,
                         const float* residual, float* dx, const float* y, const float* z, const float* mean,
                         const float* invstd, int act, float* part, int64_t part_mb, void* ws, size_t ws_bytes,
                         mx_stream_t stream) {
  int rc = conv_check(s);
  if (rc) return rc;
  MX_CHECK_ARG(s->K % 8 == 0 && s->C % 8 == 0, "conv dgrad x3: K and C must be multiples of 8");
  MX_CHECK_ARG(s->stride_h <= 2 && s->stride_w <= 2, "conv dgrad x3: strides 1 and 2 are supported");
  const bool bnb = part != nullptr;
  if (bnb) {
    MX_CHECK_ARG(s->stride_h == 1 && s->stride_w == 1, "conv dgrad x3 bnb: stride 1 only");
    MX_CHECK_ARG(y && z && mean && invstd && act >= 0 && act <= 2, "conv dgrad x3 bnb: bad BN arguments");
    MX_CHECK_ARG(part_mb == cdiv(s->N * s->H * s->W, 64), "conv dgrad x3 bnb: part rows must be cdiv(N*H*W, 64)");
  }
  DClass cl[4];
  int64_t off[4];
  int br[4], bs[4];
  const int n = dgrad_classes(s, s->C, s->K, cl, off, br, bs);
  const bool remap = s->stride_h > 1 || s->stride_w > 1;
  const int64_t plane = s->C * s->R * s->S * s->K;
  for (int i = 0; i < n; ++i) {
    const DClass& c = cl[i];
    if (c.Hc * c.Wc == 0) continue;
    ConvP p{};
    p.src = (const uint16_t*)dy; p.wt = wt + c.off; p.wt_plane = plane; p.aplanes = aplanes;
    p.M = s->N * c.Hc * c.Wc; p.Ncol = s->C; p.Kdim = (int64_t)c.Rc * c.Sc * s->K;
    p.OH = c.Hc; p.OW = c.Wc; p.IH = s->Ho; p.IW = s->Wo; p.IC = s->K;
    p.R = std::max(c.Rc, 1); p.S = std::max(c.Sc, 1); p.st_h = 1; p.st_w = 1; p.pad_h = c.dh; p.pad_w = c.dw;
    p.out = dx; p.out_f32 = 1; p.act = 0; p.residual = residual;
    if (bnb) {
      p.bnb_y = y; p.bnb_z = z; p.bnb_mean = mean; p.bnb_invstd = invstd; p.bnb_act = act; p.bnb_part = part;
      p.bnb_mb = part_mb;
    }
    p.remap = remap; p.rst_h = s->stride_h; p.rst_w = s->stride_w; p.rph = c.ph; p.rpw = c.pw;
    p.rH = s->H; p.rW = s->W;
    p.src_elems = s->N * s->Ho * s->Wo * s->K; p.wt_elems = p.Ncol * p.Kdim;
    rc = launch_igemm_x3<1>(p, make_geo_x3(p.M, p.Ncol, p.Kdim), ws, ws_bytes, (hipStream_t)stream);
    if (rc) return rc;
  }
  return MX_OK;
}

extern "C" int mx_conv2d_dgrad_x3(const mx_conv_shape* s, const float* dy, const uint16_t* wt, const float* residual,
                                  float* dx, const float* y, const float* z, const float* mean, const float* invstd,
                                  int act, float* part, int64_t part_mb, void* ws, size_t ws_bytes, mx_stream_t stream) {
  return conv_dgrad_x3(s, dy, 0, wt, residual, dx, y, z, mean, invstd, act, part, part_mb, ws, ws_bytes, stream);
}

extern "C" int mx_conv2d_dgrad_x3p(const mx_conv_shape* s, const uint16_t* dyp, const uint16_t* wt,
                                   const float* residual, float* dx, const float* y, const float* z, const float* mean,
                                   const float* invstd, int act, float* part, int64_t part_mb, void* ws,
                                   size_t ws_bytes, mx_stream_t stream) {
  return conv_dgrad_x3(s, dyp, 1, wt, residual, dx, y, z, mean, invstd, act, part, part_mb, ws, ws_bytes, stream);
}

extern "C" int mx_split_planes(const float* src, int64_t n, uint16_t* planes, mx_stream_t stream) {
  MX_CHECK_ARG(src && planes && n >= 0 && n % 8 == 0, "mx_split_planes: n must be a multiple of 8");
  if (n == 0) return MX_OK;
  split_planes_kernel<<<(unsigned)cdiv(n / 8, 256), 256, 0, (hipStream_t)stream>>>(src, n / 8, planes, planes + n);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

static int conv_wgrad_x3(const mx_conv_shape* s, const void* dy, const void* x, int planes, float* dw, int64_t Kout,
                         int64_t Cin, int layout, void* ws, size_t ws_bytes, mx_stream_t stream);
extern "C" int mx_conv2d_wgrad_x3(const mx_conv_shape* s, const float* dy, const float* x, float* dw, int64_t Kout,
                                  int64_t Cin, int layout, void* ws, size_t ws_bytes, mx_stream_t stream) {
  return conv_wgrad_x3(s, dy, x, 0, dw, Kout, Cin, layout, ws, ws_bytes, stream);
}
// dy / x already as bf16 hi / lo planes (mx_split_planes): the LDS-DMA kernel without its split passes;
// workspace = the split slab only (mx_conv_workspace_x3p)
extern "C" int mx_conv2d_wgrad_x3p(const mx_conv_shape* s, const uint16_t* dyp, const uint16_t* xp, float* dw,
                                   int64_t Kout, int64_t Cin, int layout, void* ws, size_t ws_bytes, mx_stream_t stream) {
  return conv_wgrad_x3(s, dyp, xp, 1, dw, Kout, Cin, layout, ws, ws_bytes, stream);
}
static int conv_wgrad_x3(const mx_conv_shape* s, const void* dy_, const void* x_, int planes, float* dw, int64_t Kout,
                         int64_t Cin, int layout, void* ws, size_t ws_bytes, mx_stream_t stream) {
  const float* dy = (const float*)dy_;
  const float* x = (const float*)x_;
  int rc = conv_check(s);
  if (rc) return rc;
  MX_CHECK_ARG(s->K % 8 == 0 && s->C % 8 == 0, "conv wgrad x3: K and C must be multiples of 8");
  MX_CHECK_ARG(Kout >= 1 && Kout <= s->K && Cin >= 1 && Cin <= s->C, "conv wgrad x3: Kout/Cin out of range");
  MX_CHECK_ARG(layout == 0 || layout == 1, "conv wgrad x3: layout 0 (KRSC) or 1 (KCRS)");
  MX_CHECK_ARG(s->K * s->R * s->S * s->C < (1ll << 31), "conv wgrad x3: weight too large");
  hipStream_t st = (hipStream_t)stream;
  const int dC = (int)s->C, dRS = (int)(s->R * s->S);
  bool dense;
  const mx_conv_shape sd = wgrad_shape(s, &dense);
  s = &sd;
  WgP p{};
  p.dy = (const uint16_t*)dy_; p.x = (const uint16_t*)x_; p.dw = dw;
  p.P = s->N * s->Ho * s->Wo; p.K = s->K; p.Ncol = s->R * s->S * s->C;
  p.OH = s->Ho; p.OW = s->Wo; p.H = s->H; p.W = s->W; p.C = s->C; p.N = s->N;
  p.R = (int)s->R; p.S = (int)s->S; p.st_h = s->stride_h; p.st_w = s->stride_w; p.pad_h = s->pad_h; p.pad_w = s->pad_w;
  p.Kout = Kout; p.Cin = Cin; p.layout = layout;
  p.dC = dC; p.dRS = dRS;
  const WGeo g = wgrad_geo_x3(s, planes != 0);
  p.kchunk = g.kchunk;
  const bool dma = planes || wgrad_x3_dma(), split = dma && !planes;
  const size_t slab = wgrad_x3_slab(s, g), need = slab + (split ? wgrad_x3_planes(s) : 0);
  if (need) {
    MX_CHECK_ARG(ws && ws_bytes >= need, "conv wgrad x3: workspace of %zu bytes required (mx_conv_workspace_x3)",
                 need);
  }
  if (g.splits > 1) p.slab = (float*)ws;
  if (split) {  // the operands as bf16 hi / lo planes, read by LDS-DMA
    const int64_t dyel = p.P * p.K, xel = p.N * p.H * p.W * p.C;
    uint16_t* dyp = (uint16_t*)((char*)ws + slab);
    uint16_t* xp = dyp + 2 * dyel;
    split_planes_kernel<<<(unsigned)cdiv(dyel / 8, 256), 256, 0, st>>>(dy, dyel / 8, dyp, dyp + dyel);
    MX_LAUNCH_CHECK();
    split_planes_kernel<<<(unsigned)cdiv(xel / 8, 256), 256, 0, st>>>(x, xel / 8, xp, xp + xel);
    MX_LAUNCH_CHECK();
    p.dy = dyp;
    p.x = xp;
  }
  MX_CHECK_ARG(g.tiles * g.splits < (1ll << 31), "conv wgrad x3: grid too large");
  MX_CHECK_ARG(p.P * p.K * 4 < (1ll << 31) && p.N * p.H * p.W * p.C * 4 < (1ll << 31) && p.P + 64 < (1ll << 23) &&
                   p.N * p.H * p.W < (1ll << 23) && p.K * 4 < (1ll << 24) && p.C * 4 < (1ll << 24),
               "conv wgrad x3: dy / x must each stay below 2 GiB and 8M pixels (32-bit / 24-bit offset math)");
  if (dma)
    conv_wgrad_x3d_kernel<<<(unsigned)(g.tiles * g.splits), NT, 2 * 4 * 32 * 256, st>>>(p);
  else if (wgrad_x3_ww())
    conv_wgrad_x3ww_kernel<<<(unsigned)(g.tiles * g.splits), 256, 2 * 8 * 32 * 256, st>>>(p);
  else if (wgrad_x3_wide())
    conv_wgrad_x3w_kernel<<<(unsigned)(g.tiles * g.splits), 512, 2 * 6 * 32 * 256, st>>>(p);
  else if (g_wgrad_variant == 6)
    conv_wgrad_x3_kernel<true><<<(unsigned)(g.tiles * g.splits), NT, 2 * 4 * 32 * 256, st>>>(p);
  else
    conv_wgrad_x3_kernel<false><<<(unsigned)(g.tiles * g.splits), NT, 2 * 4 * 32 * 256, st>>>(p);
  MX_LAUNCH_CHECK();
  if (g.splits > 1) {
    MX_CHECK_ARG(Kout < 65536, "conv wgrad x3: too many output channels for the split reduce");
    wgrad_reduce_kernel<<<dim3((unsigned)cdiv(p.Ncol / 4, 64), (unsigned)Kout), 256, 0, st>>>(p, (int)g.splits);
    MX_LAUNCH_CHECK();
  }
  return MX_OK;
}

extern "C" int mx_conv2d_stem_x3(const mx_conv_shape* s, const float* x, const uint16_t* w, const float* bias,
                                 int act, float* y, float* stats, mx_stream_t stream) {
  int rc = conv_check(s);
  if (rc) return rc;
  MX_CHECK_ARG(s->R == 7 && s->S == 7 && s->K == STEM_K, "conv stem x3: a 7x7 conv to 64 channels is required");
  MX_CHECK_ARG(s->C >= 4 && s->C % 4 == 0, "conv stem x3: input channel stride C=%lld must be a multiple of 4",
               (long long)s->C);
  MX_CHECK_ARG(act == 0 || act == 1, "conv stem x3: act 0 (none) or 1 (relu)");
  MX_CHECK_ARG(x && w && y, "conv stem x3: null operand");
  MX_CHECK_ARG(s->N * s->H * s->W * s->C * 4 < (1ll << 31), "conv stem x3: input must stay below 2 GiB");
  StemP p{};
  p.x = x; p.w = w; p.bias = bias; p.y = y; p.stats = stats;
  p.M = s->N * s->Ho * s->Wo;
  p.mblocks = cdiv(p.M, SROWS);
  p.H = (int)s->H; p.W = (int)s->W; p.C = (int)s->C; p.Ho = (int)s->Ho; p.Wo = (int)s->Wo;
  p.st_h = s->stride_h; p.st_w = s->stride_w; p.pad_h = s->pad_h; p.pad_w = s->pad_w; p.act = act;
  p.xbytes = (int)(s->N * s->H * s->W * s->C * 4);
  const int64_t ntiles = cdiv(p.M, 16 * STEM_T);
  const int64_t slots = 2 * (int64_t)num_cus();
  p.tiles_per_block = std::max<int64_t>(4, cdiv(ntiles, slots));  // ~2 blocks per CU, equal shares
  const int64_t blocks = cdiv(ntiles, p.tiles_per_block);
  conv_stem_x3_kernel<<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(p);
  MX_LAUNCH_CHECK();
  return MX_OK;
}
