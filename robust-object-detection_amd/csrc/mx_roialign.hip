// mx_roialign.hip — torchvision::roi_align forward/backward and MultiScaleRoIAlign, NHWC, gfx950.
//
// Restates torchvision 0.20.1 roi_align_kernel.cpp / roi_align_common.h (oracle/mx_oracle.c
// orc_roi_align_fwd/bwd): roi start/end = coord*scale (- 0.5 if aligned), size clamped to >= 1
// when !aligned, bin = size/pooled, sample at start + p*bin + (i+.5)*bin/grid, bilinear with the
// (<-1 or >H) skip and edge clamp, out = sum(((w1 f1 + w2 f2) + w3 f3) + w4 f4) / count.
// Built -ffp-contract=off so each f32 op rounds as the C++ does: with f32 features the forward is
// bit-identical to the CPU kernel (same op order per output element). Backward: a deterministic
// gather (default; fixed summation order per element, bitwise reproducible, every level-map element
// written once) or f32 atomics (deterministic = 0; the caller zero-fills the gradient maps).
//
// Serves RoIHeads.box_roi_pool = MultiScaleRoIAlign(['0','1','2','3'], 7, 2) (reached from
// train_frcnn_baseline.py:171 / eval_all.py:111), whose LevelMapper is fused here:
//   lvl = floor(4 + log2(sqrt(area)/224) + 1e-6), clamped to [k_min, k_max].
//
// Layout: features NHWC so a RoI bin's C channels are one contiguous row: one block per RoI,
// threads over channels (coalesced 2/4-byte lanes), the per-sample bilinear table (positions +
// weights, identical for every channel) computed once per RoI into LDS.
#include "mx_common.h"

namespace mx {

struct Samp {
  int32_t p1, p2, p3, p4;  // pixel offsets y*W+x; p1 < 0 -> sample outside, contributes nothing
  float w1, w2, w3, w4;
};

static constexpr int kMaxSamp = 1024;  // 32 KiB of LDS; 7x7 bins x 2x2 samples = 196
static constexpr int kMergeBins = 49, kMergeCorners = 16;  // backward corner merge: 7x7 bins, 2x2 samples

struct RoiGeo {
  float sw, sh, bw, bh, count;
  int gh, gw;
  int64_t b;
};

__device__ __forceinline__ RoiGeo roi_geo(const float* r, float scale, int PH, int PW, int sampling, int aligned) {
  RoiGeo g;
  float off = aligned ? 0.5f : 0.f;
  g.b = (int64_t)r[0];
  g.sw = r[1] * scale - off;
  g.sh = r[2] * scale - off;
  float ew = r[3] * scale - off, eh = r[4] * scale - off;
  float rw = ew - g.sw, rh = eh - g.sh;
  if (!aligned) {
    rw = fmaxf(rw, 1.f);
    rh = fmaxf(rh, 1.f);
  }
  g.bh = rh / (float)PH;
  g.bw = rw / (float)PW;
  g.gh = sampling > 0 ? sampling : (int)ceilf(rh / (float)PH);
  g.gw = sampling > 0 ? sampling : (int)ceilf(rw / (float)PW);
  int cnt = g.gh * g.gw;
  g.count = (float)(cnt < 1 ? 1 : cnt);
  return g;
}

// One bilinear sample: its corner rows/cols (yl, yh) x (xl, xh) and weights; false if the sample
// lies outside [-1, H] x [-1, W] (contributes nothing).
__device__ __forceinline__ bool sample_corners(const RoiGeo& g, int64_t H, int64_t W, int ph, int pw, int iy, int ix,
                                               int& yl, int& xl, int& yh, int& xh, float (&w)[4]) {
  float y = (g.sh + (float)ph * g.bh) + ((float)iy + .5f) * g.bh / (float)g.gh;
  float x = (g.sw + (float)pw * g.bw) + ((float)ix + .5f) * g.bw / (float)g.gw;
  if (y < -1.0f || y > (float)H || x < -1.0f || x > (float)W) return false;
  if (y <= 0) y = 0;
  if (x <= 0) x = 0;
  yl = (int)y;
  xl = (int)x;
  if (yl >= H - 1) { yh = yl = (int)H - 1; y = (float)yl; } else yh = yl + 1;
  if (xl >= W - 1) { xh = xl = (int)W - 1; x = (float)xl; } else xh = xl + 1;
  float ly = y - (float)yl, lx = x - (float)xl, hy = 1.f - ly, hx = 1.f - lx;
  w[0] = hy * hx; w[1] = hy * lx; w[2] = ly * hx; w[3] = ly * lx;
  return true;
}

__device__ __forceinline__ Samp make_samp(const RoiGeo& g, int64_t H, int64_t W, int ph, int pw, int iy, int ix) {
  Samp s;
  int yl, xl, yh, xh;
  float w[4];
  if (!sample_corners(g, H, W, ph, pw, iy, ix, yl, xl, yh, xh, w)) {
    s.p1 = -1; s.p2 = s.p3 = s.p4 = 0;
    s.w1 = s.w2 = s.w3 = s.w4 = 0.f;
    return s;
  }
  s.p1 = (int32_t)((int64_t)yl * W + xl); s.p2 = (int32_t)((int64_t)yl * W + xh);
  s.p3 = (int32_t)((int64_t)yh * W + xl); s.p4 = (int32_t)((int64_t)yh * W + xh);
  s.w1 = w[0]; s.w2 = w[1]; s.w3 = w[2]; s.w4 = w[3];
  return s;
}

struct Levels {
  const void* f[5];
  float* g[5];
  int64_t H[5], W[5];
  float scale[5];
  int n, k_min;
};

__device__ __forceinline__ int level_of(const float* r, int k_min, int n) {
  // LevelMapper: s = sqrt(box_area); floor(lvl0 + log2(s / s0) + eps), clamp, - k_min
  float area = (r[3] - r[1]) * (r[4] - r[2]);
  float s = sqrtf(area);
  float t = floorf((4.0f + log2f(s / 224.0f)) + 1e-6f);
  float lo = (float)k_min, hi = (float)(k_min + n - 1);
  t = t < lo ? lo : (t > hi ? hi : t);
  return (int)t - k_min;
}

// one block per RoI (blockIdx.x), threads stride the channels
template <typename T>
__global__ void __launch_bounds__(256) roi_align_fwd_kernel(Levels L, int64_t C, const float* __restrict__ rois, int PH,
                                                            int PW, int sampling, int aligned, int multiscale,
                                                            T* __restrict__ out, int32_t* __restrict__ lv_out) {
  __shared__ Samp tab[kMaxSamp];
  __shared__ RoiGeo sg;
  __shared__ int slv;
  const int64_t k = blockIdx.x;
  const float* r = rois + 5 * k;
  if (threadIdx.x == 0) {
    int lv = multiscale ? level_of(r, L.k_min, L.n) : 0;
    slv = lv;
    sg = roi_geo(r, L.scale[lv], PH, PW, sampling, aligned);
    if (lv_out) lv_out[k] = lv;
  }
  __syncthreads();
  const int lv = slv;
  const RoiGeo g = sg;
  const int64_t H = L.H[lv], W = L.W[lv];
  const int per_bin = g.gh * g.gw;
  const int ns = PH * PW * per_bin;
  for (int i = threadIdx.x; i < ns; i += blockDim.x) {
    int bin = i / per_bin, sidx = i % per_bin;
    tab[i] = make_samp(g, H, W, bin / PW, bin % PW, sidx / g.gw, sidx % g.gw);
  }
  __syncthreads();
  const T* f = (const T*)L.f[lv] + g.b * H * W * C;
  for (int64_t c = threadIdx.x; c < C; c += blockDim.x) {
    for (int bin = 0; bin < PH * PW; ++bin) {
      float v = 0.f;
      for (int s = 0; s < per_bin; ++s) {
        const Samp p = tab[bin * per_bin + s];
        if (p.p1 < 0) continue;
        float f1 = io<T>::ld(f + (int64_t)p.p1 * C + c), f2 = io<T>::ld(f + (int64_t)p.p2 * C + c);
        float f3 = io<T>::ld(f + (int64_t)p.p3 * C + c), f4 = io<T>::ld(f + (int64_t)p.p4 * C + c);
        v += ((p.w1 * f1 + p.w2 * f2) + p.w3 * f3) + p.w4 * f4;
      }
      io<T>::st(out + (k * PH * PW + bin) * C + c, v / g.count);
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) roi_align_bwd_kernel(Levels L, int64_t C, const float* __restrict__ rois,
                                                            const int32_t* __restrict__ lv_in, int PH, int PW, int sampling,
                                                            int aligned, const T* __restrict__ gout) {
  __shared__ Samp tab[kMaxSamp];
  __shared__ RoiGeo sg;
  __shared__ int slv;
  const int64_t k = blockIdx.x;
  const float* r = rois + 5 * k;
  if (threadIdx.x == 0) {
    int lv = lv_in ? lv_in[k] : 0;
    slv = lv;
    sg = roi_geo(r, L.scale[lv], PH, PW, sampling, aligned);
  }
  __syncthreads();
  const int lv = slv;
  const RoiGeo g = sg;
  const int64_t H = L.H[lv], W = L.W[lv];
  const int per_bin = g.gh * g.gw;
  const int ns = PH * PW * per_bin;
  for (int i = threadIdx.x; i < ns; i += blockDim.x) {
    int bin = i / per_bin, sidx = i % per_bin;
    tab[i] = make_samp(g, H, W, bin / PW, bin % PW, sidx / g.gw, sidx % g.gw);
  }
  __syncthreads();
  float* gf = L.g[lv] + g.b * H * W * C;
  const int nbins = PH * PW;
  if (nbins <= kMergeBins && per_bin * 4 <= kMergeCorners) {
    // Within a bin every sample scales the same gout value, so corners that hit the same pixel
    // (2x2 samples of a bin narrower than ~2 px share most of them) are merged first: one atomic
    // per distinct pixel with the summed bilinear weight (~2-4x fewer atomics per RoI).
    __shared__ int32_t mpix[kMergeBins][kMergeCorners];
    __shared__ float mw[kMergeBins][kMergeCorners];
    __shared__ int mcnt[kMergeBins];
    for (int bin = threadIdx.x; bin < nbins; bin += blockDim.x) {
      int n = 0;
      for (int s = 0; s < per_bin; ++s) {
        const Samp p = tab[bin * per_bin + s];
        if (p.p1 < 0) continue;
        const int32_t pp[4] = {p.p1, p.p2, p.p3, p.p4};
        const float ww[4] = {p.w1, p.w2, p.w3, p.w4};
        for (int q = 0; q < 4; ++q) {
          int j = 0;
          while (j < n && mpix[bin][j] != pp[q]) ++j;
          if (j == n) {
            mpix[bin][n] = pp[q];
            mw[bin][n] = ww[q];
            ++n;
          } else {
            mw[bin][j] += ww[q];
          }
        }
      }
      mcnt[bin] = n;
    }
    __syncthreads();
    const float inv = 1.f / g.count;
    for (int64_t c = threadIdx.x; c < C; c += blockDim.x) {
      for (int bin = 0; bin < nbins; ++bin) {
        const float go = io<T>::ld(gout + (k * nbins + bin) * C + c) * inv;
        const int n = mcnt[bin];
        for (int j = 0; j < n; ++j) atomicAdd(gf + (int64_t)mpix[bin][j] * C + c, go * mw[bin][j]);
      }
    }
    return;
  }
  for (int64_t c = threadIdx.x; c < C; c += blockDim.x) {
    for (int bin = 0; bin < nbins; ++bin) {
      float go = io<T>::ld(gout + (k * nbins + bin) * C + c);
      for (int s = 0; s < per_bin; ++s) {
        const Samp p = tab[bin * per_bin + s];
        if (p.p1 < 0) continue;
        atomicAdd(gf + (int64_t)p.p1 * C + c, go * p.w1 / g.count);
        atomicAdd(gf + (int64_t)p.p2 * C + c, go * p.w2 / g.count);
        atomicAdd(gf + (int64_t)p.p3 * C + c, go * p.w3 / g.count);
        atomicAdd(gf + (int64_t)p.p4 * C + c, go * p.w4 / g.count);
      }
    }
  }
}

// ---- vector forward, 8 channels per lane (bf16: one 16-B load, f32: two) -------------------------
// Same per-channel arithmetic (and order) as roi_align_fwd_kernel: a group of C/8 lanes covers one
// bin's channel row, 256 / (C/8) groups stride the bins, and every lane keeps its 4 samples x 4
// corners of loads independent (16-32 loads in flight per lane instead of one scalar at a time).
template <typename T>
__global__ void __launch_bounds__(256) roi_align_fwd_v8_kernel(Levels L, int64_t C, const float* __restrict__ rois, int PH,
                                                               int PW, int sampling, int aligned, int multiscale,
                                                               T* __restrict__ out, int32_t* __restrict__ lv_out) {
  extern __shared__ Samp tab[];  // [PH * PW * sampling^2] (sized at launch: more blocks per CU)
  __shared__ RoiGeo sg;
  __shared__ int slv;
  const int64_t k = blockIdx.x;
  const float* r = rois + 5 * k;
  if (threadIdx.x == 0) {
    int lv = multiscale ? level_of(r, L.k_min, L.n) : 0;
    slv = lv;
    sg = roi_geo(r, L.scale[lv], PH, PW, sampling, aligned);
    if (lv_out) lv_out[k] = lv;
  }
  __syncthreads();
  const int lv = slv;
  const RoiGeo g = sg;
  const int64_t H = L.H[lv], W = L.W[lv];
  const int per_bin = g.gh * g.gw;
  const int nbins = PH * PW;
  const int ns = nbins * per_bin;
  for (int i = threadIdx.x; i < ns; i += blockDim.x) {
    int bin = i / per_bin, sidx = i % per_bin;
    tab[i] = make_samp(g, H, W, bin / PW, bin % PW, sidx / g.gw, sidx % g.gw);
  }
  __syncthreads();
  // gridDim.y channel slices per RoI (mx_roi_fwd_set_split): more, shorter blocks in flight
  const int C8 = (int)(C / 8) / (int)gridDim.y, cb = (int)blockIdx.y * C8 * 8;
  const T* f = (const T*)L.f[lv] + g.b * H * W * C;
  for (int e = threadIdx.x; e < nbins * C8; e += blockDim.x) {
    const int bin = e / C8, c0 = cb + (e - bin * C8) * 8;
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int s = 0; s < per_bin; ++s) {
      const Samp p = tab[bin * per_bin + s];
      if (p.p1 < 0) continue;
      float f1[8], f2[8], f3[8], f4[8];
      ld8(f + (int64_t)p.p1 * C + c0, f1);
      ld8(f + (int64_t)p.p2 * C + c0, f2);
      ld8(f + (int64_t)p.p3 * C + c0, f3);
      ld8(f + (int64_t)p.p4 * C + c0, f4);
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] += ((p.w1 * f1[t] + p.w2 * f2[t]) + p.w3 * f3[t]) + p.w4 * f4[t];
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = v[t] / g.count;
    st8(out + (k * nbins + bin) * C + c0, v);
  }
}

// ---- deterministic backward (gather form, no atomics) ---------------------------------------------
// grad_feat[n, y, x, :] = sum over the RoIs k of image n at this level, their bins and the bilinear
// corners landing on (y, x) of gout[k, bin, :] / count * w. Pass 1 (one block per RoI) merges each
// bin's corners per distinct pixel (summed weights, fixed sample/corner order) into
// ent[k][bin][0..cnt) and records the RoI's pixel footprint. Pass 2 (one block per 8x8 pixel tile of
// every level map and image) walks the RoIs overlapping its tile in ascending k; wave w owns 64/G
// of the tile's pixels in an LDS f32 accumulator and adds their contributions in (k, bin, corner)
// order, so every output element has one fixed summation order: bitwise reproducible. Every pixel
// of every level map is written exactly once (untouched ones as 0): no zero-fill, no atomics.
struct BwdEnt {
  int32_t yx;  // y << 16 | x on the level map
  float w;     // summed bilinear weight of this pixel within the bin
};

// Pass 1: one block per RoI, one thread per bin: the bin's per_bin samples x 4 corners as entries in
// torchvision's loop order (iy, ix, corner 1..4; roi_align_kernel.cpp roi_align_backward_kernel_impl),
// yx = -1 for samples outside the map, plus the bin's and the RoI's pixel bbox.
__global__ void __launch_bounds__(64) roi_bwd_prep_kernel(Levels L, const float* __restrict__ rois,
                                                          const int32_t* __restrict__ lv_in, int PH, int PW, int sampling,
                                                          int aligned, int S4, BwdEnt* __restrict__ ent,
                                                          int2* __restrict__ binbox, int4* __restrict__ box,
                                                          int32_t* __restrict__ meta) {
  __shared__ int sb[4];
  const int64_t k = blockIdx.x;
  const float* r = rois + 5 * k;
  const int lv = lv_in ? lv_in[k] : 0;
  const RoiGeo g = roi_geo(r, L.scale[lv], PH, PW, sampling, aligned);
  const int64_t H = L.H[lv], W = L.W[lv];
  const int per_bin = g.gh * g.gw, nbins = PH * PW;
  if (threadIdx.x == 0) {
    sb[0] = sb[2] = 0x7fffffff;
    sb[1] = sb[3] = -1;
  }
  __syncthreads();
  int y0 = 0x7fffffff, y1 = -1, x0 = 0x7fffffff, x1 = -1;
  for (int bin = threadIdx.x; bin < nbins; bin += blockDim.x) {
    BwdEnt* e = ent + (k * nbins + bin) * S4;
    int by0 = 0x7fff, by1 = -1, bx0 = 0x7fff, bx1 = -1;
    for (int sidx = 0; sidx < per_bin; ++sidx) {
      int yl, xl, yh, xh;
      float ww[4];
      if (!sample_corners(g, H, W, bin / PW, bin % PW, sidx / g.gw, sidx % g.gw, yl, xl, yh, xh, ww)) {
        for (int q = 0; q < 4; ++q) { e[4 * sidx + q].yx = -1; e[4 * sidx + q].w = 0.f; }
        continue;
      }
      const int cy[4] = {yl, yl, yh, yh}, cx[4] = {xl, xh, xl, xh};
      for (int q = 0; q < 4; ++q) {
        e[4 * sidx + q].yx = (cy[q] << 16) | cx[q];
        e[4 * sidx + q].w = ww[q];
      }
      by0 = min(by0, yl); by1 = max(by1, yh); bx0 = min(bx0, xl); bx1 = max(bx1, xh);
    }
    for (int j = 4 * per_bin; j < S4; ++j) { e[j].yx = -1; e[j].w = 0.f; }
    binbox[k * nbins + bin] = make_int2((by0 & 0xffff) | (by1 << 16), (bx0 & 0xffff) | (bx1 << 16));
    y0 = min(y0, by0); y1 = max(y1, by1); x0 = min(x0, bx0); x1 = max(x1, bx1);
  }
  atomicMin(&sb[0], y0); atomicMax(&sb[1], y1); atomicMin(&sb[2], x0); atomicMax(&sb[3], x1);
  __syncthreads();
  if (threadIdx.x == 0) {
    box[k] = make_int4(sb[0], sb[1], sb[2], sb[3]);
    meta[k] = (int32_t)(g.b * 8 + lv);
  }
}

struct TileGrid {
  int64_t first[6];  // first tile id of each level (level-major, then image, then tile row, col)
  int tw[5], th[5];
  int n;
};

template <typename T>
__device__ __forceinline__ float4 ld4f(const T* p) {
  if constexpr (sizeof(T) == 2) {
    const uint2 u = *(const uint2*)p;
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                       __uint_as_float(u.y & 0xffff0000u));
  } else {
    return *(const float4*)p;
  }
}

// Pass 2: one block per 8x8 tile, 8 waves; wave w owns the tile's pixel row w (8 pixels, f32
// accumulators in registers), lanes = channel quads (C <= 256). The RoIs overlapping the tile
// are listed in ascending k (one ordered block compaction per 1024 RoIs); each wave then walks them
// independently (no barriers): a ballot over the RoI's bins picks those whose pixel bbox meets the
// wave's strip, 64/S4 (<= 4) such bins are loaded at once -- their corner slots one per lane and their
// gout rows one quad per lane, the next group (of this or a later RoI) prefetched while the current
// one is applied -- and the hit bits are walked in slot order with readlane: fixed order per output
// element.
template <typename T, int SW>
__global__ void __launch_bounds__(512, 2) roi_bwd_gather_kernel(Levels L, TileGrid TG, int64_t C, int64_t K, int nbins, int S4,
                                                             float count, const BwdEnt* __restrict__ ent,
                                                             const int2* __restrict__ binbox, const int4* __restrict__ box,
                                                             const int32_t* __restrict__ meta, const T* __restrict__ gout) {
  __shared__ int list[1024];
  __shared__ int wcnt[2][8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t id = blockIdx.x;
  int lv = 0;
  while (lv + 1 < TG.n && id >= TG.first[lv + 1]) ++lv;
  const int64_t rem = id - TG.first[lv];
  const int per_img = TG.th[lv] * TG.tw[lv];
  const int n = (int)(rem / per_img), t = (int)(rem % per_img);
  const int ty0 = (t / TG.tw[lv]) * 8, tx0 = (t % TG.tw[lv]) * SW;
  const int64_t H = L.H[lv], W = L.W[lv];
  const int Q = (int)(C / 4);
  const bool qa = lane < Q;  // this lane's channel quad exists
  // this wave's 8 pixels (named registers: an indexed array would go to scratch)
  float4 a0{}, a1{}, a2{}, a3{}, a4{}, a5{}, a6{}, a7{};
  const float inv = 1.f / count;
  const bool pow2 = inv * count == 1.f && (__float_as_uint(count) & 0x7fffffu) == 0;
  const int32_t want = n * 8 + lv;
  const int sy0 = ty0 + wave;  // this wave's strip: row sy0, cols tx0..tx0+SW-1
  const int NBC = min(4, 64 / S4);  // bins per load group
  const int sub = lane / S4, sj = lane - sub * S4;
  for (int64_t c0 = 0; c0 < K; c0 += 1024) {
    bool hit[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int64_t kq = c0 + r * 512 + tid;
      hit[r] = false;
      if (kq < K && meta[kq] == want) {
        const int4 b = box[kq];
        hit[r] = b.x <= ty0 + 7 && b.y >= ty0 && b.z <= tx0 + SW - 1 && b.w >= tx0;
      }
    }
    uint64_t m[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      m[r] = __ballot(hit[r]);
      if (lane == 0) wcnt[r][wave] = __popcll(m[r]);
    }
    __syncthreads();
    int base = 0;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      int pre = 0, tot = 0;
      for (int w = 0; w < 8; ++w) {
        pre += w < wave ? wcnt[r][w] : 0;
        tot += wcnt[r][w];
      }
      if (hit[r]) list[base + pre + __popcll(m[r] & ((1ull << lane) - 1))] = (int)(c0 + r * 512 + tid);
      base += tot;
    }
    const int nl = base;
    __syncthreads();
    // Pipelined walk over the listed RoIs (ascending k: the fixed summation order), 64 at a time.
    // Phase 1: each RoI's bins on this strip as a 64-bit mask in lane (j - j0), from binbox rows of 8
    // RoIs per round trip. Phase 2: the RoIs with hits in order, as a stream of (RoI, bin group)
    // loads double-buffered in two named register sets: the next group (of this or a later RoI) is in
    // flight while the current one is applied. Every load is unconditional (clamped indices, results
    // masked after) so the compiler's counted waits stay exact across the loop.
    for (int j0 = 0; j0 < nl; j0 += 64) {
      const int nb = min(64, nl - j0);
      uint32_t bml = 0, bmh = 0;
      const int bl = min(lane, nbins - 1);
      for (int r0 = 0; r0 < nb; r0 += 8) {
        int2 bb[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) bb[r] = binbox[(int64_t)list[j0 + min(r0 + r, nb - 1)] * nbins + bl];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int by0 = (int)(int16_t)(bb[r].x & 0xffff), by1 = bb[r].x >> 16;
          const int bx0 = (int)(int16_t)(bb[r].y & 0xffff), bx1 = bb[r].y >> 16;
          const bool bh = lane < nbins && r0 + r < nb && by0 <= sy0 && by1 >= sy0 && bx0 <= tx0 + SW - 1 && bx1 >= tx0;
          const uint64_t bmr = __ballot(bh);
          if (lane == r0 + r) {
            bml = (uint32_t)bmr;
            bmh = (uint32_t)(bmr >> 32);
          }
        }
      }
      uint64_t todo = __ballot((bml | bmh) != 0u);  // RoIs of this batch with a bin on the strip
      int cj = 0;                                    // cursor: RoI (batch lane) and its bins not yet loaded
      uint64_t cbm = 0;
      auto advance = [&]() -> bool {
        if (cbm == 0) {
          if (todo == 0) return false;
          cj = __builtin_ctzll(todo);
          todo &= todo - 1;
          cbm = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)bmh, cj) << 32) |
                (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)bml, cj);
        }
        return true;
      };
      // a load group: up to NBC (<= 4) bins of the cursor RoI in order; lane (sub, sj) holds corner
      // slot sj of bin sub, lane q channel quad q of each bin's gout row
      struct Grp {
        int g0, g1, g2, g3;
        bool ev;  // this lane's corner slot belongs to a loaded bin
        BwdEnt e;
        float4 o0, o1, o2, o3;  // raw rows: slots without a bin have no hits, lanes >= Q are never stored
      };
      const int qc = min(lane, Q - 1);
      auto load_group = [&](Grp& G, bool valid) {
        const int64_t kk = list[j0 + (valid ? cj : 0)];
        G.g0 = G.g1 = G.g2 = G.g3 = -1;
        if (valid) {
#define MX_TAKE(gbv, s)                        \
  if (s < NBC && cbm) {                        \
    gbv = __builtin_ctzll(cbm);                \
    cbm &= cbm - 1;                            \
  }
          MX_TAKE(G.g0, 0) MX_TAKE(G.g1, 1) MX_TAKE(G.g2, 2) MX_TAKE(G.g3, 3)
#undef MX_TAKE
        }
        const int mb = sub == 0 ? G.g0 : sub == 1 ? G.g1 : sub == 2 ? G.g2 : sub == 3 ? G.g3 : -1;
        G.ev = sub < NBC && mb >= 0;
        G.e = ent[(kk * nbins + max(mb, 0)) * S4 + (sub < NBC ? sj : 0)];
        G.o0 = ld4f(gout + (kk * nbins + max(G.g0, 0)) * C + 4 * qc);
        G.o1 = ld4f(gout + (kk * nbins + max(G.g1, 0)) * C + 4 * qc);
        G.o2 = ld4f(gout + (kk * nbins + max(G.g2, 0)) * C + 4 * qc);
        G.o3 = ld4f(gout + (kk * nbins + max(G.g3, 0)) * C + 4 * qc);
      };
      auto apply = [&](const Grp& G) {
        const BwdEnt ce = G.e;
        const int y = (ce.yx >> 16) - sy0, x = (ce.yx & 0xffff) - tx0;
        const bool inb = G.ev && ce.yx >= 0 && y == 0 && (unsigned)x < (unsigned)SW;
        const int plv = inb ? x : -1;  // pixel within the wave's 1x8 strip
        const uint64_t hm = __ballot(inb);
        if (hm) {
          // per pixel, its hits in slot order (bin-sub s ascending, then lane): the static loops keep
          // every accumulator and gout quad in named registers
          uint64_t pm[8];
#pragma unroll
          for (int p = 0; p < SW; ++p) pm[p] = __ballot(plv == p);
          const uint64_t sl = S4 >= 64 ? ~0ull : ((1ull << S4) - 1);
#define MX_RUN(sv, cgv)                                                            \
  {                                                                                \
    const float4 cg = cgv;                                                         \
    const uint64_t sm = hm & (sl << (sv * S4));                                    \
    if (sv < NBC && sm) {                                                          \
      MX_PIX(0) MX_PIX(1) MX_PIX(2) MX_PIX(3) MX_PIX(4) MX_PIX(5) MX_PIX(6) MX_PIX(7)  \
    }                                                                              \
  }
#define MX_PIX(pp)                                                                  \
  if (pp < SW) {                                                                    \
    uint64_t m = sm & pm[pp];                                                       \
    while (m) {                                                                     \
      const int b = __builtin_ctzll(m);                                             \
      m &= m - 1;                                                                   \
      const float w = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ce.w), b)); \
      float vx = cg.x * w, vy = cg.y * w, vz = cg.z * w, vw = cg.w * w;             \
      if (pow2) { vx *= inv; vy *= inv; vz *= inv; vw *= inv; }                     \
      else { vx /= count; vy /= count; vz /= count; vw /= count; }                  \
      a##pp.x += vx; a##pp.y += vy; a##pp.z += vz; a##pp.w += vw;                   \
    }                                                                               \
  }
          MX_RUN(0, G.o0) MX_RUN(1, G.o1) MX_RUN(2, G.o2) MX_RUN(3, G.o3)
#undef MX_PIX
#undef MX_RUN
        }
      };
      Grp ga, gb;
      bool ha = advance();
      load_group(ga, ha);
      while (ha) {
        const bool hb = advance();
        load_group(gb, hb);  // prefetch (a dummy load past the end: keeps the wait counts exact)
        apply(ga);
        if (!hb) break;
        ha = advance();
        load_group(ga, ha);
        apply(gb);
      }
    }
    __syncthreads();  // list rebuilt for the next 1024 RoIs
  }
  float* gmap = L.g[lv] + (int64_t)n * H * W * C;
  if (qa) {
    const float4 av[8] = {a0, a1, a2, a3, a4, a5, a6, a7};
#pragma unroll
    for (int i = 0; i < SW; ++i) {
      const int y = sy0, x = tx0 + i;
      if (y < H && x < W) *((float4*)(gmap + ((int64_t)y * W + x) * C) + lane) = av[i];
    }
  }
}

// ---- adaptive sampling grid (sampling_ratio <= 0: ceil(roi_h / PH) x ceil(roi_w / PW) per RoI) -------
// torchvision.ops.roi_align's default. The grid of a large RoI can hold thousands of samples per bin,
// so the bilinear setup is recomputed per sample instead of tabled in LDS; the per-channel
// accumulation order (iy, ix; corners 1..4) is torchvision's. One block per RoI, threads over
// (bin, channel), consecutive lanes on consecutive channels.
template <typename T>
__global__ void __launch_bounds__(256) roi_align_fwd_adaptive_kernel(Levels L, int64_t C, const float* __restrict__ rois,
                                                                     int PH, int PW, int aligned, int multiscale,
                                                                     T* __restrict__ out, int32_t* __restrict__ lv_out) {
  const int64_t k = blockIdx.x;
  const float* r = rois + 5 * k;
  const int lv = multiscale ? level_of(r, L.k_min, L.n) : 0;
  if (lv_out && threadIdx.x == 0) lv_out[k] = lv;
  const RoiGeo g = roi_geo(r, L.scale[lv], PH, PW, 0, aligned);
  const int64_t H = L.H[lv], W = L.W[lv];
  const T* f = (const T*)L.f[lv] + g.b * H * W * C;
  const int64_t nbins = (int64_t)PH * PW;
  for (int64_t e = threadIdx.x; e < nbins * C; e += blockDim.x) {
    const int bin = (int)(e / C);
    const int64_t c = e - (int64_t)bin * C;
    float v = 0.f;
    for (int iy = 0; iy < g.gh; ++iy)
      for (int ix = 0; ix < g.gw; ++ix) {
        int yl, xl, yh, xh;
        float w[4];
        if (!sample_corners(g, H, W, bin / PW, bin % PW, iy, ix, yl, xl, yh, xh, w)) continue;
        const float f1 = io<T>::ld(f + ((int64_t)yl * W + xl) * C + c), f2 = io<T>::ld(f + ((int64_t)yl * W + xh) * C + c);
        const float f3 = io<T>::ld(f + ((int64_t)yh * W + xl) * C + c), f4 = io<T>::ld(f + ((int64_t)yh * W + xh) * C + c);
        v += ((w[0] * f1 + w[1] * f2) + w[2] * f3) + w[3] * f4;
      }
    io<T>::st(out + (k * nbins + bin) * C + c, v / g.count);
  }
}

// backward with the adaptive grid: f32 atomics into zero-filled maps (torchvision's CUDA backward
// scheme; g_i = gout * w_i / count per corner)
template <typename T>
__global__ void __launch_bounds__(256) roi_align_bwd_adaptive_kernel(Levels L, int64_t C, const float* __restrict__ rois,
                                                                     const int32_t* __restrict__ lv_in, int PH, int PW,
                                                                     int aligned, const T* __restrict__ gout) {
  const int64_t k = blockIdx.x;
  const float* r = rois + 5 * k;
  const int lv = lv_in ? lv_in[k] : 0;
  const RoiGeo g = roi_geo(r, L.scale[lv], PH, PW, 0, aligned);
  const int64_t H = L.H[lv], W = L.W[lv];
  float* gf = L.g[lv] + g.b * H * W * C;
  const int64_t nbins = (int64_t)PH * PW;
  for (int64_t e = threadIdx.x; e < nbins * C; e += blockDim.x) {
    const int bin = (int)(e / C);
    const int64_t c = e - (int64_t)bin * C;
    const float go = io<T>::ld(gout + (k * nbins + bin) * C + c);
    for (int iy = 0; iy < g.gh; ++iy)
      for (int ix = 0; ix < g.gw; ++ix) {
        int yl, xl, yh, xh;
        float w[4];
        if (!sample_corners(g, H, W, bin / PW, bin % PW, iy, ix, yl, xl, yh, xh, w)) continue;
        atomicAdd(gf + ((int64_t)yl * W + xl) * C + c, go * w[0] / g.count);
        atomicAdd(gf + ((int64_t)yl * W + xh) * C + c, go * w[1] / g.count);
        atomicAdd(gf + ((int64_t)yh * W + xl) * C + c, go * w[2] / g.count);
        atomicAdd(gf + ((int64_t)yh * W + xh) * C + c, go * w[3] / g.count);
      }
  }
}

static int check_grid(int PH, int PW, int sampling) {
  if (PH <= 0 || PW <= 0) return 0;
  if (sampling > 0 && PH * PW * sampling * sampling > kMaxSamp) return 0;
  return 1;
}

}  // namespace mx

using namespace mx;

// forward: channel slices per RoI block (mx_roi_fwd_set_split: 1, 2, 4 or 8; 4 measured 65 vs 76 us cold on the
// step's 1,024 RoIs: four 64-channel blocks per RoI keep more gathers in flight per CU)
static int g_roi_fwd_split = 4;
extern "C" int mx_roi_fwd_set_split(int n) {
  MX_CHECK_ARG(n == 1 || n == 2 || n == 4 || n == 8, "mx_roi_fwd_set_split: 1, 2, 4 or 8");
  g_roi_fwd_split = n;
  return MX_OK;
}

static int launch_fwd(const Levels& L, int dtype, int64_t C, const float* rois, int64_t K, int PH, int PW, int sampling,
                      int aligned, int ms, void* out, int32_t* lv, hipStream_t s) {
  MX_CHECK_ARG(check_grid(PH, PW, sampling), "roi_align: unsupported pooled %dx%d sampling %d", PH, PW, sampling);
  MX_CHECK_ARG(dtype == MX_F32 || dtype == MX_BF16, "roi_align: bad dtype %d", dtype);
  if (K == 0) return MX_OK;
  if (sampling <= 0) {
    if (dtype == MX_F32)
      roi_align_fwd_adaptive_kernel<float><<<(unsigned)K, 256, 0, s>>>(L, C, rois, PH, PW, aligned, ms, (float*)out, lv);
    else
      roi_align_fwd_adaptive_kernel<uint16_t><<<(unsigned)K, 256, 0, s>>>(L, C, rois, PH, PW, aligned, ms,
                                                                          (uint16_t*)out, lv);
    MX_LAUNCH_CHECK();
    return MX_OK;
  }
  int threads = C >= 256 ? 256 : (int)(cdiv(C, 64) * 64);
  const int cs = (C % 8 == 0 && (C / 8) % g_roi_fwd_split == 0) ? g_roi_fwd_split : 1;
  const dim3 grid((unsigned)K, (unsigned)cs);
  const size_t tab = sizeof(Samp) * (size_t)PH * PW * sampling * sampling;
  if (C % 8 == 0 && dtype == MX_F32)
    roi_align_fwd_v8_kernel<float><<<grid, 256, tab, s>>>(L, C, rois, PH, PW, sampling, aligned, ms, (float*)out, lv);
  else if (C % 8 == 0)
    roi_align_fwd_v8_kernel<uint16_t><<<grid, 256, tab, s>>>(L, C, rois, PH, PW, sampling, aligned, ms,
                                                             (uint16_t*)out, lv);
  else if (dtype == MX_F32)
    roi_align_fwd_kernel<float><<<(unsigned)K, threads, 0, s>>>(L, C, rois, PH, PW, sampling, aligned, ms, (float*)out, lv);
  else
    roi_align_fwd_kernel<uint16_t><<<(unsigned)K, threads, 0, s>>>(L, C, rois, PH, PW, sampling, aligned, ms,
                                                                    (uint16_t*)out, lv);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

// deterministic-backward workspace: ent [K][nbins][4*sampling^2], cnt [K][nbins], box [K], meta [K]
static size_t det_ws_bytes(int64_t K, int PH, int PW, int sampling) {
  const int64_t nb = (int64_t)PH * PW, S4 = 4ll * sampling * sampling;
  return align_up(sizeof(BwdEnt) * K * nb * S4) + align_up(sizeof(int2) * K * nb) + align_up(sizeof(int4) * K) +
         align_up(sizeof(int32_t) * K);
}

// one channel quad per lane (C <= 256); 16 pixels x 4 channels of f32 accumulators per lane
static bool det_supported(int64_t C) { return C >= 4 && C <= 256 && C % 4 == 0; }

// deterministic gather tile: 8 rows x g_roi_strip columns (one wave per row strip). Narrower strips cut
// the work of the block and of each wave on tiles that many RoIs overlap (the kernel's tail) at more
// blocks (each re-scans the RoI list): mx_roi_bwd_set_strip
static int g_roi_strip = 2;
extern "C" int mx_roi_bwd_set_strip(int sw) {
  MX_CHECK_ARG(sw == 2 || sw == 4 || sw == 8, "mx_roi_bwd_set_strip: 2, 4 or 8");
  g_roi_strip = sw;
  return MX_OK;
}

static int launch_bwd(const Levels& L, int64_t N, int dtype, int64_t C, const float* rois, const int32_t* lv, int64_t K,
                      int PH, int PW, int sampling, int aligned, const void* gout, int deterministic, void* ws,
                      size_t ws_bytes, hipStream_t s) {
  MX_CHECK_ARG(check_grid(PH, PW, sampling), "roi_align: unsupported pooled %dx%d sampling %d", PH, PW, sampling);
  MX_CHECK_ARG(dtype == MX_F32 || dtype == MX_BF16, "roi_align: bad dtype %d", dtype);
  if (sampling <= 0) {  // adaptive grid: atomics only (the caller zero-fills the maps)
    MX_CHECK_ARG(!deterministic, "roi_align_bwd: the deterministic gather needs a fixed sampling_ratio in 1..4");
    if (K == 0) return MX_OK;
    if (dtype == MX_F32)
      roi_align_bwd_adaptive_kernel<float><<<(unsigned)K, 256, 0, s>>>(L, C, rois, lv, PH, PW, aligned, (const float*)gout);
    else
      roi_align_bwd_adaptive_kernel<uint16_t><<<(unsigned)K, 256, 0, s>>>(L, C, rois, lv, PH, PW, aligned,
                                                                          (const uint16_t*)gout);
    MX_LAUNCH_CHECK();
    return MX_OK;
  }
  if (deterministic) {
    MX_CHECK_ARG(det_supported(C), "roi_align_bwd deterministic: C=%lld must be a multiple of 4 in 4..256", (long long)C);
    MX_CHECK_ARG(N >= 1 && N < (1 << 27), "roi_align_bwd deterministic: bad image count");
    for (int i = 0; i < L.n; ++i)
      MX_CHECK_ARG(L.H[i] < 32768 && L.W[i] < 32768, "roi_align_bwd deterministic: level map too large");
    const size_t need = det_ws_bytes(K, PH, PW, sampling);
    MX_CHECK_ARG(K == 0 || (ws && ws_bytes >= need), "roi_align_bwd deterministic: workspace of %zu bytes required", need);
    const int nbins = PH * PW, S4 = 4 * sampling * sampling;
    MX_CHECK_ARG(nbins <= 64 && S4 <= 64, "roi_align_bwd deterministic: pooled bins <= 64 and sampling <= 4");
    char* w = (char*)ws;
    BwdEnt* ent = (BwdEnt*)w;
    w += align_up(sizeof(BwdEnt) * K * nbins * S4);
    int2* cnt = (int2*)w;
    w += align_up(sizeof(int2) * K * nbins);
    int4* box = (int4*)w;
    w += align_up(sizeof(int4) * K);
    int32_t* meta = (int32_t*)w;
    if (K > 0) {
      roi_bwd_prep_kernel<<<(unsigned)K, 64, 0, s>>>(L, rois, lv, PH, PW, sampling, aligned, S4, ent, cnt, box, meta);
      MX_LAUNCH_CHECK();
    }
    TileGrid tg{};
    tg.n = L.n;
    int64_t tot = 0;
    for (int i = 0; i < L.n; ++i) {
      tg.first[i] = tot;
      tg.th[i] = (int)cdiv(L.H[i], 8);
      tg.tw[i] = (int)cdiv(L.W[i], g_roi_strip);
      tot += N * tg.th[i] * tg.tw[i];
    }
    tg.first[L.n] = tot;
    MX_CHECK_ARG(tot < (1ll << 31), "roi_align_bwd deterministic: grid too large");
    if (tot == 0) return MX_OK;
    const float count = (float)(sampling * sampling);
#define MX_GATHER(T_, SW_)                                                                               \
  roi_bwd_gather_kernel<T_, SW_><<<(unsigned)tot, 512, 0, s>>>(L, tg, C, K, nbins, S4, count, ent, cnt, box, meta, \
                                                                (const T_*)gout)
    if (dtype == MX_F32) {
      if (g_roi_strip == 2) MX_GATHER(float, 2);
      else if (g_roi_strip == 4) MX_GATHER(float, 4);
      else MX_GATHER(float, 8);
    } else {
      if (g_roi_strip == 2) MX_GATHER(uint16_t, 2);
      else if (g_roi_strip == 4) MX_GATHER(uint16_t, 4);
      else MX_GATHER(uint16_t, 8);
    }
#undef MX_GATHER
    MX_LAUNCH_CHECK();
    return MX_OK;
  }
  if (K == 0) return MX_OK;
  int threads = C >= 256 ? 256 : (int)(cdiv(C, 64) * 64);
  if (dtype == MX_F32)
    roi_align_bwd_kernel<float><<<(unsigned)K, threads, 0, s>>>(L, C, rois, lv, PH, PW, sampling, aligned, (const float*)gout);
  else
    roi_align_bwd_kernel<uint16_t><<<(unsigned)K, threads, 0, s>>>(L, C, rois, lv, PH, PW, sampling, aligned,
                                                                    (const uint16_t*)gout);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" size_t mx_roi_align_bwd_workspace(int64_t K, int PH, int PW, int sampling) {
  if (K <= 0 || PH <= 0 || PW <= 0 || sampling <= 0) return 0;
  return det_ws_bytes(K, PH, PW, sampling);
}

extern "C" int mx_roi_align_fwd(const void* feat, int dtype, int64_t N, int64_t H, int64_t W, int64_t C, const float* rois,
                                int64_t K, float scale, int PH, int PW, int sampling, int aligned, void* out,
                                mx_stream_t stream) {
  (void)N;
  MX_CHECK_ARG(H * W < (1ll << 31), "roi_align: feature map too large");
  Levels L{};
  L.f[0] = feat; L.H[0] = H; L.W[0] = W; L.scale[0] = scale; L.n = 1; L.k_min = 0;
  return launch_fwd(L, dtype, C, rois, K, PH, PW, sampling, aligned, 0, out, nullptr, (hipStream_t)stream);
}

extern "C" int mx_roi_align_bwd(const void* gout, int dtype, int64_t N, int64_t H, int64_t W, int64_t C, const float* rois,
                                int64_t K, float scale, int PH, int PW, int sampling, int aligned, float* grad_feat,
                                int deterministic, void* ws, size_t ws_bytes, mx_stream_t stream) {
  MX_CHECK_ARG(H * W < (1ll << 31), "roi_align: feature map too large");
  Levels L{};
  L.g[0] = grad_feat; L.H[0] = H; L.W[0] = W; L.scale[0] = scale; L.n = 1; L.k_min = 0;
  return launch_bwd(L, N, dtype, C, rois, nullptr, K, PH, PW, sampling, aligned, gout, deterministic, ws, ws_bytes,
                    (hipStream_t)stream);
}

extern "C" int mx_multiscale_roi_align_fwd(const void* const* feats, const int64_t* Hs, const int64_t* Ws,
                                           const float* scales, int nlev, int k_min, int dtype, int64_t C,
                                           const float* rois, int64_t K, int PH, int PW, int sampling, void* out,
                                           int32_t* levels_out, mx_stream_t stream) {
  MX_CHECK_ARG(nlev >= 1 && nlev <= 5, "multiscale_roi_align: 1..5 levels");
  Levels L{};
  for (int i = 0; i < nlev; ++i) {
    L.f[i] = feats[i]; L.H[i] = Hs[i]; L.W[i] = Ws[i]; L.scale[i] = scales[i];
    MX_CHECK_ARG(Hs[i] * Ws[i] < (1ll << 31), "roi_align: feature map too large");
  }
  L.n = nlev; L.k_min = k_min;
  return launch_fwd(L, dtype, C, rois, K, PH, PW, sampling, 0, 1, out, levels_out, (hipStream_t)stream);
}

extern "C" int mx_multiscale_roi_align_bwd(const void* gout, int dtype, float* const* gfeats, int64_t N, const int64_t* Hs,
                                           const int64_t* Ws, const float* scales, int nlev, int64_t C, const float* rois,
                                           const int32_t* levels, int64_t K, int PH, int PW, int sampling,
                                           int deterministic, void* ws, size_t ws_bytes, mx_stream_t stream) {
  MX_CHECK_ARG(nlev >= 1 && nlev <= 5, "multiscale_roi_align: 1..5 levels");
  MX_CHECK_ARG(levels != nullptr, "multiscale_roi_align_bwd: levels from the forward are required");
  Levels L{};
  for (int i = 0; i < nlev; ++i) {
    L.g[i] = gfeats[i]; L.H[i] = Hs[i]; L.W[i] = Ws[i]; L.scale[i] = scales[i];
  }
  L.n = nlev; L.k_min = 0;
  return launch_bwd(L, N, dtype, C, rois, levels, K, PH, PW, sampling, 0, gout, deterministic, ws, ws_bytes,
                    (hipStream_t)stream);
}
