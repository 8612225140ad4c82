// mx_roialign.hip — torchvision::roi_align forward/backward and MultiScaleRoIAlign, NHWC, gfx950.
//
// Restates torchvision 0.20.1 roi_align_kernel.cpp / roi_align_common.h (oracle/mx_oracle.c
// orc_roi_align_fwd/bwd): roi start/end = coord*scale (- 0.5 if aligned), size clamped to >= 1
// when !aligned, bin = size/pooled, sample at start + p*bin + (i+.5)*bin/grid, bilinear with the
// (<-1 or >H) skip and edge clamp, out = sum(((w1 f1 + w2 f2) + w3 f3) + w4 f4) / count.
// Built -ffp-contract=off so each f32 op rounds as the C++ does: with f32 features the forward is
// bit-identical to the CPU kernel (same op order per output element). Backward uses f32 atomics.
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

__device__ __forceinline__ Samp make_samp(const RoiGeo& g, int64_t H, int64_t W, int ph, int pw, int iy, int ix) {
  Samp s;
  float y = (g.sh + (float)ph * g.bh) + ((float)iy + .5f) * g.bh / (float)g.gh;
  float x = (g.sw + (float)pw * g.bw) + ((float)ix + .5f) * g.bw / (float)g.gw;
  if (y < -1.0f || y > (float)H || x < -1.0f || x > (float)W) {
    s.p1 = -1; s.p2 = s.p3 = s.p4 = 0;
    s.w1 = s.w2 = s.w3 = s.w4 = 0.f;
    return s;
  }
  if (y <= 0) y = 0;
  if (x <= 0) x = 0;
  int64_t yl = (int64_t)y, xl = (int64_t)x, yh, xh;
  if (yl >= H - 1) { yh = yl = H - 1; y = (float)yl; } else yh = yl + 1;
  if (xl >= W - 1) { xh = xl = W - 1; x = (float)xl; } else xh = xl + 1;
  float ly = y - (float)yl, lx = x - (float)xl, hy = 1.f - ly, hx = 1.f - lx;
  s.p1 = (int32_t)(yl * W + xl); s.p2 = (int32_t)(yl * W + xh);
  s.p3 = (int32_t)(yh * W + xl); s.p4 = (int32_t)(yh * W + xh);
  s.w1 = hy * hx; s.w2 = hy * lx; s.w3 = ly * hx; s.w4 = ly * lx;
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

// ---- bf16 forward, 8 channels per lane ----------------------------------------------------------
// Same per-channel arithmetic (and order) as roi_align_fwd_kernel, 16-B loads: a group of C/8 lanes
// covers one bin's channel row, 256 / (C/8) groups stride the bins.
__global__ void __launch_bounds__(256) roi_align_fwd_v8_kernel(Levels L, int64_t C, const float* __restrict__ rois, int PH,
                                                               int PW, int sampling, int aligned, int multiscale,
                                                               uint16_t* __restrict__ out, int32_t* __restrict__ lv_out) {
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
  const int nbins = PH * PW;
  const int ns = nbins * per_bin;
  for (int i = threadIdx.x; i < ns; i += blockDim.x) {
    int bin = i / per_bin, sidx = i % per_bin;
    tab[i] = make_samp(g, H, W, bin / PW, bin % PW, sidx / g.gw, sidx % g.gw);
  }
  __syncthreads();
  const int C8 = (int)(C / 8);
  const uint16_t* f = (const uint16_t*)L.f[lv] + g.b * H * W * C;
  for (int e = threadIdx.x; e < nbins * C8; e += blockDim.x) {
    const int bin = e / C8, c0 = (e - bin * C8) * 8;
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int s = 0; s < per_bin; ++s) {
      const Samp p = tab[bin * per_bin + s];
      if (p.p1 < 0) continue;
      const uint4 u1 = *(const uint4*)(f + (int64_t)p.p1 * C + c0), u2 = *(const uint4*)(f + (int64_t)p.p2 * C + c0);
      const uint4 u3 = *(const uint4*)(f + (int64_t)p.p3 * C + c0), u4 = *(const uint4*)(f + (int64_t)p.p4 * C + c0);
      const uint16_t *h1 = (const uint16_t*)&u1, *h2 = (const uint16_t*)&u2, *h3 = (const uint16_t*)&u3,
                     *h4 = (const uint16_t*)&u4;
#pragma unroll
      for (int t = 0; t < 8; ++t)
        v[t] += ((p.w1 * bf2f(h1[t]) + p.w2 * bf2f(h2[t])) + p.w3 * bf2f(h3[t])) + p.w4 * bf2f(h4[t]);
    }
    uint4 o;
    uint16_t* oh = (uint16_t*)&o;
#pragma unroll
    for (int t = 0; t < 8; ++t) oh[t] = f2bf(v[t] / g.count);
    *(uint4*)(out + (k * nbins + bin) * C + c0) = o;
  }
}

static int check_grid(int PH, int PW, int sampling) {
  if (PH <= 0 || PW <= 0) return 0;
  if (sampling > 0 && PH * PW * sampling * sampling > kMaxSamp) return 0;
  return 1;
}

}  // namespace mx

using namespace mx;

static int launch_fwd(const Levels& L, int dtype, int64_t C, const float* rois, int64_t K, int PH, int PW, int sampling,
                      int aligned, int ms, void* out, int32_t* lv, hipStream_t s) {
  MX_CHECK_ARG(check_grid(PH, PW, sampling), "roi_align: unsupported pooled %dx%d sampling %d", PH, PW, sampling);
  MX_CHECK_ARG(sampling > 0, "roi_align: adaptive sampling (sampling_ratio<=0) not supported");
  MX_CHECK_ARG(dtype == MX_F32 || dtype == MX_BF16, "roi_align: bad dtype %d", dtype);
  if (K == 0) return MX_OK;
  int threads = C >= 256 ? 256 : (int)(cdiv(C, 64) * 64);
  if (dtype == MX_F32)
    roi_align_fwd_kernel<float><<<(unsigned)K, threads, 0, s>>>(L, C, rois, PH, PW, sampling, aligned, ms, (float*)out, lv);
  else if (C % 8 == 0)
    roi_align_fwd_v8_kernel<<<(unsigned)K, 256, 0, s>>>(L, C, rois, PH, PW, sampling, aligned, ms, (uint16_t*)out, lv);
  else
    roi_align_fwd_kernel<uint16_t><<<(unsigned)K, threads, 0, s>>>(L, C, rois, PH, PW, sampling, aligned, ms,
                                                                    (uint16_t*)out, lv);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

static int launch_bwd(const Levels& L, int dtype, int64_t C, const float* rois, const int32_t* lv, int64_t K, int PH, int PW,
                      int sampling, int aligned, const void* gout, hipStream_t s) {
  MX_CHECK_ARG(check_grid(PH, PW, sampling), "roi_align: unsupported pooled %dx%d sampling %d", PH, PW, sampling);
  MX_CHECK_ARG(sampling > 0, "roi_align: adaptive sampling (sampling_ratio<=0) not supported");
  MX_CHECK_ARG(dtype == MX_F32 || dtype == MX_BF16, "roi_align: bad dtype %d", dtype);
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
                                mx_stream_t stream) {
  (void)N;
  MX_CHECK_ARG(H * W < (1ll << 31), "roi_align: feature map too large");
  Levels L{};
  L.g[0] = grad_feat; L.H[0] = H; L.W[0] = W; L.scale[0] = scale; L.n = 1; L.k_min = 0;
  return launch_bwd(L, dtype, C, rois, nullptr, K, PH, PW, sampling, aligned, gout, (hipStream_t)stream);
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

extern "C" int mx_multiscale_roi_align_bwd(const void* gout, int dtype, float* const* gfeats, const int64_t* Hs,
                                           const int64_t* Ws, const float* scales, int nlev, int64_t C, const float* rois,
                                           const int32_t* levels, int64_t K, int PH, int PW, int sampling,
                                           mx_stream_t stream) {
  MX_CHECK_ARG(nlev >= 1 && nlev <= 5, "multiscale_roi_align: 1..5 levels");
  MX_CHECK_ARG(levels != nullptr, "multiscale_roi_align_bwd: levels from the forward are required");
  Levels L{};
  for (int i = 0; i < nlev; ++i) {
    L.g[i] = gfeats[i]; L.H[i] = Hs[i]; L.W[i] = Ws[i]; L.scale[i] = scales[i];
  }
  L.n = nlev; L.k_min = 0;
  return launch_bwd(L, dtype, C, rois, levels, K, PH, PW, sampling, 0, gout, (hipStream_t)stream);
}
