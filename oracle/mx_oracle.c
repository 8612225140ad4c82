/* mx_oracle.c — CPU restatement (TEST INFRASTRUCTURE ONLY; see mx_oracle.h header).
 *
 * Compiled with -O2 -ffp-contract=off -fno-fast-math so that every float op rounds once, in the
 * order the restated C++/ATen code evaluates it (torchvision's CPU kernels are built in ISO C++
 * mode on x86-64 baseline, which never contracts a*b+c).
 */
#include "mx_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

static inline float fmaxf_(float a, float b) { return a > b ? a : b; }
static inline float fminf_(float a, float b) { return a < b ? a : b; }

/* torchvision/ops/boxes.py box_iou + _box_inter_union:
 *   area = (x2-x1)*(y2-y1); lt = max(b1[:2], b2[:2]); rb = min(b1[2:], b2[2:]);
 *   wh = (rb-lt).clamp(min=0); inter = wh0*wh1; union = area1 + area2 - inter; iou = inter/union.
 * Serves rpn.py assign_targets_to_anchors (train_frcnn_baseline.py:171) and roi_heads.py
 * assign_targets_to_proposals. */
static inline float iou1(const float* a, const float* b) {
  float area1 = (a[2] - a[0]) * (a[3] - a[1]);
  float area2 = (b[2] - b[0]) * (b[3] - b[1]);
  float ltx = fmaxf_(a[0], b[0]), lty = fmaxf_(a[1], b[1]);
  float rbx = fminf_(a[2], b[2]), rby = fminf_(a[3], b[3]);
  float w = rbx - ltx, h = rby - lty;
  if (w < 0.f) w = 0.f;
  if (h < 0.f) h = 0.f;
  float inter = w * h;
  float uni = (area1 + area2) - inter;
  return inter / uni;
}

void orc_box_iou(const float* b1, int64_t n, const float* b2, int64_t m, float* out) {
  for (int64_t i = 0; i < n; ++i)
    for (int64_t j = 0; j < m; ++j) out[i * m + j] = iou1(b1 + 4 * i, b2 + 4 * j);
}

/* torchvision/models/detection/_utils.py Matcher.__call__ + set_low_quality_matches_:
 *   matched_vals, matches = q.max(dim=0)          (first index on ties)
 *   matches[vals < low] = -1; matches[(vals >= low) & (vals < high)] = -2
 *   if allow_low_quality: for every (g, a) with q[g,a] == q[g].max(): matches[a] = all_matches[a] */
void orc_matcher(const float* q, int64_t G, int64_t A, float high, float low, int allow_lq, int64_t* matches) {
  int64_t* all = (int64_t*)malloc(sizeof(int64_t) * (A > 0 ? A : 1));
  for (int64_t a = 0; a < A; ++a) {
    float best = q[a];
    int64_t bi = 0;
    for (int64_t g = 1; g < G; ++g) {
      float v = q[g * A + a];
      if (v > best) { best = v; bi = g; }
    }
    all[a] = bi;
    int64_t m = bi;
    if (best < low) m = -1;
    else if (best < high) m = -2;
    matches[a] = m;
  }
  if (allow_lq) {
    for (int64_t g = 0; g < G; ++g) {
      float mx = -INFINITY;
      for (int64_t a = 0; a < A; ++a) if (q[g * A + a] > mx) mx = q[g * A + a];
      for (int64_t a = 0; a < A; ++a) if (q[g * A + a] == mx) matches[a] = all[a];
    }
  }
  free(all);
}

/* ---- NMS ---------------------------------------------------------------------------------- */
typedef struct { float s; int64_t i; } si_t;
/* stable descending sort by score (torchvision nms_kernel.cpp: scores.sort(stable=true, desc)) */
static int cmp_desc(const void* x, const void* y) {
  const si_t* a = (const si_t*)x; const si_t* b = (const si_t*)y;
  if (a->s > b->s) return -1;
  if (a->s < b->s) return 1;
  return (a->i < b->i) ? -1 : (a->i > b->i);
}

/* torchvision/csrc/ops/cpu/nms_kernel.cpp nms_kernel_impl. */
int64_t orc_nms(const float* boxes, const float* scores, int64_t n, double thr, int64_t* keep) {
  if (n == 0) return 0;
  si_t* ord = (si_t*)malloc(sizeof(si_t) * n);
  float* area = (float*)malloc(sizeof(float) * n);
  char* sup = (char*)calloc(n, 1);
  for (int64_t i = 0; i < n; ++i) {
    ord[i].s = scores[i]; ord[i].i = i;
    const float* b = boxes + 4 * i;
    area[i] = (b[2] - b[0]) * (b[3] - b[1]);
  }
  qsort(ord, n, sizeof(si_t), cmp_desc);
  int64_t nk = 0;
  for (int64_t _i = 0; _i < n; ++_i) {
    int64_t i = ord[_i].i;
    if (sup[i]) continue;
    keep[nk++] = i;
    const float* bi = boxes + 4 * i;
    for (int64_t _j = _i + 1; _j < n; ++_j) {
      int64_t j = ord[_j].i;
      if (sup[j]) continue;
      const float* bj = boxes + 4 * j;
      float xx1 = fmaxf_(bi[0], bj[0]), yy1 = fmaxf_(bi[1], bj[1]);
      float xx2 = fminf_(bi[2], bj[2]), yy2 = fminf_(bi[3], bj[3]);
      float w = fmaxf_(0.f, xx2 - xx1), h = fmaxf_(0.f, yy2 - yy1);
      float inter = w * h;
      float ovr = inter / ((area[i] + area[j]) - inter);
      if ((double)ovr > thr) sup[j] = 1;
    }
  }
  free(ord); free(area); free(sup);
  return nk;
}

static int cmp_i64(const void* x, const void* y) {
  int64_t a = *(const int64_t*)x, b = *(const int64_t*)y;
  return (a > b) - (a < b);
}

/* torchvision/ops/boxes.py batched_nms (CPU threshold 4000 numel):
 *   _batched_nms_vanilla: per class id (torch.unique order) nms, keep mask, then
 *       keep_indices[scores[keep_indices].sort(descending=True)]
 *   _batched_nms_coordinate_trick: offsets = idxs.to(boxes) * (boxes.max() + 1); nms(boxes+off) */
int64_t orc_batched_nms(const float* boxes, const float* scores, const int64_t* idxs, int64_t n, double thr,
                        int64_t* keep) {
  if (n == 0) return 0;
  if (n * 4 > 4000) {
    char* km = (char*)calloc(n, 1);
    int64_t* cls = (int64_t*)malloc(sizeof(int64_t) * n);
    memcpy(cls, idxs, sizeof(int64_t) * n);
    qsort(cls, n, sizeof(int64_t), cmp_i64);
    float* cb = (float*)malloc(sizeof(float) * 4 * n);
    float* cs = (float*)malloc(sizeof(float) * n);
    int64_t* ci = (int64_t*)malloc(sizeof(int64_t) * n);
    int64_t* ck = (int64_t*)malloc(sizeof(int64_t) * n);
    for (int64_t u = 0; u < n; ++u) {
      if (u > 0 && cls[u] == cls[u - 1]) continue;
      int64_t c = cls[u], m = 0;
      for (int64_t i = 0; i < n; ++i)
        if (idxs[i] == c) {
          memcpy(cb + 4 * m, boxes + 4 * i, 16); cs[m] = scores[i]; ci[m] = i; ++m;
        }
      int64_t nk = orc_nms(cb, cs, m, thr, ck);
      for (int64_t k = 0; k < nk; ++k) km[ci[ck[k]]] = 1;
    }
    int64_t nk = 0;
    si_t* ord = (si_t*)malloc(sizeof(si_t) * n);
    for (int64_t i = 0; i < n; ++i) if (km[i]) { ord[nk].s = scores[i]; ord[nk].i = i; ++nk; }
    qsort(ord, nk, sizeof(si_t), cmp_desc);
    for (int64_t k = 0; k < nk; ++k) keep[k] = ord[k].i;
    free(km); free(cls); free(cb); free(cs); free(ci); free(ck); free(ord);
    return nk;
  }
  float mx = boxes[0];
  for (int64_t i = 1; i < 4 * n; ++i) if (boxes[i] > mx) mx = boxes[i];
  float step = mx + 1.0f;
  float* ob = (float*)malloc(sizeof(float) * 4 * n);
  for (int64_t i = 0; i < n; ++i) {
    float off = (float)idxs[i] * step;
    for (int k = 0; k < 4; ++k) ob[4 * i + k] = boxes[4 * i + k] + off;
  }
  int64_t nk = orc_nms(ob, scores, n, thr, keep);
  free(ob);
  return nk;
}

/* ---- RoIAlign ------------------------------------------------------------------------------ */
/* torchvision/csrc/ops/cpu/roi_align_common.h pre_calc_for_bilinear_interpolate and
 * roi_align_kernel.cpp roi_align_forward_kernel_impl (aligned=False in MultiScaleRoIAlign). */
typedef struct { int64_t p1, p2, p3, p4; float w1, w2, w3, w4; } pc_t;

static void bilin_pre(int64_t H, int64_t W, float y, float x, pc_t* pc) {
  if (y < -1.0f || y > (float)H || x < -1.0f || x > (float)W) {
    memset(pc, 0, sizeof(*pc));
    return;
  }
  if (y <= 0) y = 0;
  if (x <= 0) x = 0;
  int64_t yl = (int64_t)y, xl = (int64_t)x, yh, xh;
  if (yl >= H - 1) { yh = yl = H - 1; y = (float)yl; } else yh = yl + 1;
  if (xl >= W - 1) { xh = xl = W - 1; x = (float)xl; } else xh = xl + 1;
  float ly = y - (float)yl, lx = x - (float)xl, hy = 1.f - ly, hx = 1.f - lx;
  pc->p1 = yl * W + xl; pc->p2 = yl * W + xh; pc->p3 = yh * W + xl; pc->p4 = yh * W + xh;
  pc->w1 = hy * hx; pc->w2 = hy * lx; pc->w3 = ly * hx; pc->w4 = ly * lx;
}

typedef struct { float sw, sh, bw, bh; int gh, gw; float count; int64_t b; } roi_geo_t;
static roi_geo_t roi_geo(const float* r, float scale, int PH, int PW, int sampling, int aligned) {
  roi_geo_t g;
  float off = aligned ? 0.5f : 0.f;
  g.b = (int64_t)r[0];
  g.sw = r[1] * scale - off; g.sh = r[2] * scale - off;
  float ew = r[3] * scale - off, eh = r[4] * scale - off;
  float rw = ew - g.sw, rh = eh - g.sh;
  if (!aligned) { rw = fmaxf_(rw, 1.f); rh = fmaxf_(rh, 1.f); }
  g.bh = rh / (float)PH; g.bw = rw / (float)PW;
  g.gh = sampling > 0 ? sampling : (int)ceilf(rh / (float)PH);
  g.gw = sampling > 0 ? sampling : (int)ceilf(rw / (float)PW);
  int cnt = g.gh * g.gw; if (cnt < 1) cnt = 1;
  g.count = (float)cnt;
  return g;
}

static inline float sample_y(const roi_geo_t* g, int ph, int iy) {
  return (g->sh + (float)ph * g->bh) + ((float)iy + .5f) * g->bh / (float)g->gh;
}
static inline float sample_x(const roi_geo_t* g, int pw, int ix) {
  return (g->sw + (float)pw * g->bw) + ((float)ix + .5f) * g->bw / (float)g->gw;
}

void orc_roi_align_fwd(const float* in, int64_t N, int64_t C, int64_t H, int64_t W, const float* rois, int64_t K,
                       float scale, int PH, int PW, int sampling, int aligned, float* out) {
  (void)N;
  for (int64_t k = 0; k < K; ++k) {
    roi_geo_t g = roi_geo(rois + 5 * k, scale, PH, PW, sampling, aligned);
    pc_t* pre = (pc_t*)malloc(sizeof(pc_t) * PH * PW * (g.gh * g.gw > 0 ? g.gh * g.gw : 1));
    int64_t pi = 0;
    for (int ph = 0; ph < PH; ++ph)
      for (int pw = 0; pw < PW; ++pw)
        for (int iy = 0; iy < g.gh; ++iy) {
          float y = sample_y(&g, ph, iy);
          for (int ix = 0; ix < g.gw; ++ix) bilin_pre(H, W, y, sample_x(&g, pw, ix), &pre[pi++]);
        }
    for (int64_t c = 0; c < C; ++c) {
      const float* f = in + (g.b * C + c) * H * W;
      pi = 0;
      for (int ph = 0; ph < PH; ++ph)
        for (int pw = 0; pw < PW; ++pw) {
          float v = 0.f;
          for (int s = 0; s < g.gh * g.gw; ++s) {
            const pc_t* p = &pre[pi++];
            v += ((p->w1 * f[p->p1] + p->w2 * f[p->p2]) + p->w3 * f[p->p3]) + p->w4 * f[p->p4];
          }
          out[((k * C + c) * PH + ph) * PW + pw] = v / g.count;
        }
    }
    free(pre);
  }
}

/* roi_align_kernel.cpp roi_align_backward_kernel_impl + bilinear_interpolate_gradient. */
void orc_roi_align_bwd(const float* go, int64_t N, int64_t C, int64_t H, int64_t W, const float* rois, int64_t K,
                       float scale, int PH, int PW, int sampling, int aligned, float* gi) {
  (void)N;
  for (int64_t k = 0; k < K; ++k) {
    roi_geo_t g = roi_geo(rois + 5 * k, scale, PH, PW, sampling, aligned);
    for (int64_t c = 0; c < C; ++c) {
      float* f = gi + (g.b * C + c) * H * W;
      for (int ph = 0; ph < PH; ++ph)
        for (int pw = 0; pw < PW; ++pw) {
          float gv = go[((k * C + c) * PH + ph) * PW + pw];
          for (int iy = 0; iy < g.gh; ++iy) {
            float y0 = sample_y(&g, ph, iy);
            for (int ix = 0; ix < g.gw; ++ix) {
              float y = y0, x = sample_x(&g, pw, ix);
              if (y < -1.0f || y > (float)H || x < -1.0f || x > (float)W) continue;
              if (y <= 0) y = 0;
              if (x <= 0) x = 0;
              int64_t yl = (int64_t)y, xl = (int64_t)x, yh, xh;
              if (yl >= H - 1) { yh = yl = H - 1; y = (float)yl; } else yh = yl + 1;
              if (xl >= W - 1) { xh = xl = W - 1; x = (float)xl; } else xh = xl + 1;
              float ly = y - (float)yl, lx = x - (float)xl, hy = 1.f - ly, hx = 1.f - lx;
              float w1 = hy * hx, w2 = hy * lx, w3 = ly * hx, w4 = ly * lx;
              f[yl * W + xl] += gv * w1 / g.count;
              f[yl * W + xh] += gv * w2 / g.count;
              f[yh * W + xl] += gv * w3 / g.count;
              f[yh * W + xh] += gv * w4 / g.count;
            }
          }
        }
    }
  }
}

/* ---- anchors / box coder ------------------------------------------------------------------- */
/* torchvision/models/detection/anchor_utils.py generate_anchors + grid_anchors:
 *   h_ratios = sqrt(ar); w_ratios = 1/h_ratios; ws = w_ratios*size; hs = h_ratios*size;
 *   base = round(stack([-ws,-hs,ws,hs])/2)  (round half to even);
 *   shifts = (arange(gw)*stride_w, arange(gh)*stride_h) meshgrid ij; anchors = shift + base,
 *   ordered (y, x, ratio). */
void orc_anchors_level(float size, const float* ratios, int nr, int64_t gh, int64_t gw, int64_t sh, int64_t sw,
                       float* out) {
  float base[16][4];
  for (int r = 0; r < nr; ++r) {
    float hr = sqrtf(ratios[r]);
    float wr = 1.f / hr;
    float ws = wr * size, hs = hr * size;
    base[r][0] = rintf(-ws / 2.f); base[r][1] = rintf(-hs / 2.f);
    base[r][2] = rintf(ws / 2.f); base[r][3] = rintf(hs / 2.f);
  }
  int64_t o = 0;
  for (int64_t y = 0; y < gh; ++y)
    for (int64_t x = 0; x < gw; ++x)
      for (int r = 0; r < nr; ++r) {
        float sx = (float)(x * sw), sy = (float)(y * sh);
        out[o++] = sx + base[r][0]; out[o++] = sy + base[r][1];
        out[o++] = sx + base[r][2]; out[o++] = sy + base[r][3];
      }
}

/* torchvision det_utils.BoxCoder.decode_single: rel[n, ncls*4], boxes[n,4] -> out[n, ncls*4]. */
void orc_box_decode(const float* rel, const float* boxes, int64_t n, int64_t ncls, const float* w, float clip,
                    float* out) {
  for (int64_t i = 0; i < n; ++i) {
    const float* b = boxes + 4 * i;
    float widths = b[2] - b[0], heights = b[3] - b[1];
    float cx = b[0] + 0.5f * widths, cy = b[1] + 0.5f * heights;
    for (int64_t c = 0; c < ncls; ++c) {
      const float* r = rel + (i * ncls + c) * 4;
      float dx = r[0] / w[0], dy = r[1] / w[1], dw = r[2] / w[2], dh = r[3] / w[3];
      if (dw > clip) dw = clip;
      if (dh > clip) dh = clip;
      float pcx = dx * widths + cx, pcy = dy * heights + cy;
      float pw = expf(dw) * widths, ph = expf(dh) * heights;
      float hw = 0.5f * pw, hh = 0.5f * ph;
      float* o = out + (i * ncls + c) * 4;
      o[0] = pcx - hw; o[1] = pcy - hh; o[2] = pcx + hw; o[3] = pcy + hh;
    }
  }
}

/* torchvision det_utils.encode_boxes(reference_boxes=gt, proposals). */
void orc_box_encode(const float* gt, const float* prop, int64_t n, const float* w, float* out) {
  for (int64_t i = 0; i < n; ++i) {
    const float* p = prop + 4 * i; const float* g = gt + 4 * i;
    float ew = p[2] - p[0], eh = p[3] - p[1];
    float ecx = p[0] + 0.5f * ew, ecy = p[1] + 0.5f * eh;
    float gw = g[2] - g[0], gh = g[3] - g[1];
    float gcx = g[0] + 0.5f * gw, gcy = g[1] + 0.5f * gh;
    out[4 * i + 0] = w[0] * (gcx - ecx) / ew;
    out[4 * i + 1] = w[1] * (gcy - ecy) / eh;
    out[4 * i + 2] = w[2] * logf(gw / ew);
    out[4 * i + 3] = w[3] * logf(gh / eh);
  }
}

/* ---- corruption (augmentations.py) --------------------------------------------------------- */
void orc_noise_u8(const uint8_t* img, const float* noise, int64_t n, uint8_t* out) {
  for (int64_t i = 0; i < n; ++i) {
    float v = (float)img[i] + noise[i];
    if (v < 0.f) v = 0.f;
    if (v > 255.f) v = 255.f;
    out[i] = (uint8_t)v; /* numpy astype(uint8) truncates toward zero */
  }
}

static inline int64_t refl101(int64_t i, int64_t n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) { if (i < 0) i = -i; if (i >= n) i = 2 * n - 2 - i; }
  return i;
}

/* filter2D(src, -1, k) with k = 9x9, row 4 = float(1/9), BORDER_REFLECT_101: zero taps are dropped,
 * sum = sum_t float(1/9)*src in f32, saturate_cast<uchar> = round half to even. */
void orc_blur_h9_u8(const uint8_t* img, int64_t H, int64_t W, int64_t C, uint8_t* out) {
  const float k = 1.0f / 9.0f;
  for (int64_t y = 0; y < H; ++y)
    for (int64_t x = 0; x < W; ++x)
      for (int64_t c = 0; c < C; ++c) {
        float s = 0.f;
        for (int t = -4; t <= 4; ++t) s += k * (float)img[(y * W + refl101(x + t, W)) * C + c];
        float r = rintf(s);
        if (r < 0) r = 0;
        if (r > 255) r = 255;
        out[(y * W + x) * C + c] = (uint8_t)r;
      }
}

/* OpenCV imgproc/resize.cpp computeResizeAreaTab (general INTER_AREA path). */
typedef struct { int64_t di, si; float alpha; } area_t;
static int64_t area_tab(int64_t ssize, int64_t dsize, double scale, area_t* tab) {
  int64_t k = 0;
  for (int64_t dx = 0; dx < dsize; ++dx) {
    double fsx1 = dx * scale, fsx2 = fsx1 + scale;
    double cell = scale < (ssize - fsx1) ? scale : (ssize - fsx1);
    int64_t sx1 = (int64_t)ceil(fsx1), sx2 = (int64_t)floor(fsx2);
    if (sx2 > ssize - 1) sx2 = ssize - 1;
    if (sx1 > sx2) sx1 = sx2;
    if (sx1 - fsx1 > 1e-3) { tab[k].di = dx; tab[k].si = sx1 - 1; tab[k++].alpha = (float)((sx1 - fsx1) / cell); }
    for (int64_t sx = sx1; sx < sx2; ++sx) { tab[k].di = dx; tab[k].si = sx; tab[k++].alpha = (float)(1.0 / cell); }
    if (fsx2 - sx2 > 1e-3) {
      double d = fsx2 - sx2; if (d > 1.) d = 1.; if (d > cell) d = cell;
      tab[k].di = dx; tab[k].si = sx2; tab[k++].alpha = (float)(d / cell);
    }
  }
  return k;
}

/* ResizeArea_Invoker: out row = saturate(sum_y beta_y * (sum_x alpha_x * S)), f32 buffers. */
void orc_resize_area_u8(const uint8_t* src, int64_t sh, int64_t sw, int64_t C, uint8_t* dst, int64_t dh, int64_t dw) {
  double sx = (double)sw / dw, sy = (double)sh / dh;
  area_t* xt = (area_t*)malloc(sizeof(area_t) * (sw * 2 + 2));
  area_t* yt = (area_t*)malloc(sizeof(area_t) * (sh * 2 + 2));
  int64_t nx = area_tab(sw, dw, sx, xt), ny = area_tab(sh, dh, sy, yt);
  float* buf = (float*)malloc(sizeof(float) * dw * C);
  float* sum = (float*)calloc(dw * C, sizeof(float));
  int64_t prev = -1;
  for (int64_t j = 0; j < ny; ++j) {
    float beta = yt[j].alpha;
    int64_t dy = yt[j].di;
    const uint8_t* S = src + yt[j].si * sw * C;
    for (int64_t k = 0; k < dw * C; ++k) buf[k] = 0.f;
    for (int64_t k = 0; k < nx; ++k) {
      int64_t s = xt[k].si * C, d = xt[k].di * C;
      float a = xt[k].alpha;
      for (int64_t c = 0; c < C; ++c) buf[d + c] = buf[d + c] + (float)S[s + c] * a;
    }
    if (dy != prev) {
      if (prev >= 0)
        for (int64_t k = 0; k < dw * C; ++k) {
          float r = rintf(sum[k]); dst[prev * dw * C + k] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
        }
      for (int64_t k = 0; k < dw * C; ++k) sum[k] = beta * buf[k];
      prev = dy;
    } else {
      for (int64_t k = 0; k < dw * C; ++k) sum[k] = sum[k] + beta * buf[k];
    }
  }
  if (prev >= 0)
    for (int64_t k = 0; k < dw * C; ++k) {
      float r = rintf(sum[k]); dst[prev * dw * C + k] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
    }
  free(xt); free(yt); free(buf); free(sum);
}

/* INTER_LINEAR 8U: coefficients in 11-bit fixed point (INTER_RESIZE_COEF_BITS), horizontal pass
 * exact in int; vertical pass as OpenCV's SIMD VResizeLinearVec_32s8u computes it:
 *   out = sat_u8(( mulhi16(S0>>4, b0) + mulhi16(S1>>4, b1) + 2 ) >> 2)
 * (the scalar tail uses (S0*b0 + S1*b1 + 2^21) >> 22; the two differ by at most 1 LSB). */
static void lin_tab(int64_t ssize, int64_t dsize, int64_t* ofs, short* al) {
  double scale = 1.0 / ((double)dsize / ssize);
  for (int64_t d = 0; d < dsize; ++d) {
    float f = (float)((d + 0.5) * scale - 0.5);
    int64_t s = (int64_t)floorf(f);
    f -= (float)s;
    if (s < 0) { f = 0.f; s = 0; }
    if (s >= ssize - 1) { f = 0.f; s = ssize - 1; }
    ofs[d] = s;
    al[2 * d] = (short)lrintf((1.f - f) * 2048.f);
    al[2 * d + 1] = (short)lrintf(f * 2048.f);
  }
}

void orc_resize_linear_u8(const uint8_t* src, int64_t sh, int64_t sw, int64_t C, uint8_t* dst, int64_t dh, int64_t dw) {
  int64_t* xo = (int64_t*)malloc(sizeof(int64_t) * dw);
  int64_t* yo = (int64_t*)malloc(sizeof(int64_t) * dh);
  short* xa = (short*)malloc(sizeof(short) * 2 * dw);
  short* ya = (short*)malloc(sizeof(short) * 2 * dh);
  lin_tab(sw, dw, xo, xa);
  lin_tab(sh, dh, yo, ya);
  for (int64_t y = 0; y < dh; ++y) {
    int64_t r0 = yo[y], r1 = r0 + 1 < sh ? r0 + 1 : sh - 1;
    int b0 = ya[2 * y], b1 = ya[2 * y + 1];
    for (int64_t x = 0; x < dw; ++x) {
      int64_t c0 = xo[x], c1 = c0 + 1 < sw ? c0 + 1 : sw - 1;
      int a0 = xa[2 * x], a1 = xa[2 * x + 1];
      for (int64_t c = 0; c < C; ++c) {
        int S0 = src[(r0 * sw + c0) * C + c] * a0 + src[(r0 * sw + c1) * C + c] * a1;
        int S1 = src[(r1 * sw + c0) * C + c] * a0 + src[(r1 * sw + c1) * C + c] * a1;
        int v = ((((S0 >> 4) * b0) >> 16) + (((S1 >> 4) * b1) >> 16) + 2) >> 2;
        dst[(y * dw + x) * C + c] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
      }
    }
  }
  free(xo); free(yo); free(xa); free(ya);
}

/* OpenCV resize, INTER_AREA with is_area_fast (both scales exactly the integer 2): resizeAreaFast_.
 * ResizeAreaFastVec_SIMD_8u (128-bit x86-64 baseline) handles the first elements of each destination
 * row: cn 3 in steps of 48 (3 x 16 lanes, v_load_deinterleave), cn 1 in steps of 8, cn 4 in steps of
 * 16, each as v_rshr_pack<2>: (a + b + c + d + 2) >> 2. The remaining elements of the row take the
 * scalar loop: saturate_cast<uchar>(sum * (1.f / area)) = cvRound, half to even. */
void orc_resize_area_fast2_u8(const uint8_t* src, int64_t sh, int64_t sw, int64_t C, uint8_t* dst, int64_t dh,
                              int64_t dw) {
  const int64_t w = dw * C;
  const int64_t step = C == 1 ? 8 : (C == 3 ? 48 : (C == 4 ? 16 : 0));
  const int64_t vec = step ? (w / step) * step : 0;
  (void)sh;
  for (int64_t dy = 0; dy < dh; ++dy)
    for (int64_t e = 0; e < w; ++e) {
      const int64_t c = e % C, dx = e / C;
      const uint8_t* s0 = src + ((2 * dy) * sw + 2 * dx) * C + c;
      const uint8_t* s1 = s0 + sw * C;
      const int sum = (int)s0[0] + (int)s0[C] + (int)s1[0] + (int)s1[C];
      uint8_t v;
      if (e < vec) {
        v = (uint8_t)((sum + 2) >> 2);
      } else {
        const float r = rintf((float)sum * 0.25f);
        v = (uint8_t)(r > 255.f ? 255.f : r);
      }
      dst[dy * w + e] = v;
    }
}

void orc_lowres_u8(const uint8_t* img, int64_t H, int64_t W, int64_t C, double factor, uint8_t* tmp, uint8_t* out) {
  int64_t nw = (int64_t)(W * factor), nh = (int64_t)(H * factor);
  if (nw < 1) nw = 1;
  if (nh < 1) nh = 1;
  if (W == 2 * nw && H == 2 * nh)  /* cv::resize: scale_x == scale_y == 2 exactly -> fast area path */
    orc_resize_area_fast2_u8(img, H, W, C, tmp, nh, nw);
  else
    orc_resize_area_u8(img, H, W, C, tmp, nh, nw);
  orc_resize_linear_u8(tmp, nh, nw, C, out, H, W);
}

/* cv2.filter2D(src, -1, kernel), 8U -> 8U, direct (non-DFT) path, anchor at the kernel centre,
 * BORDER_REFLECT_101 (BORDER_DEFAULT): the taps are the kernel's non-zero coefficients in row-major
 * order (preprocess2DKernel), each output = saturate_cast<uchar>(sum_t coef_t * src_t) with the sum in
 * f32 starting at delta = 0 (mul and add rounded separately: -ffp-contract=off). taps: ntaps triples
 * (dy, dx, coef) relative to the anchor. */
void orc_filter2d_u8(const uint8_t* img, int64_t H, int64_t W, int64_t C, const float* taps, int ntaps, uint8_t* out) {
  for (int64_t y = 0; y < H; ++y)
    for (int64_t x = 0; x < W; ++x)
      for (int64_t c = 0; c < C; ++c) {
        float s = 0.f;
        for (int k = 0; k < ntaps; ++k) {
          const int64_t yy = refl101(y + (int64_t)taps[3 * k], H), xx = refl101(x + (int64_t)taps[3 * k + 1], W);
          s += taps[3 * k + 2] * (float)img[(yy * W + xx) * C + c];
        }
        float r = rintf(s);
        if (r < 0) r = 0;
        if (r > 255) r = 255;
        out[(y * W + x) * C + c] = (uint8_t)r;
      }
}

/* BORDER_REFLECT: fedcba|abcdefgh|hgfedcb */
static inline int64_t refl(int64_t i, int64_t n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) { if (i < 0) i = -i - 1; if (i >= n) i = 2 * n - 1 - i; }
  return i;
}
void orc_reflect_pad_u8(const uint8_t* src, int64_t H, int64_t W, int64_t C, int64_t ph, int64_t pw, uint8_t* dst) {
  int64_t W2 = W + pw;
  for (int64_t y = 0; y < H + ph; ++y)
    for (int64_t x = 0; x < W2; ++x)
      for (int64_t c = 0; c < C; ++c) dst[(y * W2 + x) * C + c] = src[(refl(y, H) * W + refl(x, W)) * C + c];
}

/* ---- augmentations.py:21-27 _motion_blur_kernel(k, angle) ----------------------------------------
 * kernel = zeros(k, k) f32, row k//2 = 1; M = cv2.getRotationMatrix2D((k/2 - 0.5, k/2 - 0.5), angle, 1);
 * kernel = cv2.warpAffine(kernel, M, (k, k)) (INTER_LINEAR, BORDER_CONSTANT 0); kernel /= kernel.sum() +
 * 1e-8 (numpy 2 scalar rules: all f32). warpAffine restated from OpenCV imgwarp.cpp: M inverted in
 * double, source coordinates in 1/32-pixel fixed point (AB_BITS 10, INTER_BITS 5, round_delta 16),
 * bilinear weights from the f32 table (1-ay)(1-ax), (1-ay)ax, ay(1-ax), ay*ax (remapBilinear, f32
 * sum in tap order), constant-0 border per tap. The sum is numpy's pairwise float32 sum (blocks of 8
 * partial sums for n <= 128). */
static int cv_round(double v) { return (int)lrint(v); }

static float np_pairwise_sum_f32(const float* a, int n) {
  if (n < 8) {
    float r = 0.f;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  float r[8];
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}

void orc_motion_blur_kernel(int k, double angle_deg, float* out /* k*k */) {
  float* src = (float*)calloc((size_t)k * k, sizeof(float));
  for (int x = 0; x < k; ++x) src[(k / 2) * k + x] = 1.f;
  const double cx = k / 2.0 - 0.5, cy = k / 2.0 - 0.5;
  const double ang = angle_deg * 3.14159265358979323846 / 180.0;
  const double alpha = cos(ang), beta = sin(ang);
  double M[6] = {alpha, beta, (1 - alpha) * cx - beta * cy, -beta, alpha, beta * cx + (1 - alpha) * cy};
  double D = M[0] * M[4] - M[1] * M[3];
  D = D != 0 ? 1. / D : 0;
  const double A11 = M[4] * D, A22 = M[0] * D;
  M[0] = A11; M[1] *= -D; M[3] *= -D; M[4] = A22;
  const double b1 = -M[0] * M[2] - M[1] * M[5], b2 = -M[3] * M[2] - M[4] * M[5];
  M[2] = b1; M[5] = b2;
  for (int y = 0; y < k; ++y) {
    const int X0 = cv_round((M[1] * y + M[2]) * 1024) + 16;
    const int Y0 = cv_round((M[4] * y + M[5]) * 1024) + 16;
    for (int x = 0; x < k; ++x) {
      const int X = (X0 + cv_round(M[0] * x * 1024)) >> 5;
      const int Y = (Y0 + cv_round(M[3] * x * 1024)) >> 5;
      const int sx = X >> 5, sy = Y >> 5;
      const float ax = (float)(X & 31) * (1.f / 32), ay = (float)(Y & 31) * (1.f / 32);
      const float w0 = (1.f - ay) * (1.f - ax), w1 = (1.f - ay) * ax, w2 = ay * (1.f - ax), w3 = ay * ax;
      float v;
      if (sx >= k || sx + 1 < 0 || sy >= k || sy + 1 < 0) {
        v = 0.f;
      } else {
        const float v0 = (sx >= 0 && sy >= 0 && sx < k && sy < k) ? src[sy * k + sx] : 0.f;
        const float v1 = (sx + 1 >= 0 && sy >= 0 && sx + 1 < k && sy < k) ? src[sy * k + sx + 1] : 0.f;
        const float v2 = (sx >= 0 && sy + 1 >= 0 && sx < k && sy + 1 < k) ? src[(sy + 1) * k + sx] : 0.f;
        const float v3 = (sx + 1 >= 0 && sy + 1 >= 0 && sx + 1 < k && sy + 1 < k) ? src[(sy + 1) * k + sx + 1] : 0.f;
        v = v0 * w0 + v1 * w1 + v2 * w2 + v3 * w3;
      }
      out[y * k + x] = v;
    }
  }
  const float den = np_pairwise_sum_f32(out, k * k) + 1e-8f;
  for (int i = 0; i < k * k; ++i) out[i] = out[i] / den;
  free(src);
}

/* ---------------------------------------------------------------------------------------------
 * JPEG pixel reconstruction from quantised coefficients, restated from libjpeg-turbo (the decoder
 * behind PIL / cv2.imread) in its own loop structure:
 *   jidctint.c jpeg_idct_islow (6b algorithm: CONST_BITS 13, PASS1_BITS 2, JLONG intermediates, the
 *   post-IDCT range-limit table of jdmaster.c prepare_range_limit_table),
 *   jdsample.c h2v1_fancy_upsample / h2v2_fancy_upsample (context rows replicated at the image
 *   edges, jdmainct.c) and the plain replicating upsamplers when downsampled_width <= 2,
 *   jdcolor.c build_ycc_rgb_table / ycc_rgb_convert.
 * TEST INFRASTRUCTURE: the checker of mx_jpeg_reconstruct, itself checked against PIL's decode.
 * ------------------------------------------------------------------------------------------- */
static unsigned char rl_table[256 * 4 + 256 + 128];  /* sample_range_limit block */
static const unsigned char* sample_range_limit;
static void prep_range_limit(void) {
  if (sample_range_limit) return;
  unsigned char* t = rl_table + 256;
  memset(t - 256, 0, 256);
  for (int i = 0; i <= 255; ++i) t[i] = (unsigned char)i;
  unsigned char* p = t + 128;
  for (int i = 128; i < 512; ++i) p[i] = 255;
  memset(p + 512, 0, 512 - 128);
  memcpy(p + 1024 - 128, t, 128);
  sample_range_limit = t;
}

#define DESCALE(x, n) (((x) + ((int64_t)1 << ((n) - 1))) >> (n))

static void islow(const int16_t* coef, const uint16_t* q, unsigned char* out, int64_t stride) {
  int ws[64];
  const unsigned char* range_limit = sample_range_limit + 128;
  for (int col = 0; col < 8; ++col) {
    const int16_t* in = coef + col;
    const uint16_t* qp = q + col;
    int64_t z1, z2, z3, z4, z5, tmp0, tmp1, tmp2, tmp3, tmp10, tmp11, tmp12, tmp13;
    z2 = (int64_t)in[16] * qp[16];
    z3 = (int64_t)in[48] * qp[48];
    z1 = (z2 + z3) * 4433;
    tmp2 = z1 + z3 * -15137;
    tmp3 = z1 + z2 * 6270;
    z2 = (int64_t)in[0] * qp[0];
    z3 = (int64_t)in[32] * qp[32];
    tmp0 = (z2 + z3) * 8192;
    tmp1 = (z2 - z3) * 8192;
    tmp10 = tmp0 + tmp3; tmp13 = tmp0 - tmp3; tmp11 = tmp1 + tmp2; tmp12 = tmp1 - tmp2;
    tmp0 = (int64_t)in[56] * qp[56];
    tmp1 = (int64_t)in[40] * qp[40];
    tmp2 = (int64_t)in[24] * qp[24];
    tmp3 = (int64_t)in[8] * qp[8];
    z1 = tmp0 + tmp3; z2 = tmp1 + tmp2; z3 = tmp0 + tmp2; z4 = tmp1 + tmp3;
    z5 = (z3 + z4) * 9633;
    tmp0 *= 2446; tmp1 *= 16819; tmp2 *= 25172; tmp3 *= 12299;
    z1 *= -7373; z2 *= -20995; z3 *= -16069; z4 *= -3196;
    z3 += z5; z4 += z5;
    tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
    ws[col] = (int)DESCALE(tmp10 + tmp3, 11);
    ws[56 + col] = (int)DESCALE(tmp10 - tmp3, 11);
    ws[8 + col] = (int)DESCALE(tmp11 + tmp2, 11);
    ws[48 + col] = (int)DESCALE(tmp11 - tmp2, 11);
    ws[16 + col] = (int)DESCALE(tmp12 + tmp1, 11);
    ws[40 + col] = (int)DESCALE(tmp12 - tmp1, 11);
    ws[24 + col] = (int)DESCALE(tmp13 + tmp0, 11);
    ws[32 + col] = (int)DESCALE(tmp13 - tmp0, 11);
  }
  for (int row = 0; row < 8; ++row) {
    const int* w = ws + row * 8;
    unsigned char* o = out + row * stride;
    int64_t z1, z2, z3, z4, z5, tmp0, tmp1, tmp2, tmp3, tmp10, tmp11, tmp12, tmp13;
    z2 = w[2]; z3 = w[6];
    z1 = (z2 + z3) * 4433;
    tmp2 = z1 + z3 * -15137;
    tmp3 = z1 + z2 * 6270;
    tmp0 = ((int64_t)w[0] + w[4]) * 8192;
    tmp1 = ((int64_t)w[0] - w[4]) * 8192;
    tmp10 = tmp0 + tmp3; tmp13 = tmp0 - tmp3; tmp11 = tmp1 + tmp2; tmp12 = tmp1 - tmp2;
    tmp0 = w[7]; tmp1 = w[5]; tmp2 = w[3]; tmp3 = w[1];
    z1 = tmp0 + tmp3; z2 = tmp1 + tmp2; z3 = tmp0 + tmp2; z4 = tmp1 + tmp3;
    z5 = (z3 + z4) * 9633;
    tmp0 *= 2446; tmp1 *= 16819; tmp2 *= 25172; tmp3 *= 12299;
    z1 *= -7373; z2 *= -20995; z3 *= -16069; z4 *= -3196;
    z3 += z5; z4 += z5;
    tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
    o[0] = range_limit[(int)DESCALE(tmp10 + tmp3, 18) & 1023];
    o[7] = range_limit[(int)DESCALE(tmp10 - tmp3, 18) & 1023];
    o[1] = range_limit[(int)DESCALE(tmp11 + tmp2, 18) & 1023];
    o[6] = range_limit[(int)DESCALE(tmp11 - tmp2, 18) & 1023];
    o[2] = range_limit[(int)DESCALE(tmp12 + tmp1, 18) & 1023];
    o[5] = range_limit[(int)DESCALE(tmp12 - tmp1, 18) & 1023];
    o[3] = range_limit[(int)DESCALE(tmp13 + tmp0, 18) & 1023];
    o[4] = range_limit[(int)DESCALE(tmp13 - tmp0, 18) & 1023];
  }
}

/* one upsampled chroma row (output width 2*dw or dw) from sample rows `in0` (nearer) / `in1` */
static void up_h2v1(const unsigned char* in, int dw, unsigned char* o) {
  if (dw <= 2) { for (int c = 0; c < dw; ++c) o[2 * c] = o[2 * c + 1] = in[c]; return; }
  int v = in[0];
  o[0] = (unsigned char)v;
  o[1] = (unsigned char)((v * 3 + in[1] + 2) >> 2);
  for (int c = 1; c < dw - 1; ++c) {
    v = in[c] * 3;
    o[2 * c] = (unsigned char)((v + in[c - 1] + 1) >> 2);
    o[2 * c + 1] = (unsigned char)((v + in[c + 1] + 2) >> 2);
  }
  v = in[dw - 1];
  o[2 * dw - 2] = (unsigned char)((v * 3 + in[dw - 2] + 1) >> 2);
  o[2 * dw - 1] = (unsigned char)v;
}

static void up_h2v2_row(const unsigned char* in0, const unsigned char* in1, int dw, unsigned char* o) {
  if (dw <= 2) { for (int c = 0; c < dw; ++c) o[2 * c] = o[2 * c + 1] = in0[c]; return; }
  int this_ = in0[0] * 3 + in1[0], next = in0[1] * 3 + in1[1], last;
  o[0] = (unsigned char)((this_ * 4 + 8) >> 4);
  o[1] = (unsigned char)((this_ * 3 + next + 7) >> 4);
  last = this_; this_ = next;
  int k = 2;
  for (int c = 2; c < dw; ++c) {
    next = in0[c] * 3 + in1[c];
    o[k++] = (unsigned char)((this_ * 3 + last + 8) >> 4);
    o[k++] = (unsigned char)((this_ * 3 + next + 7) >> 4);
    last = this_; this_ = next;
  }
  o[k++] = (unsigned char)((this_ * 3 + last + 8) >> 4);
  o[k++] = (unsigned char)((this_ * 4 + 7) >> 4);
}

int orc_jpeg_reconstruct(const int16_t* coefs, const mx_jpeg_info* info, unsigned char* out, int bgr) {
  prep_range_limit();
  const int W = info->width, H = info->height, nc = info->ncomp;
  unsigned char* plane[3] = {0, 0, 0};
  for (int c = 0; c < nc; ++c) {
    const int64_t stride = (int64_t)info->bw[c] * 8;
    plane[c] = (unsigned char*)malloc((size_t)stride * info->bh[c] * 8);
    if (!plane[c]) return -1;
    for (int by = 0; by < info->bh[c]; ++by)
      for (int bx = 0; bx < info->bw[c]; ++bx)
        islow(coefs + info->coef_off[c] + ((int64_t)by * info->bw[c] + bx) * 64, info->qt[info->tq[c]],
              plane[c] + (int64_t)by * 8 * stride + bx * 8, stride);
  }
  /* colour tables (jdcolor.c) */
  int crr[256], cbb[256], crg[256], cbg[256];
  for (int i = 0; i < 256; ++i) {
    const int x = i - 128;
    crr[i] = (91881 * x + 32768) >> 16;
    cbb[i] = (116130 * x + 32768) >> 16;
    crg[i] = -46802 * x;
    cbg[i] = -22554 * x + 32768;
  }
  const unsigned char* lim = sample_range_limit;
  unsigned char* up[3] = {0, 0, 0};
  for (int c = 1; c < nc; ++c) up[c] = (unsigned char*)malloc((size_t)2 * info->dw[c] + 16);
  for (int y = 0; y < H; ++y) {
    const unsigned char* Y = plane[0] + (int64_t)y * info->bw[0] * 8;
    const unsigned char* cb = 0;
    const unsigned char* cr = 0;
    for (int c = 1; c < nc; ++c) {
      const int hs = info->hmax / info->h[c], vs = info->vmax / info->v[c];
      const int64_t st = (int64_t)info->bw[c] * 8;
      const unsigned char* src;
      if (hs == 1 && vs == 1) {
        src = plane[c] + (int64_t)y * st;
      } else if (vs == 1) {
        up_h2v1(plane[c] + (int64_t)y * st, info->dw[c], up[c]);
        src = up[c];
      } else {
        const int r0 = y >> 1;
        int r1 = (y & 1) ? r0 + 1 : r0 - 1;
        if (r1 < 0) r1 = 0;
        if (r1 > info->dh[c] - 1) r1 = info->dh[c] - 1;
        if (info->dw[c] <= 2) r1 = r0;
        up_h2v2_row(plane[c] + (int64_t)r0 * st, plane[c] + (int64_t)r1 * st, info->dw[c], up[c]);
        src = up[c];
      }
      if (c == 1) cb = src; else cr = src;
    }
    for (int x = 0; x < W; ++x) {
      unsigned char* o = out + ((int64_t)y * W + x) * 3;
      const int yy = Y[x];
      int R, G, B;
      if (nc == 1) {
        R = G = B = yy;
      } else {
        R = lim[yy + crr[cr[x]]];
        G = lim[yy + ((cbg[cb[x]] + crg[cr[x]]) >> 16)];
        B = lim[yy + cbb[cb[x]]];
      }
      o[0] = (unsigned char)(bgr ? B : R);
      o[1] = (unsigned char)G;
      o[2] = (unsigned char)(bgr ? R : B);
    }
  }
  for (int c = 0; c < 3; ++c) { free(plane[c]); free(up[c]); }
  return 0;
}

/* GeneralizedRCNNTransform resize (torchvision 0.20.1 transform.py _resize_image_and_masks ->
 * F.interpolate(scale_factor=s, mode="bilinear", align_corners=False, recompute_scale_factor=True)),
 * on the ToDtype(scale=True) + normalize output, restating torch's CUDA upsample_bilinear2d_out_frame
 * (aten/src/ATen/native/cuda/UpSampleBilinear2d.cu; area_pixel_compute_scale / _source_index in
 * UpSample.h) in float, one rounding per op: scale = (float)in / out; src = scale * (dst + 0.5) - 0.5,
 * clamped at 0; i0 = (int)src; i1 = i0 + (i0 < in - 1); l1 = src - i0; l0 = 1 - l1;
 * v = h0 * (w0 * v00 + w1 * v01) + h1 * (w0 * v10 + w1 * v11). img u8 [H][W][3] -> out f32 [nh][nw][3]. */
static inline float rz_src(float scale, int64_t dst) {
  float s = scale * ((float)dst + 0.5f) - 0.5f;
  return s < 0.f ? 0.f : s;
}
void orc_resize_normalize(const uint8_t* img, int64_t H, int64_t W, int64_t nh, int64_t nw, const float* mean,
                          const float* stdv, float* out) {
  const float sh = (float)H / (float)nh, sw = (float)W / (float)nw;
  const float inv = (float)(1.0 / 255.0);
  for (int64_t y = 0; y < nh; ++y) {
    const float hr = rz_src(sh, y);
    const int64_t h0 = (int64_t)hr, h1 = h0 + (h0 < H - 1 ? 1 : 0);
    const float hl1 = hr - (float)h0, hl0 = 1.f - hl1;
    for (int64_t x = 0; x < nw; ++x) {
      const float wr = rz_src(sw, x);
      const int64_t w0 = (int64_t)wr, w1 = w0 + (w0 < W - 1 ? 1 : 0);
      const float wl1 = wr - (float)w0, wl0 = 1.f - wl1;
      for (int c = 0; c < 3; ++c) {
        const float a = ((float)img[(h0 * W + w0) * 3 + c] * inv - mean[c]) / stdv[c];
        const float b = ((float)img[(h0 * W + w1) * 3 + c] * inv - mean[c]) / stdv[c];
        const float d0 = ((float)img[(h1 * W + w0) * 3 + c] * inv - mean[c]) / stdv[c];
        const float d1 = ((float)img[(h1 * W + w1) * 3 + c] * inv - mean[c]) / stdv[c];
        out[(y * nw + x) * 3 + c] = hl0 * (wl0 * a + wl1 * b) + hl1 * (wl0 * d0 + wl1 * d1);
      }
    }
  }
}
