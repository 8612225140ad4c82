// mx_jpeg.hip — device half of the hybrid baseline-JPEG decoder (host half: mx_jpeg.cpp).
//
// Reproduces libjpeg-turbo's default decompression (the decoder behind PIL and cv2.imread,
// coco_detection_dataset.py:23, restore_testsets.py:99) bit for bit:
//   idct_kernel      dequantisation + jpeg_idct_islow (jidctint.c: CONST_BITS 13, PASS1_BITS 2, 64-bit
//                    intermediates like JLONG, the post-IDCT range-limit table of jdmaster.c
//                    prepare_range_limit_table indexed by x & 1023), one thread per 8x8 block, written
//                    into MCU-padded component planes;
//   colour_kernel    per output pixel: chroma "fancy" upsampling (jdsample.c h2v1_fancy_upsample /
//                    h2v2_fancy_upsample: triangle filter, rows beyond the image replicated like
//                    jdmainct.c's context rows; plain replication when downsampled_width <= 2) and
//                    ycc_rgb_convert (jdcolor.c tables, SCALEBITS 16), grey replicated to RGB.
// Both are integer kernels (no float anywhere), HBM-bound streaming work.
#include "mx_common.h"

namespace mx {

struct JpegDev {
  int32_t width, height, ncomp;
  int32_t h[3], v[3], tq[3];
  int32_t hmax, vmax;
  int32_t bw[3], bh[3], dw[3], dh[3];
  int64_t coef_off[3], plane_off[3];
  int64_t nblocks[3];
  uint16_t qt[4][64];
};

// post-IDCT range limit (jdmaster.c prepare_range_limit_table, idct table = sample_range_limit +
// CENTERJSAMPLE): x & 1023 -> [0,128): x+128, [128,512): 255, [512,896): 0, [896,1024): x-896
__device__ __forceinline__ uint8_t idct_limit(int64_t x) {
  const int i = (int)(x & 1023);
  return i < 128 ? (uint8_t)(i + 128) : (i < 512 ? 255 : (i < 896 ? 0 : (uint8_t)(i - 896)));
}

#define FIX_0_298631336 2446
#define FIX_0_390180644 3196
#define FIX_0_541196100 4433
#define FIX_0_765366865 6270
#define FIX_0_899976223 7373
#define FIX_1_175875602 9633
#define FIX_1_501321110 12299
#define FIX_1_847759065 15137
#define FIX_1_961570560 16069
#define FIX_2_053119869 16819
#define FIX_2_562915447 20995
#define FIX_3_072711026 25172

__device__ __forceinline__ int64_t descale(int64_t x, int n) { return (x + ((int64_t)1 << (n - 1))) >> n; }

// one 1-D islow pass over in[0..7] (stride-free), CONST_BITS 13; returns the 8 outputs before the
// final descale (shared by both passes)
__device__ __forceinline__ void idct8(const int64_t* in, int64_t* o) {
  int64_t z2 = in[2], z3 = in[6];
  int64_t z1 = (z2 + z3) * FIX_0_541196100;
  const int64_t tmp2e = z1 + z3 * (-FIX_1_847759065);
  const int64_t tmp3e = z1 + z2 * FIX_0_765366865;
  const int64_t tmp0e = (in[0] + in[4]) * 8192;
  const int64_t tmp1e = (in[0] - in[4]) * 8192;
  const int64_t tmp10 = tmp0e + tmp3e, tmp13 = tmp0e - tmp3e, tmp11 = tmp1e + tmp2e, tmp12 = tmp1e - tmp2e;
  int64_t tmp0 = in[7], tmp1 = in[5], tmp2 = in[3], tmp3 = in[1];
  z1 = tmp0 + tmp3;
  z2 = tmp1 + tmp2;
  z3 = tmp0 + tmp2;
  int64_t z4 = tmp1 + tmp3;
  const int64_t z5 = (z3 + z4) * FIX_1_175875602;
  tmp0 = tmp0 * FIX_0_298631336;
  tmp1 = tmp1 * FIX_2_053119869;
  tmp2 = tmp2 * FIX_3_072711026;
  tmp3 = tmp3 * FIX_1_501321110;
  z1 = z1 * (-FIX_0_899976223);
  z2 = z2 * (-FIX_2_562915447);
  z3 = z3 * (-FIX_1_961570560);
  z4 = z4 * (-FIX_0_390180644);
  z3 += z5;
  z4 += z5;
  tmp0 += z1 + z3;
  tmp1 += z2 + z4;
  tmp2 += z2 + z3;
  tmp3 += z1 + z4;
  o[0] = tmp10 + tmp3;
  o[7] = tmp10 - tmp3;
  o[1] = tmp11 + tmp2;
  o[6] = tmp11 - tmp2;
  o[2] = tmp12 + tmp1;
  o[5] = tmp12 - tmp1;
  o[3] = tmp13 + tmp0;
  o[4] = tmp13 - tmp0;
}

__global__ void __launch_bounds__(256) jpeg_idct_kernel(const int16_t* __restrict__ coefs, JpegDev j,
                                                        uint8_t* __restrict__ planes) {
  int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int c = 0;
  while (c < j.ncomp && b >= j.nblocks[c]) b -= j.nblocks[c++];
  if (c >= j.ncomp) return;
  const int16_t* src = coefs + j.coef_off[c] + b * 64;
  const uint16_t* q = j.qt[j.tq[c]];
  int16_t cf[64];
#pragma unroll
  for (int i = 0; i < 8; ++i) *(uint4*)&cf[8 * i] = ((const uint4*)src)[i];
  int64_t ws[64];
  // pass 1: columns (DEQUANTIZE = coef * q), outputs descaled by CONST_BITS - PASS1_BITS
#pragma unroll
  for (int col = 0; col < 8; ++col) {
    int64_t in[8], o[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) in[r] = (int64_t)cf[r * 8 + col] * q[r * 8 + col];
    idct8(in, o);
#pragma unroll
    for (int r = 0; r < 8; ++r) ws[r * 8 + col] = (int64_t)(int32_t)descale(o[r], 11);
  }
  const int64_t by = b / j.bw[c], bx = b % j.bw[c];
  const int64_t stride = (int64_t)j.bw[c] * 8;
  uint8_t* dst = planes + j.plane_off[c] + by * 8 * stride + bx * 8;
  // pass 2: rows, descaled by CONST_BITS + PASS1_BITS + 3, range-limited
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    int64_t o[8];
    idct8(&ws[r * 8], o);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      lo |= (uint32_t)idct_limit(descale(o[t], 18)) << (8 * t);
      hi |= (uint32_t)idct_limit(descale(o[t + 4], 18)) << (8 * t);
    }
    *(uint2*)(dst + r * stride) = make_uint2(lo, hi);
  }
}

__device__ __forceinline__ int clamp255(int x) { return x < 0 ? 0 : (x > 255 ? 255 : x); }

// upsampled chroma sample at output (x, y) of component c (jdsample.c)
__device__ __forceinline__ int chroma(const uint8_t* pl, int64_t stride, int hs, int vs, int dw, int dh, int x, int y) {
  if (hs == 1 && vs == 1) return pl[(int64_t)y * stride + x];
  const bool fancy = dw > 2;
  if (!fancy) return pl[(int64_t)(y / vs) * stride + x / hs];  // h2v1_upsample / h2v2_upsample: replicate
  const int cx = x >> 1;
  if (vs == 1) {  // h2v1 fancy
    const uint8_t* row = pl + (int64_t)y * stride;
    const int v0 = row[cx];
    if ((x & 1) == 0) return cx == 0 ? v0 : (v0 * 3 + row[cx - 1] + 1) >> 2;
    return cx == dw - 1 ? v0 : (v0 * 3 + row[cx + 1] + 2) >> 2;
  }
  // h2v2 fancy: the nearer sample row (3/4) and the other row (1/4), rows clamped to the image
  const int r0 = y >> 1;
  int r1 = (y & 1) ? r0 + 1 : r0 - 1;
  r1 = r1 < 0 ? 0 : (r1 > dh - 1 ? dh - 1 : r1);
  const uint8_t* a = pl + (int64_t)r0 * stride;
  const uint8_t* b = pl + (int64_t)r1 * stride;
  const int cs = a[cx] * 3 + b[cx];
  if ((x & 1) == 0) {
    if (cx == 0) return (cs * 4 + 8) >> 4;
    return (cs * 3 + a[cx - 1] * 3 + b[cx - 1] + 8) >> 4;
  }
  if (cx == dw - 1) return (cs * 4 + 7) >> 4;
  return (cs * 3 + a[cx + 1] * 3 + b[cx + 1] + 7) >> 4;
}

__global__ void __launch_bounds__(256) jpeg_colour_kernel(const uint8_t* __restrict__ planes, JpegDev j, int bgr,
                                                          uint8_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)j.width * j.height) return;
  const int x = (int)(i % j.width), y = (int)(i / j.width);
  const int Y = planes[j.plane_off[0] + (int64_t)y * j.bw[0] * 8 + x];
  int R, G, B;
  if (j.ncomp == 1) {
    R = G = B = Y;
  } else {
    const int hs = j.hmax / j.h[1], vs = j.vmax / j.v[1];  // chroma components share one sampling
    const int cb = chroma(planes + j.plane_off[1], (int64_t)j.bw[1] * 8, hs, vs, j.dw[1], j.dh[1], x, y);
    const int cr = chroma(planes + j.plane_off[2], (int64_t)j.bw[2] * 8, hs, vs, j.dw[2], j.dh[2], x, y);
    // jdcolor.c build_ycc_rgb_table (FIX(x) = (int)(x * 65536 + 0.5), ONE_HALF = 1 << 15)
    const int xcr = cr - 128, xcb = cb - 128;
    const int crr = (91881 * xcr + 32768) >> 16;
    const int cbb = (116130 * xcb + 32768) >> 16;
    const int g = (-46802 * xcr + (-22554 * xcb + 32768)) >> 16;
    R = clamp255(Y + crr);
    G = clamp255(Y + g);
    B = clamp255(Y + cbb);
  }
  uint8_t* o = out + i * 3;
  o[0] = (uint8_t)(bgr ? B : R);
  o[1] = (uint8_t)G;
  o[2] = (uint8_t)(bgr ? R : B);
}

static void to_dev(const mx_jpeg_info* in, JpegDev* j, int64_t* plane_bytes) {
  j->width = in->width;
  j->height = in->height;
  j->ncomp = in->ncomp;
  j->hmax = in->hmax;
  j->vmax = in->vmax;
  int64_t off = 0;
  for (int c = 0; c < 3; ++c) {
    const bool on = c < in->ncomp;
    j->h[c] = on ? in->h[c] : 1;
    j->v[c] = on ? in->v[c] : 1;
    j->tq[c] = on ? in->tq[c] : 0;
    j->bw[c] = on ? in->bw[c] : 0;
    j->bh[c] = on ? in->bh[c] : 0;
    j->dw[c] = on ? in->dw[c] : 0;
    j->dh[c] = on ? in->dh[c] : 0;
    j->coef_off[c] = on ? in->coef_off[c] : 0;
    j->nblocks[c] = on ? (int64_t)in->bw[c] * in->bh[c] : 0;
    j->plane_off[c] = off;
    off += j->nblocks[c] * 64;
  }
  for (int t = 0; t < 4; ++t)
    for (int k = 0; k < 64; ++k) j->qt[t][k] = in->qt[t][k];
  *plane_bytes = off;
}

}  // namespace mx

using namespace mx;

extern "C" size_t mx_jpeg_workspace(const mx_jpeg_info* info) {
  if (!info) return 0;
  JpegDev j;
  int64_t bytes = 0;
  to_dev(info, &j, &bytes);
  return (size_t)bytes;
}

extern "C" int mx_jpeg_reconstruct(const int16_t* coefs, const mx_jpeg_info* info, void* ws, size_t ws_bytes,
                                   uint8_t* out, int bgr, mx_stream_t stream) {
  MX_CHECK_ARG(coefs && info && out, "jpeg_reconstruct: null argument");
  MX_CHECK_ARG(info->ncomp == 1 || info->ncomp == 3, "jpeg_reconstruct: 1 or 3 components");
  MX_CHECK_ARG(info->width > 0 && info->height > 0 && info->coef_total > 0, "jpeg_reconstruct: parse the image first");
  JpegDev j;
  int64_t need = 0;
  to_dev(info, &j, &need);
  MX_CHECK_ARG(ws && (int64_t)ws_bytes >= need, "jpeg_reconstruct: workspace of %lld bytes required", (long long)need);
  const int64_t nb = j.nblocks[0] + j.nblocks[1] + j.nblocks[2];
  hipStream_t st = (hipStream_t)stream;
  jpeg_idct_kernel<<<(unsigned)cdiv(nb, 256), 256, 0, st>>>(coefs, j, (uint8_t*)ws);
  MX_LAUNCH_CHECK();
  const int64_t np = (int64_t)j.width * j.height;
  jpeg_colour_kernel<<<(unsigned)cdiv(np, 256), 256, 0, st>>>((const uint8_t*)ws, j, bgr, out);
  MX_LAUNCH_CHECK();
  return MX_OK;
}
