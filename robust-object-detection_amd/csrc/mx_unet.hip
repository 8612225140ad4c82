// mx_unet.hip — device-side pieces of the restoration pre-pass (gfx950).
//
// Reference: scripts/restore_testsets.py:53-79 restore_image + scripts/restoration_net.py:44-106.
//   reflect_pad:  cv2.copyMakeBorder(img, 0, ph, 0, pw, BORDER_REFLECT) (fedcba|abcdefgh|hgfedcb)
//   up_concat:    ConvTranspose2d(k=2, s=2) output, computed as a 1x1 conv with 4*Cout channels
//                 ordered (i, j, co), scattered to (2h+i, 2w+j) and concatenated with the skip map
//                 along channels (torch.cat([x, skip], dim=1), restoration_net.py:56)
//   restore_finish: clamp(x + residual, 0, 1) (restoration_net.py:105-106) with x = u8/255.0f, then
//                 *255.0, clip, truncation to uint8 and the crop back to (H, W) (restore_testsets.py:71-77)
#include "mx_common.h"

namespace mx {

__device__ __forceinline__ int64_t reflect(int64_t i, int64_t n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) {
    if (i < 0) i = -i - 1;
    if (i >= n) i = 2 * n - 1 - i;
  }
  return i;
}

__global__ void reflect_pad_kernel(const uint8_t* __restrict__ src, int64_t B, int64_t H, int64_t W, int64_t C, int64_t Hp,
                                   int64_t Wp, uint8_t* __restrict__ dst) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * Hp * Wp * C) return;
  int64_t c = i % C, x = (i / C) % Wp, y = (i / (C * Wp)) % Hp, b = i / (C * Wp * Hp);
  dst[i] = src[((b * H + reflect(y, H)) * W + reflect(x, W)) * C + c];
}

// up [N,H,W,4*Cu] (i,j,co) + skip [N,2H,2W,Cs] -> out [N,2H,2W,Cu+Cs]; 8 channels per thread (a copy:
// bf16 or f32 storage, 16 or 32 B per thread)
template <typename T>
__global__ void up_concat_kernel(const T* __restrict__ up, const T* __restrict__ skip, int64_t N, int64_t H,
                                 int64_t W, int64_t Cu, int64_t Cs, T* __restrict__ out) {
  const int64_t Co = Cu + Cs, C8 = Co / 8;
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N * 2 * H * 2 * W * C8) return;
  int64_t c0 = (e % C8) * 8, p = e / C8;
  int64_t x = p % (2 * W), y = (p / (2 * W)) % (2 * H), n = p / (4 * H * W);
  const T* src;
  if (c0 < Cu) {
    int64_t q = (y & 1) * 2 + (x & 1);
    src = up + ((n * H + (y >> 1)) * W + (x >> 1)) * 4 * Cu + q * Cu + c0;
  } else {
    src = skip + p * Cs + (c0 - Cu);
  }
  constexpr int V = sizeof(T) / 2;  // 16-B vectors per 8 elements
#pragma unroll
  for (int i = 0; i < V; ++i) ((uint4*)(out + p * Co + c0))[i] = ((const uint4*)src)[i];
}

// Backward of up_concat (U-Net training, train_restoration.py:199-205): gcat [N,2H,2W,Cu+Cs] ->
// gup [N,H,W,4*Cu] (the same (i, j, co) channel order: the gradient of the 1x1 conv's output) and
// gskip [N,2H,2W,Cs]. Every element of gcat is read once and written to exactly one place (8 channels
// per thread, 16/32-B vectors).
template <typename T>
__global__ void up_concat_bwd_kernel(const T* __restrict__ g, int64_t N, int64_t H, int64_t W, int64_t Cu, int64_t Cs,
                                     T* __restrict__ gup, T* __restrict__ gskip) {
  const int64_t Co = Cu + Cs, C8 = Co / 8;
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N * 2 * H * 2 * W * C8) return;
  int64_t c0 = (e % C8) * 8, p = e / C8;
  int64_t x = p % (2 * W), y = (p / (2 * W)) % (2 * H), n = p / (4 * H * W);
  T* dst;
  if (c0 < Cu) {
    int64_t q = (y & 1) * 2 + (x & 1);
    dst = gup + ((n * H + (y >> 1)) * W + (x >> 1)) * 4 * Cu + q * Cu + c0;
  } else {
    if (gskip == nullptr) return;
    dst = gskip + p * Cs + (c0 - Cu);
  }
  constexpr int V = sizeof(T) / 2;
#pragma unroll
  for (int i = 0; i < V; ++i) ((uint4*)dst)[i] = ((const uint4*)(g + p * Co + c0))[i];
}

__global__ void restore_finish_kernel(const uint8_t* __restrict__ img, int64_t B, int64_t Hp, int64_t Wp, const float* __restrict__ res,
                                      int64_t H, int64_t W, uint8_t* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * H * W * 3) return;
  int64_t c = i % 3, x = (i / 3) % W, y = (i / (3 * W)) % H, b = i / (3 * W * H);
  int64_t pi = ((b * Hp + y) * Wp + x) * 3 + c;
  float v = (float)img[pi] / 255.0f + res[pi];
  v = v < 0.f ? 0.f : (v > 1.f ? 1.f : v);
  v = v * 255.0f;
  v = v < 0.f ? 0.f : (v > 255.f ? 255.f : v);
  out[i] = (uint8_t)v;
}

}  // namespace mx

using namespace mx;

extern "C" int mx_reflect_pad_u8(const uint8_t* src, int64_t B, int64_t H, int64_t W, int64_t C, int64_t Hp, int64_t Wp,
                                 uint8_t* dst, mx_stream_t stream) {
  MX_CHECK_ARG(Hp >= H && Wp >= W && H > 0 && W > 0, "reflect_pad: bad sizes");
  int64_t n = B * Hp * Wp * C;
  if (n == 0) return MX_OK;
  reflect_pad_kernel<<<(unsigned)cdiv(n, 256), 256, 0, (hipStream_t)stream>>>(src, B, H, W, C, Hp, Wp, dst);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

template <typename T>
static void up_concat_launch(const void* up, const void* skip, int64_t N, int64_t H, int64_t W, int64_t Cu, int64_t Cs,
                             void* out, int64_t n, hipStream_t s) {
  up_concat_kernel<T><<<(unsigned)cdiv(n, 256), 256, 0, s>>>((const T*)up, (const T*)skip, N, H, W, Cu, Cs, (T*)out);
}

extern "C" int mx_up_concat(const void* up, const void* skip, int dtype, int64_t N, int64_t H, int64_t W, int64_t Cu,
                            int64_t Cs, void* out, mx_stream_t stream) {
  MX_CHECK_ARG(Cu % 8 == 0 && Cs % 8 == 0, "up_concat: channel counts must be multiples of 8");
  int64_t n = N * 4 * H * W * ((Cu + Cs) / 8);
  if (n == 0) return MX_OK;
  MX_DT_DISPATCH(dtype, up_concat_launch, up, skip, N, H, W, Cu, Cs, out, n, (hipStream_t)stream);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

template <typename T>
static void up_concat_bwd_launch(const void* g, int64_t N, int64_t H, int64_t W, int64_t Cu, int64_t Cs, void* gup,
                                 void* gskip, int64_t n, hipStream_t s) {
  up_concat_bwd_kernel<T><<<(unsigned)cdiv(n, 256), 256, 0, s>>>((const T*)g, N, H, W, Cu, Cs, (T*)gup, (T*)gskip);
}

extern "C" int mx_up_concat_bwd(const void* gcat, int dtype, int64_t N, int64_t H, int64_t W, int64_t Cu, int64_t Cs,
                                void* gup, void* gskip, mx_stream_t stream) {
  MX_CHECK_ARG(Cu % 8 == 0 && Cs % 8 == 0, "up_concat_bwd: channel counts must be multiples of 8");
  MX_CHECK_ARG(gup != nullptr, "up_concat_bwd: gup is required");
  int64_t n = N * 4 * H * W * ((Cu + Cs) / 8);
  if (n == 0) return MX_OK;
  MX_DT_DISPATCH(dtype, up_concat_bwd_launch, gcat, N, H, W, Cu, Cs, gup, gskip, n, (hipStream_t)stream);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_restore_finish(const uint8_t* img_padded, int64_t B, int64_t Hp, int64_t Wp, const float* residual, int64_t H,
                                 int64_t W, uint8_t* out, mx_stream_t stream) {
  MX_CHECK_ARG(Hp >= H && Wp >= W, "restore_finish: bad sizes");
  int64_t n = B * H * W * 3;
  if (n == 0) return MX_OK;
  restore_finish_kernel<<<(unsigned)cdiv(n, 256), 256, 0, (hipStream_t)stream>>>(img_padded, B, Hp, Wp, residual, H, W, out);
  MX_LAUNCH_CHECK();
  return MX_OK;
}
