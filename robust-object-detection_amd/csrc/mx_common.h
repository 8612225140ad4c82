// mx_common.h — shared helpers for the libmx_det HIP kernels (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/mx_det.h"

namespace mx {

void set_error(const char* fmt, ...);

#define MX_CHECK_ARG(cond, ...)            \
  do {                                     \
    if (!(cond)) {                         \
      ::mx::set_error(__VA_ARGS__);        \
      return MX_EINVAL;                    \
    }                                      \
  } while (0)

#define MX_HIP(call)                                                              \
  do {                                                                            \
    hipError_t e_ = (call);                                                       \
    if (e_ != hipSuccess) {                                                       \
      ::mx::set_error("%s:%d %s: %s", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
      return MX_EHIP;                                                             \
    }                                                                             \
  } while (0)

#define MX_LAUNCH_CHECK() MX_HIP(hipGetLastError())

// bf16 helpers (bit-level; round-to-nearest-even like v_cvt_pk_bf16_f32)
// XCD-aware bijective remap of a linear block id (cdna_hip_programming.md §5 / T1): the blocks one
// XCD receives (id % 8) get one contiguous run of work indices, in dispatch order
__device__ __forceinline__ int64_t xcd_remap(int64_t id, int64_t nwg) {
  if (nwg < 8) return id;
  int64_t q = nwg / 8, r = nwg % 8, xcd = id % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + id / 8;
}

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

template <typename T> struct io;
template <> struct io<float> {
  static __device__ __forceinline__ float ld(const float* p) { return *p; }
  static __device__ __forceinline__ void st(float* p, float v) { *p = v; }
};
template <> struct io<uint16_t> {
  static __device__ __forceinline__ float ld(const uint16_t* p) { return bf2f(*p); }
  static __device__ __forceinline__ void st(uint16_t* p, float v) { *p = f2bf(v); }
};

// 8 consecutive activation elements of storage type T (bf16 bits or f32) <-> float[8]: one 16-B
// access for bf16, two for f32 (NHWC rows are 8-element aligned everywhere: C % 8 == 0)
template <typename T>
__device__ __forceinline__ void ld8(const T* p, float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    const uint4 u = *(const uint4*)p;
    const uint16_t* h = (const uint16_t*)&u;
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = bf2f(h[q]);
  } else {
    *(float4*)&v[0] = *(const float4*)p;
    *(float4*)&v[4] = *(const float4*)(p + 4);
  }
}
template <typename T>
__device__ __forceinline__ void st8(T* p, const float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    uint4 u;
    uint16_t* h = (uint16_t*)&u;
#pragma unroll
    for (int q = 0; q < 8; ++q) h[q] = f2bf(v[q]);
    *(uint4*)p = u;
  } else {
    *(float4*)p = *(const float4*)&v[0];
    *(float4*)(p + 4) = *(const float4*)&v[4];
  }
}
// storage element as stored (no rounding when T is f32)
template <typename T>
__device__ __forceinline__ float ld1(const T* p) {
  if constexpr (sizeof(T) == 2) return bf2f(*p);
  else return *p;
}
template <typename T>
__device__ __forceinline__ void st1(T* p, float v) {
  if constexpr (sizeof(T) == 2) *p = f2bf(v);
  else *p = v;
}

// bf16x3 split of f32 operands (precision-faithful conv mode): x = hi + lo + O(2^-17 |x|), hi = RNE
// bf16(x), lo = RNE bf16(x - hi); products hi*hi + hi*lo + lo*hi in f32 accumulation differ from the
// f32 product by O(2^-16) relative (TF32 rounds each operand to 2^-11). One v_cvt_pk_bf16_f32 per
// pair and plane.
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  typedef float f2_t __attribute__((ext_vector_type(2)));
  typedef __bf16 b2_t __attribute__((ext_vector_type(2)));
  const b2_t r = __builtin_convertvector((f2_t){a, b}, b2_t);
  return __builtin_bit_cast(uint32_t, r);
}
// scalar v_sub_f32: plain `a - b` pairs get SLP-packed into v_pk_add_f32, which costs ~13 extra
// cycles per instruction beside MFMAs (MI355X_MICROARCH.md, filler prices)
__device__ __forceinline__ float sub_f32(float a, float b) {
  float r;
  asm("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ void split2(float a, float b, uint32_t& hi, uint32_t& lo) {
  hi = pk_bf16(a, b);
  const float ha = __uint_as_float(hi << 16), hb = __uint_as_float(hi & 0xffff0000u);
  lo = pk_bf16(sub_f32(a, ha), sub_f32(b, hb));
}
// 8 f32 -> 8 bf16 hi (16 B) + 8 bf16 lo (16 B)
__device__ __forceinline__ void split8(const float4 a, const float4 b, uint4& hi, uint4& lo) {
  split2(a.x, a.y, hi.x, lo.x);
  split2(a.z, a.w, hi.y, lo.y);
  split2(b.x, b.y, hi.z, lo.z);
  split2(b.z, b.w, hi.w, lo.w);
}

// host: call F<uint16_t> (MX_BF16) or F<float> (MX_F32) with the arguments; other codes -> MX_EINVAL
#define MX_DT_DISPATCH(dt, F, ...)                                   \
  do {                                                              \
    MX_CHECK_ARG((dt) == MX_BF16 || (dt) == MX_F32, "bad dtype %d", (int)(dt)); \
    if ((dt) == MX_BF16) F<uint16_t>(__VA_ARGS__);                  \
    else F<float>(__VA_ARGS__);                                     \
  } while (0)

// torch.optim.SGD's update of one element (scripts/train_frcnn_baseline.py:149-153):
//   d = g + wd * p;  buf = first ? d : momentum * buf + (1 - dampening) * d;
//   d = nesterov ? d + momentum * buf : buf;  p -= lr * d
// Shared by sgd_kernel (mx_optim.hip) and the pack-fused sgd_pack_kernel (mx_conv.hip), both built with
// the same flags, so the two paths produce the same bits.
__device__ __forceinline__ float sgd_update(float& p, float g, float& b, bool first, float lr, float momentum,
                                            float dampening, float wd, int nesterov) {
  // explicit fused multiply-adds: the same rounding in every kernel that inlines this, whatever
  // contraction the compiler would pick around it
  const float d = __fmaf_rn(wd, p, g);
  b = first ? d : __fmaf_rn(momentum, b, __fmul_rn(1.f - dampening, d));
  const float u = nesterov ? __fmaf_rn(momentum, b, d) : b;
  p = __fmaf_rn(-lr, u, p);
  return p;
}

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline size_t align_up(size_t v, size_t a = 256) { return (v + a - 1) / a * a; }

// Carves a caller-owned workspace into aligned slabs.
struct Carver {
  char* base;
  size_t cap, off = 0;
  Carver(void* b, size_t c) : base((char*)b), cap(c) {}
  template <typename T> T* take(size_t count) {
    size_t o = align_up(off);
    off = o + sizeof(T) * count;
    return base ? (T*)(base + o) : nullptr;
  }
  bool ok() const { return off <= cap; }
};

}  // namespace mx
