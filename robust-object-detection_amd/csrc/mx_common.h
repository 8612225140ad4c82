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
