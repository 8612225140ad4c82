// mx_optim.hip — multi-tensor SGD (momentum, weight decay) in one launch per 64 tensors (gfx950).
//
// torch.optim.SGD semantics (the reference: SGD(params, lr=0.005, momentum=0.9, weight_decay=5e-4),
// scripts/train_frcnn_baseline.py:149-153, step at :176):
//   d = g + wd * p;  buf = first ? d : momentum * buf + (1 - dampening) * d;
//   d = nesterov ? d + momentum * buf : buf;  p -= lr * d
// Replaces the three multi_tensor_apply launches (plus their host-side grouping) of torch's foreach
// path with one streaming pass: 20 B of HBM traffic per parameter (p, g, buf read; p, buf written).
#include "mx_common.h"

namespace mx {

static constexpr int SGD_CHUNK = 64;      // tensors per launch (kernel-argument struct < 4 KiB)
static constexpr int SGD_PER_BLOCK = 2048; // elements per 256-thread block

struct SgdArgs {
  float* p[SGD_CHUNK];
  const float* g[SGD_CHUNK];
  float* buf[SGD_CHUNK];
  int64_t n[SGD_CHUNK];
  int32_t first_block[SGD_CHUNK + 1];  // prefix of blocks per tensor
  uint64_t first_mask;                 // bit t: tensor t takes its first momentum step
  int count;
  float lr, momentum, dampening, wd;
  int nesterov;
};

__device__ __forceinline__ float sgd1(float& p, float g, float& b, bool first, const SgdArgs& a) {
  return sgd_update(p, g, b, first, a.lr, a.momentum, a.dampening, a.wd, a.nesterov);
}

__global__ void __launch_bounds__(256) sgd_kernel(SgdArgs a) {
  const int blk = blockIdx.x;
  int lo = 0, hi = a.count - 1;  // tensor t with first_block[t] <= blk < first_block[t+1]
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (a.first_block[mid] <= blk) lo = mid;
    else hi = mid - 1;
  }
  const int t = lo;
  const int64_t n = a.n[t];
  const int64_t e0 = (int64_t)(blk - a.first_block[t]) * SGD_PER_BLOCK;
  const int64_t e1 = min<int64_t>(n, e0 + SGD_PER_BLOCK);
  float* __restrict__ p = a.p[t];
  const float* __restrict__ g = a.g[t];
  float* __restrict__ b = a.buf[t];
  const bool first = (a.first_mask >> t) & 1ull;
  const bool vec = ((((uintptr_t)p) | ((uintptr_t)g) | ((uintptr_t)b)) & 15u) == 0;
  if (vec) {
    for (int64_t e = e0 + threadIdx.x * 4; e + 3 < e1; e += 256 * 4) {
      float4 pv = *(float4*)(p + e), bv = *(float4*)(b + e);
      const float4 gv = *(const float4*)(g + e);
      sgd1(pv.x, gv.x, bv.x, first, a);
      sgd1(pv.y, gv.y, bv.y, first, a);
      sgd1(pv.z, gv.z, bv.z, first, a);
      sgd1(pv.w, gv.w, bv.w, first, a);
      *(float4*)(p + e) = pv;
      *(float4*)(b + e) = bv;
    }
    const int64_t tail = e0 + ((e1 - e0) & ~(int64_t)3);
    for (int64_t e = tail + threadIdx.x; e < e1; e += 256) sgd1(p[e], g[e], b[e], first, a);
  } else {
    for (int64_t e = e0 + threadIdx.x; e < e1; e += 256) sgd1(p[e], g[e], b[e], first, a);
  }
}

}  // namespace mx

using namespace mx;

extern "C" int mx_sgd_step(float* const* params, const float* const* grads, float* const* bufs, const int64_t* numels,
                           const uint8_t* first, int64_t count, float lr, float momentum, float dampening,
                           float weight_decay, int nesterov, mx_stream_t stream) {
  MX_CHECK_ARG(count >= 0 && (count == 0 || (params && grads && bufs && numels && first)), "sgd_step: bad tensor lists");
  for (int64_t c0 = 0; c0 < count; c0 += SGD_CHUNK) {
    SgdArgs a{};
    a.count = (int)std::min<int64_t>(SGD_CHUNK, count - c0);
    a.lr = lr; a.momentum = momentum; a.dampening = dampening; a.wd = weight_decay; a.nesterov = nesterov;
    int64_t blocks = 0;
    for (int i = 0; i < a.count; ++i) {
      const int64_t j = c0 + i;
      MX_CHECK_ARG(params[j] && grads[j] && bufs[j] && numels[j] > 0, "sgd_step: tensor %lld empty or null", (long long)j);
      a.p[i] = params[j]; a.g[i] = grads[j]; a.buf[i] = bufs[j]; a.n[i] = numels[j];
      if (first[j]) a.first_mask |= 1ull << i;
      a.first_block[i] = (int32_t)blocks;
      blocks += cdiv(numels[j], SGD_PER_BLOCK);
      MX_CHECK_ARG(blocks < (1ll << 31), "sgd_step: too many elements");
    }
    a.first_block[a.count] = (int32_t)blocks;
    sgd_kernel<<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(a);
    MX_LAUNCH_CHECK();
  }
  return MX_OK;
}
