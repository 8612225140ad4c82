// mx_ssim.hip — the U-Net restoration loss L1 + w·(1 − SSIM) (train_restoration.py:142-178, §8f row 4)
// as two fused gfx950 kernels over NHWC f32 images, one workgroup per 32×32 output tile of one channel
// plane:
//   forward: the tile plus its window halo is staged in LDS; a horizontal pass of the separable
//     Gaussian window (11 taps, σ 1.5) forms the five moments (x, y, x², y², xy) per halo row, a
//     vertical pass finishes the five window sums per pixel; the SSIM map, its derivatives with respect
//     to the three moments that depend on the prediction (∂S/∂μx, ∂S/∂E[x²], ∂S/∂E[xy]) and the tile's
//     Σ SSIM and Σ|x−y| come out of the same pass (per-tile f64 partials, one fixed-order finish block:
//     deterministic, no atomics);
//   backward: the three derivative maps are window-summed again (the window is symmetric, zero padding
//     = the forward's) and combined per pixel: dx = g·(c_s·(W⊛a + 2x·W⊛b + y·W⊛c) + c_l·sign(x−y)).
// Window sums, the SSIM algebra and the derivative maps are f64 on the f32 inputs (the three gradient
// terms cancel heavily where the SSIM map is flat, so f32 maps would cost ~1e-5 of the gradient), so
// the loss and gradient track the f64 evaluation of the reference formula (the reference's own f32 depthwise convs lose ~1e-4 relative
// in the variance terms E[x²] − μ² on flat regions).
#include "mx_common.h"

namespace mx {
namespace {

constexpr int kTile = 32;
constexpr int kMaxR = 7;  // window sizes up to 15
constexpr int kRows = kTile + 2 * kMaxR;

struct Taps {
  double g[16];
  int r;  // window radius (size = 2r + 1)
};

__global__ __launch_bounds__(256) void ssim_fwd_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                       int H, int W, int C, int ntw, Taps t, double c1, double c2,
                                                       double* __restrict__ ma, double* __restrict__ mb,
                                                       double* __restrict__ mc, double* __restrict__ part) {
  __shared__ float xs[kRows][kRows + 1], ys[kRows][kRows + 1];
  __shared__ double hs[5][kRows][kTile];
  __shared__ double red[2][4];
  __shared__ double g[16];
  if (threadIdx.x < 16) g[threadIdx.x] = t.g[threadIdx.x];
  const int r = t.r, n2 = kTile + 2 * r;
  const int plane = blockIdx.y, n = plane / C, c = plane - n * C;
  const int h0 = (blockIdx.x / ntw) * kTile, w0 = (blockIdx.x % ntw) * kTile;
  const int64_t base = (int64_t)n * H * W * C + c;
  for (int i = threadIdx.x; i < n2 * n2; i += 256) {
    const int rr = i / n2, cc = i - rr * n2;
    const int h = h0 - r + rr, w = w0 - r + cc;
    float xv = 0.f, yv = 0.f;
    if (h >= 0 && h < H && w >= 0 && w < W) {
      const int64_t o = base + ((int64_t)h * W + w) * C;
      xv = x[o];
      yv = y[o];
    }
    xs[rr][cc] = xv;
    ys[rr][cc] = yv;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n2 * kTile; i += 256) {
    const int rr = i / kTile, cc = i - rr * kTile;
    double s0 = 0, s1 = 0, s2 = 0, s3 = 0, s4 = 0;
    for (int k = 0; k <= 2 * r; ++k) {
      const double a = xs[rr][cc + k], b = ys[rr][cc + k], wk = g[k];
      s0 += wk * a;
      s1 += wk * b;
      s2 += wk * (a * a);
      s3 += wk * (b * b);
      s4 += wk * (a * b);
    }
    hs[0][rr][cc] = s0;
    hs[1][rr][cc] = s1;
    hs[2][rr][cc] = s2;
    hs[3][rr][cc] = s3;
    hs[4][rr][cc] = s4;
  }
  __syncthreads();
  double accS = 0, accL = 0;
  for (int i = threadIdx.x; i < kTile * kTile; i += 256) {
    const int rr = i / kTile, cc = i - rr * kTile;
    const int h = h0 + rr, w = w0 + cc;
    if (h >= H || w >= W) continue;
    double mu1 = 0, mu2 = 0, e11 = 0, e22 = 0, e12 = 0;
    for (int k = 0; k <= 2 * r; ++k) {
      const double wk = g[k];
      mu1 += wk * hs[0][rr + k][cc];
      mu2 += wk * hs[1][rr + k][cc];
      e11 += wk * hs[2][rr + k][cc];
      e22 += wk * hs[3][rr + k][cc];
      e12 += wk * hs[4][rr + k][cc];
    }
    // train_restoration.py:155-164 algebra: sigma = E[.] - mu^2, S = (2 mu12 + C1)(2 s12 + C2) / ...
    const double mu1s = mu1 * mu1, mu2s = mu2 * mu2, mu12 = mu1 * mu2;
    const double s1 = e11 - mu1s, s2 = e22 - mu2s, s12 = e12 - mu12;
    const double A1 = 2 * mu12 + c1, A2 = 2 * s12 + c2, B1 = mu1s + mu2s + c1, B2 = s1 + s2 + c2;
    const double D = B1 * B2, S = A1 * A2 / D;
    accS += S;
    const double xv = xs[rr + r][cc + r], yv = ys[rr + r][cc + r];
    accL += fabs(xv - yv);
    if (ma) {
      const double dA1 = A2 / D, dA2 = A1 / D, dB1 = -S / B1, dB2 = -S / B2;
      const int64_t o = base + ((int64_t)h * W + w) * C;
      ma[o] = 2 * mu2 * dA1 - 2 * mu2 * dA2 + 2 * mu1 * dB1 - 2 * mu1 * dB2;  // dS/dmu1
      mb[o] = dB2;                                                             // dS/dE[x^2]
      mc[o] = 2 * dA2;                                                         // dS/dE[xy]
    }
  }
  // block sum in a fixed order: wave shuffles, then the four wave partials in order
  for (int off = 32; off > 0; off >>= 1) {
    accS += __shfl_down(accS, off, 64);
    accL += __shfl_down(accL, off, 64);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wv] = accS;
    red[1][wv] = accL;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int64_t b = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
    part[2 * b] = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
    part[2 * b + 1] = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
  }
}

// one block: out[0] = mean SSIM, out[1] = mean |x - y|, out[2] = out[1] + weight * (1 - out[0])
__global__ __launch_bounds__(1024) void ssim_finish_kernel(const double* __restrict__ part, int64_t nblk, double inv_n,
                                                           float weight, float* __restrict__ out) {
  __shared__ double red[2][16];
  double s = 0, l = 0;
  for (int64_t b = threadIdx.x; b < nblk; b += 1024) {
    s += part[2 * b];
    l += part[2 * b + 1];
  }
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_down(s, off, 64);
    l += __shfl_down(l, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s;
    red[1][threadIdx.x >> 6] = l;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double ts = 0, tl = 0;
    for (int k = 0; k < 16; ++k) {
      ts += red[0][k];
      tl += red[1][k];
    }
    const double ssim = ts * inv_n, l1 = tl * inv_n;
    out[0] = (float)ssim;
    out[1] = (float)l1;
    out[2] = (float)(l1 + (double)weight * (1.0 - ssim));
  }
}

__global__ __launch_bounds__(256) void ssim_bwd_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                       const double* __restrict__ ma, const double* __restrict__ mb,
                                                       const double* __restrict__ mc, int H, int W, int C, int ntw,
                                                       Taps t, const float* __restrict__ gout, float cs, float cl,
                                                       float* __restrict__ gx) {
  __shared__ double as[3][kRows][kRows + 1];
  __shared__ double hs[3][kRows][kTile];
  __shared__ double g[16];
  if (threadIdx.x < 16) g[threadIdx.x] = t.g[threadIdx.x];
  const int r = t.r, n2 = kTile + 2 * r;
  const int plane = blockIdx.y, n = plane / C, c = plane - n * C;
  const int h0 = (blockIdx.x / ntw) * kTile, w0 = (blockIdx.x % ntw) * kTile;
  const int64_t base = (int64_t)n * H * W * C + c;
  for (int i = threadIdx.x; i < n2 * n2; i += 256) {
    const int rr = i / n2, cc = i - rr * n2;
    const int h = h0 - r + rr, w = w0 - r + cc;
    double a = 0, b = 0, d = 0;
    if (h >= 0 && h < H && w >= 0 && w < W) {
      const int64_t o = base + ((int64_t)h * W + w) * C;
      a = ma[o];
      b = mb[o];
      d = mc[o];
    }
    as[0][rr][cc] = a;
    as[1][rr][cc] = b;
    as[2][rr][cc] = d;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n2 * kTile; i += 256) {
    const int rr = i / kTile, cc = i - rr * kTile;
    double s0 = 0, s1 = 0, s2 = 0;
    for (int k = 0; k <= 2 * r; ++k) {
      const double wk = g[k];
      s0 += wk * as[0][rr][cc + k];
      s1 += wk * as[1][rr][cc + k];
      s2 += wk * as[2][rr][cc + k];
    }
    hs[0][rr][cc] = s0;
    hs[1][rr][cc] = s1;
    hs[2][rr][cc] = s2;
  }
  __syncthreads();
  const double go = (double)gout[0];
  for (int i = threadIdx.x; i < kTile * kTile; i += 256) {
    const int rr = i / kTile, cc = i - rr * kTile;
    const int h = h0 + rr, w = w0 + cc;
    if (h >= H || w >= W) continue;
    double wa = 0, wb = 0, wc = 0;
    for (int k = 0; k <= 2 * r; ++k) {
      const double wk = g[k];
      wa += wk * hs[0][rr + k][cc];
      wb += wk * hs[1][rr + k][cc];
      wc += wk * hs[2][rr + k][cc];
    }
    const int64_t o = base + ((int64_t)h * W + w) * C;
    const double xv = x[o], yv = y[o];
    const double sg = xv > yv ? 1.0 : (xv < yv ? -1.0 : 0.0);  // torch.sign: 0 at x == y
    gx[o] = (float)(go * ((double)cs * (wa + 2.0 * xv * wb + yv * wc) + (double)cl * sg));
  }
}

// The reference window (train_restoration.py:135-139): coords = arange(size) - size // 2,
// g = exp(-coords^2 / (2 sigma^2)), w2 = outer(g, g) / sum -- separable: w2[i][j] = (g[i] / sum g) (g[j] /
// sum g). Evaluated in f64 (the f64 reading of the formula; the reference builds it in f32, whose
// per-element rounding of the 2-D window (~6e-8) is below every tolerance except the cancelling
// mean-SSIM gradient's).
bool make_taps(int window, float sigma, Taps* t) {
  if (window < 1 || window > 2 * kMaxR + 1 || (window & 1) == 0 || !(sigma > 0.f)) return false;
  t->r = window / 2;
  double s = 0;
  double gg[16];
  const double sg = (double)sigma;
  for (int k = 0; k < window; ++k) {
    const double c = (double)(k - window / 2);
    gg[k] = exp(-(c * c) / (2.0 * sg * sg));
    s += gg[k];
  }
  for (int k = 0; k < 16; ++k) t->g[k] = k < window ? gg[k] / s : 0.0;
  return true;
}

}  // namespace
}  // namespace mx

using namespace mx;

extern "C" size_t mx_ssim_workspace(int64_t N, int64_t H, int64_t W, int64_t C) {
  const int64_t tiles = cdiv(H, kTile) * cdiv(W, kTile);
  return (size_t)(N * C * tiles) * 2 * sizeof(double);
}

extern "C" int mx_ssim_l1_fwd(const float* pred, const float* target, int64_t N, int64_t H, int64_t W, int64_t C,
                              int window, float sigma, float c1, float c2, float weight, float* out3, double* dmaps,
                              void* ws, size_t ws_bytes, mx_stream_t stream) {
  Taps t;
  MX_CHECK_ARG(make_taps(window, sigma, &t), "ssim: window must be odd and <= 15, sigma > 0");
  MX_CHECK_ARG(N > 0 && H > 0 && W > 0 && C > 0 && H * W < (1ll << 31), "ssim: bad sizes");
  MX_CHECK_ARG(ws_bytes >= mx_ssim_workspace(N, H, W, C), "ssim: workspace too small");
  const int ntw = (int)cdiv(W, kTile), nth = (int)cdiv(H, kTile);
  const int64_t planes = N * C, npx = N * H * W * C;
  MX_CHECK_ARG(planes < 65536, "ssim: at most 65535 channel planes per call");
  hipStream_t s = (hipStream_t)stream;
  double* ma = dmaps;
  double* mb = dmaps ? dmaps + npx : nullptr;
  double* mc = dmaps ? dmaps + 2 * npx : nullptr;
  ssim_fwd_kernel<<<dim3(ntw * nth, (unsigned)planes), 256, 0, s>>>(pred, target, (int)H, (int)W, (int)C, ntw, t,
                                                                     (double)c1, (double)c2, ma, mb, mc, (double*)ws);
  MX_LAUNCH_CHECK();
  ssim_finish_kernel<<<1, 1024, 0, s>>>((const double*)ws, (int64_t)ntw * nth * planes, 1.0 / (double)npx, weight, out3);
  MX_LAUNCH_CHECK();
  return MX_OK;
}

extern "C" int mx_ssim_l1_bwd(const float* pred, const float* target, const double* dmaps, int64_t N, int64_t H,
                              int64_t W, int64_t C, int window, float sigma, const float* gout, float cs, float cl,
                              float* grad, mx_stream_t stream) {
  Taps t;
  MX_CHECK_ARG(make_taps(window, sigma, &t), "ssim: window must be odd and <= 15, sigma > 0");
  MX_CHECK_ARG(N > 0 && H > 0 && W > 0 && C > 0 && H * W < (1ll << 31), "ssim: bad sizes");
  MX_CHECK_ARG(dmaps && gout && grad, "ssim_bwd: maps, gout and grad are required");
  const int ntw = (int)cdiv(W, kTile), nth = (int)cdiv(H, kTile);
  const int64_t planes = N * C, npx = N * H * W * C;
  MX_CHECK_ARG(planes < 65536, "ssim: at most 65535 channel planes per call");
  ssim_bwd_kernel<<<dim3(ntw * nth, (unsigned)planes), 256, 0, (hipStream_t)stream>>>(
      pred, target, dmaps, dmaps + npx, dmaps + 2 * npx, (int)H, (int)W, (int)C, ntw, t, gout, cs, cl, grad);
  MX_LAUNCH_CHECK();
  return MX_OK;
}
