// MobileNetV3-Small body kernels that are not GEMM-shaped (gfx950).
//
//   * stem: conv3x3 s2 (Cin 1|3 -> 16) + folded BN + hardswish, reads the
//     caller's NCHW fp32 image directly and writes NHWC (fused layout change).
//     torchvision mobilenet_v3_small features.0 (reference backbone.py:250-254).
//   * dwconv: depthwise k3/k5 s1/s2 + folded BN + ReLU/hardswish, NHWC, four
//     channels per lane (16-byte loads/stores along C).  features.N.block.dw.
//   * se: squeeze (global average) + fc1/ReLU + fc2/hardsigmoid, one workgroup
//     per image; the excitation is applied later inside the project conv's
//     A-load (conv_mfma.hip, a_scale), so the scaled tensor never hits HBM.
//   * channel_stats: per-image channel sum/max partials for ChannelAttention
//     when the FPN conv epilogue cannot produce them (H*W not a tile multiple).
#include "kpd_common.h"
#include "kpd_kernels.h"

namespace {

__global__ __launch_bounds__(256) void stem_kernel(const float* __restrict__ img, int N, int Cin, int H,
                                                   int W, const float* __restrict__ w,
                                                   const float* __restrict__ b, float* __restrict__ out,
                                                   int Ho, int Wo) {
  __shared__ float sw[16 * 27];
  __shared__ float sb[16];
  const int nw = 16 * Cin * 9;
  for (int i = threadIdx.x; i < nw; i += blockDim.x) sw[i] = w[i];
  if (threadIdx.x < 16) sb[threadIdx.x] = b[threadIdx.x];
  __syncthreads();
  const int pix = blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= N * Ho * Wo) return;
  const int n = pix / (Ho * Wo), r = pix - n * Ho * Wo, oy = r / Wo, ox = r - oy * Wo;
  float in[27];
  for (int c = 0; c < Cin; ++c)
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int iy = oy * 2 - 1 + ky, ix = ox * 2 - 1 + kx;
        in[c * 9 + ky * 3 + kx] = (iy >= 0 && iy < H && ix >= 0 && ix < W)
                                      ? img[((size_t)(n * Cin + c) * H + iy) * W + ix] : 0.f;
      }
  float o[16];
#pragma unroll
  for (int co = 0; co < 16; ++co) {
    float a = 0.f;
    for (int k = 0; k < Cin * 9; ++k) a = fmaf(in[k], sw[co * Cin * 9 + k], a);
    o[co] = kpd_act(a + sb[co], ACT_HSWISH);
  }
  float4* dst = reinterpret_cast<float4*>(out + (size_t)pix * 16);
#pragma unroll
  for (int q = 0; q < 4; ++q) dst[q] = make_float4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
}

template <int K, int S>
__global__ __launch_bounds__(256) void dwconv_kernel(const float* __restrict__ in, const float* __restrict__ w,
                                                     const float* __restrict__ b, float* __restrict__ out,
                                                     int N, int H, int W, int Cp, int Ho, int Wo, int act) {
  const int nq = Cp >> 2;
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t total = (size_t)N * Ho * Wo * nq;
  if (idx >= total) return;
  const int q = idx % nq;
  const size_t pix = idx / nq;
  const int n = pix / (Ho * Wo), r = pix - (size_t)n * Ho * Wo, oy = r / Wo, ox = r - oy * Wo;
  constexpr int P = (K - 1) / 2;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int ky = 0; ky < K; ++ky) {
    const int iy = oy * S - P + ky;
    if (iy < 0 || iy >= H) continue;
#pragma unroll
    for (int kx = 0; kx < K; ++kx) {
      const int ix = ox * S - P + kx;
      if (ix < 0 || ix >= W) continue;
      const float4 v = *reinterpret_cast<const float4*>(in + ((size_t)(n * H + iy) * W + ix) * Cp + q * 4);
      const float4 k = *reinterpret_cast<const float4*>(w + (ky * K + kx) * Cp + q * 4);
      acc.x = fmaf(v.x, k.x, acc.x); acc.y = fmaf(v.y, k.y, acc.y);
      acc.z = fmaf(v.z, k.z, acc.z); acc.w = fmaf(v.w, k.w, acc.w);
    }
  }
  const float4 bb = *reinterpret_cast<const float4*>(b + q * 4);
  float4 o;
  o.x = kpd_act(acc.x + bb.x, act); o.y = kpd_act(acc.y + bb.y, act);
  o.z = kpd_act(acc.z + bb.z, act); o.w = kpd_act(acc.w + bb.w, act);
  *reinterpret_cast<float4*>(out + pix * Cp + q * 4) = o;
}

// One workgroup per image.  x: [N][HW][Cp]; w1: [sq][C]; w2: [C][sq].
__global__ __launch_bounds__(256) void se_kernel(const float* __restrict__ x, int HW, int C, int Cp,
                                                 const float* __restrict__ w1, const float* __restrict__ b1,
                                                 const float* __restrict__ w2, const float* __restrict__ b2,
                                                 int sq, float* __restrict__ scale) {
  __shared__ float4 part[256];
  __shared__ float mean[1024];
  __shared__ float hid[256];
  const int n = blockIdx.x, tid = threadIdx.x;
  const int nq = Cp >> 2;                 // <= 256 (host checks Cp <= 1024)
  const int rows = 256 / nq;              // pixel strides sharing one channel quad
  const float* xb = x + (size_t)n * HW * Cp;
  {
    const int q = tid % nq, pr = tid / nq;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (pr < rows) {
      for (int p = pr; p < HW; p += rows) {
        const float4 v = *reinterpret_cast<const float4*>(xb + (size_t)p * Cp + q * 4);
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
    }
    part[tid] = s;
  }
  __syncthreads();
  if (tid < nq) {
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int r = 0; r < rows; ++r) {
      const float4 v = part[r * nq + tid];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    const float hw = (float)HW;
    mean[tid * 4 + 0] = t.x / hw; mean[tid * 4 + 1] = t.y / hw;
    mean[tid * 4 + 2] = t.z / hw; mean[tid * 4 + 3] = t.w / hw;
  }
  __syncthreads();
  // fc1 / fc2: one thread per output streaming its weight row with 16-byte
  // loads (C and sq are multiples of 4 in MobileNetV3-Small), two partial sums.
  for (int j = tid; j < sq; j += 256) {
    const float4* wr = reinterpret_cast<const float4*>(w1 + (size_t)j * C);
    float a0 = 0.f, a1 = 0.f;
#pragma unroll 4
    for (int q = 0; q < C / 4; ++q) {
      const float4 w = wr[q];
      a0 = fmaf(w.x, mean[4 * q], a0); a1 = fmaf(w.y, mean[4 * q + 1], a1);
      a0 = fmaf(w.z, mean[4 * q + 2], a0); a1 = fmaf(w.w, mean[4 * q + 3], a1);
    }
    hid[j] = fmaxf(a0 + a1 + b1[j], 0.f);
  }
  __syncthreads();
  for (int c = tid; c < Cp; c += 256) {
    float v = 0.f;
    if (c < C) {
      const float4* wr = reinterpret_cast<const float4*>(w2 + (size_t)c * sq);
      float a0 = 0.f, a1 = 0.f;
#pragma unroll 4
      for (int q = 0; q < sq / 4; ++q) {
        const float4 w = wr[q];
        a0 = fmaf(w.x, hid[4 * q], a0); a1 = fmaf(w.y, hid[4 * q + 1], a1);
        a0 = fmaf(w.z, hid[4 * q + 2], a0); a1 = fmaf(w.w, hid[4 * q + 3], a1);
      }
      v = kpd_hsigmoid(a0 + a1 + b2[c]);
    }
    scale[(size_t)n * Cp + c] = v;
  }
}

// stats: [N][tiles][2][Cp]; grid (tiles, N); each block reduces HW/tiles pixels.
__global__ __launch_bounds__(256) void channel_stats_kernel(const float* __restrict__ x, int HW, int Cp,
                                                            int tiles, float* __restrict__ stats) {
  const int t = blockIdx.x, n = blockIdx.y;
  const int per = (HW + tiles - 1) / tiles;
  const int p0 = t * per, p1 = min(HW, p0 + per);
  for (int c = threadIdx.x; c < Cp; c += blockDim.x) {
    float s = 0.f, m = -INFINITY;
    for (int p = p0; p < p1; ++p) {
      const float v = x[((size_t)n * HW + p) * Cp + c];
      s += v; m = fmaxf(m, v);
    }
    float* st = stats + ((size_t)n * tiles + t) * 2 * Cp;
    st[c] = s;
    st[Cp + c] = m;
  }
}

}  // namespace

hipError_t launch_stem(const float* img, int N, int Cin, int H, int W, const float* w, const float* b,
                       float* out, int Ho, int Wo, hipStream_t st) {
  const int total = N * Ho * Wo;
  hipLaunchKernelGGL(stem_kernel, dim3((total + 255) / 256), dim3(256), 0, st, img, N, Cin, H, W, w, b, out,
                     Ho, Wo);
  return hipGetLastError();
}

hipError_t launch_dwconv(const float* in, const float* w, const float* b, float* out, int N, int H, int W,
                         int Cp, int Ho, int Wo, int k, int s, int act, hipStream_t st) {
  const size_t total = (size_t)N * Ho * Wo * (Cp / 4);
  const dim3 grid((unsigned)((total + 255) / 256));
#define DW(K, S) hipLaunchKernelGGL((dwconv_kernel<K, S>), grid, dim3(256), 0, st, in, w, b, out, N, H, W, Cp, Ho, Wo, act)
  if (k == 3 && s == 1) DW(3, 1);
  else if (k == 3 && s == 2) DW(3, 2);
  else if (k == 5 && s == 1) DW(5, 1);
  else if (k == 5 && s == 2) DW(5, 2);
  else return hipErrorInvalidValue;
#undef DW
  return hipGetLastError();
}

hipError_t launch_se(const float* x, int N, int HW, int C, int Cp, const float* w1, const float* b1,
                     const float* w2, const float* b2, int sq, float* scale, hipStream_t st) {
  if (Cp > 1024 || sq > 256 || C % 4 || sq % 4) return hipErrorInvalidValue;
  hipLaunchKernelGGL(se_kernel, dim3(N), dim3(256), 0, st, x, HW, C, Cp, w1, b1, w2, b2, sq, scale);
  return hipGetLastError();
}

hipError_t launch_channel_stats(const float* x, int N, int HW, int Cp, int tiles, float* stats,
                                hipStream_t st) {
  hipLaunchKernelGGL(channel_stats_kernel, dim3(tiles, N), dim3(128), 0, st, x, HW, Cp, tiles, stats);
  return hipGetLastError();
}
