// The HeatmapHead's 3x3 convolution (nn.Conv2d(k=3, padding=1), reference
// dll/models/heatmap_head.py:31-45,55-66) forward and backward on NCHW fp32
// tensors -- SURVEY §8(f) rank 4, "backward of K6".  The reference gets these
// gradients from autograd inside Trainer.train (dll/training/trainer.py:263,
// 272); here they are explicit kernels (gfx950):
//   forward  y[n][o][p]  = sum_{c,t} w[o][c][t] x[n][c][p + d(t)] + b[o]
//   dgrad    gx[n][c][p] = sum_{o,t} w[o][c][t] gy[n][o][p - d(t)]
//   wgrad    gw[o][c][t] = sum_{n,p} gy[n][o][p] x[n][c][p + d(t)]
//   bias     gb[o]       = sum_{n,p} gy[n][o][p]
// (t = ky*3 + kx, d(t) = (ky - 1, kx - 1), zero outside the map).  All three
// are one implicit GEMM kernel on v_mfma_f32_16x16x4_f32 (exact fp32
// products, fp32 accumulation): 64 x 64 output tiles, K in steps of 16 staged
// through LDS by coalesced gathers along each operand's contiguous axis, four
// waves of 2 x 2 fragments.  wgrad splits K (images x pixels) into fixed
// slices whose partial sums are added in slice order, and the bias sums run
// in a fixed tree: every result is deterministic.  Training is outside the
// hot path; these kernels are correctness-first and
// MFMA-tiled, not tuned.
#include <algorithm>

#include "kpd_common.h"
#include "kpd_kernels.h"

namespace {

constexpr int TB = 64, TK = 16;

enum { C3_FWD = 0, C3_DGRAD = 1, C3_WGRAD = 2 };

// map offset of pixel p shifted by tap t (sign +1: p + d(t), -1: p - d(t)); -1 outside
__device__ __forceinline__ int shift_px(int p, int t, int sgn, int H, int W) {
  const int y = p / W, x = p - y * W;
  const int yy = y + sgn * (t / 3 - 1), xx = x + sgn * (t % 3 - 1);
  return (yy >= 0 && yy < H && xx >= 0 && xx < W) ? yy * W + xx : -1;
}

// MODE C3_FWD:   M = O, N = HW, K = 9C, per image (blockIdx.z)
// MODE C3_DGRAD: M = C, N = HW, K = 9O, per image
// MODE C3_WGRAD: M = O, N = 9C, K = NI*HW, K slice blockIdx.z of length kslice
template <int MODE>
__global__ __launch_bounds__(256) void conv3_gemm_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                         const float* __restrict__ gy, const float* __restrict__ bias,
                                                         int C, int H, int W, int O, int kslice, int ktot,
                                                         float* __restrict__ out) {
  __shared__ float As[TK][TB + 4], Bs[TK][TB + 4];
  const int HW = H * W;
  const int M = MODE == C3_DGRAD ? C : O;
  const int Nn = MODE == C3_WGRAD ? 9 * C : HW;
  const int K = MODE == C3_FWD ? 9 * C : MODE == C3_DGRAD ? 9 * O : 0;
  const int m0 = blockIdx.y * TB, n0 = blockIdx.x * TB, z = blockIdx.z;
  const int k_begin = MODE == C3_WGRAD ? z * kslice : 0;
  const int k_end = MODE == C3_WGRAD ? min(k_begin + kslice, ktot) : K;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, g = lane >> 4, r16 = lane & 15;

  // A[m][k] and B[k][n] element loaders (0 outside the operand)
  auto ldA = [&](int m, int k) -> float {
    if (m >= M || k >= k_end) return 0.f;
    if constexpr (MODE == C3_FWD) {
      return w[(size_t)m * K + k];
    } else if constexpr (MODE == C3_DGRAD) {
      const int o = k / 9, t = k - o * 9;
      return w[((size_t)o * C + m) * 9 + t];
    } else {
      const int n = k / HW, p = k - n * HW;
      return gy[((size_t)n * O + m) * HW + p];
    }
  };
  auto ldB = [&](int k, int nn) -> float {
    if (nn >= Nn || k >= k_end) return 0.f;
    if constexpr (MODE == C3_FWD) {
      const int c = k / 9, t = k - c * 9, q = shift_px(nn, t, 1, H, W);
      return q < 0 ? 0.f : x[((size_t)z * C + c) * HW + q];
    } else if constexpr (MODE == C3_DGRAD) {
      const int o = k / 9, t = k - o * 9, q = shift_px(nn, t, -1, H, W);
      return q < 0 ? 0.f : gy[((size_t)z * O + o) * HW + q];
    } else {
      const int n = k / HW, p = k - n * HW, c = nn / 9, t = nn - c * 9, q = shift_px(p, t, 1, H, W);
      return q < 0 ? 0.f : x[((size_t)n * C + c) * HW + q];
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // register-staged double buffer: the next K-step's 4 + 4 elements per
  // thread load while this step's MFMAs run
  float ra[4], rb[4];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u;
      // A: k fastest (contiguous for forward / wgrad weights and gy rows)
      ra[u] = ldA(m0 + e / TK, k0 + e % TK);
      // B: forward / dgrad contiguous along n (pixels), wgrad along k (pixels)
      if constexpr (MODE == C3_WGRAD) rb[u] = ldB(k0 + e % TK, n0 + e / TK);
      else rb[u] = ldB(k0 + e / TB, n0 + e % TB);
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u;
      As[e % TK][e / TK] = ra[u];
      if constexpr (MODE == C3_WGRAD) Bs[e % TK][e / TK] = rb[u];
      else Bs[e / TB][e % TB] = rb[u];
    }
  };
  fetch(k_begin);
  for (int k0 = k_begin; k0 < k_end; k0 += TK) {
    __syncthreads();   // the previous step's fragment reads are done
    stash();
    __syncthreads();
    if (k0 + TK < k_end) fetch(k0 + TK);
#pragma unroll
    for (int kk = 0; kk < TK; kk += 4) {
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[kk + g][wm * 32 + i * 16 + r16];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[kk + g][wn * 32 + j * 16 + r16];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
  // lane (g, r16) holds rows 4g + e, column r16 of each 16 x 16 fragment
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm * 32 + i * 16 + g * 4 + e, nn = n0 + wn * 32 + j * 16 + r16;
        if (m >= M || nn >= Nn) continue;
        float v = acc[i][j][e];
        if constexpr (MODE == C3_FWD) v += bias ? bias[m] : 0.f;
        out[((size_t)z * M + m) * Nn + nn] = v;
      }
}

// gw[i] = sum over slices s = 0 .. S-1 (in order) of part[s][i]
__global__ void slice_sum_kernel(const float* __restrict__ part, int S, long n, float* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = 0.f;
  for (int k = 0; k < S; ++k) s += part[(size_t)k * n + i];
  out[i] = s;
}

// gb[o] = sum_{n,p} gy[n][o][p]: one workgroup per o, per-thread strided
// partial sums in a fixed order, then a fixed-shape tree
__global__ __launch_bounds__(256) void bias_grad_kernel(const float* __restrict__ gy, int N, int O, int HW,
                                                        float* __restrict__ gb) {
  __shared__ float red[256];
  const int o = blockIdx.x, tid = threadIdx.x;
  float s = 0.f;
  for (int n = 0; n < N; ++n) {
    const float* src = gy + ((size_t)n * O + o) * HW;
    for (int p = tid; p < HW; p += 256) s += src[p];
  }
  red[tid] = s;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (tid < h) red[tid] += red[tid + h];
    __syncthreads();
  }
  if (tid == 0) gb[o] = red[0];
}

}  // namespace

hipError_t launch_conv3_forward(const float* x, const float* w, const float* b, int N, int C, int H, int W, int O,
                                float* y, hipStream_t st) {
  if (N <= 0) return hipSuccess;
  const dim3 grid((unsigned)((H * W + TB - 1) / TB), (unsigned)((O + TB - 1) / TB), (unsigned)N);
  hipLaunchKernelGGL(conv3_gemm_kernel<C3_FWD>, grid, dim3(256), 0, st, x, w, nullptr, b, C, H, W, O, 0, 0, y);
  return hipGetLastError();
}

size_t conv3_wgrad_slices(int N, int H, int W) {
  const long K = (long)N * H * W;
  const long ks = 4096;
  return (size_t)((K + ks - 1) / ks);
}

hipError_t launch_conv3_backward(const float* x, const float* w, const float* gy, int N, int C, int H, int W, int O,
                                 float* gx, float* gw, float* gb, float* wgrad_part, hipStream_t st) {
  if (N <= 0) return hipSuccess;
  const int HW = H * W;
  if (gx) {
    const dim3 grid((unsigned)((HW + TB - 1) / TB), (unsigned)((C + TB - 1) / TB), (unsigned)N);
    hipLaunchKernelGGL(conv3_gemm_kernel<C3_DGRAD>, grid, dim3(256), 0, st, nullptr, w, gy, nullptr, C, H, W, O, 0, 0,
                       gx);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (gw) {
    if (!wgrad_part) return hipErrorInvalidValue;
    const int S = (int)conv3_wgrad_slices(N, H, W);
    const int ks = 4096;   // a multiple of the K step (16); the last slice ends at N * H * W
    const dim3 grid((unsigned)((9 * C + TB - 1) / TB), (unsigned)((O + TB - 1) / TB), (unsigned)S);
    hipLaunchKernelGGL(conv3_gemm_kernel<C3_WGRAD>, grid, dim3(256), 0, st, x, nullptr, gy, nullptr, C, H, W, O, ks,
                       N * HW, wgrad_part);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const long n = (long)O * 9 * C;
    hipLaunchKernelGGL(slice_sum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, wgrad_part, S, n, gw);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (gb) {
    hipLaunchKernelGGL(bias_grad_kernel, dim3((unsigned)O), dim3(256), 0, st, gy, N, O, HW, gb);
    return hipGetLastError();
  }
  return hipSuccess;
}
