// The HeatmapHead's 3x3 convolution (nn.Conv2d(k=3, padding=1), reference
// dll/models/heatmap_head.py:31-45,55-66) forward and backward on NCHW fp32
// tensors -- SURVEY §8(f) rank 4, "backward of K6".  The reference gets these
// gradients from autograd inside Trainer.train (dll/training/trainer.py:263,
// 272); here they are explicit kernels (gfx950):
//   forward  y[n][o][p]  = sum_{c,t} w[o][c][t] x[n][c][p + d(t)] + b[o]
//   dgrad    gx[n][c][p] = sum_{o,t} w[o][c][t] gy[n][o][p - d(t)]
//   wgrad    gw[o][c][t] = sum_{n,p} gy[n][o][p] x[n][c][p + d(t)]
//   bias     gb[o]       = sum_{n,p} gy[n][o][p]
// (t = ky*3 + kx, d(t) = (ky - 1, kx - 1), zero outside the map).
// Default paths (round 5): forward and dgrad at the heatmap
// convs' 56 x 56 shapes (cin 64 | 256 -> cout 64 | 256) on the split hmconv
// kernel in its linear epilogue mode (three f16 products per MAC, fp32
// accumulation: the forward heatmap convs' arithmetic); wgrad (any shape) as
// a per-tap GEMM over zero-padded planes on the same split products; the bias
// from per-plane sums.  Fallback for other forward / dgrad shapes, and for all
// three under KPD_K6_GENERIC (diagnostic build): one implicit GEMM kernel on
// v_mfma_f32_16x16x4_f32 (exact fp32 products): 64 x 64 output tiles, K in
// steps of 16 staged through LDS, four waves of 2 x 2 fragments.  wgrad sums
// fixed K slices in slice order and the bias sums run in fixed orders: every
// result is deterministic.
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

// ===================================================================== fast paths (round 5)
// forward / dgrad at the heatmap convs' 56 x 56 shape (cin 64 | 256 -> cout
// 256): the split hmconv kernel in its linear mode (three f16 MFMA products
// of hi / lo operand splits, fp32 accumulation -- the forward heatmap convs'
// fp32-accurate arithmetic) on the zero-bordered hmconv layout,
// then an NHWC -> NCHW transpose.  wgrad for any shape: an fp32 MFMA GEMM over
// zero-padded planes (exact products), per tap, split over image slices that
// are summed in order.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
constexpr int kHmSide = 56;

// per-image max|x| -> hsc[n * 4] (float bits; hsc zeroed)
__global__ __launch_bounds__(256) void k6_amax_kernel(const float* __restrict__ x, long per_img,
                                                      float* __restrict__ hsc) {
  const float* src = x + (size_t)blockIdx.y * per_img;
  float m = 0.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < per_img; i += (long)gridDim.x * 256)
    m = fmaxf(m, fabsf(src[i]));
  __shared__ float red[4];
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  if (threadIdx.x == 0 && m > 0.f)   // one atomic per workgroup (64 per image)
    atomicMax(reinterpret_cast<unsigned*>(hsc + (size_t)blockIdx.y * 4), __float_as_uint(m));
}

// Per image n: the input scale exponent a (hsc[n][2], an exact small integer
// as float: k6_to_hm_kernel scales by 2^a) and hsc[n][1], the bound whose
// split_exp_of is a + w_exp, so that hmconv_kernel (in_idx 1, w_exp 0)
// unscales by 2^-(a + w_exp) with the weights' exponent computed on the
// device (no host round trip).  a = split_exp_of(max |x_n|), lowered where
// a + w_exp would pass split_exp_of's clamp at 100 (max|x| * max|w| below
// ~2^-72): then hsc[n][1] = 0, whose split_exp_of is 100 = a + w_exp exactly
// (a smaller scale only lowers the split's precision floor).
__global__ __launch_bounds__(256) void k6_bound_kernel(float* __restrict__ hsc, int N, const float* __restrict__ wmax) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const int we = split_exp_of(*wmax);
  int a = split_exp_of(hsc[(size_t)n * 4]);
  float bound = ldexpf(hsc[(size_t)n * 4], -we);
  if (a + we > 100) {
    a = 100 - we;
    bound = 0.f;
  }
  hsc[(size_t)n * 4 + 1] = bound;
  hsc[(size_t)n * 4 + 2] = (float)a;
}

// x [N][C][56][56] fp32 -> the hmconv split layout [N * 3249][C / 32][hi32 | lo32]
// f16 at interior positions (borders zeroed by the caller), image n scaled by
// 2^hsc[n * 4 + 2] (k6_bound_kernel) -- the scale hmconv_kernel's split mode unscales by
__global__ __launch_bounds__(256) void k6_to_hm_kernel(const float* __restrict__ x, int C,
                                                       const float* __restrict__ hsc, _Float16* __restrict__ out) {
  __shared__ float t[32][65];
  const int n = blockIdx.z, cg = blockIdx.y, p0 = blockIdx.x * 64, tid = threadIdx.x;
  const float* src = x + ((size_t)n * C + cg * 32) * (kHmSide * kHmSide);
  for (int i = tid; i < 32 * 64; i += 256) {
    const int c = i >> 6, pp = i & 63;
    t[c][pp] = p0 + pp < kHmSide * kHmSide ? src[(size_t)c * (kHmSide * kHmSide) + p0 + pp] : 0.f;
  }
  __syncthreads();
  const int pp = tid >> 2, c8 = (tid & 3) * 8, p = p0 + pp;
  if (p >= kHmSide * kHmSide) return;
  const float sc = ldexpf(1.f, (int)hsc[(size_t)n * 4 + 2]);
  const int y = p / kHmSide, xx = p - y * kHmSide;
  f16x8 hi, lo;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float v = t[c8 + e][pp] * sc;
    hi[e] = (_Float16)v;
    lo[e] = (_Float16)(v - (float)hi[e]);
  }
  char* dst = reinterpret_cast<char*>(out) + ((size_t)n * kHmRoiPos + (y + 1) * kHmPitch + xx) * ((size_t)C * 4) +
              cg * 128 + c8 * 2;
  *reinterpret_cast<f16x8*>(dst) = hi;
  *reinterpret_cast<f16x8*>(dst + 64) = lo;
}

// the hmconv layout's border positions of image n (row 0: 57 positions; the
// shared zero column 56 of rows 1 .. 56) set to zero; C channels x 4 bytes each
__global__ __launch_bounds__(256) void k6_hm_border_kernel(_Float16* __restrict__ out, int C) {
  const int n = blockIdx.x, per = C / 4;   // 16-byte pieces per position
  uint4* base = reinterpret_cast<uint4*>(out) + (size_t)n * kHmRoiPos * per;
  for (int i = threadIdx.x; i < (kHmPitch + kHmSide) * per; i += 256) {
    const int k = i / per, piece = i - k * per;
    const int pos = k < kHmPitch ? k : (k - kHmPitch + 1) * kHmPitch + kHmSide;
    base[(size_t)pos * per + piece] = uint4{0u, 0u, 0u, 0u};
  }
}

__global__ __launch_bounds__(256) void k6_max_kernel(const float* __restrict__ w, long n, float* __restrict__ out) {
  float m = 0.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) m = fmaxf(m, fabsf(w[i]));
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0 && m > 0.f) atomicMax(reinterpret_cast<unsigned*>(out), __float_as_uint(m));
}

// w [O][C][3][3] -> split weights [co'][9][ci'] as [hi32 | lo32] groups scaled
// 2^w_exp, w_exp = split_exp_of(max |w|) (pack_split_hm's layout), rows
// co' >= cout zero up to cout_p; flip: the dgrad conv's weights, co' = c,
// ci' = o, tap t <- 8 - t (d(8 - t) = -d(t))
__global__ __launch_bounds__(256) void k6_pack_w_kernel(const float* __restrict__ w, int O, int C, int flip,
                                                        const float* __restrict__ wmax, int cout_p,
                                                        _Float16* __restrict__ ws) {
  const int w_exp = split_exp_of(*wmax);
  const int cin = flip ? O : C, cout = flip ? C : O;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)cout_p * 9 * cin) return;
  const int ci = (int)(i % cin);
  const long r = i / cin;
  const int t = (int)(r % 9), co = (int)(r / 9);
  const float v = co >= cout ? 0.f : flip ? w[((size_t)ci * C + co) * 9 + (8 - t)] : w[((size_t)co * C + ci) * 9 + t];
  const float xs = ldexpf(v, w_exp);
  const _Float16 hi = (_Float16)xs, lo = (_Float16)(xs - (float)hi);
  const size_t o = (size_t)r * 2 * cin + (size_t)(ci / 32) * 64 + ci % 32;
  ws[o] = hi;
  ws[o + 32] = lo;
}

// [N][3136][Op] (the first O of Op channels) -> [N][O][3136]
__global__ __launch_bounds__(256) void k6_nhwc_nchw_kernel(const float* __restrict__ in, int O, int Op,
                                                           float* __restrict__ out) {
  __shared__ float t[64][65];
  constexpr int HW = kHmSide * kHmSide;
  const int n = blockIdx.z, o0 = blockIdx.y * 64, p0 = blockIdx.x * 64, tid = threadIdx.x;
  for (int i = tid; i < 64 * 64; i += 256) {
    const int pp = i >> 6, oo = i & 63;
    t[pp][oo] = (p0 + pp < HW && o0 + oo < O) ? in[((size_t)n * HW + p0 + pp) * Op + o0 + oo] : 0.f;
  }
  __syncthreads();
  for (int i = tid; i < 64 * 64; i += 256) {
    const int oo = i >> 6, pp = i & 63;
    if (p0 + pp < HW && o0 + oo < O) out[((size_t)n * O + o0 + oo) * HW + p0 + pp] = t[pp][oo];
  }
}

// in [N][Ch][H][W] -> out [N][Chp][Qs]: pixel (y, x) at (y + 1) (W + 2) + x + 1,
// zero elsewhere (borders, the tail to Qs, planes ch >= Ch); one workgroup
// per plane (ch, n), coalesced reads and writes.  Also: the plane's max |in|
// into amax[n][ch] (amax non-null) and, psum non-null, the
// plane's sum psum[n][ch] (fixed order: a thread's positions ascending, then
// an LDS tree) -- the bias gradient's partials.  out null: sums / max only.
__global__ __launch_bounds__(256) void k6_plane_kernel(const float* __restrict__ in, int Ch, int H, int W, int Chp,
                                                       int Qs, float* __restrict__ out, float* __restrict__ amax,
                                                       float* __restrict__ psum) {
  __shared__ float red[256];
  const int ch = blockIdx.x, n = blockIdx.y, tid = threadIdx.x, W2 = W + 2;
  const bool live = ch < Ch;
  const float* src = in + ((size_t)n * Ch + (live ? ch : 0)) * H * W;
  float* dst = out ? out + ((size_t)n * Chp + ch) * Qs : nullptr;
  float m = 0.f, sum = 0.f;
  for (int q = tid; q < Qs; q += 256) {
    const int yy = q / W2 - 1, xx = q - (yy + 1) * W2 - 1;
    float v = 0.f;
    if (live && yy >= 0 && yy < H && xx >= 0 && xx < W) {
      v = src[yy * W + xx];
      m = fmaxf(m, fabsf(v));
      sum += v;
    }
    if (dst) dst[q] = v;
  }
  if (amax) {   // per-plane max |in| (k6_max_finish_kernel reduces them: no same-address atomics)
    m = wave_max(m);
    if ((tid & 63) == 0) red[tid >> 6] = m;
    __syncthreads();
    if (tid == 0) amax[(size_t)n * Chp + ch] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    __syncthreads();
  }
  if (psum && live) {
    red[tid] = sum;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
      if (tid < h) red[tid] += red[tid + h];
      __syncthreads();
    }
    if (tid == 0) psum[(size_t)n * Ch + ch] = red[0];
  }
}

// out[0] = max of m[0 .. n)
__global__ __launch_bounds__(256) void k6_max_finish_kernel(const float* __restrict__ m, long n, float* __restrict__ out) {
  __shared__ float red[4];
  float v = 0.f;
  for (long i = threadIdx.x; i < n; i += 256) v = fmaxf(v, m[i]);
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// gb[o] = sum over n (in order) of psum[n][o]
__global__ __launch_bounds__(256) void k6_bias_finish_kernel(const float* __restrict__ psum, int N, int O,
                                                             float* __restrict__ gb) {
  const int o = blockIdx.x * 256 + threadIdx.x;
  if (o >= O) return;
  float s = 0.f;
  for (int n = 0; n < N; ++n) s += psum[(size_t)n * O + o];
  gb[o] = s;
}

// wgrad partials: part[s][o][c][t] = sum over the images of slice s and the
// padded positions q of gyP[n][o][q] * xP[n][c][q + off(t)] (gyP is zero on
// the border positions, so the border q add nothing and a shifted read past an
// image's plane is multiplied by zero; xP carries a guard of W + 3 floats at
// both ends of the buffer).  128 x 128 tiles per tap, 4 waves of 64 x 64,
// K-steps of 16 positions: a lane's 16-byte LDS read feeds four MFMAs (its K
// index 4 g + j in step j, on A and B alike).  Exact fp32 products.
constexpr int kWgT = 128, kWgK = 16, kWgLd = kWgK + 4;
__global__ __launch_bounds__(256) void k6_wgrad_kernel(const float* __restrict__ gyP, const float* __restrict__ xP,
                                                       int N, int Op, int Cp, int O, int C, int W2, int Qs, int ips,
                                                       float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float As[2][kWgT][kWgLd];
  __shared__ __attribute__((aligned(16))) float Bs[2][kWgT][kWgLd];
  const int c0 = blockIdx.x * kWgT, o0 = blockIdx.y * kWgT, t = blockIdx.z % 9, s = blockIdx.z / 9;
  const int off = (t / 3 - 1) * W2 + (t % 3 - 1);
  const int n0 = s * ips, n1 = min(N, n0 + ips);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4, r16 = lane & 15;
  const int lrow = tid >> 2, lq = (tid & 3) * 4;   // loader: rows lrow, lrow + 64; positions lq .. lq + 3
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int total = (n1 - n0) * (Qs / kWgK);
  // running load pointers (row lrow; row lrow + 64 is 64 planes on): K-steps
  // walk a plane, then jump to the same row of the next image
  const float* pa = gyP + ((size_t)n0 * Op + o0 + lrow) * Qs + lq;
  const float* pb = xP + ((size_t)n0 * Cp + c0 + lrow) * Qs + lq + off;
  const size_t ra64 = (size_t)64 * Qs, ajump = (size_t)(Op - 1) * Qs, bjump = (size_t)(Cp - 1) * Qs;
  int fq = 0;
  float4 ra0, ra1, rb0, rb1;
#define K6_FETCH()                                                                   \
  do {                                                                               \
    ra0 = *reinterpret_cast<const float4*>(pa);                                      \
    ra1 = *reinterpret_cast<const float4*>(pa + ra64);                               \
    rb0 = make_float4(pb[0], pb[1], pb[2], pb[3]);                                   \
    rb1 = make_float4(pb[ra64], pb[ra64 + 1], pb[ra64 + 2], pb[ra64 + 3]);           \
    pa += kWgK;                                                                      \
    pb += kWgK;                                                                      \
    if ((fq += kWgK) == Qs) { fq = 0; pa += ajump; pb += bjump; }                    \
  } while (0)
#define K6_STASH(b)                                                                  \
  do {                                                                               \
    *reinterpret_cast<float4*>(&As[b][lrow][lq]) = ra0;                              \
    *reinterpret_cast<float4*>(&As[b][lrow + 64][lq]) = ra1;                         \
    *reinterpret_cast<float4*>(&Bs[b][lrow][lq]) = rb0;                              \
    *reinterpret_cast<float4*>(&Bs[b][lrow + 64][lq]) = rb1;                         \
  } while (0)
  if (total > 0) {
    K6_FETCH();
    K6_STASH(0);
  }
  __syncthreads();
  for (int st = 0; st < total; ++st) {
    const int b = st & 1;
    if (st + 1 < total) K6_FETCH();
    float4 a4[4], b4[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a4[i] = *reinterpret_cast<const float4*>(&As[b][wm * 64 + i * 16 + r16][4 * g]);
#pragma unroll
    for (int j = 0; j < 4; ++j) b4[j] = *reinterpret_cast<const float4*>(&Bs[b][wn * 64 + j * 16 + r16][4 * g]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[i].x, b4[j].x, acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[i].y, b4[j].y, acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[i].z, b4[j].z, acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[i].w, b4[j].w, acc[i][j], 0, 0, 0);
      }
    if (st + 1 < total) K6_STASH(b ^ 1);
    __syncthreads();
  }
#undef K6_FETCH
#undef K6_STASH
  // lane (g, r16) holds rows 4 g + e (o), column r16 (c) of each fragment
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int o = o0 + wm * 64 + i * 16 + g * 4 + e, c = c0 + wn * 64 + j * 16 + r16;
        if (o < O && c < C) part[(((size_t)s * O + o) * C + c) * 9 + t] = acc[i][j][e];
      }
}

// wgrad partials on split f16 products: the same GEMM as k6_wgrad_kernel with
// the operands scaled by powers of two (2^a on gy, 2^b on x, a / b from the
// tensors' max |.|: split_exp_of) and split into f16 hi + lo while they are
// staged (fp32 loads, as above), three v_mfma_f32_16x16x32_f16 products per
// fragment pair (lo.hi, hi.hi, hi.lo: the heatmap convs' fp32-accurate
// split), fp32 accumulation, unscaled by 2^-(a + b) at the
// store.  K-steps of 32 positions; an LDS row = [hi 32 | lo 32] f16 + 16 B pad
// (conflict-free b128 fragment reads).
// NWM x NWN waves of 64 x 16 FJ: tiles of 64 NWM (o) x 16 FJ NWN (c); the
// larger tiles stage fewer operand bytes per MFMA (256 x 256: half of 128 x
// 128's)
constexpr int kWsK = 32, kWsRow = 144;
template <int NWM, int NWN, int FJ>
__global__ __launch_bounds__(64 * NWM * NWN) void k6_wgrad_split_kernel(const float* __restrict__ gyP,
                                                                        const float* __restrict__ xP,
                                                                        const float* __restrict__ amax, int N, int Op,
                                                                        int Cp, int O, int C, int W2, int Qs, int ips,
                                                                        float* __restrict__ part) {
  constexpr int NT = 64 * NWM * NWN, TM = 64 * NWM, TN = 16 * FJ * NWN, RP = NT / 8, UA = TM / RP, UBn = TN / RP;
  __shared__ __attribute__((aligned(16))) char As[2][TM * kWsRow];
  __shared__ __attribute__((aligned(16))) char Bs[2][TN * kWsRow];
  const int c0 = blockIdx.x * TN, o0 = blockIdx.y * TM, t = blockIdx.z % 9, s = blockIdx.z / 9;
  const int off = (t / 3 - 1) * W2 + (t % 3 - 1);
  const int n0 = s * ips, n1 = min(N, n0 + ips);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave / NWN, wn = wave % NWN;
  const int g = lane >> 4, r16 = lane & 15;
  const int lrow = tid >> 3, lq = (tid & 7) * 4;   // loader: rows lrow + RP u; positions lq .. lq + 3
  const int ea = split_exp_of(amax[0]), eb = split_exp_of(amax[1]);
  const float sa = ldexpf(1.f, ea), sb = ldexpf(1.f, eb), us = ldexpf(1.f, -(ea + eb));
  f32x4 acc[4][FJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int total = (n1 - n0) * (Qs / kWsK);
  const float* pa = gyP + ((size_t)n0 * Op + o0 + lrow) * Qs + lq;
  const float* pb = xP + ((size_t)n0 * Cp + c0 + lrow) * Qs + lq + off;
  const size_t r32 = (size_t)RP * Qs, ajump = (size_t)(Op - 1) * Qs, bjump = (size_t)(Cp - 1) * Qs;
  int fq = 0;
  float4 ra[UA], rb[UBn];
#define K6S_FETCH()                                                                                   \
  do {                                                                                                \
    _Pragma("unroll") for (int u = 0; u < UA; ++u)                                                    \
      ra[u] = *reinterpret_cast<const float4*>(pa + u * r32);                                         \
    _Pragma("unroll") for (int u = 0; u < UBn; ++u) {                                                 \
      const float* q = pb + u * r32;                                                                  \
      rb[u] = make_float4(q[0], q[1], q[2], q[3]);                                                    \
    }                                                                                                 \
    pa += kWsK;                                                                                       \
    pb += kWsK;                                                                                       \
    if ((fq += kWsK) == Qs) { fq = 0; pa += ajump; pb += bjump; }                                     \
  } while (0)
#define K6S_PUT(dst, v, sc)                                                                           \
  do {                                                                                                \
    const float e4[4] = {(v).x * (sc), (v).y * (sc), (v).z * (sc), (v).w * (sc)};                     \
    f16x4 hi, lo;                                                                                     \
    _Pragma("unroll") for (int e = 0; e < 4; ++e) {                                                   \
      hi[e] = (_Float16)e4[e];                                                                        \
      lo[e] = (_Float16)(e4[e] - (float)hi[e]);                                                       \
    }                                                                                                 \
    *reinterpret_cast<f16x4*>(dst) = hi;                                                              \
    *reinterpret_cast<f16x4*>((dst) + 64) = lo;                                                       \
  } while (0)
#define K6S_STASH(b)                                                                                  \
  do {                                                                                                \
    _Pragma("unroll") for (int u = 0; u < UA; ++u)                                                    \
      K6S_PUT(&As[b][(lrow + RP * u) * kWsRow + lq * 2], ra[u], sa);                                  \
    _Pragma("unroll") for (int u = 0; u < UBn; ++u)                                                   \
      K6S_PUT(&Bs[b][(lrow + RP * u) * kWsRow + lq * 2], rb[u], sb);                                  \
  } while (0)
  if (total > 0) {
    K6S_FETCH();
    K6S_STASH(0);
  }
  __syncthreads();
  for (int st = 0; st < total; ++st) {
    const int b = st & 1;
    if (st + 1 < total) K6S_FETCH();
    f16x8 ah[4], al[4], bh[FJ], bl[FJ];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const char* q = &As[b][(wm * 64 + i * 16 + r16) * kWsRow + g * 16];
      ah[i] = *reinterpret_cast<const f16x8*>(q);
      al[i] = *reinterpret_cast<const f16x8*>(q + 64);
    }
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const char* q = &Bs[b][(wn * 16 * FJ + j * 16 + r16) * kWsRow + g * 16];
      bh[j] = *reinterpret_cast<const f16x8*>(q);
      bl[j] = *reinterpret_cast<const f16x8*>(q + 64);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
      }
    if (st + 1 < total) K6S_STASH(b ^ 1);
    __syncthreads();
  }
#undef K6S_FETCH
#undef K6S_PUT
#undef K6S_STASH
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int o = o0 + wm * 64 + i * 16 + g * 4 + e, c = c0 + wn * 16 * FJ + j * 16 + r16;
        if (o < O && c < C) part[(((size_t)s * O + o) * C + c) * 9 + t] = acc[i][j][e] * us;
      }
}

}  // namespace

// split forward / dgrad shape: 56 x 56 maps, cin 64 | 256, cout 64 | 256
// (64 runs as a 128-column tile with zero weights in columns 64 .. 127)
static bool k6_split_ok(int N, int cin, int cout, int H, int W) {
  return H == kHmSide && W == kHmSide && (cin == 64 || cin == 256) && (cout == 64 || cout == 256) &&
         (long)N * kHmRoiPos * cin * 4 < (1L << 31);
}

static bool k6_generic() {   // A/B switch (diagnostic build): the round-3 fp32 kernels for all three
  static const bool g = kpd_diag_env("KPD_K6_GENERIC") != nullptr;
  return g;
}

// y [N][cout][56][56] = conv3x3(x [N][cin][56][56], w) (+ b) on the split
// hmconv path; w already oriented [cout][cin][3][3] unless flip (dgrad: w is
// the forward's [cin][cout][3][3] and is transposed / tap-reversed here)
static hipError_t k6_split_conv(const float* x, const float* w, const float* b, int N, int cin, int cout, int flip,
                                float* y, hipStream_t st) {
  const int cout_p = cout == 64 ? 128 : cout;
  const size_t hm_bytes = (size_t)N * kHmRoiPos * cin * 4, ws_elems = (size_t)cout_p * 9 * cin * 2;
  const size_t nhwc = (size_t)N * kHmSide * kHmSide * cout_p;
  char* buf = nullptr;
  const size_t total = hm_bytes + ws_elems * 2 + nhwc * 4 + (size_t)N * 16 + (size_t)cout_p * 4 + 256 * 5;
  hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&buf), total, st);
  if (e != hipSuccess) return e;
  auto carve = [&](size_t bytes) { char* r = buf; buf += (bytes + 255) / 256 * 256; return r; };
  char* base = buf;
  _Float16* hm = reinterpret_cast<_Float16*>(carve(hm_bytes));
  _Float16* ws = reinterpret_cast<_Float16*>(carve(ws_elems * 2));
  float* yn = reinterpret_cast<float*>(carve(nhwc * 4));
  float* hsc = reinterpret_cast<float*>(carve((size_t)N * 16));
  float* zb = reinterpret_cast<float*>(carve((size_t)cout_p * 4));
  float* mx = reinterpret_cast<float*>(carve(4));
  do {
    hipLaunchKernelGGL(k6_hm_border_kernel, dim3((unsigned)N), dim3(256), 0, st, hm, cin);
    if ((e = hipMemsetAsync(hsc, 0, (size_t)N * 16, st)) != hipSuccess) break;
    if (!b || cout_p != cout) {   // the bias padded to the tile's columns (zero for dgrad)
      if ((e = hipMemsetAsync(zb, 0, (size_t)cout_p * 4, st)) != hipSuccess) break;
      if (b && (e = hipMemcpyAsync(zb, b, (size_t)cout * 4, hipMemcpyDeviceToDevice, st)) != hipSuccess) break;
      b = zb;
    }
    const long per_img = (long)cin * kHmSide * kHmSide;
    hipLaunchKernelGGL(k6_amax_kernel, dim3(64, (unsigned)N), dim3(256), 0, st, x, per_img, hsc);
    if ((e = hipGetLastError()) != hipSuccess) break;
    if ((e = hipMemsetAsync(mx, 0, sizeof(float), st)) != hipSuccess) break;
    hipLaunchKernelGGL(k6_max_kernel, dim3(64), dim3(256), 0, st, w, (long)cin * cout * 9, mx);
    hipLaunchKernelGGL(k6_bound_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, hsc, N, mx);
    hipLaunchKernelGGL(k6_to_hm_kernel, dim3((kHmSide * kHmSide + 63) / 64, (unsigned)(cin / 32), (unsigned)N), dim3(256),
                       0, st, x, cin, hsc, hm);
    const long nw = (long)cout_p * 9 * cin;
    hipLaunchKernelGGL(k6_pack_w_kernel, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, st, w, flip ? cin : cout,
                       flip ? cout : cin, flip, mx, cout_p, ws);
    if ((e = hipGetLastError()) != hipSuccess) break;
    HmConvArgs h{};
    h.in = hm; h.wt = ws; h.bias = b; h.outf = yn; h.R = N; h.cin = cin; h.cout = cout_p;
    h.split = 1; h.hsc = hsc; h.in_c = 0.f; h.in_s = 1.f; h.in_idx = 1; h.out_idx = -1; h.amax_idx = -1;
    h.w_exp = 0;
    if ((e = launch_hmconv(h, st)) != hipSuccess) break;
    hipLaunchKernelGGL(k6_nhwc_nchw_kernel, dim3((kHmSide * kHmSide + 63) / 64, (unsigned)((cout + 63) / 64), (unsigned)N),
                       dim3(256), 0, st, yn, cout, cout_p, y);
    e = hipGetLastError();
  } while (false);
  const hipError_t ef = hipFreeAsync(base, st);
  return e != hipSuccess ? e : ef;
}

// gw [O][C][3][3] (and gb [O] when non-null, from the gy plane pass) on the
// padded-plane GEMM (any shape)
static hipError_t k6_wgrad(const float* x, const float* gy, int N, int C, int H, int W, int O, float* gw, float* gb,
                           hipStream_t st) {
  // split f16 products (default) or exact fp32 products (KPD_K6_WG32, diagnostic A/B)
  static const bool fp32 = kpd_diag_env("KPD_K6_WG32") != nullptr;
  const int W2 = W + 2, Qs = ((H + 2) * W2 + kWsK - 1) / kWsK * kWsK, G = W + 3;
  // split tiles: 256 rows / columns where the channel count exceeds 128
  // (conv 2: one 256 x 256 tile per tap), else 128
  const int TM = (!fp32 && O > kWgT) ? 256 : kWgT, TN = (!fp32 && C > kWgT) ? 256 : kWgT;
  const int Cp = (C + TN - 1) / TN * TN, Op = (O + TM - 1) / TM * TM;
  const int tiles = (Cp / TN) * (Op / TM) * 9;
  // images per K slice: the fewest-rounds x longest-slice product over the
  // resident slots (split: 72 KB of LDS, 2 workgroups per CU; fp32: 4)
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
  }
  const long slots = (long)ncu * (fp32 ? 4 : TM * TN > kWgT * kWgT ? 1 : 2);   // resident per CU (LDS)
  int ips = N;
  long best = -1;
  for (int i = 1; i <= N; ++i) {
    const long S = (N + i - 1) / i, cost = ((S * tiles + slots - 1) / slots) * i;
    if (best < 0 || cost < best) { best = cost; ips = i; }
  }
  const int S = (N + ips - 1) / ips;
  const size_t xb = ((size_t)N * Cp * Qs + 2 * G) * 4, gyb = (size_t)N * Op * Qs * 4, pb = (size_t)S * O * C * 9 * 4;
  const size_t sb = gb ? (size_t)N * O * 4 : 0, mb = (size_t)N * (Cp + Op) * 4;
  char* buf = nullptr;
  hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&buf), xb + gyb + pb + sb + mb + 1536, st);
  if (e != hipSuccess) return e;
  char* base = buf;
  auto carve = [&](size_t bytes) { char* r = buf; buf += (bytes + 255) / 256 * 256; return r; };
  float* xP = reinterpret_cast<float*>(carve(xb));
  float* gyP = reinterpret_cast<float*>(carve(gyb));
  float* part = reinterpret_cast<float*>(carve(pb));
  float* mx = reinterpret_cast<float*>(carve(8));
  float* psum = gb ? reinterpret_cast<float*>(carve(sb)) : nullptr;
  float* pmx = reinterpret_cast<float*>(carve(mb));   // per-plane max |.|: x planes, then gy planes
  do {
    // the guards at both ends of xP; max |gy|, max |x| from the plane passes
    if ((e = hipMemsetAsync(xP, 0, (size_t)G * 4, st)) != hipSuccess) break;
    if ((e = hipMemsetAsync(xP + G + (size_t)N * Cp * Qs, 0, (size_t)G * 4, st)) != hipSuccess) break;
    hipLaunchKernelGGL(k6_plane_kernel, dim3((unsigned)Cp, (unsigned)N), dim3(256), 0, st, x, C, H, W, Cp, Qs, xP + G,
                       pmx, nullptr);
    hipLaunchKernelGGL(k6_plane_kernel, dim3((unsigned)Op, (unsigned)N), dim3(256), 0, st, gy, O, H, W, Op, Qs, gyP,
                       pmx + (size_t)N * Cp, psum);
    hipLaunchKernelGGL(k6_max_finish_kernel, dim3(1), dim3(256), 0, st, pmx + (size_t)N * Cp, (long)N * Op, mx);
    hipLaunchKernelGGL(k6_max_finish_kernel, dim3(1), dim3(256), 0, st, pmx, (long)N * Cp, mx + 1);
    if (gb) hipLaunchKernelGGL(k6_bias_finish_kernel, dim3((unsigned)((O + 255) / 256)), dim3(256), 0, st, psum, N, O, gb);
    const dim3 grid((unsigned)(Cp / TN), (unsigned)(Op / TM), (unsigned)(9 * S));
    if (fp32) {
      hipLaunchKernelGGL(k6_wgrad_kernel, grid, dim3(256), 0, st, gyP, xP + G, N, Op, Cp, O, C, W2, Qs, ips, part);
    } else {
#define K6S_LAUNCH(M_, N_, F_)                                                                              \
  hipLaunchKernelGGL((k6_wgrad_split_kernel<M_, N_, F_>), grid, dim3(64 * M_ * N_), 0, st, gyP, xP + G, mx, N, Op, \
                     Cp, O, C, W2, Qs, ips, part)
      if (TM == 256 && TN == 256) K6S_LAUNCH(4, 2, 8);
      else if (TM == 256) K6S_LAUNCH(4, 2, 4);
      else if (TN == 256) K6S_LAUNCH(2, 4, 4);
      else K6S_LAUNCH(2, 2, 4);
#undef K6S_LAUNCH
    }
    const long n = (long)O * C * 9;
    hipLaunchKernelGGL(slice_sum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, part, S, n, gw);
    e = hipGetLastError();
  } while (false);
  const hipError_t ef = hipFreeAsync(base, st);
  return e != hipSuccess ? e : ef;
}

// gb [O] alone: plane sums of gy, summed over the images in order
static hipError_t k6_bias(const float* gy, int N, int O, int H, int W, float* gb, hipStream_t st) {
  float* psum = nullptr;
  hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&psum), (size_t)N * O * 4, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k6_plane_kernel, dim3((unsigned)O, (unsigned)N), dim3(256), 0, st, gy, O, H, W, O,
                     (H + 2) * (W + 2), nullptr, nullptr, psum);
  hipLaunchKernelGGL(k6_bias_finish_kernel, dim3((unsigned)((O + 255) / 256)), dim3(256), 0, st, psum, N, O, gb);
  e = hipGetLastError();
  const hipError_t ef = hipFreeAsync(psum, st);
  return e != hipSuccess ? e : ef;
}

hipError_t launch_conv3_forward(const float* x, const float* w, const float* b, int N, int C, int H, int W, int O,
                                float* y, hipStream_t st) {
  if (N <= 0) return hipSuccess;
  if (!k6_generic() && k6_split_ok(N, C, O, H, W)) return k6_split_conv(x, w, b, N, C, O, 0, y, st);
  const dim3 grid((unsigned)((H * W + TB - 1) / TB), (unsigned)((O + TB - 1) / TB), (unsigned)N);
  hipLaunchKernelGGL(conv3_gemm_kernel<C3_FWD>, grid, dim3(256), 0, st, x, w, nullptr, b, C, H, W, O, 0, 0, y);
  return hipGetLastError();
}

size_t conv3_wgrad_slices(int N, int H, int W) {
  if (!k6_generic()) return 0;   // the fast wgrad allocates its own scratch
  const long K = (long)N * H * W;
  const long ks = 4096;
  return (size_t)((K + ks - 1) / ks);
}

hipError_t launch_conv3_backward(const float* x, const float* w, const float* gy, int N, int C, int H, int W, int O,
                                 float* gx, float* gw, float* gb, float* wgrad_part, hipStream_t st) {
  if (N <= 0) return hipSuccess;
  const int HW = H * W;
  const bool generic = k6_generic();
  if (gx && !generic && k6_split_ok(N, O, C, H, W)) {
    const hipError_t e = k6_split_conv(gy, w, nullptr, N, O, C, 1, gx, st);
    if (e != hipSuccess) return e;
    gx = nullptr;
  }
  if (gw && !generic) {
    const hipError_t e = k6_wgrad(x, gy, N, C, H, W, O, gw, gb, st);
    if (e != hipSuccess) return e;
    gw = gb = nullptr;
  }
  if (gb && !generic) {
    const hipError_t e = k6_bias(gy, N, O, H, W, gb, st);
    if (e != hipSuccess) return e;
    gb = nullptr;
  }
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
