// Preprocessing on the GPU: the reference's ITransform (dll/data/transforms.py:
// 9-113) without OpenCV or PIL on the host.
//
//   uint8 HWC image (device) --[RGB->gray]--[CLAHE per plane]--[edge blend]
//       --[Gaussian 3x3]--PIL-exact bilinear resize--ToTensor/Normalize--> fp32 CHW (device)
//
// * Resize reproduces Pillow's ImagingResample for 8-bit images bit for bit
//   (Resample.c): coefficients from precompute_coeffs in double, converted to
//   22-bit fixed point by normalize_coeffs_8bpc; horizontal pass first with the
//   intermediate rounded and clipped to uint8, then the vertical pass.  The
//   coefficients are computed on the device in IEEE double with contraction
//   off, so they equal Pillow's.  Pinned by tests/golden/preprocess.npz (real
//   Pillow 12.2 outputs).
// * ToTensor / Normalize: x = (u8 / 255.f - mean) / std, the same fp32 ops as
//   torchvision (a division, not a reciprocal multiply).
// * CLAHE follows OpenCV's cv::CLAHE for CV_8U (clahe.cpp): reflect-101 pad
//   to a tile multiple, 256-bin tile histograms (integer LDS atomics, so the
//   counts are deterministic), clip + batch/strided-residual redistribution,
//   LUT = saturate_cast<uchar>(cumsum * (255 / area)), bilinear blend of four
//   tile LUTs in fp32 without contraction, round-half-even.  Gray conversion is
//   cv::cvtColor(RGB2GRAY) fixed point; Gaussian blurs follow GaussianBlur's
//   8U fixed-point path; the grayscale edge blend is GaussianBlur 5x5 ->
//   medianBlur 5 -> Canny(100, 200, L1) -> (dilate, erode) x 2 -> GaussianBlur
//   3x3 -> scale to 255 -> addWeighted(0.7, 0.3).
//   OpenCV is absent here and on the GPU box: these stages are parity
//   unpinned (see oracle/preprocess_oracle.py).
#include <algorithm>
#include <cmath>
#include <vector>

#include "../../include/kpd.h"
#include "kpd_common.h"
#include "kpd_kernels.h"

#pragma clang fp contract(off)

namespace {

constexpr int kPrecisionBits = 32 - 8 - 2;

// Pillow precompute_coeffs (bilinear, support 1) + normalize_coeffs_8bpc.
// One thread per output coordinate; bounds [out][2], kk [out][ksize] int32.
__global__ void resize_coeffs_kernel(int in_size, int out_size, int ksize, int* bounds, int* kk) {
  const int xx = blockIdx.x * blockDim.x + threadIdx.x;
  if (xx >= out_size) return;
  const double scale = (double)in_size / (double)out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = filterscale;
  const double center = (xx + 0.5) * scale;
  const double ss = 1.0 / filterscale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  xmax -= xmin;
  double w[64];
  double ww = 0.0;
  for (int x = 0; x < xmax && x < 64; ++x) {
    double t = (x + xmin - center + 0.5) * ss;
    t = t < 0.0 ? -t : t;
    w[x] = t < 1.0 ? 1.0 - t : 0.0;
    ww += w[x];
  }
  for (int x = 0; x < ksize; ++x) {
    int v = 0;
    if (x < xmax) {
      const double k = ww != 0.0 ? w[x] / ww : w[x];
      v = k < 0 ? (int)(-0.5 + k * (1 << kPrecisionBits)) : (int)(0.5 + k * (1 << kPrecisionBits));
    }
    kk[xx * ksize + x] = v;
  }
  bounds[2 * xx] = xmin;
  bounds[2 * xx + 1] = xmax;
}

__device__ __forceinline__ unsigned char clip8(int v) {
  if (v >= (1 << kPrecisionBits << 8)) return 255;
  if (v <= 0) return 0;
  return (unsigned char)(v >> kPrecisionBits);
}

// horizontal pass: rows [y0, y0 + rows) of src -> tmp [rows][OW][C]
__global__ void resize_h_kernel(const unsigned char* __restrict__ src, int pitch, int C, int y0, int rows, int OW,
                                int ksize, const int* __restrict__ bounds, const int* __restrict__ kk,
                                unsigned char* __restrict__ tmp) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)rows * OW * C) return;
  const int c = i % C, xx = (i / C) % OW, y = (int)(i / ((long)C * OW));
  const int xmin = bounds[2 * xx], n = bounds[2 * xx + 1];
  const unsigned char* row = src + (size_t)(y0 + y) * pitch;
  int acc = 1 << (kPrecisionBits - 1);
  for (int x = 0; x < n; ++x) acc += (int)row[(xmin + x) * C + c] * kk[xx * ksize + x];
  tmp[i] = clip8(acc);
}

// vertical pass + ToTensor + Normalize: tmp [rows][OW][C] -> dst fp32 [C][OH][OW]
__global__ void resize_v_norm_kernel(const unsigned char* __restrict__ tmp, int OW, int C, int OH, int ksize,
                                     const int* __restrict__ bounds, const int* __restrict__ kk, int y_shift,
                                     float m0, float m1, float m2, float s0, float s1, float s2,
                                     float* __restrict__ dst) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)OH * OW * C) return;
  const int xx = i % OW, yy = (i / OW) % OH, c = (int)(i / ((long)OW * OH));
  const int ymin = bounds[2 * yy] - y_shift, n = bounds[2 * yy + 1];
  int acc = 1 << (kPrecisionBits - 1);
  for (int y = 0; y < n; ++y) acc += (int)tmp[((size_t)(ymin + y) * OW + xx) * C + c] * kk[yy * ksize + y];
  const float mean = c == 0 ? m0 : (c == 1 ? m1 : m2), sd = c == 0 ? s0 : (c == 1 ? s1 : s2);
  const float x = (float)clip8(acc) / 255.f;
  dst[i] = (x - mean) / sd;
}

// cv::cvtColor(RGB2GRAY), 8U fixed point (yuv coefficients << 14)
__global__ void rgb2gray_kernel(const unsigned char* __restrict__ src, int pitch, int H, int W,
                                unsigned char* __restrict__ dst) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= H * W) return;
  const int y = i / W, x = i - y * W;
  const unsigned char* p = src + (size_t)y * pitch + x * 3;
  dst[i] = (unsigned char)((p[0] * 4899 + p[1] * 9617 + p[2] * 1868 + (1 << 13)) >> 14);
}

__device__ __forceinline__ int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
}

// one workgroup per (tile, plane): histogram -> clip/redistribute -> LUT
__global__ __launch_bounds__(256) void clahe_lut_kernel(const unsigned char* __restrict__ src, int pitch, int C,
                                                        int H, int W, int tiles_x, int tiles_y, int tw, int th,
                                                        int clip, unsigned char* __restrict__ luts) {
  __shared__ int hist[256];
  const int tx = blockIdx.x, ty = blockIdx.y, c = blockIdx.z, tid = threadIdx.x;
  hist[tid] = 0;
  __syncthreads();
  for (int i = tid; i < tw * th; i += 256) {
    const int y = reflect101(ty * th + i / tw, H), x = reflect101(tx * tw + i % tw, W);
    atomicAdd(&hist[src[(size_t)y * pitch + x * C + c]], 1);
  }
  __syncthreads();
  if (tid == 0) {
    if (clip > 0) {
      int clipped = 0;
      for (int i = 0; i < 256; ++i)
        if (hist[i] > clip) { clipped += hist[i] - clip; hist[i] = clip; }
      const int batch = clipped / 256;
      int residual = clipped - batch * 256;
      for (int i = 0; i < 256; ++i) hist[i] += batch;
      if (residual != 0) {
        const int step = max(256 / residual, 1);
        for (int i = 0; i < 256 && residual > 0; i += step, --residual) hist[i]++;
      }
    }
    const float lut_scale = 255.f / (float)(tw * th);
    int sum = 0;
    unsigned char* lut = luts + ((size_t)(c * tiles_y + ty) * tiles_x + tx) * 256;
    for (int i = 0; i < 256; ++i) {
      sum += hist[i];
      lut[i] = (unsigned char)min(max(__float2int_rn((float)sum * lut_scale), 0), 255);
    }
  }
}

__global__ void clahe_apply_kernel(const unsigned char* __restrict__ src, int pitch, int C, int H, int W,
                                   int tiles_x, int tiles_y, int tw, int th, const unsigned char* __restrict__ luts,
                                   unsigned char* __restrict__ dst) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)H * W * C) return;
  const int c = i % C, x = (i / C) % W, y = (int)(i / ((long)C * W));
  const float inv_tw = 1.f / (float)tw, inv_th = 1.f / (float)th;
  const float tyf = (float)y * inv_th - 0.5f, txf = (float)x * inv_tw - 0.5f;
  int ty1 = (int)floorf(tyf), tx1 = (int)floorf(txf);
  const float ya = tyf - (float)ty1, ya1 = 1.f - ya, xa = txf - (float)tx1, xa1 = 1.f - xa;
  const int ty2 = min(ty1 + 1, tiles_y - 1), tx2 = min(tx1 + 1, tiles_x - 1);
  ty1 = max(ty1, 0);
  tx1 = max(tx1, 0);
  const int v = src[(size_t)y * pitch + x * C + c];
  const unsigned char* lp = luts + (size_t)c * tiles_y * tiles_x * 256;
  const float l11 = lp[(ty1 * tiles_x + tx1) * 256 + v], l12 = lp[(ty1 * tiles_x + tx2) * 256 + v];
  const float l21 = lp[(ty2 * tiles_x + tx1) * 256 + v], l22 = lp[(ty2 * tiles_x + tx2) * 256 + v];
  const float r = (l11 * xa1 + l12 * xa) * ya1 + (l21 * xa1 + l22 * xa) * ya;
  dst[i] = (unsigned char)min(max(__float2int_rn(r), 0), 255);
}

// cv::GaussianBlur for CV_8U (the fixed-point path): kernel taps carry 8
// fraction bits and sum to 256; the row sum and the column sum are exact
// integers, the result is rounded half up from 16 fraction bits.  Reflect-101.
struct GaussTaps {
  int n;
  int k[7];
};

__global__ void gauss_fixed_kernel(const unsigned char* __restrict__ src, int pitch, int C, int H, int W, GaussTaps g,
                                   unsigned char* __restrict__ dst) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)H * W * C) return;
  const int c = i % C, x = (i / C) % W, y = (int)(i / ((long)C * W));
  const int r = g.n / 2;
  int v = 0;
  for (int dy = 0; dy < g.n; ++dy) {
    const unsigned char* row = src + (size_t)reflect101(y + dy - r, H) * pitch;
    int h = 0;
    for (int dx = 0; dx < g.n; ++dx) h += g.k[dx] * (int)row[reflect101(x + dx - r, W) * C + c];
    v += g.k[dy] * h;
  }
  dst[i] = (unsigned char)min((v + (1 << 15)) >> 16, 255);
}

// cv::medianBlur(5) on one plane, replicated border.  The median is the value
// whose rank window [#less, #less-or-equal) holds 12; fully unrolled compares
// keep the 25 samples in registers.
__global__ void median5_kernel(const unsigned char* __restrict__ src, int H, int W, unsigned char* __restrict__ dst) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= H * W) return;
  const int y = i / W, x = i - y * W;
  int v[25];
#pragma unroll
  for (int dy = 0; dy < 5; ++dy) {
    const unsigned char* row = src + (size_t)min(max(y + dy - 2, 0), H - 1) * W;
#pragma unroll
    for (int dx = 0; dx < 5; ++dx) v[dy * 5 + dx] = row[min(max(x + dx - 2, 0), W - 1)];
  }
  int med = v[0];
#pragma unroll
  for (int a = 0; a < 25; ++a) {
    int lt = 0, le = 0;
#pragma unroll
    for (int b = 0; b < 25; ++b) {
      lt += v[b] < v[a];
      le += v[b] <= v[a];
    }
    med = (lt <= 12 && le > 12) ? v[a] : med;
  }
  dst[i] = (unsigned char)med;
}

// Canny step 1: 3x3 Sobel (replicated border), L1 magnitude.
__global__ void canny_grad_kernel(const unsigned char* __restrict__ src, int H, int W, int* __restrict__ dxy,
                                  int* __restrict__ mag) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= H * W) return;
  const int y = i / W, x = i - y * W;
  const int y0 = max(y - 1, 0), y2 = min(y + 1, H - 1), x0 = max(x - 1, 0), x2 = min(x + 1, W - 1);
  auto at = [&](int yy, int xx) { return (int)src[(size_t)yy * W + xx]; };
  const int dx = (at(y0, x2) + 2 * at(y, x2) + at(y2, x2)) - (at(y0, x0) + 2 * at(y, x0) + at(y2, x0));
  const int dy = (at(y2, x0) + 2 * at(y2, x) + at(y2, x2)) - (at(y0, x0) + 2 * at(y0, x) + at(y0, x2));
  dxy[2 * i] = dx;
  dxy[2 * i + 1] = dy;
  mag[i] = abs(dx) + abs(dy);
}

// Canny step 2: non-maximum suppression with OpenCV's fixed-point sector
// test (tan 22.5 deg in Q15), magnitude 0 outside the image.  map: 0 = not
// an edge, 1 = candidate (m > low), 2 = seed (m > high, appended to queue).
constexpr int kCannyTg22 = 13573;   // (int)(tan(22.5 deg) * 2^15 + 0.5)

__global__ void canny_nms_kernel(const int* __restrict__ dxy, const int* __restrict__ mag, int H, int W, int low,
                                 int high, int* __restrict__ map, int* __restrict__ queue, int* __restrict__ qn) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= H * W) return;
  const int y = i / W, x = i - y * W;
  auto M = [&](int yy, int xx) { return (yy < 0 || yy >= H || xx < 0 || xx >= W) ? 0 : mag[(size_t)yy * W + xx]; };
  const int m = mag[i];
  int state = 0;
  if (m > low) {
    const int dx = dxy[2 * i], dy = dxy[2 * i + 1];
    const long ax = abs(dx), ay = (long)abs(dy) << 15;
    const long tg22x = ax * kCannyTg22, tg67x = tg22x + (ax << 16);
    bool keep;
    if (ay < tg22x) {
      keep = m > M(y, x - 1) && m >= M(y, x + 1);
    } else if (ay > tg67x) {
      keep = m > M(y - 1, x) && m >= M(y + 1, x);
    } else {
      const int s = (dx ^ dy) < 0 ? -1 : 1;
      keep = m > M(y - 1, x - s) && m > M(y + 1, x + s);
    }
    if (keep) state = m > high ? 2 : 1;
  }
  map[i] = state;
  if (state == 2) queue[atomicAdd(qn, 1)] = i;
}

// Canny step 3: hysteresis as a breadth-first flood from the seeds over
// 8-connected candidates, in one workgroup (level-synchronous; each pixel
// enters the queue once, so the loop ends after at most H*W pushes).
__global__ __launch_bounds__(1024) void canny_hyst_kernel(int H, int W, int* __restrict__ map,
                                                          int* __restrict__ queue, const int* __restrict__ qn) {
  __shared__ int s_tail;
  const int tid = threadIdx.x;
  if (tid == 0) s_tail = *qn;
  __syncthreads();
  int head = 0, tail = s_tail;
  while (head < tail) {
    for (int q = head + tid; q < tail; q += 1024) {
      const int p = queue[q], y = p / W, x = p - y * W;
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
          const int yy = y + dy, xx = x + dx;
          if ((dy | dx) == 0 || yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
          const int n = yy * W + xx;
          if (map[n] == 1 && atomicCAS(&map[n], 1, 2) == 1) queue[atomicAdd(&s_tail, 1)] = n;
        }
    }
    __syncthreads();
    head = tail;
    tail = s_tail;
    __syncthreads();
  }
}

// 3x3 ones dilate (DIL) / erode on one plane; the out-of-image value never
// wins.  FROM_MAP reads the Canny map (2 -> 255) instead of a u8 image.
template <bool DIL, bool FROM_MAP>
__global__ void morph3_kernel(const void* __restrict__ src_, int H, int W, unsigned char* __restrict__ dst) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= H * W) return;
  const int y = i / W, x = i - y * W;
  int r = DIL ? 0 : 255;
  for (int yy = max(y - 1, 0); yy <= min(y + 1, H - 1); ++yy)
    for (int xx = max(x - 1, 0); xx <= min(x + 1, W - 1); ++xx) {
      const size_t j = (size_t)yy * W + xx;
      const int v = FROM_MAP ? (static_cast<const int*>(src_)[j] == 2 ? 255 : 0)
                             : (int)static_cast<const unsigned char*>(src_)[j];
      r = DIL ? max(r, v) : min(r, v);
    }
  dst[i] = (unsigned char)r;
}

__global__ void max_u8_kernel(const unsigned char* __restrict__ src, int n, int* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  int v = i < n ? (int)src[i] : 0;
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  if ((threadIdx.x & 63) == 0 && v > 0) atomicMax(out, v);
}

// normalized_edges = uint8(edges / max * 255) in double (truncating), then
// cv::addWeighted(base, 0.7, edges, 0.3, 0): fp32 fma(a, .7f, fma(b, .3f, 0)),
// round half even, saturate.
__global__ void edge_blend_kernel(const unsigned char* __restrict__ base, const unsigned char* __restrict__ edges,
                                  const int* __restrict__ maxp, int n, unsigned char* __restrict__ dst) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int mx = *maxp;
  int e = edges[i];
  if (mx > 0) e = (int)((double)e / (double)mx * 255.0);
  const float t = __fmaf_rn((float)base[i], 0.7f, __fmaf_rn((float)e, 0.3f, 0.f));
  dst[i] = (unsigned char)min(max(__float2int_rn(t), 0), 255);
}

// cv::getGaussianKernelBitExact + getGaussianKernelFixedPoint_ED (8 bits)
GaussTaps gauss_taps(int n, double sigma) {
  double r[7] = {0};
  const int n2 = (n - 1) / 2;
  if (sigma <= 0 && n <= 7) {
    static const double t3[] = {0.25, 0.5, 0.25}, t5[] = {0.0625, 0.25, 0.375, 0.25, 0.0625},
                        t7[] = {0.03125, 0.109375, 0.21875, 0.28125, 0.21875, 0.109375, 0.03125};
    const double* t = n == 3 ? t3 : (n == 5 ? t5 : t7);
    for (int i = 0; i < n; ++i) r[i] = n == 1 ? 1.0 : t[i];
  } else {
    const double sig = sigma > 0 ? sigma : n * 0.15 + 0.35, scale2x = -0.125 / (sig * sig);
    double vals[3], sum = 0.0;
    for (int i = 0; i < n2; ++i) {
      const int x = 2 * i + 1 - n;
      vals[i] = std::exp((double)(x * x) * scale2x);
      sum += vals[i];
    }
    sum = sum * 2.0 + 1.0;
    const double mul1 = 1.0 / sum;
    for (int i = 0; i < n2; ++i) r[i] = r[n - 1 - i] = vals[i] * mul1;
    r[n2] = mul1;
  }
  GaussTaps g{};
  g.n = n;
  double err = 0.0;
  int s = 0;
  for (int i = 0; i < n2; ++i) {
    const double adj = r[i] * 256.0 + err;
    const int v0 = (int)std::nearbyint(adj);   // cvRound (half to even)
    err = adj - v0;
    g.k[i] = g.k[n - 1 - i] = v0;
    s += v0;
  }
  g.k[n2] = 256 - 2 * s;
  return g;
}

inline unsigned blocks(long n) { return (unsigned)((n + 255) / 256); }

// host copy of precompute_coeffs' bounds for one output coordinate (same
// double arithmetic as resize_coeffs_kernel): first source row and count
void pil_bounds(int in_size, int out_size, int xx, int* xmin_out, int* n_out) {
  const double scale = (double)in_size / (double)out_size;
  const double support = scale < 1.0 ? 1.0 : scale;
  const double center = (xx + 0.5) * scale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  *xmin_out = xmin;
  *n_out = xmax - xmin;
}

}  // namespace

extern "C" int kpd_preprocess(const uint8_t* src, int H, int W, int C, int pitch, int flags, float clip_limit,
                              int tiles_x, int tiles_y, int out_h, int out_w, const float* mean, const float* std_,
                              float* dst, void* stream) {
  if (!src || !dst || !mean || !std_ || H <= 0 || W <= 0 || out_h <= 0 || out_w <= 0 || (C != 1 && C != 3) ||
      pitch < W * C)
    return kpd_fail_einval("kpd_preprocess: bad arguments");
  if ((flags & KPD_PRE_GRAY) && C != 3) return kpd_fail_einval("kpd_preprocess: GRAY needs a 3-channel image");
  if ((flags & KPD_PRE_EDGES) && !((flags & KPD_PRE_GRAY) || C == 1))
    return kpd_fail_einval("kpd_preprocess: EDGES needs a single-plane (gray) pipeline");
  if ((flags & KPD_PRE_CLAHE) && (tiles_x <= 0 || tiles_y <= 0 || tiles_x > W || tiles_y > H))
    return kpd_fail_einval("kpd_preprocess: bad CLAHE tile grid");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int Co = (flags & KPD_PRE_GRAY) ? 1 : C;
  std::vector<void*> scratch;
  auto alloc = [&](size_t bytes) -> void* {
    void* p = nullptr;
    if (hipMallocAsync(&p, std::max<size_t>(bytes, 16), st) != hipSuccess) return nullptr;
    scratch.push_back(p);
    return p;
  };
  int rc = KPD_OK;
  auto fail_hip = [&](hipError_t e) {
    if (e != hipSuccess && rc == KPD_OK) rc = kpd_fail_hip(e, "kpd_preprocess");
  };
  const unsigned char* cur = src;
  int cur_pitch = pitch;
  do {
    if (flags & KPD_PRE_GRAY) {
      auto* g = static_cast<unsigned char*>(alloc((size_t)H * W));
      if (!g) { rc = kpd_fail_einval("kpd_preprocess: out of device memory"); break; }
      hipLaunchKernelGGL(rgb2gray_kernel, dim3(blocks((long)H * W)), dim3(256), 0, st, cur, cur_pitch, H, W, g);
      fail_hip(hipGetLastError());
      cur = g;
      cur_pitch = W;
    }
    if (flags & KPD_PRE_CLAHE) {
      const int Hp = H % tiles_y ? H + tiles_y - H % tiles_y : H, Wp = W % tiles_x ? W + tiles_x - W % tiles_x : W;
      const int tw = Wp / tiles_x, th = Hp / tiles_y, area = tw * th;
      const int clip = clip_limit > 0.f ? std::max((int)(clip_limit * area / 256), 1) : 0;
      auto* luts = static_cast<unsigned char*>(alloc((size_t)Co * tiles_y * tiles_x * 256));
      auto* out = static_cast<unsigned char*>(alloc((size_t)H * W * Co));
      if (!luts || !out) { rc = kpd_fail_einval("kpd_preprocess: out of device memory"); break; }
      hipLaunchKernelGGL(clahe_lut_kernel, dim3(tiles_x, tiles_y, Co), dim3(256), 0, st, cur, cur_pitch, Co, H, W,
                         tiles_x, tiles_y, tw, th, clip, luts);
      fail_hip(hipGetLastError());
      hipLaunchKernelGGL(clahe_apply_kernel, dim3(blocks((long)H * W * Co)), dim3(256), 0, st, cur, cur_pitch, Co, H,
                         W, tiles_x, tiles_y, tw, th, luts, out);
      fail_hip(hipGetLastError());
      cur = out;
      cur_pitch = W * Co;
    }
    if (flags & KPD_PRE_EDGES) {   // to_grayscale_clahe's edge blend (transforms.py:55-73)
      const int n = H * W;
      auto* d0 = static_cast<unsigned char*>(alloc((size_t)n));
      auto* d1 = static_cast<unsigned char*>(alloc((size_t)n));
      auto* out = static_cast<unsigned char*>(alloc((size_t)n));
      auto* dxy = static_cast<int*>(alloc(sizeof(int) * 2 * (size_t)n));
      auto* mag = static_cast<int*>(alloc(sizeof(int) * (size_t)n));
      auto* map = static_cast<int*>(alloc(sizeof(int) * (size_t)n));
      auto* queue = static_cast<int*>(alloc(sizeof(int) * (size_t)n));
      auto* cnt = static_cast<int*>(alloc(sizeof(int) * 2));
      if (!d0 || !d1 || !out || !dxy || !mag || !map || !queue || !cnt) {
        rc = kpd_fail_einval("kpd_preprocess: out of device memory");
        break;
      }
      if (cur_pitch != W) {   // the edge kernels read a dense plane
        fail_hip(hipMemcpy2DAsync(out, W, cur, cur_pitch, W, H, hipMemcpyDeviceToDevice, st));
        cur = out;
        cur_pitch = W;
        out = static_cast<unsigned char*>(alloc((size_t)n));
        if (!out) { rc = kpd_fail_einval("kpd_preprocess: out of device memory"); break; }
      }
      fail_hip(hipMemsetAsync(cnt, 0, sizeof(int) * 2, st));
      const unsigned nb = blocks(n);
      hipLaunchKernelGGL(gauss_fixed_kernel, dim3(nb), dim3(256), 0, st, cur, W, 1, H, W, gauss_taps(5, 1.5), d0);
      hipLaunchKernelGGL(median5_kernel, dim3(nb), dim3(256), 0, st, d0, H, W, d1);
      hipLaunchKernelGGL(canny_grad_kernel, dim3(nb), dim3(256), 0, st, d1, H, W, dxy, mag);
      hipLaunchKernelGGL(canny_nms_kernel, dim3(nb), dim3(256), 0, st, dxy, mag, H, W, 100, 200, map, queue, cnt);
      hipLaunchKernelGGL(canny_hyst_kernel, dim3(1), dim3(1024), 0, st, H, W, map, queue, cnt);
      hipLaunchKernelGGL((morph3_kernel<true, true>), dim3(nb), dim3(256), 0, st, map, H, W, d0);
      hipLaunchKernelGGL((morph3_kernel<false, false>), dim3(nb), dim3(256), 0, st, d0, H, W, d1);
      hipLaunchKernelGGL((morph3_kernel<true, false>), dim3(nb), dim3(256), 0, st, d1, H, W, d0);
      hipLaunchKernelGGL((morph3_kernel<false, false>), dim3(nb), dim3(256), 0, st, d0, H, W, d1);
      hipLaunchKernelGGL(gauss_fixed_kernel, dim3(nb), dim3(256), 0, st, d1, W, 1, H, W, gauss_taps(3, 0.0), d0);
      hipLaunchKernelGGL(max_u8_kernel, dim3(nb), dim3(256), 0, st, d0, n, cnt + 1);
      hipLaunchKernelGGL(edge_blend_kernel, dim3(nb), dim3(256), 0, st, cur, d0, cnt + 1, n, out);
      fail_hip(hipGetLastError());
      cur = out;
    }
    if (flags & KPD_PRE_BLUR) {   // GaussianBlur((3, 3), 0.5) of to_rgb_clahe
      auto* out = static_cast<unsigned char*>(alloc((size_t)H * W * Co));
      if (!out) { rc = kpd_fail_einval("kpd_preprocess: out of device memory"); break; }
      hipLaunchKernelGGL(gauss_fixed_kernel, dim3(blocks((long)H * W * Co)), dim3(256), 0, st, cur, cur_pitch, Co, H,
                         W, gauss_taps(3, 0.5), out);
      fail_hip(hipGetLastError());
      cur = out;
      cur_pitch = W * Co;
    }
    // PIL bilinear resize (horizontal pass first) + ToTensor + Normalize
    const double sx = (double)W / out_w, sy = (double)H / out_h;
    const int kx = (int)std::ceil(std::max(sx, 1.0)) * 2 + 1, ky = (int)std::ceil(std::max(sy, 1.0)) * 2 + 1;
    if (kx > 64 || ky > 64) { rc = kpd_fail_einval("kpd_preprocess: downscale factor > 31 not supported"); break; }
    auto* bx = static_cast<int*>(alloc(sizeof(int) * 2 * out_w));
    auto* kkx = static_cast<int*>(alloc(sizeof(int) * (size_t)out_w * kx));
    auto* by = static_cast<int*>(alloc(sizeof(int) * 2 * out_h));
    auto* kky = static_cast<int*>(alloc(sizeof(int) * (size_t)out_h * ky));
    if (!bx || !kkx || !by || !kky) { rc = kpd_fail_einval("kpd_preprocess: out of device memory"); break; }
    hipLaunchKernelGGL(resize_coeffs_kernel, dim3(blocks(out_w)), dim3(256), 0, st, W, out_w, kx, bx, kkx);
    hipLaunchKernelGGL(resize_coeffs_kernel, dim3(blocks(out_h)), dim3(256), 0, st, H, out_h, ky, by, kky);
    fail_hip(hipGetLastError());
    const unsigned char* tmp = cur;
    int y_shift = 0;
    if (out_w != W) {   // rows the vertical pass reads: PIL's ybox [first, last)
      int f0, fn, l0, ln;
      pil_bounds(H, out_h, 0, &f0, &fn);
      pil_bounds(H, out_h, out_h - 1, &l0, &ln);
      const int y0 = out_h != H ? f0 : 0, y1 = out_h != H ? l0 + ln : H;
      auto* t = static_cast<unsigned char*>(alloc((size_t)(y1 - y0) * out_w * Co));
      if (!t) { rc = kpd_fail_einval("kpd_preprocess: out of device memory"); break; }
      hipLaunchKernelGGL(resize_h_kernel, dim3(blocks((long)(y1 - y0) * out_w * Co)), dim3(256), 0, st, cur, cur_pitch,
                         Co, y0, y1 - y0, out_w, kx, bx, kkx, t);
      fail_hip(hipGetLastError());
      tmp = t;
      y_shift = y0;
    } else if (cur_pitch != W * Co) {   // the vertical kernel reads a dense [rows][W][C] image
      auto* t = static_cast<unsigned char*>(alloc((size_t)H * W * Co));
      if (!t) { rc = kpd_fail_einval("kpd_preprocess: out of device memory"); break; }
      fail_hip(hipMemcpy2DAsync(t, (size_t)W * Co, cur, cur_pitch, (size_t)W * Co, H, hipMemcpyDeviceToDevice, st));
      tmp = t;
    }
    const float m1 = Co > 1 ? mean[1] : 0.f, m2 = Co > 2 ? mean[2] : 0.f;
    const float s1 = Co > 1 ? std_[1] : 1.f, s2 = Co > 2 ? std_[2] : 1.f;
    hipLaunchKernelGGL(resize_v_norm_kernel, dim3(blocks((long)out_h * out_w * Co)), dim3(256), 0, st, tmp, out_w, Co,
                       out_h, ky, by, kky, y_shift, mean[0], m1, m2, std_[0], s1, s2, dst);
    fail_hip(hipGetLastError());
  } while (false);
  for (void* p : scratch) (void)hipFreeAsync(p, st);
  return rc;
}
