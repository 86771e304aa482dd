// Preprocessing on the GPU: the reference's ITransform (dll/data/transforms.py:
// 9-113) without OpenCV or PIL on the host.
//
//   uint8 HWC image (device) --[RGB->gray]--[CLAHE per plane]--[Gaussian 3x3]
//       --PIL-exact bilinear resize--ToTensor/Normalize--> fp32 CHW (device)
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
//   cv::cvtColor(RGB2GRAY) fixed point; Gaussian 3x3 is fp32 separable.
//   OpenCV is absent here and on the GPU box: these stages are parity
//   unpinned (see oracle/preprocess_oracle.py).
#include <algorithm>
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

// separable 3x3 Gaussian, reflect-101, fp32, round half even (unpinned vs OpenCV)
__global__ void gauss3_kernel(const unsigned char* __restrict__ src, int pitch, int C, int H, int W, float k0, float k1,
                              unsigned char* __restrict__ dst) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)H * W * C) return;
  const int c = i % C, x = (i / C) % W, y = (int)(i / ((long)C * W));
  const float k[3] = {k0, k1, k0};
  float v = 0.f;
  for (int dy = 0; dy < 3; ++dy) {
    const unsigned char* row = src + (size_t)reflect101(y + dy - 1, H) * pitch;
    float h = 0.f;
    for (int dx = 0; dx < 3; ++dx) h += k[dx] * (float)row[reflect101(x + dx - 1, W) * C + c];
    v += k[dy] * h;
  }
  dst[i] = (unsigned char)min(max(__float2int_rn(v), 0), 255);
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
    if (flags & KPD_PRE_BLUR) {   // GaussianBlur((3, 3), 0.5) of to_rgb_clahe
      const double e = std::exp(-1.0 / (2.0 * 0.25)), s = (e + 1.0) + e;   // summed in index order
      auto* out = static_cast<unsigned char*>(alloc((size_t)H * W * Co));
      if (!out) { rc = kpd_fail_einval("kpd_preprocess: out of device memory"); break; }
      hipLaunchKernelGGL(gauss3_kernel, dim3(blocks((long)H * W * Co)), dim3(256), 0, st, cur, cur_pitch, Co, H, W,
                         (float)(e / s), (float)(1.0 / s), out);
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
