// Kernels behind the stand-alone operator entry points of the C ABI (the
// reference's submodule forwards and helper functions, called outside
// MultiPersonKeypointModel.forward): heatmap decoders, a generic ROI align,
// NCHW <-> NHWC layout changes, channel statistics / gathers and a 1x1 conv.
//
// Reference (file:line under /root/reference):
//   decode_heatmaps / _subpixel / _soft_argmax  dll/models/heatmap_head.py:265-413
//   decode_heatmap / _soft_argmax (model)       dll/models/keypoint_model.py:250-313
//   extract_roi_features -> torchvision roi_align  dll/models/keypoint_model.py:212-228
//   select_top_k_channels                       dll/models/keypoint_model.py:653-661
//   PERSON_HEAD.forward (box_heads[-1])         dll/models/person_head.py:141-166
#include <algorithm>

#include "../../include/kpd.h"
#include "kpd_common.h"
#include "kpd_kernels.h"

namespace {

constexpr int DT = 256;   // decoder threads per plane

// (value, index) max with torch.max's rules: the first maximal index wins on
// ties, and a NaN counts as the maximum (torch propagates it).
__device__ __forceinline__ bool better(float v, int i, float bv, int bi) {
  const bool vn = v != v, bn = bv != bv;
  if (vn != bn) return vn;
  if (vn) return i < bi;
  return v > bv || (v == bv && i < bi);
}

template <int MODE>
__global__ __launch_bounds__(DT) void decode_planes_kernel(const float* __restrict__ heat, int H, int W, float param,
                                                           float* __restrict__ kpts, float* __restrict__ scores,
                                                           float* __restrict__ vis) {
  __shared__ float sv[DT], s1[DT], s2[DT];
  __shared__ int si[DT];
  const int plane = blockIdx.x, tid = threadIdx.x, n = H * W;
  const float* hp = heat + (size_t)plane * n;
  // rough maximum (argmax) -- every mode needs the maximum value
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int i = tid; i < n; i += DT) {
    const float v = hp[i];
    if (better(v, i, bv, bi)) { bv = v; bi = i; }
  }
  sv[tid] = bv;
  si[tid] = bi;
  __syncthreads();
  for (int o = DT / 2; o > 0; o >>= 1) {
    if (tid < o && better(sv[tid + o], si[tid + o], sv[tid], si[tid])) {
      sv[tid] = sv[tid + o];
      si[tid] = si[tid + o];
    }
    __syncthreads();
  }
  const float mx = sv[0];
  const int mi = si[0] == 0x7fffffff ? 0 : si[0];
  __syncthreads();
  if constexpr (MODE == KPD_DECODE_ARGMAX) {
    if (tid == 0) {
      kpts[plane * 2 + 0] = (float)(mi % W) / (float)(W - 1);
      kpts[plane * 2 + 1] = (float)(mi / W) / (float)(H - 1);
      if (scores) scores[plane] = mx;
    }
  } else if constexpr (MODE == KPD_DECODE_SUBPIXEL) {
    // mass-weighted mean of the window around the maximum (row-major sums)
    if (tid == 0) {
      // pad = window_size // 2 (Python floor: a negative window is empty -> zeros, as the reference)
      const int pad = (int)floorf(param * 0.5f), xc = mi % W, yc = mi / W;
      const int x0 = max(0, xc - pad), x1 = min(W, xc + pad + 1), y0 = max(0, yc - pad), y1 = min(H, yc + pad + 1);
      float tot = 0.f, sx = 0.f, sy = 0.f, wm = -INFINITY;
      for (int y = y0; y < y1; ++y)
        for (int x = x0; x < x1; ++x) tot += hp[y * W + x];
      float rx = 0.f, ry = 0.f, sc = 0.f;
      if (tot > 0.f) {
        for (int y = y0; y < y1; ++y)
          for (int x = x0; x < x1; ++x) {
            const float v = hp[y * W + x];
            sx += (float)x * v;
            sy += (float)y * v;
            wm = (v > wm || v != v) ? v : wm;
          }
        rx = sx / tot;
        ry = sy / tot;
        sc = wm;
      }
      kpts[plane * 2 + 0] = rx / (float)(W - 1);
      kpts[plane * 2 + 1] = ry / (float)(H - 1);
      if (scores) scores[plane] = sc;
    }
  } else {
    // soft-argmax: softmax over the plane (of h / T), expected x and y
    const float T = MODE == KPD_DECODE_SOFTARGMAX ? param : 1.f;
    float m = -INFINITY;
    for (int i = tid; i < n; i += DT) m = fmaxf(m, MODE == KPD_DECODE_SOFTARGMAX ? hp[i] / T : hp[i]);
    sv[tid] = m;
    __syncthreads();
    for (int o = DT / 2; o > 0; o >>= 1) {
      if (tid < o) sv[tid] = fmaxf(sv[tid], sv[tid + o]);
      __syncthreads();
    }
    m = sv[0];
    __syncthreads();
    float se = 0.f, sx = 0.f, sy = 0.f;
    for (int i = tid; i < n; i += DT) {
      const float e = expf((MODE == KPD_DECODE_SOFTARGMAX ? hp[i] / T : hp[i]) - m);
      se += e;
      sx = fmaf(e, (float)(i % W), sx);
      sy = fmaf(e, (float)(i / W), sy);
    }
    sv[tid] = se;
    s1[tid] = sx;
    s2[tid] = sy;
    __syncthreads();
    for (int o = DT / 2; o > 0; o >>= 1) {
      if (tid < o) {
        sv[tid] += sv[tid + o];
        s1[tid] += s1[tid + o];
        s2[tid] += s2[tid + o];
      }
      __syncthreads();
    }
    if (tid == 0) {
      kpts[plane * 2 + 0] = (s1[0] / sv[0]) / (float)(W - 1);
      kpts[plane * 2 + 1] = (s2[0] / sv[0]) / (float)(H - 1);
      if (scores) scores[plane] = mx;
      if (MODE == KPD_DECODE_MODEL && vis) {
        // keypoint_model.py:268-280: conf = sigmoid(max), classes < 0.3 / < 0.7 / else
        const float conf = kpd_sigmoid(mx);
        // compared as the reference does: conf.item() (a double) against 0.3 / 0.7
        const int cls = (double)conf < 0.3 ? 0 : ((double)conf < 0.7 ? 1 : 2);
        vis[plane * 3 + 0] = cls == 0 ? 1.f : 0.f;
        vis[plane * 3 + 1] = cls == 1 ? 1.f : 0.f;
        vis[plane * 3 + 2] = cls == 2 ? 1.f : 0.f;
      }
    }
  }
}

// torchvision roi_align (CPU/CUDA reference semantics), NCHW features,
// rois [R][5] = (batch index, x1, y1, x2, y2) in input coordinates.  One
// thread per output element; samples summed in (iy, ix) order, / count.
__global__ __launch_bounds__(256) void roi_align_nchw_kernel(const float* __restrict__ feat, int C, int H, int W,
                                                             const float* __restrict__ rois, int R, int oh, int ow,
                                                             float scale, int sr, int aligned, float* __restrict__ out) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x, total = (long)R * C * oh * ow;
  if (idx >= total) return;
  const int pw = (int)(idx % ow), ph = (int)((idx / ow) % oh), c = (int)((idx / ((long)ow * oh)) % C);
  const int r = (int)(idx / ((long)ow * oh * C));
  const float* ro = rois + (size_t)r * 5;
  const int b = (int)ro[0];
  const float off = aligned ? 0.5f : 0.f;
  const float x1 = ro[1] * scale - off, y1 = ro[2] * scale - off, x2 = ro[3] * scale - off, y2 = ro[4] * scale - off;
  float rw = x2 - x1, rh = y2 - y1;
  if (!aligned) {
    rw = fmaxf(rw, 1.f);
    rh = fmaxf(rh, 1.f);
  }
  const float bh = rh / (float)oh, bw = rw / (float)ow;
  const int gh = sr > 0 ? sr : (int)ceilf(rh / (float)oh), gw = sr > 0 ? sr : (int)ceilf(rw / (float)ow);
  const float count = (float)max(gh * gw, 1);
  const float* fp = feat + ((size_t)b * C + c) * H * W;
  float acc = 0.f;
  for (int iy = 0; iy < gh; ++iy) {
    const float y0 = y1 + (float)ph * bh + ((float)iy + 0.5f) * bh / (float)gh;
    for (int ix = 0; ix < gw; ++ix) {
      const float x0 = x1 + (float)pw * bw + ((float)ix + 0.5f) * bw / (float)gw;
      if (y0 < -1.f || y0 > (float)H || x0 < -1.f || x0 > (float)W) continue;
      float y = y0 <= 0.f ? 0.f : y0, x = x0 <= 0.f ? 0.f : x0;
      int yl = (int)y, xl = (int)x, yh, xh;
      if (yl >= H - 1) { yh = yl = H - 1; y = (float)yl; } else yh = yl + 1;
      if (xl >= W - 1) { xh = xl = W - 1; x = (float)xl; } else xh = xl + 1;
      const float ly = y - (float)yl, lx = x - (float)xl, hy = 1.f - ly, hx = 1.f - lx;
      acc += hy * hx * fp[yl * W + xl] + hy * lx * fp[yl * W + xh] + ly * hx * fp[yh * W + xl] +
             ly * lx * fp[yh * W + xh];
    }
  }
  out[idx] = acc / count;
}

// [N][C][H][W] -> [N][H][W][C], one image row per workgroup (W <= 64,
// C <= 128) through LDS; optional per-row channel sum / max in the layout
// roi_align_kernel writes for the HeatmapHead attention: stats [N][H][2][C];
// optional amax[n * amax_stride] = max |x| of image n (float bits, atomicMax:
// the caller zeroes it) -- the split heatmap convs' operand bound when the
// input may be negative (the stand-alone HeatmapHead).
__global__ __launch_bounds__(256) void nchw_rows_to_nhwc_kernel(const float* __restrict__ in, int C, int H, int W,
                                                                float* __restrict__ out, float* __restrict__ stats,
                                                                float* __restrict__ amax, int amax_stride) {
  __shared__ float t[128][65];
  const int y = blockIdx.x, n = blockIdx.y, tid = threadIdx.x;
  for (int e = tid; e < C * W; e += 256) {
    const int c = e / W, x = e - c * W;
    t[c][x] = in[(((size_t)n * C + c) * H + y) * W + x];
  }
  __syncthreads();
  for (int e = tid; e < C * W; e += 256) {
    const int x = e / C, c = e - x * C;
    out[(((size_t)n * H + y) * W + x) * C + c] = t[c][x];
  }
  if (stats && tid < C) {
    float s = 0.f, m = -INFINITY;
    for (int x = 0; x < W; ++x) {
      s += t[tid][x];
      m = fmaxf(m, t[tid][x]);
    }
    float* st = stats + ((size_t)n * H + y) * 2 * C;
    st[tid] = s;
    st[C + tid] = m;
  }
  if (amax) {
    float a = 0.f;
    for (int e = tid; e < C * W; e += 256) {
      const int c = e / W, x = e - c * W;
      a = fmaxf(a, fabsf(t[c][x]));
    }
    a = wave_max(a);
    if ((tid & 63) == 0)
      atomicMax(reinterpret_cast<unsigned*>(amax + (size_t)n * amax_stride), __float_as_uint(a));
  }
}

// [N][HW][C] -> [N][C][HW], 32 pixels x C (<= 128) channels per workgroup
__global__ __launch_bounds__(256) void nhwc_to_nchw_kernel(const float* __restrict__ in, int HW, int C,
                                                           float* __restrict__ out) {
  __shared__ float t[32][129];
  const int p0 = blockIdx.x * 32, n = blockIdx.y, tid = threadIdx.x, np = min(32, HW - p0);
  for (int e = tid; e < np * C; e += 256) {
    const int p = e / C, c = e - p * C;
    t[p][c] = in[((size_t)n * HW + p0 + p) * C + c];
  }
  __syncthreads();
  for (int e = tid; e < np * C; e += 256) {
    const int c = e / np, p = e - c * np;
    out[((size_t)n * C + c) * HW + p0 + p] = t[p][c];
  }
}

// [N][HW][Cp] (channels padded to Cp) -> [N][C][HW]: a 32-pixel x 32-channel
// tile per workgroup (grid: pixel tiles, channel tiles, images); the body taps
// of MobileNetV3Wrapper.body (up to 576 channels)
__global__ __launch_bounds__(256) void nhwc_pad_to_nchw_kernel(const float* __restrict__ in, int HW, int C, int Cp,
                                                               float* __restrict__ out) {
  __shared__ float t[32][33];
  const int p0 = blockIdx.x * 32, c0 = blockIdx.y * 32, n = blockIdx.z, tid = threadIdx.x;
  const int np = min(32, HW - p0), nc = min(32, C - c0);
  for (int e = tid; e < 32 * 32; e += 256) {
    const int p = e >> 5, c = e & 31;
    if (p < np && c < nc) t[p][c] = in[((size_t)n * HW + p0 + p) * Cp + c0 + c];
  }
  __syncthreads();
  for (int e = tid; e < 32 * 32; e += 256) {
    const int c = e >> 5, p = e & 31;
    if (p < np && c < nc) out[((size_t)n * C + c0 + c) * HW + p0 + p] = t[p][c];
  }
}

// [N][C][HW] -> [N][HW][Cp], zero in the padding channels C..Cp-1 (the body
// layout the FPN convs read: LightweightFPN.forward on caller taps)
__global__ __launch_bounds__(256) void nchw_to_nhwc_pad_kernel(const float* __restrict__ in, int HW, int C, int Cp,
                                                               float* __restrict__ out) {
  __shared__ float t[32][33];
  const int p0 = blockIdx.x * 32, c0 = blockIdx.y * 32, n = blockIdx.z, tid = threadIdx.x;
  const int np = min(32, HW - p0), nc = min(32, Cp - c0);
  for (int e = tid; e < 32 * 32; e += 256) {
    const int c = e >> 5, p = e & 31;
    if (p < np && c < nc) t[p][c] = c0 + c < C ? in[((size_t)n * C + c0 + c) * HW + p0 + p] : 0.f;
  }
  __syncthreads();
  for (int e = tid; e < 32 * 32; e += 256) {
    const int p = e >> 5, c = e & 31;
    if (p < np && c < nc) out[((size_t)n * HW + p0 + p) * Cp + c0 + c] = t[p][c];
  }
}

// per (image, channel) plane: sum and max over HW -> stats [N][1][2][C]
// (the layout topk_kernel reads, one "tile" per image)
__global__ __launch_bounds__(256) void nchw_channel_stats_kernel(const float* __restrict__ x, int C, int HW,
                                                                 float* __restrict__ stats) {
  __shared__ float ss[256], sm[256];
  const int c = blockIdx.x, n = blockIdx.y, tid = threadIdx.x;
  const float* p = x + ((size_t)n * C + c) * HW;
  float s = 0.f, m = -INFINITY;
  for (int i = tid; i < HW; i += 256) {
    s += p[i];
    m = fmaxf(m, p[i]);
  }
  ss[tid] = s;
  sm[tid] = m;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
      ss[tid] += ss[tid + o];
      sm[tid] = fmaxf(sm[tid], sm[tid + o]);
    }
    __syncthreads();
  }
  if (tid == 0) {
    stats[(size_t)n * 2 * C + c] = ss[0];
    stats[(size_t)n * 2 * C + C + c] = sm[0];
  }
}

// out[n][k] = x[n][idx[n][k]] (whole HW planes)
__global__ __launch_bounds__(256) void gather_planes_kernel(const float* __restrict__ x, int C, int HW,
                                                            const int32_t* __restrict__ idx, int K,
                                                            float* __restrict__ out) {
  const int k = blockIdx.y, n = blockIdx.z;
  const float* src = x + ((size_t)n * C + idx[n * K + k]) * HW;
  float* dst = out + ((size_t)n * K + k) * HW;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < HW; i += gridDim.x * 256) dst[i] = src[i];
}

// 1x1 conv on NCHW: out[n][co][p] = b[co] + sum_ci w[co][ci] x[n][ci][p] (ci ascending)
__global__ __launch_bounds__(256) void conv1x1_nchw_kernel(const float* __restrict__ x, int Cin, int HW,
                                                           const float* __restrict__ w, const float* __restrict__ b,
                                                           int Cout, float* __restrict__ out) {
  const int p = blockIdx.x * 256 + threadIdx.x, co = blockIdx.y, n = blockIdx.z;
  if (p >= HW) return;
  const float* xp = x + (size_t)n * Cin * HW + p;
  float a = 0.f;
  for (int ci = 0; ci < Cin; ++ci) a = fmaf(w[(size_t)co * Cin + ci], xp[(size_t)ci * HW], a);
  out[((size_t)n * Cout + co) * HW + p] = a + (b ? b[co] : 0.f);
}

__global__ __launch_bounds__(256) void fill_kernel(float* __restrict__ p, long n, float v) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] = v;
}

}  // namespace

hipError_t launch_fill(float* p, long n, float v, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(fill_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, p, n, v);
  return hipGetLastError();
}

hipError_t launch_decode_planes(const float* heat, int planes, int H, int W, int mode, float param, float* kpts,
                                float* scores, float* vis, hipStream_t st) {
  if (planes <= 0) return hipSuccess;
  if (H < 2 || W < 2 || !heat || !kpts) return hipErrorInvalidValue;
#define DEC(M) hipLaunchKernelGGL(decode_planes_kernel<M>, dim3(planes), dim3(DT), 0, st, heat, H, W, param, kpts, \
                                  scores, vis)
  switch (mode) {
    case KPD_DECODE_ARGMAX: DEC(KPD_DECODE_ARGMAX); break;
    case KPD_DECODE_SUBPIXEL:
      if (!(fabsf(param) < 1e9f)) return hipErrorInvalidValue;   // any finite window size (0: 1x1)
      DEC(KPD_DECODE_SUBPIXEL);
      break;
    case KPD_DECODE_SOFTARGMAX:
      if (!(param != 0.f)) return hipErrorInvalidValue;
      DEC(KPD_DECODE_SOFTARGMAX);
      break;
    case KPD_DECODE_MODEL: DEC(KPD_DECODE_MODEL); break;
    default: return hipErrorInvalidValue;
  }
#undef DEC
  return hipGetLastError();
}

hipError_t launch_roi_align_nchw(const float* feat, int C, int H, int W, const float* rois, int R, int oh, int ow,
                                 float scale, int sr, int aligned, float* out, hipStream_t st) {
  const long total = (long)R * C * oh * ow;
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(roi_align_nchw_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, feat, C, H, W,
                     rois, R, oh, ow, scale, sr, aligned, out);
  return hipGetLastError();
}

hipError_t launch_nchw_rows_to_nhwc(const float* in, int N, int C, int H, int W, float* out, float* stats,
                                    hipStream_t st, float* amax, int amax_stride) {
  if (N <= 0) return hipSuccess;
  if (C > 128 || W > 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(nchw_rows_to_nhwc_kernel, dim3(H, N), dim3(256), 0, st, in, C, H, W, out, stats, amax,
                     amax_stride);
  return hipGetLastError();
}

hipError_t launch_nhwc_to_nchw(const float* in, int N, int HW, int C, float* out, hipStream_t st) {
  if (N <= 0 || HW <= 0) return hipSuccess;
  if (C > 128) return hipErrorInvalidValue;
  hipLaunchKernelGGL(nhwc_to_nchw_kernel, dim3((HW + 31) / 32, N), dim3(256), 0, st, in, HW, C, out);
  return hipGetLastError();
}

hipError_t launch_nhwc_pad_to_nchw(const float* in, int N, int HW, int C, int Cp, float* out, hipStream_t st) {
  if (N <= 0 || HW <= 0 || C <= 0) return hipSuccess;
  if (Cp < C || N > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL(nhwc_pad_to_nchw_kernel, dim3((HW + 31) / 32, (C + 31) / 32, N), dim3(256), 0, st, in, HW, C, Cp,
                     out);
  return hipGetLastError();
}

hipError_t launch_nchw_to_nhwc_pad(const float* in, int N, int HW, int C, int Cp, float* out, hipStream_t st) {
  if (N <= 0 || HW <= 0 || Cp <= 0) return hipSuccess;
  if (Cp < C || N > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL(nchw_to_nhwc_pad_kernel, dim3((HW + 31) / 32, (Cp + 31) / 32, N), dim3(256), 0, st, in, HW, C, Cp,
                     out);
  return hipGetLastError();
}

hipError_t launch_nchw_channel_stats(const float* x, int N, int C, int HW, float* stats, hipStream_t st) {
  if (N <= 0) return hipSuccess;
  hipLaunchKernelGGL(nchw_channel_stats_kernel, dim3(C, N), dim3(256), 0, st, x, C, HW, stats);
  return hipGetLastError();
}

hipError_t launch_gather_planes(const float* x, int N, int C, int HW, const int32_t* idx, int K, float* out,
                                hipStream_t st) {
  if (N <= 0 || K <= 0) return hipSuccess;
  hipLaunchKernelGGL(gather_planes_kernel, dim3(std::min((HW + 255) / 256, 64), K, N), dim3(256), 0, st, x, C, HW,
                     idx, K, out);
  return hipGetLastError();
}

hipError_t launch_conv1x1_nchw(const float* x, int N, int Cin, int HW, const float* w, const float* b, int Cout,
                               float* out, hipStream_t st) {
  if (N <= 0 || HW <= 0) return hipSuccess;
  hipLaunchKernelGGL(conv1x1_nchw_kernel, dim3((HW + 255) / 256, Cout, N), dim3(256), 0, st, x, Cin, HW, w, b, Cout,
                     out);
  return hipGetLastError();
}
