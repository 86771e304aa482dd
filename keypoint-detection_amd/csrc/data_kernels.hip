// Data-side kernels around the hot path: training /
// evaluation targets and the validation metrics, on the device.
//
// * kpd_target_heatmaps restates generate_target_heatmap
//   (dll/models/heatmap_head.py:163-224) with get_gaussian_kernel (:153-161):
//   per (person, keypoint) plane, the normalised (6*int(sigma)+1)^2 Gaussian is
//   pasted with its centre at (floor(x*W), floor(y*H)) and cropped at the
//   borders; planes whose keypoint lies outside [0, W) x [0, H) stay zero.
//   One thread writes four consecutive pixels of a row (HBM-bound: the output
//   is the only traffic).
// * kpd_keypoint_metrics restates Trainer._calculate_validation_metrics
//   (dll/training/trainer.py:384-429): dist = ||pred - gt|| in fp32, ADE =
//   mean dist over visible keypoints, PCK_t = #(dist <= t and visible) / numel
//   (the reference divides by all keypoints, not the visible ones).  One
//   workgroup, double accumulators, fixed-order tree reduction; the thresholds
//   (host floats) travel as kernel arguments.
#include <cmath>
#include <vector>

#include "../../include/kpd.h"
#include "kpd_common.h"
#include "kpd_kernels.h"

#pragma clang fp contract(off)

namespace {

__global__ void target_heatmap_kernel(const float* __restrict__ kpts, int planes, int H, int W, int ks,
                                      const float* __restrict__ gk, float* __restrict__ out) {
  const int Wq = (W + 3) / 4;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)planes * H * Wq) return;
  const int xq = (int)(i % Wq), y = (int)((i / Wq) % H), p = (int)(i / ((long)Wq * H));
  const float x0 = kpts[2 * p] * (float)W, y0 = kpts[2 * p + 1] * (float)H;
  const bool inside = x0 >= 0.f && y0 >= 0.f && x0 < (float)W && y0 < (float)H;   // NaN: outside
  const int fx = inside ? (int)x0 : 0, fy = inside ? (int)y0 : 0, r = ks / 2;
  const int ky = y - fy + r;
  float v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int kx = xq * 4 + j - fx + r;
    v[j] = (inside && ky >= 0 && ky < ks && kx >= 0 && kx < ks) ? gk[ky * ks + kx] : 0.f;
  }
  float* o = out + ((size_t)p * H + y) * W + xq * 4;
  if ((W & 3) == 0) {
    *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    for (int j = 0; j < 4 && xq * 4 + j < W; ++j) o[j] = v[j];
  }
}

constexpr int kMaxPck = 16;
constexpr int kMetricThreads = 256;

struct PckThresholds {
  float t[kMaxPck];
};

__global__ __launch_bounds__(kMetricThreads) void keypoint_metrics_kernel(const float* __restrict__ pred,
                                                                          const float* __restrict__ gt,
                                                                          const float* __restrict__ vis, long n,
                                                                          int nt, PckThresholds thr,
                                                                          float* __restrict__ out) {
  __shared__ double s_sum[kMetricThreads];
  __shared__ long s_cnt[kMetricThreads][kMaxPck + 1];
  const int tid = threadIdx.x;
  double sum = 0.0;
  long cnt[kMaxPck + 1] = {0};
  for (long i = tid; i < n; i += kMetricThreads) {
    const float dx = pred[2 * i] - gt[2 * i], dy = pred[2 * i + 1] - gt[2 * i + 1];
    const float d = sqrtf(dx * dx + dy * dy);
    if (vis[i] > 0.f) {
      sum += (double)d;
      cnt[0] += 1;
      for (int t = 0; t < nt; ++t) cnt[1 + t] += d <= thr.t[t];
    }
  }
  s_sum[tid] = sum;
  for (int t = 0; t <= nt; ++t) s_cnt[tid][t] = cnt[t];
  __syncthreads();
  for (int s = kMetricThreads / 2; s > 0; s >>= 1) {
    if (tid < s) {
      s_sum[tid] += s_sum[tid + s];
      for (int t = 0; t <= nt; ++t) s_cnt[tid][t] += s_cnt[tid + s][t];
    }
    __syncthreads();
  }
  if (tid == 0) {
    const long nv = s_cnt[0][0];
    out[0] = nv > 0 ? (float)(s_sum[0] / (double)nv) : 0.f;
    for (int t = 0; t < nt; ++t) out[1 + t] = nv > 0 ? (float)((double)s_cnt[0][1 + t] / (double)n) : 0.f;
  }
}

}  // namespace

extern "C" int kpd_target_heatmaps(const float* kpts, int planes, int H, int W, float sigma, float* out,
                                   void* stream) {
  if (!out || (planes > 0 && !kpts) || planes < 0 || H <= 0 || W <= 0 || !(sigma > 0.f) || sigma > 64.f)
    return kpd_fail_einval("kpd_target_heatmaps: bad arguments");
  if (planes == 0) return KPD_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // get_gaussian_kernel(6*int(sigma)+1, sigma) in fp32: coords i - (ks-1)/2,
  // exp(-(cy^2 + cx^2) / (2 sigma^2)), divided by its sum (summed in double,
  // rounded once).
  const int ks = 6 * (int)sigma + 1;
  std::vector<float> g((size_t)ks * ks);
  const float den = (float)(2.0 * (double)sigma * (double)sigma);
  double sum = 0.0;
  for (int a = 0; a < ks; ++a)
    for (int b = 0; b < ks; ++b) {
      const float ca = (float)a - (float)((ks - 1) / 2.0), cb = (float)b - (float)((ks - 1) / 2.0);
      const float e = std::exp(-(ca * ca + cb * cb) / den);
      g[(size_t)a * ks + b] = e;
      sum += e;
    }
  const float fs = (float)sum;
  for (float& v : g) v = v / fs;
  float* dg = nullptr;
  hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&dg), g.size() * sizeof(float), st);
  if (e != hipSuccess) return kpd_fail_hip(e, "kpd_target_heatmaps alloc");
  e = hipMemcpyAsync(dg, g.data(), g.size() * sizeof(float), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) {
    const long n = (long)planes * H * ((W + 3) / 4);
    hipLaunchKernelGGL(target_heatmap_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, kpts, planes, H,
                       W, ks, dg, out);
    e = hipGetLastError();
  }
  // the table lives in pageable host memory: finish the copy before it goes away
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  (void)hipFreeAsync(dg, st);
  return e == hipSuccess ? KPD_OK : kpd_fail_hip(e, "kpd_target_heatmaps");
}

extern "C" int kpd_keypoint_metrics(const float* pred, const float* gt, const float* vis, long n,
                                    const float* thresholds, int n_thresholds, float* out, void* stream) {
  if (!out || !thresholds || n < 0 || n_thresholds < 0 || n_thresholds > kMaxPck || (n > 0 && (!pred || !gt || !vis)))
    return kpd_fail_einval("kpd_keypoint_metrics: bad arguments (at most 16 thresholds)");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  PckThresholds thr{};
  for (int t = 0; t < n_thresholds; ++t) thr.t[t] = thresholds[t];
  hipLaunchKernelGGL(keypoint_metrics_kernel, dim3(1), dim3(kMetricThreads), 0, st, pred, gt, vis, n, n_thresholds,
                     thr, out);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? KPD_OK : kpd_fail_hip(e, "kpd_keypoint_metrics");
}
