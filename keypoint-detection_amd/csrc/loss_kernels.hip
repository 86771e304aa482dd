// Training-side loss: AdaptiveHeatmapLoss
// (dll/losses/keypoint_loss.py:202-280) forward, plus its gradient with
// respect to the predicted heatmaps (the seed of a heatmap-head backward).
//
//   thr  = clamp(quantile(gt, 0.9), 0.05, 0.3)  (adaptive; else 0.1)   :229-236
//   mse  = (pred - gt)^2                                              :260
//   wl   = mse * [gt > thr] * kw + mse * [gt <= thr] * bw              :263-264
//   wl  *= (1 - exp(-mse))^alpha          (alpha > 0)                  :267-270
//   wl  *= target_weight[b, k]            (when given)                 :273-277
//   loss = mean(wl)                                                    :279
//
// quantile: torch.quantile's linear interpolation on the sorted values, with
// the rank 0.9 * (n - 1) and the lerp evaluated in fp32 as torch does
// (q and the sorted values share the input dtype).  The order statistics come
// from a radix select over the order-preserving unsigned image of the floats:
// 4 passes of 8 bits (global histogram of the candidates, one workgroup picks
// the bucket), then the successor of the selected value when the rank above
// it is needed (count of equal values, min of the larger ones).
//
// Reductions are deterministic: a fixed grid of LOSS_BLOCKS workgroups sums
// its elements in a fixed order into double partials, and one workgroup adds
// the partials in index order.  HBM-bound: 4 select passes + 1 loss pass read
// gt (4 + 1) times and pred once, ~6 x 13 MB at B = 64, 17 x 64 x 48.
#include <cstdint>
#include <cmath>

#include <algorithm>

#include "../../include/kpd.h"
#include "kpd_common.h"
#include "kpd_kernels.h"

namespace {

constexpr int LOSS_BLOCKS = 1024, LOSS_NT = 256;

__device__ __forceinline__ unsigned f2key(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// select state: [0] prefix, [1] mask, [2] rank still to skip inside the
// prefix, [3] count of elements equal to the selected value (after pass 4),
// [4] min key above the selected value, [5..] spare; hist[256] after it
struct SelState {
  unsigned prefix, mask, rank, eq, above, pad[3];
  unsigned hist[256];
};

__global__ __launch_bounds__(LOSS_NT) void sel_init_kernel(SelState* s, unsigned rank) {
  const int t = threadIdx.x;
  if (t == 0) {
    s->prefix = 0u;
    s->mask = 0u;
    s->rank = rank;
    s->eq = 0u;
    s->above = 0xffffffffu;
  }
  s->hist[t] = 0u;
}

__global__ __launch_bounds__(LOSS_NT) void sel_hist_kernel(const float* __restrict__ x, long n, SelState* s,
                                                            int shift) {
  __shared__ unsigned h[256];
  h[threadIdx.x] = 0u;
  __syncthreads();
  const unsigned prefix = s->prefix, mask = s->mask;
  for (long i = (long)blockIdx.x * LOSS_NT + threadIdx.x; i < n; i += (long)gridDim.x * LOSS_NT) {
    const unsigned k = f2key(x[i]);
    if ((k & mask) == prefix) atomicAdd(&h[(k >> shift) & 255u], 1u);
  }
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd(&s->hist[threadIdx.x], h[threadIdx.x]);
}

// one workgroup: the bucket holding the rank, then clear the histogram
__global__ __launch_bounds__(LOSS_NT) void sel_pick_kernel(SelState* s, int shift) {
  __shared__ unsigned c[256];
  const int t = threadIdx.x;
  c[t] = s->hist[t];
  __syncthreads();
  if (t == 0) {
    unsigned r = s->rank, b = 0;
    for (; b < 255u && r >= c[b]; ++b) r -= c[b];
    s->rank = r;
    s->prefix |= b << shift;
    s->mask |= 255u << shift;
    if (shift == 0) s->eq = c[b];
  }
  __syncthreads();
  s->hist[t] = 0u;
}

// min key strictly above the selected one (needed only when the rank above
// it is not another copy of the same value)
__global__ __launch_bounds__(LOSS_NT) void sel_above_kernel(const float* __restrict__ x, long n, SelState* s) {
  __shared__ unsigned m[LOSS_NT];
  const unsigned sel = s->prefix;
  unsigned best = 0xffffffffu;
  for (long i = (long)blockIdx.x * LOSS_NT + threadIdx.x; i < n; i += (long)gridDim.x * LOSS_NT) {
    const unsigned k = f2key(x[i]);
    if (k > sel && k < best) best = k;
  }
  m[threadIdx.x] = best;
  __syncthreads();
  for (int w = LOSS_NT / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) m[threadIdx.x] = min(m[threadIdx.x], m[threadIdx.x + w]);
    __syncthreads();
  }
  if (threadIdx.x == 0 && m[0] != 0xffffffffu) atomicMin(&s->above, m[0]);
}

// threshold from the order statistics: torch.lerp(lo, hi, w) in fp32, clamp
__global__ void sel_threshold_kernel(const SelState* s, float w, int need_above, float* thr) {
  if (threadIdx.x != 0) return;
  const float lo = key2f(s->prefix);
  float hi = lo;
  if (need_above && s->rank + 1u >= s->eq && s->above != 0xffffffffu) hi = key2f(s->above);
  // at::lerp (scalar path, one element): weight < 0.5 ? self + weight * (end - self)
  // : end - (end - self) * (1 - weight), each operation rounded (no contraction)
  const float dlt = __fsub_rn(hi, lo);
  const float q = w < 0.5f ? __fadd_rn(lo, __fmul_rn(w, dlt)) : __fsub_rn(hi, __fmul_rn(dlt, __fsub_rn(1.f, w)));
  *thr = fminf(fmaxf(q, 0.05f), 0.3f);
}

__global__ void thr_const_kernel(float* thr, float v) {
  if (threadIdx.x == 0) *thr = v;
}

// per element: weighted focal MSE; d/dpred of the mean when grad != null
__global__ __launch_bounds__(LOSS_NT) void loss_kernel(const float* __restrict__ pred, const float* __restrict__ gt,
                                                       const float* __restrict__ tw, long n, long hw,
                                                       const float* __restrict__ thr_p, float kw, float bw,
                                                       float alpha, float* __restrict__ grad, double* __restrict__ part) {
  __shared__ double red[LOSS_NT];
  const float thr = *thr_p;
  const float inv_n = (float)(1.0 / (double)n);
  double acc = 0.0;
  for (long i = (long)blockIdx.x * LOSS_NT + threadIdx.x; i < n; i += (long)gridDim.x * LOSS_NT) {
    const float p = pred[i], g = gt[i];
    const float d = p - g, mse = d * d;
    const bool kp = g > thr;
    const float km = kp ? 1.f : 0.f, bm = kp ? 0.f : 1.f;
    const float wr = mse * km * kw + mse * bm * bw;   // the reference's two products (0 * x terms included)
    float wl = wr, fw = 1.f, pt = 1.f;
    if (alpha > 0.f) {
      pt = expf(-mse);
      const float om = 1.f - pt;
      fw = alpha == 2.f ? om * om : powf(om, alpha);
      wl = wl * fw;
    }
    const float t = tw ? tw[i / hw] : 1.f;
    if (tw) wl = wl * t;
    acc += (double)wl;
    if (grad) {
      // d wl / d p = t * w * [dmse * fw + mse * alpha * (1 - pt)^(alpha-1) * pt * dmse], dmse = 2 d
      const float wsel = km * kw + bm * bw;
      float dfw = 0.f;
      if (alpha > 0.f) {
        const float om = 1.f - pt;
        dfw = alpha == 2.f ? 2.f * om * pt : alpha * powf(om, alpha - 1.f) * pt;
      }
      const float dm = 2.f * d;
      grad[i] = t * wsel * (dm * fw + mse * dfw * dm) * inv_n;
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = LOSS_NT / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ __launch_bounds__(LOSS_NT) void loss_final_kernel(const double* __restrict__ part, int nb, long n,
                                                             float* __restrict__ out) {
  __shared__ double red[LOSS_NT];
  double a = 0.0;
  for (int i = threadIdx.x; i < nb; i += LOSS_NT) a += part[i];
  red[threadIdx.x] = a;
  __syncthreads();
  for (int w = LOSS_NT / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = (float)(red[0] / (double)n);
}

}  // namespace

extern "C" int kpd_adaptive_heatmap_loss(const float* pred, const float* gt, const float* target_weight, int B,
                                         int K, int H, int W, float keypoint_weight, float background_weight,
                                         int adaptive_threshold, float focal_alpha, float* loss_out,
                                         float* grad_pred, float* threshold_out, void* stream) {
  const long hw = (long)H * W, n = (long)B * K * hw;
  if (!pred || !gt || !loss_out || B <= 0 || K <= 0 || H <= 0 || W <= 0 || !(focal_alpha >= 0.f) ||
      n >= (1L << 31))
    return kpd_fail_einval("kpd_adaptive_heatmap_loss: bad arguments");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const size_t scratch = sizeof(SelState) + sizeof(double) * LOSS_BLOCKS + sizeof(float);
  char* ws = nullptr;
  hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&ws), scratch, st);
  if (e != hipSuccess) return kpd_fail_hip(e, "kpd_adaptive_heatmap_loss alloc");
  SelState* s = reinterpret_cast<SelState*>(ws);
  double* part = reinterpret_cast<double*>(ws + sizeof(SelState));
  float* thr = reinterpret_cast<float*>(ws + sizeof(SelState) + sizeof(double) * LOSS_BLOCKS);
  const unsigned grid = (unsigned)std::min<long>(LOSS_BLOCKS, (n + LOSS_NT - 1) / LOSS_NT);
  if (adaptive_threshold) {
    // torch.quantile(q=0.9): ranks = q * (n - 1) in fp32, below = floor, weight = ranks - below
    const float rank = 0.9f * (float)(n - 1);
    const long below = (long)rank;
    const float w = rank - (float)below;
    const int need_above = (float)below != rank;
    hipLaunchKernelGGL(sel_init_kernel, dim3(1), dim3(LOSS_NT), 0, st, s, (unsigned)below);
    for (int shift = 24; shift >= 0; shift -= 8) {
      hipLaunchKernelGGL(sel_hist_kernel, dim3(grid), dim3(LOSS_NT), 0, st, gt, n, s, shift);
      hipLaunchKernelGGL(sel_pick_kernel, dim3(1), dim3(LOSS_NT), 0, st, s, shift);
    }
    if (need_above) hipLaunchKernelGGL(sel_above_kernel, dim3(grid), dim3(LOSS_NT), 0, st, gt, n, s);
    hipLaunchKernelGGL(sel_threshold_kernel, dim3(1), dim3(64), 0, st, s, w, need_above, thr);
  } else {
    hipLaunchKernelGGL(thr_const_kernel, dim3(1), dim3(64), 0, st, thr, 0.1f);
  }
  hipLaunchKernelGGL(loss_kernel, dim3(grid), dim3(LOSS_NT), 0, st, pred, gt, target_weight, n, hw, thr,
                     keypoint_weight, background_weight, focal_alpha, grad_pred, part);
  hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(LOSS_NT), 0, st, part, (int)grid, n, loss_out);
  if (threshold_out) e = hipMemcpyAsync(threshold_out, thr, sizeof(float), hipMemcpyDeviceToDevice, st);
  if (e == hipSuccess) e = hipGetLastError();
  (void)hipFreeAsync(ws, st);
  return e == hipSuccess ? KPD_OK : kpd_fail_hip(e, "kpd_adaptive_heatmap_loss");
}
