// Greedy per-set NMS on gfx950 (reference: dll/models/person_head.py:54-139).
//
// Semantics (bit-matched to PERSON_HEAD.non_max_suppression):
//   order = scores sorted descending (ties: lower index first);
//   repeat: keep the best remaining box; stop if max_output reached;
//           drop every remaining box whose IoU with it is NOT <= thr.
//   IoU on cxcywh boxes in fp32 exactly as box_iou (:54-94), eps 1e-16.
//
// Instead of a full sort, each round is a workgroup-wide arg-max over the
// still-alive candidates (score desc, index asc) followed by one suppression
// sweep.  Rounds = boxes kept, so with max_output = 5 (the person-head glue)
// it is five passes over the candidates; no host round trip, one launch per
// batch (grid = sets).
#include "kpd_common.h"
#include "kpd_kernels.h"

namespace {

__device__ __forceinline__ void corners(const float* b, float& x1, float& y1, float& x2, float& y2) {
  x1 = b[0] - b[2] / 2.f; y1 = b[1] - b[3] / 2.f;
  x2 = b[0] + b[2] / 2.f; y2 = b[1] + b[3] / 2.f;
}

__device__ __forceinline__ float iou_cxcywh(const float* a, const float* b) {
  float ax1, ay1, ax2, ay2, bx1, by1, bx2, by2;
  corners(a, ax1, ay1, ax2, ay2);
  corners(b, bx1, by1, bx2, by2);
  const float iw = fmaxf(fminf(ax2, bx2) - fmaxf(ax1, bx1), 0.f);
  const float ih = fmaxf(fminf(ay2, by2) - fmaxf(ay1, by1), 0.f);
  const float inter = iw * ih;
  const float a1 = (ax2 - ax1) * (ay2 - ay1);
  const float a2 = (bx2 - bx1) * (by2 - by1);
  return inter / (a1 + a2 - inter + 1e-16f);
}

// better(a, b): a ranks before b in a descending sort with index tie-break
__device__ __forceinline__ bool better(float sa, int ia, float sb, int ib) {
  return sa > sb || (sa == sb && ia < ib);
}

// One workgroup (1024 threads) per set.  alive flags live in global scratch.
// boxes [sets][n][4], scores [sets][n]; keep [sets][max_keep]; n_keep [sets].
__global__ __launch_bounds__(1024) void nms_kernel(const float* __restrict__ boxes, const float* __restrict__ scores,
                                                   int n, float thr, int max_out, int max_keep,
                                                   int32_t* __restrict__ keep, int32_t* __restrict__ n_keep,
                                                   uint8_t* __restrict__ alive_all, int filter,
                                                   float* __restrict__ out_boxes, float* __restrict__ out_scores) {
  __shared__ float ws[16];
  __shared__ int wi[16];
  __shared__ int best_s;
  const int set = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* bx = boxes + (size_t)set * n * 4;
  const float* sc = scores + (size_t)set * n;
  uint8_t* alive = alive_all + (size_t)set * n;
  // filter: candidates whose score is -inf (below the detector's conf threshold) start dead
  for (int i = tid; i < n; i += 1024) alive[i] = filter ? (sc[i] > -INFINITY) : 1;
  __syncthreads();
  int kept = 0;
  const int limit = max_out > 0 ? min(max_out, max_keep) : max_keep;
  while (kept < limit) {
    float bs = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = tid; i < n; i += 1024)
      if (alive[i] && better(sc[i], i, bs, bi)) { bs = sc[i]; bi = i; }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float s2 = __shfl_xor(bs, o, 64);
      const int i2 = __shfl_xor(bi, o, 64);
      if (better(s2, i2, bs, bi)) { bs = s2; bi = i2; }
    }
    if (lane == 0) { ws[wave] = bs; wi[wave] = bi; }
    __syncthreads();
    if (tid == 0) {
      float s = ws[0];
      int b = wi[0];
      for (int w = 1; w < 16; ++w)
        if (better(ws[w], wi[w], s, b)) { s = ws[w]; b = wi[w]; }
      best_s = b;
    }
    __syncthreads();
    const int b = best_s;
    if (b == 0x7fffffff) break;  // nothing alive
    if (tid == 0) keep[(size_t)set * max_keep + kept] = b;
    ++kept;
    float kb[4] = {bx[b * 4], bx[b * 4 + 1], bx[b * 4 + 2], bx[b * 4 + 3]};
    for (int i = tid; i < n; i += 1024) {
      if (!alive[i]) continue;
      if (i == b) { alive[i] = 0; continue; }
      const float iou = iou_cxcywh(kb, bx + (size_t)i * 4);
      if (!(iou <= thr)) alive[i] = 0;
    }
    __syncthreads();
  }
  if (tid == 0) n_keep[set] = kept;
  if (out_boxes) {   // gather kept boxes, zero padded to max_keep (zero boxes are skipped downstream)
    __syncthreads();
    for (int t = tid; t < max_keep; t += 1024) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      float s = 0.f;
      if (t < kept) {
        const int k = keep[(size_t)set * max_keep + t];
        v = *reinterpret_cast<const float4*>(bx + (size_t)k * 4);
        s = sc[k];
      }
      *reinterpret_cast<float4*>(out_boxes + ((size_t)set * max_keep + t) * 4) = v;
      if (out_scores) out_scores[(size_t)set * max_keep + t] = s;
    }
  }
}

}  // namespace

size_t nms_scratch_bytes(int n) { return (size_t)n; }

hipError_t launch_nms_sets(const float* boxes, const float* scores, int sets, int n, float thr, int max_out,
                           int max_keep, int32_t* keep, int32_t* n_keep, void* scratch, hipStream_t st, int filter,
                           float* out_boxes, float* out_scores) {
  if (n <= 0) {
    return hipMemsetAsync(n_keep, 0, sizeof(int32_t) * sets, st);
  }
  hipLaunchKernelGGL(nms_kernel, dim3(sets), dim3(1024), 0, st, boxes, scores, n, thr, max_out, max_keep, keep,
                     n_keep, reinterpret_cast<uint8_t*>(scratch), filter, out_boxes, out_scores);
  return hipGetLastError();
}

hipError_t launch_nms(const float* boxes, const float* scores, int n, float thr, int max_out, int32_t* keep,
                      int32_t* n_keep, void* scratch, size_t scratch_bytes, hipStream_t st) {
  if (scratch_bytes < nms_scratch_bytes(n)) return hipErrorInvalidValue;
  return launch_nms_sets(boxes, scores, 1, n, thr, max_out, n, keep, n_keep, scratch, st, 0, nullptr, nullptr);
}
