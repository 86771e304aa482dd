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

// Register-resident variant for n <= 1024 * 32 (the detector glue: 28,224
// candidates per image).  Thread t owns candidates t + 1024 k: their scores
// live in registers, their alive flags in one 32-bit mask, and each round is
// ONE pass that applies the previous round's suppression (IoU against the box
// kept last) and finds the best survivor at the same time -- the same
// keep-best / drop-IoU>thr sequence as nms_kernel (same IoU arithmetic and
// tie-break), without its global alive array and two sweeps per kept box.
// slot of this lane in a list that every wave appends to: one LDS atomic per
// wave (the lanes with `in` set take consecutive slots in lane order)
__device__ __forceinline__ int wave_append(bool in, int* counter, int lane) {
  const unsigned long long m = __ballot(in);
  if (!m) return 0;
  const int leader = __ffsll((long long)m) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(counter, (int)__popcll(m));
  base = __shfl(base, leader, 64);
  return base + (int)__popcll(m & ((1ull << lane) - 1ull));
}
constexpr int kNmsRegSlots = 32;
constexpr int kNmsPrefix = 1024;   // target size of the fast path's prefix S
constexpr int kNmsList = 2048;     // LDS list capacity for S (ties at its threshold included)
__global__ __launch_bounds__(1024) void nms_reg_kernel(const float* __restrict__ boxes,
                                                       const float* __restrict__ scores, int n, float thr,
                                                       int max_out, int max_keep, int32_t* __restrict__ keep,
                                                       int32_t* __restrict__ n_keep, int filter,
                                                       float* __restrict__ out_boxes, float* __restrict__ out_scores) {
  __shared__ float ws[16];
  __shared__ int wi[16];
  __shared__ int best_s;
  const int set = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* bx = boxes + (size_t)set * n * 4;
  const float* sc = scores + (size_t)set * n;
  float s[kNmsRegSlots];
  unsigned alive = 0u;
#pragma unroll
  for (int k = 0; k < kNmsRegSlots; ++k) {
    const int i = tid + k * 1024;
    s[k] = -INFINITY;
    if (i < n) {
      s[k] = sc[i];
      if (!filter || s[k] > -INFINITY) alive |= 1u << k;
    }
  }
  int kept = 0;
  const int limit = max_out > 0 ? min(max_out, max_keep) : max_keep;
  // ---- fast path: greedy NMS on a prefix of the (score desc, index asc)
  // order.  Every decision about a candidate depends only on the candidates
  // ranked above it, so once `limit` boxes are kept inside a prefix S (all
  // candidates whose sortable score key is >= tau), the full pass would keep
  // the same boxes.  S: radix select of the kNmsPrefix-th largest key (8-bit
  // digits, LDS histograms), ties at tau included while S fits the LDS list.
  // If S runs dry before `limit` and does not hold every alive candidate, the
  // full register pass below runs from the start.
  {
    __shared__ unsigned hist[16 * 257];   // per-wave histograms (stride 257: each wave's bins on other banks)
    __shared__ unsigned sh_prefix, sh_need, sh_total;
    __shared__ int sh_cnt;
    __shared__ int l_idx[kNmsList];
    __shared__ float l_sc[kNmsList];
    auto key_of = [](float x) {   // order-preserving map of a float to unsigned (every alive key >= 0x007fffff)
      const unsigned b = __float_as_uint(x);
      return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
    };
    if (tid == 0) { sh_total = 0u; sh_cnt = 0; sh_prefix = 0u; sh_need = kNmsPrefix; }
    __syncthreads();
    {
      unsigned c = __popc(alive);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
      if (lane == 0) atomicAdd(&sh_total, c);
    }
    __syncthreads();
    const unsigned total = sh_total;
    unsigned tau = 0u;                      // S = alive keys >= tau (0: every alive candidate)
    if (total > (unsigned)kNmsPrefix) {
      unsigned mask = 0u;
      for (int shift = 24; shift >= 0; shift -= 8) {
        for (int i = tid; i < 16 * 257; i += 1024) hist[i] = 0u;
        __syncthreads();
        const unsigned prefix = sh_prefix;
        unsigned* wh = hist + wave * 257;
#pragma unroll
        for (int k = 0; k < kNmsRegSlots; ++k) {
          if (!((alive >> k) & 1u)) continue;
          const unsigned key = key_of(s[k]);
          if ((key & mask) == prefix) atomicAdd(&wh[(key >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (tid < 256) {   // merge the wave histograms into wave 0's
          unsigned c = 0u;
          for (int w = 0; w < 16; ++w) c += hist[w * 257 + tid];
          hist[tid] = c;
        }
        __syncthreads();
        if (wave == 0) {
          // the digit holding the need-th largest key: lane l sums bins
          // 255 - 4l .. 252 - 4l, a wave prefix sum over the lanes (descending
          // bins) finds the lane, then its four bins
          unsigned c[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) c[j] = hist[255 - (4 * lane + j)];
          const unsigned tot = c[0] + c[1] + c[2] + c[3];
          unsigned pre = tot;
#pragma unroll
          for (int o = 1; o < 64; o <<= 1) {
            const unsigned v = __shfl_up(pre, o, 64);
            if (lane >= o) pre += v;
          }
          const unsigned need = sh_need, excl = pre - tot;
          if (excl < need && pre >= need) {
            unsigned r = need - excl;
            int j = 0;
            for (; j < 3; ++j) {
              if (r <= c[j]) break;
              r -= c[j];
            }
            sh_prefix = prefix | ((unsigned)(255 - (4 * lane + j)) << shift);
            sh_need = r;
          }
        }
        mask |= 0xffu << shift;
        __syncthreads();
      }
      tau = sh_prefix;                      // the kNmsPrefix-th largest key
    }
    // compact S into the LDS list (ties at tau too, while they fit)
    for (int pass = 0; pass < 2; ++pass) {   // pass 0: keys > tau, pass 1: keys == tau
#pragma unroll
      for (int k = 0; k < kNmsRegSlots; ++k) {
        const unsigned key = key_of(s[k]);
        const bool in = ((alive >> k) & 1u) &&
                        (pass == 0 ? (tau == 0u || key > tau) : (tau != 0u && key == tau));
        const int pos = wave_append(in, &sh_cnt, lane);
        if (in && pos < kNmsList) { l_idx[pos] = tid + k * 1024; l_sc[pos] = s[k]; }
      }
      __syncthreads();
      if (pass == 0 && sh_cnt > kNmsList) break;   // (cannot happen: keys > tau number < kNmsPrefix)
    }
    int m = sh_cnt;
    // S holds every alive candidate and fits the list.  Decided before the
    // re-compaction below: after a tie overflow the list holds only keys > tau,
    // a strict prefix, so running dry there must fall back to the full pass.
    const bool covered = m == (int)total && m <= kNmsList;
    if (m > kNmsList) {                         // the ties overflowed: keep only keys > tau (a prefix too)
      __syncthreads();
      if (tid == 0) sh_cnt = 0;
      __syncthreads();
#pragma unroll
      for (int k = 0; k < kNmsRegSlots; ++k) {
        const bool in = ((alive >> k) & 1u) && key_of(s[k]) > tau;
        const int pos = wave_append(in, &sh_cnt, lane);
        if (in) { l_idx[pos] = tid + k * 1024; l_sc[pos] = s[k]; }
      }
      __syncthreads();
      m = sh_cnt;
    }
    // greedy rounds over the list: thread t holds entries t and t + 1024
    constexpr int PER = kNmsList / 1024;
    int li[PER];
    float ls[PER];
    float4 lb[PER];
    unsigned la = 0u;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int e = tid + u * 1024;
      li[u] = 0x7fffffff;
      ls[u] = -INFINITY;
      lb[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < m) {
        li[u] = l_idx[e];
        ls[u] = l_sc[e];
        lb[u] = *reinterpret_cast<const float4*>(bx + (size_t)li[u] * 4);
        la |= 1u << u;
      }
    }
    bool have = false;
    float fb[4] = {0.f, 0.f, 0.f, 0.f};
    int fk = 0;
    while (fk < limit) {
      float bs = -INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        if (!((la >> u) & 1u)) continue;
        if (have) {
          const float bb[4] = {lb[u].x, lb[u].y, lb[u].z, lb[u].w};
          if (!(iou_cxcywh(fb, bb) <= thr)) { la &= ~(1u << u); continue; }
        }
        if (better(ls[u], li[u], bs, bi)) { bs = ls[u]; bi = li[u]; }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float s2 = __shfl_xor(bs, o, 64);
        const int i2 = __shfl_xor(bi, o, 64);
        if (better(s2, i2, bs, bi)) { bs = s2; bi = i2; }
      }
      if (lane == 0) { ws[wave] = bs; wi[wave] = bi; }
      __syncthreads();
      if (tid == 0) {
        float sb = ws[0];
        int b = wi[0];
        for (int w = 1; w < 16; ++w)
          if (better(ws[w], wi[w], sb, b)) { sb = ws[w]; b = wi[w]; }
        best_s = b;
      }
      __syncthreads();
      const int b = best_s;
      if (b == 0x7fffffff) break;
      if (tid == 0) keep[(size_t)set * max_keep + fk] = b;
      ++fk;
#pragma unroll
      for (int u = 0; u < PER; ++u)
        if (li[u] == b) la &= ~(1u << u);
      const float4 v = *reinterpret_cast<const float4*>(bx + (size_t)b * 4);
      fb[0] = v.x; fb[1] = v.y; fb[2] = v.z; fb[3] = v.w;
      have = true;
    }
    if (fk >= limit || covered) {
      kept = fk;
      goto done;
    }
  }
  {
  float kb[4] = {0.f, 0.f, 0.f, 0.f};
  bool have_kb = false;
  while (kept < limit) {
    float bs = -INFINITY;
    int bi = 0x7fffffff;
    // groups of 4 slots: the group's box loads are all issued before its IoUs
#pragma unroll
    for (int k0 = 0; k0 < kNmsRegSlots; k0 += 4) {
      if (!((alive >> k0) & 0xfu)) continue;
      float4 v[4];
      if (have_kb) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if ((alive >> (k0 + u)) & 1u) v[u] = *reinterpret_cast<const float4*>(bx + (size_t)(tid + (k0 + u) * 1024) * 4);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = k0 + u;
        if (!((alive >> k) & 1u)) continue;
        const int i = tid + k * 1024;
        if (have_kb) {
          const float bb[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
          if (!(iou_cxcywh(kb, bb) <= thr)) {
            alive &= ~(1u << k);
            continue;
          }
        }
        if (better(s[k], i, bs, bi)) { bs = s[k]; bi = i; }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float s2 = __shfl_xor(bs, o, 64);
      const int i2 = __shfl_xor(bi, o, 64);
      if (better(s2, i2, bs, bi)) { bs = s2; bi = i2; }
    }
    if (lane == 0) { ws[wave] = bs; wi[wave] = bi; }
    __syncthreads();
    if (tid == 0) {
      float sb = ws[0];
      int b = wi[0];
      for (int w = 1; w < 16; ++w)
        if (better(ws[w], wi[w], sb, b)) { sb = ws[w]; b = wi[w]; }
      best_s = b;
    }
    __syncthreads();
    const int b = best_s;
    if (b == 0x7fffffff) break;   // nothing alive
    if (tid == 0) keep[(size_t)set * max_keep + kept] = b;
    ++kept;
    if ((b & 1023) == tid) alive &= ~(1u << (b >> 10));   // the kept box leaves the candidates
    const float4 v = *reinterpret_cast<const float4*>(bx + (size_t)b * 4);
    kb[0] = v.x; kb[1] = v.y; kb[2] = v.z; kb[3] = v.w;
    have_kb = true;
  }
  }
done:
  if (tid == 0) n_keep[set] = kept;
  if (out_boxes) {   // kept boxes, zero padded to max_keep (zero boxes are skipped downstream)
    __syncthreads();
    for (int t = tid; t < max_keep; t += 1024) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      float sv = 0.f;
      if (t < kept) {
        const int k = keep[(size_t)set * max_keep + t];
        v = *reinterpret_cast<const float4*>(bx + (size_t)k * 4);
        sv = sc[k];
      }
      *reinterpret_cast<float4*>(out_boxes + ((size_t)set * max_keep + t) * 4) = v;
      if (out_scores) out_scores[(size_t)set * max_keep + t] = sv;
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
  // KPD_NMS_SWEEP=1: the two-sweep kernel with the global alive array for every n (A/B)
  static const bool sweep = kpd_diag_env("KPD_NMS_SWEEP") != nullptr;
  if (n <= 1024 * kNmsRegSlots && !sweep)
    hipLaunchKernelGGL(nms_reg_kernel, dim3(sets), dim3(1024), 0, st, boxes, scores, n, thr, max_out, max_keep, keep,
                       n_keep, filter, out_boxes, out_scores);
  else
    hipLaunchKernelGGL(nms_kernel, dim3(sets), dim3(1024), 0, st, boxes, scores, n, thr, max_out, max_keep, keep,
                       n_keep, reinterpret_cast<uint8_t*>(scratch), filter, out_boxes, out_scores);
  return hipGetLastError();
}

hipError_t launch_nms(const float* boxes, const float* scores, int n, float thr, int max_out, int32_t* keep,
                      int32_t* n_keep, void* scratch, size_t scratch_bytes, hipStream_t st) {
  if (scratch_bytes < nms_scratch_bytes(n)) return hipErrorInvalidValue;
  return launch_nms_sets(boxes, scores, 1, n, thr, max_out, n, keep, n_keep, scratch, st, 0, nullptr, nullptr);
}
