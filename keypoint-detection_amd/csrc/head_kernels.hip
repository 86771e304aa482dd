// Channel attention + top-k, batched ROI-align, HeatmapHead attention, final
// 1x1 + sigmoid, and fused soft-argmax / visibility / coordinate decode (gfx950).
//
// Reference (file:line under /root/reference):
//   ChannelAttention + select_top_k_channels  dll/models/keypoint_model.py:18-44,653-661
//   extract_roi_features / box corners        dll/models/keypoint_model.py:212-228,630-638
//   torchvision roi_align (aligned=False, sampling_ratio=-1), restated
//   HeatmapHead channel/spatial attention     dll/models/heatmap_head.py:94-102,115-151
//   final 1x1 + sigmoid                       dll/models/heatmap_head.py:40-44,111
//   decode_heatmap / _soft_argmax             dll/models/keypoint_model.py:250-313
//   convert_to_original_coords                dll/models/keypoint_model.py:230-248
//   zero-box skip / dummy / padding rules     dll/models/keypoint_model.py:149-199,640-651
//
// All ROIs of a batch are processed together as one [R,56,56,C] NHWC tensor
// (R = B*P); the reference's per-box Python loop becomes grid dimensions.
#include <algorithm>

#include "kpd_common.h"
#include "kpd_kernels.h"

namespace {
constexpr int HM = 56;              // ROI / heatmap side
static_assert(HM % 4 == 0, "hm_spool / hm_sapply take 4 pixels per load instruction");
constexpr int HMP = HM * HM;        // 3136
constexpr int NK = 17;              // keypoints
constexpr int TOPK = 64;
constexpr int FC = 128;             // FPN channels

// ---------------------------------------------------------------- top-k
// ChannelAttention + select_top_k_channels (keypoint_model.py:18-44,
// 653-661).  One 256-thread workgroup per image.  stats: [N][tiles][2][128]
// partial channel sums / maxima from the FPN level-0 epilogue.  A thread
// takes one (sum | max, channel) column of the partials, loads 48 tiles of it
// into registers at once and reduces them in tile order; both FC weights go
// to LDS in the same round trip.
__device__ __forceinline__ void slotmap_image(const float* __restrict__ boxes, int b, int P, int32_t* __restrict__ slot);
__global__ __launch_bounds__(256) void topk_kernel(const float* __restrict__ stats, int tiles, int HW,
                                                   const float* __restrict__ w0, const float* __restrict__ b0,
                                                   const float* __restrict__ w2, const float* __restrict__ b2,
                                                   int32_t* __restrict__ topk, float* __restrict__ scores_out,
                                                   const float* __restrict__ boxes, int P, int32_t* __restrict__ slot,
                                                   float* __restrict__ imax, float* __restrict__ sc_zero, int sc_n) {
  extern __shared__ __attribute__((aligned(16))) float tsm[];
  float* sw0 = tsm;                        // [8][FC]
  float* sw2 = sw0 + 8 * FC;               // [FC][8]
  __shared__ float avg[FC], mx[FC], h[16], sc[FC];
  const int n = blockIdx.x, tid = threadIdx.x, c = tid;
  {
    // both FC weights -> LDS (2 float4 per thread), issued with the partials
    float4 wv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = tid + u * 256;
      wv[u] = i < 256 ? reinterpret_cast<const float4*>(w0)[i] : reinterpret_cast<const float4*>(w2)[i - 256];
    }
    // partials straight into registers: thread (kind = sum / max, channel)
    // loads its column of every tile in batches of TB tiles, all in flight
    // together (one round trip per batch instead of one per LDS staging pass),
    // and reduces them in tile order as before
    const int kind = tid >> 7, ch = tid & (FC - 1);
    const float* col = stats + (size_t)n * tiles * 2 * FC + kind * FC + ch;
    constexpr int TB = 48;
    float acc = kind ? -INFINITY : 0.f;
    for (int t0 = 0; t0 < tiles; t0 += TB) {
      float v[TB];
#pragma unroll
      for (int u = 0; u < TB; ++u) v[u] = col[(size_t)min(t0 + u, tiles - 1) * 2 * FC];
#pragma unroll
      for (int u = 0; u < TB; ++u)
        if (t0 + u < tiles) acc = kind ? fmaxf(acc, v[u]) : acc + v[u];
    }
    if (kind) mx[ch] = acc;
    else avg[ch] = acc / (float)HW;
#pragma unroll
    for (int u = 0; u < 2; ++u) reinterpret_cast<float4*>(tsm)[tid + u * 256] = wv[u];
  }
  __syncthreads();
  if (c < 16) {  // hidden units: 0..7 for avg branch, 8..15 for max branch
    const int j = c & 7;
    const float* vv = (c < 8) ? avg : mx;
    float a = b0[j];
#pragma unroll 32
    for (int k = 0; k < FC; ++k) a = fmaf(sw0[j * FC + k], vv[k], a);
    h[c] = fmaxf(a, 0.f);
  }
  __syncthreads();
  if (c >= FC) {
    // (optional) the image's box slot map (slotmap_kernel's work) on a thread
    // of the otherwise idle upper waves: one launch less per forward
    if (slot && c == 255) slotmap_image(boxes, n, P, slot);
    // (optional) the image's max over FPN level 0 (its channel maxima; the map
    // follows a ReLU, so this is max |x|): the bound of the KEYPOINT_HEAD's
    // split operand, whose ROI features interpolate this map
    // (optional) zero the image's split-scale slots (max |tap0|, max |lateral 1|,
    // atomicMax targets of the stem and lateral-1 conv): FPN level 0 has read
    // them, and the next forward's producers need them zero (no memset launch)
    if (sc_zero && c == 129) {
      sc_zero[(size_t)n * kAmaxStride] = 0.f;
      sc_zero[(size_t)(sc_n + n) * kAmaxStride] = 0.f;
    }
    if (imax && c == 128) {
      float M = 0.f;
      for (int k = 0; k < FC; ++k) M = fmaxf(M, mx[k]);
      imax[n] = M;
    }
    return;
  }
  float oa = b2[c], om = b2[c];
  for (int j = 0; j < 8; ++j) {
    oa = fmaf(sw2[c * 8 + j], h[j], oa);
    om = fmaf(sw2[c * 8 + j], h[8 + j], om);
  }
  const float score = kpd_sigmoid(oa + om);
  sc[c] = score;
  __syncthreads();   // waves 2-3 (c >= 128) have exited: the barrier counts waves 0-1
  // rank = number of channels ordered before c (score desc, index asc on ties)
  int rank = 0;
#pragma unroll 32
  for (int k = 0; k < FC; ++k) {
    const float o = sc[k];
    rank += (o > score) || (o == score && k < c);
  }
  if (rank < TOPK) topk[n * TOPK + rank] = c;
  if (scores_out) scores_out[n * FC + c] = score;
}

// ---------------------------------------------------------------- slot map
// One thread per image: compaction of non-zero boxes (keypoint_model.py:149-153),
// and the "no valid person" dummy (vis class 0 = 1, :171-179).
__device__ __forceinline__ void slotmap_image(const float* __restrict__ boxes, int b, int P, int32_t* __restrict__ slot) {
  int cnt = 0;
  for (int p = 0; p < P; ++p) {
    const float* bx = boxes + ((size_t)b * P + p) * 4;
    if (!(bx[0] == 0.f && bx[1] == 0.f && bx[2] == 0.f && bx[3] == 0.f)) ++cnt;
  }
  int valid = 0, empty = cnt;
  for (int p = 0; p < P; ++p) {
    const float* bx = boxes + ((size_t)b * P + p) * 4;
    const bool zero = bx[0] == 0.f && bx[1] == 0.f && bx[2] == 0.f && bx[3] == 0.f;
    if (zero) {
      slot[b * P + p] = slot_empty(empty, cnt == 0 && empty == 0);   // the dummy person sits at position 0
      ++empty;
    } else {
      slot[b * P + p] = valid++;
    }
  }
}
__global__ void slotmap_kernel(const float* __restrict__ boxes, int B, int P, int32_t* __restrict__ slot) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  slotmap_image(boxes, b, P, slot);
}

// ---------------------------------------------------------------- ROI align
// grid (56 output rows, R); 256 threads = 4 waves; lane = selected channel.
// feat: FPN level-0 NHWC [B][Hf][Wf][Cf]; channel gather through topk (the
// reference materialises features[b, topk] first -- here it is an index).
// Also emits per-(roi,row) channel sum/max partials for HeatmapHead attention.
// CW = channels per lane: 1 -> the 64 top-k channels (HeatmapHead input),
// 2 -> all 128 FPN channels in order (KEYPOINT_HEAD input, topk == nullptr).
constexpr int kRoiStageFloats = 12800;   // 50 KB (one interpolated row: 200 columns x 64 / 100 x 128 channels): 3 workgroups per CU
// One output row ph of ROI r (all 56 bins) for CW x 64 channels: torchvision
// roi_align sampling (aligned=False, sampling_ratio=-1) summed per bin in
// acc[j][q] (bin pw = wave + 4 j, channel lane + 64 q, or topk[b][lane]);
// divide by *count for the average.  stage: the dynamic LDS of stage_cap
// floats for the separable path (stage_cap 0: direct gathers).
template <int CW>
__device__ __forceinline__ void roi_row_sample(const float* __restrict__ feat, int Hf, int Wf, int Cf,
                                               const int32_t* __restrict__ topk, const float* __restrict__ boxes,
                                               int ph, int r, int b, int stage_cap, float* stage,
                                               float (&acc)[HM / 4][CW], float* count_out,
                                               unsigned long long* __restrict__ stamps) {
  auto stamp = [&](int i) {
    if (stamps && threadIdx.x == 0)
      stamps[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 + i] = __builtin_amdgcn_s_memrealtime();
  };
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int CO = TOPK * CW;
  const float* bx = boxes + (size_t)r * 4;
  const float cx = bx[0], cy = bx[1], bw = bx[2], bh = bx[3];
  const float x1 = fminf(fmaxf(cx - bw / 2.f, 0.f), 1.f) * (float)Wf;
  const float y1 = fminf(fmaxf(cy - bh / 2.f, 0.f), 1.f) * (float)Hf;
  const float x2 = fminf(fmaxf(cx + bw / 2.f, 0.f), 1.f) * (float)Wf;
  const float y2 = fminf(fmaxf(cy + bh / 2.f, 0.f), 1.f) * (float)Hf;
  const float roi_w = fmaxf(x2 - x1, 1.f), roi_h = fmaxf(y2 - y1, 1.f);
  const float bin_w = roi_w / (float)HM, bin_h = roi_h / (float)HM;
  const int gw = (int)ceilf(roi_w / (float)HM), gh = (int)ceilf(roi_h / (float)HM);
  const float count = (float)max(gw * gh, 1);
  *count_out = count;
  const float* fb = feat + (size_t)b * Hf * Wf * Cf;

  // The wave's 14 bins (pw = wave + 4 j) advance together through the
  // sampling grid: for each (iy, ix) the 4 corner loads of all 14 bins are
  // issued before any is used (56 gathers in flight per lane instead of one
  // bin's 4), and every bin still sums its samples in (iy, ix) order, i.e. the
  // arithmetic is the scalar loop's.  A sample outside [-1, H] x [-1, W]
  // contributes 0 (torchvision's skip).
  constexpr int NB = HM / 4;
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int q = 0; q < CW; ++q) acc[j][q] = 0.f;
  // Staged (separable) path: bilinear sampling is separable -- a sample's
  // value is hx (hy F[yl][xl] + ly F[yh][xl]) + lx (hy F[yl][xh] + ly F[yh][xh])
  // and the validity test is (y in range) && (x in range) -- so for each
  // sample row iy the vertically interpolated row T[x] = hy F[yl][x] +
  // ly F[yh][x] over the row's column span [xlo, xhi] is built in LDS once
  // (each source element read from L2 once per sample row, not once per
  // output bin and corner: ~3x fewer L1 / L2 loads), then every bin reads T at
  // its two columns.  Same sample positions and weights as the direct path
  // (the sums associate differently: fp32 rounding only).  Column spans wider
  // than the stage fall back to the direct gathers.
  auto sample_y = [&](int iy, bool& yin, int& yl, int& yh, float& ly, float& hy) {
    const float y = y1 + (float)ph * bin_h + ((float)iy + 0.5f) * bin_h / (float)gh;
    yin = !(y < -1.f || y > (float)Hf);
    float yy = y <= 0.f ? 0.f : y;
    yl = (int)yy;
    if (yl >= Hf - 1) { yh = yl = Hf - 1; yy = (float)yl; } else yh = yl + 1;
    ly = yy - (float)yl;
    hy = 1.f - ly;
  };
  auto sample_x = [&](int pw, int ix, int& xl, int& xh, float& lx, float& hx, bool& xin) {
    const float x = x1 + (float)pw * bin_w + ((float)ix + 0.5f) * bin_w / (float)gw;
    xin = !(x < -1.f || x > (float)Wf);
    float xx = x <= 0.f ? 0.f : x;
    xl = (int)xx;
    if (xl >= Wf - 1) { xh = xl = Wf - 1; xx = (float)xl; } else xh = xl + 1;
    lx = xx - (float)xl;
    hx = 1.f - lx;
  };
  bool staged = false;
  int xlo = 0, nc = 0;
  {
    bool t0;
    int a0, xhi, d0;
    float f0, f1;
    sample_x(0, 0, xlo, d0, f0, f1, t0);
    sample_x(HM - 1, gw - 1, a0, xhi, f0, f1, t0);
    nc = xhi - xlo + 1;
    staged = nc > 0 && nc * CO <= stage_cap;   // stage_cap: the launch's dynamic LDS (floats)
  }
  if (staged) {
    int chs[CW];
#pragma unroll
    for (int q = 0; q < CW; ++q) chs[q] = topk ? topk[b * TOPK + lane] : lane + TOPK * q;
    for (int iy = 0; iy < gh; ++iy) {
      bool yin;
      int yl, yh;
      float ly, hy;
      sample_y(iy, yin, yl, yh, ly, hy);
      if (iy) __syncthreads();   // every bin finished reading the previous row's T
      const float* r1 = fb + (size_t)yl * Wf * Cf;
      const float* r2 = fb + (size_t)yh * Wf * Cf;
      if (topk == nullptr && Cf == CO) {
        // every channel in order (CW 2: the 128-channel KEYPOINT_HEAD rows):
        // 16-byte loads, lane = (column, channel quad), CPI columns per
        // wave-instruction -- a quarter of the load / LDS-store instructions of
        // the per-channel form below, the same T values
        constexpr int QPC = CO / 4, CPI = 64 / QPC, UB4 = 4;
        const int qd = lane % QPC, cs = lane / QPC;
        for (int base = wave * CPI; base < nc; base += 4 * CPI * UB4) {
          float4 v1[UB4], v2[UB4];
#pragma unroll
          for (int u = 0; u < UB4; ++u) {
            const int px = min(base + u * 4 * CPI + cs, nc - 1);
            const size_t o = (size_t)(xlo + px) * Cf + qd * 4;
            v1[u] = *reinterpret_cast<const float4*>(r1 + o);
            v2[u] = *reinterpret_cast<const float4*>(r2 + o);
          }
#pragma unroll
          for (int u = 0; u < UB4; ++u) {
            const int px = base + u * 4 * CPI + cs;
            if (px < nc) {
              float4 t;
              t.x = yin ? hy * v1[u].x + ly * v2[u].x : 0.f;
              t.y = yin ? hy * v1[u].y + ly * v2[u].y : 0.f;
              t.z = yin ? hy * v1[u].z + ly * v2[u].z : 0.f;
              t.w = yin ? hy * v1[u].w + ly * v2[u].w : 0.f;
              *reinterpret_cast<float4*>(stage + px * CO + qd * 4) = t;
            }
          }
        }
      } else {
      // 8 columns per wave per batch, every load of a batch in flight before
      // the first use (one L2 round trip per batch instead of per column)
      constexpr int UB = 8;
      for (int base = wave; base < nc; base += 4 * UB) {
        float v1[UB][CW], v2[UB][CW];
#pragma unroll
        for (int u = 0; u < UB; ++u) {
          const int px = min(base + 4 * u, nc - 1);
          const size_t o = (size_t)(xlo + px) * Cf;
#pragma unroll
          for (int q = 0; q < CW; ++q) {
            v1[u][q] = r1[o + chs[q]];
            v2[u][q] = r2[o + chs[q]];
          }
        }
#pragma unroll
        for (int u = 0; u < UB; ++u) {
          const int px = base + 4 * u;
          if (px < nc)
#pragma unroll
            for (int q = 0; q < CW; ++q) stage[px * CO + lane + TOPK * q] = yin ? hy * v1[u][q] + ly * v2[u][q] : 0.f;
        }
      }
      }
      __syncthreads();
      if (iy == 0) stamp(1);
      for (int ix = 0; ix < gw; ++ix) {
        // a bin's sample column is the same for every channel: lane j < NB
        // computes bin wave + 4 j's (sample_x) and the bins take theirs by lane
        // broadcasts, instead of every lane repeating all 14 bins' arithmetic
        int cxl = 0, cxh = 0, cin = 0;
        float clx = 0.f, chx = 0.f;
        if (lane < NB) {
          int xl, xh;
          float lx, hx;
          bool xin;
          sample_x(wave + 4 * lane, ix, xl, xh, lx, hx, xin);
          cxl = (xl - xlo) * CO;
          cxh = (xh - xlo) * CO;
          clx = lx;
          chx = hx;
          cin = xin ? 1 : 0;
        }
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const int oxl = __builtin_amdgcn_readlane(cxl, j), oxh = __builtin_amdgcn_readlane(cxh, j);
          const float lx = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, clx), j));
          const float hx = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, chx), j));
          const bool xin = __builtin_amdgcn_readlane(cin, j) != 0;
#pragma unroll
          for (int q = 0; q < CW; ++q) {
            const float v = hx * stage[oxl + lane + TOPK * q] + lx * stage[oxh + lane + TOPK * q];
            acc[j][q] += xin ? v : 0.f;
          }
        }
      }
    }
  }
  if (!staged) {
  int ch[CW];
#pragma unroll
  for (int q = 0; q < CW; ++q) ch[q] = topk ? topk[b * TOPK + lane] : lane + TOPK * q;
  for (int iy = 0; iy < gh; ++iy) {
    float y = y1 + (float)ph * bin_h + ((float)iy + 0.5f) * bin_h / (float)gh;
    const bool yin = !(y < -1.f || y > (float)Hf);
    float yy = y <= 0.f ? 0.f : y;
    int yl = (int)yy, yh;
    if (yl >= Hf - 1) { yh = yl = Hf - 1; yy = (float)yl; } else yh = yl + 1;
    const float ly = yy - (float)yl, hy = 1.f - ly;
    // the bins in groups of NBG; each bin still sums its samples in (iy, ix)
    // order.  CW 2 (roi_kh_kernel): one bin at a time -- this direct-gather
    // fallback only runs for maps wider than the stage (Wf > 100), and its
    // gathers in flight set the kernel's register peak (168 VGPRs with
    // spills at two groups of 7; 127 at one bin: four workgroups per CU)
    constexpr int NBG = CW == 2 ? 1 : NB;
    for (int ix = 0; ix < gw; ++ix)
#pragma unroll
    for (int j0 = 0; j0 < NB; j0 += NBG) {
      float v[NBG][4][CW], wgt[NBG][4];
#pragma unroll
      for (int jj = 0; jj < NBG; ++jj) {
        const int j = j0 + jj, pw = wave + 4 * j;
        float x = x1 + (float)pw * bin_w + ((float)ix + 0.5f) * bin_w / (float)gw;
        const bool in = yin && !(x < -1.f || x > (float)Wf);
        float xx = x <= 0.f ? 0.f : x;
        int xl = (int)xx, xh;
        if (xl >= Wf - 1) { xh = xl = Wf - 1; xx = (float)xl; } else xh = xl + 1;
        const float lx = xx - (float)xl, hx = 1.f - lx;
        wgt[jj][0] = in ? hy * hx : 0.f; wgt[jj][1] = in ? hy * lx : 0.f;
        wgt[jj][2] = in ? ly * hx : 0.f; wgt[jj][3] = in ? ly * lx : 0.f;
        const float* p1 = fb + ((size_t)yl * Wf + xl) * Cf;
        const float* p2 = fb + ((size_t)yl * Wf + xh) * Cf;
        const float* p3 = fb + ((size_t)yh * Wf + xl) * Cf;
        const float* p4 = fb + ((size_t)yh * Wf + xh) * Cf;
#pragma unroll
        for (int q = 0; q < CW; ++q) {
          v[jj][0][q] = p1[ch[q]]; v[jj][1][q] = p2[ch[q]]; v[jj][2][q] = p3[ch[q]]; v[jj][3][q] = p4[ch[q]];
        }
      }
#pragma unroll
      for (int jj = 0; jj < NBG; ++jj)
#pragma unroll
        for (int q = 0; q < CW; ++q)
          acc[j0 + jj][q] += wgt[jj][0] * v[jj][0][q] + wgt[jj][1] * v[jj][1][q] + wgt[jj][2] * v[jj][2][q] +
                             wgt[jj][3] * v[jj][3][q];
    }
  }
  }
}

template <int CW>
__global__ __launch_bounds__(256) void roi_align_kernel(const float* __restrict__ feat, int Hf, int Wf, int Cf,
                                                        const int32_t* __restrict__ topk,
                                                        const float* __restrict__ boxes, int P,
                                                        float* __restrict__ roi, float* __restrict__ roi_stats,
                                                        int stage_cap, unsigned long long* __restrict__ stamps) {
  __shared__ float red[4][2][TOPK];
  extern __shared__ float stage[];
  constexpr int CO = TOPK * CW, NB = HM / 4;
  const int ph = blockIdx.x, r = blockIdx.y, b = r / P;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (stamps && threadIdx.x == 0)
    stamps[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8] = __builtin_amdgcn_s_memrealtime();
  float acc[NB][CW], count;
  roi_row_sample<CW>(feat, Hf, Wf, Cf, topk, boxes, ph, r, b, stage_cap, stage, acc, &count, stamps);
  auto stamp = [&](int i) {
    if (stamps && threadIdx.x == 0)
      stamps[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 + i] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(2);
  float s_sum = 0.f, s_max = -INFINITY;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int pw = wave + 4 * j;
#pragma unroll
    for (int q = 0; q < CW; ++q) {
      const float v = acc[j][q] / count;
      roi[(((size_t)r * HM + ph) * HM + pw) * CO + lane + TOPK * q] = v;
      s_sum += v;
      s_max = fmaxf(s_max, v);
    }
  }
  if (roi_stats == nullptr) return;   // (CW == 1 only) HeatmapHead attention partials
  red[wave][0][lane] = s_sum;
  red[wave][1][lane] = s_max;
  __syncthreads();
  if (wave == 0) {
    const float s = red[0][0][lane] + red[1][0][lane] + red[2][0][lane] + red[3][0][lane];
    const float m = fmaxf(fmaxf(red[0][1][lane], red[1][1][lane]), fmaxf(red[2][1][lane], red[3][1][lane]));
    float* st = roi_stats + ((size_t)r * HM + ph) * 2 * TOPK;
    st[lane] = s;
    st[TOPK + lane] = m;
  }
  stamp(3);
}

// ---------------------------------------------------------------- ROI align + KEYPOINT_HEAD attention
// Dual-head forward, split precision: the two ROI aligns of a box (the 64
// top-k channels for HeatmapHead, all 128 FPN channels for KEYPOINT_HEAD,
// keypoint_model.py:212-228 / keypoint_head.py:51-54) sample the same
// positions, so one pass over the 128 channels serves both, and
// KEYPOINT_HEAD's spatial attention (keypoint_head.py:15-20,53-54:
// att = sigmoid(b2 + w2 . relu6(W1 x + b1)), x * att) is per pixel, so it runs
// on the row while it is in registers.  grid (56 rows, R), 256 threads; lane
// = channels lane, lane + 64 (roi_row_sample<2>).  Outputs:
//   roi / roi_stats: the top-k channels (lane <- channel topk[b][lane] by a
//     cross-lane read), as roi_align_kernel<1> writes them;
//   out: x * att * 2^a as the split [hi32 | lo32] operand of the first
//     KEYPOINT_HEAD conv, interior of the zero-bordered [R][57 x 57][128] map
//     (a = split_exp_of(bound of the image), hsc[r][2] = that bound), staged
//     in LDS and stored as whole 28 KB rows;
// replacing roi_align_kernel<1>, roi_align_kernel<2> (whose 128-channel fp32
// map went through HBM twice) and kh_att2_kernel.  The attention's 1x1 128 ->
// 64 runs on v_mfma_f32_16x16x32_f16 with the three split products (lo.hi,
// hi.hi, hi.lo) and the 64 -> 1 dot by 16-lane butterflies and a 4-wave sum:
// the arithmetic of kh_att2_kernel.
constexpr int kKaRow = 528;   // LDS bytes per pixel of the attention operand: hi 256 | lo 256 | 16 pad
constexpr int kRoiKhLds = 64 * kKaRow;   // (>= 56 x 512 output staging)
__global__ __launch_bounds__(256, 4) void roi_kh_kernel(const float* __restrict__ feat, int Hf, int Wf,
                                                     const int32_t* __restrict__ topk,
                                                     const float* __restrict__ boxes, int P,
                                                     float* __restrict__ roi, float* __restrict__ roi_stats,
                                                     int stage_cap, const _Float16* __restrict__ w1s, int w1_exp,
                                                     const float* __restrict__ b1, const float* __restrict__ w2,
                                                     const float* __restrict__ b2, const float* __restrict__ bound,
                                                     int bdiv, int bstride, float* __restrict__ hsc,
                                                     _Float16* __restrict__ out,
                                                     unsigned long long* __restrict__ stamps) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  // KPD_STAMPS (diagnostic): start | first T row | sampled | top-k + stats |
  // attention | stored (vmcnt drained)
  auto stamp = [&](int i) {
    if (stamps && threadIdx.x == 0)
      stamps[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 + i] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  __shared__ float red[4][2][TOPK];
  __shared__ float spart[4][64];
  __shared__ float satt[64];
  extern __shared__ __attribute__((aligned(16))) float stage[];
  constexpr int NB = HM / 4;
  const int ph = blockIdx.x, r = blockIdx.y, b = r / P;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, r16 = lane & 15;
  const int co = wave * 16 + r16;
  const int tch = topk[b * TOPK + lane];
  const float bnd = bound[(size_t)(r / bdiv) * bstride];
  if (tid == 0 && ph == 0) hsc[(size_t)r * 4 + 2] = bnd;

  float acc[NB][2], count;
  roi_row_sample<2>(feat, Hf, Wf, 2 * TOPK, nullptr, boxes, ph, r, b, stage_cap, stage, acc, &count, stamps);
  stamp(2);
  // attention weights (wave w: output channels 16 w .. 16 w + 15), loaded
  // after the sampling (held through it they cost the kernel its occupancy);
  // their latency overlaps the top-k / statistics phase below
  h8 bh[4], bl[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const _Float16* wp = w1s + (size_t)co * 256 + c * 64 + g * 8;
    bh[c] = *reinterpret_cast<const h8*>(wp);
    bl[c] = *reinterpret_cast<const h8*>(wp + 32);
  }
  const float bias1 = b1[co], wo2 = w2[co], bias2 = b2[0];
  const int ea = split_exp_of(bnd);
  const float sc = ldexpf(1.f, ea), us = ldexpf(1.f, -(ea + w1_exp));
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    acc[j][0] /= count;
    acc[j][1] /= count;
  }
  // HeatmapHead input: channel topk[lane] of the row (held by lane tch & 63,
  // slot tch >> 6 of the same wave) + the per-row channel sum / max partials
  {
    const int src = (tch & 63) * 4;
    const bool hi_half = tch >= 64;
    float s_sum = 0.f, s_max = -INFINITY;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const float a0 = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(acc[j][0])));
      const float a1 = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(acc[j][1])));
      const float v = hi_half ? a1 : a0;
      roi[(((size_t)r * HM + ph) * HM + wave + 4 * j) * TOPK + lane] = v;
      s_sum += v;
      s_max = fmaxf(s_max, v);
    }
    red[wave][0][lane] = s_sum;
    red[wave][1][lane] = s_max;
  }
  __syncthreads();   // every wave's reads of the sampling stage are done: it becomes the operand image
  if (wave == 0) {
    const float s = red[0][0][lane] + red[1][0][lane] + red[2][0][lane] + red[3][0][lane];
    const float m = fmaxf(fmaxf(red[0][1][lane], red[1][1][lane]), fmaxf(red[2][1][lane], red[3][1][lane]));
    float* st = roi_stats + ((size_t)r * HM + ph) * 2 * TOPK;
    st[lane] = s;
    st[TOPK + lane] = m;
  }
  stamp(3);
  char* img = reinterpret_cast<char*>(stage);
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float xs = acc[j][q] * sc;
      const _Float16 hi = (_Float16)xs, lo = (_Float16)(xs - (float)hi);
      char* rowp = img + (wave + 4 * j) * kKaRow + (lane + TOPK * q) * 2;
      *reinterpret_cast<_Float16*>(rowp) = hi;
      *reinterpret_cast<_Float16*>(rowp + 256) = lo;
    }
  __syncthreads();
  // 1x1 128 -> 64 on 64 pixel rows (rows 56-63 are don't-care: every MFMA row
  // depends on its own A row only, and their results are dropped)
  f32x4 am[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) am[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const char* rowp = img + (i * 16 + r16) * kKaRow + c * 64 + g * 16;
      const h8 ah = *reinterpret_cast<const h8*>(rowp), al = *reinterpret_cast<const h8*>(rowp + 256);
      am[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[c], am[i], 0, 0, 0);
      am[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[c], am[i], 0, 0, 0);
      am[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[c], am[i], 0, 0, 0);
    }
  // lane (g, r16) holds pixels 16 i + 4 g + e of output channel co
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float pv = wo2 * fminf(fmaxf(fmaf(am[i][e], us, bias1), 0.f), 6.f);
      pv = row16_sum(pv);   // the 16 output channels of the wave (DPP butterfly)
      if (r16 == 0) spart[wave][i * 16 + g * 4 + e] = pv;
    }
  __syncthreads();   // (also: every wave's operand reads are done -- the image becomes the output stage)
  if (tid < 64) satt[tid] = kpd_sigmoid(bias2 + ((spart[0][tid] + spart[1][tid]) + (spart[2][tid] + spart[3][tid])));
  __syncthreads();
  stamp(4);
  // x * att * 2^a as f16 hi / lo in the [hi32 | lo32] groups of the padded map's row
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int pw = wave + 4 * j;
    const float att = satt[pw];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c = lane + TOPK * q;
      const float xs = (acc[j][q] * att) * sc;
      const _Float16 hi = (_Float16)xs, lo = (_Float16)(xs - (float)hi);
      char* o = img + pw * 512 + (c >> 5) * 128 + (c & 31) * 2;
      *reinterpret_cast<_Float16*>(o) = hi;
      *reinterpret_cast<_Float16*>(o + 64) = lo;
    }
  }
  __syncthreads();
  // the 56 pixels of row ph are one contiguous 28 KB run of the hmconv layout
  uint4* dst = reinterpret_cast<uint4*>(out + hm_pos(r, ph, 0) * 256);
  const uint4* srcs = reinterpret_cast<const uint4*>(img);
#pragma unroll
  for (int k = 0; k < HM * 512 / 16 / 256; ++k) dst[tid + 256 * k] = srcs[tid + 256 * k];
  if (stamps) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(5);
  }
}

// ---------------------------------------------------------------- HeatmapHead channel attention
// grid R, 64 threads.  cw[r][c] = sigmoid(fc(avg) + fc(max)), fc = 64->4 ReLU ->64.
__global__ __launch_bounds__(64) void hm_chattn_kernel(const float* __restrict__ roi_stats,
                                                       const float* __restrict__ w0, const float* __restrict__ b0,
                                                       const float* __restrict__ w2, const float* __restrict__ b2,
                                                       float* __restrict__ cw, float* __restrict__ hsc,
                                                       int abs_in) {
  __shared__ float avg[TOPK], mx[TOPK], h[8];
  const int r = blockIdx.x, c = threadIdx.x;
  const float* st = roi_stats + (size_t)r * HM * 2 * TOPK;
  float s = 0.f, m = -INFINITY;
  // rows in batches of 14: 28 loads in flight, sums still in row order
  constexpr int RB = 14;
  static_assert(HM % RB == 0, "row batches");
  for (int row0 = 0; row0 < HM; row0 += RB) {
    float vs[RB], vm[RB];
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      vs[u] = st[(row0 + u) * 2 * TOPK + c];
      vm[u] = st[(row0 + u) * 2 * TOPK + TOPK + c];
    }
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      s += vs[u];
      m = fmaxf(m, vm[u]);
    }
  }
  avg[c] = s / (float)HMP;
  mx[c] = m;
  if (hsc) {   // split heatmap convs: U0 = max of the ROI features bounds |xs| (sigmoid gates <= 1)
    float u0 = fmaxf(wave_max(m), 0.f);
    if (abs_in) u0 = fmaxf(u0, hsc[(size_t)r * 4 + 2]);   // features of either sign: max |x|
    if (c == 0) {
      hsc[(size_t)r * 4] = u0;
      hsc[(size_t)r * 4 + 1] = 0.f;   // max|h1|, published by heatmap conv 1
    }
  }
  __syncthreads();
  if (c < 8) {
    const int j = c & 3;
    const float* v = (c < 4) ? avg : mx;
    float a = b0[j];
#pragma unroll 16
    for (int k = 0; k < TOPK; ++k) a = fmaf(w0[j * TOPK + k], v[k], a);
    h[c] = fmaxf(a, 0.f);
  }
  __syncthreads();
  float oa = b2[c], om = b2[c];
  for (int j = 0; j < 4; ++j) {
    oa = fmaf(w2[c * 4 + j], h[j], oa);
    om = fmaf(w2[c * 4 + j], h[4 + j], om);
  }
  cw[(size_t)r * TOPK + c] = kpd_sigmoid(oa + om);
}

template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}

// ---------------------------------------------------------------- spatial pool
// grid (56 rows, R), one wave.  smap[r][y][x] = {mean_c, max_c} of roi*cw.
// Lane (p, c) = (lane >> 4, lane & 15) holds channels 4c .. 4c+3 of pixel
// 4i + p: every load instruction reads 4 whole 256-byte pixel rows (1 KiB
// contiguous; a pixel per lane touched 64 lines per instruction), and all 14
// loads of the row are in flight before the first use.  The channel sum runs
// 4-wide in the lane, then over the 16 lanes of the pixel (xor 1, 2, 4, 8).
__global__ __launch_bounds__(64) void hm_spool_kernel(const float* __restrict__ roi, const float* __restrict__ cw,
                                                      float* __restrict__ smap) {
  constexpr int NI = HM / 4;
  const int y = blockIdx.x, r = blockIdx.y, lane = threadIdx.x, pp = lane >> 4, c = lane & 15;
  const float4* src = reinterpret_cast<const float4*>(roi + ((size_t)r * HM + y) * HM * TOPK);
  float4 v[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) v[i] = src[(4 * i + pp) * (TOPK / 4) + c];
  const float4 w = reinterpret_cast<const float4*>(cw + (size_t)r * TOPK)[c];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const float a = v[i].x * w.x, b = v[i].y * w.y, cc = v[i].z * w.z, d = v[i].w * w.w;
    float s = (a + b) + (cc + d), m = fmaxf(fmaxf(a, b), fmaxf(cc, d));
    // all-reduce inside the 16-lane row by DPP (quad xor 1, 2; row rotate 4, 8)
    s += dpp_f<0xB1>(s); m = fmaxf(m, dpp_f<0xB1>(m));
    s += dpp_f<0x4E>(s); m = fmaxf(m, dpp_f<0x4E>(m));
    s += dpp_f<0x124>(s); m = fmaxf(m, dpp_f<0x124>(m));
    s += dpp_f<0x128>(s); m = fmaxf(m, dpp_f<0x128>(m));
    if (c == 0) {
      const size_t pix = ((size_t)r * HM + y) * HM + 4 * i + pp;
      *reinterpret_cast<float2*>(smap + pix * 2) = make_float2(s / (float)TOPK, m);
    }
  }
}

// ---------------------------------------------------------------- spatial apply
// grid (56 rows, R), one wave.  sw = sigmoid(conv7x7([mean,max]) + b) per
// pixel (lane x < 56, LDS), then xs = (roi * cw) * sw with lane (p, c) on
// channels 4c .. 4c+3 of pixel 4i + p (1 KiB contiguous per load, the roi row
// loads issued first), stored as the first heatmap conv's operand: bf16
// zero-bordered [R][57 x 57][64] (out_bf16 == 2), bf16 [R][3136][64] (1),
// f32 (0), or (3) zero-bordered f16 hi | lo of xs * 2^a0(r), 32-channel
// [hi32 | lo32] groups, a0 = split_exp_of(hsc[r][0]) (split heatmap convs).
__global__ __launch_bounds__(64) void hm_sapply_kernel(const float* __restrict__ roi, const float* __restrict__ cw,
                                                       const float* __restrict__ smap, const float* __restrict__ saw,
                                                       const float* __restrict__ sab, void* __restrict__ xs,
                                                       int out_bf16, const float* __restrict__ hsc, int use_sp,
                                                       float* __restrict__ sw_out) {
  constexpr int NI = HM / 4;
  __shared__ float w[98];
  __shared__ float2 srow[7][HM + 6];   // the 7 smap rows around y, zero-padded by 3 columns
  __shared__ float ssw[HM];
  const int y = blockIdx.x, r = blockIdx.y, x = threadIdx.x, pp = x >> 4, c = x & 15;
  const float* sm = smap + (size_t)r * HMP * 2;
  const float4* src = reinterpret_cast<const float4*>(roi + ((size_t)r * HM + y) * HM * TOPK);
  float4 v[NI];
  {   // every load of the workgroup issued before the first LDS store
#pragma unroll
    for (int i = 0; i < NI; ++i) v[i] = src[(4 * i + pp) * (TOPK / 4) + c];
    float2 sv[7];
#pragma unroll
    for (int ky = 0; ky < 7; ++ky) {
      const int iy = y + ky - 3;
      sv[ky] = (x < HM && iy >= 0 && iy < HM) ? *reinterpret_cast<const float2*>(sm + (iy * HM + x) * 2)
                                                : make_float2(0.f, 0.f);
    }
    const float w0v = saw[x], w1v = x + 64 < 98 ? saw[x + 64] : 0.f;
#pragma unroll
    for (int ky = 0; ky < 7; ++ky) {
      if (x < HM) srow[ky][x + 3] = sv[ky];
      if (x < 3) { srow[ky][x] = make_float2(0.f, 0.f); srow[ky][HM + 3 + x] = make_float2(0.f, 0.f); }
    }
    w[x] = w0v;
    if (x + 64 < 98) w[x + 64] = w1v;
  }
  __syncthreads();
  if (x < HM) {
    // same tap order (ky, kx) as the reference conv; out-of-image taps add 0
    float a = 0.f;
#pragma unroll
    for (int ky = 0; ky < 7; ++ky) {
      const int iy = y + ky - 3;
      if (iy < 0 || iy >= HM) continue;
#pragma unroll
      for (int kx = 0; kx < 7; ++kx) {
        const int ix = x + kx - 3;
        if (ix < 0 || ix >= HM) continue;
        const float2 sv2 = srow[ky][x + kx];
        a = fmaf(w[ky * 7 + kx], sv2.x, a);
        a = fmaf(w[49 + ky * 7 + kx], sv2.y, a);
      }
    }
    ssw[x] = use_sp ? kpd_sigmoid(a + sab[0]) : 1.f;
    if (sw_out) sw_out[((size_t)r * HM + y) * HM + x] = ssw[x];
  }
  const float4 cq = reinterpret_cast<const float4*>(cw + (size_t)r * TOPK)[c];
  const float ssc = out_bf16 == 3 ? ldexpf(1.f, split_exp_of(hsc[(size_t)r * 4])) : 1.f;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int px = 4 * i + pp;
    const float sw = ssw[px];
    const float4 o = make_float4((v[i].x * cq.x) * sw, (v[i].y * cq.y) * sw, (v[i].z * cq.z) * sw, (v[i].w * cq.w) * sw);
    if (out_bf16 == 3) {
      const size_t opix = hm_pos(r, y, px);
      const float ov[4] = {o.x * ssc, o.y * ssc, o.z * ssc, o.w * ssc};
      f16x4 hi, lo;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        hi[e] = (_Float16)ov[e];
        lo[e] = (_Float16)(ov[e] - (float)hi[e]);
      }
      _Float16* ob = reinterpret_cast<_Float16*>(xs) + opix * 2 * TOPK + (c >> 3) * 64 + (c & 7) * 4;
      *reinterpret_cast<f16x4*>(ob) = hi;
      *reinterpret_cast<f16x4*>(ob + 32) = lo;
    } else if (out_bf16) {
      const size_t opix = out_bf16 == 2 ? hm_pos(r, y, px)
                                        : ((size_t)r * HM + y) * HM + px;
      bf16x4 ob;
      ob[0] = (__bf16)o.x; ob[1] = (__bf16)o.y; ob[2] = (__bf16)o.z; ob[3] = (__bf16)o.w;
      *reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(xs) + opix * TOPK + 4 * c) = ob;
    } else {
      reinterpret_cast<float4*>(reinterpret_cast<float*>(xs) + (((size_t)r * HM + y) * HM + px) * TOPK)[c] = o;
    }
  }
}

// ---------------------------------------------------------------- spatial pool + apply, fused
// hm_spool_kernel and hm_sapply_kernel in one launch: a 512-thread workgroup
// takes a band of BR = 8 rows of one ROI.  (A) its waves pool the band's rows
// and the 3-row halo on either side (mean and max over channels of roi * cw,
// as hm_spool_kernel: same lane layout and reduction order) into LDS;
// (B) sw for the band's pixels (the 7x7 conv, same tap order as
// hm_sapply_kernel); (C) one wave per band row re-reads that row (the same
// workgroup read it in (A): an L2 hit) and applies cw * sw with the same
// output modes.  The map never reaches HBM and the ROI features leave HBM
// once.  Bands of one ROI are consecutive logical workgroups and a ROI's
// bands share an XCD (xcd-contiguous order; every ROI is the same work), so
// the halo rows a neighbour band re-reads are L2 hits.
constexpr int kAttBR = 8;
__global__ __launch_bounds__(512) void hm_attn_kernel(const float* __restrict__ roi, const float* __restrict__ cw,
                                                      const float* __restrict__ saw, const float* __restrict__ sab,
                                                      void* __restrict__ xs, int out_bf16, const float* __restrict__ hsc,
                                                      int use_sp, float* __restrict__ sw_out) {
  constexpr int NI = HM / 4, BR = kAttBR, PR = BR + 6;
  __shared__ float w[98];
  __shared__ float2 pool[PR][HM + 6];   // pooled rows y0 - 3 .. y0 + BR + 2, zero-padded by 3 columns
  __shared__ float ssw[BR][HM];
  const int nb = HM / BR;
  const int nblk = gridDim.x, L = blockIdx.x;
  // xcd-contiguous logical order (dispatch round-robins the 8 XCDs)
  const int qx = nblk / 8, rx = nblk % 8, x8 = L % 8, k8 = L / 8;
  const int g = (x8 < rx ? x8 * (qx + 1) : rx * (qx + 1) + (x8 - rx) * qx) + k8;
  const int r = g / nb, y0 = (g - r * nb) * BR;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, pp = lane >> 4, c = lane & 15;
  const float4 cq = reinterpret_cast<const float4*>(cw + (size_t)r * TOPK)[c];
  if (tid < 98) w[tid] = saw[tid];
  // zero padding columns of the pooled rows
  for (int i = tid; i < PR * 6; i += 512) {
    const int rr = i / 6, cc = i - rr * 6;
    pool[rr][cc < 3 ? cc : HM + cc] = make_float2(0.f, 0.f);
  }
  // (A) pooled rows: wave w takes rows y0 - 3 + w and + 8 (zero outside the ROI)
  for (int pr = wave; pr < PR; pr += 8) {
    const int y = y0 - 3 + pr;
    if (y < 0 || y >= HM) {
      if (lane < HM) pool[pr][lane + 3] = make_float2(0.f, 0.f);
      continue;
    }
    const float4* src = reinterpret_cast<const float4*>(roi + ((size_t)r * HM + y) * HM * TOPK);
    float4 v[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) v[i] = src[(4 * i + pp) * (TOPK / 4) + c];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const float a = v[i].x * cq.x, b = v[i].y * cq.y, cc = v[i].z * cq.z, d = v[i].w * cq.w;
      float sm = (a + b) + (cc + d), m = fmaxf(fmaxf(a, b), fmaxf(cc, d));
      sm += dpp_f<0xB1>(sm); m = fmaxf(m, dpp_f<0xB1>(m));
      sm += dpp_f<0x4E>(sm); m = fmaxf(m, dpp_f<0x4E>(m));
      sm += dpp_f<0x124>(sm); m = fmaxf(m, dpp_f<0x124>(m));
      sm += dpp_f<0x128>(sm); m = fmaxf(m, dpp_f<0x128>(m));
      if (c == 0) pool[pr][4 * i + pp + 3] = make_float2(sm / (float)TOPK, m);
    }
  }
  __syncthreads();
  // (B) sw of the band's pixels
  if (tid < BR * HM) {
    const int j = tid / HM, x = tid - j * HM, y = y0 + j;
    float a = 0.f;
#pragma unroll
    for (int ky = 0; ky < 7; ++ky) {
      const int iy = y + ky - 3;
      if (iy < 0 || iy >= HM) continue;
#pragma unroll
      for (int kx = 0; kx < 7; ++kx) {
        const int ix = x + kx - 3;
        if (ix < 0 || ix >= HM) continue;
        const float2 sv2 = pool[j + ky][x + kx];
        a = fmaf(w[ky * 7 + kx], sv2.x, a);
        a = fmaf(w[49 + ky * 7 + kx], sv2.y, a);
      }
    }
    ssw[j][x] = use_sp ? kpd_sigmoid(a + sab[0]) : 1.f;
    if (sw_out) sw_out[((size_t)r * HM + y) * HM + x] = ssw[j][x];
  }
  const float ssc = out_bf16 == 3 ? ldexpf(1.f, split_exp_of(hsc[(size_t)r * 4])) : 1.f;
  __syncthreads();
  // (C) band row wave: roi * cw * sw -> the first heatmap conv's operand
  {
    const int j = wave, y = y0 + j;
    const float4* src = reinterpret_cast<const float4*>(roi + ((size_t)r * HM + y) * HM * TOPK);
    float4 v[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) v[i] = src[(4 * i + pp) * (TOPK / 4) + c];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int px = 4 * i + pp;
      const float sw = ssw[j][px];
      const float4 o = make_float4((v[i].x * cq.x) * sw, (v[i].y * cq.y) * sw, (v[i].z * cq.z) * sw, (v[i].w * cq.w) * sw);
      if (out_bf16 == 3) {
        const size_t opix = hm_pos(r, y, px);
        const float ov[4] = {o.x * ssc, o.y * ssc, o.z * ssc, o.w * ssc};
        f16x4 hi, lo;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          hi[e] = (_Float16)ov[e];
          lo[e] = (_Float16)(ov[e] - (float)hi[e]);
        }
        _Float16* ob = reinterpret_cast<_Float16*>(xs) + opix * 2 * TOPK + (c >> 3) * 64 + (c & 7) * 4;
        *reinterpret_cast<f16x4*>(ob) = hi;
        *reinterpret_cast<f16x4*>(ob + 32) = lo;
      } else if (out_bf16) {
        const size_t opix = out_bf16 == 2 ? hm_pos(r, y, px)
                                          : ((size_t)r * HM + y) * HM + px;
        bf16x4 ob;
        ob[0] = (__bf16)o.x; ob[1] = (__bf16)o.y; ob[2] = (__bf16)o.z; ob[3] = (__bf16)o.w;
        *reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(xs) + opix * TOPK + 4 * c) = ob;
      } else {
        reinterpret_cast<float4*>(reinterpret_cast<float*>(xs) + (((size_t)r * HM + y) * HM + px) * TOPK)[c] = o;
      }
    }
  }
}

// ---------------------------------------------------------------- final 1x1 + sigmoid
// grid (56 rows, R), 64 threads (pixel x).  h3: [R][3136][64] f32.
// heat_out: [B][P][17][56][56] written at the box's compacted slot.
__global__ __launch_bounds__(64) void hm_final_kernel(const float* __restrict__ h3, const float* __restrict__ w,
                                                      const float* __restrict__ b, const int32_t* __restrict__ slot,
                                                      int P, float* __restrict__ heat_out) {
  __shared__ float sw[NK * TOPK];
  __shared__ float sb[NK];
  const int y = blockIdx.x, r = blockIdx.y, x = threadIdx.x;
  const int sl = slot[r];
  if (sl < 0) {   // all-zero box (skipped by the reference): its padding slot gets zeros
    if (x < HM) {
      float* dst = heat_out + ((size_t)((r / P) * P + slot_pos(sl)) * NK) * HMP + y * HM + x;
      for (int k = 0; k < NK; ++k) dst[(size_t)k * HMP] = 0.f;
    }
    return;
  }
  for (int i = x; i < NK * TOPK; i += 64) sw[i] = w[i];
  if (x < NK) sb[x] = b[x];
  __syncthreads();
  if (x >= HM) return;
  const int bimg = r / P;
  const size_t pix = ((size_t)r * HM + y) * HM + x;
  float v[TOPK];
  const float4* src = reinterpret_cast<const float4*>(h3 + pix * TOPK);
#pragma unroll
  for (int q = 0; q < TOPK / 4; ++q) {
    const float4 u = src[q];
    v[4 * q] = u.x; v[4 * q + 1] = u.y; v[4 * q + 2] = u.z; v[4 * q + 3] = u.w;
  }
  float* dst = heat_out + ((size_t)(bimg * P + sl) * NK) * HMP + y * HM + x;
  for (int k = 0; k < NK; ++k) {
    float a = 0.f;
#pragma unroll
    for (int c = 0; c < TOPK; ++c) a = fmaf(sw[k * TOPK + c], v[c], a);
    dst[(size_t)k * HMP] = kpd_sigmoid(a + sb[k]);
  }
}

// ---------------------------------------------------------------- decode
// grid (R, 17), one wave per (roi, keypoint); single pass over the 3136
// heatmap values with an online (running-max) softmax per lane, lanes then
// merged pairwise -- the heatmap is read once.
__global__ __launch_bounds__(64) void decode_kernel(const float* __restrict__ heat_out,
                                                    const float* __restrict__ boxes,
                                                    const int32_t* __restrict__ slot, int P,
                                                    float* __restrict__ kpts_out, float* __restrict__ vis_out) {
  const int r = blockIdx.x, k = blockIdx.y, lane = threadIdx.x;
  const int sl = slot[r];
  const int bimg = r / P;
  if (sl < 0) {   // padding slot: zeros; the dummy person of a box-less image is visibility class 0
    if (lane == 0) {
      const size_t o = (size_t)(bimg * P + slot_pos(sl)) * NK + k;
      kpts_out[o * 2 + 0] = 0.f;
      kpts_out[o * 2 + 1] = 0.f;
      vis_out[o * 3 + 0] = slot_dummy(sl) ? 1.f : 0.f;
      vis_out[o * 3 + 1] = 0.f;
      vis_out[o * 3 + 2] = 0.f;
    }
    return;
  }
  const size_t o = (size_t)(bimg * P + sl) * NK;
  const float cx = boxes[r * 4 + 0], cy = boxes[r * 4 + 1], bw = boxes[r * 4 + 2], bh = boxes[r * 4 + 3];
  {
    const float* hp = heat_out + (o + k) * HMP;
    // all 49 values of the lane loaded at once, then a two-pass softmax:
    // the wave max first, then the exp-weighted sums (butterfly-reduced)
    constexpr int NV = HMP / 64;
    static_assert(HMP % 64 == 0, "decode layout");
    float v[NV];
#pragma unroll
    for (int t = 0; t < NV; ++t) v[t] = hp[lane + 64 * t];
    float m = -INFINITY;
#pragma unroll
    for (int t = 0; t < NV; ++t) m = fmaxf(m, v[t]);
    m = wave_max(m);
    float se = 0.f, sx = 0.f, sy = 0.f;
#pragma unroll
    for (int t = 0; t < NV; ++t) {
      const int i = lane + 64 * t;
      const float e = expf(v[t] - m);
      se += e;
      sx = fmaf(e, (float)(i % HM), sx);
      sy = fmaf(e, (float)(i / HM), sy);
    }
    se = wave_sum(se);
    sx = wave_sum(sx);
    sy = wave_sum(sy);
    if (lane == 0) {
      const float kx = (sx / se) / (float)(HM - 1);
      const float ky = (sy / se) / (float)(HM - 1);
      const float px = fminf(fmaxf(kx * bw + (cx - bw / 2.f), 0.f), 1.f);
      const float py = fminf(fmaxf(ky * bh + (cy - bh / 2.f), 0.f), 1.f);
      kpts_out[(o + k) * 2 + 0] = px;
      kpts_out[(o + k) * 2 + 1] = py;
      const float conf = kpd_sigmoid(m);
      // compared as the reference does: conf.item() (a double) against 0.3 / 0.7
      const int cls = (double)conf < 0.3 ? 0 : ((double)conf < 0.7 ? 1 : 2);
      vis_out[(o + k) * 3 + 0] = cls == 0 ? 1.f : 0.f;
      vis_out[(o + k) * 3 + 1] = cls == 1 ? 1.f : 0.f;
      vis_out[(o + k) * 3 + 2] = cls == 2 ? 1.f : 0.f;
    }
  }
}

}  // namespace

hipError_t launch_topk(const float* stats, int N, int tiles, int HW, const float* w0, const float* b0,
                       const float* w2, const float* b2, int32_t* topk, float* scores, hipStream_t st,
                       const float* boxes, int P, int32_t* slot, float* imax, float* sc_zero, int sc_n) {
  if (slot && (!boxes || P <= 0 || P > 0xFFFF)) return hipErrorInvalidValue;
  const size_t lds = (size_t)2 * 8 * FC * 4;   // the two FC weights
  hipLaunchKernelGGL(topk_kernel, dim3(N), dim3(256), lds, st, stats, tiles, HW, w0, b0, w2, b2, topk, scores,
                     boxes, P, slot, imax, sc_zero, sc_n);
  return hipGetLastError();
}
hipError_t launch_slotmap(const float* boxes, int B, int P, int32_t* slot, hipStream_t st) {
  if (P > 0xFFFF) return hipErrorInvalidValue;
  hipLaunchKernelGGL(slotmap_kernel, dim3((B + 63) / 64), dim3(64), 0, st, boxes, B, P, slot);
  return hipGetLastError();
}
hipError_t launch_roi_align(const float* feat, int Hf, int Wf, int Cf, const int32_t* topk, const float* boxes,
                            int R, int P, float* roi, float* roi_stats, hipStream_t st, unsigned long long* stamps) {
  // the stage holds at most the map's width of interpolated columns: sized to
  // that (64 channels at Wf 96: 24 KB, 6 workgroups per CU instead of 3)
  static const bool full_cap = kpd_diag_env("KPD_ROI_FULLCAP") != nullptr;   // A/B: the fixed 50 KB stage
  if (topk) {
    static const bool direct = kpd_diag_env("KPD_ROI_DIRECT") != nullptr;   // A/B: no LDS stage
    const int cap = direct ? 0 : full_cap ? kRoiStageFloats : std::min(kRoiStageFloats, Wf * TOPK);
    hipLaunchKernelGGL((roi_align_kernel<1>), dim3(HM, R), dim3(256), cap * 4, st, feat, Hf, Wf, Cf, topk, boxes, P,
                       roi, roi_stats, cap, stamps);
  } else {
    if (Cf != 2 * TOPK) return hipErrorInvalidValue;
    static const bool direct = kpd_diag_env("KPD_ROI_DIRECT") != nullptr;   // A/B: no LDS stage
    const int cap = direct ? 0 : full_cap ? kRoiStageFloats : std::min(kRoiStageFloats, Wf * 2 * TOPK);
    hipLaunchKernelGGL((roi_align_kernel<2>), dim3(HM, R), dim3(256), cap * 4, st, feat, Hf, Wf, Cf, nullptr, boxes, P,
                       roi, nullptr, cap, stamps);
  }
  return hipGetLastError();
}
hipError_t launch_roi_kh(const float* feat, int Hf, int Wf, const int32_t* topk, const float* boxes, int R, int P,
                        float* roi, float* roi_stats, const void* w1s, int w1_exp, const float* b1, const float* w2,
                        const float* b2, const float* bound, int bdiv, int bstride, float* hsc, void* out,
                        hipStream_t st, unsigned long long* stamps) {
  if (R <= 0) return hipSuccess;
  if (!topk || !roi || !roi_stats || !w1s || !bound || bdiv < 1 || bstride < 1 || !hsc || !out)
    return hipErrorInvalidValue;
  // the sampling stage sized to the map width (128 channels), at least the
  // attention operand image it becomes afterwards
  const int cap = std::min(kRoiStageFloats, Wf * 2 * TOPK);
  const size_t lds = std::max<size_t>((size_t)cap * 4, kRoiKhLds);
  hipLaunchKernelGGL(roi_kh_kernel, dim3(HM, R), dim3(256), lds, st, feat, Hf, Wf, topk, boxes, P, roi, roi_stats,
                     cap, static_cast<const _Float16*>(w1s), w1_exp, b1, w2, b2, bound, bdiv, bstride, hsc,
                     static_cast<_Float16*>(out), stamps);
  return hipGetLastError();
}
hipError_t launch_hm_chattn(const float* roi_stats, int R, const float* w0, const float* b0, const float* w2,
                            const float* b2, float* cw, float* hsc, hipStream_t st, int abs_in) {
  hipLaunchKernelGGL(hm_chattn_kernel, dim3(R), dim3(64), 0, st, roi_stats, w0, b0, w2, b2, cw, hsc, abs_in);
  return hipGetLastError();
}
hipError_t launch_hm_spool(const float* roi, const float* cw, int R, float* smap, hipStream_t st) {
  hipLaunchKernelGGL(hm_spool_kernel, dim3(HM, R), dim3(64), 0, st, roi, cw, smap);
  return hipGetLastError();
}
hipError_t launch_hm_sapply(const float* roi, const float* cw, const float* smap, const float* saw,
                            const float* sab, int R, void* xs, int out_bf16, hipStream_t st, const float* hsc,
                            int use_sp, float* sw_out) {
  hipLaunchKernelGGL(hm_sapply_kernel, dim3(HM, R), dim3(64), 0, st, roi, cw, smap, saw, sab, xs, out_bf16, hsc,
                     use_sp, sw_out);
  return hipGetLastError();
}
hipError_t launch_hm_attn(const float* roi, const float* cw, const float* saw, const float* sab, int R, void* xs,
                          int out_bf16, hipStream_t st, const float* hsc, int use_sp, float* sw_out) {
  static_assert(HM % kAttBR == 0 && kAttBR == 8, "one wave per band row");
  if (R <= 0) return hipSuccess;
  hipLaunchKernelGGL(hm_attn_kernel, dim3((unsigned)(R * (HM / kAttBR))), dim3(512), 0, st, roi, cw, saw, sab, xs,
                     out_bf16, hsc, use_sp, sw_out);
  return hipGetLastError();
}
hipError_t launch_hm_final(const float* h3, int R, const float* w, const float* b, const int32_t* slot, int P,
                           float* heat_out, hipStream_t st) {
  hipLaunchKernelGGL(hm_final_kernel, dim3(HM, R), dim3(64), 0, st, h3, w, b, slot, P, heat_out);
  return hipGetLastError();
}
hipError_t launch_decode(const float* heat_out, const float* boxes, const int32_t* slot, int R, int P,
                         float* kpts_out, float* vis_out, hipStream_t st) {
  hipLaunchKernelGGL(decode_kernel, dim3(R, NK), dim3(64), 0, st, heat_out, boxes, slot, P, kpts_out, vis_out);
  return hipGetLastError();
}
