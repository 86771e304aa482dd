// Person-detector glue and KEYPOINT_HEAD ("dual head") kernels (gfx950).
//
// Person detector (reference PERSON_HEAD, dll/models/person_head.py:7-166; the
// reference never decodes or NMSes inside forward, so the glue is
// build-defined -- DESIGN.md §C3, oracle.kpd_oracle.person_detect):
//   pool:   FPN level 0 adaptive-avg-pooled to the 56x56 anchor grid
//   heads:  box_heads[0] / cls_heads[0] as one 1x1 MFMA conv (conv_mfma.hip)
//   decode: sigmoid score, threshold, anchor decode (this file)
//   NMS:    nms.hip, one workgroup per image, max_persons kept, zero padded
//
// KEYPOINT_HEAD (dll/models/keypoint_head.py:9-90) on the 128-channel ROI
// features: spatial attention apply (this file), ResidualBlocks and 3x3 convs
// on the MFMA conv kernel (post-affine epilogue for ResidualBlock.bn1),
// adaptive pools (this file), the two Linear layers as MFMA GEMMs, and
// LayerNorm + ReLU6 + Linear + sigmoid tails (this file).
#include <algorithm>

#include "kpd_common.h"
#include "kpd_kernels.h"
#include "conv_epilogue.h"

namespace {
constexpr int G = 56, GP = G * G, NA = 9;

// [B][Hf][Wf][C] -> [B][56][56][C], PyTorch adaptive_avg_pool2d bins; thread per (cell, channel quad).
// Summed as person_detect_kernel sums (column sums over y, then over x), so
// the pooled features of the KPD_PD_UNFUSED diagnostic path round exactly as
// the fused default's; its 1x1 heads (conv_mfma) still sum K in another order,
// so the two paths' scores agree to fp32 rounding, not bit for bit.
__global__ __launch_bounds__(256) void adaptive_pool56_kernel(const float* __restrict__ in, int B, int Hf, int Wf,
                                                              int C, float* __restrict__ out) {
  const int nq = C / 4;
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (size_t)B * GP * nq) return;
  const int q = idx % nq;
  const size_t cell = idx / nq;
  const int b = cell / GP, r = cell - (size_t)b * GP, i = r / G, j = r - i * G;
  const int y0 = (i * Hf) / G, y1 = ((i + 1) * Hf + G - 1) / G;
  const int x0 = (j * Wf) / G, x1 = ((j + 1) * Wf + G - 1) / G;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int x = x0; x < x1; ++x) {
    float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int y = y0; y < y1; ++y) {
      const float4 v = *reinterpret_cast<const float4*>(in + (((size_t)b * Hf + y) * Wf + x) * C + q * 4);
      cs.x += v.x; cs.y += v.y; cs.z += v.z; cs.w += v.w;
    }
    s.x += cs.x; s.y += cs.y; s.z += cs.z; s.w += cs.w;
  }
  const float cnt = (float)((y1 - y0) * (x1 - x0));
  *reinterpret_cast<float4*>(out + cell * C + q * 4) = make_float4(s.x / cnt, s.y / cnt, s.z / cnt, s.w / cnt);
}

// head output [B][56*56][hc] (channels 0..35 box deltas (anchor a, coord c at a*4+c), 36..44 logits)
// -> candidates [B][56*56*9][4] boxes, [B][..] scores (-inf when <= conf)
__global__ __launch_bounds__(256) void person_decode_kernel(const float* __restrict__ head, int B, int hc,
                                                            const float* __restrict__ anchors, float inv_w,
                                                            float inv_h, float conf, float* __restrict__ cand_boxes,
                                                            float* __restrict__ cand_scores) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (size_t)B * GP * NA) return;
  const int a = idx % NA;
  const size_t cell = idx / NA;             // b*GP + (i*56+j)
  const int anc = (int)(cell % GP) * NA + a;
  const float* h = head + cell * hc;
  const float logit = h[36 + a];
  const float score = kpd_sigmoid(logit);
  const float ax = anchors[anc * 4 + 0], ay = anchors[anc * 4 + 1];
  const float aw = anchors[anc * 4 + 2] * inv_w, ah = anchors[anc * 4 + 3] * inv_h;
  const float clip = 4.135166556742356f;   // log(1000/16)
  const float cx = ax + h[a * 4 + 0] * aw;
  const float cy = ay + h[a * 4 + 1] * ah;
  const float w = aw * expf(fminf(h[a * 4 + 2], clip));
  const float hh = ah * expf(fminf(h[a * 4 + 3], clip));
  *reinterpret_cast<float4*>(cand_boxes + idx * 4) = make_float4(cx, cy, w, hh);
  cand_scores[idx] = score > conf ? score : -INFINITY;
}

// The whole detector front end in one pass (replaces adaptive_pool56_kernel ->
// the 45-column 1x1 conv -> person_decode_kernel, whose pooled [B][3136][128]
// and head [B][3136][48] maps went through HBM).  One 512-thread workgroup per
// (image, grid row i), XCD-contiguous in i (neighbouring rows' bins share an
// input row, which then hits the same L2):
//   1. column sums of the row's input rows [y0, y1) for every x and channel
//      quad (coalesced 512-byte pixel rows, 4 rows' loads in flight per item)
//      -> LDS [Wf][128];
//   2. bins: sum of the column sums over [x0, x1), / count (adaptive-avg-pool
//      bins; the sum runs over columns of row sums instead of row-major);
//   3. box_heads[0] ++ cls_heads[0] on v_mfma_f32_16x16x4_f32 (exact fp32
//      products), waves 0-3: columns 0-31 of bin block w, 4-7: columns 32-47;
//   4. the row's 504 anchors decoded as person_decode_kernel does.
// in: FPN level 0 [B][Hf][Wf][128] fp32; w: [48][128] (rows 45..47 zero), bias
// [48].  Dynamic LDS: person_detect_lds(Wf).
constexpr int kPdPP = 128 + 4, kPdHS = 49;
inline size_t person_detect_lds(int Wf) {
  return std::max<size_t>((size_t)Wf * 128 * 4, (size_t)G * kPdHS * 4) + (size_t)G * kPdPP * 4;
}
__global__ __launch_bounds__(512) void person_detect_kernel(const float* __restrict__ in, int Hf, int Wf,
                                                            const float* __restrict__ w, const float* __restrict__ bias,
                                                            const float* __restrict__ anchors, float inv_w,
                                                            float inv_h, float conf, float* __restrict__ cand_boxes,
                                                            float* __restrict__ cand_scores) {
  constexpr int C = 128, PP = kPdPP, HC = 45, HS = kPdHS, NT = 512;
  extern __shared__ __attribute__((aligned(16))) float pd_lds[];
  float* colsum = pd_lds;                                  // [Wf][128]; later the head outputs [56][49]
  float* pool = pd_lds + std::max(Wf * C, G * HS);         // [56][132]
  const int L = xcd_remap(blockIdx.x, gridDim.x), b = L / G, i = L - b * G, tid = threadIdx.x;
  const int y0 = (i * Hf) / G, y1 = ((i + 1) * Hf + G - 1) / G;
  const float* src = in + (size_t)b * Hf * Wf * C;
  // 1. column sums, 3 items x 4 rows of loads in flight per thread
  for (int base = 0; base < Wf * 32; base += 3 * NT) {
    float4 s[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) s[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int ys = y0; ys < y1; ys += 4) {
      float4 v[3][4];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int it = base + k * NT + tid, x = it >> 5, q = it & 31;
#pragma unroll
        for (int u = 0; u < 4; ++u)
          v[k][u] = (it < Wf * 32 && ys + u < y1)
                        ? *reinterpret_cast<const float4*>(src + ((size_t)(ys + u) * Wf + x) * C + q * 4)
                        : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          s[k].x += v[k][u].x; s[k].y += v[k][u].y; s[k].z += v[k][u].z; s[k].w += v[k][u].w;
        }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int it = base + k * NT + tid;
      if (it < Wf * 32) *reinterpret_cast<float4*>(colsum + (it >> 5) * C + (it & 31) * 4) = s[k];
    }
  }
  __syncthreads();
  // 2. bins
  for (int it = tid; it < G * 32; it += NT) {
    const int j = it >> 5, q = it & 31;
    const int x0 = (j * Wf) / G, x1 = ((j + 1) * Wf + G - 1) / G;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int x = x0; x < x1; ++x) {
      const float4 v = *reinterpret_cast<const float4*>(colsum + x * C + q * 4);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    const float cnt = (float)((y1 - y0) * (x1 - x0));
    *reinterpret_cast<float4*>(pool + j * PP + q * 4) = make_float4(s.x / cnt, s.y / cnt, s.z / cnt, s.w / cnt);
  }
  __syncthreads();
  // 3. heads (the head outputs overwrite the dead column sums)
  float* head = colsum;
  {
    const int lane = tid & 63, wave = tid >> 6, g = lane >> 4, r16 = lane & 15;
    const int rb = wave & 3, nb0 = wave < 4 ? 0 : 2, nnb = wave < 4 ? 2 : 1;
    const int row = rb * 16 + r16;
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int kc = 0; kc < C / 16; ++kc) {
      // lane (g, r16) supplies A[bin r16][16 kc + 4g .. +3] and B[col r16][same k]
      const float4 a = row < G ? *reinterpret_cast<const float4*>(pool + row * PP + kc * 16 + g * 4)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        if (n >= nnb) continue;
        const float4 bw = *reinterpret_cast<const float4*>(w + (size_t)((nb0 + n) * 16 + r16) * C + kc * 16 + g * 4);
        acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, bw.x, acc[n], 0, 0, 0);
        acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, bw.y, acc[n], 0, 0, 0);
        acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, bw.z, acc[n], 0, 0, 0);
        acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, bw.w, acc[n], 0, 0, 0);
      }
    }
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int col = (nb0 + n) * 16 + r16;
      if (n >= nnb || col >= HC) continue;
      const float bb = bias[col];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int j = rb * 16 + g * 4 + e;   // D: lane holds rows 4g + e of its block, column r16
        if (j < G) head[j * HS + col] = acc[n][e] + bb;
      }
    }
  }
  __syncthreads();
  // 4. decode
  for (int it = tid; it < G * NA; it += NT) {
    const int j = it / NA, a = it - j * NA;
    const float* h = head + j * HS;
    const size_t idx = ((size_t)b * GP + i * G + j) * NA + a;
    const int anc = (i * G + j) * NA + a;
    const float score = kpd_sigmoid(h[36 + a]);
    const float ax = anchors[anc * 4 + 0], ay = anchors[anc * 4 + 1];
    const float aw = anchors[anc * 4 + 2] * inv_w, ah = anchors[anc * 4 + 3] * inv_h;
    const float clip = 4.135166556742356f;   // log(1000/16)
    const float cx = ax + h[a * 4 + 0] * aw;
    const float cy = ay + h[a * 4 + 1] * ah;
    const float bw = aw * expf(fminf(h[a * 4 + 2], clip));
    const float bh = ah * expf(fminf(h[a * 4 + 3], clip));
    *reinterpret_cast<float4*>(cand_boxes + idx * 4) = make_float4(cx, cy, bw, bh);
    cand_scores[idx] = score > conf ? score : -INFINITY;
  }
}

// x'[c] = x[c] * sigmoid(b + sum_k w[k] * sa1[k]) in place; thread per pixel.
__global__ __launch_bounds__(256) void kh_att_kernel(float* __restrict__ x, const float* __restrict__ sa1,
                                                     const float* __restrict__ w, const float* __restrict__ b,
                                                     size_t npix) {
  __shared__ float sw[64];
  if (threadIdx.x < 64) sw[threadIdx.x] = w[threadIdx.x];
  __syncthreads();
  const size_t pix = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= npix) return;
  const float4* s = reinterpret_cast<const float4*>(sa1 + pix * 64);
  float a = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const float4 v = s[q];
    a = fmaf(sw[4 * q], v.x, a); a = fmaf(sw[4 * q + 1], v.y, a);
    a = fmaf(sw[4 * q + 2], v.z, a); a = fmaf(sw[4 * q + 3], v.w, a);
  }
  const float att = kpd_sigmoid(a + b[0]);
  float4* xp = reinterpret_cast<float4*>(x + pix * 128);
#pragma unroll
  for (int q = 0; q < 32; ++q) {
    float4 v = xp[q];
    v.x *= att; v.y *= att; v.z *= att; v.w *= att;
    xp[q] = v;
  }
}

// Split-operand variant (KEYPOINT_HEAD on hmconv_kernel, MODE 2): the same
// x * att (fp32), scaled by ROI r's power of two and written as f16 hi + lo in
// [hi32 | lo32] groups at the pixel's position of the hmconv layout (kHmPitch;
// the zero borders are never written).  |x * att| <= |x| <= bound: the
// scale 2^a, a = split_exp_of(bound), keeps hi below 2^15; the first conv's
// input unscale reads the same bound from hsc[r][2].
__global__ __launch_bounds__(256) void kh_att_split_kernel(const float* __restrict__ x, const float* __restrict__ sa1,
                                                           const float* __restrict__ w, const float* __restrict__ b,
                                                           const float* __restrict__ bound, int bdiv, int bstride,
                                                           float* __restrict__ hsc, int R, _Float16* __restrict__ out) {
  __shared__ float sw[64];
  if (threadIdx.x < 64) sw[threadIdx.x] = w[threadIdx.x];
  __syncthreads();
  const size_t pix = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= (size_t)R * GP) return;
  const int r = (int)(pix / GP), rem = (int)(pix - (size_t)r * GP), yy = rem / G, xx = rem - yy * G;
  const float4* s = reinterpret_cast<const float4*>(sa1 + pix * 64);
  float a = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const float4 v = s[q];
    a = fmaf(sw[4 * q], v.x, a); a = fmaf(sw[4 * q + 1], v.y, a);
    a = fmaf(sw[4 * q + 2], v.z, a); a = fmaf(sw[4 * q + 3], v.w, a);
  }
  const float att = kpd_sigmoid(a + b[0]);
  const float bnd = bound[(size_t)(r / bdiv) * bstride];
  if (rem == 0) hsc[(size_t)r * 4 + 2] = bnd;
  const float sc = ldexpf(1.f, split_exp_of(bnd));
  const float4* xp = reinterpret_cast<const float4*>(x + pix * 128);
  _Float16* o = out + hm_pos(r, yy, xx) * 256;
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
#pragma unroll
  for (int q8 = 0; q8 < 16; ++q8) {   // 8 channels per step: one 16-byte hi and lo store each
    const float4 u0 = xp[2 * q8], u1 = xp[2 * q8 + 1];
    const float v[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
    h8 hi, lo;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float xs = (v[e] * att) * sc;
      hi[e] = (_Float16)xs;
      lo[e] = (_Float16)(xs - (float)hi[e]);
    }
    const int c = q8 * 8;
    *reinterpret_cast<h8*>(o + (c / 32) * 64 + c % 32) = hi;
    *reinterpret_cast<h8*>(o + (c / 32) * 64 + 32 + c % 32) = lo;
  }
}

// KEYPOINT_HEAD spatial attention fused (keypoint_head.py:15-20, 53-54):
// att = sigmoid(b2 + w2 . relu6(W1 x + b1)) per pixel and xa = x * att written
// as the split operand of the first KH hmconv (as kh_att_split_kernel).  A
// workgroup takes 64 pixels of one ROI (3136 = 49 x 64; persistent over
// tiles): x (fp32) stays in registers; x * 2^a as f16 hi / lo rows in LDS; the
// 1x1 128 -> 64 on v_mfma_f32_16x16x32_f16 with three products (lo.hi, hi.hi,
// hi.lo: fp32-accurate, the heatmap convs' split), wave w owning output
// channels 16w .. 16w+15 with W1's fragments in registers for the whole launch;
// the 64 -> 1 dot by 16-lane butterflies and a 4-wave LDS sum.  Replaces the
// fp32 1x1 conv (whose [R][3136][64] output went through HBM) and one pass.
constexpr int KA_ROW = 528;   // LDS bytes per pixel: hi 256 | lo 256 | 16 pad (b128 reads conflict-free)
__global__ __launch_bounds__(256) void kh_att2_kernel(const float* __restrict__ x, const _Float16* __restrict__ w1s,
                                                      int w1_exp, const float* __restrict__ b1,
                                                      const float* __restrict__ w2, const float* __restrict__ b2,
                                                      const float* __restrict__ bound, int bdiv, int bstride,
                                                      float* __restrict__ hsc, int R, _Float16* __restrict__ out) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  __shared__ __attribute__((aligned(16))) char sx[64 * KA_ROW];
  __shared__ float spart[4][64];
  __shared__ float satt[64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, r16 = lane & 15;
  const int co = wave * 16 + r16;
  h8 bh[4], bl[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const _Float16* wp = w1s + (size_t)co * 256 + c * 64 + g * 8;
    bh[c] = *reinterpret_cast<const h8*>(wp);
    bl[c] = *reinterpret_cast<const h8*>(wp + 32);
  }
  const float bias1 = b1[co], wo2 = w2[co], bias2 = b2[0];
  const int ntiles = R * 49, c4 = (tid & 31) * 4;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int r = tile / 49, p0 = (tile - r * 49) * 64;
    const float bnd = bound[(size_t)(r / bdiv) * bstride];
    const int a = split_exp_of(bnd);
    const float sc = ldexpf(1.f, a), us = ldexpf(1.f, -(a + w1_exp));
    if (tid == 0 && p0 == 0) hsc[(size_t)r * 4 + 2] = bnd;
    const float4* xp = reinterpret_cast<const float4*>(x + ((size_t)r * GP + p0) * 128);
    float4 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = xp[tid + 256 * i];   // pixel (tid >> 5) + 8 i, channels c4 .. c4 + 3
    __syncthreads();   // the previous tile's LDS reads are done
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float e4[4] = {v[i].x * sc, v[i].y * sc, v[i].z * sc, v[i].w * sc};
      f16x4 hi, lo;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        hi[e] = (_Float16)e4[e];
        lo[e] = (_Float16)(e4[e] - (float)hi[e]);
      }
      char* rowp = sx + ((tid >> 5) + 8 * i) * KA_ROW + c4 * 2;
      *reinterpret_cast<f16x4*>(rowp) = hi;
      *reinterpret_cast<f16x4*>(rowp + 256) = lo;
    }
    __syncthreads();
    f32x4 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const char* rowp = sx + (i * 16 + r16) * KA_ROW + c * 64 + g * 16;
        const h8 ah = *reinterpret_cast<const h8*>(rowp), al = *reinterpret_cast<const h8*>(rowp + 256);
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[c], acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[c], acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[c], acc[i], 0, 0, 0);
      }
    // lane (g, r16) holds pixels 16 i + 4 g + e of output channel co
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float pv = wo2 * fminf(fmaxf(fmaf(acc[i][e], us, bias1), 0.f), 6.f);
        pv = row16_sum(pv);   // the 16 output channels of the wave (DPP butterfly)
        if (r16 == 0) spart[wave][i * 16 + g * 4 + e] = pv;
      }
    __syncthreads();
    if (tid < 64) satt[tid] = kpd_sigmoid(bias2 + ((spart[0][tid] + spart[1][tid]) + (spart[2][tid] + spart[3][tid])));
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int px = (tid >> 5) + 8 * i, pix = p0 + px, yy = pix / G, xx = pix - yy * G;
      const float att = satt[px];
      const float e4[4] = {(v[i].x * att) * sc, (v[i].y * att) * sc, (v[i].z * att) * sc, (v[i].w * att) * sc};
      f16x4 hi, lo;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        hi[e] = (_Float16)e4[e];
        lo[e] = (_Float16)(e4[e] - (float)hi[e]);
      }
      _Float16* o = out + hm_pos(r, yy, xx) * 256 + (c4 / 32) * 64 + c4 % 32;
      *reinterpret_cast<f16x4*>(o) = hi;
      *reinterpret_cast<f16x4*>(o + 32) = lo;
    }
  }
}

// adaptive avg pool of an NHWC [R][56][56][C] map to (o x o), written in
// NCHW-flatten order (c*o*o + y*o + x) as nn.Flatten after the pool does.
// grid R, 256 threads.  Pass 1: item = (cell, source row, channel quad) sums
// its row's columns with 16-byte loads (4 lanes read a pixel's 64 bytes)
// into an LDS partial; pass 2: each output sums its cell's row partials in
// row order.  LDS: o*o cells x rows-per-cell x C floats (host-sized).
__global__ __launch_bounds__(256) void kh_pool_kernel(const float* __restrict__ in, int C, int o,
                                                      float* __restrict__ out, int out_stride) {
  extern __shared__ float part[];   // [cell][row in cell][C]
  const int r = blockIdx.x, nq = C / 4, rpc = (G + o - 1) / o + 1;   // rows per cell (upper bound)
  const float* src = in + (size_t)r * GP * C;
  const int items = o * o * rpc * nq;
  // IU items per thread at a time, XB columns of each: IU * XB loads in
  // flight per batch (one memory round trip), each item still summed in x
  // order
  constexpr int IU = 4, XB = 2;
  for (int t0 = threadIdx.x; t0 < items; t0 += IU * blockDim.x) {
    const float* rowp[IU];
    int len[IU], dst[IU], lmax = 0;
#pragma unroll
    for (int k = 0; k < IU; ++k) {
      const int t = t0 + k * blockDim.x;
      const int tt = min(t, items - 1);
      const int q = tt % nq, rest = tt / nq, dy = rest % rpc, cell = rest / rpc, i = cell / o, j = cell - i * o;
      const int y0 = (i * G) / o, y1 = ((i + 1) * G + o - 1) / o;
      const int x0 = (j * G) / o, x1 = ((j + 1) * G + o - 1) / o;
      const int y = y0 + dy;
      len[k] = t < items && y < y1 ? x1 - x0 : 0;
      rowp[k] = src + ((size_t)min(y, G - 1) * G + x0) * C + q * 4;
      dst[k] = t < items ? (cell * rpc + dy) * C + q * 4 : -1;
      lmax = max(lmax, len[k]);
    }
    float4 s[IU];
#pragma unroll
    for (int k = 0; k < IU; ++k) s[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int xb = 0; xb < lmax; xb += XB) {
      float4 v[IU][XB];
#pragma unroll
      for (int k = 0; k < IU; ++k)
#pragma unroll
        for (int u = 0; u < XB; ++u)
          if (xb + u < len[k]) v[k][u] = *reinterpret_cast<const float4*>(rowp[k] + (size_t)(xb + u) * C);
#pragma unroll
      for (int k = 0; k < IU; ++k)
#pragma unroll
        for (int u = 0; u < XB; ++u)
          if (xb + u < len[k]) { s[k].x += v[k][u].x; s[k].y += v[k][u].y; s[k].z += v[k][u].z; s[k].w += v[k][u].w; }
    }
#pragma unroll
    for (int k = 0; k < IU; ++k)
      if (dst[k] >= 0) *reinterpret_cast<float4*>(part + dst[k]) = s[k];
  }
  __syncthreads();
  const int n = C * o * o;
  for (int t = threadIdx.x; t < n; t += blockDim.x) {
    const int c = t / (o * o), cell = t - c * o * o, i = cell / o, j = cell - i * o;
    const int y0 = (i * G) / o, y1 = ((i + 1) * G + o - 1) / o;
    const int x0 = (j * G) / o, x1 = ((j + 1) * G + o - 1) / o;
    float s = 0.f;
    for (int dy = 0; dy < y1 - y0; ++dy) s += part[((size_t)cell * rpc + dy) * C + c];
    out[(size_t)r * out_stride + t] = s / (float)((y1 - y0) * (x1 - x0));
  }
}

// LayerNorm(n) (eps 1e-5, biased variance) + ReLU6 + Linear(n -> m) + sigmoid for one ROI.
__device__ void ln_linear_sigmoid(const float* __restrict__ y, int n, const float* __restrict__ g,
                                  const float* __restrict__ bb, const float* __restrict__ w,
                                  const float* __restrict__ b, int m, float* __restrict__ dst, float* sh) {
  const int tid = threadIdx.x;
  __shared__ float red[2][4];
  float s = 0.f;
  for (int i = tid; i < n; i += 256) s += y[i];
  s = wave_sum(s);
  if ((tid & 63) == 0) red[0][tid >> 6] = s;
  __syncthreads();
  const float mean = (red[0][0] + red[0][1] + red[0][2] + red[0][3]) / (float)n;
  float v = 0.f;
  for (int i = tid; i < n; i += 256) { const float d = y[i] - mean; v += d * d; }
  v = wave_sum(v);
  if ((tid & 63) == 0) red[1][tid >> 6] = v;
  __syncthreads();
  const float var = (red[1][0] + red[1][1] + red[1][2] + red[1][3]) / (float)n;
  const float inv = 1.f / sqrtf(var + 1e-5f);
  for (int i = tid; i < n; i += 256) sh[i] = fminf(fmaxf((y[i] - mean) * inv * g[i] + bb[i], 0.f), 6.f);
  __syncthreads();
  for (int k = tid; k < m; k += 256) {
    float a = b[k];
    for (int i = 0; i < n; ++i) a = fmaf(w[k * n + i], sh[i], a);
    dst[k] = kpd_sigmoid(a);
  }
  __syncthreads();
}

// grid R.  lin_r [R][256] (regression Linear out), lin_v [R][128] (visibility).
__global__ __launch_bounds__(256) void kh_final_kernel(const float* __restrict__ lin_r, int r_stride,
                                                       const float* __restrict__ lin_v, int v_stride,
                                                       const float* ln_rg, const float* ln_rb, const float* w_r,
                                                       const float* b_r, const float* ln_vg, const float* ln_vb,
                                                       const float* w_v, const float* b_v,
                                                       const int32_t* __restrict__ slot, int P,
                                                       float* __restrict__ kh_kpts, float* __restrict__ kh_vis) {
  __shared__ float sh[256];
  const int r = blockIdx.x;
  const int sl = slot[r];
  if (sl < 0) {   // padding slot: zeros
    const size_t o = (size_t)((r / P) * P + slot_pos(sl)) * 17;
    for (int i = threadIdx.x; i < 17 * 5; i += blockDim.x) {
      if (i < 34) kh_kpts[o * 2 + i] = 0.f;
      else kh_vis[o * 3 + (i - 34)] = 0.f;
    }
    return;
  }
  const size_t o = (size_t)((r / P) * P + sl) * 17;
  ln_linear_sigmoid(lin_r + (size_t)r * r_stride, 256, ln_rg, ln_rb, w_r, b_r, 34, kh_kpts + o * 2, sh);
  ln_linear_sigmoid(lin_v + (size_t)r * v_stride, 128, ln_vg, ln_vb, w_v, b_v, 51, kh_vis + o * 3, sh);
}

}  // namespace

hipError_t launch_adaptive_pool56(const float* in, int B, int Hf, int Wf, int C, float* out, hipStream_t st) {
  if (C % 4) return hipErrorInvalidValue;
  const size_t total = (size_t)B * GP * (C / 4);
  hipLaunchKernelGGL(adaptive_pool56_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, in, B, Hf, Wf,
                     C, out);
  return hipGetLastError();
}

bool person_detect_fits(int Wf) { return Wf >= 1 && person_detect_lds(Wf) <= 160 * 1024; }

hipError_t launch_person_detect(const float* feat, int B, int Hf, int Wf, const float* w, const float* bias,
                                const float* anchors, int img_h, int img_w, float conf, float* cand_boxes,
                                float* cand_scores, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  if (Hf < 1 || Wf < 1 || !w || !bias || !anchors) return hipErrorInvalidValue;
  const size_t lds = person_detect_lds(Wf);
  if (lds > 160 * 1024) return hipErrorInvalidValue;   // (the caller takes the unfused path)
  hipLaunchKernelGGL(person_detect_kernel, dim3((unsigned)(B * G)), dim3(512), lds, st, feat, Hf, Wf, w, bias,
                     anchors, 1.f / (float)img_w, 1.f / (float)img_h, conf, cand_boxes, cand_scores);
  return hipGetLastError();
}

hipError_t launch_person_decode(const float* head, int B, int hc, const float* anchors, int img_h, int img_w,
                                float conf, float* cand_boxes, float* cand_scores, hipStream_t st) {
  const size_t total = (size_t)B * GP * NA;
  hipLaunchKernelGGL(person_decode_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, head, B, hc,
                     anchors, 1.f / (float)img_w, 1.f / (float)img_h, conf, cand_boxes, cand_scores);
  return hipGetLastError();
}

hipError_t launch_kh_att(float* x, const float* sa1, const float* w, const float* b, size_t npix, hipStream_t st) {
  hipLaunchKernelGGL(kh_att_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, st, x, sa1, w, b, npix);
  return hipGetLastError();
}

hipError_t launch_kh_att_split(const float* x, const float* sa1, const float* w, const float* b, int R,
                               const float* bound, int bdiv, int bstride, float* hsc, void* out, hipStream_t st) {
  if (R <= 0) return hipSuccess;
  if (!bound || bdiv < 1 || bstride < 1 || !hsc || !out) return hipErrorInvalidValue;
  const size_t n = (size_t)R * GP;
  hipLaunchKernelGGL(kh_att_split_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, sa1, w, b, bound,
                     bdiv, bstride, hsc, R, static_cast<_Float16*>(out));
  return hipGetLastError();
}

hipError_t launch_kh_att2(const float* x, const void* w1s, int w1_exp, const float* b1, const float* w2,
                          const float* b2, int R, const float* bound, int bdiv, int bstride, float* hsc, void* out,
                          hipStream_t st) {
  if (R <= 0) return hipSuccess;
  if (!w1s || !bound || bdiv < 1 || bstride < 1 || !hsc || !out) return hipErrorInvalidValue;
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
  }
  const long tiles = (long)R * 49;
  const unsigned grid = (unsigned)std::min<long>(tiles, 4L * ncu);
  hipLaunchKernelGGL(kh_att2_kernel, dim3(grid), dim3(256), 0, st, x, static_cast<const _Float16*>(w1s), w1_exp, b1,
                     w2, b2, bound, bdiv, bstride, hsc, R, static_cast<_Float16*>(out));
  return hipGetLastError();
}

hipError_t launch_kh_pool(const float* in, int R, int C, int o, float* out, int out_stride, hipStream_t st) {
  if (C % 4 || o < 1 || o > G) return hipErrorInvalidValue;
  const size_t lds = (size_t)o * o * ((G + o - 1) / o + 1) * C * sizeof(float);
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kh_pool_kernel, dim3(R), dim3(256), lds, st, in, C, o, out, out_stride);
  return hipGetLastError();
}

hipError_t launch_kh_final(const float* lin_r, int r_stride, const float* lin_v, int v_stride, const float* ln_rg,
                           const float* ln_rb, const float* w_r, const float* b_r, const float* ln_vg,
                           const float* ln_vb, const float* w_v, const float* b_v, const int32_t* slot, int R, int P,
                           float* kh_kpts, float* kh_vis, hipStream_t st) {
  hipLaunchKernelGGL(kh_final_kernel, dim3(R), dim3(256), 0, st, lin_r, r_stride, lin_v, v_stride, ln_rg, ln_rb, w_r,
                     b_r, ln_vg, ln_vb, w_v, b_v, slot, P, kh_kpts, kh_vis);
  return hipGetLastError();
}
