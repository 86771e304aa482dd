// features.2 + features.3 of mobilenet_v3_small in one launch (backbone.py:250-254
// via torchvision's InvertedResidual): the two SE-less blocks between the
// 64 x 48 and the 32 x 24 maps (at 256 x 192), stride-2 then stride-1, both
// expand 1x1 + ReLU -> depthwise 3x3 + ReLU -> project 1x1 (+ residual).
//
// A workgroup takes T output rows of features.3 for one image.  It recomputes
// the features.2 rows those need (the 3x3 halo: T + 2 rows, clipped to the
// map) from the features.1 rows those need (2 (T + 2) + 1 rows), so neither
// the 72-channel expanded tensors nor the features.2 output reach HBM: one
// read of the features.1 rows and one write of features.3 (tap 1 of the FPN)
// per tile.  It replaces fir_kernel (features.2: five channel slices, each an
// LDS-bound VALU expand / project) plus exdw_kernel + pw_small_kernel
// (features.3).
//
// All four 1x1 convs run on v_mfma_f32_16x16x4_f32 (exact fp32 products) as
// transposed GEMMs: M = 16 output channels, N = 16 pixels, so a lane's
// accumulator is 4 consecutive channels of one pixel (one 16-byte LDS store)
// and a lane's B operand is 4 consecutive channels of one pixel (one 16-byte
// LDS or global read).  The K order inside a K-step is permuted identically
// for A and B (lane group g supplies channels 4g .. 4g + 3, one per step).
// The depthwise 3x3 convs run on VALU (4 channels x one pixel per item).
//
// LDS rows are 16 (or 32) floats per pixel, 16-byte chunks XOR-swizzled by
// the pixel (chunk ^ (px >> 2) & 3, or ^ (px >> 1) & 7 for 32-float rows):
// 16 lanes reading one chunk of 16 consecutive pixels hit 16 different bank
// quads.  Sums run in a fixed order (MFMA K order, taps ky-major), so an
// image's result does not depend on the batch or the tile grid's position.
#include "kpd_common.h"
#include "kpd_kernels.h"

namespace {

// 16 waves: 4 per SIMD, so one workgroup's MFMA chains, LDS round trips and
// depthwise items interleave; every thread owns at most one depthwise item of
// each block (the tile bounds below keep NPX2, NPX3 <= 256 pixels)
constexpr int F23_NW = 16, F23_NT = 64 * F23_NW;
constexpr int F23_MAXT1 = 4;   // features.1 pixel tiles per wave (held in registers)
constexpr int F23_MAXT2 = 1;   // features.2 output pixel tiles per wave (f3 expand operands in registers)
constexpr int F23_MAXP = 2;    // project (channel tile, pixel tile) pairs per wave

// chunk swizzles for ds_read_b128 / ds_write_b128, whose 16-lane bank groups
// are lanes {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} and the same + 32
// (MI355X_MICROARCH.md, LDS): conflict-free for the MFMA operand pattern (lane
// = (chunk group lg, pixel lr), 16-aligned pixel base) and, for 16-float rows,
// for 64 lanes reading one chunk of 64 consecutive pixels at any base --
// verified exhaustively for the permutation tables {0,2,3,1} of (px >> 2) & 3
// and {0,1,4,5,6,7,2,3} of (px >> 1) & 7 (a plain XOR with those bits leaves
// 2-way conflicts: SQ_LDS_BANK_CONFLICT was 32 % of the LDS cycles)
__device__ __forceinline__ int a16(int px, int c) { return px * 16 + 4 * (c ^ ((0x78 >> (2 * ((px >> 2) & 3))) & 3)); }
__device__ __forceinline__ int a32(int px, int c) { return px * 32 + 4 * (c ^ ((0x6beb08 >> (3 * ((px >> 1) & 7))) & 7)); }

// diagnostic phase stamps (KPD_STAMPS, diagnostic build): 0 start, 1 operands
// staged, 2 / 3 first features.2 expand / depthwise done, 4 features.2 done,
// 5 Y2 stored, 6 features.3 done, 7 end
__device__ __forceinline__ void f23_stamp(unsigned long long* st, int i) {
  if (st && threadIdx.x == 0) st[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 + i] = __builtin_amdgcn_s_memrealtime();
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
// RELU: every activation of both blocks is ReLU (mobilenet_v3_small's
// features.2 / .3), a compile-time max instead of kpd_act's runtime switch
template <bool RELU>
__device__ __forceinline__ float4 act4(float4 v, int act) {
  if constexpr (RELU)
    return make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
  return make_float4(kpd_act(v.x, act), kpd_act(v.y, act), kpd_act(v.z, act), kpd_act(v.w, act));
}

// region sizes in floats for the largest (interior) tile of T rows
struct F23Lds {
  int bd2, be2, ra, wd3, bd3, be3, rb, total;
};
__host__ __device__ inline F23Lds f23_lds(const Fir23Args& a) {
  const int ny2 = min(a.T + 2, a.H2), ny1 = min(2 * ny2 + 1, a.H1);
  const int npx1 = ny1 * a.W1, npx2 = ny2 * a.W2, npx3 = min(a.T, a.H2) * a.W2;
  F23Lds L;
  L.bd2 = 9 * a.E2;                  // wd2 [9][E2] at 0, then bd2 [E2], be2 [E2]
  L.be2 = 10 * a.E2;
  L.ra = (11 * a.E2 + 3) / 4 * 4;
  // region A: two features.2 expanded slices (each followed by a zero chunk,
  // what out-of-map depthwise taps read); later two features.3 expanded
  // slices, two features.3 depthwise slices and wd3 / bd3 / be3
  L.wd3 = L.ra + 2 * (npx2 * 16 + 4) + 2 * npx3 * 16;
  L.bd3 = L.wd3 + 9 * a.E3;
  L.be3 = L.bd3 + a.E3;
  L.rb = L.ra + max(2 * (npx1 * 16 + 4), (L.be3 + a.E3 - L.ra + 3) / 4 * 4);
  // region B: two features.2 depthwise slices, later the features.2 output (32 floats per pixel)
  L.total = L.rb + npx2 * 32;
  return L;
}

// One thread's depthwise item (pixel p of the output rows, channel quad q),
// fixed for every channel slice: the LDS float offset of each tap's source
// chunk inside an expanded-slice buffer (16-bit pairs), taps outside the map
// pointing at the buffer's zero chunk -- no masks, no per-slice address math
struct DwItem {
  unsigned off[5];
  int q, p;
};

// fill an item: tap t reads source pixel base + (t / 3) * W + t % 3 when
// (mask >> t) & 1, else the zero chunk at float offset zoff
__device__ __forceinline__ void dw_setup(DwItem& d, int base, int W, int mask, int zoff) {
#pragma unroll
  for (int i = 0; i < 5; ++i) d.off[i] = 0;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const unsigned o = ((mask >> t) & 1) ? (unsigned)a16(base + (t / 3) * W + t % 3, d.q) : (unsigned)zoff;
    d.off[t >> 1] |= o << (16 * (t & 1));
  }
}

// 3x3 depthwise of one item: taps ky-major, bias, activation -> 4 channels.
// wq = the slice's depthwise weights at channel quad q (tap t at wq + t * E).
template <bool RELU>
__device__ __forceinline__ float4 dw_item(const float* src, const float* wq, int E, float4 b, const DwItem& d,
                                          int act) {
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    float4 e[3], w[3];
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int t = ky * 3 + kx;
      e[kx] = ld4(src + ((d.off[t >> 1] >> (16 * (t & 1))) & 0xffff));
      w[kx] = ld4(wq + t * E);
    }
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      s.x = fmaf(e[kx].x, w[kx].x, s.x); s.y = fmaf(e[kx].y, w[kx].y, s.y);
      s.z = fmaf(e[kx].z, w[kx].z, s.z); s.w = fmaf(e[kx].w, w[kx].w, s.w);
    }
    __builtin_amdgcn_sched_barrier(0);   // row by row: all 18 loads hoisted spill registers
  }
  return act4<RELU>(make_float4(s.x + b.x, s.y + b.y, s.z + b.z, s.w + b.w), act);
}

// project: acc += W (16 channels of tile ct, 4 K-steps) . B (the pair's
// pixel tile of a 16-channel depthwise slice)
__device__ __forceinline__ void project_slice(f32x4 (&acc)[F23_MAXP], const float4& w, const float* D, int npx,
                                              int wave, int lr, int lg) {
  float4 b[F23_MAXP];
#pragma unroll
  for (int i = 0; i < F23_MAXP; ++i) {
    const int px = ((wave >> 1) + (F23_NW / 2) * i) * 16 + lr;
    b[i] = px < npx ? ld4(D + a16(px, lg)) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int i = 0; i < F23_MAXP; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, b[i].x, acc[i], 0, 0, 0);
#pragma unroll
  for (int i = 0; i < F23_MAXP; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, b[i].y, acc[i], 0, 0, 0);
#pragma unroll
  for (int i = 0; i < F23_MAXP; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, b[i].z, acc[i], 0, 0, 0);
#pragma unroll
  for (int i = 0; i < F23_MAXP; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, b[i].w, acc[i], 0, 0, 0);
}

// Software pipeline, one barrier per 16-channel slice s of each block:
//   project(s - 1) [MFMA, depthwise slice (s - 1) & 1]
//   expand(s + 1)  [MFMA -> expanded slice (s + 1) & 1]
//   depthwise(s)   [VALU, expanded slice s & 1 -> depthwise slice s & 1]
// so the matrix pipe works while the depthwise items wait on LDS.
template <bool RELU>
__global__ __launch_bounds__(F23_NT) void fir23_kernel(const Fir23Args a) {
  extern __shared__ float4 f23_sm4[];
  float* sm = reinterpret_cast<float*>(f23_sm4);
  const F23Lds L = f23_lds(a);
  f23_stamp(a.stamps, 0);
  const int n = blockIdx.y, r0 = blockIdx.x * a.T, tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  const int H1 = a.H1, W1 = a.W1, H2 = a.H2, W2 = a.W2, E2 = a.E2, E3 = a.E3;
  const int T3 = min(a.T, H2 - r0);
  const int y2a = max(r0 - 1, 0), y2b = min(r0 + T3 + 1, H2);
  const int e1a = max(2 * y2a - 1, 0), e1b = min(2 * y2b, H1);
  const int NPX1 = (e1b - e1a) * W1, NPX2 = (y2b - y2a) * W2, NPX3 = T3 * W2;
  const int S2 = E2 / 16, S3 = E3 / 16;
  float* RA = sm + L.ra;
  float* RB = sm + L.rb;
  const int ct = wave & 1;   // the channel tile of this wave's project pairs

  // this wave's features.1 pixel tiles: the B operand of every features.2
  // expand slice (issued first: they land while the weights are staged)
  const float* x1 = a.x + ((size_t)n * H1 + e1a) * W1 * 16;
  float4 af[F23_MAXT1];
#pragma unroll
  for (int i = 0; i < F23_MAXT1; ++i) {
    const int px = (wave + F23_NW * i) * 16 + lr;
    af[i] = px < NPX1 ? ld4(x1 + (size_t)px * 16 + 4 * lg) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // expand A = We2[c0 + lr][4 lg ..] (slices 0 and 1; the bias from LDS),
  // project A = Wp2[16 ct + lr][c0 + 4 lg ..]
  const float4 we_c = ld4(a.we2 + (size_t)lr * 16 + 4 * lg);
  float4 we_n = S2 > 1 ? ld4(a.we2 + (size_t)(16 + lr) * 16 + 4 * lg) : we_c;
  float4 wp_n = ld4(a.wp2 + (size_t)(16 * ct + lr) * E2 + 4 * lg);
  for (int i = tid; i < 9 * E2; i += F23_NT) sm[i] = a.wd2[i];
  for (int i = tid; i < E2; i += F23_NT) {
    sm[L.bd2 + i] = a.bd2[i];
    sm[L.be2 + i] = a.be2[i];
  }
  if (tid < 2) st4(RA + tid * (NPX1 * 16 + 4) + NPX1 * 16, make_float4(0.f, 0.f, 0.f, 0.f));

  // depthwise items (pixel-fastest over the threads: a wave's 16-lane groups
  // read 16 neighbouring pixels of one chunk)
  DwItem d2{};
  const int ES2 = NPX1 * 16 + 4;   // expanded-slice buffer stride (zero chunk at NPX1 * 16)
  const bool has2 = tid < NPX2 * 4;
  if (has2) {
    d2.q = tid / NPX2;
    d2.p = tid - d2.q * NPX2;
    const int yy = y2a + d2.p / W2, xx = d2.p % W2;
    int mask = 0;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int iy = 2 * yy - 1 + t / 3, ix = 2 * xx - 1 + t % 3;
      mask |= (iy >= e1a && iy < e1b && ix >= 0 && ix < W1) ? 1 << t : 0;
    }
    dw_setup(d2, (2 * yy - 1 - e1a) * W1 + 2 * xx - 1, W1, mask, NPX1 * 16);
  }

  // expand of one features.2 slice: the wave's tiles as independent
  // accumulator chains, step-major (tiles past the map multiply zeros and are
  // not stored)
  auto expand2 = [&](const float4& we, f32x4 (&e)[F23_MAXT1]) {
#pragma unroll
    for (int i = 0; i < F23_MAXT1; ++i) e[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < F23_MAXT1; ++i) e[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(we.x, af[i].x, e[i], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < F23_MAXT1; ++i) e[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(we.y, af[i].y, e[i], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < F23_MAXT1; ++i) e[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(we.z, af[i].z, e[i], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < F23_MAXT1; ++i) e[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(we.w, af[i].w, e[i], 0, 0, 0);
  };
  auto store_e2 = [&](const f32x4 (&e)[F23_MAXT1], int c0, float* E) {
    const float4 be = ld4(sm + L.be2 + c0 + 4 * lg);
#pragma unroll
    for (int i = 0; i < F23_MAXT1; ++i) {
      const int px = (wave + F23_NW * i) * 16 + lr;
      if (px < NPX1)
        st4(E + a16(px, lg), act4<RELU>(make_float4(e[i][0] + be.x, e[i][1] + be.y, e[i][2] + be.z, e[i][3] + be.w),
                                  a.act2e));
    }
  };

  // ---------------- features.2 ----------------
  f32x4 acc[F23_MAXP];
#pragma unroll
  for (int i = 0; i < F23_MAXP; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  {
    f32x4 e[F23_MAXT1];
    expand2(we_c, e);
    __syncthreads();   // the depthwise weights and the expand bias staged
    store_e2(e, 0, RA);
  }
  __syncthreads();   // expanded slice 0 staged
  f23_stamp(a.stamps, 1);
  float4 wp_c = wp_n;
  for (int sl = 0; sl < S2; ++sl) {
    // operands of the next step: project(sl) and expand(sl + 2)
    const float4 wp_p = wp_c, we_x = we_n;
    wp_c = wp_n;
    if (sl + 1 < S2) wp_n = ld4(a.wp2 + (size_t)(16 * ct + lr) * E2 + (sl + 1) * 16 + 4 * lg);
    if (sl + 2 < S2) we_n = ld4(a.we2 + (size_t)((sl + 2) * 16 + lr) * 16 + 4 * lg);
    // (the matrix work first: while this wave waits for its MFMA results, the
    // SIMD's other waves run their depthwise items)
    if (sl + 1 < S2) {
      f32x4 e[F23_MAXT1];
      expand2(we_x, e);
      if (sl > 0) project_slice(acc, wp_p, RB + ((sl - 1) & 1) * NPX2 * 16, NPX2, wave, lr, lg);
      store_e2(e, (sl + 1) * 16, RA + ((sl + 1) & 1) * ES2);
    } else if (sl > 0) {
      project_slice(acc, wp_p, RB + ((sl - 1) & 1) * NPX2 * 16, NPX2, wave, lr, lg);
    }
    if (has2)
      st4(RB + (sl & 1) * NPX2 * 16 + a16(d2.p, d2.q),
          dw_item<RELU>(RA + (sl & 1) * ES2, sm + sl * 16 + 4 * d2.q, E2, ld4(sm + L.bd2 + sl * 16 + 4 * d2.q), d2,
                        a.act2d));
    if (sl == 0) f23_stamp(a.stamps, 2);
    __syncthreads();
  }
  // features.3 depthwise weights / bias (to LDS below) and items
  float w3r[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = tid + u * F23_NT;
    w3r[u] = i < 9 * E3 ? a.wd3[i] : i < 10 * E3 ? a.bd3[i - 9 * E3] : i < 11 * E3 ? a.be3[i - 10 * E3] : 0.f;
  }
  project_slice(acc, wp_c, RB + ((S2 - 1) & 1) * NPX2 * 16, NPX2, wave, lr, lg);
  DwItem d3{};
  const bool has3 = tid < NPX3 * 4;
  if (has3) {
    d3.q = tid / NPX3;
    d3.p = tid - d3.q * NPX3;
    const int yy = r0 + d3.p / W2, xx = d3.p % W2;
    int mask = 0;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int iy = yy - 1 + t / 3, ix = xx - 1 + t % 3;
      mask |= (iy >= y2a && iy < y2b && ix >= 0 && ix < W2) ? 1 << t : 0;
    }
    dw_setup(d3, (yy - 1 - y2a) * W2 + xx - 1, W2, mask, NPX2 * 16);
  }
  f23_stamp(a.stamps, 4);
  // features.3 operands of slices 0 / 1 (issued before the barrier)
  float4 we3_c0 = ld4(a.we3 + (size_t)lr * 32 + 8 * lg), we3_c1 = ld4(a.we3 + (size_t)lr * 32 + 8 * lg + 4);
  float4 we3_n0 = we3_c0, we3_n1 = we3_c1;
  if (S3 > 1) {
    we3_n0 = ld4(a.we3 + (size_t)(16 + lr) * 32 + 8 * lg);
    we3_n1 = ld4(a.we3 + (size_t)(16 + lr) * 32 + 8 * lg + 4);
  }
  float4 wp3_n = ld4(a.wp3 + (size_t)(16 * ct + lr) * E3 + 4 * lg);
  const float4 bp2 = ld4(a.bp2 + 16 * ct + 4 * lg), bp3 = ld4(a.bp3 + 16 * ct + 4 * lg);
  // region A is free (the last depthwise read it before the loop's last barrier): wd3 / bd3
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = tid + u * F23_NT;
    if (i < 11 * E3) sm[L.wd3 + i] = w3r[u];
  }
  __syncthreads();   // every wave's last project read of region B done: it becomes Y2
  // features.2 output Y2 [px][32] = acc + bp2 (no activation)
#pragma unroll
  for (int i = 0; i < F23_MAXP; ++i) {
    const int px = ((wave >> 1) + (F23_NW / 2) * i) * 16 + lr;
    if (px < NPX2)
      st4(RB + a32(px, 4 * ct + lg), make_float4(acc[i][0] + bp2.x, acc[i][1] + bp2.y, acc[i][2] + bp2.z,
                                                 acc[i][3] + bp2.w));
  }
  __syncthreads();
  f23_stamp(a.stamps, 5);

  // ---------------- features.3 ----------------
  // this wave's Y2 pixel tile: the B operand of every features.3 expand slice
  // (K = 32: lane group g supplies channels 8 g .. 8 g + 7 over 8 steps)
  float4 yf[F23_MAXT2][2];
#pragma unroll
  for (int i = 0; i < F23_MAXT2; ++i) {
    const int px = (wave + F23_NW * i) * 16 + lr;
    yf[i][0] = px < NPX2 ? ld4(RB + a32(px, 2 * lg)) : make_float4(0.f, 0.f, 0.f, 0.f);
    yf[i][1] = px < NPX2 ? ld4(RB + a32(px, 2 * lg + 1)) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  auto expand3 = [&](const float4& w0, const float4& w1, f32x4 (&e)[F23_MAXT2]) {
#pragma unroll
    for (int i = 0; i < F23_MAXT2; ++i) e[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float4 w = h ? w1 : w0;
#pragma unroll
      for (int i = 0; i < F23_MAXT2; ++i) e[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, yf[i][h].x, e[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < F23_MAXT2; ++i) e[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, yf[i][h].y, e[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < F23_MAXT2; ++i) e[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, yf[i][h].z, e[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < F23_MAXT2; ++i) e[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, yf[i][h].w, e[i], 0, 0, 0);
    }
  };
  auto store_e3 = [&](const f32x4 (&e)[F23_MAXT2], int c0, float* E) {
    const float4 be = ld4(sm + L.be3 + c0 + 4 * lg);
#pragma unroll
    for (int i = 0; i < F23_MAXT2; ++i) {
      const int px = (wave + F23_NW * i) * 16 + lr;
      if (px < NPX2)
        st4(E + a16(px, lg), act4<RELU>(make_float4(e[i][0] + be.x, e[i][1] + be.y, e[i][2] + be.z, e[i][3] + be.w),
                                  a.act3e));
    }
  };
  const int ES3 = NPX2 * 16 + 4;         // expanded-slice buffer stride (zero chunk at NPX2 * 16)
  float* E3b = RA;                       // two expanded slices [NPX2][16] + zero chunk
  float* D3b = RA + 2 * ES3;             // two depthwise slices [NPX3][16]
#pragma unroll
  for (int i = 0; i < F23_MAXP; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  {
    f32x4 e[F23_MAXT2];
    expand3(we3_c0, we3_c1, e);
    store_e3(e, 0, E3b);
    if (tid < 2) st4(E3b + tid * ES3 + NPX2 * 16, make_float4(0.f, 0.f, 0.f, 0.f));
  }
  __syncthreads();
  float4 wp3_c = wp3_n;
  for (int sl = 0; sl < S3; ++sl) {
    const float4 wp_p = wp3_c, w0x = we3_n0, w1x = we3_n1;
    wp3_c = wp3_n;
    if (sl + 1 < S3) wp3_n = ld4(a.wp3 + (size_t)(16 * ct + lr) * E3 + (sl + 1) * 16 + 4 * lg);
    if (sl + 2 < S3) {
      we3_n0 = ld4(a.we3 + (size_t)((sl + 2) * 16 + lr) * 32 + 8 * lg);
      we3_n1 = ld4(a.we3 + (size_t)((sl + 2) * 16 + lr) * 32 + 8 * lg + 4);
    }
    if (sl + 1 < S3) {
      f32x4 e[F23_MAXT2];
      expand3(w0x, w1x, e);
      if (sl > 0) project_slice(acc, wp_p, D3b + ((sl - 1) & 1) * NPX3 * 16, NPX3, wave, lr, lg);
      store_e3(e, (sl + 1) * 16, E3b + ((sl + 1) & 1) * ES3);
    } else if (sl > 0) {
      project_slice(acc, wp_p, D3b + ((sl - 1) & 1) * NPX3 * 16, NPX3, wave, lr, lg);
    }
    if (has3)
      st4(D3b + (sl & 1) * NPX3 * 16 + a16(d3.p, d3.q),
          dw_item<RELU>(E3b + (sl & 1) * ES3, sm + L.wd3 + sl * 16 + 4 * d3.q, E3,
                        ld4(sm + L.bd3 + sl * 16 + 4 * d3.q), d3, a.act3d));
    __syncthreads();
  }
  project_slice(acc, wp3_c, D3b + ((S3 - 1) & 1) * NPX3 * 16, NPX3, wave, lr, lg);
  f23_stamp(a.stamps, 6);
  // features.3 output = acc + bp3 + Y2 (residual; Y2 is still in region B)
#pragma unroll
  for (int i = 0; i < F23_MAXP; ++i) {
    const int px = ((wave >> 1) + (F23_NW / 2) * i) * 16 + lr;
    if (px >= NPX3) continue;
    const int yy = r0 + px / W2, xx = px - (px / W2) * W2;
    const float4 r = ld4(RB + a32((yy - y2a) * W2 + xx, 4 * ct + lg));
    st4(a.out + (((size_t)n * H2 + yy) * W2 + xx) * 32 + 16 * ct + 4 * lg,
        make_float4(acc[i][0] + bp3.x + r.x, acc[i][1] + bp3.y + r.y, acc[i][2] + bp3.z + r.z,
                    acc[i][3] + bp3.w + r.w));
  }
  f23_stamp(a.stamps, 7);
}

}  // namespace

// features.3 rows per workgroup: the largest T in {8, 4, 2, 1} whose tile fits
// the register tiles (features.1 pixels <= 16 x 8 x 8 per workgroup, project
// pairs <= 4 per wave, f3 expand tiles <= 2 per wave) and 160 KB of LDS; 0
// when none does (the caller keeps the per-block kernels)
int fir23_pick_rows(Fir23Args& a) {
  // (the ReLU blocks of mobilenet_v3_small; other activations keep the per-block kernels)
  if (a.act2e != ACT_RELU || a.act2d != ACT_RELU || a.act3e != ACT_RELU || a.act3d != ACT_RELU) return 0;
  if (a.E2 % 16 || a.E3 % 16 || a.E2 <= 0 || a.E3 <= 0 || 11 * a.E3 > 2 * F23_NT || a.H2 != (a.H1 - 1) / 2 + 1 || a.W2 != (a.W1 - 1) / 2 + 1)
    return 0;
  static const int t_env = kpd_diag_env("KPD_FIR23_T") ? atoi(kpd_diag_env("KPD_FIR23_T")) : 0;   // A/B sweeps
  for (int t = 8; t >= 1; t /= 2) {
    if (t_env > 0 && t > t_env) continue;
    a.T = t;
    const int ny2 = std::min(t + 2, a.H2), ny1 = std::min(2 * ny2 + 1, a.H1);
    const int npx1 = ny1 * a.W1, npx2 = ny2 * a.W2, npx3 = std::min(t, a.H2) * a.W2;
    const bool regs = (npx1 + 15) / 16 <= F23_NW * F23_MAXT1 && (npx2 + 15) / 16 <= F23_NW * F23_MAXT2 &&
                      2 * ((npx2 + 15) / 16) <= F23_NW * F23_MAXP && 2 * ((npx3 + 15) / 16) <= F23_NW * F23_MAXP;
    if (regs && (size_t)f23_lds(a).total * 4 <= 160 * 1024) return t;
  }
  a.T = 0;
  return 0;
}

hipError_t launch_fir23(const Fir23Args& a, int N, hipStream_t st) {
  if (a.T <= 0 || N <= 0 || N > 65535 || 11 * a.E3 > 2 * F23_NT || a.E2 % 16 || a.E3 % 16) return hipErrorInvalidValue;
  Fir23Args c = a;
  const int T = a.T;
  const int ny2 = std::min(T + 2, a.H2), ny1 = std::min(2 * ny2 + 1, a.H1);
  if ((ny1 * a.W1 + 15) / 16 > F23_NW * F23_MAXT1 || (ny2 * a.W2 + 15) / 16 > F23_NW * F23_MAXT2 ||
      2 * ((ny2 * a.W2 + 15) / 16) > F23_NW * F23_MAXP || 2 * ((std::min(T, a.H2) * a.W2 + 15) / 16) > F23_NW * F23_MAXP)
    return hipErrorInvalidValue;
  const size_t lds = (size_t)f23_lds(c).total * 4;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (!(a.act2e == ACT_RELU && a.act2d == ACT_RELU && a.act3e == ACT_RELU && a.act3d == ACT_RELU))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(fir23_kernel<true>, dim3((a.H2 + T - 1) / T, N), dim3(F23_NT), lds, st, c);
  return hipGetLastError();
}
