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

__device__ __forceinline__ int a16(int px, int c) { return px * 16 + 4 * (c ^ ((px >> 2) & 3)); }
__device__ __forceinline__ int a32(int px, int c) { return px * 32 + 4 * (c ^ ((px >> 1) & 7)); }

// diagnostic phase stamps (KPD_STAMPS, diagnostic build): 0 start, 1 operands
// staged, 2 / 3 first features.2 expand / depthwise done, 4 features.2 done,
// 5 Y2 stored, 6 features.3 done, 7 end
__device__ __forceinline__ void f23_stamp(unsigned long long* st, int i) {
  if (st && threadIdx.x == 0) st[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 + i] = __builtin_amdgcn_s_memrealtime();
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float4 act4(float4 v, int act) {
  return make_float4(kpd_act(v.x, act), kpd_act(v.y, act), kpd_act(v.z, act), kpd_act(v.w, act));
}

// region sizes in floats for the largest (interior) tile of T rows
struct F23Lds {
  int wd2, bd2, wd3, bd3, ra, rb, total;
};
__host__ __device__ inline F23Lds f23_lds(const Fir23Args& a) {
  const int ny2 = min(a.T + 2, a.H2), ny1 = min(2 * ny2 + 1, a.H1);
  const int npx1 = ny1 * a.W1, npx2 = ny2 * a.W2, npx3 = min(a.T, a.H2) * a.W2;
  F23Lds L;
  L.wd2 = 0;
  L.bd2 = L.wd2 + 9 * a.E2;
  L.wd3 = L.bd2 + a.E2;
  L.bd3 = L.wd3 + 9 * a.E3;
  L.ra = (L.bd3 + a.E3 + 3) / 4 * 4;
  // region A: the features.2 expanded slice, later the features.3 expanded slice + 2 depthwise slices
  const int ra = max(npx1 * 16, npx2 * 16 + 2 * npx3 * 16);
  L.rb = L.ra + ra;
  // region B: 2 features.2 depthwise slices, later the features.2 output (32 floats per pixel)
  L.total = L.rb + npx2 * 32;
  return L;
}

// One thread's depthwise item (pixel p of the output rows, channel quad q),
// fixed for every channel slice: the source tile pixel of tap (0, 0) (row
// pitch W, may lie outside the tile) and a mask of the taps inside the map
// (outside: the tap reads a valid pixel and is skipped)
struct DwItem {
  int base, mask, q, p;
};

// 3x3 depthwise of one item: taps ky-major, bias, activation -> 4 channels
__device__ __forceinline__ float4 dw_item(const float* src, int W, const float* wd, int E, const float* bd, int c0,
                                          const DwItem& d, int act) {
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    float4 e[3], w[3];
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int t = ky * 3 + kx;
      e[kx] = ld4(src + a16(((d.mask >> t) & 1) ? d.base + ky * W + kx : 0, d.q));
      w[kx] = ld4(wd + t * E + c0 + 4 * d.q);
    }
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      if (!((d.mask >> (ky * 3 + kx)) & 1)) continue;
      s.x = fmaf(e[kx].x, w[kx].x, s.x); s.y = fmaf(e[kx].y, w[kx].y, s.y);
      s.z = fmaf(e[kx].z, w[kx].z, s.z); s.w = fmaf(e[kx].w, w[kx].w, s.w);
    }
  }
  const float4 b = ld4(bd + c0 + 4 * d.q);
  return act4(make_float4(s.x + b.x, s.y + b.y, s.z + b.z, s.w + b.w), act);
}

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
  float* RA = sm + L.ra;
  float* RB = sm + L.rb;

  // this wave's features.1 pixel tiles: the B operand of every features.2
  // expand slice (issued first: they land while the weights are staged)
  const float* x1 = a.x + ((size_t)n * H1 + e1a) * W1 * 16;
  float4 af[F23_MAXT1];
#pragma unroll
  for (int i = 0; i < F23_MAXT1; ++i) {
    const int px = (wave + F23_NW * i) * 16 + lr;
    af[i] = px < NPX1 ? ld4(x1 + (size_t)px * 16 + 4 * lg) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // per-slice operands of features.2 (one slice ahead): expand A =
  // We2[c0 + lr][4 lg ..], its bias for this lane's output channels, project
  // A = Wp2[16 ct + lr][c0 + 4 lg ..] (ct = the wave's parity, below)
  const int ct = wave & 1;
  float4 we_n = ld4(a.we2 + (size_t)lr * 16 + 4 * lg), be_n = ld4(a.be2 + 4 * lg);
  float4 wp_n = ld4(a.wp2 + (size_t)(16 * ct + lr) * E2 + 4 * lg);
  // depthwise weights and biases of both blocks -> LDS
  for (int i = tid; i < 9 * E2; i += F23_NT) sm[L.wd2 + i] = a.wd2[i];
  for (int i = tid; i < E2; i += F23_NT) sm[L.bd2 + i] = a.bd2[i];
  for (int i = tid; i < 9 * E3; i += F23_NT) sm[L.wd3 + i] = a.wd3[i];
  for (int i = tid; i < E3; i += F23_NT) sm[L.bd3 + i] = a.bd3[i];

  // depthwise items (pixel-fastest over the threads: a wave's 16-lane groups
  // read 16 neighbouring pixels of one chunk)
  DwItem d2{}, d3{};
  const bool has2 = tid < NPX2 * 4, has3 = tid < NPX3 * 4;
  if (has2) {
    d2.q = tid / NPX2;
    d2.p = tid - d2.q * NPX2;
    const int yy = y2a + d2.p / W2, xx = d2.p % W2;
    d2.base = (2 * yy - 1 - e1a) * W1 + 2 * xx - 1;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int iy = 2 * yy - 1 + t / 3, ix = 2 * xx - 1 + t % 3;
      d2.mask |= (iy >= e1a && iy < e1b && ix >= 0 && ix < W1) ? 1 << t : 0;
    }
  }
  if (has3) {
    d3.q = tid / NPX3;
    d3.p = tid - d3.q * NPX3;
    const int yy = r0 + d3.p / W2, xx = d3.p % W2;
    d3.base = (yy - 1 - y2a) * W2 + xx - 1;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int iy = yy - 1 + t / 3, ix = xx - 1 + t % 3;
      d3.mask |= (iy >= y2a && iy < y2b && ix >= 0 && ix < W2) ? 1 << t : 0;
    }
  }

  // ---------------- features.2: 16 expanded channels per slice ----------------
  f32x4 acc[F23_MAXP];
#pragma unroll
  for (int i = 0; i < F23_MAXP; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();   // depthwise weights staged
  f23_stamp(a.stamps, 1);
  for (int c0 = 0, sl = 0; c0 < E2; c0 += 16, ++sl) {
    const float4 we = we_n, be = be_n, wp = wp_n;
    if (c0 + 16 < E2) {
      const int c1 = c0 + 16;
      we_n = ld4(a.we2 + (size_t)(c1 + lr) * 16 + 4 * lg);
      be_n = ld4(a.be2 + c1 + 4 * lg);
      wp_n = ld4(a.wp2 + (size_t)(16 * ct + lr) * E2 + c1 + 4 * lg);
    }
    // expand: E2 slice [px][16] = act(We2 slice . X1 + be2); the wave's tiles
    // as independent accumulator chains, step-major (tiles past the map
    // multiply zeros and are not stored)
    {
      f32x4 e[F23_MAXT1];
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
#pragma unroll
      for (int i = 0; i < F23_MAXT1; ++i) {
        const int px = (wave + F23_NW * i) * 16 + lr;
        if (px < NPX1)
          st4(RA + a16(px, lg), act4(make_float4(e[i][0] + be.x, e[i][1] + be.y, e[i][2] + be.z, e[i][3] + be.w),
                                     a.act2e));
      }
    }
    if (sl == 0) f23_stamp(a.stamps, 2);
    __syncthreads();
    // depthwise 3x3 stride 2 (zero outside the features.1 map)
    float* D2 = RB + (sl & 1) * NPX2 * 16;
    if (has2) st4(D2 + a16(d2.p, d2.q), dw_item(RA, W1, sm + L.wd2, E2, sm + L.bd2, c0, d2, a.act2d));
    if (sl == 0) f23_stamp(a.stamps, 3);
    __syncthreads();
    // project: Y2 += Wp2 slice . D2 slice (accumulators persist across slices;
    // D2 is double-buffered, so the next slice's expand needs no barrier here).
    // Pair i of the wave = (channel tile ct, pixel tile (wave >> 1) + 8 i)
    {
      float4 b[F23_MAXP];
#pragma unroll
      for (int i = 0; i < F23_MAXP; ++i) {
        const int px = ((wave >> 1) + (F23_NW / 2) * i) * 16 + lr;
        b[i] = px < NPX2 ? ld4(D2 + a16(px, lg)) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int i = 0; i < F23_MAXP; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(wp.x, b[i].x, acc[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < F23_MAXP; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(wp.y, b[i].y, acc[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < F23_MAXP; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(wp.z, b[i].z, acc[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < F23_MAXP; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(wp.w, b[i].w, acc[i], 0, 0, 0);
    }
  }
  f23_stamp(a.stamps, 4);
  // features.3 per-slice operands, first slice (issued before the barrier)
  float4 we3_n0 = ld4(a.we3 + (size_t)lr * 32 + 8 * lg), we3_n1 = ld4(a.we3 + (size_t)lr * 32 + 8 * lg + 4);
  float4 be3_n = ld4(a.be3 + 4 * lg);
  float4 wp3_n = ld4(a.wp3 + (size_t)(16 * ct + lr) * E3 + 4 * lg);
  const float4 bp2 = ld4(a.bp2 + 16 * ct + 4 * lg), bp3 = ld4(a.bp3 + 16 * ct + 4 * lg);
  __syncthreads();   // every wave's last project read of D2 done: region B becomes Y2
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

  // ---------------- features.3: 16 expanded channels per slice ----------------
  // this wave's Y2 pixel tile: the B operand of every features.3 expand slice
  // (K = 32: lane group g supplies channels 8 g .. 8 g + 7 over 8 steps)
  float4 yf[F23_MAXT2][2];
#pragma unroll
  for (int i = 0; i < F23_MAXT2; ++i) {
    const int px = (wave + F23_NW * i) * 16 + lr;
    yf[i][0] = px < NPX2 ? ld4(RB + a32(px, 2 * lg)) : make_float4(0.f, 0.f, 0.f, 0.f);
    yf[i][1] = px < NPX2 ? ld4(RB + a32(px, 2 * lg + 1)) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int i = 0; i < F23_MAXP; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float* E3s = RA;
  for (int c0 = 0, sl = 0; c0 < E3; c0 += 16, ++sl) {
    const float4 w0 = we3_n0, w1 = we3_n1, be = be3_n, wp = wp3_n;
    if (c0 + 16 < E3) {
      const int c1 = c0 + 16;
      we3_n0 = ld4(a.we3 + (size_t)(c1 + lr) * 32 + 8 * lg);
      we3_n1 = ld4(a.we3 + (size_t)(c1 + lr) * 32 + 8 * lg + 4);
      be3_n = ld4(a.be3 + c1 + 4 * lg);
      wp3_n = ld4(a.wp3 + (size_t)(16 * ct + lr) * E3 + c1 + 4 * lg);
    }
    // expand: E3 slice [px][16] over the Y2 rows (all inside the map)
    {
      f32x4 e[F23_MAXT2];
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
#pragma unroll
      for (int i = 0; i < F23_MAXT2; ++i) {
        const int px = (wave + F23_NW * i) * 16 + lr;
        if (px < NPX2)
          st4(E3s + a16(px, lg), act4(make_float4(e[i][0] + be.x, e[i][1] + be.y, e[i][2] + be.z, e[i][3] + be.w),
                                      a.act3e));
      }
    }
    __syncthreads();
    // depthwise 3x3 stride 1 (zero outside the features.2 map)
    float* D3 = RA + NPX2 * 16 + (sl & 1) * NPX3 * 16;
    if (has3) st4(D3 + a16(d3.p, d3.q), dw_item(E3s, W2, sm + L.wd3, E3, sm + L.bd3, c0, d3, a.act3d));
    __syncthreads();
    {
      float4 b[F23_MAXP];
#pragma unroll
      for (int i = 0; i < F23_MAXP; ++i) {
        const int px = ((wave >> 1) + (F23_NW / 2) * i) * 16 + lr;
        b[i] = px < NPX3 ? ld4(D3 + a16(px, lg)) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int i = 0; i < F23_MAXP; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(wp.x, b[i].x, acc[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < F23_MAXP; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(wp.y, b[i].y, acc[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < F23_MAXP; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(wp.z, b[i].z, acc[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < F23_MAXP; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(wp.w, b[i].w, acc[i], 0, 0, 0);
    }
  }
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
  if (a.E2 % 16 || a.E3 % 16 || a.E2 <= 0 || a.E3 <= 0 || a.H2 != (a.H1 - 1) / 2 + 1 || a.W2 != (a.W1 - 1) / 2 + 1)
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
  if (a.T <= 0 || N <= 0 || N > 65535) return hipErrorInvalidValue;
  Fir23Args c = a;
  const int T = a.T;
  const int ny2 = std::min(T + 2, a.H2), ny1 = std::min(2 * ny2 + 1, a.H1);
  if ((ny1 * a.W1 + 15) / 16 > F23_NW * F23_MAXT1 || (ny2 * a.W2 + 15) / 16 > F23_NW * F23_MAXT2 ||
      2 * ((ny2 * a.W2 + 15) / 16) > F23_NW * F23_MAXP || 2 * ((std::min(T, a.H2) * a.W2 + 15) / 16) > F23_NW * F23_MAXP)
    return hipErrorInvalidValue;
  const size_t lds = (size_t)f23_lds(c).total * 4;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fir23_kernel, dim3((a.H2 + T - 1) / T, N), dim3(F23_NT), lds, st, c);
  return hipGetLastError();
}
