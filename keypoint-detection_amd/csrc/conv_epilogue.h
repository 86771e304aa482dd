// Conv epilogue shared by the MFMA conv kernels: the block's accumulator tile
// is staged through LDS so that every global store is a 16-byte-per-lane,
// full-row store (a 16x16 MFMA fragment alone would give 64-byte segments),
// and bias / activation / residual / channel statistics are applied in the
// coalesced pass.
#pragma once
#include "kpd_common.h"

struct EpiArgs {
  const float* bias;   // [cout_p]
  void* out;           // NHWC rows of out_cstride elements
  const float* res;    // optional residual NHWC [N][rh][rw][cout_p] (nearest-upsampled when rh != H)
  float* stats;        // optional [N][tiles_per_img][2][cout_p] (requires HW % BM == 0)
  float* amax;         // optional per-image max|out| (amax_publish_img)
  float scale;         // acc multiplier before bias (split16 unscale), 1 otherwise
  int M, H, W, cout_p, out_cstride, rh, rw, act, tiles_per_img;
  // optional second per-channel affine after the activation (an un-foldable BN
  // behind a non-linearity, KEYPOINT_HEAD ResidualBlock.bn1) and its act,
  // then the residual, then a final activation:
  //   v = act3( act2( act(acc*scale + bias) * post_scale + post_shift ) + res )
  const float* post_scale;
  const float* post_shift;
  int act2, act3;
};

// Physical 16-byte chunk of logical chunk c in LDS row r (rows of CPR chunks):
// an XOR swizzle that makes the MFMA fragment reads (ds_read_b128, 4 lane
// groups of 16 on gfx950) and the staging writes bank-conflict free.
template <int CPR>
__device__ __forceinline__ int lds_chunk(int r, int c) {
  if constexpr (CPR == 8) return c ^ (r & 7);
  else if constexpr (CPR == 4) return c ^ ((r ^ (r >> 1)) & 3);
  else return c;
}

// XCD-aware block order: workgroups are dealt round-robin over the 8 XCDs
// (block b and b+8 share one), so map the blocks of one XCD to CONSECUTIVE
// logical tiles -- neighbouring implicit-GEMM tiles share 3x3 halo rows and
// A tiles, which then hit the same 4 MiB L2.  Bijective for any nblk; a
// placement other than round-robin only changes speed, never results.
__device__ __forceinline__ int xcd_remap(int b, int nblk) {
  const int q = nblk / 8, r = nblk % 8, x = b % 8, k = b / 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
}

// fp32 tile [BM][BN+4] plus the per-thread channel-statistics partials
template <int BM, int BN, int NT = 256>
constexpr int epi_lds_bytes() { return (BM * (BN + 4) + 2 * NT) * 4; }

// acc[FM][FN] of wave (wm, wn) -> LDS tile [BM][BN+4] (fp32)
template <int FM, int FN, int WM, int WN, int BN>
__device__ __forceinline__ void acc_to_lds(float* tile, const f32x4 (&acc)[FM][FN], int wm, int wn, int lane) {
  constexpr int P = BN + 4;
  const int g = lane >> 4, r16 = lane & 15;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        tile[(wm * WM + i * 16 + g * 4 + e) * P + wn * WN + j * 16 + r16] = acc[i][j][e];
}

template <typename TO>
__device__ __forceinline__ void store4(TO* dst, const float4& v);
template <>
__device__ __forceinline__ void store4<float>(float* dst, const float4& v) {
  *reinterpret_cast<float4*>(dst) = v;
}
template <>
__device__ __forceinline__ void store4<__bf16>(__bf16* dst, const float4& v) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  bf16x4 o;
  o[0] = (__bf16)v.x; o[1] = (__bf16)v.y; o[2] = (__bf16)v.z; o[3] = (__bf16)v.w;
  *reinterpret_cast<bf16x4*>(dst) = o;
}

// Requires a __syncthreads() between acc_to_lds and this call (done inside).
// NT = threads of the workgroup; LDS behind the tile holds 2*NT stats floats.
// Two passes over a fixed per-thread set of (row, 4-column) cells: every
// global load (bias, second affine, residual) is issued before the first
// store -- hipcc cannot prove `out` does not alias them, so interleaving loads
// and stores would serialise one memory round trip per cell.
template <typename TO, int BM, int BN, int NT = 256>
__device__ __forceinline__ void tile_store(float* tile, const EpiArgs& p, int m0, int n0) {
  constexpr int P = BN + 4, C4 = BN / 4;
  static_assert(NT % C4 == 0 && (BM * C4) % NT == 0, "epilogue layout");
  constexpr int RS = NT / C4, IT = BM / RS;   // rows per pass, cells per thread
  const int tid = threadIdx.x;
  const int c4 = tid % C4, row0 = tid / C4;
  const int co = n0 + c4 * 4;
  const bool col_ok = co < p.cout_p;
  __syncthreads();
  float amax = 0.f;
  TO* out = reinterpret_cast<TO*>(p.out);
  const int HW = p.H * p.W;
  float4 b = make_float4(0.f, 0.f, 0.f, 0.f), ps = b, pt = b;
  if (col_ok) {
    b = *reinterpret_cast<const float4*>(p.bias + co);
    if (p.post_scale) {
      ps = *reinterpret_cast<const float4*>(p.post_scale + co);
      pt = *reinterpret_cast<const float4*>(p.post_shift + co);
    }
  }
  float4 v[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int row = row0 + it * RS, m = m0 + row;
    float4 x = *reinterpret_cast<const float4*>(tile + row * P + c4 * 4);
    x.x = kpd_act(x.x * p.scale + b.x, p.act);
    x.y = kpd_act(x.y * p.scale + b.y, p.act);
    x.z = kpd_act(x.z * p.scale + b.z, p.act);
    x.w = kpd_act(x.w * p.scale + b.w, p.act);
    if (p.post_scale) {
      x.x = kpd_act(x.x * ps.x + pt.x, p.act2); x.y = kpd_act(x.y * ps.y + pt.y, p.act2);
      x.z = kpd_act(x.z * ps.z + pt.z, p.act2); x.w = kpd_act(x.w * ps.w + pt.w, p.act2);
    }
    if (p.res && col_ok && m < p.M) {
      const int n = m / HW, r = m - n * HW, y = r / p.W, xx = r - y * p.W;
      int sy = y, sx = xx;
      if (p.rh != p.H) sy = min((int)floorf((float)y * ((float)p.rh / (float)p.H)), p.rh - 1);
      if (p.rw != p.W) sx = min((int)floorf((float)xx * ((float)p.rw / (float)p.W)), p.rw - 1);
      const float4 q = *reinterpret_cast<const float4*>(p.res + ((size_t)(n * p.rh + sy) * p.rw + sx) * p.cout_p + co);
      x.x += q.x; x.y += q.y; x.z += q.z; x.w += q.w;
    }
    if (p.act3) {
      x.x = kpd_act(x.x, p.act3); x.y = kpd_act(x.y, p.act3);
      x.z = kpd_act(x.z, p.act3); x.w = kpd_act(x.w, p.act3);
    }
    v[it] = x;
  }
  // per-image max|out|: cells of the tile's first image reduce over the
  // wave, cells of a later image (a tile straddling images) publish directly
  const int nb = m0 / HW;
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int row = row0 + it * RS, m = m0 + row;
    if (m >= p.M || !col_ok) continue;
    const float4 x = v[it];
    const float mc = fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w)));
    if (p.amax && m / HW != nb) amax_publish_img(p.amax, m / HW, mc);
    else amax = fmaxf(amax, mc);
    store4<TO>(out + (size_t)m * p.out_cstride + co, x);
    if (p.stats) *reinterpret_cast<float4*>(tile + row * P + c4 * 4) = x;
  }
  if (p.amax) {
    const float w = wave_max(amax);
    if ((tid & 63) == 0) amax_publish_img(p.amax, nb, w);
  }
  if (p.stats) {
    // column sums / maxima: NT/BN row groups in parallel, then one combine
    constexpr int RG = NT / BN;
    static_assert(RG >= 1 && BM % RG == 0, "stats layout");
    float* part = tile + BM * P;
    __syncthreads();
    {
      const int col = tid % BN, rg = tid / BN;
      float s = 0.f, mx = -INFINITY;
      for (int r = rg; r < BM; r += RG) {
        const float v = tile[r * P + col];
        s += v;
        mx = fmaxf(mx, v);
      }
      part[rg * BN + col] = s;
      part[NT + rg * BN + col] = mx;
    }
    __syncthreads();
    if (tid < BN && n0 + tid < p.cout_p) {
      float s = part[tid], mx = part[NT + tid];
#pragma unroll
      for (int g = 1; g < RG; ++g) {
        s += part[g * BN + tid];
        mx = fmaxf(mx, part[NT + g * BN + tid]);
      }
      const int n = m0 / HW, t = (m0 - n * HW) / BM;
      float* st = p.stats + ((size_t)n * p.tiles_per_img + t) * 2 * p.cout_p;
      st[n0 + tid] = s;
      st[p.cout_p + n0 + tid] = mx;
    }
  }
}
