// LightweightFPN laterals as one launch (reference dll/models/backbone.py:
// 29-39): lat3 = L3 . tap3, lat2 = L2 . tap2 + up(lat3), lat1 = L1 . tap1 +
// up(lat2) (1x1 convs without bias, nearest top-down upsampling as
// F.interpolate(size=...)).  The top-down adds are channel-wise, so a
// workgroup takes one image and 16 output channels and runs the whole chain
// with lat3 / lat2 in LDS: only lat1 reaches HBM (the split-mode FPN level 0
// reads lat1 and the stem tap; lateral 0 is never materialised).  Replaces
// five launches (lateral 3 split-K GEMM + reduce, lateral 2, lateral 1) whose
// cost was latency, not work.  gfx950:
//   * 1x1 convs on v_mfma_f32_16x16x4_f32 (exact fp32 products; a lane's
//     float4 of 4 consecutive input channels feeds 4 MFMAs, with the weights
//     permuted alike), operands straight from L2;
//   * lat3 (few pixels, K = 576) splits K over the 4 waves, partial sums added
//     in wave order; lat2 / lat1 split the pixel tiles over the waves;
//   * per-image max |lat1| published for the split FPN scale (as the generic
//     conv epilogue did).
#include <algorithm>

#include "kpd_common.h"
#include "kpd_kernels.h"

namespace {

constexpr int LG = 16;   // output channels per workgroup

__device__ __forceinline__ int up_index(int y, int H, int h) {   // nearest, F.interpolate(size=(H, .)) from h
  return H == h ? y : min((int)floorf((float)y * ((float)h / (float)H)), h - 1);
}

// diagnostic phase stamps (KPD_STAMPS): thread 0, s_memrealtime, row [8] per workgroup
__device__ __forceinline__ void stamp(unsigned long long* st, int i) {
  if (st && threadIdx.x == 0)
    st[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 + i] = __builtin_amdgcn_s_memrealtime();
}

// MFMA over one 16-channel K chunk: lane (g, r16) supplies A[px r16][4g .. 4g+3]
// and B[co r16][4g .. 4g+3]
__device__ __forceinline__ f32x4 mfma_k16(const float4 a, const float4 b, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc, 0, 0, 0);
}

// NK1 / NK2 / NK3: 16-channel K chunks of laterals 1 / 2 / 3 (the model's 24
// -> 32, 48 and 576 input channels); T3: lateral-3 tiles (at most 16 * T3
// pixels); T1: lateral-1 tiles per wave and load batch.  Eight waves; every phase
// issues all its independent loads before its MFMAs, so a phase costs about
// one memory round trip: the chain is latency (and fp32-MFMA rate), not
// bandwidth (a 256x192 image's whole chain reads 0.3 MB).
//
// SPLIT: lateral 1 leaves as the f16 hi|lo rows fpn0x_kernel reads (the
// layout of split_rows_kernel), scaled by 2^a_l from fpn0x_exps(max|tap0|,
// bound).  The bound is S1 m1 + S2 m2 + S3 m3 >= max|lateral 1| (S_i = max
// over output channels of sum |L_i|, m_i = max|tap_i| of the image): every
// workgroup of the image reads all of its taps, so all eight compute the same
// bound without talking to each other, and it is published in place of the
// max (slot amax[n * kAmaxStride]) for the consumers' unscale.  A bound
// looser than the max only lowers the split's precision floor, which sits
// ~2^-39 of the largest scaled operand: 2^12 of slack still leaves it below
// fp32 rounding.
constexpr int NW = 8;

// REUSE (SPLIT, lateral 1 in one load batch per wave): the max|tap1| scan's
// registers are lateral 1's A operands (the same pixels, tiles wave + NW j,
// in the same lane layout), so lateral 1 issues no tap1 loads of its own.
template <int NK1, int NK2, int NK3, int T3, int T1, bool SPLIT, bool REUSE = false>
__global__ __launch_bounds__(NW * 64) void lateral_chain_kernel(const LatChainArgs p) {
  static_assert(!REUSE || (SPLIT && T1 == 6), "tap1 registers reused as lateral 1's A: one 6-tile batch");
  extern __shared__ __attribute__((aligned(16))) float lsm[];
  const int P1 = p.h1 * p.w1, P2 = p.h2 * p.w2, P3 = p.h3 * p.w3;
  float* l3 = lsm;                      // [P3][16]
  float* l2 = l3 + P3 * LG;             // [P2][16]
  float* red = l2;                      // [NW][P3][16] lat3 partials (dead before l2 is written)
  float* mx = l2 + max(P2, NW * P3) * LG;   // [3][NW] per-wave tap maxima
  // SPLIT: per-wave transpose scratch of one lateral-1 tile (16 pixels x
  // [hi16 | lo16] halves, 1 KB), so that a lane stores 16 contiguous bytes
  _Float16* tsc = reinterpret_cast<_Float16*>(mx + 4 * NW) + (threadIdx.x >> 6) * (16 * 2 * LG);
  // grid (B rounded up to 8, 8): workgroup id b + Bp * cg sits on XCD b % 8,
  // so an image's 8 channel groups share one L2 and its taps leave HBM once
  const int b = blockIdx.x, cg = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (b >= p.n) return;
  const int g = lane >> 4, r16 = lane & 15, co = cg * LG + r16;
  const float* t1 = p.t1 + (size_t)b * P1 * (NK1 * 16) + 4 * g;
  const float* t2 = p.t2 + (size_t)b * P2 * (NK2 * 16) + 4 * g;
  const float* t3 = p.t3 + (size_t)b * P3 * (NK3 * 16) + 4 * g;
  // max |x| over the real input channels (c0 = this float4's first channel)
  auto amax4 = [](float m, const float4 v, int c0, int creal) {
    if (c0 + 0 < creal) m = fmaxf(m, fabsf(v.x));
    if (c0 + 1 < creal) m = fmaxf(m, fabsf(v.y));
    if (c0 + 2 < creal) m = fmaxf(m, fabsf(v.z));
    if (c0 + 3 < creal) m = fmaxf(m, fabsf(v.w));
    return m;
  };
  float m1 = 0.f, m2 = 0.f, m3 = 0.f;
  stamp(p.stamps, 0);

  // lat3: every tile at once, K chunks q = wave + NW * u (partials added in wave order)
  {
    constexpr int U3 = (NK3 + NW - 1) / NW, UB = T3 <= 3 ? 3 : 1;   // K chunks per wave, per load batch
    const int nt3 = (P3 + 15) / 16;
    const float* brow = p.L3 + (size_t)co * (NK3 * 16) + 4 * g;
    f32x4 acc[T3];
#pragma unroll
    for (int t = 0; t < T3; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u0 = 0; u0 < U3; u0 += UB) {
      float4 bb[UB], a[UB][T3];
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int q = min(wave + NW * (u0 + u), NK3 - 1);
        bb[u] = *reinterpret_cast<const float4*>(brow + q * 16);
#pragma unroll
        for (int t = 0; t < T3; ++t)
          a[u][t] = *reinterpret_cast<const float4*>(t3 + (size_t)min(t * 16 + r16, P3 - 1) * (NK3 * 16) + q * 16);
      }
#pragma unroll
      for (int u = 0; u < UB; ++u)
        if (u0 + u < U3 && wave + NW * (u0 + u) < NK3)
#pragma unroll
          for (int t = 0; t < T3; ++t) {
            acc[t] = mfma_k16(a[u][t], bb[u], acc[t]);
            if (SPLIT) m3 = amax4(m3, a[u][t], (wave + NW * (u0 + u)) * 16 + 4 * g, p.c3r);
          }
    }
#pragma unroll
    for (int t = 0; t < T3; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int pp = t * 16 + 4 * g + e;
        if (t < nt3 && pp < P3) red[(wave * P3 + pp) * LG + r16] = acc[t][e];
      }
  }
  float4 v[6][NK1];   // REUSE: tap1 tiles wave + NW j, kept for lateral 1
#pragma unroll
  for (int j = 0; j < 6; ++j)
#pragma unroll
    for (int k = 0; k < NK1; ++k) v[j][k] = make_float4(0.f, 0.f, 0.f, 0.f);   // (lanes past the map: no load)
  if (SPLIT) {
    // max |tap1| of the image over the real channels: wave w scans pixels w, w + NW, ...
    // (batches of 6 pixel rows per lane, loads issued together)
    for (int px0 = wave * 16 + r16; px0 < P1; px0 += 6 * NW * 16) {
#pragma unroll
      for (int j = 0; j < 6; ++j)
#pragma unroll
        for (int k = 0; k < NK1; ++k)
          v[j][k] = *reinterpret_cast<const float4*>(t1 + (size_t)min(px0 + j * NW * 16, P1 - 1) * (NK1 * 16) + 16 * k);
#pragma unroll
      for (int j = 0; j < 6; ++j)
#pragma unroll
        for (int k = 0; k < NK1; ++k) m1 = amax4(m1, v[j][k], 16 * k + 4 * g, p.c1r);
    }
    m1 = wave_max(m1);
    m3 = wave_max(m3);
    if (lane == 0) {
      mx[wave] = m1;
      mx[2 * NW + wave] = m3;
    }
  }
  stamp(p.stamps, 1);
  __syncthreads();
  for (int i = tid; i < P3 * LG; i += NW * 64) {
    float v = red[i];
#pragma unroll
    for (int w = 1; w < NW; ++w) v += red[w * P3 * LG + i];
    l3[i] = v;
  }
  __syncthreads();
  stamp(p.stamps, 2);

  // lat2 = L2 . tap2 + up(lat3): wave takes tiles wave + NW * j in batches of JB
  {
    constexpr int JB = 2;
    float4 bw[NK2];
#pragma unroll
    for (int k = 0; k < NK2; ++k) bw[k] = *reinterpret_cast<const float4*>(p.L2 + (size_t)co * (NK2 * 16) + 4 * g + 16 * k);
    const int nt2 = (P2 + 15) / 16;
    for (int t0 = wave; t0 < nt2; t0 += NW * JB) {
      float4 a[JB][NK2];
#pragma unroll
      for (int j = 0; j < JB; ++j) {
        const int px = min((t0 + NW * j) * 16 + r16, P2 - 1);
#pragma unroll
        for (int k = 0; k < NK2; ++k) a[j][k] = *reinterpret_cast<const float4*>(t2 + (size_t)px * (NK2 * 16) + 16 * k);
      }
#pragma unroll
      for (int j = 0; j < JB; ++j) {
        const int t = t0 + NW * j;
        if (t >= nt2) break;
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < NK2; ++k) {
          acc = mfma_k16(a[j][k], bw[k], acc);
          if (SPLIT) m2 = amax4(m2, a[j][k], 16 * k + 4 * g, p.c2r);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int pp = t * 16 + 4 * g + e;
          if (pp >= P2) continue;
          const int y = pp / p.w2, x = pp - y * p.w2;
          const int sy = up_index(y, p.h2, p.h3), sx = up_index(x, p.w2, p.w3);
          l2[pp * LG + r16] = acc[e] + l3[(sy * p.w3 + sx) * LG + r16];
        }
      }
    }
  }
  if (SPLIT) {
    m2 = wave_max(m2);
    if (lane == 0) mx[NW + wave] = m2;
  }
  stamp(p.stamps, 3);
  __syncthreads();

  // lat1 = L1 . tap1 + up(lat2) -> HBM (fp32, or split by the image's bound)
  float s_l = 1.f, s_f = 1.f;
  _Float16* outs = nullptr;
  const int part = lane & 3;
  if constexpr (SPLIT) {
    float M1 = mx[0], M2 = mx[NW], M3 = mx[2 * NW];
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      M1 = fmaxf(M1, mx[w]);
      M2 = fmaxf(M2, mx[NW + w]);
      M3 = fmaxf(M3, mx[2 * NW + w]);
    }
    const float bound = fmaf(p.S1, M1, fmaf(p.S2, M2, p.S3 * M3));
    int a_f, a_l, P;
    fpn0x_exps(p.amax[(size_t)b * kAmaxStride], bound, p.w_exp0, p.w_expE, &a_f, &a_l, &P);
    s_l = ldexpf(1.f, a_l);
    s_f = ldexpf(1.f, a_f);
    if (tid == 0) amax_publish_img(p.amax + (size_t)p.n * kAmaxStride, b, bound);
    // hi|lo rows: pixel pp at halves [pp][2 * 128]; channel co in group co / 32: hi at +co % 32, lo 32 further.
    // A lane stores 8 halves: pixel lane / 4, part lane % 4 = (hi | lo) x (channels 0-7 | 8-15) of the group
    outs = p.lat1_split + (size_t)b * P1 * 256 + (cg >> 1) * 64 + (cg & 1) * 16 + (part >> 1) * 32 + (part & 1) * 8;
  }
  {
    constexpr int JB = T1;
    float4 bw[NK1];
#pragma unroll
    for (int k = 0; k < NK1; ++k) bw[k] = *reinterpret_cast<const float4*>(p.L1 + (size_t)co * (NK1 * 16) + 4 * g + 16 * k);
    const int nt1 = (P1 + 15) / 16;
    float* out = p.lat1 + (size_t)b * P1 * 128 + co;
    for (int t0 = wave; t0 < nt1; t0 += NW * JB) {
      float4 a[JB][NK1];
#pragma unroll
      for (int j = 0; j < JB; ++j) {
        const int px = min((t0 + NW * j) * 16 + r16, P1 - 1);
#pragma unroll
        for (int k = 0; k < NK1; ++k)
          a[j][k] = REUSE ? v[j][k] : *reinterpret_cast<const float4*>(t1 + (size_t)px * (NK1 * 16) + 16 * k);
      }
#pragma unroll
      for (int j = 0; j < JB; ++j) {
        const int t = t0 + NW * j;
        if (t >= nt1) break;
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < NK1; ++k) acc = mfma_k16(a[j][k], bw[k], acc);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int pp = t * 16 + 4 * g + e;
          if (pp >= P1) continue;
          const int y = pp / p.w1, x = pp - y * p.w1;
          const int sy = up_index(y, p.h1, p.h2), sx = up_index(x, p.w1, p.w2);
          const float v = acc[e] + l2[(sy * p.w2 + sx) * LG + r16];
          if constexpr (SPLIT) {
            const float xs = v * s_l;
            const _Float16 hi = (_Float16)xs;
            tsc[(4 * g + e) * 32 + r16] = hi;
            tsc[(4 * g + e) * 32 + 16 + r16] = (_Float16)(xs - (float)hi);
          } else {
            out[(size_t)pp * 128] = v;
          }
        }
        if constexpr (SPLIT) {
          // (LDS operations of one wave complete in order: the reads see
          // every lane's writes, and the next tile's writes follow them)
          const int q = lane >> 2, pp = t * 16 + q;
          const uint4 v = *reinterpret_cast<const uint4*>(tsc + q * 32 + part * 8);
          if (pp < P1) *reinterpret_cast<uint4*>(outs + (size_t)pp * 256) = v;
        }
      }
    }
  }
  stamp(p.stamps, 4);
  if constexpr (SPLIT) {
    // the stem tap's split rows (split_rows_kernel's layout for 16 channels:
    // [hi16 | lo16] per pixel) with 2^a_f: channel group cg converts its
    // eighth of the image's pixels, 8 channels per item, loads batched; this
    // streams beside the latency-bound chain instead of as its own launch
    if (p.t0) {
      const int P0 = p.P0, n8 = P0 * 2, per = (n8 + 7) / 8, i0 = cg * per, i1 = min(i0 + per, n8);
      const float* src = p.t0 + (size_t)b * P0 * 16;
      _Float16* dst = p.t0_split + (size_t)b * P0 * 32;
      typedef _Float16 f16x8v __attribute__((ext_vector_type(8)));
      for (int j0 = i0 + tid; j0 < i1; j0 += 4 * NW * 64) {
        float4 u[4][2];
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int j = min(j0 + v * NW * 64, i1 - 1), px = j >> 1, c = (j & 1) * 8;
          u[v][0] = *reinterpret_cast<const float4*>(src + (size_t)px * 16 + c);
          u[v][1] = *reinterpret_cast<const float4*>(src + (size_t)px * 16 + c + 4);
        }
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int j = j0 + v * NW * 64, px = j >> 1, c = (j & 1) * 8;
          if (j >= i1) continue;
          const float x[8] = {u[v][0].x, u[v][0].y, u[v][0].z, u[v][0].w, u[v][1].x, u[v][1].y, u[v][1].z, u[v][1].w};
          f16x8v hi, lo;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float xs = x[e] * s_f;
            hi[e] = (_Float16)xs;
            lo[e] = (_Float16)(xs - (float)hi[e]);
          }
          _Float16* o = dst + (size_t)px * 32 + c;
          *reinterpret_cast<f16x8v*>(o) = hi;
          *reinterpret_cast<f16x8v*>(o + 16) = lo;
        }
      }
    }
  }
  stamp(p.stamps, 5);
}

}  // namespace

size_t lateral_chain_lds_bytes(const LatChainArgs& a) {
  const size_t P2 = (size_t)a.h2 * a.w2, P3 = (size_t)a.h3 * a.w3;
  // (+ the split path's per-wave transpose tiles: 16 x 32 halves per wave)
  return (P3 * LG + std::max(P2, NW * P3) * LG + 4 * NW) * sizeof(float) + (size_t)NW * 16 * 2 * LG * 2;
}

bool lateral_chain_ok(const LatChainArgs& a) {
  return a.c1 == 32 && a.c2 == 48 && a.c3 == 576 && a.h1 > 0 && a.w1 > 0 && a.h2 > 0 && a.w2 > 0 && a.h3 > 0 &&
         a.w3 > 0 && a.h3 * a.w3 <= 16 * 8 && lateral_chain_lds_bytes(a) <= 80 * 1024 &&
         (!a.lat1_split || a.amax);
}

hipError_t launch_lateral_chain(const LatChainArgs& a, int B, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  if (!lateral_chain_ok(a)) return hipErrorInvalidValue;
  LatChainArgs q = a;
  q.n = B;
  const dim3 grid((unsigned)((B + 7) / 8 * 8), 128 / LG), block(NW * 64);
  const size_t lds = lateral_chain_lds_bytes(a);
  const bool small = a.h3 * a.w3 <= 16 * 3;
  // REUSE when lateral 1 is one 6-tile batch per wave (A/B: KPD_LC_NOREUSE=1 off)
  static const bool noreuse = kpd_diag_env("KPD_LC_NOREUSE") != nullptr;
  const bool reuse = !noreuse && (long)a.h1 * a.w1 <= 6 * NW * 16;
  if (a.lat1_split && small && reuse) {
    hipLaunchKernelGGL((lateral_chain_kernel<2, 3, 36, 3, 6, true, true>), grid, block, lds, st, q);
  } else if (a.lat1_split && reuse) {
    hipLaunchKernelGGL((lateral_chain_kernel<2, 3, 36, 8, 6, true, true>), grid, block, lds, st, q);
  } else if (a.lat1_split) {
    if (small) hipLaunchKernelGGL((lateral_chain_kernel<2, 3, 36, 3, 6, true>), grid, block, lds, st, q);
    else hipLaunchKernelGGL((lateral_chain_kernel<2, 3, 36, 8, 6, true>), grid, block, lds, st, q);
  } else {
    if (small) hipLaunchKernelGGL((lateral_chain_kernel<2, 3, 36, 3, 6, false>), grid, block, lds, st, q);
    else hipLaunchKernelGGL((lateral_chain_kernel<2, 3, 36, 8, 6, false>), grid, block, lds, st, q);
  }
  return hipGetLastError();
}
