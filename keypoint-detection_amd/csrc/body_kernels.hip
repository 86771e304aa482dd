// MobileNetV3-Small body kernels that are not GEMM-shaped (gfx950).
//
//   * stem: conv3x3 s2 (Cin 1|3 -> 16) + folded BN + hardswish, reads the
//     caller's NCHW fp32 image directly and writes NHWC (fused layout change).
//     torchvision mobilenet_v3_small features.0 (reference backbone.py:250-254).
//   * dwconv: depthwise k3/k5 s1/s2 + folded BN + ReLU/hardswish, NHWC, four
//     channels per lane (16-byte loads/stores along C).  features.N.block.dw.
//   * se: squeeze (global average) + fc1/ReLU + fc2/hardsigmoid, one workgroup
//     per image; the excitation is applied later inside the project conv's
//     A-load (conv_mfma.hip, a_scale), so the scaled tensor never hits HBM.
//   * channel_stats: per-image channel sum/max partials for ChannelAttention
//     when the FPN conv epilogue cannot produce them (H*W not a tile multiple).
#include <algorithm>
#include <cstdlib>

#include "kpd_common.h"
#include "kpd_kernels.h"
#include "kpd_dma.h"

namespace {

constexpr int kSeExcitePart = 6144;   // fc1 partial floats per image staged by se_excite_kernel

// In-kernel phase stamps (diagnostic, KPD_STAMPS): thread 0 of each workgroup
// records s_memrealtime (100 MHz) at phase boundaries into its own 8-slot row
// of a buffer no other code reads.
__device__ __forceinline__ void stamp(unsigned long long* st, int i) {
  if (st && threadIdx.x == 0)
    st[(((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 8 + i] = __builtin_amdgcn_s_memrealtime();
}

// Stem: 3x3 stride-2 conv (CIN -> 16) + folded BN + h-swish, NCHW image in,
// NHWC out; CIN is a template argument so the 9*CIN inputs stay in registers.
template <int CIN>
__global__ __launch_bounds__(256) void stem_kernel(const float* __restrict__ img, int N, int H, int W,
                                                   const float* __restrict__ w, const float* __restrict__ b,
                                                   float* __restrict__ out, int Ho, int Wo,
                                                   float* __restrict__ amax) {
  constexpr int Cin = CIN, PT = 2;   // PT output pixels per thread: pix0 + t and pix0 + 256 + t
  typedef float f2 __attribute__((ext_vector_type(2)));
  __shared__ float4 so[256 * PT * 4];
  __shared__ float red[4];
  const int t = threadIdx.x, total = N * Ho * Wo;
  const int pix0 = blockIdx.x * 256 * PT;
  // all 9*CIN loads of both pixels issued unconditionally (clamped address,
  // zero selected afterwards): no exec-mask branch per tap
  f2 in[Cin * 9];
  bool live[PT];
#pragma unroll
  for (int u = 0; u < PT; ++u) {
    const int pix = pix0 + u * 256 + t;
    live[u] = pix < total;
    const int pc = live[u] ? pix : 0;
    const int n = pc / (Ho * Wo), r = pc - n * Ho * Wo, oy = r / Wo, ox = r - oy * Wo;
    const float* ib = img + (size_t)n * Cin * H * W;
#pragma unroll
    for (int c = 0; c < Cin; ++c)
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int iy = oy * 2 - 1 + ky, ix = ox * 2 - 1 + kx;
          const bool ok = live[u] && iy >= 0 && iy < H && ix >= 0 && ix < W;
          const float v = ib[((size_t)c * H + min(max(iy, 0), H - 1)) * W + min(max(ix, 0), W - 1)];
          in[c * 9 + ky * 3 + kx][u] = ok ? v : 0.f;
        }
  }
  // weights and bias at wave-uniform addresses (scalar loads); the two pixels
  // share each weight in one packed FMA
  f2 o[16];
  float m_abs[PT] = {0.f, 0.f};
#pragma unroll
  for (int co = 0; co < 16; ++co) {
    f2 a = f2{0.f, 0.f};
#pragma unroll
    for (int k = 0; k < Cin * 9; ++k) {
      const float wk = w[co * Cin * 9 + k];
      a = __builtin_elementwise_fma(in[k], f2{wk, wk}, a);
    }
#pragma unroll
    for (int u = 0; u < PT; ++u) {
      o[co][u] = kpd_act(a[u] + b[co], ACT_HSWISH);
      if (live[u]) m_abs[u] = fmaxf(m_abs[u], fabsf(o[co][u]));
    }
  }
  // stage the block's 512 x 64-byte outputs in LDS (XOR-swizzled quads), then
  // store them as one contiguous 32 KB run: each store instruction covers
  // 1 KB of consecutive addresses instead of a 16-byte piece of every 64
#pragma unroll
  for (int u = 0; u < PT; ++u) {
    const int lp = u * 256 + t;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      so[lp * 4 + (q ^ (lp & 3))] = make_float4(o[4 * q][u], o[4 * q + 1][u], o[4 * q + 2][u], o[4 * q + 3][u]);
  }
  __syncthreads();
  const int npx = min(256 * PT, total - pix0);
  float4* dst = reinterpret_cast<float4*>(out + (size_t)pix0 * 16);
#pragma unroll
  for (int q = 0; q < 4 * PT; ++q) {
    const int i = q * 256 + t, px = i >> 2, qq = i & 3;
    if (px < npx) dst[i] = so[px * 4 + (qq ^ (px & 3))];
  }
  if (amax) {   // per-image max|tap0| for the split FPN scale (conv_glds.hip, fpn0x_kernel)
    // the block's first image reduces over the workgroup; pixels of a later
    // image (a block straddling an image boundary) publish one by one
    const int HWo = Ho * Wo, nb = pix0 / HWo;
    float mb = 0.f;
#pragma unroll
    for (int u = 0; u < PT; ++u) {
      const int pix = pix0 + u * 256 + t;
      if (!live[u]) continue;
      const int n = pix / HWo;
      if (n == nb) mb = fmaxf(mb, m_abs[u]);
      else amax_publish_img(amax, n, m_abs[u]);
    }
    const float wm = wave_max(mb);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = wm;
    __syncthreads();
    if (threadIdx.x == 0) amax_publish_img(amax, nb, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
  }
}

// Depthwise KxK conv, stride S, "same" padding, + folded BN + act.  A thread
// owns 4 channels (one 16-byte quad) x XT consecutive output columns: each
// input column loaded feeds up to ceil(K/S) outputs from registers, so a 5x5
// stride-1 row costs 8 loads for 4 outputs instead of 20.
template <int K, int S, int XT = 4>
__global__ __launch_bounds__(256) void dwconv_kernel(const float* __restrict__ in, const float* __restrict__ w,
                                                     const float* __restrict__ b, float* __restrict__ out,
                                                     int N, int H, int W, int Cp, int Ho, int Wo, int act) {
  constexpr int P = (K - 1) / 2, NC = (XT - 1) * S + K;   // input columns per row
  const int nq = Cp >> 2, wx = (Wo + XT - 1) / XT;
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t total = (size_t)N * Ho * wx * nq;
  if (idx >= total) return;
  const int q = idx % nq;
  const size_t rest = idx / nq;
  const int xt = rest % wx;
  const int nr = rest / wx, n = nr / Ho, oy = nr - n * Ho, ox0 = xt * XT;
  const int ix0 = ox0 * S - P;
  float4 acc[XT];
#pragma unroll
  for (int o = 0; o < XT; ++o) acc[o] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int ky = 0; ky < K; ++ky) {
    const int iy = oy * S - P + ky;
    if (iy < 0 || iy >= H) continue;
    const float* row = in + ((size_t)(n * H + iy) * W) * Cp + q * 4;
    float4 col[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ix = ix0 + c;
      col[c] = (ix >= 0 && ix < W) ? *reinterpret_cast<const float4*>(row + (size_t)ix * Cp)
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int kx = 0; kx < K; ++kx) {
      const float4 k = *reinterpret_cast<const float4*>(w + (ky * K + kx) * Cp + q * 4);
#pragma unroll
      for (int o = 0; o < XT; ++o) {
        const float4 v = col[o * S + kx];
        acc[o].x = fmaf(v.x, k.x, acc[o].x); acc[o].y = fmaf(v.y, k.y, acc[o].y);
        acc[o].z = fmaf(v.z, k.z, acc[o].z); acc[o].w = fmaf(v.w, k.w, acc[o].w);
      }
    }
  }
  const float4 bb = *reinterpret_cast<const float4*>(b + q * 4);
  float* op = out + ((size_t)(n * Ho + oy) * Wo + ox0) * Cp + q * 4;
#pragma unroll
  for (int o = 0; o < XT; ++o) {
    if (ox0 + o >= Wo) break;
    float4 r;
    r.x = kpd_act(acc[o].x + bb.x, act); r.y = kpd_act(acc[o].y + bb.y, act);
    r.z = kpd_act(acc[o].z + bb.z, act); r.w = kpd_act(acc[o].w + bb.w, act);
    *reinterpret_cast<float4*>(op + (size_t)o * Cp) = r;
  }
}

// SE excitation from the channel means (in LDS): fc1 + ReLU, fc2 +
// hardsigmoid.  NT threads; the arithmetic order does not depend on NT (a
// row of fc1 is one wave's reduction, an output of fc2 one thread's chain).
// (A fused "last slice of the image runs the excitation" tail in exdw_kernel
// was measured and dropped: the device-scope fence it needs writes back the
// XCD's L2 and made the kernel 6x slower.)
template <int NT, int IPW>
__device__ __forceinline__ void se_fc(const float* mean, float* hid, int nimg, int C, int Cp,
                                      const float* __restrict__ w1, const float* __restrict__ b1,
                                      const float* __restrict__ w2t, const float* __restrict__ b2, int sq,
                                      float* __restrict__ scale) {
  // mean: [IPW][Cp] (LDS), hid: [IPW][256] (LDS), scale: [IPW][Cp] rows (global)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // (2) fc1 + ReLU: wave per output row, lanes split K with 16-byte loads;
  // up to 3 rows x 4 K-chunks (C <= 1024) issued before the reductions; each
  // weight load serves the IPW images
  const int nch = (C + 255) / 256;
  for (int j0 = wave * 3; j0 < sq; j0 += (NT / 64) * 3) {
    float acc[3][IPW];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int m = 0; m < IPW; ++m) acc[r][m] = 0.f;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int j = j0 + r;
      if (j < sq) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int c = t * 256 + lane * 4;
          if (t < nch && c < C) {
            const float4 wv = *reinterpret_cast<const float4*>(w1 + (size_t)j * C + c);
#pragma unroll
            for (int m = 0; m < IPW; ++m) {
              const float4 mv = *reinterpret_cast<const float4*>(mean + m * Cp + c);
              acc[r][m] = fmaf(wv.x, mv.x, fmaf(wv.y, mv.y, fmaf(wv.z, mv.z, fmaf(wv.w, mv.w, acc[r][m]))));
            }
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int m = 0; m < IPW; ++m) {
        const float v = wave_sum(acc[r][m]);
        if (lane == 0 && j0 + r < sq) hid[m * 256 + j0 + r] = fmaxf(v + b1[j0 + r], 0.f);
      }
  }
  __syncthreads();
  // (3) fc2 + hardsigmoid: thread per output over the transposed weights
  // (coalesced rows), K unrolled with two accumulators per image
  for (int c = tid; c < Cp; c += NT) {
    float a0[IPW], a1[IPW];
#pragma unroll
    for (int m = 0; m < IPW; ++m) a0[m] = a1[m] = 0.f;
    if (c < C) {
#pragma unroll 4
      for (int j = 0; j < sq; j += 2) {
        const float wa = w2t[(size_t)j * C + c], wb = w2t[(size_t)(j + 1) * C + c];
#pragma unroll
        for (int m = 0; m < IPW; ++m) {
          a0[m] = fmaf(wa, hid[m * 256 + j], a0[m]);
          a1[m] = fmaf(wb, hid[m * 256 + j + 1], a1[m]);
        }
      }
    }
#pragma unroll
    for (int m = 0; m < IPW; ++m)
      if (m < nimg) scale[(size_t)m * Cp + c] = c < C ? kpd_hsigmoid(a0[m] + a1[m] + b2[c]) : 0.f;
  }
}

// Fused MobileNetV3 inverted-residual front half for the coarse maps:
// expand 1x1 (+ folded BN + act) -> depthwise KxK stride S (+ folded BN + act)
// -> output, plus the per-image channel means the SE block needs and, when
// p.part is set, the SE fc1 partial products of this slice's channels
// (fc1 is linear in the means, so fc1(mean) = sum over slices of
// w1[:, slice] . mean[slice]; seproj_kernel finishes it).  One workgroup per
// (image, slice of CS = 16 * NTC expanded channels).  torchvision
// InvertedResidual (backbone.py:250-254 via mobilenet_v3_small).
//   * every weight / input load of a phase is issued before its first use
//     (register batches): the phases are latency chains, not throughput;
//   * expand on v_mfma_f32_16x16x4_f32 (exact fp32 products): A = 16 input
//     pixels x 16 channels of x straight from L2 (16 bytes per lane), B = the
//     slice's expand weights, kept in registers for all M tiles;
//   * the expanded slice lives in LDS only, rows padded to CS + 4 floats so the
//     depthwise's 16-byte reads of 4 column groups hit distinct banks;
//   * channel means reduced in a fixed order (deterministic, batch-independent).
// LDS row stride (floats) of the expanded slice: CS + 4 pads the depthwise's
// 16-byte reads apart; for the 32-channel stride-1 slices (features.10 / 11)
// 48, which a simulation of the ds_read_b128 lane groups (lanes {0-3, 12-15,
// 20-27}, {4-11, 16-19, 28-31} and + 32, MI355X_MICROARCH.md) over the
// kernel's item -> lane map shows conflict-free (36: 2.2-way average)
__host__ __device__ constexpr int exdw_estr(int CS, int S) { return CS == 32 && S == 1 ? 48 : CS + 4; }

// BL (the 576-channel blocks, features.10 / 11): the expand's B fragments come
// from LDS (staged by LDS-DMA with the first round trip, rows cin_p + 8 floats
// apart: conflict-free fragment reads) instead of 48 registers, and the fc1
// partial reads its weight columns from L2 instead of an LDS copy, so that
// five workgroups fit a CU (LDS <= 32 KB, VGPRs <= 96): the launch's 1,152
// workgroups in one round instead of two
// ACT >= 0: both activations that compile-time constant (the runtime switch
// of kpd_act costs a branch tree per element), else p.act_e / p.act_d
template <int K, int S, int NTC, int XT, int KC, bool BL = false, int ACT = -1>
__global__ __launch_bounds__(256) void exdw_kernel(const ExDwArgs p) {
  const int act_e = ACT >= 0 ? ACT : p.act_e, act_d = ACT >= 0 ? ACT : p.act_d;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  // KC = cin_p / 16 k chunks; DA = M tiles whose A loads are in flight per wave
  constexpr int CS = 16 * NTC, CQ = CS / 4, ESTR = exdw_estr(CS, S), DA = KC <= 3 ? 4 : 1, WBS = 16 * KC + 8;
  const int n = blockIdx.y, c0 = blockIdx.x * CS, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int PD = (K - 1) / 2;
  // row band (blockIdx.z of gridDim.z; no SE): output rows [oy0, oy1), from
  // input rows [iy_lo, iy_hi) -- the depthwise halo rows are expanded by both
  // neighbouring bands
  const int oy0 = blockIdx.z * p.Ho / gridDim.z, oy1 = (blockIdx.z + 1) * p.Ho / gridDim.z;
  const int iy_lo = max(0, oy0 * S - PD), iy_hi = min(p.Hi, (oy1 - 1) * S - PD + K);
  const int Pin = (iy_hi - iy_lo) * p.Wi, Po = p.Ho * p.Wo, cin_p = p.cin_p;
  float* es = sm;                                  // [Pin][ESTR]
  float* wds = es + Pin * ESTR;                    // [K*K][CS] depthwise weights, then [CS] its bias
  float* ds = wds + (K * K + 1) * CS;              // [Po][CS] (pooled)
  float* w1s = ds + (p.pooled ? Po * CS : 0);      // [sq][CS] (part; BL: [CS][WBS] expand weights)
  const float* xg = p.x + ((size_t)n * p.Hi + iy_lo) * p.Wi * cin_p;
  stamp(p.stamps, 0);
  const int r = lane & 15, g = lane >> 4;
  const int nmt = (Pin + 15) / 16, ntw = (nmt - wave + 3) / 4;   // M tiles of this wave: wave + 4 t
  // one round trip for everything the expand needs: B fragments (all k
  // chunks, all N tiles) and the first DA M tiles' A fragments -> registers,
  // then the depthwise weights and the fc1 columns -> LDS
  float4 bw[BL ? 1 : NTC][BL ? 1 : KC];
  if constexpr (!BL) {
#pragma unroll
    for (int nt = 0; nt < NTC; ++nt)
#pragma unroll
      for (int kc = 0; kc < KC; ++kc)
        bw[nt][kc] = *reinterpret_cast<const float4*>(p.we + (size_t)(c0 + nt * 16 + r) * cin_p + kc * 16 + g * 4);
  } else {
    // the slice's expand weight rows by LDS-DMA: 16-byte piece e of [CS][WBS]
    // is row e / (WBS / 4), column piece e % (WBS / 4) (the last two: padding)
    const i32x4 rwe = make_rsrc(p.we + (size_t)c0 * cin_p, CS * cin_p * 4);
    const unsigned wb_lds = lds_addr(w1s);
    constexpr int NPR = WBS / 4, NPC = (CS * NPR + 63) / 64;
    for (int i = wave; i < NPC; i += 4) {
      const int e = i * 64 + lane, row = e / NPR, cp = e - row * NPR;
      const unsigned voff = (row < CS && cp < 4 * KC) ? (unsigned)((row * cin_p + cp * 4) * 4) : 0x80000000u;
      glds16(rwe, __builtin_amdgcn_readfirstlane(wb_lds + i * 1024), voff, 0);
    }
  }
  float be[NTC];   // expand bias, loaded with the first round trip
#pragma unroll
  for (int nt = 0; nt < NTC; ++nt) be[nt] = p.be[c0 + nt * 16 + r];
  float4 av[DA][KC];
  auto load_a = [&](int t, float4* a4) {
    if (t < ntw) {
      const int px = min((wave + 4 * t) * 16 + r, Pin - 1);
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) a4[kc] = *reinterpret_cast<const float4*>(xg + (size_t)px * cin_p + kc * 16 + g * 4);
    }
  };
#pragma unroll
  for (int d = 0; d < DA; ++d) load_a(d, av[d]);
  {
    // the depthwise weights and (row K*K) its bias
    constexpr int NW = ((K * K + 1) * CQ + 255) / 256;
    float4 v[NW];
#pragma unroll
    for (int u = 0; u < NW; ++u) {
      const int i = tid + u * 256, t = i / CQ, q = i - t * CQ;
      if (i < K * K * CQ) v[u] = *reinterpret_cast<const float4*>(p.wd + (size_t)t * p.Ep + c0 + q * 4);
      else if (i < (K * K + 1) * CQ) v[u] = *reinterpret_cast<const float4*>(p.bd + c0 + q * 4);
    }
    // the fc1 columns by LDS-DMA (no registers; waited for after the expand):
    // 16-byte piece e of w1s = [sq][CS] is w1[j][c0 + 4 q], e = j * CQ + q,
    // padding channels (>= C) load zeros through the range check
    if (!BL && p.part) {
      const i32x4 rw1 = make_rsrc(p.w1, p.sq * p.C * 4);
      const unsigned w1s_lds = lds_addr(w1s);
      const int npc = (p.sq * CQ + 63) / 64;   // wave-instructions (1 KiB each)
      for (int i = wave; i < npc; i += 4) {
        const int e = i * 64 + lane, j = e / CQ, q = e - j * CQ;
        const unsigned voff = (j < p.sq && c0 + q * 4 < p.C) ? (unsigned)((j * p.C + c0 + q * 4) * 4) : 0x80000000u;
        glds16(rw1, __builtin_amdgcn_readfirstlane(w1s_lds + i * 1024), voff, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < NW; ++u) {
      const int i = tid + u * 256;
      if (i < (K * K + 1) * CQ) reinterpret_cast<float4*>(wds)[i] = v[u];
    }
  }
  if constexpr (BL) {   // the expand weights' DMA landed (every wave's pieces)
    wait_vmcnt<0>();
    __syncthreads();
  }
  stamp(p.stamps, 1);
  // expand: DA M tiles of A in flight per wave; a tile's slot is refilled
  // with the tile DA ahead right after its MFMAs
  {
    for (int t0 = 0; t0 < ntw; t0 += DA) {
#pragma unroll
      for (int d = 0; d < DA; ++d) {
        const int t = t0 + d;
        if (t < ntw) {
          f32x4 acc[NTC];
#pragma unroll
          for (int nt = 0; nt < NTC; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kc = 0; kc < KC; ++kc)
#pragma unroll
            for (int nt = 0; nt < NTC; ++nt) {
              const float4 b4 = BL ? *reinterpret_cast<const float4*>(w1s + (nt * 16 + r) * WBS + kc * 16 + g * 4)
                                   : bw[BL ? 0 : nt][BL ? 0 : kc];
              acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[d][kc].x, b4.x, acc[nt], 0, 0, 0);
              acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[d][kc].y, b4.y, acc[nt], 0, 0, 0);
              acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[d][kc].z, b4.z, acc[nt], 0, 0, 0);
              acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[d][kc].w, b4.w, acc[nt], 0, 0, 0);
            }
          load_a(t + DA, av[d]);
          // C layout: col = lane & 15 (channel), row = 4 * (lane >> 4) + i (pixel)
          const int mt = wave + 4 * t;
#pragma unroll
          for (int nt = 0; nt < NTC; ++nt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int px = mt * 16 + g * 4 + i;
              if (px < Pin) es[px * ESTR + nt * 16 + r] = kpd_act(acc[nt][i] + be[nt], act_e);
            }
        }
      }
    }
  }
  if (!BL && p.part) wait_vmcnt<0>();   // the fc1-column DMA (issued at the start; long landed)
  __syncthreads();
  stamp(p.stamps, 2);
  // depthwise from LDS, XT consecutive output columns per thread (input
  // columns reused from registers as in dwconv_kernel)
  constexpr int NC = (XT - 1) * S + K;
  const int wx = (p.Wo + XT - 1) / XT;
  for (int i = tid; i < (oy1 - oy0) * wx * CQ; i += 256) {
    const int q = i % CQ, rr = i / CQ, xt = rr % wx, oy = oy0 + rr / wx, ox0 = xt * XT, ix0 = ox0 * S - PD;
    float4 a[XT];
#pragma unroll
    for (int o = 0; o < XT; ++o) a[o] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      const int iy = oy * S - PD + ky;
      if (iy < 0 || iy >= p.Hi) continue;
      float4 col[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int ix = ix0 + c;
        col[c] = (ix >= 0 && ix < p.Wi) ? *reinterpret_cast<const float4*>(es + ((iy - iy_lo) * p.Wi + ix) * ESTR + q * 4)
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int kx = 0; kx < K; ++kx) {
        const float4 w = reinterpret_cast<const float4*>(wds)[(ky * K + kx) * CQ + q];
#pragma unroll
        for (int o = 0; o < XT; ++o) {
          const float4 v = col[o * S + kx];
          a[o].x = fmaf(v.x, w.x, a[o].x); a[o].y = fmaf(v.y, w.y, a[o].y);
          a[o].z = fmaf(v.z, w.z, a[o].z); a[o].w = fmaf(v.w, w.w, a[o].w);
        }
      }
    }
    const float4 b = reinterpret_cast<const float4*>(wds)[K * K * CQ + q];
#pragma unroll
    for (int o = 0; o < XT; ++o) {
      if (ox0 + o >= p.Wo) break;
      float4 v;
      v.x = kpd_act(a[o].x + b.x, act_d); v.y = kpd_act(a[o].y + b.y, act_d);
      v.z = kpd_act(a[o].z + b.z, act_d); v.w = kpd_act(a[o].w + b.w, act_d);
      const int op = oy * p.Wo + ox0 + o;
      *reinterpret_cast<float4*>(p.out + ((size_t)n * Po + op) * p.Ep + c0 + q * 4) = v;
      if (p.pooled) reinterpret_cast<float4*>(ds)[op * CQ + q] = v;
    }
  }
  if (p.pooled) {   // channel means: 256/CS row groups in parallel, then a fixed-order combine
    __syncthreads();
    stamp(p.stamps, 3);
    constexpr int groups = 256 / CS;
    const int c = tid % CS, gg0 = tid / CS;
    float sum = 0.f;
    for (int op = gg0; op < Po; op += groups) sum += ds[op * CS + c];
    __syncthreads();
    ds[gg0 * CS + c] = sum;
    __syncthreads();
    if (tid < CS) {
      float t = 0.f;
#pragma unroll
      for (int gg = 0; gg < groups; ++gg) t += ds[gg * CS + tid];
      t /= (float)Po;
      p.pooled[(size_t)n * p.Ep + c0 + tid] = t;
      ds[tid] = t;   // column tid of ds is read only by this thread above
    }
    if (p.part) {   // SE fc1 partial of this slice, one output row per thread
      __syncthreads();
      const int nsl = gridDim.x;
      for (int j = tid; j < p.sq; j += 256) {
        float acc = 0.f;
        if constexpr (BL) {   // the fc1 columns from L2 (padding channels: zero weights)
          float4 w4[CQ];
#pragma unroll
          for (int q = 0; q < CQ; ++q)
            w4[q] = c0 + 4 * q < p.C ? *reinterpret_cast<const float4*>(p.w1 + (size_t)j * p.C + c0 + 4 * q)
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int q = 0; q < CQ; ++q) {
            acc = fmaf(w4[q].x, ds[4 * q + 0], acc);
            acc = fmaf(w4[q].y, ds[4 * q + 1], acc);
            acc = fmaf(w4[q].z, ds[4 * q + 2], acc);
            acc = fmaf(w4[q].w, ds[4 * q + 3], acc);
          }
        } else {
#pragma unroll
          for (int c2 = 0; c2 < CS; ++c2) acc = fmaf(w1s[j * CS + c2], ds[c2], acc);
        }
        p.part[((size_t)n * nsl + blockIdx.x) * p.sq + j] = acc;
      }
    }
  }
  stamp(p.stamps, 4);
}

// Squeeze-excitation excitation + project 1x1 (+ residual) for the coarse
// maps (features.4..11 of mobilenet_v3_small; torchvision SqueezeExcitation +
// InvertedResidual, backbone.py:250-254).  One workgroup per (image, NTT*16
// output channels):
//   hid = ReLU(b1 + sum over slices of exdw_kernel's fc1 partials)  (fixed order)
//   s   = hardsigmoid(b2 + W2 . hid)                                  (all Ep channels, LDS)
//   out = (d * s) . Wp^T + bp (+ x)
// (with a.sesc set, s comes precomputed from se_excite_kernel instead).
// The project GEMM runs on v_mfma_f32_16x16x4_f32 (exact fp32 products): each
// lane loads 16 bytes of a d row and of a Wp row per 16-wide k chunk and feeds
// them to 4 MFMAs (k-step t takes element t; A and B use the same k
// permutation).  The 4 waves split the k chunks; their partial tiles are summed
// in LDS in wave order (deterministic, independent of the batch).  The first
// D chunks' loads do not depend on s and are issued before the excitation, so
// their latency hides under it; each chunk's slot is refilled D chunks ahead.
template <int MT, int NTT, int NWV = 4>
__global__ __launch_bounds__(NWV * 64) void seproj_kernel(const SeProjArgs a) {
  constexpr int NTH = NWV * 64;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr int NT = NTT * 16, MP = MT * 16;
  constexpr int D = (28 / (MT + NTT)) < 1 ? 1 : ((28 / (MT + NTT)) > 4 ? 4 : 28 / (MT + NTT));
  const int n = blockIdx.y, o0 = blockIdx.x * NT, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int Ep = a.Ep, Po = a.Po;
  float* sS = sm;                    // [Ep] excitation
  float* hid = sS + Ep;              // [256]
  float* red = hid + 256;            // [NWV][MP][NT] partial tiles / SE scratch
  stamp(a.stamps, 0);
  const int r = lane & 15, g = lane >> 4;
  // rows of this workgroup: [m0, m0 + MP) of the image (blockIdx.z splits M)
  const int m0 = blockIdx.z * MP, Pr = min(MP, Po - m0);
  const float* dbase = a.d + ((size_t)n * Po + m0) * Ep;
  const int nkc = Ep / 16, ncw = (nkc - wave + NWV - 1) / NWV;   // this wave's k chunks: wave + NWV t
  // the excitation's biases with the first round trip (loaded behind its
  // barriers they were two more dependent round trips)
  const float b1v = a.sesc ? 0.f : a.b1[min(tid, a.sq - 1)];
  constexpr int NB2 = 1024 / NTH;   // Ep <= 1024
  float b2v[NB2];
#pragma unroll
  for (int u = 0; u < NB2; ++u) b2v[u] = a.sesc ? 0.f : a.b2[min(tid + u * NTH, a.C - 1)];
  float4 av[D][MT], bv[D][NTT];
  auto load_chunk = [&](int t, float4* a4, float4* b4) {
    if (t < ncw) {
      const int k = (wave + NWV * t) * 16 + g * 4;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int px = mt * 16 + r;
        a4[mt] = px < Pr ? *reinterpret_cast<const float4*>(dbase + (size_t)px * Ep + k) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int nt = 0; nt < NTT; ++nt) b4[nt] = *reinterpret_cast<const float4*>(a.wp + (size_t)(o0 + nt * 16 + r) * Ep + k);
    }
  };
#pragma unroll
  for (int dd = 0; dd < D; ++dd) load_chunk(dd, av[dd], bv[dd]);
  if (a.sesc) {   // precomputed excitation
    for (int c = tid; c < Ep / 4; c += NTH)
      reinterpret_cast<float4*>(sS)[c] = reinterpret_cast<const float4*>(a.sesc + (size_t)n * Ep)[c];
    __syncthreads();
  } else {
    // (1) hid = ReLU(b1 + sum of the slice partials): the image's partials
    // staged in LDS first (all loads in flight), then summed in slice order
    const int npart = a.nsl * a.sq;
    const float* part = a.part + (size_t)n * npart;
    {
      constexpr int NP = 6 * 256 / NTH;   // npart / 4 <= 1536 (kSePartFloats / 4 / ... checked at launch)
      float4 v[NP];
#pragma unroll
      for (int u = 0; u < NP; ++u)   // clamped (unconditional) loads keep v in registers
        v[u] = reinterpret_cast<const float4*>(part)[min(tid + u * NTH, npart / 4 - 1)];
#pragma unroll
      for (int u = 0; u < NP; ++u) {
        const int i = tid + u * NTH;
        if (i < npart / 4) reinterpret_cast<float4*>(red)[i] = v[u];
      }
    }
    __syncthreads();
    if (tid < a.sq) {   // (sq <= 144 <= NTH)
      float h = 0.f;
      for (int s2 = 0; s2 < a.nsl; ++s2) h += red[s2 * a.sq + tid];
      hid[tid] = fmaxf(h + b1v, 0.f);
    }
    __syncthreads();
    stamp(a.stamps, 1);
    // (2) s = hardsigmoid(b2 + W2 . hid), W2 transposed [sq][C]: a work item is
    // (channel quad, j group); the group's rows are loaded together (16-byte
    // loads), the j groups' partial sums meet in LDS in group order
    {
      const int nq4 = a.C / 4, ngrp = max(1, min(16, 256 / nq4)), items = nq4 * ngrp;
      const int jper = (a.sq + ngrp - 1) / ngrp;
      float* fsum = red;   // [ngrp][C]
      for (int it = tid; it < items; it += NTH) {
        const int q = it % nq4, gi = it / nq4, j0 = gi * jper, j1 = min(a.sq, j0 + jper);
        float4 acc4 = make_float4(0.f, 0.f, 0.f, 0.f);
        constexpr int JU = 16;
        for (int j = j0; j < j1; j += JU) {
          float4 wv[JU];
#pragma unroll
          for (int u = 0; u < JU; ++u)
            if (j + u < j1) wv[u] = *reinterpret_cast<const float4*>(a.w2t + (size_t)(j + u) * a.C + q * 4);
#pragma unroll
          for (int u = 0; u < JU; ++u)
            if (j + u < j1) {
              const float h = hid[j + u];
              acc4.x = fmaf(wv[u].x, h, acc4.x); acc4.y = fmaf(wv[u].y, h, acc4.y);
              acc4.z = fmaf(wv[u].z, h, acc4.z); acc4.w = fmaf(wv[u].w, h, acc4.w);
            }
        }
        reinterpret_cast<float4*>(fsum + (size_t)gi * a.C)[q] = acc4;
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < NB2; ++u) {
        const int c = tid + u * NTH;
        if (c >= Ep) break;
        float t = 0.f;
        if (c < a.C)
          for (int gi = 0; gi < ngrp; ++gi) t += fsum[(size_t)gi * a.C + c];
        sS[c] = c < a.C ? kpd_hsigmoid(t + b2v[u]) : 0.f;
      }
      __syncthreads();
    }
  }
  stamp(a.stamps, 2);
  // the epilogue's bias and residual quads, loaded before the K loop (their
  // latency hides under it instead of ending the workgroup)
  constexpr int NQ = NT / 4, IT = (MP * NQ + NTH - 1) / NTH;
  float4 ep_b[IT], ep_r[IT];
  {
    const float* res0 = a.res ? a.res + ((size_t)n * Po + m0) * a.cout_p + o0 : nullptr;
#pragma unroll
    for (int u = 0; u < IT; ++u) {
      const int i = min(tid + u * NTH, Pr * NQ - 1), px = i / NQ, q = i - px * NQ;
      ep_b[u] = *reinterpret_cast<const float4*>(a.bp + o0 + q * 4);
      ep_r[u] = res0 ? *reinterpret_cast<const float4*>(res0 + (size_t)px * a.cout_p + q * 4)
                     : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  // (3) project on MFMA
  f32x4 acc[MT][NTT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NTT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int t0 = 0; t0 < ncw; t0 += D) {
#pragma unroll
    for (int dd = 0; dd < D; ++dd) {
      const int t = t0 + dd;
      if (t < ncw) {
        const float4 sv = *reinterpret_cast<const float4*>(sS + (wave + NWV * t) * 16 + g * 4);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const float4 x4 = make_float4(av[dd][mt].x * sv.x, av[dd][mt].y * sv.y, av[dd][mt].z * sv.z,
                                        av[dd][mt].w * sv.w);
#pragma unroll
          for (int nt = 0; nt < NTT; ++nt) {
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(x4.x, bv[dd][nt].x, acc[mt][nt], 0, 0, 0);
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(x4.y, bv[dd][nt].y, acc[mt][nt], 0, 0, 0);
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(x4.z, bv[dd][nt].z, acc[mt][nt], 0, 0, 0);
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(x4.w, bv[dd][nt].w, acc[mt][nt], 0, 0, 0);
          }
        }
        load_chunk(t + D, av[dd], bv[dd]);
      }
    }
  }
  __syncthreads();   // (red held the SE scratch)
  // partial tiles -> LDS (C layout: col = lane & 15, row = 4 * (lane >> 4) + i)
  float* rw = red + (size_t)wave * MP * NT;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NTT; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) rw[(mt * 16 + g * 4 + i) * NT + nt * 16 + r] = acc[mt][nt][i];
  __syncthreads();
  stamp(a.stamps, 3);
  // (4) sum the NWV waves in order, bias, residual; 4 channels per thread
  float* out = a.out + ((size_t)n * Po + m0) * a.cout_p + o0;
#pragma unroll
  for (int u = 0; u < IT; ++u) {
    const int i = tid + u * NTH;
    if (i >= Pr * NQ) break;
    const int px = i / NQ, q = i - px * NQ;
    float4 v = *reinterpret_cast<const float4*>(red + px * NT + q * 4);
#pragma unroll
    for (int w = 1; w < NWV; ++w) {
      const float4 t = *reinterpret_cast<const float4*>(red + ((size_t)w * MP + px) * NT + q * 4);
      v.x += t.x; v.y += t.y; v.z += t.z; v.w += t.w;
    }
    const float4 b = ep_b[u];
    v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
    if (a.res) {
      const float4 x = ep_r[u];
      v.x += x.x; v.y += x.y; v.z += x.z; v.w += x.w;
    }
    *reinterpret_cast<float4*>(out + (size_t)px * a.cout_p + q * 4) = v;
  }
  stamp(a.stamps, 4);
}

// SE excitation for the wide blocks (features.9..11, C >= 288, whose fc2 is
// too large to recompute in every project workgroup): one workgroup per
// (image, 64 channels).  The image's fc1 partials and the 64-column slice of
// W2 are loaded in one round trip; hid is summed in slice order, the slice's
// excitation in j-group order (deterministic).  Writes sesc [N][Ep].
__global__ __launch_bounds__(256) void se_excite_kernel(const SeProjArgs a, float* __restrict__ sesc) {
  __shared__ __attribute__((aligned(16))) float spart[kSeExcitePart];
  __shared__ float hid[256];
  __shared__ __attribute__((aligned(16))) float fsum[16 * 64];
  const int n = blockIdx.y, c0 = blockIdx.x * 64, tid = threadIdx.x;
  const int npart = a.nsl * a.sq;
  const float* part = a.part + (size_t)n * npart;
  // work item: thread (q = channel quad of 16, grp = j group of 16)
  const int q = tid & 15, grp = tid >> 4, jper = (a.sq + 15) / 16, j0 = grp * jper, j1 = min(a.sq, j0 + jper);
  const bool qlive = c0 + q * 4 < a.C;
  // the biases with the first round trip (behind the barriers they were two
  // more dependent round trips)
  const float b1v = a.b1[min(tid, a.sq - 1)], b2v = a.b2[min(c0 + tid, a.C - 1)];
  constexpr int JMAX = 9;   // sq <= 144
  float4 wv[JMAX];
#pragma unroll
  for (int u = 0; u < JMAX; ++u)
    if (qlive && j0 + u < j1) wv[u] = *reinterpret_cast<const float4*>(a.w2t + (size_t)(j0 + u) * a.C + c0 + q * 4);
  {
    constexpr int NP = kSeExcitePart / 4 / 256;
    float4 v[NP];
#pragma unroll
    for (int u = 0; u < NP; ++u)   // clamped (unconditional) loads keep v in registers
      v[u] = reinterpret_cast<const float4*>(part)[min(tid + u * 256, npart / 4 - 1)];
#pragma unroll
    for (int u = 0; u < NP; ++u) {
      const int i = tid + u * 256;
      if (i < npart / 4) reinterpret_cast<float4*>(spart)[i] = v[u];
    }
  }
  __syncthreads();
  if (tid < a.sq) {   // (sq <= 144)
    float h = 0.f;
    for (int s2 = 0; s2 < a.nsl; ++s2) h += spart[s2 * a.sq + tid];
    hid[tid] = fmaxf(h + b1v, 0.f);
  }
  __syncthreads();
  float4 acc4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int u = 0; u < JMAX; ++u)
    if (qlive && j0 + u < j1) {
      const float h = hid[j0 + u];
      acc4.x = fmaf(wv[u].x, h, acc4.x); acc4.y = fmaf(wv[u].y, h, acc4.y);
      acc4.z = fmaf(wv[u].z, h, acc4.z); acc4.w = fmaf(wv[u].w, h, acc4.w);
    }
  reinterpret_cast<float4*>(fsum)[grp * 16 + q] = acc4;
  __syncthreads();
  if (tid < 64) {
    const int c = c0 + tid;
    float t = 0.f;
#pragma unroll
    for (int gi = 0; gi < 16; ++gi) t += fsum[gi * 64 + tid];
    if (c < a.Ep) sesc[(size_t)n * a.Ep + c] = c < a.C ? kpd_hsigmoid(t + b2v) : 0.f;
  }
}

// The narrow SE block without expand (features.1 of mobilenet_v3_small:
// 16 -> 16 channels, depthwise 3x3 stride 2 + ReLU, SE 16 -> 8 -> 16,
// project 1x1, no residual; torchvision InvertedResidual via backbone.py:
// 250-254) in two launches instead of three:
//   dwsum_kernel: depthwise on tiles of TH output rows x the full width of one
//     image, plus the tile's per-channel sums (fixed order) for the squeeze;
//   se16_proj_kernel: the excitation from those partial sums (every workgroup
//     recomputes it: 16 x 8 x 2 MACs) and the project 1x1 with the excitation
//     applied to its input, one pixel per thread.
constexpr int kDwsTH = 4;   // output rows per dwsum workgroup
template <int K, int S, int ACT = -1>   // ACT >= 0: the activation as a compile-time constant
__global__ __launch_bounds__(256) void dwsum_kernel(const float* __restrict__ in, int Hi, int Wi,
                                                    const float* __restrict__ w, const float* __restrict__ b, int act_rt,
                                                    float* __restrict__ out, int Ho, int Wo,
                                                    float* __restrict__ part) {
  constexpr int C = 16, CQ = 4, XT = 4, P = (K - 1) / 2, NC = (XT - 1) * S + K;
  const int act = ACT >= 0 ? ACT : act_rt;
  __shared__ float4 red[256];
  const int n = blockIdx.y, tile = blockIdx.x, tid = threadIdx.x;
  const int wx = (Wo + XT - 1) / XT, units = kDwsTH * wx * CQ;
  const int q = tid % CQ, rest = tid / CQ, xt = rest % wx, orow = rest / wx;
  const int oy = tile * kDwsTH + orow, ox0 = xt * XT, ix0 = ox0 * S - P;
  float4 sum = make_float4(0.f, 0.f, 0.f, 0.f);
  if (tid < units && oy < Ho) {
    float4 acc[XT];
#pragma unroll
    for (int o = 0; o < XT; ++o) acc[o] = make_float4(0.f, 0.f, 0.f, 0.f);
    // row by row (36 VGPRs of inputs): occupancy hides the load latency
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      const int iy = oy * S - P + ky;
      if (iy < 0 || iy >= Hi) continue;
      float4 col[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int ix = ix0 + c;
        col[c] = (ix >= 0 && ix < Wi) ? *reinterpret_cast<const float4*>(in + (((size_t)n * Hi + iy) * Wi + ix) * C + q * 4)
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int kx = 0; kx < K; ++kx) {
        const float4 k4 = *reinterpret_cast<const float4*>(w + (ky * K + kx) * C + q * 4);
#pragma unroll
        for (int o = 0; o < XT; ++o) {
          const float4 v = col[o * S + kx];
          acc[o].x = fmaf(v.x, k4.x, acc[o].x); acc[o].y = fmaf(v.y, k4.y, acc[o].y);
          acc[o].z = fmaf(v.z, k4.z, acc[o].z); acc[o].w = fmaf(v.w, k4.w, acc[o].w);
        }
      }
    }
    const float4 bb = *reinterpret_cast<const float4*>(b + q * 4);
    float* op = out + (((size_t)n * Ho + oy) * Wo + ox0) * C + q * 4;
#pragma unroll
    for (int o = 0; o < XT; ++o) {
      if (ox0 + o >= Wo) break;
      float4 r;
      r.x = kpd_act(acc[o].x + bb.x, act); r.y = kpd_act(acc[o].y + bb.y, act);
      r.z = kpd_act(acc[o].z + bb.z, act); r.w = kpd_act(acc[o].w + bb.w, act);
      *reinterpret_cast<float4*>(op + (size_t)o * C) = r;
      sum.x += r.x; sum.y += r.y; sum.z += r.z; sum.w += r.w;
    }
  }
  // tile channel sums: the 16 lanes of a wave that share a quad (lane bits
  // 2-5) by xor shuffles, then the 4 waves in order (fixed order throughout)
#pragma unroll
  for (int o = 4; o < 64; o <<= 1) {
    sum.x += __shfl_xor(sum.x, o); sum.y += __shfl_xor(sum.y, o);
    sum.z += __shfl_xor(sum.z, o); sum.w += __shfl_xor(sum.w, o);
  }
  if ((tid & 63) < CQ) red[(tid >> 6) * CQ + (tid & 63)] = sum;
  __syncthreads();
  if (tid < C) {
    const int cq = tid >> 2, e = tid & 3;
    float t = 0.f;
#pragma unroll
    for (int wv = 0; wv < 4; ++wv) {
      const float4 v = red[wv * CQ + cq];
      t += e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w;
    }
    part[((size_t)n * gridDim.x + tile) * C + tid] = t;
  }
}

__global__ __launch_bounds__(256) void se16_proj_kernel(const float* __restrict__ d, int npx, int ntiles,
                                                        const float* __restrict__ part, const float* __restrict__ w1,
                                                        const float* __restrict__ b1, const float* __restrict__ w2t,
                                                        const float* __restrict__ b2, int sq,
                                                        const float* __restrict__ wp, const float* __restrict__ bp,
                                                        float* __restrict__ out) {
  constexpr int C = 16;
  __shared__ float mean[C], hid[16], sc[C], wps[C * C], bps[C], w1s[16 * C], w2s[16 * C], b1s[16], b2s[C];
  const int n = blockIdx.y, tid = threadIdx.x;
  const int px = blockIdx.x * 256 + tid;
  // this thread's pixel first (its latency overlaps the excitation)
  float4 v[4];
  const bool live = px < npx;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    v[k] = reinterpret_cast<const float4*>(d + ((size_t)n * npx + min(px, npx - 1)) * C)[k];
  // the image's tile partials (ntiles x 16 <= 1024 floats) staged in one load
  // round trip, then summed in tile order
  __shared__ float sp[1024];
  {
    const float* pp = part + (size_t)n * ntiles * C;
    float t4[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) t4[u] = pp[min(tid + u * 256, ntiles * C - 1)];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (tid + u * 256 < ntiles * C) sp[tid + u * 256] = t4[u];
  }
  // every weight of the excitation and the projection in the same round trip
  // (loaded lazily they were two more dependent round trips behind barriers)
  if (tid < C * C) wps[tid] = wp[tid];
  if (tid < C) bps[tid] = bp[tid];
  if (tid < sq * C) {
    w1s[tid] = w1[tid];
    w2s[tid] = w2t[tid];
  }
  if (tid < sq) b1s[tid] = b1[tid];
  if (tid < C) b2s[tid] = b2[tid];
  __syncthreads();
  if (tid < C) {
    float t = 0.f;
    for (int i = 0; i < ntiles; ++i) t += sp[i * C + tid];
    mean[tid] = t / (float)npx;
  }
  __syncthreads();
  if (tid < sq) {
    float a = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) a = fmaf(w1s[tid * C + c], mean[c], a);
    hid[tid] = fmaxf(a + b1s[tid], 0.f);
  }
  __syncthreads();
  if (tid < C) {
    float a = 0.f;
    for (int j = 0; j < sq; ++j) a = fmaf(w2s[j * C + tid], hid[j], a);
    sc[tid] = kpd_hsigmoid(a + b2s[tid]);
  }
  __syncthreads();
  if (!live) return;
  float x[C];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    x[4 * k] = v[k].x * sc[4 * k]; x[4 * k + 1] = v[k].y * sc[4 * k + 1];
    x[4 * k + 2] = v[k].z * sc[4 * k + 2]; x[4 * k + 3] = v[k].w * sc[4 * k + 3];
  }
  float o[C];
#pragma unroll
  for (int co = 0; co < C; ++co) {
    float a = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) a = fmaf(x[c], wps[co * C + c], a);
    o[co] = a + bps[co];
  }
  float4* op = reinterpret_cast<float4*>(out + ((size_t)n * npx + px) * C);
#pragma unroll
  for (int k = 0; k < 4; ++k) op[k] = make_float4(o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]);
}

// Small-K 1x1 conv (cin_p <= 96, cout_p % 64 == 0) + bias + act (+ nearest-
// upsampled residual, + max|out|): the FPN laterals 1 / 2 (backbone.py:33-37,
// top-down add) and features.12 (the last 96 -> 576 conv).  The generic
// implicit-GEMM kernel stages through LDS and pays a K-loop prologue for a
// single K-tile; here every operand goes straight from L2 to MFMA fragments
// in one load round trip.  Workgroup = 64 pixels x 64 output channels; wave w
// owns pixels 16w..16w+15 and all four 16-channel tiles.  fp32 operands on
// v_mfma_f32_16x16x4_f32 (exact products), k-step t of a 16-wide chunk takes
// element t of each lane's 16-byte load (same permutation for A and B).
constexpr int kPwKC = 6;   // 16-wide k chunks (cin_p <= 96)
template <int ACT = -1>   // ACT >= 0: the activation as a compile-time constant (features.12: hardswish)
__global__ __launch_bounds__(256) void pw_small_kernel(const ConvArgs a) {
  const int act = ACT >= 0 ? ACT : a.act;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  const int m0 = blockIdx.x * 64 + wave * 16, n0 = blockIdx.y * 64;
  const int nkc = a.cin_p / 16, M = a.M;
  const float* x = static_cast<const float*>(a.in);
  const float* w = static_cast<const float*>(a.wt);
  float4 av[kPwKC], bv[4][kPwKC];
  const int pa = min(m0 + r, M - 1);
#pragma unroll
  for (int kc = 0; kc < kPwKC; ++kc)
    av[kc] = kc < nkc ? *reinterpret_cast<const float4*>(x + (size_t)pa * a.in_cstride + kc * 16 + g * 4)
                      : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int kc = 0; kc < kPwKC; ++kc)
      bv[nt][kc] = kc < nkc ? *reinterpret_cast<const float4*>(w + (size_t)(n0 + nt * 16 + r) * a.cin_p + kc * 16 + g * 4)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
  // epilogue inputs issued before the MFMAs: bias, and the residual rows
  float bias[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) bias[nt] = a.bias[n0 + nt * 16 + r];
  const int HW = a.H * a.W;
  float resv[4][4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) resv[nt][i] = 0.f;
  if (a.res) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = min(m0 + g * 4 + i, M - 1);
      const int n = m / HW, rr = m - n * HW, y = rr / a.W, xx = rr - y * a.W;
      int sy = y, sx = xx;
      if (a.rh != a.H) sy = min((int)floorf((float)y * ((float)a.rh / (float)a.H)), a.rh - 1);
      if (a.rw != a.W) sx = min((int)floorf((float)xx * ((float)a.rw / (float)a.W)), a.rw - 1);
      const float* rp = a.res + ((size_t)(n * a.rh + sy) * a.rw + sx) * a.cout_p + n0 + r;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) resv[nt][i] = rp[nt * 16];
    }
  }
  f32x4 acc[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kc = 0; kc < kPwKC; ++kc)
    if (kc < nkc) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kc].x, bv[nt][kc].x, acc[nt], 0, 0, 0);
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kc].y, bv[nt][kc].y, acc[nt], 0, 0, 0);
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kc].z, bv[nt][kc].z, acc[nt], 0, 0, 0);
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kc].w, bv[nt][kc].w, acc[nt], 0, 0, 0);
      }
    }
  // C layout: col = lane & 15 (channel), row = 4 * (lane >> 4) + i (pixel)
  float* out = static_cast<float*>(a.out);
  // per-image max|out| (split FPN scale): rows of the block's first image
  // reduce over the workgroup, rows of a later image publish directly
  const int nb = blockIdx.x * 64 / HW;
  float m_abs = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + g * 4 + i;
    if (m >= M) continue;
    float mr = 0.f;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const float v = kpd_act(acc[nt][i] + bias[nt], act) + resv[nt][i];
      out[(size_t)m * a.out_cstride + n0 + nt * 16 + r] = v;
      mr = fmaxf(mr, fabsf(v));
    }
    if (a.amax && m / HW != nb) amax_publish_img(a.amax, m / HW, mr);
    else m_abs = fmaxf(m_abs, mr);
  }
  if (a.amax) {
    __shared__ float red[4];
    const float wm = wave_max(m_abs);
    if (lane == 0) red[wave] = wm;
    __syncthreads();
    if (tid == 0) amax_publish_img(a.amax, nb, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
  }
}

// Fused MobileNetV3 inverted residual without SE (features.2 / features.3 of
// mobilenet_v3_small, backbone.py:250-254): expand 1x1 + act, depthwise KxK
// stride S + act, project 1x1 (+ residual), on a tile of TH output rows x the
// full width of one image.  The expanded channels are processed in slices of
// FIR_CS: a slice is expanded (input rows of the tile incl. the depthwise halo,
// zero outside the image), filtered, and folded into the project accumulators
// that each thread keeps for 2 pixels x 8 output channels -- the expanded and
// depthwise tensors never touch HBM (the unfused path writes and re-reads
// them: 2 launches and ~75 MB per step at 256x192).  Sums run in a fixed order
// (input channel, tap, expanded channel), so results do not depend on the batch.
constexpr int FIR_CS = 16;
template <int K, int S>
__global__ __launch_bounds__(256) void fir_kernel(const FirArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  typedef float f2 __attribute__((ext_vector_type(2)));
  constexpr int PD = (K - 1) / 2, CS = FIR_CS, CQ = CS / 4;
  const int n = blockIdx.y, oy0 = blockIdx.x * a.TH, tid = threadIdx.x;
  const int TH = min(a.TH, a.Ho - oy0), Wi = a.Wi, Wo = a.Wo, cin_p = a.cin_p, cout_p = a.cout_p;
  const int iy0 = oy0 * S - PD, THin = (a.TH - 1) * S + K;
  const int npx_in = THin * Wi, npx = TH * Wo;
  // LDS: [xs: npx_in x cin_p] [es: npx_in x CS] [ds: TH*Wo x CS] [weT: cin_p x CS] [wds: K*K x CS] [wpT: CS x cout_p]
  float* xs = sm;
  float* es = xs + npx_in * cin_p;
  float* ds = es + (npx_in + 3) / 4 * 4 * CS;
  float* weT = ds + a.TH * Wo * CS;
  float* wds = weT + cin_p * CS;
  float* wpT = wds + K * K * CS;
  float* sb = wpT + CS * cout_p;   // [be slice: CS][bd slice: CS]
  // es pixel p lives at row esw(p): the depthwise threads of one ds_read_b128
  // lane group read pixels XT * S apart, which would share banks; the swizzle
  // (a permutation within aligned groups of 4 rows, es padded to a multiple of
  // 4) spreads them over the 4 bank quarters
  constexpr int SWS = S == 2 ? 3 : 2;
  auto esw = [](int p) { return p ^ ((p >> SWS) & 3); };
  // the input rows of the tile (zero outside the image)
  const float* xg = a.x + (size_t)n * a.Hi * Wi * cin_p;
  stamp(a.stamps, 0);
  // (batches of 8 loads per thread issued together, then the LDS stores)
  const int cq_in = cin_p / 4, nxq = npx_in * cq_in;
  for (int i0 = 0; i0 < nxq; i0 += 8 * 256) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = min(i0 + u * 256 + tid, nxq - 1);
      const int px = i / cq_in, q = i - px * cq_in, iy = iy0 + px / Wi;
      v[u] = *reinterpret_cast<const float4*>(xg + ((size_t)min(max(iy, 0), a.Hi - 1) * Wi + px % Wi) * cin_p + q * 4);
      if (iy < 0 || iy >= a.Hi) v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * 256 + tid;
      if (i < nxq) reinterpret_cast<float4*>(xs)[i] = v[u];
    }
  }
  // project accumulators: unit = (pixel pair, 8 output channels)
  const int nco8 = cout_p / 8, npair = (npx + 1) / 2, units = npair * nco8;
  const bool has_unit = tid < units;
  const int u_pair = tid / nco8, u_co = (tid - u_pair * nco8) * 8;
  const int px0 = min(u_pair * 2, npx - 1), px1 = min(u_pair * 2 + 1, npx - 1);
  f2 acc[2][4];   // (channel pairs: packed FMAs)
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[r][j] = f2{0.f, 0.f};

  // a slice's weights are loaded into registers one slice ahead (issued
  // before this slice's compute, stored to LDS after its barrier), so no
  // slice waits on a global round trip for its weights.  (Padding the LDS
  // pixel rows against bank conflicts with a one-pixel expand mapping
  // measured 84 vs 51 us: more LDS reads per FMA; not kept.)
  constexpr int PE = 4, PP = 4;   // cin_p * CS <= 1024, CS * cout_p <= 1024 (fir_pick_rows)
  float pe[PE], pp[PP];
  float4 pd = make_float4(0.f, 0.f, 0.f, 0.f), pb = make_float4(0.f, 0.f, 0.f, 0.f);
  auto prefetch = [&](int c0) {
    // the slice's expand / depthwise biases ride along (no global round trip inside a phase)
    if (tid >= 256 - 2 * CQ) {
      const int v = tid - (256 - 2 * CQ);
      pb = *reinterpret_cast<const float4*>((v < CQ ? a.be : a.bd) + c0 + (v % CQ) * 4);
    }
#pragma unroll
    for (int u = 0; u < PE; ++u) {
      const int i = tid + u * 256, c = i / cin_p, k = i - c * cin_p;
      pe[u] = i < cin_p * CS ? a.we[(size_t)(c0 + c) * cin_p + k] : 0.f;
    }
    if (tid < K * K * CQ) {
      const int t = tid / CQ, q = tid - t * CQ;
      pd = *reinterpret_cast<const float4*>(a.wd + (size_t)t * a.Ep + c0 + q * 4);
    }
#pragma unroll
    for (int u = 0; u < PP; ++u) {
      const int i = tid + u * 256, co = i / CS, c = i - co * CS;
      pp[u] = i < CS * cout_p ? a.wp[(size_t)co * a.Ep + c0 + c] : 0.f;
    }
  };
  prefetch(0);
  for (int c0 = 0; c0 < a.Ep; c0 += CS) {
    __syncthreads();   // previous slice's es / ds / weights fully consumed (and xs staged)
#pragma unroll
    for (int u = 0; u < PE; ++u) {
      const int i = tid + u * 256, c = i / cin_p, k = i - c * cin_p;
      if (i < cin_p * CS) weT[k * CS + c] = pe[u];
    }
    if (tid < K * K * CQ) reinterpret_cast<float4*>(wds)[tid] = pd;
    if (tid >= 256 - 2 * CQ) reinterpret_cast<float4*>(sb)[tid - (256 - 2 * CQ)] = pb;
#pragma unroll
    for (int u = 0; u < PP; ++u) {
      const int i = tid + u * 256, co = i / CS, c = i - co * CS;
      if (i < CS * cout_p) wpT[c * cout_p + co] = pp[u];
    }
    if (c0 + CS < a.Ep) prefetch(c0 + CS);
    __syncthreads();
    if (c0 == 0) stamp(a.stamps, 1);
    // expand: 4 pixels x 4 channels per thread, weights from LDS
    const int pg_n = (npx_in + 3) / 4;
    for (int i = tid; i < pg_n * CQ; i += 256) {
      const int pg = i / CQ, q = i - pg * CQ;
      // (v_pk_fma_f32: channel pairs (x, y) / (z, w) in one packed FMA, the
      // pixel value broadcast -- the same fma per element, half the VALU issue;
      // the kernel is bound by its FMA issue)
      const float4 b = reinterpret_cast<const float4*>(sb)[q];
      f2 acc_e[4][2];
#pragma unroll
      for (int r = 0; r < 4; ++r) { acc_e[r][0] = f2{b.x, b.y}; acc_e[r][1] = f2{b.z, b.w}; }
      int pxr[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) pxr[r] = min(r * pg_n + pg, npx_in - 1);   // pixels pg_n apart: conflict-free xs reads
      for (int k = 0; k < cin_p; k += 4) {
        float4 xv[4], wv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) xv[r] = *reinterpret_cast<const float4*>(xs + pxr[r] * cin_p + k);
#pragma unroll
        for (int j = 0; j < 4; ++j) wv[j] = *reinterpret_cast<const float4*>(weT + (k + j) * CS + q * 4);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float xk[4] = {xv[r].x, xv[r].y, xv[r].z, xv[r].w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc_e[r][0] = __builtin_elementwise_fma(f2{xk[j], xk[j]}, f2{wv[j].x, wv[j].y}, acc_e[r][0]);
            acc_e[r][1] = __builtin_elementwise_fma(f2{xk[j], xk[j]}, f2{wv[j].z, wv[j].w}, acc_e[r][1]);
          }
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int px = r * pg_n + pg;
        if (px >= npx_in) break;
        const int iy = iy0 + px / Wi;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);   // the depthwise zero padding of the expanded tensor
        if (iy >= 0 && iy < a.Hi)
          v = make_float4(kpd_act(acc_e[r][0].x, a.act_e), kpd_act(acc_e[r][0].y, a.act_e),
                          kpd_act(acc_e[r][1].x, a.act_e), kpd_act(acc_e[r][1].y, a.act_e));
        reinterpret_cast<float4*>(es)[esw(px) * CQ + q] = v;
      }
    }
    __syncthreads();
    if (c0 == 0) stamp(a.stamps, 2);
    // depthwise: 4 consecutive output columns x 4 channels per thread
    constexpr int XT = 4, NC = (XT - 1) * S + K;
    const int wx = (Wo + XT - 1) / XT;
    for (int i = tid; i < TH * wx * CQ; i += 256) {
      const int q = i % CQ, r = i / CQ, xt = r % wx, oy = r / wx, ox0 = xt * XT, ix0 = ox0 * S - PD;
      f2 d[XT][2];
#pragma unroll
      for (int o = 0; o < XT; ++o) d[o][0] = d[o][1] = f2{0.f, 0.f};
#pragma unroll
      for (int ky = 0; ky < K; ++ky) {
        const int ly = oy * S + ky;   // row in the tile (iy = iy0 + ly)
        float4 col[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int ix = ix0 + c;
          col[c] = (ix >= 0 && ix < Wi) ? reinterpret_cast<const float4*>(es)[esw(ly * Wi + ix) * CQ + q]
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
          const float4 w = reinterpret_cast<const float4*>(wds)[(ky * K + kx) * CQ + q];
#pragma unroll
          for (int o = 0; o < XT; ++o) {
            const float4 v = col[o * S + kx];
            d[o][0] = __builtin_elementwise_fma(f2{v.x, v.y}, f2{w.x, w.y}, d[o][0]);
            d[o][1] = __builtin_elementwise_fma(f2{v.z, v.w}, f2{w.z, w.w}, d[o][1]);
          }
        }
      }
      const float4 b = reinterpret_cast<const float4*>(sb)[CQ + q];
#pragma unroll
      for (int o = 0; o < XT; ++o) {
        if (ox0 + o >= Wo) break;
        float4 v;
        v.x = kpd_act(d[o][0].x + b.x, a.act_d); v.y = kpd_act(d[o][0].y + b.y, a.act_d);
        v.z = kpd_act(d[o][1].x + b.z, a.act_d); v.w = kpd_act(d[o][1].y + b.w, a.act_d);
        reinterpret_cast<float4*>(ds)[(oy * Wo + ox0 + o) * CQ + q] = v;
      }
    }
    __syncthreads();
    if (c0 == 0) stamp(a.stamps, 3);
    // project: fold this slice into the accumulators
    if (has_unit) {
#pragma unroll
      for (int c4 = 0; c4 < CQ; ++c4) {
        const float4 d0 = reinterpret_cast<const float4*>(ds)[px0 * CQ + c4];
        const float4 d1 = reinterpret_cast<const float4*>(ds)[px1 * CQ + c4];
        const float dv0[4] = {d0.x, d0.y, d0.z, d0.w}, dv1[4] = {d1.x, d1.y, d1.z, d1.w};
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
          const float4 w0 = *reinterpret_cast<const float4*>(wpT + (c4 * 4 + cc) * cout_p + u_co);
          const float4 w1 = *reinterpret_cast<const float4*>(wpT + (c4 * 4 + cc) * cout_p + u_co + 4);
          const f2 wv[4] = {f2{w0.x, w0.y}, f2{w0.z, w0.w}, f2{w1.x, w1.y}, f2{w1.z, w1.w}};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[0][j] = __builtin_elementwise_fma(f2{dv0[cc], dv0[cc]}, wv[j], acc[0][j]);
            acc[1][j] = __builtin_elementwise_fma(f2{dv1[cc], dv1[cc]}, wv[j], acc[1][j]);
          }
        }
      }
    }
  }
  stamp(a.stamps, 4);
  if (!has_unit) return;
  const float4 b0 = *reinterpret_cast<const float4*>(a.bp + u_co), b1 = *reinterpret_cast<const float4*>(a.bp + u_co + 4);
  const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int px = u_pair * 2 + r;
    if (px >= npx) break;
    const int oy = oy0 + px / Wo, ox = px % Wo;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = acc[r][j / 2][j % 2] + bv[j];
    if (a.res) {   // stride 1: the residual pixel is the output pixel
      const float* xr = xg + ((size_t)oy * Wi + ox) * cin_p + u_co;
      const float4 r0 = *reinterpret_cast<const float4*>(xr), r1 = *reinterpret_cast<const float4*>(xr + 4);
      v[0] += r0.x; v[1] += r0.y; v[2] += r0.z; v[3] += r0.w;
      v[4] += r1.x; v[5] += r1.y; v[6] += r1.z; v[7] += r1.w;
    }
    float* op = a.out + (((size_t)n * a.Ho + oy) * Wo + ox) * cout_p + u_co;
    *reinterpret_cast<float4*>(op) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(op + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }  stamp(a.stamps, 5);
}

// Squeeze-excitation, one 1024-thread workgroup (16 waves) per kSeImages
// images (the fc weights are the bulk of the traffic, so each weight load
// serves several images).  The three steps are dependent, so each is laid
// out for memory-level parallelism (all of a step's loads in flight
// together) rather than per-thread loops.
//   x: [N][HW][Cp]; w1 = fc1 [sq][C] (row-major, as stored); w2t = fc2
//   TRANSPOSED [sq][C]; scale out: [N][Cp] (hardsigmoid, 0 in padding).
// torchvision SqueezeExcitation (backbone.py:250 via mobilenet_v3_small).
constexpr int kSeThreads = 1024;
constexpr int kSeImages = 1;   // images per workgroup (4 was measured slower: 16 workgroups, longer chains)
__global__ __launch_bounds__(kSeThreads) void se_kernel(const float* __restrict__ x, int N, int HW, int C, int Cp,
                                                        const float* __restrict__ w1, const float* __restrict__ b1,
                                                        const float* __restrict__ w2t, const float* __restrict__ b2,
                                                        int sq, float* __restrict__ scale,
                                                        const float* __restrict__ pooled) {
  __shared__ float4 part[kSeThreads];
  __shared__ __attribute__((aligned(16))) float mean[kSeImages * 1024];
  __shared__ float hid[kSeImages * 256];
  const int n0 = blockIdx.x * kSeImages, tid = threadIdx.x;
  const int nimg = min(kSeImages, N - n0);
  if (pooled) {   // means already reduced by the fused expand+depthwise kernel
    for (int i = tid; i < kSeImages * Cp; i += kSeThreads) {
      const int m = i / Cp;
      mean[i] = m < nimg ? pooled[(size_t)n0 * Cp + i] : 0.f;
    }
    __syncthreads();
  } else {
    const int nq = Cp >> 2;                       // <= 256
    const int groups = kSeThreads / nq;           // pixel groups sharing a channel quad
    for (int m = 0; m < kSeImages; ++m) {
      if (m >= nimg) {
        for (int c = tid; c < Cp; c += kSeThreads) mean[m * Cp + c] = 0.f;
        continue;
      }
      const float* xb = x + (size_t)(n0 + m) * HW * Cp;
      // (1) pool: thread (q, g) sums pixels g, g + groups, ... -- loads independent
      {
        const int q = tid % nq, g = tid / nq;
        float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
        if (g < groups) {
          int pix = g;
          for (; pix + groups < HW; pix += 2 * groups) {
            const float4 a = *reinterpret_cast<const float4*>(xb + (size_t)pix * Cp + q * 4);
            const float4 b = *reinterpret_cast<const float4*>(xb + (size_t)(pix + groups) * Cp + q * 4);
            s0.x += a.x; s0.y += a.y; s0.z += a.z; s0.w += a.w;
            s1.x += b.x; s1.y += b.y; s1.z += b.z; s1.w += b.w;
          }
          if (pix < HW) {
            const float4 a = *reinterpret_cast<const float4*>(xb + (size_t)pix * Cp + q * 4);
            s0.x += a.x; s0.y += a.y; s0.z += a.z; s0.w += a.w;
          }
          s0.x += s1.x; s0.y += s1.y; s0.z += s1.z; s0.w += s1.w;
        }
        part[tid] = s0;
      }
      __syncthreads();
      if (tid < nq) {
        float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int g = 0; g < groups; ++g) {
          const float4 v = part[g * nq + tid];
          t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
        }
        const float hw = (float)HW;
        *reinterpret_cast<float4*>(mean + m * Cp + tid * 4) = make_float4(t.x / hw, t.y / hw, t.z / hw, t.w / hw);
      }
      __syncthreads();
    }
  }
  se_fc<kSeThreads, kSeImages>(mean, hid, nimg, C, Cp, w1, b1, w2t, b2, sq, scale + (size_t)n0 * Cp);
}

// FPN lateral 1x1 conv with a small input width (cin_p <= 32) and 128 outputs,
// plus the nearest-upsampled top-down residual (backbone.py:33-37).  Pure
// streaming (it writes the largest tensor of the pass): a thread owns 8 output
// channels of kLatPix pixels, all their inputs are loaded before the first
// store, and every store is 16 bytes.  Weights transposed in LDS once per
// workgroup; the grid is capped (kLatBlocks) and each workgroup strides over
// chunks of 16 x kLatPix pixels, so the weight staging and the barrier are
// amortised over many chunks.  fp32 FPN level 0 only: the split (mixed)
// precision never materialises lateral 0 (fpn0x_kernel works by linearity).
constexpr int kLatPix = 2;   // pixels per thread (4 doubles the registers and halves occupancy: slower)
constexpr int kLatBlocks = 2048;
template <int CIN4>          // cin_p / 4
__global__ __launch_bounds__(256) void lateral_stream_kernel(const float* __restrict__ in,
                                                             const float* __restrict__ w,
                                                             const float* __restrict__ bias,
                                                             const float* __restrict__ res, int H, int W, int rh,
                                                             int rw, int M, float* __restrict__ out, int nt_store) {
  __shared__ __attribute__((aligned(16))) float sw[32 * 128];
  const int tid = threadIdx.x;
  constexpr int cin_p = CIN4 * 4;
  for (int i = tid; i < cin_p * 128; i += 256) {
    const int co = i / cin_p, k = i - co * cin_p;
    sw[k * 128 + co] = w[i];
  }
  __syncthreads();
  const int c8 = tid & 15, sub = tid >> 4, co = c8 * 8;
  const float4 b0 = *reinterpret_cast<const float4*>(bias + co), b1 = *reinterpret_cast<const float4*>(bias + co + 4);
  const int HW = H * W;
  const float sy = (float)rh / (float)H, sx = (float)rw / (float)W;
  const int chunks = (M + 16 * kLatPix - 1) / (16 * kLatPix);
  for (int chunk = blockIdx.x; chunk < chunks; chunk += gridDim.x) {
    // load phase: inputs and residuals of this thread's pixels
    float4 xin[kLatPix][CIN4];
    float4 r0[kLatPix], r1[kLatPix];
    int mm[kLatPix];
#pragma unroll
    for (int it = 0; it < kLatPix; ++it) {
      const int m = chunk * (16 * kLatPix) + it * 16 + sub;
      mm[it] = m;
      r0[it] = r1[it] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int k = 0; k < CIN4; ++k) xin[it][k] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (m >= M) continue;
#pragma unroll
      for (int k = 0; k < CIN4; ++k) xin[it][k] = *reinterpret_cast<const float4*>(in + (size_t)m * cin_p + k * 4);
      if (res) {
        const int n = m / HW, r = m - n * HW, y = r / W, x = r - y * W;
        const int yy = rh == H ? y : min((int)floorf((float)y * sy), rh - 1);
        const int xx = rw == W ? x : min((int)floorf((float)x * sx), rw - 1);
        const float* rp = res + ((size_t)(n * rh + yy) * rw + xx) * 128 + co;
        r0[it] = *reinterpret_cast<const float4*>(rp);
        r1[it] = *reinterpret_cast<const float4*>(rp + 4);
      }
    }
#pragma unroll
    for (int it = 0; it < kLatPix; ++it) {
      const int m = mm[it];
      if (m >= M) continue;
      float a[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int k4 = 0; k4 < CIN4; ++k4) {
        const float xs[4] = {xin[it][k4].x, xin[it][k4].y, xin[it][k4].z, xin[it][k4].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 w0 = *reinterpret_cast<const float4*>(sw + (k4 * 4 + q) * 128 + co);
          const float4 w1 = *reinterpret_cast<const float4*>(sw + (k4 * 4 + q) * 128 + co + 4);
          a[0] = fmaf(xs[q], w0.x, a[0]); a[1] = fmaf(xs[q], w0.y, a[1]);
          a[2] = fmaf(xs[q], w0.z, a[2]); a[3] = fmaf(xs[q], w0.w, a[3]);
          a[4] = fmaf(xs[q], w1.x, a[4]); a[5] = fmaf(xs[q], w1.y, a[5]);
          a[6] = fmaf(xs[q], w1.z, a[6]); a[7] = fmaf(xs[q], w1.w, a[7]);
        }
      }
      a[0] += r0[it].x; a[1] += r0[it].y; a[2] += r0[it].z; a[3] += r0[it].w;
      a[4] += r1[it].x; a[5] += r1[it].y; a[6] += r1[it].z; a[7] += r1[it].w;
      float* op = out + (size_t)m * 128 + co;
      if (nt_store) {   // streamed past the caches (KPD_LAT_NT, A/B)
        __builtin_nontemporal_store(f32x4{a[0], a[1], a[2], a[3]}, reinterpret_cast<f32x4*>(op));
        __builtin_nontemporal_store(f32x4{a[4], a[5], a[6], a[7]}, reinterpret_cast<f32x4*>(op + 4));
      } else {
        *reinterpret_cast<float4*>(op) = make_float4(a[0], a[1], a[2], a[3]);
        *reinterpret_cast<float4*>(op + 4) = make_float4(a[4], a[5], a[6], a[7]);
      }
    }
  }
}

// stats: [N][tiles][2][Cp]; grid (tiles, N); each block reduces HW/tiles pixels.
__global__ __launch_bounds__(256) void channel_stats_kernel(const float* __restrict__ x, int HW, int Cp,
                                                            int tiles, float* __restrict__ stats) {
  const int t = blockIdx.x, n = blockIdx.y;
  const int per = (HW + tiles - 1) / tiles;
  const int p0 = t * per, p1 = min(HW, p0 + per);
  for (int c = threadIdx.x; c < Cp; c += blockDim.x) {
    float s = 0.f, m = -INFINITY;
    for (int p = p0; p < p1; ++p) {
      const float v = x[((size_t)n * HW + p) * Cp + c];
      s += v; m = fmaxf(m, v);
    }
    float* st = stats + ((size_t)n * tiles + t) * 2 * Cp;
    st[c] = s;
    st[Cp + c] = m;
  }
}

}  // namespace

hipError_t launch_stem(const float* img, int N, int Cin, int H, int W, const float* w, const float* b,
                       float* out, int Ho, int Wo, float* amax, hipStream_t st) {
  const int total = N * Ho * Wo;
  if (Cin == 3)
    hipLaunchKernelGGL(stem_kernel<3>, dim3((total + 511) / 512), dim3(256), 0, st, img, N, H, W, w, b, out, Ho,
                       Wo, amax);
  else if (Cin == 1)
    hipLaunchKernelGGL(stem_kernel<1>, dim3((total + 511) / 512), dim3(256), 0, st, img, N, H, W, w, b, out, Ho,
                       Wo, amax);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_dwconv(const float* in, const float* w, const float* b, float* out, int N, int H, int W,
                         int Cp, int Ho, int Wo, int k, int s, int act, hipStream_t st) {
  const size_t total = (size_t)N * Ho * ((Wo + 3) / 4) * (Cp / 4);
  const dim3 grid((unsigned)((total + 255) / 256));
#define DW(K, S) hipLaunchKernelGGL((dwconv_kernel<K, S>), grid, dim3(256), 0, st, in, w, b, out, N, H, W, Cp, Ho, Wo, act)
  if (k == 3 && s == 1) DW(3, 1);
  else if (k == 3 && s == 2) DW(3, 2);
  else if (k == 5 && s == 1) DW(5, 1);
  else if (k == 5 && s == 2) DW(5, 2);
  else return hipErrorInvalidValue;
#undef DW
  return hipGetLastError();
}

hipError_t launch_se(const float* x, int N, int HW, int C, int Cp, const float* w1, const float* b1,
                     const float* w2, const float* b2, int sq, float* scale, hipStream_t st, const float* pooled) {
  if (Cp > 1024 || sq > 256 || C % 4 || sq % 2) return hipErrorInvalidValue;
  hipLaunchKernelGGL(se_kernel, dim3((N + kSeImages - 1) / kSeImages), dim3(kSeThreads), 0, st, x, N, HW, C, Cp, w1,
                     b1, w2, b2, sq, scale, pooled);
  return hipGetLastError();
}

hipError_t launch_lateral_stream(const float* in, int cin_p, const float* w, const float* bias, const float* res,
                                 int N, int H, int W, int rh, int rw, void* out, hipStream_t st) {
  if (cin_p != 16 && cin_p != 32) return hipErrorInvalidValue;
  const int M = N * H * W;
  const int chunks = (M + 16 * kLatPix - 1) / (16 * kLatPix);
  static const int blocks_env = kpd_diag_env("KPD_LAT_BLOCKS") ? atoi(kpd_diag_env("KPD_LAT_BLOCKS")) : kLatBlocks;
  static const int nt_env = kpd_diag_env("KPD_LAT_NT") ? atoi(kpd_diag_env("KPD_LAT_NT")) : 0;
  const int nblk = std::max(1, std::min(chunks, blocks_env));
#define LAT(C4) hipLaunchKernelGGL(lateral_stream_kernel<C4>, dim3(nblk), dim3(256), 0, st, in, w, bias, res, H, \
                                  W, rh, rw, M, static_cast<float*>(out), nt_env)
  switch (cin_p / 4) {
    case 4: LAT(4); break;
    case 8: LAT(8); break;
    default: return hipErrorInvalidValue;
  }
#undef LAT
  return hipGetLastError();
}

hipError_t launch_channel_stats(const float* x, int N, int HW, int Cp, int tiles, float* stats,
                                hipStream_t st) {
  hipLaunchKernelGGL(channel_stats_kernel, dim3(tiles, N), dim3(128), 0, st, x, HW, Cp, tiles, stats);
  return hipGetLastError();
}

size_t fir_lds_bytes(const FirArgs& a, int K, int S) {
  const size_t THin = (size_t)(a.TH - 1) * S + K;
  return 4 * (THin * a.Wi * a.cin_p + (THin * a.Wi + 3) / 4 * 4 * FIR_CS + (size_t)a.TH * a.Wo * FIR_CS + (size_t)a.cin_p * FIR_CS +
              (size_t)K * K * FIR_CS + (size_t)FIR_CS * a.cout_p + 2 * FIR_CS);
}

int fir_pick_rows(FirArgs& a, int K, int S) {
  if (a.cin_p % 4 || a.Ep % FIR_CS || a.cout_p % 8 || (a.res && (S != 1 || a.cin_p != a.cout_p)) ||
      a.cin_p * FIR_CS > 1024 || FIR_CS * a.cout_p > 1024 || K * K * FIR_CS / 4 > 256)
    return 0;
  static const int th_env = kpd_diag_env("KPD_FIR_TH") ? atoi(kpd_diag_env("KPD_FIR_TH")) : 0;   // A/B sweeps
  for (int th = std::min(a.Ho, th_env > 0 ? th_env : 16); th >= 1; --th) {
    a.TH = th;
    const int units = (th * a.Wo + 1) / 2 * (a.cout_p / 8);
    if (units <= 256 && fir_lds_bytes(a, K, S) <= 64 * 1024) return th;
  }
  a.TH = 0;
  return 0;
}

hipError_t launch_fir(const FirArgs& a, int N, int K, int S, hipStream_t st) {
  if (a.TH <= 0 || (a.TH * a.Wo + 1) / 2 * (a.cout_p / 8) > 256) return hipErrorInvalidValue;
  const size_t lds = fir_lds_bytes(a, K, S);
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  const dim3 grid((a.Ho + a.TH - 1) / a.TH, N);
#define FIR(KK, SS) hipLaunchKernelGGL((fir_kernel<KK, SS>), grid, dim3(256), lds, st, a)
  if (K == 3 && S == 1) FIR(3, 1);
  else if (K == 3 && S == 2) FIR(3, 2);
  else if (K == 5 && S == 1) FIR(5, 1);
  else if (K == 5 && S == 2) FIR(5, 2);
  else return hipErrorInvalidValue;
#undef FIR
  return hipGetLastError();
}

// the BL variant of exdw_kernel: the 576-wide stride-1 SE blocks (32-channel
// slices of a 96-channel input; KPD_EXDW_NOBL=1, diagnostic build: off)
bool exdw_bl(const ExDwArgs& a, int K) {
  static const bool off = kpd_diag_env("KPD_EXDW_NOBL") != nullptr;
  return !off && K == 5 && a.Hi == a.Ho && a.CS == 32 && a.cin_p == 96 && a.pooled && a.part && a.nband <= 1;
}

size_t exdw_lds_bytes(const ExDwArgs& a, int K) {
  // a band's input rows: at most ceil(Ho / nband) output rows' worth
  const int nb = a.nband > 1 ? a.nband : 1, S = a.Hi > a.Ho ? 2 : 1;
  const int Pin = std::min(a.Hi, ((a.Ho + nb - 1) / nb - 1) * S + K) * a.Wi, Po = a.Ho * a.Wo;
  // the fc1 columns are filled by 1 KiB LDS-DMA pieces: round up to whole pieces
  const size_t w1f = exdw_bl(a, K) ? ((size_t)a.CS * (a.cin_p + 8) + 255) / 256 * 256
                   : a.part ? ((size_t)a.sq * a.CS + 255) / 256 * 256 : 0;
  const size_t main = (size_t)Pin * exdw_estr(a.CS, S) + (size_t)(K * K + 1) * a.CS + (a.pooled ? (size_t)Po * a.CS : 0) + w1f;
  return 4 * main;
}

hipError_t launch_exdw(const ExDwArgs& a, int N, int K, int S, hipStream_t st) {
  const int kc = a.cin_p / 16;
  if ((a.CS != 16 && a.CS != 32 && a.CS != 48) || a.Ep % a.CS || a.cin_p % 16 || (kc != 2 && kc != 3 && kc != 6) ||
      !a.we ||
      (a.part && (!a.pooled || !a.w1 || a.sq <= 0 || a.sq > 144 || a.C % 4)) ||
      (a.nband > 1 && (a.pooled || a.part || a.nband > a.Ho)))
    return hipErrorInvalidValue;
  const size_t lds = exdw_lds_bytes(a, K);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const dim3 grid(a.Ep / a.CS, N, a.nband > 1 ? a.nband : 1);
  const bool xt4 = a.Wo >= 12;
  // the coarse SE blocks (features.4..11) use hardswish for both: that
  // instance compiled with the constant (KPD_EXDW_RTACT=1, diagnostic build: the runtime switch)
  static const bool rtact = kpd_diag_env("KPD_EXDW_RTACT") != nullptr;
  const bool hs = !rtact && a.act_e == ACT_HSWISH && a.act_d == ACT_HSWISH;
  if (exdw_bl(a, K)) {
    if (hs && xt4) hipLaunchKernelGGL((exdw_kernel<5, 1, 2, 4, 6, true, ACT_HSWISH>), grid, dim3(256), lds, st, a);
    else if (hs) hipLaunchKernelGGL((exdw_kernel<5, 1, 2, 2, 6, true, ACT_HSWISH>), grid, dim3(256), lds, st, a);
    else if (xt4) hipLaunchKernelGGL((exdw_kernel<5, 1, 2, 4, 6, true>), grid, dim3(256), lds, st, a);
    else hipLaunchKernelGGL((exdw_kernel<5, 1, 2, 2, 6, true>), grid, dim3(256), lds, st, a);
    return hipGetLastError();
  }
  // the hardswish instances the model's blocks take: features.4 (5x5 s2, 16-channel slices of 32
  // input channels), .5-.8 (5x5 s1, 16-channel slices, 48 input channels), .9 (5x5 s2, 32-channel slices)
  if (hs && K == 5 && S == 2 && a.CS == 16 && kc == 2 && xt4) {
    hipLaunchKernelGGL((exdw_kernel<5, 2, 1, 4, 2, false, ACT_HSWISH>), grid, dim3(256), lds, st, a);
    return hipGetLastError();
  }
  if (hs && K == 5 && S == 1 && a.CS == 16 && kc == 3 && xt4) {
    hipLaunchKernelGGL((exdw_kernel<5, 1, 1, 4, 3, false, ACT_HSWISH>), grid, dim3(256), lds, st, a);
    return hipGetLastError();
  }
  if (hs && K == 5 && S == 2 && a.CS == 32 && kc == 3 && !xt4) {
    hipLaunchKernelGGL((exdw_kernel<5, 2, 2, 2, 3, false, ACT_HSWISH>), grid, dim3(256), lds, st, a);
    return hipGetLastError();
  }
#define EXDW_KC(KK, SS, NTC, XT)                                                                        \
  do {                                                                                                  \
    if (kc == 2) hipLaunchKernelGGL((exdw_kernel<KK, SS, NTC, XT, 2>), grid, dim3(256), lds, st, a);   \
    else if (kc == 3) hipLaunchKernelGGL((exdw_kernel<KK, SS, NTC, XT, 3>), grid, dim3(256), lds, st, a); \
    else hipLaunchKernelGGL((exdw_kernel<KK, SS, NTC, XT, 6>), grid, dim3(256), lds, st, a);           \
  } while (0)
#define EXDW(KK, SS)                                    \
  do {                                                  \
    if (a.CS == 16) {                                   \
      if (xt4) EXDW_KC(KK, SS, 1, 4);                   \
      else EXDW_KC(KK, SS, 1, 2);                       \
    } else if (a.CS == 32) {                            \
      if (xt4) EXDW_KC(KK, SS, 2, 4);                   \
      else EXDW_KC(KK, SS, 2, 2);                       \
    } else {                                            \
      EXDW_KC(KK, SS, 3, 2);                            \
    }                                                   \
  } while (0)
  if (K == 3 && S == 1) EXDW(3, 1);
  else if (K == 5 && S == 1) EXDW(5, 1);
  else if (K == 5 && S == 2) EXDW(5, 2);
  else return hipErrorInvalidValue;
#undef EXDW
#undef EXDW_KC
  return hipGetLastError();
}

size_t seproj_lds_bytes(const SeProjArgs& a) {
  const int mt = (a.Po + 15) / 16;
  const size_t nq4 = a.C / 4, ngrp = std::max<size_t>(1, std::min<size_t>(16, 256 / nq4));
  const size_t red = std::max({(size_t)4 * mt * 16 * a.NT, (size_t)a.nsl * a.sq, ngrp * a.C});
  return 4 * ((size_t)a.Ep + 256 + red);
}

hipError_t launch_seproj(const SeProjArgs& a, int N, hipStream_t st) {
  const int mt_all = (a.Po + 15) / 16;
  if (a.Ep % 16 || a.NT % 16 || a.cout_p % a.NT || a.sq > 144 || a.C > a.Ep || a.C % 4 ||
      (size_t)a.nsl * a.sq > 6 * 256 * 4 || (a.nsl * a.sq) % 4)
    return hipErrorInvalidValue;
  // the 192-pixel maps split their rows over workgroups, each recomputing the
  // excitation: with 48-column tiles (all of features.4..8's outputs) four
  // groups of 48 rows (256 workgroups at 64 images, 4 excitations per image),
  // with 16-column tiles two (384 workgroups, 6 excitations per image)
  static const int msplit_env = kpd_diag_env("KPD_SEPROJ_MSPLIT") ? atoi(kpd_diag_env("KPD_SEPROJ_MSPLIT")) : 0;
  const int msplit = mt_all == 12 ? (msplit_env > 0 ? msplit_env : (a.NT >= 48 ? 4 : 2)) : 1;
  const int mt = (mt_all + msplit - 1) / msplit;
  SeProjArgs b = a;
  // the 48-pixel maps (3 row tiles): eight waves split the project's K
  // chunks (one wave per SIMD at four leaves the fp32-MFMA K loop exposed):
  // 12.1 -> 9.6 us per launch.  The 192-pixel maps (6 row tiles per
  // workgroup) measured 13.5 -> 16.9 us with eight, so they keep four.
  // KPD_SEPROJ_NWV = 4 / 8 forces one (A/B).
  static const int nwv_env = kpd_diag_env("KPD_SEPROJ_NWV") ? atoi(kpd_diag_env("KPD_SEPROJ_NWV")) : 0;
  const int nwv = nwv_env == 4 || nwv_env == 8 ? nwv_env : (mt == 3 ? 8 : 4);
  const size_t lds_m = 4 * ((size_t)a.Ep + 256 + std::max({(size_t)nwv * mt * 16 * a.NT, (size_t)a.nsl * a.sq,
                                                             std::max<size_t>(1, std::min<size_t>(16, 256 / (a.C / 4))) * a.C}));
  if (lds_m > 160 * 1024) return hipErrorInvalidValue;
  const dim3 grid(a.cout_p / a.NT, N, msplit);
  const int ntt = a.NT / 16;
#define SEP(M, T)                                                                                   \
  do {                                                                                              \
    if (nwv == 8) hipLaunchKernelGGL((seproj_kernel<M, T, 8>), grid, dim3(512), lds_m, st, b);     \
    else hipLaunchKernelGGL((seproj_kernel<M, T, 4>), grid, dim3(256), lds_m, st, b);              \
  } while (0)
  if (mt == 3 && ntt == 1) SEP(3, 1);
  else if (mt == 3 && ntt == 2) SEP(3, 2);
  else if (mt == 3 && ntt == 3) SEP(3, 3);
  else if (mt == 6 && ntt == 1) SEP(6, 1);
  else if (mt == 4 && ntt == 1) SEP(4, 1);
  else if (mt == 12 && ntt == 1) SEP(12, 1);
  else if (mt == 12 && ntt == 3) SEP(12, 3);
  else return hipErrorInvalidValue;
#undef SEP
  return hipGetLastError();
}

hipError_t launch_dwsum(const float* in, int N, int Hi, int Wi, const float* w, const float* b, int act, float* out,
                         int Ho, int Wo, int k, int s, float* part, int* ntiles, hipStream_t st) {
  if (kDwsTH * ((Wo + 3) / 4) * 4 > 256) return hipErrorInvalidValue;
  const dim3 grid((Ho + kDwsTH - 1) / kDwsTH, N);
  *ntiles = (int)grid.x;
  if (k == 3 && s == 2 && act == ACT_RELU)   // features.1 of mobilenet_v3_small
    hipLaunchKernelGGL((dwsum_kernel<3, 2, ACT_RELU>), grid, dim3(256), 0, st, in, Hi, Wi, w, b, act, out, Ho, Wo, part);
  else if (k == 3 && s == 2) hipLaunchKernelGGL((dwsum_kernel<3, 2>), grid, dim3(256), 0, st, in, Hi, Wi, w, b, act, out, Ho, Wo, part);
  else if (k == 3 && s == 1) hipLaunchKernelGGL((dwsum_kernel<3, 1>), grid, dim3(256), 0, st, in, Hi, Wi, w, b, act, out, Ho, Wo, part);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_se16_proj(const float* d, int N, int npx, int ntiles, const float* part, const float* w1,
                            const float* b1, const float* w2t, const float* b2, int sq, const float* wp,
                            const float* bp, float* out, hipStream_t st) {
  if (sq > 16 || ntiles * 16 > 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(se16_proj_kernel, dim3((npx + 255) / 256, N), dim3(256), 0, st, d, npx, ntiles, part, w1, b1, w2t,
                     b2, sq, wp, bp, out);
  return hipGetLastError();
}

bool pw_small_ok(const ConvArgs& a) {
  static const bool off = kpd_diag_env("KPD_NO_PWSMALL") != nullptr;   // A/B switch
  // large outputs keep the generic kernel's LDS-staged 16-byte stores: lateral
  // 1 (6.3 M outputs at 64 images) measured 18.9 us here vs 17.6 us there;
  // lateral 2 (1.6 M) 8.2 vs 17, the last conv (1.8 M) 12.9 vs 18
  return !off && a.cin_p % 16 == 0 && a.cin_p <= 16 * kPwKC && a.cout_p % 64 == 0 && !a.a_scale && !a.stats &&
         !a.post_scale && a.act3 == 0 && a.out_cstride >= a.cout_p && a.in_cstride % 4 == 0 && a.M > 0 &&
         (long)a.M * a.cout_p <= (4L << 20);
}

hipError_t launch_pw_small(const ConvArgs& a, hipStream_t st) {
  if (!pw_small_ok(a)) return hipErrorInvalidValue;
  const dim3 grid((a.M + 63) / 64, a.cout_p / 64);
  if (a.act == ACT_HSWISH) hipLaunchKernelGGL(pw_small_kernel<ACT_HSWISH>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(pw_small_kernel<>, grid, dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_se_excite(const SeProjArgs& a, int N, float* sesc, hipStream_t st) {
  if (a.sq > 144 || a.C % 4 || a.C > a.Ep || (size_t)a.nsl * a.sq > kSeExcitePart || (a.nsl * a.sq) % 4)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(se_excite_kernel, dim3((a.Ep + 63) / 64, N), dim3(256), 0, st, a, sesc);
  return hipGetLastError();
}

