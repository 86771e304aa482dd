// Coarse MobileNetV3-Small body in one launch (gfx950): features.5..11 -- the
// squeeze-excitation inverted residuals on the 1/16 and 1/32 maps -- and
// features.12 (1x1 96 -> 576 + hardswish), torchvision mobilenet_v3_small as
// the reference builds it (backbone.py:250-254).
//
// The batched path runs these layers as ~20 launches (exdw -> se_excite ->
// seproj per block), each a few microseconds of latency-bound work on tensors
// of a few hundred kilobytes.  Here one 512-thread workgroup owns one image
// for the whole chain: the block input lives in LDS, every phase is separated
// by a workgroup barrier instead of a kernel boundary, and nothing but the
// depthwise output (the SE needs all of it before the project can start)
// leaves the CU.  An image's result depends on that image alone.
//
// Per block (Ep expanded channels, in rounds of RW = 64):
//   XS    = f16 hi | lo split of the block input X * 2^ex (ex from max|X|)
//   round: expand 1x1 on v_mfma_f32_16x16x32_f16, three products per K-step
//          (lo.hi + hi.hi + hi.lo, fp32 accumulate; fp32-accurate, the
//          hmconv / fpn0x numerics) -> act -> E (LDS)
//          depthwise k x k from E (fp32 VALU) -> act -> D (per-image global
//          scratch, L2-resident) + per-channel sums (fixed-order) + max|d|
//   SE:    fc1 / ReLU / fc2 / hardsigmoid on the channel means (fp32)
//   project 1x1 on the split MFMA with A = D * s (split on the fly, scale from
//          max|d|: s <= 1), + bias (+ residual X) -> X (in place)
// features.12 reads XS of the last block output and writes the FPN tap.
#include <algorithm>

#include "kpd_common.h"
#include "kpd_kernels.h"

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int NT = 512, NW = NT / 64;
constexpr int RW = 64;             // expanded channels per round
constexpr int ESTR = RW + 4;       // LDS row of the expanded slice (floats): 16-byte reads of 4 quads on distinct banks
constexpr int kMaxEp = 576, kMaxSq = 160, kMaxKK = 25;

struct CbLds { int x, xs, e, wd, red, mean, sc, hid, misc, total; };

__host__ __device__ inline int rup(int v, int a) { return (v + a - 1) / a * a; }
__host__ __device__ inline int imax(int a, int b) { return a > b ? a : b; }

__host__ __device__ inline CbLds cb_layout(const CbodyArgs& a) {
  int xf = 0, xsb = 0, ef = 0;
  for (int l = 0; l < a.nl; ++l) {
    const CbLayer& L = a.L[l];
    const int pin = L.Hi * L.Wi, po = L.Ho * L.Wo;
    xf = imax(xf, imax(pin * L.cin_p, po * L.cout_p));
    xsb = imax(xsb, L.kc_in * pin * 128);
    ef = imax(ef, pin * ESTR);
  }
  const CbLayer& Z = a.L[a.nl - 1];
  xsb = imax(xsb, a.last_kc * Z.Ho * Z.Wo * 128);
  CbLds o;
  int off = 0;
  o.x = off;    off = rup(off + xf * 4, 16);
  o.xs = off;   off = rup(off + xsb, 16);
  o.e = off;    off = rup(off + ef * 4, 16);
  o.wd = off;   off += kMaxKK * RW * 4;
  o.red = off;  off += NW * RW * 4;
  o.mean = off; off += kMaxEp * 4;
  o.sc = off;   off += kMaxEp * 4;
  o.hid = off;  off += kMaxSq * 4;
  o.misc = off; off += 64;
  o.total = off;
  return o;
}

__device__ __forceinline__ void cstamp(unsigned long long* st, int i) {
  if (st && threadIdx.x == 0) st[(size_t)blockIdx.x * 128 + (i & 127)] = __builtin_amdgcn_s_memrealtime();
}

__device__ __forceinline__ void split8(const float* v, float sc, f16x8& hi, f16x8& lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float x = v[e] * sc;
    const _Float16 h = (_Float16)x;
    hi[e] = h;
    lo[e] = (_Float16)(x - (float)h);
  }
}

__device__ __forceinline__ f32x4 mma3(const f16x8& ah, const f16x8& al, const f16x8& bh, const f16x8& bl, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, c, 0, 0, 0);
}

// XS row piece of (K chunk kc, pixel px): 128 bytes = 8 units of 16 B (hi
// units 0-3, lo units 4-7 of 8 channels each), unit u at u ^ (px & 7)
__device__ __forceinline__ const char* xs_unit(const char* XS, int P, int kc, int px, int u) {
  return XS + ((size_t)kc * P + px) * 128 + ((u ^ (px & 7)) << 4);
}

// X [P][cin_p] fp32 -> XS (kc chunks of 32 channels, zero past cin_p) with
// the scale 2^ex, ex = split_exp_of(max|X|) (max in *xmax_bits)
__device__ int build_xs(const float* X, char* XS, int P, int cin_p, int kc, const unsigned* xmax_bits) {
  const int ex = split_exp_of(__uint_as_float(*xmax_bits));
  const float sc = ldexpf(1.f, ex);
  const int items = kc * P * 4;
  for (int i = threadIdx.x; i < items; i += NT) {
    const int g4 = i & 3, rest = i >> 2, px = rest % P, k = rest / P, c0 = k * 32 + g4 * 8;
    float v[8];
    if (c0 < cin_p) {
      const float4 a = *reinterpret_cast<const float4*>(X + (size_t)px * cin_p + c0);
      const float4 b = *reinterpret_cast<const float4*>(X + (size_t)px * cin_p + c0 + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 0.f;
    }
    f16x8 hi, lo;
    split8(v, sc, hi, lo);
    *reinterpret_cast<f16x8*>(const_cast<char*>(xs_unit(XS, P, k, px, g4))) = hi;
    *reinterpret_cast<f16x8*>(const_cast<char*>(xs_unit(XS, P, k, px, 4 + g4))) = lo;
  }
  return ex;
}

// workgroup barrier that orders LDS only: the wave's global stores and
// prefetch loads stay in flight across it (they are waited for where used)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ void lds_max(unsigned* slot, float v) {
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0 && v > 0.f) atomicMax(slot, __float_as_uint(v));
}

// depthwise k x k (stride S, XT output columns per work item) of the round's RW channels from E [Pin][ESTR]
// with the round's weights WD [k*k][RW]; work item (output row, XT-column
// tile, channel quad q = tid % 16).  Output -> D [Po][EpK] (+ c0), the
// item's channel sums reduced over the wave's lanes of the same quad in a
// fixed butterfly, per wave into RED [NW][RW]; max|d| into *dmax.
template <int K, int S, int XT>
__device__ void depthwise_round(const CbLayer& L, const float* E, const float* WD, float* D, float* RED,
                                unsigned* dmax, int c0, int rc, int dbg) {
  constexpr int PD = (K - 1) / 2, NC = (XT - 1) * S + K;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = tid & 15;
  const int nxt = (L.Wo + XT - 1) / XT, nsp = L.Ho * nxt;
  const bool qlive = q * 4 < rc;
  float4 psum = make_float4(0.f, 0.f, 0.f, 0.f);
  float m = 0.f;
  const float4 b = qlive ? *reinterpret_cast<const float4*>(L.bd + c0 + q * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int sp = tid >> 4; sp < nsp; sp += NT / 16) {
    if (!qlive) continue;
    const int oy = sp / nxt, ox0 = (sp - oy * nxt) * XT, ix0 = ox0 * S - PD;
    float4 a[XT];
#pragma unroll
    for (int o = 0; o < XT; ++o) a[o] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      const int iy = oy * S - PD + ky;
      if (iy < 0 || iy >= L.Hi) continue;
      float4 col[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int ix = ix0 + c;
        col[c] = (ix >= 0 && ix < L.Wi) ? *reinterpret_cast<const float4*>(E + (iy * L.Wi + ix) * ESTR + q * 4)
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int kx = 0; kx < K; ++kx) {
        const float4 w = *reinterpret_cast<const float4*>(WD + (ky * K + kx) * RW + q * 4);
#pragma unroll
        for (int o = 0; o < XT; ++o) {
          const float4 v = col[o * S + kx];
          a[o].x = fmaf(v.x, w.x, a[o].x); a[o].y = fmaf(v.y, w.y, a[o].y);
          a[o].z = fmaf(v.z, w.z, a[o].z); a[o].w = fmaf(v.w, w.w, a[o].w);
        }
      }
    }
#pragma unroll
    for (int o = 0; o < XT; ++o) {
      if (ox0 + o >= L.Wo) break;
      float4 v;
      v.x = kpd_act(a[o].x + b.x, ACT_HSWISH); v.y = kpd_act(a[o].y + b.y, ACT_HSWISH);
      v.z = kpd_act(a[o].z + b.z, ACT_HSWISH); v.w = kpd_act(a[o].w + b.w, ACT_HSWISH);
      const int op = oy * L.Wo + ox0 + o;
      if (!(dbg & 1)) *reinterpret_cast<float4*>(D + (size_t)op * L.EpK + c0 + q * 4) = v;
      psum.x += v.x; psum.y += v.y; psum.z += v.z; psum.w += v.w;
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
  }
  // lanes q, q + 16, q + 32, q + 48 hold the same channel quad
#pragma unroll
  for (int o = 16; o <= 32; o <<= 1) {
    psum.x += __shfl_xor(psum.x, o, 64); psum.y += __shfl_xor(psum.y, o, 64);
    psum.z += __shfl_xor(psum.z, o, 64); psum.w += __shfl_xor(psum.w, o, 64);
  }
  if (lane < 16) *reinterpret_cast<float4*>(RED + wave * RW + lane * 4) = psum;
  lds_max(dmax, m);
}

__device__ __forceinline__ float hswish(float v) { return kpd_act(v, ACT_HSWISH); }

struct Smem {
  float *X, *E, *WD, *RED, *MEAN, *SC, *HID;
  char* XS;
  unsigned* MISC;
};

// expand weights of one round for this wave's N tile (wave & 3): KC K chunks
// of 8 f16 hi + 8 f16 lo (the lane's MFMA B fragment), and the tile's bias
template <int KC>
struct BFrag { f16x8 h[KC], l[KC]; float bias; };

template <int KC>
__device__ __forceinline__ void load_bfrag(const CbLayer& L, int c0, int rc, BFrag<KC>& b) {
  const int lane = threadIdx.x & 63, nt = (threadIdx.x >> 6) & 3;
  if (nt * 16 < rc) {
    const int row = c0 + nt * 16 + (lane & 15);
    const char* wr = reinterpret_cast<const char*>(L.we) + (size_t)row * KC * 128 + (lane >> 4) * 16;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      b.h[kc] = *reinterpret_cast<const f16x8*>(wr + kc * 128);
      b.l[kc] = *reinterpret_cast<const f16x8*>(wr + kc * 128 + 64);
    }
    b.bias = L.be[row];
  }
}

// one thread's float4 of a round's depthwise weights (k*k*rc/4 of them)
__device__ __forceinline__ float4 load_wd(const CbLayer& L, int c0, int rc) {
  const int i = threadIdx.x, nq = rc / 4;
  if (i >= L.k * L.k * nq) return make_float4(0.f, 0.f, 0.f, 0.f);
  const int t = i / nq, qq = i - t * nq;
  return *reinterpret_cast<const float4*>(L.wd + (size_t)t * L.Ep + c0 + qq * 4);
}
__device__ __forceinline__ void store_wd(const CbLayer& L, float* WD, int rc, float4 v) {
  const int i = threadIdx.x, nq = rc / 4;
  if (i >= L.k * L.k * nq) return;
  const int t = i / nq, qq = i - t * nq;
  *reinterpret_cast<float4*>(WD + t * RW + qq * 4) = v;
}

// the expand + depthwise rounds of one block; leaves MEAN [Ep] (channel
// means of the depthwise output) and max|d| in MISC[1].  Round r+1's expand
// weights, bias and depthwise weights are loaded into registers while round
// r's depthwise runs.
template <int KC>
__device__ void block_rounds(const CbLayer& L, const Smem& s, float* D, int ex, unsigned long long* stamps, int& st,
                             int& st2, int dbg) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r16 = lane & 15, g = lane >> 4;
  const int Pin = L.Hi * L.Wi, Po = L.Ho * L.Wo, mtin = (Pin + 15) / 16, nt = wave & 3;
  const float eunsc = ldexpf(1.f, -(ex + L.we_exp));
  const int nr = (L.Ep + RW - 1) / RW;
  BFrag<KC> bcur, bnext;
  load_bfrag<KC>(L, 0, min(RW, L.Ep), bcur);
  float4 wdr = load_wd(L, 0, min(RW, L.Ep));
  int rc_prev = 0;
  for (int r = 0; r < nr; ++r) {
    const int c0 = r * RW, rc = min(RW, L.Ep - c0);
    store_wd(L, s.WD, rc, wdr);
    if (tid < rc_prev) {   // channel means of round r - 1, wave partials summed in wave order
      float sum = 0.f;
#pragma unroll 4
      for (int w = 0; w < NW; ++w) sum += s.RED[w * RW + tid];
      s.MEAN[c0 - RW + tid] = sum / (float)Po;
    }
    // expand: wave (N tile nt, M tiles wave / 4 + 4 i), B fragments in registers
    if (nt * 16 < rc) {
      for (int mt = wave >> 2; mt < mtin; mt += NW / 4) {
        const int pxa = min(mt * 16 + r16, Pin - 1);
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          const f16x8 ah = *reinterpret_cast<const f16x8*>(xs_unit(s.XS, Pin, kc, pxa, g));
          const f16x8 al = *reinterpret_cast<const f16x8*>(xs_unit(s.XS, Pin, kc, pxa, 4 + g));
          acc = mma3(ah, al, bcur.h[kc], bcur.l[kc], acc);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int px = mt * 16 + g * 4 + i;
          if (px < Pin) s.E[px * ESTR + nt * 16 + r16] = hswish(fmaf(acc[i], eunsc, bcur.bias));
        }
      }
    }
    if (dbg & 2) lds_barrier();
    else __syncthreads();
    if (st2 < 64) cstamp(stamps, 64 + st2);
    ++st2;
    if (r + 1 < nr) {   // next round's operands in flight during this depthwise
      const int rcn = min(RW, L.Ep - c0 - RW);
      load_bfrag<KC>(L, c0 + RW, rcn, bnext);
      wdr = load_wd(L, c0 + RW, rcn);
    }
    if (L.s == 1) depthwise_round<5, 1, 4>(L, s.E, s.WD, D, s.RED, &s.MISC[1], c0, rc, dbg);
    else depthwise_round<5, 2, 2>(L, s.E, s.WD, D, s.RED, &s.MISC[1], c0, rc, dbg);
    if (dbg & 2) lds_barrier();
    else __syncthreads();
    if (st2 < 64) cstamp(stamps, 64 + st2);
    ++st2;
    bcur = bnext;
    rc_prev = rc;
  }
  if (tid < rc_prev) {
    float sum = 0.f;
#pragma unroll 4
    for (int w = 0; w < NW; ++w) sum += s.RED[w * RW + tid];
    s.MEAN[(nr - 1) * RW + tid] = sum / (float)Po;
  }
  cstamp(stamps, st++);
  __syncthreads();
}

// squeeze-excitation: SC[c] = hardsigmoid(b2 + W2 relu(b1 + W1 mean)), 0 for
// c >= C.  fc1: item (j, part of 8), strided channels, the 8 parts of a j in
// adjacent lanes reduced by a fixed butterfly; fc2: item (channel quad, j
// group), group partials through LDS (E is free) summed in group order.
__device__ void squeeze_excite(const CbLayer& L, const Smem& s) {
  const int tid = threadIdx.x;
  for (int it = tid; it < ((L.sq * 8 + 63) / 64) * 64; it += NT) {   // whole waves per pass (shuffles)
    const int j = it >> 3, part = it & 7;
    float acc = 0.f;
    if (j < L.sq) {
      const float* w = L.w1 + (size_t)j * L.C;
#pragma unroll 8
      for (int c = part; c < L.C; c += 8) acc = fmaf(w[c], s.MEAN[c], acc);
    }
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
    acc += __shfl_xor(acc, 4, 64);
    if (j < L.sq && part == 0) s.HID[j] = fmaxf(acc + L.b1[j], 0.f);
  }
  __syncthreads();
  const int nq = L.C / 4, jg = max(1, min(16, NT / nq)), jper = (L.sq + jg - 1) / jg;
  float* part = s.E;   // [jg][C]
  for (int it = tid; it < nq * jg; it += NT) {
    const int q = it % nq, grp = it / nq, j0 = grp * jper, j1 = min(L.sq, j0 + jper);
    float4 a4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
    for (int j = j0; j < j1; ++j) {
      const float4 w = *reinterpret_cast<const float4*>(L.w2t + (size_t)j * L.C + q * 4);
      const float h = s.HID[j];
      a4.x = fmaf(w.x, h, a4.x); a4.y = fmaf(w.y, h, a4.y); a4.z = fmaf(w.z, h, a4.z); a4.w = fmaf(w.w, h, a4.w);
    }
    *reinterpret_cast<float4*>(part + (size_t)grp * L.C + q * 4) = a4;
  }
  __syncthreads();
  for (int c = tid; c < L.EpK; c += NT) {
    float t = 0.f;
    if (c < L.C) {
      for (int grp = 0; grp < jg; ++grp) t += part[(size_t)grp * L.C + c];
      s.SC[c] = kpd_hsigmoid(t + L.b2[c]);
    } else {
      s.SC[c] = 0.f;
    }
  }
  __syncthreads();
}

// project 1x1: X[px][o] = (D * s)[px][:] . Wp[o][:] 2^-(ed + wp_exp) + bp (+ X)
// unit = (M tile, NG N tiles); the K loop is software-pipelined two chunks
// deep (each chunk: 8 d values of the lane's row + NG B fragments)
template <int NG>
__device__ __forceinline__ void proj_load(const float* drow, const char* wbase, int kc, int kcp, float4& d0, float4& d1,
                                          f16x8 (&bh)[NG], f16x8 (&bl)[NG]) {
  // always in bounds (rows are EpK wide); channels >= Ep are zeroed in proj_compute
  d0 = *reinterpret_cast<const float4*>(drow + kc * 32);
  d1 = *reinterpret_cast<const float4*>(drow + kc * 32 + 4);
#pragma unroll
  for (int j = 0; j < NG; ++j) {
    const char* wr = wbase + ((size_t)j * 16 * kcp + kc) * 128;
    bh[j] = *reinterpret_cast<const f16x8*>(wr);
    bl[j] = *reinterpret_cast<const f16x8*>(wr + 64);
  }
}

template <int NG>
__device__ __forceinline__ void proj_compute(const float* SC, int kc, int g, float dsc, bool live, float4 d0, float4 d1,
                                             const f16x8 (&bh)[NG], const f16x8 (&bl)[NG], f32x4 (&acc)[NG]) {
  const float4 s0 = *reinterpret_cast<const float4*>(SC + (live ? kc * 32 + g * 8 : 0));
  const float4 s1 = *reinterpret_cast<const float4*>(SC + (live ? kc * 32 + g * 8 + 4 : 0));
  if (!live) {   // padding channels of D hold no data: SC is 0 there, but 0 * garbage may be NaN
    d0 = make_float4(0.f, 0.f, 0.f, 0.f);
    d1 = d0;
  }
  f16x8 ah, al;
  {
    const float v0 = d0.x * s0.x * dsc, v1 = d0.y * s0.y * dsc, v2 = d0.z * s0.z * dsc, v3 = d0.w * s0.w * dsc;
    const float v4 = d1.x * s1.x * dsc, v5 = d1.y * s1.y * dsc, v6 = d1.z * s1.z * dsc, v7 = d1.w * s1.w * dsc;
    ah[0] = (_Float16)v0; ah[1] = (_Float16)v1; ah[2] = (_Float16)v2; ah[3] = (_Float16)v3;
    ah[4] = (_Float16)v4; ah[5] = (_Float16)v5; ah[6] = (_Float16)v6; ah[7] = (_Float16)v7;
    al[0] = (_Float16)(v0 - (float)ah[0]); al[1] = (_Float16)(v1 - (float)ah[1]);
    al[2] = (_Float16)(v2 - (float)ah[2]); al[3] = (_Float16)(v3 - (float)ah[3]);
    al[4] = (_Float16)(v4 - (float)ah[4]); al[5] = (_Float16)(v5 - (float)ah[5]);
    al[6] = (_Float16)(v6 - (float)ah[6]); al[7] = (_Float16)(v7 - (float)ah[7]);
  }
#pragma unroll
  for (int j = 0; j < NG; ++j) acc[j] = mma3(ah, al, bh[j], bl[j], acc[j]);
}

// project 1x1: X[px][o] = (D * s)[px][:] . Wp[o][:] 2^-(ed + wp_exp) + bp (+ X)
// unit = (M tile, NG N tiles); the K loop is software-pipelined two chunks
// deep (each chunk: 8 d values of the lane's row + NG B fragments)
template <int NG>
__device__ void project(const CbLayer& L, const Smem& s, const float* D) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r16 = lane & 15, g = lane >> 4;
  const int Po = L.Ho * L.Wo, mto = (Po + 15) / 16, ntiles = L.cout_p / 16, kcp = L.EpK / 32;
  const int units = mto * (ntiles / NG);
  const int ed = split_exp_of(__uint_as_float(s.MISC[1]));
  const float dsc = ldexpf(1.f, ed), punsc = ldexpf(1.f, -(ed + L.wp_exp));
  float m = 0.f;
  for (int u = wave; u < units; u += NW) {
    const int mt = u % mto, nt0 = (u / mto) * NG;
    const int pxa = min(mt * 16 + r16, Po - 1);
    const float* drow = D + (size_t)pxa * L.EpK + g * 8;
    const char* wbase = reinterpret_cast<const char*>(L.wp) + ((size_t)(nt0 * 16 + r16) * kcp) * 128 + g * 16;
    f32x4 acc[NG];
#pragma unroll
    for (int j = 0; j < NG; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float4 da0, da1, db0, db1;
    f16x8 bha[NG], bla[NG], bhb[NG], blb[NG];
    // straight-line double-buffered loop: every load unconditional (the chunk
    // index clamped; an out-of-range chunk computes with live = false, i.e. a
    // zero A), so the compiler's vmcnt waits stay exact across iterations
    proj_load<NG>(drow, wbase, 0, kcp, da0, da1, bha, bla);
    proj_load<NG>(drow, wbase, min(1, kcp - 1), kcp, db0, db1, bhb, blb);
    for (int kc = 0; kc < kcp; kc += 2) {
      proj_compute<NG>(s.SC, kc, g, dsc, kc * 32 + g * 8 < L.Ep, da0, da1, bha, bla, acc);
      proj_load<NG>(drow, wbase, min(kc + 2, kcp - 1), kcp, da0, da1, bha, bla);
      proj_compute<NG>(s.SC, kc + 1, g, dsc, kc + 1 < kcp && (kc + 1) * 32 + g * 8 < L.Ep, db0, db1, bhb, blb, acc);
      proj_load<NG>(drow, wbase, min(kc + 3, kcp - 1), kcp, db0, db1, bhb, blb);
    }
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      const int oc = (nt0 + j) * 16 + r16;
      const float bj = L.bp[oc];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int px = mt * 16 + g * 4 + i;
        if (px < Po) {
          float v = fmaf(acc[j][i], punsc, bj);
          if (L.res) v += s.X[(size_t)px * L.cout_p + oc];
          s.X[(size_t)px * L.cout_p + oc] = v;
          m = fmaxf(m, fabsf(v));
        }
      }
    }
  }
  lds_max(&s.MISC[0], m);
}

__global__ __launch_bounds__(NT) void cbody_kernel(const CbodyArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const CbLds o = cb_layout(a);
  Smem s;
  s.X = reinterpret_cast<float*>(lds + o.x);
  s.XS = lds + o.xs;
  s.E = reinterpret_cast<float*>(lds + o.e);
  s.WD = reinterpret_cast<float*>(lds + o.wd);
  s.RED = reinterpret_cast<float*>(lds + o.red);
  s.MEAN = reinterpret_cast<float*>(lds + o.mean);
  s.SC = reinterpret_cast<float*>(lds + o.sc);
  s.HID = reinterpret_cast<float*>(lds + o.hid);
  s.MISC = reinterpret_cast<unsigned*>(lds + o.misc);   // [0] max|X| bits, [1] max|d| bits
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  float* D = a.dscr + (size_t)n * a.dscr_floats;
  int st = 0, st2 = 0;   // stamp slots: phases 0.., rounds 64..
  cstamp(a.stamps, st++);
  if (tid < 16) s.MISC[tid] = 0u;
  __syncthreads();
  {   // X = features.4 output
    const int nx4 = a.L[0].Hi * a.L[0].Wi * a.L[0].cin_p / 4;
    const float4* src = reinterpret_cast<const float4*>(a.x) + (size_t)n * nx4;
    float m = 0.f;
    for (int i = tid; i < nx4; i += NT) {
      const float4 v = src[i];
      reinterpret_cast<float4*>(s.X)[i] = v;
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    lds_max(&s.MISC[0], m);
  }
  __syncthreads();
  for (int l = 0; l < a.nl; ++l) {
    const CbLayer L = a.L[l];
    const int Pin = L.Hi * L.Wi, Po = L.Ho * L.Wo;
    const int ex = build_xs(s.X, s.XS, Pin, L.cin_p, L.kc_in, &s.MISC[0]);
    __syncthreads();
    if (tid == 0) { s.MISC[0] = 0u; s.MISC[1] = 0u; }
    cstamp(a.stamps, st++);
    if (L.kc_in == 2) block_rounds<2>(L, s, D, ex, a.stamps, st, st2, a.dbg);
    else block_rounds<3>(L, s, D, ex, a.stamps, st, st2, a.dbg);
    squeeze_excite(L, s);
    cstamp(a.stamps, st++);
    const int mto = (Po + 15) / 16;
    if (mto >= 8 && L.cout_p % 48 == 0) project<3>(L, s, D);
    else project<1>(L, s, D);
    __syncthreads();
    cstamp(a.stamps, st++);
    if (L.tap) {   // FPN tap (features.8 output)
      const int n4 = Po * L.cout_p / 4;
      float4* dst = reinterpret_cast<float4*>(L.tap) + (size_t)n * n4;
      for (int i = tid; i < n4; i += NT) dst[i] = reinterpret_cast<const float4*>(s.X)[i];
    }
  }
  // features.12: 1x1 96 -> 576 + hardswish -> tap3; unit = (M tile, 4 N tiles),
  // the unit's B fragments of all K chunks loaded before its MFMAs, the next
  // unit's while this one computes
  {
    const CbLayer& Z = a.L[a.nl - 1];
    const int P = Z.Ho * Z.Wo, kcl = a.last_kc;
    const int ex = build_xs(s.X, s.XS, P, a.last_cin_p, kcl, &s.MISC[0]);
    __syncthreads();
    const float unsc = ldexpf(1.f, -(ex + a.wl_exp));
    const int mt_n = (P + 15) / 16, ngr = a.last_cout / 64, units = mt_n * ngr;
    float* out = a.tap3 + (size_t)n * P * a.last_cout;
    constexpr int KL = 3;   // launch_cbody checks last_kc == 3
    struct LStage { f16x8 h[4][KL], l[4][KL]; float b[4]; };
    auto load = [&](int u, LStage& S) {
      const int c0 = (u / mt_n) * 64;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int oc = c0 + j * 16 + r16;
        const char* wr = reinterpret_cast<const char*>(a.wl) + (size_t)oc * KL * 128 + g * 16;
#pragma unroll
        for (int kc = 0; kc < KL; ++kc) {
          S.h[j][kc] = *reinterpret_cast<const f16x8*>(wr + kc * 128);
          S.l[j][kc] = *reinterpret_cast<const f16x8*>(wr + kc * 128 + 64);
        }
        S.b[j] = a.bl[oc];
      }
    };
    LStage S;
    load(min(wave, units - 1), S);
    for (int u = wave; u < units; u += NW) {
      const int mt = u % mt_n, c0 = (u / mt_n) * 64;
      const int pxa = min(mt * 16 + r16, P - 1);
      f32x4 acc[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KL; ++kc) {
        const f16x8 ah = *reinterpret_cast<const f16x8*>(xs_unit(s.XS, P, kc, pxa, g));
        const f16x8 al = *reinterpret_cast<const f16x8*>(xs_unit(s.XS, P, kc, pxa, 4 + g));
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = mma3(ah, al, S.h[j][kc], S.l[j][kc], acc[j]);
      }
      float bb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bb[j] = S.b[j];
      load(min(u + NW, units - 1), S);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int oc = c0 + j * 16 + r16;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int px = mt * 16 + g * 4 + i;
          if (px < P) out[(size_t)px * a.last_cout + oc] = hswish(fmaf(acc[j][i], unsc, bb[j]));
        }
      }
    }
  }
  cstamp(a.stamps, st++);
}

}  // namespace

size_t cbody_lds_bytes(const CbodyArgs& a) { return (size_t)cb_layout(a).total; }

hipError_t launch_cbody(const CbodyArgs& a, int N, hipStream_t st) {
  if (N <= 0) return hipSuccess;
  if (a.nl < 1 || a.nl > kCbMaxLayers || !a.x || !a.tap3 || !a.dscr || !a.wl || !a.bl || a.last_cout % 64 ||
      a.last_kc != 3 || a.last_kc * 32 < a.last_cin_p)
    return hipErrorInvalidValue;
  long dneed = 0;
  for (int l = 0; l < a.nl; ++l) {
    const CbLayer& L = a.L[l];
    const bool ok = L.act == ACT_HSWISH && (L.kc_in == 2 || L.kc_in == 3) && L.cin_p % 16 == 0 && L.kc_in * 32 >= L.cin_p && L.Ep % 16 == 0 && L.EpK % 32 == 0 &&
                    L.EpK >= L.Ep && L.Ep <= kMaxEp && L.EpK <= kMaxEp && L.C <= L.Ep && L.cout_p % 16 == 0 &&
                    L.cout_p <= 96 && L.k == 5 && (L.s == 1 || L.s == 2) && L.sq <= kMaxSq &&
                    L.we && L.be && L.wd && L.bd && L.wp && L.bp && (!L.se || (L.w1 && L.b1 && L.w2t && L.b2)) &&
                    (!L.res || (L.cin_p == L.cout_p && L.Hi == L.Ho && L.Wi == L.Wo)) &&
                    (l == 0 || (a.L[l - 1].Ho == L.Hi && a.L[l - 1].Wo == L.Wi && a.L[l - 1].cout_p == L.cin_p));
    if (!ok) return hipErrorInvalidValue;
    dneed = std::max(dneed, (long)L.Ho * L.Wo * L.EpK);
  }
  if (dneed > a.dscr_floats || a.L[a.nl - 1].cout_p != a.last_cin_p) return hipErrorInvalidValue;
  const size_t lds = cbody_lds_bytes(a);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(cbody_kernel, dim3(N), dim3(NT), lds, st, a);
  return hipGetLastError();
}
