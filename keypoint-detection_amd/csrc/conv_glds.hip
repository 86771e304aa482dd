// 16-bit-operand implicit-GEMM convolution with LDS-DMA staging (gfx950).
//
//   out[m, co] = act( scale * sum_k A[m, k] * Bw[co, k] + bias[co] )
//   m = pixel (n, y, x) of an NHWC tensor, k = (tap, ci), tap = (ky, kx)
//
// Users (reference file:line):
//   * FPN level-0 3x3 128->128 + BN + ReLU (dll/models/backbone.py:20-27,39),
//     fp32-accurate "split" mode: every operand is carried as f16 hi + lo
//     (x*s = hi + lo, power-of-two s) and each 16x16x32 k-step issues three
//     v_mfma_f32_16x16x32_f16 (hi*lo, lo*hi, hi*hi) into one fp32 accumulator;
//     f16 x f16 products are exact in fp32 and the dropped lo*lo term is
//     ~2^-22 relative, so the result matches an fp32 conv to fp32 rounding.
//     That keeps ChannelAttention's top-64 channel ORDER (keypoint_model.py:
//     653-661) identical to the reference.
//   * HeatmapHead 3x3 convs 64->256->256->64 (dll/models/heatmap_head.py:
//     31-45,55-66) in bf16 ("mixed" precision), v_mfma_f32_16x16x32_bf16.
//
// Design (DESIGN.md "K6b"):
//   * 512-thread workgroups (8 waves, 2 per SIMD at one workgroup per CU),
//     BM = 256 pixels x BN in {64,128,256} output channels; every wave owns a
//     (256/WAVES_M) x 64 tile of 16x16 fragments.
//   * One K-tile = one 128-byte row per pixel / per output channel: 64 bf16
//     input channels of one tap, or (split) 32 channels as [hi32 | lo32] f16
//     -- the producer writes that interleaved layout, so staging is a pure copy.
//   * Staging is LDS-DMA (buffer_load_dwordx4 ... lds): no VGPRs, no
//     ds_write, no VALU conversion.  The 3x3 halo and the M tail come from the
//     buffer descriptor's range check (an out-of-range offset loads zeros).
//     The LDS image is XOR-swizzled (16-byte chunk c of row r at c ^ (r & 7),
//     conflict-free ds_read_b128) by permuting the per-lane SOURCE chunk,
//     because an LDS-DMA writes 1 KiB lane-linearly.
//   * S-stage ring with a counted s_waitcnt vmcnt and a raw s_barrier: S-1
//     K-tiles are in flight while the MFMAs of the current one run, and the
//     single barrier per K-tile never drains the pipeline.
//   * Epilogue (fp32 out) straight from the accumulators: fused bias / ReLU /
//     unscale, channel sum+max by cross-lane reduction (+ a 2*WAVES_M*BN-float
//     LDS exchange), and a DPP quad transpose for 16-byte row stores; bf16
//     outputs stage the tile through LDS (conv_epilogue.h), which measured
//     faster for them.
#include <algorithm>
#include <type_traits>

#include "kpd_common.h"
#include "kpd_kernels.h"
#include "conv_epilogue.h"
#include "kpd_dma.h"

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int BM = 256, NT = 512, ROWB = 128;
constexpr unsigned OOB = 0x80000000u;   // out-of-range voffset: the buffer load returns 0

// diagnostic phase stamps (KPD_STAMPS): thread 0 records s_memrealtime
__device__ __forceinline__ void stamp16(unsigned long long* st, int i, unsigned long long v = 0, int row = -1) {
  if (st && threadIdx.x == 0)
    st[(size_t)(row < 0 ? blockIdx.x : row) * 8 + i] = v ? v : __builtin_amdgcn_s_memrealtime();
}

// 4x4 transpose inside each quad of lanes: lane t holds v[e] = C[e][t] of a
// 4x4 block on entry and C[t][e] on exit (two DPP butterflies, xor 1 / xor 2).
// Turns a 16x16 MFMA accumulator (a lane = 4 rows of one column) into a lane =
// 4 consecutive columns of one row, i.e. one 16-byte store per row piece.
__device__ __forceinline__ float dpp_xor1(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, true));   // quad_perm 1,0,3,2
}
__device__ __forceinline__ float dpp_xor2(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x4E, 0xF, 0xF, true));   // quad_perm 2,3,0,1
}
template <int N>
__device__ __forceinline__ float dpp_row_ror(float x) {   // row rotate right: lane l <- lane (l - N) mod 16
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x120 + N, 0xF, 0xF, false));
}
// x + (lane l ^ 4) + (lane l ^ 8) + (lane l ^ 12) within a 16-lane row as a
// symmetric butterfly: every lane of the group computes (x_a + x_b) + (x_c +
// x_d) with the same pairs, so the sum is bit-identical in all four lanes and
// does not depend on which lane a pixel landed in (a rotation sum associates
// differently per lane: a result would then depend on the pixel's position in
// the tile, i.e. on what the ROI is batched with).  xor 4 = ror 4 or ror 12
// by bit 2 of the lane (l ^ 4 = l - 4 when bit 2 is set); xor 8 = ror 8.
// Both rotations run unconditionally with the whole wave active and a plain
// select picks one: a DPP inside a divergent branch reads the inactive lanes
// of the other side as 0.
__device__ __forceinline__ float dpp_sum_xor4_8(float x, int lane) {
  const float r4 = dpp_row_ror<4>(x), r12 = dpp_row_ror<12>(x);
  const unsigned sel = 0u - (unsigned)((lane >> 2) & 1);
  const float u = __uint_as_float((__float_as_uint(r4) & sel) | (__float_as_uint(r12) & ~sel));
  const float s = x + u;
  return s + dpp_row_ror<8>(s);
}
// 1 / (1 + e^-v) with the hardware reciprocal and one Newton step (within an
// ulp or two of the IEEE quotient; the division sequence is ~10 instructions)
// For v < ~-88, e^-v overflows: d = inf, rcp = 0 and the Newton step would
// give 0 * (1 - inf * 0) = NaN, so that case returns 0 like 1 / inf does.
__device__ __forceinline__ float sigmoid_rcp(float v) {
  const float d = 1.f + expf(-v);
  const float r = __builtin_amdgcn_rcpf(d);
  return d < INFINITY ? fmaf(r, fmaf(-d, r, 1.f), r) : 0.f;
}
__device__ __forceinline__ void quad_transpose(f32x4& v, int t) {
  const bool b0 = t & 1, b1 = t & 2;
  float r = dpp_xor1(b0 ? v[0] : v[1]);
  if (b0) v[0] = r; else v[1] = r;
  r = dpp_xor1(b0 ? v[2] : v[3]);
  if (b0) v[2] = r; else v[3] = r;
  r = dpp_xor2(b1 ? v[0] : v[2]);
  if (b1) v[0] = r; else v[2] = r;
  r = dpp_xor2(b1 ? v[1] : v[3]);
  if (b1) v[1] = r; else v[3] = r;
}

// DBG (kpd_bench_conv16 only): 1 = no LDS-DMA in the K loop, 2 = no MFMA,
// 4 = every block reads the same 256 A rows (L2-resident working set),
// 8 = no epilogue (one value per lane stored), 16 = no K loop
template <bool SPLIT, typename TO, int KS, int BN, int S, bool PF, int DBG = 0>
__global__ __launch_bounds__(NT) void conv16_kernel(const Conv16Args p) {
  constexpr int WAVES_N = BN / 64, WAVES_M = 8 / WAVES_N;
  constexpr int WM = BM / WAVES_M, FM = WM / 16, FN = 4;
  constexpr int A_LD = 4, B_LD = BN / 64;          // LDS-DMA wave-instructions per K-tile per wave
  constexpr int LPT = A_LD + B_LD;
  constexpr int STAGE = (BM + BN) * ROWB;
  constexpr int RING = S * STAGE;
  // bf16 outputs keep the LDS-staged epilogue (conv_epilogue.h: measured 3%
  // faster there); fp32 outputs use the register epilogue (1% faster on
  // FPN0).  DBG 4096 forces the staged one for A/B runs.
  constexpr bool STAGED = !std::is_same<TO, float>::value || (DBG & 4096) != 0;
  constexpr int EPI_BN = BN > 128 ? 128 : BN;
  constexpr int EPI = STAGED ? epi_lds_bytes<BM, EPI_BN, NT>() : 0;
  constexpr int LDS_REG = RING + 2 * WAVES_M * BN * 4;   // ring + the register epilogue's statistics exchange
  constexpr int LDS = LDS_REG > EPI ? LDS_REG : EPI;
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static_assert(S >= 2 && (S - 2) * LPT < 64, "stages");
  __shared__ __attribute__((aligned(1024))) char lds[LDS];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int NTL = p.cout_p / BN;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (L / NTL) * BM, n0 = (L % NTL) * BN;
  const int H = p.H, W = p.W, HW = H * W, M = p.M;
  const int cin_e = p.cin_e;

  const i32x4 rin = make_rsrc(p.in, p.in_bytes), rwt = make_rsrc(p.wt, p.wt_bytes);
  // wave-uniform LDS byte address of this wave's first A / B staging row
  const unsigned lds0 = (unsigned)reinterpret_cast<unsigned long long>((lds_void*)lds);
  const unsigned a_dst = __builtin_amdgcn_readfirstlane(lds0 + wave * 32 * ROWB);
  const unsigned b_dst = __builtin_amdgcn_readfirstlane(lds0 + (BM + wave * (BN / 8)) * ROWB);

  // LDS-DMA geometry: one wave-instruction fills 8 rows x 128 B; lane l lands
  // in row (l >> 3), physical chunk (l & 7), so it fetches logical chunk
  // (l & 7) ^ (row & 7) of that row (rows start at multiples of 8).
  const int lrow = lane >> 3, lchunk = (lane & 7) ^ lrow;
  unsigned a_off[A_LD], a_taps[A_LD];
#pragma unroll
  for (int i = 0; i < A_LD; ++i) {
    const int m = m0 + wave * 32 + i * 8 + lrow;
    a_off[i] = 0;
    a_taps[i] = 0;
    if (m < M) {
      const int n = m / HW, r = m - n * HW, y = r / W, x = r - y * W;
      const int ms = (DBG & 4) ? (m % BM) + W + 1 : m;
      a_off[i] = (unsigned)(ms * p.in_cstride * 2 + lchunk * 16);
#pragma unroll
      for (int t = 0; t < KS * KS; ++t) {
        const int yy = y + t / KS - KS / 2, xx = x + t % KS - KS / 2;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W) a_taps[i] |= 1u << t;
      }
    }
  }
  unsigned b_off[B_LD];
#pragma unroll
  for (int i = 0; i < B_LD; ++i) {
    const int co = n0 + wave * (BN / 8) + i * 8 + lrow;
    b_off[i] = (unsigned)((co * KS * KS * cin_e) * 2 + lchunk * 16);
  }
  const int kc_per_tap = cin_e / 64;
  const int KT = (DBG & 16) ? 0 : KS * KS * kc_per_tap;
  // fused final layer: its [17][64] weights + [17] bias, loaded now (3 per
  // thread) so the epilogue does not wait on a global round trip
  float fin_pre[3] = {0.f, 0.f, 0.f};
  if constexpr (BN == 64 && std::is_same<TO, float>::value) {
    if (p.fin_w) {
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int i = tid + u * NT;
        if (i < 17 * 64) fin_pre[u] = p.fin_w[i];
        else if (i < 17 * 65) fin_pre[u] = p.fin_b[i - 17 * 64];
      }
    }
  }

  // loader state (wave-uniform): next K-tile to issue as (tap, kc)
  int ld_tap = 0, ld_kc = 0;
  auto issue = [&](int stage) {
    if constexpr ((DBG & 1) != 0) return;
    const int dy = ld_tap / KS - KS / 2, dx = ld_tap % KS - KS / 2;
    const int delta = ((dy * W + dx) * p.in_cstride + ld_kc * 64) * 2;
    const unsigned so = stage * STAGE;
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const unsigned voff = ((a_taps[i] >> ld_tap) & 1u) ? a_off[i] + delta : OOB;
      glds16(rin, a_dst + so + i * 8 * ROWB, voff, 0);
    }
    const int soff = (ld_tap * cin_e + ld_kc * 64) * 2;
#pragma unroll
    for (int i = 0; i < B_LD; ++i) glds16(rwt, b_dst + so + i * 8 * ROWB, b_off[i], soff);
    // taps inner, channel chunks outer: the 9 shifted reads of one chunk's
    // halo rows come in 9 consecutive K-tiles and hit the XCD's L2
    if (++ld_tap == KS * KS) {
      ld_tap = 0;
      ++ld_kc;
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, r16 = lane & 15;
  const int a_row = (wm * WM + r16) * ROWB, b_row = (BM + wn * 64 + r16) * ROWB;
  // A K-tile row is 8 chunks; lane group g reads chunk g (q = 0) and 4 + g
  // (q = 1): bf16 = k-steps 0 / 1, split = hi / lo of one 32-channel k-step.
  const int ch0 = ((g ^ (r16 & 7)) << 4), ch1 = (((4 + g) ^ (r16 & 7)) << 4);
  struct Frag {
    uint4 a[2][FM], b[2][FN];
  };
  auto load_frags = [&](int stage, Frag& f) {
    const char* sb = lds + stage * STAGE;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      f.a[0][i] = *reinterpret_cast<const uint4*>(sb + a_row + i * 16 * ROWB + ch0);
      f.a[1][i] = *reinterpret_cast<const uint4*>(sb + a_row + i * 16 * ROWB + ch1);
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      f.b[0][j] = *reinterpret_cast<const uint4*>(sb + b_row + j * 16 * ROWB + ch0);
      f.b[1][j] = *reinterpret_cast<const uint4*>(sb + b_row + j * 16 * ROWB + ch1);
    }
  };
  auto mma = [&](const Frag& f) {
    if constexpr ((DBG & 2) != 0) {
      acc[0][0][0] += __uint_as_float(f.a[0][0].x ^ f.b[1][FN - 1].w);   // keep the fragment reads alive
      return;
    }
    if constexpr (SPLIT) {
      // three passes over the accumulators so consecutive MFMAs are independent
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, f.a[0][i]),
                                                             __builtin_bit_cast(f16x8, f.b[1][j]), acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, f.a[1][i]),
                                                             __builtin_bit_cast(f16x8, f.b[0][j]), acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, f.a[0][i]),
                                                             __builtin_bit_cast(f16x8, f.b[0][j]), acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, f.a[q][i]),
                                                                __builtin_bit_cast(bf16x8, f.b[q][j]), acc[i][j], 0,
                                                                0, 0);
    }
  };
  auto tile_ready = [&](int k) {   // every wave's LDS-DMA of tile k landed + all fragment reads done
    if (k + S - 2 < KT) wait_vmcnt<(S - 2) * LPT>();
    else wait_vmcnt<0>();
    // lgkmcnt(0) as the builtin (vmcnt/expcnt fields at max), so hipcc knows the
    // fragment registers are complete and adds no waits inside the MFMA block
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < KT) issue(s);
  if constexpr (PF) {
    // Fragment prefetch: after barrier k the waves read tile k+1's fragments
    // while the MFMAs of tile k (already in registers) run, so a barrier never
    // leaves the MFMA pipe waiting on LDS latency.  Tile k+S-1 goes into the
    // stage of tile k-1, whose fragments every wave finished reading before
    // barrier k-1 (lgkmcnt(0) ahead of each barrier).
    Frag f0, f1;
    tile_ready(0);
    load_frags(0, f0);
    int is = S - 1, rs = 1;   // stage the next issue writes / the next fragment read uses
    auto step = [&](int kt, Frag& cur, Frag& nxt) {
      if (kt + S - 1 < KT) issue(is);
      is = is + 1 == S ? 0 : is + 1;
      __builtin_amdgcn_s_waitcnt(0xC07F);   // cur's fragments complete on every path
      if (kt + 1 < KT) {
        tile_ready(kt + 1);
        load_frags(rs, nxt);
        rs = rs + 1 == S ? 0 : rs + 1;
      }
      __builtin_amdgcn_s_setprio(1);
      mma(cur);
      __builtin_amdgcn_s_setprio(0);
    };
    int kt = 0;
    for (; kt + 1 < KT; kt += 2) {
      step(kt, f0, f1);
      step(kt + 1, f1, f0);
    }
    if (kt < KT) step(kt, f0, f1);
  } else if constexpr (!SPLIT && (DBG & 0x10000) == 0) {
    // Half-tile phases (bf16): the two 32-deep k-steps q = 0 / 1 of a K-tile
    // use separate fragment registers, so the reads of one overlap the MFMAs
    // of the other and the pipe never waits on LDS latency behind a barrier:
    //   reads (kt, q1) | MFMAs (kt, q0) | barrier kt+1 | reads (kt+1, q0) | MFMAs (kt, q1)
    // Same registers as one whole-tile fragment set.  The stage of tile kt is
    // free at barrier kt+1 (every wave's reads of it retired by the lgkmcnt(0)
    // in front of that barrier), which is where tile kt+S is issued into it.
    struct Half { uint4 a[FM], b[FN]; };
    auto load_half = [&](int stage, int q, Half& f) {
      const char* sb = lds + stage * STAGE;
      const int chq = q ? ch1 : ch0;
#pragma unroll
      for (int j = 0; j < FN; ++j) f.b[j] = *reinterpret_cast<const uint4*>(sb + b_row + j * 16 * ROWB + chq);
#pragma unroll
      for (int i = 0; i < FM; ++i) f.a[i] = *reinterpret_cast<const uint4*>(sb + a_row + i * 16 * ROWB + chq);
    };
    auto mma_half = [&](const Half& f) {
      if constexpr ((DBG & 2) != 0) {
        acc[0][0][0] += __uint_as_float(f.a[0].x ^ f.b[FN - 1].w);
        return;
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, f.a[i]),
                                                              __builtin_bit_cast(bf16x8, f.b[j]), acc[i][j], 0, 0, 0);
    };
    Half f0, f1;
    int cs = 0, is = S - 1;
    if (KT > 0) {
      tile_ready(0);
      if (S - 1 < KT) issue(is);   // tile S-1 into the never-used stage S-1
      is = is + 1 == S ? 0 : is + 1;
      load_half(0, 0, f0);
    }
    for (int kt = 0; kt < KT; ++kt) {
      load_half(cs, 1, f1);
      __builtin_amdgcn_s_setprio(1);
      mma_half(f0);
      __builtin_amdgcn_s_setprio(0);
      cs = cs + 1 == S ? 0 : cs + 1;
      if (kt + 1 < KT) {
        tile_ready(kt + 1);   // f1 complete, tile kt+1 visible, stage of tile kt free
        if (kt + S < KT) issue(is);
        is = is + 1 == S ? 0 : is + 1;
        load_half(cs, 0, f0);
      } else {
        __builtin_amdgcn_s_waitcnt(0xC07F);
      }
      __builtin_amdgcn_s_setprio(1);
      mma_half(f1);
      __builtin_amdgcn_s_setprio(0);
    }
  } else {
    int cs = 0, is = S - 1;
    for (int kt = 0; kt < KT; ++kt) {
      tile_ready(kt);   // tile kt visible to all; stage of tile kt-1 free
      if (kt + S - 1 < KT) issue(is);
      Frag f;
      load_frags(cs, f);
      mma(f);
      cs = cs + 1 == S ? 0 : cs + 1;
      is = is + 1 == S ? 0 : is + 1;
    }
  }
  __syncthreads();   // all waves leave the K loop together (measured: the stores of early waves slow the rest)
  if constexpr ((DBG & 8) != 0) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    reinterpret_cast<float*>(p.out)[(size_t)blockIdx.x * NT + tid] = s;
    return;
  }

  // ---------------- epilogue ----------------
  float scale = 1.f;
  if constexpr (SPLIT) scale = p.split_scale;
  if constexpr (STAGED) {
    EpiArgs e;
    e.bias = p.bias; e.out = p.out; e.res = nullptr; e.stats = p.stats; e.amax = nullptr; e.scale = scale;
    e.M = M; e.H = H; e.W = W; e.cout_p = p.cout_p; e.out_cstride = p.out_cstride; e.rh = H; e.rw = W;
    e.act = p.act; e.tiles_per_img = p.tiles_per_img;
    e.post_scale = nullptr; e.post_shift = nullptr; e.act2 = 0; e.act3 = 0;
    float* tile = reinterpret_cast<float*>(lds);
    constexpr int HALVES = BN / EPI_BN, WN_PER = EPI_BN / 64;
#pragma unroll
    for (int h = 0; h < HALVES; ++h) {
      if (h) __syncthreads();
      if (wn / WN_PER == h) acc_to_lds<FM, FN, WM, 64, EPI_BN>(tile, acc, wm, wn % WN_PER, lane);
      tile_store<TO, BM, EPI_BN, NT>(tile, e, m0, n0 + h * EPI_BN);
    }
    return;
  }
  // Register epilogue: bias / activation / unscale on the accumulators, the
  // per-tile channel sum+max (top-k statistics) from cross-lane reductions and
  // a small LDS exchange between the WAVES_M waves of a column block, then a
  // DPP quad transpose so each lane stores 16 bytes of one output row.  No
  // LDS staging of the tile, so the ring can stay as it is.
  const int t4 = lane & 3, q4 = r16 >> 2;
  const bool stats = (DBG & 128) == 0 && p.stats != nullptr;   // requires H*W % BM == 0
  float* sts = reinterpret_cast<float*>(lds + RING);            // [2][WAVES_M][BN]
  TO* out = reinterpret_cast<TO*>(p.out);
  // (1) bias + act in place, per-column partials (sum, max) of this wave's
  // rows: lanes 0-15 after the xor-16/32 reductions
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int col = n0 + wn * 64 + j * 16;
    const float bj = p.bias[col + r16];
    float sm = 0.f, mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v = kpd_act(acc[i][j][e] * scale + bj, p.act);
        acc[i][j][e] = v;
        sm += v;
        mx = fmaxf(mx, v);
      }
    if (stats) {
      sm += __shfl_xor(sm, 16);
      mx = fmaxf(mx, __shfl_xor(mx, 16));
      sm += __shfl_xor(sm, 32);
      mx = fmaxf(mx, __shfl_xor(mx, 32));
      if (g == 0) {
        sts[wm * BN + wn * 64 + j * 16 + r16] = sm;
        sts[(WAVES_M + wm) * BN + wn * 64 + j * 16 + r16] = mx;
      }
    }
  }
  // (2) combine the WAVES_M row blocks in a fixed order -- before any output
  // store is issued: a barrier behind the stores waits for the slowest wave's
  // store queue (measured +4 us per tile)
  if (stats) {
    __builtin_amdgcn_s_waitcnt(0xC07F);   // LDS-only barrier (no vmcnt wait)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (tid < BN) {
      float sm = sts[tid], mx = sts[WAVES_M * BN + tid];
#pragma unroll
      for (int w = 1; w < WAVES_M; ++w) {
        sm += sts[w * BN + tid];
        mx = fmaxf(mx, sts[(WAVES_M + w) * BN + tid]);
      }
      const int n = m0 / HW, t = (m0 - n * HW) / BM;
      float* st = p.stats + ((size_t)n * p.tiles_per_img + t) * 2 * p.cout_p;
      st[n0 + tid] = sm;
      st[p.cout_p + n0 + tid] = mx;
    }
  }
  // (3') HeatmapHead final_layer fused (heatmap_head.py:41-45; mixed mode,
  // BN = 64 = all conv-3 channels of a pixel in the tile): per pixel 17 dot
  // products of length 64 + sigmoid, written straight into the reference's
  // [B][P][17][56][56] heatmap at the box's slot (zeros for a padding slot).
  // After the quad transpose a lane holds channels j*16 + 4*q4 .. +3 of one
  // pixel; the 4 lanes of a pixel (q4 = lane bits 2-3) combine by two xor
  // shuffles.  conv 3's own output is never written.
  if constexpr (BN == 64 && std::is_same<TO, float>::value) {
    if (p.fin_w) {
      constexpr int NKF = 17;
      float* fw = reinterpret_cast<float*>(lds);   // [17][64] + [17]: the ring is free after the K loop
      __syncthreads();
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int i = tid + u * NT;
        if (i < NKF * 65) fw[i] = fin_pre[u];
      }
      __syncthreads();
      f32x4 v[FM][FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          v[i][j] = acc[i][j];
          quad_transpose(v[i][j], t4);
        }
      float o[FM][NKF];
#pragma unroll
      for (int k = 0; k < NKF; ++k) {
        float a[FM];
#pragma unroll
        for (int i = 0; i < FM; ++i) a[i] = 0.f;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const float4 w4 = *reinterpret_cast<const float4*>(fw + k * 64 + j * 16 + q4 * 4);
#pragma unroll
          for (int i = 0; i < FM; ++i) {
            a[i] = fmaf(w4.x, v[i][j][0], a[i]); a[i] = fmaf(w4.y, v[i][j][1], a[i]);
            a[i] = fmaf(w4.z, v[i][j][2], a[i]); a[i] = fmaf(w4.w, v[i][j][3], a[i]);
          }
        }
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          a[i] += __shfl_xor(a[i], 4);
          a[i] += __shfl_xor(a[i], 8);
          o[i][k] = a[i];
        }
      }
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int row = m0 + wm * WM + i * 16 + g * 4 + t4;
        if (row < M) {
          const int rl = row / HW, pix = row - rl * HW, r = p.r0 + rl;   // r0: the launch chunk's first ROI
          const int sl = p.slot[r], bimg = r / p.P;
          const int pos = sl >= 0 ? sl : slot_pos(sl);
          float* dst = p.heat + ((size_t)(bimg * p.P + pos) * NKF) * HW + pix;
          // lane q4 stores k = q4, q4 + 4, ... (every store instruction has all lanes active)
#pragma unroll
          for (int s4 = 0; s4 < (NKF + 3) / 4; ++s4) {
            const int k = s4 * 4 + q4;
            float val = q4 == 0 ? o[i][s4 * 4] : 0.f;
            if (s4 * 4 + 1 < NKF && q4 == 1) val = o[i][s4 * 4 + 1];
            if (s4 * 4 + 2 < NKF && q4 == 2) val = o[i][s4 * 4 + 2];
            if (s4 * 4 + 3 < NKF && q4 == 3) val = o[i][s4 * 4 + 3];
            if (k < NKF) dst[(size_t)k * HW] = sl >= 0 ? kpd_sigmoid(val + fw[NKF * 64 + k]) : 0.f;
          }
        }
      }
      return;
    }
  }
  // (3) transposed 16-byte row stores
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      f32x4 v = acc[i][j];
      quad_transpose(v, t4);
      const int row = m0 + wm * WM + i * 16 + g * 4 + t4;
      if (row < M)
        store4<TO>(out + (size_t)row * p.out_cstride + n0 + wn * 64 + j * 16 + q4 * 4,
                   make_float4(v[0], v[1], v[2], v[3]));
    }
}

// ---------------------------------------------------------------- FPN level 0 by linearity
// out = ReLU(conv3x3(lat0) + b) with lat0 = L0(tap0) + up4(lat1) (backbone.py:
// 29-39; the 1x1 laterals have no bias).  Linearity splits the conv into
//   (1) conv3x3 with the composite weights W3.L0 on the 16-channel tap0
//       (K = 9 taps x 16 = 144 instead of 9 x 128), and
//   (2) for output pixel (4Y + a, 4X + b) a sum over the lat1 pixels its nine
//       taps read after the 4x nearest upsample: (Y + oy, X + ox) with the taps
//       that land there summed into one weight matrix -- 1, 2 or 4 groups of
//       128 input channels depending on the position class (a, b).
// Both parts accumulate into the same MFMA tile; the tile's 256 pixels are of
// ONE class (consecutive lat1-grid pixels of one image), so each K-tile has
// one B operand.  2.6x fewer MACs than the 3x3 conv over lat0, and lat0 (403
// MB per step at C2) is never written.  Same fp32-accurate f16 hi/lo products
// as conv16_kernel<split>; zero padding comes from the buffer range checks
// (with an exact 4x upsample the taps outside the image are exactly the lat1
// rows / columns outside the grid).  Register epilogue with the channel
// statistics; rows past the image's class grid are masked out of them.
// DBG (ablations, KPD_FPN0X_DBG; wrong results by design): 1 = no MFMA, 2 = no K-loop DMA,
// 4 = output stores of one piece only (the others go to an out-of-range offset)
template <int DBG>
__global__ __launch_bounds__(NT) void fpn0x_kernel(const Fpn0xArgs p) {
  constexpr int BN = 128, S = 3, WAVES_N = 2, WAVES_M = 4;
  constexpr int WM = BM / WAVES_M, FM = WM / 16, FN = 4;
  constexpr int A_LD = 4, B_LD = BN / 64, LPT = A_LD + B_LD;
  constexpr int STAGE = (BM + BN) * ROWB, RING = S * STAGE;
  // ring | stats exchange [2][WAVES_M][BN] | bias [BN] | class tables (ng, woff, g[4]) x 16
  constexpr int SMISC = RING + 2 * WAVES_M * BN * 4;
  // + per-image unscale + per-image store rectangle (x0 | x1 << 16, y0 | y1 << 16)
  constexpr int LDS = SMISC + BN * 4 + 16 * 6 * 4 + kFpn0xMaxImg * 4 + kFpn0xMaxImg * 8;
  static_assert(LDS <= 160 * 1024, "LDS budget");
  constexpr int KT0 = 5;                          // tap0 K-tiles: taps (2k, 2k+1)
  __shared__ __attribute__((aligned(1024))) char lds[LDS];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int Hf = p.Hf, Wf = p.Wf, rh = p.rh, rw = p.rw, RG = rh * rw;
  // Persistent: one workgroup per CU walks rounds k = 0, 1, ... of the tile
  // space; in round k it takes logical tile k*G + (rb + k) % G.  Within a
  // round the tiles of one XCD are consecutive (xcd_remap) and the position
  // class is fastest, so the 16 classes of an (image, row block) -- which read
  // the same tap0 / lateral-1 pixels -- run together on one XCD and share its
  // L2; the (rb + k) rotation walks every workgroup through the classes, so
  // the per-class K-tile counts (9 / 13 / 21) balance out.  The next tile's
  // first K-tiles are issued right after the K loop, so their LDS-DMA
  // latency overlaps this tile's epilogue.
  const int ntiles = 16 * p.N * p.tpc, G = gridDim.x;
  const int rb = xcd_remap(blockIdx.x, G);
  // Class-half order (p.order == 1): rounds come in pairs over the same G / 8
  // (image, row block) pairs, the first round of a pair taking position
  // classes 0-7, the second 8-15.  An XCD then holds 4 row blocks x 8
  // classes per round: half the per-class weights (the 2.3 MB of 16 classes
  // re-fetched by every XCD every round dominated the kernel's HBM reads),
  // while the row blocks' input rows stay in its L2 for the second half.
  // The (rb + k) rotation still walks each workgroup through the classes.
  const int NJ = p.N * p.tpc, NJR = G >> 3;
  auto tile_at = [&](int k) {
    if (!p.order) return k * G + (rb + k) % G;
    const int r = (rb + k) % G, nj = (k >> 1) * NJR + (r >> 3);
    return nj < NJ ? nj * 16 + (k & 1) * 8 + (r & 7) : ntiles;
  };

  const i32x4 rf = make_rsrc(p.f_split, p.f_bytes), rl = make_rsrc(p.l_split, p.l_bytes);
  const i32x4 rw0 = make_rsrc(p.w0, p.w0_bytes), rwe = make_rsrc(p.weff, p.weff_bytes);
  const __amdgpu_buffer_rsrc_t rout =
      __builtin_amdgcn_make_buffer_rsrc(p.out, (short)0, p.N * Hf * Wf * BN * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rst =
      __builtin_amdgcn_make_buffer_rsrc(p.stats, (short)0, p.N * 16 * p.tpc * 2 * BN * 4, 0x00020000);
  const unsigned lds0 = (unsigned)reinterpret_cast<unsigned long long>((lds_void*)lds);
  const unsigned a_dst = __builtin_amdgcn_readfirstlane(lds0 + wave * 32 * ROWB);
  const unsigned b_dst = __builtin_amdgcn_readfirstlane(lds0 + (BM + wave * (BN / 8)) * ROWB);
  const int lrow = lane >> 3, lchunk = (lane & 7) ^ lrow;
  // once per workgroup: the unscale of the split products (a kernel-wide
  // constant), the bias and the per-class tables in LDS (the per-tile setup
  // then reads LDS instead of dependent kernel-argument loads)
  float* s_bias = reinterpret_cast<float*>(lds + SMISC);
  int* s_ng = reinterpret_cast<int*>(lds + SMISC + BN * 4);
  int* s_woff = s_ng + 16;
  int* s_g = s_ng + 32;   // [16][4]
  if (tid < BN) s_bias[tid] = p.bias[tid];
  if (tid < 16) {
    s_ng[tid] = p.cls_ng[tid];
    s_woff[tid] = p.cls_woff[tid];
#pragma unroll
    for (int gi = 0; gi < kFpn0xMaxGroups; ++gi) s_g[tid * 4 + gi] = p.cls_g[tid][gi];
  }
  // unscale 2^-P of the split products, per image (from that image's own
  // max|tap0| and max|lateral 1|): a table in LDS for the whole launch, so
  // no global load enters the K loop's counted vmcnt waits
  float* s_unscale = reinterpret_cast<float*>(lds + SMISC + BN * 4 + 16 * 6 * 4);
  for (int u = tid; u < p.N; u += NT) {
    int a_f, a_l, P;
    fpn0x_exps(p.sc[(size_t)u * kAmaxStride], p.sc[(size_t)(p.sc_n + u) * kAmaxStride], p.w_exp0, p.w_expE, &a_f,
               &a_l, &P);
    s_unscale[u] = ldexpf(1.f, -P);
  }
  // store rectangle of image u: every pixel roi_align (keypoint_model.py:
  // 212-228; the same corner / extent formulas as roi_row_sample) can read
  // for one of the image's boxes -- rows floor(y1) .. floor(y1 + roi_h) + 1
  // (+ one pixel of margin each side) -- or the whole map without boxes
  int2* s_fp = reinterpret_cast<int2*>(lds + SMISC + BN * 4 + 16 * 6 * 4 + kFpn0xMaxImg * 4);
  for (int u = tid; u < p.N; u += NT) {
    int x0 = 0, x1 = Wf - 1, y0 = 0, y1 = Hf - 1;
    if (p.fp_boxes) {
      x0 = y0 = 1 << 15;
      x1 = y1 = -1;
      for (int q = 0; u < p.fp_NB && q < p.fp_P; ++q) {
        const float* bx = p.fp_boxes + ((size_t)u * p.fp_P + q) * 4;
        const float cx = bx[0], cy = bx[1], bw = bx[2], bh = bx[3];
        if (cx == 0.f && cy == 0.f && bw == 0.f && bh == 0.f) continue;   // skipped box (keypoint_model.py:149-153)
        const float fx1 = fminf(fmaxf(cx - bw / 2.f, 0.f), 1.f) * (float)Wf;
        const float fy1 = fminf(fmaxf(cy - bh / 2.f, 0.f), 1.f) * (float)Hf;
        const float fx2 = fminf(fmaxf(cx + bw / 2.f, 0.f), 1.f) * (float)Wf;
        const float fy2 = fminf(fmaxf(cy + bh / 2.f, 0.f), 1.f) * (float)Hf;
        const float rw_ = fmaxf(fx2 - fx1, 1.f), rh_ = fmaxf(fy2 - fy1, 1.f);
        x0 = min(x0, max((int)floorf(fx1) - 1, 0));
        y0 = min(y0, max((int)floorf(fy1) - 1, 0));
        x1 = max(x1, min((int)floorf(fx1 + rw_) + 2, Wf - 1));
        y1 = max(y1, min((int)floorf(fy1 + rh_) + 2, Hf - 1));
      }
    }
    s_fp[u] = make_int2(x0 | (x1 << 16), y0 | (y1 << 16));
  }
  __syncthreads();
  // this lane's 16-byte piece of a tap0 K-row: chunks 0-1 hi(t1), 2-3 hi(t2),
  // 4-5 lo(t1), 6-7 lo(t2); a tap0 pixel row is [hi16 | lo16] (64 bytes)
  const int f_tsel = (lchunk >> 1) & 1;                       // 0: t1, 1: t2
  const unsigned f_byte = (unsigned)((lchunk >> 2) * 32 + (lchunk & 1) * 16);
  const int co_b = wave * (BN / 8) + lrow;                     // B rows of this lane (+ 8 i)

  // per-tile state
  int cls = 0, n = 0, jt = 0, ca = 0, cb = 0, q0 = 0, NG = 1, KT = 0, ld = 0;
  // masks packed: bits 0-8 = tap0 taps in the image, bits 9-12 = lat1 groups in the grid
  unsigned f_off[A_LD], l_off[A_LD], mask[A_LD];
  const float inv_rw = 1.f / (float)rw;   // q / rw by a float product: exact for q < 2^16 (host check)
  // Per-row offsets and masks of tile L (VALU only, no divides, one uniform
  // LDS read of the class's group table).  Computed for the NEXT tile inside
  // the K loop, where it overlaps the MFMAs, not between tiles where both
  // waves of a SIMD would run it side by side (measured 3.6 us per tile).
  auto rows = [&](int L, unsigned* fo, unsigned* lo, unsigned* mk) {
    const int c = L & 15, nj = L >> 4, nn = nj / p.tpc, j = nj - nn * p.tpc;
    const int a_ = c >> 2, b_ = c & 3, qb = j * BM, ng = s_ng[c];
    const int4 gq = *reinterpret_cast<const int4*>(s_g + c * 4);
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const int q = qb + wave * 32 + i * 8 + lrow;
      const int Y = (int)(((float)q + 0.5f) * inv_rw), X = q - Y * rw, y = 4 * Y + a_, x = 4 * X + b_;
      fo[i] = (unsigned)(((nn * Hf + y) * Wf + x) * 64);
      lo[i] = (unsigned)(((nn * rh + Y) * rw + X) * 512);
      // validity of rows / columns -1, 0, +1 around (y, x) and (Y, X) as 3-bit sets
      const unsigned ry = (y > 0 ? 1u : 0u) | 2u | (y + 1 < Hf ? 4u : 0u);
      const unsigned cx = (x > 0 ? 1u : 0u) | 2u | (x + 1 < Wf ? 4u : 0u);
      const unsigned ryl = (Y > 0 ? 1u : 0u) | 2u | (Y + 1 < rh ? 4u : 0u);
      const unsigned cxl = (X > 0 ? 1u : 0u) | 2u | (X + 1 < rw ? 4u : 0u);
      unsigned m = (ry & 1u ? cx : 0u) | (ry & 2u ? cx << 3 : 0u) | (ry & 4u ? cx << 6 : 0u);
      const int gg[4] = {gq.x, gq.y, gq.z, gq.w};
#pragma unroll
      for (int g = 0; g < kFpn0xMaxGroups; ++g) {
        const int oy1 = (gg[g] * 11) >> 5, ox1 = gg[g] - 3 * oy1;   // gg / 3, gg % 3 for gg < 9
        if (g < ng && ((ryl >> oy1) & (cxl >> ox1) & 1u)) m |= 1u << (9 + g);
      }
      mk[i] = q < RG ? m : 0u;
    }
  };
  auto setup = [&](int L) {
    cls = L & 15;
    const int nj = L >> 4;
    n = nj / p.tpc;
    jt = nj - n * p.tpc;
    ca = cls >> 2;
    cb = cls & 3;
    q0 = jt * BM;                                  // first lat1-grid pixel of the tile
    NG = s_ng[cls];
    KT = KT0 + 4 * NG;
    ld = 0;
  };
  // tap0 K-tile k (taps 2k, 2k+1) of a tile with rows fo / mk (class-independent B)
  auto issue_tap0 = [&](int stage, int k, const unsigned* fo, const unsigned* mk) {
    const unsigned so = stage * STAGE;
    const int t = 2 * k + f_tsel;
    const int dy = t / 3 - 1, dx = t % 3 - 1;
    const int delta = (dy * Wf + dx) * 64 + (int)f_byte;
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const unsigned voff = (t < 9 && ((mk[i] >> t) & 1u)) ? fo[i] + delta : OOB;
      glds16(rf, a_dst + so + i * 8 * ROWB, voff, 0);
    }
#pragma unroll
    for (int i = 0; i < B_LD; ++i)
      glds16(rw0, b_dst + so + i * 8 * ROWB, (unsigned)(((co_b + i * 8) * KT0 + k) * ROWB + lchunk * 16), 0);
  };
  auto issue = [&](int stage) {
    const unsigned so = stage * STAGE;
    if (ld < KT0) {
      issue_tap0(stage, ld, f_off, mask);
    } else {
      const int k = ld - KT0, g = k >> 2, kc = k & 3;
      const int gg = s_g[cls * 4 + g], oy = gg / 3 - 1, ox = gg % 3 - 1;
      const int delta = (oy * rw + ox) * 512 + kc * 128 + lchunk * 16;
#pragma unroll
      for (int i = 0; i < A_LD; ++i) {
        const unsigned voff = ((mask[i] >> (9 + g)) & 1u) ? l_off[i] + delta : OOB;
        glds16(rl, a_dst + so + i * 8 * ROWB, voff, 0);
      }
      const int wbase = s_woff[cls] * 2;   // bytes
#pragma unroll
      for (int i = 0; i < B_LD; ++i)
        glds16(rwe, b_dst + so + i * 8 * ROWB,
               (unsigned)(wbase + (((co_b + i * 8) * NG + g) * 4 + kc) * ROWB + lchunk * 16), 0);
    }
    ++ld;
  };

  f32x4 acc[FM][FN];
  const int g = lane >> 4, r16 = lane & 15;
  const int a_row = (wm * WM + r16) * ROWB, b_row = (BM + wn * 64 + r16) * ROWB;
  const int ch0 = ((g ^ (r16 & 7)) << 4), ch1 = (((4 + g) ^ (r16 & 7)) << 4);
  // One fragment set: a0/a1 (hi/lo of A), b0/b1 (hi/lo of B).  The three
  // product passes of K-tile k run as a1.b0 | a0.b1 | a0.b0, and each
  // register group is refilled with tile k+1 as soon as its last pass of
  // tile k has issued (a1 after pass 1, b1 after pass 2, a0 / b0 after pass
  // 3): the reads of the next tile overlap the MFMAs of this one with half
  // the registers of a double-buffered set (no spills beside the persistent
  // loop's next-tile state).
  uint4 fa0[FM], fa1[FM], fb0[FN], fb1[FN];
  auto rd_a = [&](int stage, int hl, uint4* f) {
    const char* sb = lds + stage * STAGE;
#pragma unroll
    for (int i = 0; i < FM; ++i) f[i] = *reinterpret_cast<const uint4*>(sb + a_row + i * 16 * ROWB + (hl ? ch1 : ch0));
  };
  auto rd_b = [&](int stage, int hl, uint4* f) {
    const char* sb = lds + stage * STAGE;
#pragma unroll
    for (int j = 0; j < FN; ++j) f[j] = *reinterpret_cast<const uint4*>(sb + b_row + j * 16 * ROWB + (hl ? ch1 : ch0));
  };
  auto pass = [&](const uint4* a, const uint4* b) {
    if (DBG == 1) return;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a[i]), __builtin_bit_cast(f16x8, b[j]),
                                                           acc[i][j], 0, 0, 0);
  };
  auto barrier_lds = [&]() {
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // The DMAs of K-tile k (k >= 1) landed.  vmcnt retires in issue order; the
  // ops younger than tile k are: the next K-tile (tile k+1, or the next
  // tile's K-tile 0 when k is the last), and for k = 1, 2 of a round > 0
  // the previous tile's FM*FN + 1 epilogue stores (issued after this tile's
  // K-tile 2, which the previous round prefetched).
  constexpr int NST = FM * FN + 1;
  auto tile_ready = [&](int k, bool younger, bool after_stores) {
    if (!younger) wait_vmcnt<0>();
    else if (after_stores) wait_vmcnt<LPT + NST>();
    else wait_vmcnt<LPT>();
    barrier_lds();
  };

  int L = tile_at(0);
  if (L >= ntiles) return;
  setup(L);
  rows(L, f_off, l_off, mask);
  float scale = s_unscale[n], nscale = scale;
  static_assert(KT0 >= S, "the prefetched K-tiles of the next tile are tap0 K-tiles");
  // Every round starts with its first S K-tiles issued: round 0 here, later
  // rounds by the previous round (two inside its K loop, one after it).
#pragma unroll
  for (int s2 = 0; s2 < S; ++s2) issue(s2);
  unsigned nf_off[A_LD], nl_off[A_LD], nmask[A_LD];   // the next tile's rows
  int sb = 0;                                          // ring stage of this tile's K-tile 0
  const bool late = p.stagger && __builtin_amdgcn_readfirstlane(wave) >= 4;   // wave-uniform (see the K loop)
  unsigned long long mt0 = 0;                          // KPD_STAMPS: shader clock at the K loop's start
  for (int round = 0; L < ntiles; ++round) {
    const int Lnext = tile_at(round + 1);
    const bool has_next = Lnext < ntiles;
    stamp16(p.stamps, 0, 0, L);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    {
      // K-tile 0 landed: younger are K-tiles 1, 2 (and in a round > 0 the
      // previous tile's stores)
      if (round == 0) wait_vmcnt<(S - 1) * LPT>();
      else wait_vmcnt<(S - 1) * LPT + NST>();
      barrier_lds();
      stamp16(p.stamps, 1, 0, L);
      mt0 = p.stamps ? __builtin_amdgcn_s_memtime() : 0ull;
      rd_a(sb, 1, fa1); rd_b(sb, 0, fb0); rd_b(sb, 1, fb1); rd_a(sb, 0, fa0);
      // Each K-tile is issued as soon as its stage is free: after barrier
      // kt+1 every wave has read tile kt into registers, so tile kt+S (or,
      // near the end, the next tile's K-tile kt+S-KT) goes into its stage.
      int is = sb, rs = sb;   // stage the next issue writes / stage of the current tile
      for (int kt = 0; kt < KT; ++kt) {
        const int ns = rs + 1 == S ? 0 : rs + 1;
        const bool more = kt + 1 < KT;
        __builtin_amdgcn_s_setprio(1);
        pass(fa1, fb0);
        __builtin_amdgcn_s_setprio(0);
        // Stagger (KPD_FPN0X_NOSTAGGER: off): waves 0-3 issue this barrier's DMA
        // pieces right after it, their SIMD partners 4-7 after pass 2, so one
        // wave of each SIMD pair issues while the other one's MFMAs run
        // (MI355X_MICROARCH.md "Two waves that run the SAME program").  The
        // stage written was freed at this barrier; the pieces still precede
        // the next barrier, so the counted waits are unchanged.
        auto issue_k = [&]() {
          if (DBG != 2) {
            if (kt + S < KT) issue(is);
            else if (has_next) issue_tap0(is, kt + S - KT, nf_off, nmask);
          }
          is = is + 1 == S ? 0 : is + 1;
        };
        if (more) {
          tile_ready(kt + 1, kt + 2 < KT || has_next, round > 0 && kt + 1 <= 2);
          if (!late) issue_k();
          rd_a(ns, 1, fa1);
        }
        __builtin_amdgcn_s_setprio(1);
        pass(fa0, fb1);
        __builtin_amdgcn_s_setprio(0);
        if (more && late) issue_k();
        if (kt == 0 && has_next) {
          rows(Lnext, nf_off, nl_off, nmask);
          nscale = s_unscale[(Lnext >> 4) / p.tpc];
        }
        if (more) rd_b(ns, 1, fb1);
        __builtin_amdgcn_s_setprio(1);
        pass(fa0, fb0);
        __builtin_amdgcn_s_setprio(0);
        if (more) {
          rd_b(ns, 0, fb0);
          rd_a(ns, 0, fa0);
        }
        rs = ns;
      }
    }
    barrier_lds();   // every wave's fragment reads of the ring retired: the stage of the last K-tile is free
    stamp16(p.stamps, 2, 0, L);
    stamp16(p.stamps, 5, (unsigned long long)KT, L);
    if (p.stamps) stamp16(p.stamps, 4, __builtin_amdgcn_s_memtime() - mt0, L);   // K loop in shader cycles
    // this tile's geometry for the epilogue; then the next tile's prologue
    const int e_cls = cls, e_n = n, e_jt = jt, e_ca = ca, e_cb = cb, e_q0 = q0;
    const float e_scale = scale;
    if (has_next) {
      scale = nscale;
      const int last = sb + KT - 1;   // the stage of this tile's last K-tile
      sb = (sb + KT) % S;
      setup(Lnext);
#pragma unroll
      for (int i = 0; i < A_LD; ++i) {
        f_off[i] = nf_off[i];
        l_off[i] = nl_off[i];
        mask[i] = nmask[i];
      }
      ld = S - 1;
      if (DBG != 2) issue(last % S);   // the next tile's K-tile S-1 (0 .. S-2 went out inside the K loop)
      else ++ld;
    }
    stamp16(p.stamps, 6, 0, L);

    // ---------------- register epilogue ----------------
    const int t4 = lane & 3;
    float* sts = reinterpret_cast<float*>(lds + RING);
    const int row_lim = RG - (e_q0 + wm * WM + g * 4);
    const bool full = e_q0 + BM <= RG;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = wn * 64 + j * 16;
      const float bj = s_bias[col + r16];
      float sm = 0.f, mx = -INFINITY;
      if (full) {   // every row of the tile is in the grid: no masks, max3 pairs
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            const float v0 = fmaxf(acc[i][j][e] * e_scale + bj, 0.f), v1 = fmaxf(acc[i][j][e + 1] * e_scale + bj, 0.f);
            acc[i][j][e] = v0;
            acc[i][j][e + 1] = v1;
            sm += v0;
            sm += v1;
            mx = fmaxf(mx, fmaxf(v0, v1));
          }
      } else {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float v = fmaxf(acc[i][j][e] * e_scale + bj, 0.f);
            acc[i][j][e] = v;
            const bool row_ok = i * 16 + e < row_lim;
            sm += row_ok ? v : 0.f;
            mx = row_ok ? fmaxf(mx, v) : mx;
          }
      }
      sm += __shfl_xor(sm, 16);
      mx = fmaxf(mx, __shfl_xor(mx, 16));
      sm += __shfl_xor(sm, 32);
      mx = fmaxf(mx, __shfl_xor(mx, 32));
      if (g == 0) {
        sts[wm * BN + col + r16] = sm;
        sts[(WAVES_M + wm) * BN + col + r16] = mx;
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    stamp16(p.stamps, 7, 0, L);
    // Stats and output leave by buffer stores issued by EVERY wave in a fixed
    // count (an out-of-range row goes to an out-of-range offset, dropped by
    // the range check): the next tile's first tile_ready counts them (vmcnt
    // retires loads, stores and LDS-DMA in issue order), so it waits for the
    // next tile's first K-tile only, not for this tile's stores.
    {
      float v = 0.f;
      if (tid < 2 * BN) {
        const int c = tid & (BN - 1), mxs = tid >= BN;
        v = sts[mxs * WAVES_M * BN + c];
#pragma unroll
        for (int w = 1; w < WAVES_M; ++w) {
          const float u = sts[(mxs * WAVES_M + w) * BN + c];
          v = mxs ? fmaxf(v, u) : v + u;
        }
      }
      const unsigned so = (unsigned)(((e_n * 16 + e_cls) * p.tpc + e_jt) * 2 * BN) * 4u;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rst, tid < 2 * BN ? so + tid * 4 : OOB, 0, 0);
    }
    stamp16(p.stamps, 3, 0, L);
    // Output pieces of 4 pixels x 64 channels (256 contiguous bytes per
    // pixel, whole 128-byte lines): piece (i, e) gathers acc[i][0..3][e]
    // (lane (g, r16): channels r16 + 16 j of pixel 16 i + 4 g + e), a quad
    // transpose and a lane transpose inside each 16-lane row (lane 4p+q <-
    // 4q+p, ds_bpermute) leave lane (g, c) with channels 4c .. 4c+3.  The
    // 64-byte pieces of the plain fragment layout took ~35 us more per launch.
    const int src4 = ((lane & 0x30) | ((lane & 3) << 2) | ((lane >> 2) & 3)) * 4;
    const int2 fp = s_fp[e_n];
    const int fx0 = fp.x & 0xFFFF, fx1 = fp.x >> 16, fy0 = fp.y & 0xFFFF, fy1 = fp.y >> 16;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        f32x4 v = f32x4{acc[i][0][e], acc[i][1][e], acc[i][2][e], acc[i][3][e]};
        quad_transpose(v, t4);
        f32x4 w;
#pragma unroll
        for (int k = 0; k < 4; ++k) w[k] = __int_as_float(__builtin_amdgcn_ds_bpermute(src4, __float_as_int(v[k])));
        const int q = e_q0 + wm * WM + i * 16 + g * 4 + e;
        const int Y = (int)(((float)q + 0.5f) * inv_rw), X = q - Y * rw;
        const unsigned o =
            (unsigned)((((e_n * Hf + 4 * Y + e_ca) * Wf + 4 * X + e_cb) * BN + wn * 64 + r16 * 4) * 4);
        const int py = 4 * Y + e_ca, px = 4 * X + e_cb;
        const bool keep = q < RG && py >= fy0 && py <= fy1 && px >= fx0 && px <= fx1;
        const unsigned so = keep && (DBG != 4 || (i | e) == 0) ? o : OOB;
        // nt: the 403 MB of output streams past the L2 instead of evicting the
        // weights and the next rounds' input rows (p.out_nt, A/B switch)
        if (p.out_nt) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, w), rout, so, 0, 2);
        else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, w), rout, so, 0, 0);
      }
    // the stats exchange region is rewritten by the next tile only after the
    // barriers of its K loop
    L = Lnext;
  }
}

// fp32 rows -> f16 hi|lo rows (groups of G = 32 channels, 16 when cin == 16),
// pixel px of image px / hw scaled by that image's power of two for operand
// `which` (0: tap0, 1: lateral 1) -- fpn0x_exps on the image's own maxima
__global__ __launch_bounds__(256) void split_rows_kernel(const float* __restrict__ in, int N, long hw, int cin,
                                                         const float* __restrict__ sc, int which, int w_exp0,
                                                         int w_expE, _Float16* __restrict__ out) {
  const int G = cin == 16 ? 16 : 32, c8n = cin / 8;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)N * hw * c8n) return;
  const long px = i / c8n;
  const int c = (int)(i - px * c8n) * 8, n = (int)(px / hw);
  int a_f, a_l, P;
  fpn0x_exps(sc[(size_t)n * kAmaxStride], sc[(size_t)(N + n) * kAmaxStride], w_exp0, w_expE, &a_f, &a_l, &P);
  const float s = ldexpf(1.f, which ? a_l : a_f);
  const float4 u = *reinterpret_cast<const float4*>(in + px * cin + c);
  const float4 v = *reinterpret_cast<const float4*>(in + px * cin + c + 4);
  const float x[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
  typedef _Float16 f16x8v __attribute__((ext_vector_type(8)));
  f16x8v hi, lo;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float xs = x[e] * s;
    hi[e] = (_Float16)xs;
    lo[e] = (_Float16)(xs - (float)hi[e]);
  }
  _Float16* o = out + px * 2 * cin + (c / G) * 2 * G + c % G;
  *reinterpret_cast<f16x8v*>(o) = hi;
  *reinterpret_cast<f16x8v*>(o + G) = lo;
}

// ---------------------------------------------------------------- HeatmapHead convs, padded ROI maps
// 3x3 conv + folded BN + ReLU on the 56x56 ROI maps of HeatmapHead
// (heatmap_head.py:31-45,55-66), bf16 operands, fp32 accumulation.  The
// activations are stored in the hmconv layout (kpd_kernels.h: rows of 57
// positions, one zero column and one zero row shared between neighbours), so
// a tap (dy, dx) of output position m is input position m + 57 dy + dx with
// the zero padding already in memory.  A GEMM row is a position; a tile is
// 256 consecutive positions, and its A operand for ALL nine taps of a
// 64-channel chunk is one window of 384 positions (m0 - 64 .. m0 + 319) staged
// once per chunk -- the per-tap A staging of the generic kernel (9 x 256 rows)
// becomes 384 rows, so the LDS-DMA bytes per MFMA drop 1.7x (BN 256) to 3x
// (BN 64): the generic kernel is bound by the ~70 GB/s per CU an L2 -> LDS
// DMA stream sustains (tools/conv16_probe.py ablations).  The border row and
// column positions of the GEMM are computed and discarded (the tile range
// starts at row 1 of ROI 0; 113 of 3249 positions per ROI, 3.5 % extra MFMA
// work; a 58 x 58 frame had 6.8 %); outputs are stored to the interior only,
// so the zero borders written once at workspace creation stay.
//   BN 256: bf16 output (conv 1, 2), LDS-staged epilogue.
//   BN 64 : conv 3 with the final 1x1 64->17 + sigmoid fused (mixed mode),
//           written to the [B][P][17][56][56] heatmap at the ROI's slot.
constexpr int HP = kHmPitch, HPP = kHmRoiPos;   // row pitch, positions per ROI (kpd_kernels.h)
constexpr int HMS = 56;                          // ROI side
constexpr int AWIN = 384;               // A window rows per chunk (tiles of <= 256 rows)
// A window rows of a BMH-row tile: 64 halo rows above, >= 64 below (a tap
// reads rows 64 - 59 .. 64 + 59 + BMH - 1 of the window)
template <int BMH>
constexpr int hm_awin() { return BMH + 128 <= AWIN ? AWIN : BMH + 128; }
// epilogue (MODE 0) row parts: a 384-row tile stages its fp32 accumulators
// through LDS in two 192-row halves (one [384][132] tile exceeds the LDS)
template <int BMH>
constexpr int hm_epi_parts() { return BMH > 256 ? 2 : 1; }
// DBG (A/B ablations, KPD_HMCONV_DBG): 1 = no MFMA, 2 = no weight / window
// DMA inside the K loop (the prologue's still lands)
// BMH: GEMM rows per tile (256, or 224 so that the tile count packs the CUs'
// rounds better -- launch_hmconv picks it; the window stays 384 rows)
// CIN: input channels as a compile-time constant (0 = p.cin): the K loop's
// trip count is then known to the compiler, and conv 1 / conv 2 are separate
// kernels in a trace
// TPS (SPLIT only): taps per K-step -- the weights of TPS consecutive taps of
// a chunk are staged together and one barrier serves all of them (the BN = 64
// conv 3 has too few MFMAs per tap to amortise a barrier).
// DB (SPLIT only): double-buffered fragment sets -- step k+1's operands are
// all read while step k's three passes run (conv 3: few MFMAs per pass and
// registers to spare; the BN = 256 tiles have no room for a second set).
// NW: waves per workgroup (8; 4 for conv 3: 64 x 64 wave tiles, 1.5x fewer
// LDS fragment bytes per MFMA than 8 waves of 32 x 64, one wave per SIMD).
// MODE: epilogue -- 0 bias + ReLU, re-split (or bf16) for the next conv; 1 the
// fused final 1x1 + sigmoid (heatmap); 2 KEYPOINT_HEAD (keypoint_head.py:
// 64-90): bias + ReLU6, the ResidualBlock's bn1 affine + ReLU6, the
// downsample residual + ReLU6, outputs split (next conv) and / or fp32 (pools).
// -1: 1 for BN = 64, else 0.
// NTAP (MODE 2): 10 = the 3x3 taps plus the ResidualBlock's 1x1 downsample as
// a tenth K-step per chunk (the centre tap's A rows, its own weights) into a
// second accumulator set.
// A-window buffers: 2 (chunk c + 1's window lands while chunk c's taps run),
// 1 when the input is a single 128-byte chunk (CIN 32 split: one window per tile)
template <int CIN, bool SPLIT>
constexpr int hm_nab() { return (CIN > 0 && (SPLIT ? CIN * 4 : CIN * 2) == 128) ? 1 : 2; }
// KEYPOINT_HEAD epilogue (MODE 2, BN 128) row parts and staged bytes: the
// fp32 accumulators of BMH / parts rows x BN columns, plus the downsample's of
// the first 64 columns
template <int BMH>
constexpr int kh_epi_parts() { return BMH > 128 ? 2 : 1; }
template <int BN, int BMH>
constexpr int kh_epi_bytes() { return BMH / kh_epi_parts<BMH>() * ((BN + 4) + 68) * 4; }
template <int BN, int SB, int BMH, bool SPLIT, int TPS, int NW, int MODE, int NAB = 2>
constexpr int hmconv_lds_bytes() {
  constexpr int EMODE = MODE >= 0 ? MODE : (BN == 64 ? 1 : 0);
  constexpr int RING = NAB * hm_awin<BMH>() * ROWB + SB * BN * ROWB * TPS;
  constexpr int EPI = EMODE == 2 ? (BN == 128 ? kh_epi_bytes<BN, BMH>() : 0)
                      : EMODE != 0 && EMODE != 3 ? 0 : epi_lds_bytes<BMH / hm_epi_parts<BMH>(), 128, NW * 64>();
  return RING > EPI ? RING : EPI;
}

// One tile: logical tile L of the launch's tile space, rows from padded
// position HP + m_off + (L / (cout / BN)) * BMH; lds: the workgroup's LDS
// (hmconv_lds_bytes), declared by the calling kernel so that kernels running
// tiles of two heights (hmconv_mixed_kernel) share one allocation.
// PST (persistent kernel, hmconv_persist_kernel): LDS as [A0 | B0 | A1 | B1]
// (window buffer c & 1 beside weight stage c & 1), so that after the K loop
// A0 + B0 take the NEXT tile's prologue (chunk 0 window, B(0): issued before
// this tile's epilogue when next_m0 >= 0) while the epilogue stages through
// A1 + B1 in four 112-row x 128-column parts; the epilogue's VMEM operations
// are a fixed count per wave (buffer stores with out-of-range offsets for
// border rows, both amax atomics always), so the next tile's first barrier
// waits for its prologue with a counted vmcnt, not for these stores.
// pre: this tile's prologue was issued by the previous tile.
template <int BMH>
constexpr int hm_pst_stores() { return 2 * 2 * ((BMH / 2 + 31) / 32) * 2; }   // parts x IT x (hi, lo)
template <int BN, int SB, int DBG, int BMH, bool SPLIT, int CIN, int TPS, bool DB, int NW, int MODE, int NTAP,
          bool PST = false>
__device__ __forceinline__ void hmconv_tile(const HmConvArgs& p, char* lds, const int L, const int m_off,
                                            const bool pre = false, const int next_m0 = -1) {
  constexpr int NTH = NW * 64;
  constexpr int EMODE = MODE >= 0 ? MODE : (BN == 64 ? 1 : 0);
  static_assert(NTAP == 9 || (NTAP == 10 && EMODE == 2 && SPLIT && !DB), "tenth tap: KH downsample");
  static_assert(EMODE != 2 || (SPLIT && !DB), "KH epilogue: split, single fragment set");
  static_assert(EMODE != 3 || SPLIT, "linear fp32 epilogue: split");
  constexpr int WAVES_N = BN / 64, WAVES_M = NW / WAVES_N;
  constexpr int WM = BMH / WAVES_M, FM = WM / 16, FN = 4;
  constexpr int AW = hm_awin<BMH>();
  static_assert(WM % 16 == 0 && BMH + 128 <= AW && AW % (8 * NW) == 0, "tile rows");
  static_assert(NW == 8 || (BN == 64 && SPLIT && DB), "4 waves: the conv 3 split DB variant only");
  constexpr int A_LD = AW / 8 / NW;                      // A-window DMA wave-instructions per wave (6; 8 at 384 rows; NW 4: 12)
  static_assert(A_LD <= 9 || TPS > 1, "window pieces: one per tap");
  constexpr int B_LD = BN / 8 / NW;                      // B DMA wave-instructions per wave per K-step
  constexpr int ABUF = AW * ROWB, BSTAGE = BN * ROWB * TPS;
  static_assert(TPS == 1 || (SPLIT && NTAP % TPS == 0), "taps per step");
  constexpr bool FINAL = EMODE == 1;
  constexpr int NAB = hm_nab<CIN, SPLIT>();
  static_assert(hmconv_lds_bytes<BN, SB, BMH, SPLIT, TPS, NW, MODE, NAB>() <= 160 * 1024, "LDS budget");
  static_assert(!PST || NAB == 2, "persistent tiles: two window buffers");
  static_assert(!PST || (SPLIT && EMODE == 0 && SB == 2 && TPS == 1 && !DB && NW == 8 && NTAP == 9 && BN == 256 &&
                         BMH <= 224 && DBG == 0), "persistent tiles: split conv 1 / conv 2 (BN = cout = 256)");
  // window buffer of chunk c, weight stage s (PST: [A0 | B0 | A1 | B1])
  auto a_at = [&](int c) { return PST ? (c & 1) * (ABUF + BSTAGE) : NAB == 1 ? 0 : (c & 1) * ABUF; };
  auto b_at = [&](int st) { return PST ? st * (ABUF + BSTAGE) + ABUF : NAB * ABUF + st * BSTAGE; };

  int tid = threadIdx.x;
  // PST: per tile, tid is opaque, so that the lane-dependent offsets are
  // recomputed in every tile instead of hoisted out of the persistent loop
  // and held (with the tile's own working set they overflow the registers)
  if constexpr (PST) asm volatile("" : "+v"(tid));
  const int lane = tid & 63, wave = tid >> 6;
  // KH mode: column groups by wave halves (waves w and w + 4 share a SIMD, so
  // a group with fewer live columns pairs with a full one on every SIMD)
  const int wm = EMODE == 2 ? wave % WAVES_M : wave / WAVES_N, wn = EMODE == 2 ? wave / WAVES_M : wave % WAVES_N;
  const int NTL = p.cout / BN;
  const int m0 = HP + m_off + (L / NTL) * BMH, n0 = (L % NTL) * BN;   // GEMM rows: positions [HP, R*HPP)
  if (m0 >= p.R * HPP) return;   // (a padding tile of hmconv_mixed_kernel's tail)
  // a K-step reads one 128-byte row piece: 64 bf16 channels, or (SPLIT) 32
  // channels as [hi32 | lo32] f16
  const int Mtot = p.R * HPP, cin = CIN ? CIN : p.cin, RB = SPLIT ? cin * 4 : cin * 2, NC = RB / 128, KT = NTAP * NC;
  stamp16(p.stamps, 0);
  // the input descriptor starts at this tile's window (a 64-bit base), so
  // the 31-bit buffer extent bounds the window, not the whole R-ROI tensor:
  // one launch takes any number of ROIs (no per-chunk launches, each with
  // its own partial last round of tiles)
  const int wbase = max(m0 - 64, 0);
  const i32x4 rin = make_rsrc(static_cast<const char*>(p.in) + (size_t)wbase * RB,
                              (int)min(((long)Mtot - wbase) * RB, 0x7fffffffL));
  const i32x4 rwt = make_rsrc(p.wt, p.wt_bytes);
  const unsigned lds0 = (unsigned)reinterpret_cast<unsigned long long>((lds_void*)lds);
  const int lrow = lane >> 3, lchunk = (lane & 7) ^ lrow;
  // A window: wave w fills rows [48 w, 48 w + 48) of the window
  unsigned a_off[A_LD];
#pragma unroll
  for (int i = 0; i < A_LD; ++i) {
    const int m = m0 - 64 + wave * (AW / NW) + i * 8 + lrow;
    a_off[i] = (m >= 0 && m < Mtot) ? (unsigned)((m - wbase) * RB + lchunk * 16) : OOB;
  }
  unsigned b_off[B_LD];
#pragma unroll
  for (int i = 0; i < B_LD; ++i) {
    const int co = n0 + wave * (BN / NW) + i * 8 + lrow;
    b_off[i] = (unsigned)(co * NTAP * RB + lchunk * 16);
  }
  auto issue_a = [&](int c, int i) {   // A window of chunk c, wave-instruction i
    const unsigned dst = __builtin_amdgcn_readfirstlane(lds0 + a_at(c) + (wave * (AW / NW) + i * 8) * ROWB);
    glds16(rin, dst, a_off[i] == OOB ? OOB : a_off[i] + c * 128, 0);
  };
  // KH mode, 2-stage ring (every barrier waits vmcnt(0), so a wave's count of
  // pieces does not matter): a wave whose weight rows are all zero-padding
  // columns (>= ns + nf) loads none of them -- their fragments are never read
  const bool b_dead = EMODE == 2 && SB == 2 && n0 + wave * (BN / NW) >= p.ns + p.nf;
  auto issue_b = [&](int k) {          // B of K-step k (TPS taps of one chunk) into stage k % SB
    if (b_dead) return;
#pragma unroll
    for (int u = 0; u < TPS; ++u) {
      const int sk = k * TPS + u, c = sk / NTAP, t = sk - c * NTAP;
      const unsigned dst = __builtin_amdgcn_readfirstlane(lds0 + b_at(k % SB) + u * BN * ROWB + wave * (BN / NW) * ROWB);
#pragma unroll
      for (int i = 0; i < B_LD; ++i) glds16(rwt, dst + i * 8 * ROWB, b_off[i], t * RB + c * 128);
    }
  };
  // Barrier of K-step k: B(k) landed.  A-window pieces are issued before the
  // B of the same batch, so every DMA younger than B(k) is among the
  // (SB - 2) * B_LD weight loads of later steps or an A piece issued after
  // them: vmcnt((SB - 2) * B_LD) retires B(k) -- and the window of k's chunk,
  // whose last piece (tap 5 of the previous chunk) precedes B(k) whenever
  // SB <= 4.  Then every fragment read retired, all waves here.
  static_assert(SB >= 2 && SB <= 4, "weight ring");
  auto barrier_k = [&](bool tail) {
    if (tail) wait_vmcnt<0>();
    else wait_vmcnt<(SB - 2) * B_LD * TPS>();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  f32x4 acc[FM][FN], acc2[FM][FN];   // acc2: the downsample (NTAP 10)
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, r16 = lane & 15;
  const int b_row = (wn * 64 + r16) * ROWB;
  const int bch0 = ((g ^ (r16 & 7)) << 4), bch1 = (((4 + g) ^ (r16 & 7)) << 4);
  struct Half { uint4 a[FM], b[FN]; };
  // half q of K-step k: A rows shifted by the tap offset (swizzle by the row)
  auto load_half = [&](int k, int q, Half& f) {
    const int c = k / 9, t = k - c * 9, off = (t / 3 - 1) * HP + (t % 3 - 1);
    const char* ab = lds + a_at(c);
    const char* bb = lds + b_at(k % SB);
#pragma unroll
    for (int j = 0; j < FN; ++j) f.b[j] = *reinterpret_cast<const uint4*>(bb + b_row + j * 16 * ROWB + (q ? bch1 : bch0));
    const int r0w = wm * WM + r16 + 64 + off;   // window row of fragment 0 (rows of fragment i: + 16 i)
    const int ach = (((q ? 4 : 0) + g) ^ (r0w & 7)) << 4;
#pragma unroll
    for (int i = 0; i < FM; ++i) f.a[i] = *reinterpret_cast<const uint4*>(ab + (r0w + i * 16) * ROWB + ach);
  };
  auto mma_half = [&](const Half& f) {
    if constexpr ((DBG & 1) != 0) {
      acc[0][0][0] += __uint_as_float(f.a[0].x ^ f.b[FN - 1].w);   // keep the fragment reads alive
      return;
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, f.a[i]),
                                                            __builtin_bit_cast(bf16x8, f.b[j]), acc[i][j], 0, 0, 0);
  };
  // fused final layer weights, loaded before the K loop (3 or 5 per thread)
  constexpr int FPRE = (17 * 65 + NTH - 1) / NTH;
  float fin_pre[FPRE];
#pragma unroll
  for (int u = 0; u < FPRE; ++u) fin_pre[u] = 0.f;
  if constexpr (FINAL) {
#pragma unroll
    for (int u = 0; u < FPRE; ++u) {
      const int i = tid + u * NTH;
      if (i < 17 * 64) fin_pre[u] = p.fin_w[i];
      else if (i < 17 * 65) fin_pre[u] = p.fin_b[i - 17 * 64];
    }
  }
  // SPLIT: per-ROI power-of-two scales of the tile's (at most two) ROIs,
  // loaded before the K loop.  Input unscale 2^-(a_in + w_exp), output scale
  // 2^a_out, a = split_exp_of(bound), bound = c + s * hsc[r][idx] (HmConvArgs).
  const int rlo = m0 / HPP;                 // local ROI of the tile's first row (rows span <= 2 ROIs)
  float us[2] = {1.f, 1.f}, os[2] = {1.f, 1.f};
  if constexpr (SPLIT) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int rg = p.r0 + min(rlo + q, p.R - 1);
      const float ui = p.in_c + p.in_s * p.hsc[(size_t)rg * 4 + p.in_idx];
      us[q] = ldexpf(1.f, -(split_exp_of(ui) + p.w_exp));
      if (p.out_idx >= 0) os[q] = ldexpf(1.f, split_exp_of(p.out_c + p.out_s * p.hsc[(size_t)rg * 4 + p.out_idx]));
    }
  }
  const int rbound = (rlo + 1) * HPP;       // first padded position of the tile's second ROI
  // prologue: chunk 0's window and the first SB-1 K-steps' weights
  const int KS = KT / TPS;                  // K-steps (barriers)
  if (!PST || !pre) {
#pragma unroll
    for (int i = 0; i < A_LD; ++i) issue_a(0, i);
#pragma unroll
    for (int k = 0; k < SB - 1; ++k)
      if (k < KS) issue_b(k);
    barrier_k(KS < SB - 1);
  } else {
    // prologue issued by the previous tile, before its epilogue's fixed count
    // of VMEM operations (hm_pst_stores<224> stores + 2 amax atomics)
    if (p.amax_idx >= 0) wait_vmcnt<hm_pst_stores<224>() + 2>();
    else wait_vmcnt<hm_pst_stores<224>()>();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  stamp16(p.stamps, 1);
  stamp16(p.stamps, 6, __builtin_amdgcn_s_memtime());   // shader clock (K-loop clock rate)
  // the next chunk's window, spread over this chunk's K-steps: pieces of
  // K-step k1 (TPS = 1: piece t1 at taps 0-5; else an equal share per step)
  auto issue_a_at = [&](int k1) {
    const int s1 = k1 * TPS, c1 = s1 / NTAP, jj = (s1 - c1 * NTAP) / TPS;
    if (c1 + 1 >= NC) return;
    if constexpr (TPS == 1) {
      if (jj < A_LD) issue_a(c1 + 1, jj);
    } else {
      constexpr int NST = 9 / TPS;
#pragma unroll
      for (int i = 0; i < A_LD; ++i)
        if (i >= jj * A_LD / NST && i < (jj + 1) * A_LD / NST) issue_a(c1 + 1, i);
    }
  };
  issue_a_at(0);
  if (SB - 1 < KS) issue_b(SB - 1);
  // DMA issue at barrier k1 (same schedule in both loops): the next chunk's
  // window pieces, and B(k1 + SB - 1) into the stage of B(k1 - 1), whose
  // fragment reads every wave finished before barrier k1
  auto issue_at = [&](int k1) {
    if constexpr ((DBG & 2) == 0) {
      issue_a_at(k1);
      if (k1 + SB - 1 < KS) issue_b(k1 + SB - 1);
    }
  };
  if constexpr (!SPLIT) {
    Half f0, f1;
    load_half(0, 0, f0);
    // K-step k: reads (k, q1) | MFMAs (k, q0) | barrier k+1 + DMA issue | reads (k+1, q0) | MFMAs (k, q1)
    for (int k = 0; k < KT; ++k) {
      load_half(k, 1, f1);
      __builtin_amdgcn_s_setprio(1);
      mma_half(f0);
      __builtin_amdgcn_s_setprio(0);
      if (k + 1 < KT) {
        const int k1 = k + 1;
        barrier_k(k1 + SB - 2 >= KT);   // B(k1) and its chunk's window landed; reads of k retired
        issue_at(k1);
        load_half(k1, 0, f0);
      } else {
        __builtin_amdgcn_s_waitcnt(0xC07F);
      }
      // (threading the DMA pieces between the MFMA rows measured 2 % slower:
      // the weights then land later than the next barrier wants them)
      __builtin_amdgcn_s_setprio(1);
      mma_half(f1);
      __builtin_amdgcn_s_setprio(0);
    }
  } else {
    // Split products per K-step: lo.hi | hi.hi | hi.lo (the lo.lo term, ~2^-22
    // relative, is dropped) on v_mfma_f32_16x16x32_f16.  One fragment set;
    // each register group is refilled with step k+1 as soon as its last pass
    // of step k has issued, so every pass finds its operands read one or two
    // passes earlier:  P1 al.bh | barrier k+1, DMA, read al' | P2 ah.bh |
    // read bh' | P3 ah.bl | read ah', bl'.
    uint4 ah[FM], al[FM], bh[FN], bl[FN];
    auto rd_a = [&](int k, int q, uint4* f) {
      const int c = k / NTAP, t = k - c * NTAP, off = t == 9 ? 0 : (t / 3 - 1) * HP + (t % 3 - 1);
      const char* ab = lds + a_at(c);
      const int r0w = wm * WM + r16 + 64 + off;
      const int ach = (((q ? 4 : 0) + g) ^ (r0w & 7)) << 4;
#pragma unroll
      for (int i = 0; i < FM; ++i) f[i] = *reinterpret_cast<const uint4*>(ab + (r0w + i * 16) * ROWB + ach);
    };
    // stagger (HmConvArgs::stagger): waves 4-7 issue a barrier's DMA pieces
    // after pass 2 instead of right after the barrier, so one wave of each
    // SIMD pair issues while its partner's MFMAs run (conv 1 / 2 K step
    // 1.84 / 1.81 -> 1.75 / 1.77 us)
    const bool late = p.stagger && __builtin_amdgcn_readfirstlane(wave) >= 4;
    auto pass = [&](f32x4 (&A)[FM][FN], const uint4* a, const uint4* b) {
      if constexpr ((DBG & 1) != 0) {
        A[0][0][0] += __uint_as_float(a[0].x ^ b[FN - 1].w);
        return;
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          A[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a[i]), __builtin_bit_cast(f16x8, b[j]),
                                                           A[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    };
    if constexpr (DB) {
      // Taps unrolled (two chunks per iteration, so the fragment set and the
      // weight stage of every sub-step are compile-time) with the per-lane A
      // offsets of the nine taps precomputed: the operand addressing is one
      // add per read, and every pass's operands were read a whole step ago.
      static_assert(SB == 2 && 9 % TPS == 0, "DB loop: 2-stage ring");
      int aoff[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int r0w = wm * WM + r16 + 64 + (t / 3 - 1) * HP + (t % 3 - 1);
        aoff[t] = r0w * ROWB + ((g ^ (r0w & 7)) << 4);   // q = 1 (lo): chunk ^ 4, byte ^ 64
      }
      struct Frag { uint4 ah[FM], al[FM], bh[FN], bl[FN]; };
      auto rd_all = [&](int c, int t, int stage, Frag& f) {
        const char* ab = lds + a_at(c);
        const char* bb = lds + b_at(stage) + (t % TPS) * BN * ROWB + b_row;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          f.al[i] = *reinterpret_cast<const uint4*>(ab + (aoff[t] ^ 64) + i * 16 * ROWB);
          f.ah[i] = *reinterpret_cast<const uint4*>(ab + aoff[t] + i * 16 * ROWB);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          f.bh[j] = *reinterpret_cast<const uint4*>(bb + j * 16 * ROWB + bch0);
          f.bl[j] = *reinterpret_cast<const uint4*>(bb + j * 16 * ROWB + bch1);
        }
      };
      Frag f0, f1;
      rd_all(0, 0, 0, f0);
      for (int c = 0; c < NC; c += 2) {   // NC even (host check): c even at the top
#pragma unroll
        for (int tt = 0; tt < 18; ++tt) {
          const int cc = c + tt / 9, t = tt % 9, k = cc * 9 + t;
          Frag& cur = (tt & 1) ? f1 : f0;
          Frag& nxt = (tt & 1) ? f0 : f1;
          pass(acc, cur.al, cur.bh);
          const bool kstep = k + 1 < KT && (t + 1) % TPS == 0;
          if (k + 1 < KT) {
            const int tn = (tt + 1) % 18, cn = c + (tt + 1) / 9;   // next sub-step (chunk cn, tap tn % 9)
            if (kstep) {
              const int k1 = (k + 1) / TPS;
              barrier_k(k1 + SB - 2 >= KS);
              if (!late) issue_at(k1);
            }
            // stage of the next sub-step: (its K-step) % 2 = (tn / 9 + (tn % 9) / TPS) % 2 with c even
            rd_all(cn, tn % 9, ((tn / 9) * (9 / TPS) + (tn % 9) / TPS) & 1, nxt);
          }
          pass(acc, cur.ah, cur.bh);
          if (kstep && late) issue_at((k + 1) / TPS);
          pass(acc, cur.ah, cur.bl);
        }
      }
    } else {
    // The K loop with NB_ weight fragments read per step and NM_ / NM9_ of
    // them multiplied (taps 0-8 / the downsample tap): KH mode skips the
    // fragments of its zero-padded columns (wave-uniform counts); elsewhere all FN.
    auto run_loop = [&](auto NBc, auto NMc, auto NM9c) {
      constexpr int NB_ = decltype(NBc)::value;
      auto rd_bn = [&](int k, int q, uint4* f) {
        const char* bb = lds + b_at((k / TPS) % SB) + (k % TPS) * BN * ROWB;
#pragma unroll
        for (int j = 0; j < NB_; ++j)
          f[j] = *reinterpret_cast<const uint4*>(bb + b_row + j * 16 * ROWB + (q ? bch1 : bch0));
      };
      auto passn = [&](f32x4 (&A)[FM][FN], const uint4* a, const uint4* b, auto NMx) {
        constexpr int NM_ = decltype(NMx)::value;
        if constexpr (NM_ == FN) {
          pass(A, a, b);
        } else if constexpr (NM_ > 0) {
          if constexpr ((DBG & 1) != 0) {
            A[0][0][0] += __uint_as_float(a[0].x ^ b[0].w);
            return;
          }
          __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < NM_; ++j)
              A[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a[i]),
                                                               __builtin_bit_cast(f16x8, b[j]), A[i][j], 0, 0, 0);
          __builtin_amdgcn_s_setprio(0);
        }
      };
      rd_a(0, 1, al);
      rd_bn(0, 0, bh);
      rd_a(0, 0, ah);
      rd_bn(0, 1, bl);
      // tap sub-step k into the accumulator set A; a barrier where a K-step begins
      auto sub = [&](int k, f32x4 (&A)[FM][FN], auto NMx) {
        const bool more = k + 1 < KT, kstep = more && (k + 1) % TPS == 0;
        passn(A, al, bh, NMx);
        if (more) {
          if (kstep) {
            const int k1 = (k + 1) / TPS;
            barrier_k(k1 + SB - 2 >= KS);   // B(k1) and its chunk's window landed; reads of k1 - 1 retired
            if (!late) issue_at(k1);
          }
          rd_a(k + 1, 1, al);
        }
        passn(A, ah, bh, NMx);
        if (kstep && late) issue_at((k + 1) / TPS);
        if (more) rd_bn(k + 1, 0, bh);
        passn(A, ah, bl, NMx);
        if (more) {
          rd_a(k + 1, 0, ah);
          rd_bn(k + 1, 1, bl);
        }
      };
      if constexpr (NTAP == 10) {
        for (int c = 0; c < NC; ++c) {
          for (int t = 0; t < 9; ++t) sub(c * NTAP + t, acc, NMc);
          sub(c * NTAP + 9, acc2, NM9c);   // the 1x1 downsample: centre-tap rows, its own weights
        }
      } else {
        for (int k = 0; k < KT; ++k) sub(k, acc, NMc);
      }
    };
    using IFN = std::integral_constant<int, FN>;
    if constexpr (EMODE == 2) {
      // live fragments of this wave's columns: [0, ns + nf) for the 3x3 taps,
      // [0, ns) (the ResidualBlock columns) for the downsample tap
      const int c0 = __builtin_amdgcn_readfirstlane(n0 + wn * 64);
      const int nact = min(max((p.ns + p.nf - c0 + 15) / 16, 0), FN), nact9 = min(max((p.ns - c0 + 15) / 16, 0), FN);
      using I0 = std::integral_constant<int, 0>;
      using I1 = std::integral_constant<int, 1>;
      using I2 = std::integral_constant<int, 2>;
      // the column plans in use (launch_hmconv_kh): [64 + ds | 32 + 32 zero] at
      // BN 128, [32 + ds | 32 zero] and [16 | 48 zero] at BN 64
      if (BN == 128 && nact == 2 && nact9 == 0) {
        if constexpr (BN == 128) run_loop(I2{}, I2{}, I0{});
      } else if (BN == 64 && NTAP == 10 && nact == 2 && nact9 == 2) {
        if constexpr (BN == 64 && NTAP == 10) run_loop(I2{}, I2{}, I2{});
      } else if (BN == 64 && NTAP == 9 && nact == 1) {
        if constexpr (BN == 64 && NTAP == 9) run_loop(I1{}, I1{}, I1{});
      } else {
        run_loop(IFN{}, IFN{}, IFN{});
      }
    } else {
      run_loop(IFN{}, IFN{}, IFN{});
    }
    }
  }
  stamp16(p.stamps, 7, __builtin_amdgcn_s_memtime());
  __syncthreads();
  stamp16(p.stamps, 2);
  float pbias[PST ? 2 : 1][8];
  if constexpr (PST) {
    // the loads of this tile are consumed here (no compiler wait lands behind
    // the prefetch below)
    // the epilogue's bias (this thread's 8 channels of each 128-column half)
    // is read before the prefetch too (L2 hits, ~0.4 us)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int co = n0 + h * 128 + (tid % 16) * 8;
      const float4 b0 = *reinterpret_cast<const float4*>(p.bias + co);
      const float4 b1 = *reinterpret_cast<const float4*>(p.bias + co + 4);
      pbias[h][0] = b0.x; pbias[h][1] = b0.y; pbias[h][2] = b0.z; pbias[h][3] = b0.w;
      pbias[h][4] = b1.x; pbias[h][5] = b1.y; pbias[h][6] = b1.z; pbias[h][7] = b1.w;
    }
    asm volatile("" ::"v"(us[0]), "v"(us[1]), "v"(os[0]), "v"(os[1]));
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < 8; ++e) asm volatile("" ::"v"(pbias[h][e]));
    // the next tile's prologue into A0 / B0 (free: the last K-step used A1 / B1)
    if (next_m0 >= 0) {
      const int nwb = max(next_m0 - 64, 0);
      const i32x4 nrin = make_rsrc(static_cast<const char*>(p.in) + (size_t)nwb * RB,
                                   (int)min(((long)Mtot - nwb) * RB, 0x7fffffffL));
#pragma unroll
      for (int i = 0; i < A_LD; ++i) {
        const int m = next_m0 - 64 + wave * (AW / NW) + i * 8 + lrow;
        const unsigned off = (m >= 0 && m < Mtot) ? (unsigned)((m - nwb) * RB + lchunk * 16) : OOB;
        const unsigned dst = __builtin_amdgcn_readfirstlane(lds0 + a_at(0) + (wave * (AW / NW) + i * 8) * ROWB);
        glds16(nrin, dst, off, 0);
      }
      issue_b(0);
    }
  }

  // interior test of a padded position: ROI row/column 1..56
  auto interior = [&](int m, int& r, int& yy, int& xx) {
    r = m / HPP;
    const int rem = m - r * HPP;
    yy = rem / HP - 1;
    xx = rem - (yy + 1) * HP;
    return m < Mtot && yy >= 0 && xx < HMS;
  };
  if constexpr (PST) {
    // four parts of 112 rows x 128 columns staged through A1 + B1; every
    // wave issues exactly hm_pst_stores<BMH>() stores (border / out-of-tile
    // rows to an out-of-range offset) and, with amax, two atomics
    float* tile = reinterpret_cast<float*>(lds + ABUF + BSTAGE);
    constexpr int P4 = 128 + 4, C8 = 16, RS = NTH / C8, IT = (WM + RS - 1) / RS;
    static_assert(WAVES_M == 2 && WM * P4 * 4 <= ABUF + BSTAGE && 4 * IT * 2 == hm_pst_stores<BMH>(), "PST epilogue");
    const int obytes = p.cout * 4;
    const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(static_cast<char*>(p.out) + (size_t)m0 * obytes,
                                                                          (short)0, BMH * obytes, 0x00020000);
    float mx[2] = {0.f, 0.f};
    const int c8 = tid % C8, row0 = tid / C8;
#pragma unroll
    for (int pp = 0; pp < 4; ++pp) {
      const int pr = pp >> 1, h = pp & 1;
      if (pp) __syncthreads();
      if (wn / 2 == h && wm == pr) acc_to_lds<FM, FN, WM, 64, 128>(tile, acc, 0, wn % 2, lane);
      __syncthreads();
      const int co = n0 + h * 128 + c8 * 8;
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int row = row0 + it * RS, m = m0 + pr * WM + row;
        int r, yy, xx;
        const bool ok = row < WM && interior(m, r, yy, xx);
        const float4 x0 = *reinterpret_cast<const float4*>(tile + min(row, WM - 1) * P4 + c8 * 8);
        const float4 x1 = *reinterpret_cast<const float4*>(tile + min(row, WM - 1) * P4 + c8 * 8 + 4);
        const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        const int q = m >= rbound;
        const float u = q ? us[1] : us[0], sc = q ? os[1] : os[0];
        f16x8 hi, lo;
        float mc = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = fmaxf(fmaf(xv[e], u, pbias[h][e]), 0.f);
          mc = fmaxf(mc, v);
          const float xs = v * sc;
          hi[e] = (_Float16)xs;
          lo[e] = (_Float16)(xs - (float)hi[e]);
        }
        const unsigned off = ok ? (unsigned)((m - m0) * obytes + (co >> 5) * 128 + (co & 31) * 2) : OOB;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, hi), rout, off, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, lo), rout, ok ? off + 64 : OOB, 0, 0);
        if (ok) {
          if (q) mx[1] = fmaxf(mx[1], mc); else mx[0] = fmaxf(mx[0], mc);
        }
      }
    }
    if (p.amax_idx >= 0) {   // per-ROI max|out| for the next conv's output scale: two atomics per wave, always
      const float w0 = wave_max(mx[0]), w1 = wave_max(mx[1]);
      if (lane == 0) {
        const bool two = rlo + 1 < p.R;
        unsigned* a0 = reinterpret_cast<unsigned*>(p.hsc + (size_t)(p.r0 + rlo) * 4 + p.amax_idx);
        unsigned* a1 = reinterpret_cast<unsigned*>(p.hsc + (size_t)(p.r0 + rlo + (two ? 1 : 0)) * 4 + p.amax_idx);
        atomicMax(a0, __float_as_uint(w0));
        atomicMax(a1, __float_as_uint(two ? w1 : 0.f));
      }
    }
  } else if constexpr (EMODE == 0 || EMODE == 3) {
    // bias + ReLU through the LDS tile (two 128-column halves): bf16 16-byte
    // row stores, or (SPLIT) the unscaled fp32 value re-split for the next
    // conv: x * 2^a_out(ROI) as f16 hi / lo into the [hi32 | lo32] groups
    float* tile = reinterpret_cast<float*>(lds);
    // a thread takes 8 consecutive channels of a row: 16-byte stores (the
    // epilogue's store tail is issue-bound when every CU stores at once:
    // half the store instructions of 8-byte pieces)
    // (RP row parts of BR rows: the waves of part pr stage, all threads store)
    constexpr int RP = hm_epi_parts<BMH>(), BR = BMH / RP, WPR = WAVES_M / RP;
    static_assert(WAVES_M % RP == 0, "epilogue row parts");
    constexpr int P4 = 128 + 4, C8 = 16, RS = NTH / C8, IT = (BR + RS - 1) / RS;
    __bf16* out = reinterpret_cast<__bf16*>(p.out);
    float mx[2] = {0.f, 0.f};   // SPLIT: max|out| of the tile's two ROIs (>= 0 after ReLU)
#pragma unroll
    for (int ph = 0; ph < RP * (BN / 128); ++ph) {
      const int pr = ph / (BN / 128), h = ph % (BN / 128);
      if (ph) __syncthreads();
      if (wn / 2 == h && wm / WPR == pr) acc_to_lds<FM, FN, WM, 64, 128>(tile, acc, wm % WPR, wn % 2, lane);
      __syncthreads();
      const int c8 = tid % C8, row0 = tid / C8, co = n0 + h * 128 + c8 * 8;
      const float4 b0 = *reinterpret_cast<const float4*>(p.bias + co);
      const float4 b1 = *reinterpret_cast<const float4*>(p.bias + co + 4);
      const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int row = row0 + it * RS, m = m0 + pr * BR + row;
        int r, yy, xx;
        if (row >= BR || !interior(m, r, yy, xx)) continue;
        const float4 x0 = *reinterpret_cast<const float4*>(tile + row * P4 + c8 * 8);
        const float4 x1 = *reinterpret_cast<const float4*>(tile + row * P4 + c8 * 8 + 4);
        float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        if constexpr (EMODE == 3) {
          // linear fp32 output (conv3x3 forward / dgrad of K6, conv3_grad.hip):
          // acc * u + bias at NHWC [R][56][56][cout]
          const float u = m >= rbound ? us[1] : us[0];
          float* of = p.outf + ((size_t)r * HMS * HMS + yy * HMS + xx) * p.cout + co;
          *reinterpret_cast<float4*>(of) = make_float4(fmaf(xv[0], u, bv[0]), fmaf(xv[1], u, bv[1]),
                                                       fmaf(xv[2], u, bv[2]), fmaf(xv[3], u, bv[3]));
          *reinterpret_cast<float4*>(of + 4) = make_float4(fmaf(xv[4], u, bv[4]), fmaf(xv[5], u, bv[5]),
                                                           fmaf(xv[6], u, bv[6]), fmaf(xv[7], u, bv[7]));
        } else if constexpr (SPLIT) {
          const int q = m >= rbound;
          const float u = q ? us[1] : us[0], sc = q ? os[1] : os[0];
          f16x8 hi, lo;
          float mc = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            xv[e] = fmaxf(fmaf(xv[e], u, bv[e]), 0.f);
            mc = fmaxf(mc, xv[e]);
            const float xs = xv[e] * sc;
            hi[e] = (_Float16)xs;
            lo[e] = (_Float16)(xs - (float)hi[e]);
          }
          char* ob = static_cast<char*>(p.out) + (size_t)m * (p.cout * 4) + (co >> 5) * 128 + (co & 31) * 2;
          *reinterpret_cast<f16x8*>(ob) = hi;
          *reinterpret_cast<f16x8*>(ob + 64) = lo;
          if (q) mx[1] = fmaxf(mx[1], mc); else mx[0] = fmaxf(mx[0], mc);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) xv[e] = fmaxf(xv[e] + bv[e], 0.f);
          store4<__bf16>(out + (size_t)m * p.cout + co, make_float4(xv[0], xv[1], xv[2], xv[3]));
          store4<__bf16>(out + (size_t)m * p.cout + co + 4, make_float4(xv[4], xv[5], xv[6], xv[7]));
        }
      }
    }
    if constexpr (SPLIT && EMODE == 0) {
      if (p.amax_idx >= 0) {   // per-ROI max|out| for the next conv's output scale
        float w0 = wave_max(mx[0]), w1 = wave_max(mx[1]);
        // the tile's maxima combined in LDS first: two atomics per tile instead
        // of two per wave (a round of tiles ends together, and same-address
        // atomics serialise at the L2)
        float* red = reinterpret_cast<float*>(lds);
        __syncthreads();   // every wave's reads of the staged tile are done
        if (lane == 0) {
          red[2 * wave] = w0;
          red[2 * wave + 1] = w1;
        }
        __syncthreads();
        if (tid == 0) {
#pragma unroll
          for (int w = 1; w < NW; ++w) {
            w0 = fmaxf(w0, red[2 * w]);
            w1 = fmaxf(w1, red[2 * w + 1]);
          }
          if (w0 > 0.f)
            atomicMax(reinterpret_cast<unsigned*>(p.hsc + (size_t)(p.r0 + rlo) * 4 + p.amax_idx), __float_as_uint(w0));
          if (w1 > 0.f && rlo + 1 < p.R)
            atomicMax(reinterpret_cast<unsigned*>(p.hsc + (size_t)(p.r0 + rlo + 1) * 4 + p.amax_idx),
                      __float_as_uint(w1));
        }
      }
    }
  } else if constexpr (EMODE == 1) {
    // conv 3 (64 channels, bias + ReLU) -> final 1x1 64->17 + sigmoid per pixel
    constexpr int NKF = 17;
    float* fw = reinterpret_cast<float*>(lds);
#pragma unroll
    for (int u = 0; u < FPRE; ++u) {
      const int i = tid + u * NTH;
      if (i < NKF * 65) fw[i] = fin_pre[u];
    }
    __syncthreads();
    const int t4 = lane & 3, q4 = r16 >> 2;
    f32x4 v[FM][FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const float bj = p.bias[j * 16 + r16];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if constexpr (SPLIT) {
            const float u = m0 + wm * WM + i * 16 + g * 4 + e >= rbound ? us[1] : us[0];
            acc[i][j][e] = fmaxf(fmaf(acc[i][j][e], u, bj), 0.f);
          } else {
            acc[i][j][e] = fmaxf(acc[i][j][e] + bj, 0.f);
          }
        }
        v[i][j] = acc[i][j];
        quad_transpose(v[i][j], t4);
      }
    }
    float o[FM][NKF];
#pragma unroll
    for (int k = 0; k < NKF; ++k) {
      float a[FM];
#pragma unroll
      for (int i = 0; i < FM; ++i) a[i] = 0.f;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const float4 w4 = *reinterpret_cast<const float4*>(fw + k * 64 + j * 16 + q4 * 4);
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          a[i] = fmaf(w4.x, v[i][j][0], a[i]); a[i] = fmaf(w4.y, v[i][j][1], a[i]);
          a[i] = fmaf(w4.z, v[i][j][2], a[i]); a[i] = fmaf(w4.w, v[i][j][3], a[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        // sum over the 4 lanes of the row with the same (lane & 3): DPP
        // butterfly (no LDS round trip as with a shuffle), lane-symmetric
        a[i] = dpp_sum_xor4_8(a[i], lane);
        o[i][k] = a[i];
      }
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = m0 + wm * WM + i * 16 + g * 4 + t4;
      int rl, yy, xx;
      if (!interior(m, rl, yy, xx)) continue;
      const int r = p.r0 + rl, sl = p.slot[r], bimg = r / p.P;
      const int pos = sl >= 0 ? sl : slot_pos(sl);
      float* dst = p.heat + ((size_t)(bimg * p.P + pos) * NKF) * (HMS * HMS) + yy * HMS + xx;
#pragma unroll
      for (int s4 = 0; s4 < (NKF + 3) / 4; ++s4) {
        const int k = s4 * 4 + q4;
        float val = q4 == 0 ? o[i][s4 * 4] : 0.f;
        if (s4 * 4 + 1 < NKF && q4 == 1) val = o[i][s4 * 4 + 1];
        if (s4 * 4 + 2 < NKF && q4 == 2) val = o[i][s4 * 4 + 2];
        if (s4 * 4 + 3 < NKF && q4 == 3) val = o[i][s4 * 4 + 3];
        if (k < NKF) dst[(size_t)k * (HMS * HMS)] = sl >= 0 ? sigmoid_rcp(val + fw[NKF * 64 + k]) : 0.f;
      }
    }
  } else {
    // KEYPOINT_HEAD (keypoint_head.py:64-90, :25-27, :38-40), per output column co:
    //   v = relu6(conv * u + b[co]); v = relu6(v * ps[co] + pt[co])   (ResidualBlock.bn1; 1, 0 elsewhere)
    //   NTAP 10: v = relu6(v + downsample * u + bd[co])               (identity branch)
    // columns [0, ns) -> the next conv's split operand (padded map, scale os);
    // [ns, ns + nf) -> fp32 [R][56][56][nf] (adaptive-pool inputs); beyond: padding.
    if constexpr (BN == 128) {
      // The accumulators go through LDS in row parts (and the downsample's for
      // the first 64 columns), then a thread takes 8 consecutive columns of a
      // row: 16-byte stores of whole [hi32 | lo32] pieces / fp32 runs (the
      // per-fragment 8-byte stores took 16 % of a ResidualBlock-1 tile: 7.2 ->
      // 5.4 us; the 64-column convs with 16 / 32 live columns keep the
      // per-fragment stores, which skip the padding fragments)
      constexpr int KRP = kh_epi_parts<BMH>(), BR = BMH / KRP, WPR = WAVES_M / KRP, P1 = BN + 4, P2 = 68;
      static_assert(WAVES_M % KRP == 0 && BR % WM == 0, "KEYPOINT_HEAD epilogue row parts");
      static_assert(kh_epi_bytes<BN, BMH>() <= hmconv_lds_bytes<BN, SB, BMH, SPLIT, TPS, NW, MODE, NAB>(),
                    "KEYPOINT_HEAD epilogue stage");
      float* t1 = reinterpret_cast<float*>(lds);
      float* t2 = t1 + BR * P1;
      constexpr int C8 = BN / 8, RS = NTH / C8, IT = (BR + RS - 1) / RS;
      const int c8 = tid % C8, row0 = tid / C8, cl = c8 * 8, co = n0 + cl;
      const bool live = co < p.ns + p.nf;   // ns % 32 == 0, nf % 16 == 0: a group is all split, all fp32 or padding
      auto relu6 = [](float x) { return fminf(fmaxf(x, 0.f), 6.f); };
      float bv[8], sv[8], tv[8], dv[8];
  #pragma unroll
      for (int e = 0; e < 8; ++e) bv[e] = sv[e] = tv[e] = dv[e] = 0.f;
      if (live) {
  #pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float4 bb = *reinterpret_cast<const float4*>(p.bias + co + 4 * h);
          const float4 ps = *reinterpret_cast<const float4*>(p.kh_ps + co + 4 * h);
          const float4 pt = *reinterpret_cast<const float4*>(p.kh_pt + co + 4 * h);
          bv[4 * h] = bb.x; bv[4 * h + 1] = bb.y; bv[4 * h + 2] = bb.z; bv[4 * h + 3] = bb.w;
          sv[4 * h] = ps.x; sv[4 * h + 1] = ps.y; sv[4 * h + 2] = ps.z; sv[4 * h + 3] = ps.w;
          tv[4 * h] = pt.x; tv[4 * h + 1] = pt.y; tv[4 * h + 2] = pt.z; tv[4 * h + 3] = pt.w;
          if constexpr (NTAP == 10) {
            const float4 bd = *reinterpret_cast<const float4*>(p.kh_bd + co + 4 * h);
            dv[4 * h] = bd.x; dv[4 * h + 1] = bd.y; dv[4 * h + 2] = bd.z; dv[4 * h + 3] = bd.w;
          }
        }
      }
  #pragma unroll
      for (int pr = 0; pr < KRP; ++pr) {
        if (pr) __syncthreads();   // the previous part's reads are done
        if (wm / WPR == pr) {
          acc_to_lds<FM, FN, WM, 64, BN>(t1, acc, wm % WPR, wn, lane);
          if constexpr (NTAP == 10)
            if (wn == 0) acc_to_lds<FM, FN, WM, 64, 64>(t2, acc2, wm % WPR, 0, lane);
        }
        __syncthreads();
        if (!live) continue;
  #pragma unroll
        for (int it = 0; it < IT; ++it) {
          const int row = row0 + it * RS, m = m0 + pr * BR + row;
          int r, yy, xx;
          if (row >= BR || !interior(m, r, yy, xx)) continue;
          const int q = m >= rbound;
          const float u = q ? us[1] : us[0];
          const float4 x0 = *reinterpret_cast<const float4*>(t1 + row * P1 + cl);
          const float4 x1 = *reinterpret_cast<const float4*>(t1 + row * P1 + cl + 4);
          const float xa[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
          float da[8];
  #pragma unroll
          for (int e = 0; e < 8; ++e) da[e] = 0.f;
          if constexpr (NTAP == 10) {
            if (cl < 64) {
              const float4 d0 = *reinterpret_cast<const float4*>(t2 + row * P2 + cl);
              const float4 d1 = *reinterpret_cast<const float4*>(t2 + row * P2 + cl + 4);
              da[0] = d0.x; da[1] = d0.y; da[2] = d0.z; da[3] = d0.w;
              da[4] = d1.x; da[5] = d1.y; da[6] = d1.z; da[7] = d1.w;
            }
          }
          float o[8];
  #pragma unroll
          for (int e = 0; e < 8; ++e) {
            float x = relu6(fmaf(xa[e], u, bv[e]));
            x = relu6(fmaf(x, sv[e], tv[e]));
            if constexpr (NTAP == 10) x = relu6(x + fmaf(da[e], u, dv[e]));
            o[e] = x;
          }
          if (co < p.ns) {
            const float sc = q ? os[1] : os[0];
            f16x8 hi, lo;
  #pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float xs = o[e] * sc;
              hi[e] = (_Float16)xs;
              lo[e] = (_Float16)(xs - (float)hi[e]);
            }
            char* ob = static_cast<char*>(p.out) + (size_t)m * (p.ns * 4) + (co >> 5) * 128 + (co & 31) * 2;
            *reinterpret_cast<f16x8*>(ob) = hi;
            *reinterpret_cast<f16x8*>(ob + 64) = lo;
          } else {
            float* of = p.outf + ((size_t)r * HMS * HMS + yy * HMS + xx) * p.nf + (co - p.ns);
            *reinterpret_cast<float4*>(of) = make_float4(o[0], o[1], o[2], o[3]);
            *reinterpret_cast<float4*>(of + 4) = make_float4(o[4], o[5], o[6], o[7]);
          }
        }
      }
  
    } else {
      // A DPP quad transpose gives each lane 4 consecutive columns of one row.
      const int t4 = lane & 3, q4 = r16 >> 2;
  #pragma unroll
      for (int i = 0; i < FM; ++i)
  #pragma unroll
        for (int j = 0; j < FN; ++j) {
          quad_transpose(acc[i][j], t4);
          if constexpr (NTAP == 10) quad_transpose(acc2[i][j], t4);
        }
      auto relu6 = [](float x) { return fminf(fmaxf(x, 0.f), 6.f); };
  #pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int co = n0 + wn * 64 + j * 16 + q4 * 4;
        if (co >= p.ns + p.nf) continue;
        const float4 bb = *reinterpret_cast<const float4*>(p.bias + co);
        const float4 ps = *reinterpret_cast<const float4*>(p.kh_ps + co);
        const float4 pt = *reinterpret_cast<const float4*>(p.kh_pt + co);
        float4 bd = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (NTAP == 10) bd = *reinterpret_cast<const float4*>(p.kh_bd + co);
        const float bv[4] = {bb.x, bb.y, bb.z, bb.w}, sv[4] = {ps.x, ps.y, ps.z, ps.w}, tv[4] = {pt.x, pt.y, pt.z, pt.w};
        const float dv[4] = {bd.x, bd.y, bd.z, bd.w};
  #pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int m = m0 + wm * WM + i * 16 + g * 4 + t4;
          int r, yy, xx;
          if (!interior(m, r, yy, xx)) continue;
          const int q = m >= rbound;
          const float u = q ? us[1] : us[0];
          float o[4];
  #pragma unroll
          for (int e = 0; e < 4; ++e) {
            float x = relu6(fmaf(acc[i][j][e], u, bv[e]));
            x = relu6(fmaf(x, sv[e], tv[e]));
            if constexpr (NTAP == 10) x = relu6(x + fmaf(acc2[i][j][e], u, dv[e]));
            o[e] = x;
          }
          if (co < p.ns) {
            const float sc = q ? os[1] : os[0];
            f16x4 hi, lo;
  #pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float xs = o[e] * sc;
              hi[e] = (_Float16)xs;
              lo[e] = (_Float16)(xs - (float)hi[e]);
            }
            char* ob = static_cast<char*>(p.out) + (size_t)m * (p.ns * 4) + (co >> 5) * 128 + (co & 31) * 2;
            *reinterpret_cast<f16x4*>(ob) = hi;
            *reinterpret_cast<f16x4*>(ob + 64) = lo;
          } else {
            *reinterpret_cast<float4*>(p.outf + ((size_t)r * HMS * HMS + yy * HMS + xx) * p.nf +
                                       (co - p.ns)) = make_float4(o[0], o[1], o[2], o[3]);
          }
        }
      }
  
    }
  }
  if (p.stamps) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp16(p.stamps, 3);
    stamp16(p.stamps, 5, (unsigned long long)KT);
  }
}

template <int BN, int SB, int DBG = 0, int BMH = BM, bool SPLIT = false, int CIN = 0, int TPS = 1, bool DB = false,
          int NW = 8, int MODE = -1, int NTAP = 9>
__global__ __launch_bounds__(NW * 64) void hmconv_kernel(const HmConvArgs p) {
  __shared__ __attribute__((aligned(1024))) char lds[hmconv_lds_bytes<BN, SB, BMH, SPLIT, TPS, NW, MODE,
                                                                      hm_nab<CIN, SPLIT>()>()];
  hmconv_tile<BN, SB, DBG, BMH, SPLIT, CIN, TPS, DB, NW, MODE, NTAP>(p, lds, xcd_remap(blockIdx.x, gridDim.x),
                                                                        p.m_off);
}

// Persistent heatmap conv 1 / conv 2 (split, BN = cout = 256): one
// workgroup per CU walks full 224-row tiles t = w, w + G, ... (w: the
// XCD-contiguous rank of the workgroup, as xcd_remap) and then tail tile w of
// 192 rows if w < mix_H; each tile issues the next one's prologue (chunk 0
// window + B(0)) before its epilogue (hmconv_tile PST).  mix_F full tiles
// (whole rounds), mix_H tail tiles (exact count, <= G).
// the kernel's argument block re-read from the kernarg segment (scalar loads;
// the asm hides the pointer's provenance so that nothing is kept live across
// a persistent loop's iterations)
template <typename T>
__device__ __forceinline__ void kernarg_copy(T& dst) {
  typedef const __attribute__((address_space(4))) unsigned* KaPtr;
  KaPtr ka = (KaPtr)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(ka));
  static_assert(sizeof(T) % 4 == 0, "argument block");
  unsigned* d = reinterpret_cast<unsigned*>(&dst);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); ++i) d[i] = ka[i];
}

template <int CIN>
__global__ __launch_bounds__(512) void hmconv_persist_kernel(const HmConvArgs p) {
  __shared__ __attribute__((aligned(1024))) char lds[hmconv_lds_bytes<256, 2, 224, true, 1, 8, -1>()];
  const int G = gridDim.x, w = xcd_remap(blockIdx.x, G);
  const int F = p.mix_F, H = p.mix_H, tail_off = p.m_off + F * 224;
  bool pre = false;
  for (int t = w; t < F; t += G) {
    // the arguments are re-read from the kernarg segment every tile (scalar
    // loads) instead of held in SGPRs across the loop: the held copy pushed
    // the tile body past the register budget (spills)
    HmConvArgs pl;
    kernarg_copy(pl);
    const int nt = t + G;
    const int next_m0 = nt < F ? HP + pl.m_off + nt * 224 : (w < H ? HP + tail_off + w * 192 : -1);
    hmconv_tile<256, 2, 0, 224, true, CIN, 1, false, 8, -1, 9, true>(pl, lds, t, pl.m_off, pre, next_m0);
    pre = next_m0 >= 0;
  }
  if (w < H) {
    HmConvArgs pl;
    kernarg_copy(pl);
    hmconv_tile<256, 2, 0, 192, true, CIN, 1, false, 8, -1, 9, true>(pl, lds, w, tail_off, pre, -1);
  }
  wait_vmcnt<0>();
}

// Full rounds of BMH-row tiles and a last round of BMT-row tiles (the rows
// left over), in ONE launch whose first round mixes the two: on every XCD
// half of the first round's workgroups take a short tail tile, so those CUs
// run a tail-tile's length ahead of the others from then on.  The epilogues
// of a round (every CU writing its tile at once: 59 MB for heatmap conv 1 /
// 2 at 64 ROIs, HBM-bound) then come as two half bursts instead of one.  The
// makespan is the two-launch schedule's (each CU: full tiles + one tail).
// mix_F full tiles and mix_H tail tiles (multiples of 8: one share per XCD);
// per XCD x (blockIdx % 8) the blocks run in the order: mix_lead pairs (tail,
// full), the remaining full tiles, the remaining tail tiles; tile indices
// stay contiguous per XCD (L2 sharing of neighbouring windows, as xcd_remap).
template <int BN, int SB, int BMH, int BMT, int CIN, int TPS, bool DB, int MODE>
__global__ __launch_bounds__(512) void hmconv_mixed_kernel(const HmConvArgs p) {
  constexpr int LB = hmconv_lds_bytes<BN, SB, BMH, true, TPS, 8, MODE>(),
                LT = hmconv_lds_bytes<BN, SB, BMT, true, TPS, 8, MODE>();
  __shared__ __attribute__((aligned(1024))) char lds[LB > LT ? LB : LT];
  const int x = blockIdx.x % 8, k = blockIdx.x / 8;
  const int Fx = p.mix_F / 8, Hx = p.mix_H / 8, h0 = min(Hx, p.mix_lead);
  bool tail;
  int idx;
  if (k < 2 * h0) {
    tail = (k & 1) == 0;
    idx = k >> 1;
  } else if (k - 2 * h0 < Fx - h0) {
    tail = false;
    idx = h0 + (k - 2 * h0);
  } else {
    tail = true;
    idx = h0 + (k - 2 * h0 - (Fx - h0));
  }
  // (tile indices count M-tiles x column tiles: the full tiles cover mix_F / NTL M-tiles)
  if (tail) hmconv_tile<BN, SB, 0, BMT, true, CIN, TPS, DB, 8, MODE, 9>(p, lds, x * Hx + idx,
                                                                       p.m_off + (p.mix_F / (p.cout / BN)) * BMH);
  else hmconv_tile<BN, SB, 0, BMH, true, CIN, TPS, DB, 8, MODE, 9>(p, lds, x * Fx + idx, p.m_off);
}

constexpr long kMaxDesc = 0x7fffffffL;   // buffer descriptors take 31-bit extents

template <bool SPLIT, typename TO, int KS, int BN, int S, bool PF = (BN <= 128)>
hipError_t launch(const Conv16Args& a0, hipStream_t st) {
  constexpr long OS = sizeof(TO);
  Conv16Args a = a0;
  const long wt_bytes = (long)a.cout_p * KS * KS * a.cin_e * 2;
  const long HW = (long)a.H * a.W;
  const long img_bytes = HW * a.in_cstride * 2;
  if (wt_bytes > kMaxDesc || img_bytes > kMaxDesc) return hipErrorInvalidValue;
  a.wt_bytes = (int)wt_bytes;
  const int chunk = (int)std::min<long>(a.N, kMaxDesc / img_bytes);
  for (int n0 = 0; n0 < a0.N; n0 += chunk) {
    const int nb = std::min(chunk, a0.N - n0);
    a.N = nb;
    a.M = (int)(nb * HW);
    a.in = static_cast<const char*>(a0.in) + n0 * img_bytes;
    a.out = static_cast<char*>(a0.out) + n0 * HW * a.out_cstride * OS;
    a.stats = a0.stats ? a0.stats + (long)n0 * a.tiles_per_img * 2 * a.cout_p : nullptr;
    a.in_bytes = (int)(nb * img_bytes);
    a.r0 = a0.r0 + n0;
    dim3 grid(((a.M + BM - 1) / BM) * (a.cout_p / BN));
    hipLaunchKernelGGL((conv16_kernel<SPLIT, TO, KS, BN, S, PF>), grid, dim3(NT), 0, st, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace

int conv16_tile_m() { return BM; }

hipError_t launch_conv16(const Conv16Args& a, int split, int out_bf16, hipStream_t st) {
  if (a.M <= 0) return hipSuccess;
  if (a.cin_e % 64 != 0 || a.in_cstride % 8 != 0 || (a.stats && (a.H * a.W) % BM != 0))
    return hipErrorInvalidValue;
  if (split) {   // diagnostics only (kpd_bench_conv16)
    if (out_bf16 || a.cout_p != 128) return hipErrorInvalidValue;
    return launch<true, float, 3, 128, 3>(a, st);
  }
  if (a.cout_p % 256 == 0)
    return out_bf16 ? launch<false, __bf16, 3, 256, 2>(a, st) : launch<false, float, 3, 256, 2>(a, st);
  if (a.cout_p % 128 == 0)
    return out_bf16 ? launch<false, __bf16, 3, 128, 3>(a, st) : launch<false, float, 3, 128, 3>(a, st);
  if (a.cout_p % 64 == 0)
    return out_bf16 ? launch<false, __bf16, 3, 64, 3>(a, st) : launch<false, float, 3, 64, 3>(a, st);
  return hipErrorInvalidValue;
}

// KEYPOINT_HEAD convs (MODE 2): cin 128 / 64 / 32 (compile-time), cout 128 or
// 64 (one column tile), the downsample as a tenth tap or not
static hipError_t launch_hmconv_kh(const HmConvArgs& a0, hipStream_t st) {
  if (!a0.split || !a0.hsc || a0.in_idx < 0 || a0.in_idx > 3 || (a0.ns > 0 && (!a0.out || a0.out_idx < 0 ||
      a0.out_idx > 3 || a0.ns % 32)) || (a0.nf > 0 && !a0.outf) || a0.nf % 16 || a0.ns + a0.nf > a0.cout ||
      (a0.ntap != 9 && a0.ntap != 10) || (a0.ntap == 10 && !a0.kh_bd) || !a0.kh_pt || !a0.bias)
    return hipErrorInvalidValue;
  const int sel = (a0.cin == 128 && a0.cout == 128 && a0.ntap == 10) ? 1
                : (a0.cin == 64 && a0.cout == 64 && a0.ntap == 10) ? 2
                : (a0.cin == 32 && a0.cout == 64 && a0.ntap == 9) ? 3 : 0;
  if (!sel) return hipErrorInvalidValue;
  // the staged BN = 128 epilogue adds the downsample (tenth-tap) accumulator
  // to columns 0..63 only: a wider identity branch is not expressible there
  if (sel == 1 && a0.ns > 64) return hipErrorInvalidValue;
  HmConvArgs a = a0;
  const long wt_bytes = (long)a.cout * a.ntap * a.cin * 4, roi_bytes = (long)HPP * a.cin * 4;
  if (wt_bytes > kMaxDesc) return hipErrorInvalidValue;
  a.wt_bytes = (int)wt_bytes;
  a.m_off = 0;
  // staggered DMA issue (waves 4-7 one pass later, as the heatmap convs):
  // KEYPOINT_HEAD stage at C3 4.41 / 4.51 vs 4.53 / 4.58 ms (same-box A/B,
  // KPD_KH_NOSTAGGER=1: off)
  static const bool kh_nostagger = kpd_diag_env("KPD_KH_NOSTAGGER") != nullptr;
  a.stagger = kh_nostagger ? 0 : 1;
  // one launch for all ROIs (the kernel's input descriptor is per tile); the
  // GEMM row index stays a 32-bit int
  if ((long)a0.R * HPP >= 0x7fffffffL) return hipErrorInvalidValue;
  const int chunk = a0.R;
  for (int r0 = 0; r0 < a0.R; r0 += chunk) {
    const int nr = std::min(chunk, a0.R - r0);
    a.R = nr;
    a.r0 = a0.r0 + r0;
    a.in = static_cast<const char*>(a0.in) + (size_t)r0 * roi_bytes;
    if (a0.out) a.out = static_cast<char*>(a0.out) + (size_t)r0 * HPP * a.ns * 4;
    if (a0.outf) a.outf = a0.outf + (size_t)r0 * HMS * HMS * a.nf;
    a.in_bytes = (int)std::min<long>((long)nr * roi_bytes, kMaxDesc);   // (unused: per-tile descriptors)
    const long rows = (long)nr * HPP - HP;
    const dim3 grid((unsigned)((rows + BM - 1) / BM));
    // the regression conv (cin 32: one input chunk, one window per tile)
    // takes 512-row tiles: 64 x 64 per wave (0.83 fragment reads per MFMA
    // instead of 1.0) and half the per-tile prologues / epilogues of its
    // 3 K-steps
    const dim3 grid512((unsigned)((rows + 511) / 512));
    // ResidualBlock 2 (cin 64, 32 live columns): 384-row tiles, 48 x 64 per
    // wave (a 512-row window pair + two weight stages fill the 160 KB)
    const dim3 grid384((unsigned)((rows + 383) / 384));
    static const bool kh_bm256 = kpd_diag_env("KPD_KH_BM256") != nullptr;   // A/B: 256-row tiles for both
    // two taps per K-step (three for the 32-channel conv): one barrier per
    // 2-3 taps of MFMAs -- these convs have 96 / 32 / 16 live output columns,
    // so a single tap's MFMAs are too few to amortise a barrier and the DMA
    // issue (MFMA busy 0.37 at one tap per step).  KPD_KH_TPS1=1: one tap (A/B).
    static const bool tps1 = kpd_diag_env("KPD_KH_TPS1") != nullptr;
    if (tps1) {
      if (sel == 1) hipLaunchKernelGGL((hmconv_kernel<128, 3, 0, BM, true, 128, 1, false, 8, 2, 10>), grid, dim3(NT), 0, st, a);
      else if (sel == 2) hipLaunchKernelGGL((hmconv_kernel<64, 4, 0, BM, true, 64, 1, false, 8, 2, 10>), grid, dim3(NT), 0, st, a);
      else hipLaunchKernelGGL((hmconv_kernel<64, 4, 0, BM, true, 32, 1, false, 8, 2, 9>), grid, dim3(NT), 0, st, a);
    } else if (kh_bm256) {
      if (sel == 1) hipLaunchKernelGGL((hmconv_kernel<128, 2, 0, BM, true, 128, 2, false, 8, 2, 10>), grid, dim3(NT), 0, st, a);
      else if (sel == 2) hipLaunchKernelGGL((hmconv_kernel<64, 2, 0, BM, true, 64, 2, false, 8, 2, 10>), grid, dim3(NT), 0, st, a);
      else hipLaunchKernelGGL((hmconv_kernel<64, 2, 0, BM, true, 32, 3, false, 8, 2, 9>), grid, dim3(NT), 0, st, a);
    } else {
      if (sel == 1) hipLaunchKernelGGL((hmconv_kernel<128, 2, 0, BM, true, 128, 2, false, 8, 2, 10>), grid, dim3(NT), 0, st, a);
      else if (sel == 2) hipLaunchKernelGGL((hmconv_kernel<64, 2, 0, 384, true, 64, 2, false, 8, 2, 10>), grid384, dim3(NT), 0, st, a);
      else hipLaunchKernelGGL((hmconv_kernel<64, 2, 0, 512, true, 32, 3, false, 8, 2, 9>), grid512, dim3(NT), 0, st, a);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// Linear mode (outf set, out / fin / kh_ps null; split): fp32 NHWC output of
// acc * u + bias, no activation -- the conv3x3 forward and dgrad of K6
// (conv3_grad.hip) on the heatmap convs' 56 x 56 maps; cin 64 or 256, cout 256
// (or 128: a 64-channel output padded with zero weights).
static hipError_t launch_hmconv_linear(const HmConvArgs& a0, hipStream_t st) {
  if (!a0.split || !a0.hsc || a0.in_idx < 0 || a0.in_idx > 3 || !a0.bias || (a0.cout != 256 && a0.cout != 128) ||
      (a0.cin != 64 && a0.cin != 256) || (long)a0.R * HPP >= 0x7fffffffL)
    return hipErrorInvalidValue;
  HmConvArgs a = a0;
  const long wt_bytes = (long)a.cout * 9 * a.cin * 4;
  if (wt_bytes > kMaxDesc) return hipErrorInvalidValue;
  a.wt_bytes = (int)wt_bytes;
  a.m_off = 0;
  a.r0 = 0;
  a.stagger = 1;
  a.out_idx = -1;
  a.amax_idx = -1;
  a.in_bytes = (int)std::min<long>((long)a.R * HPP * a.cin * 4, kMaxDesc);
  const long rows = (long)a.R * HPP - HP;
  // cout 256: the heatmap conv 1 / 2 tiles (224 x 256, 2-stage weight ring);
  // cout 128: 256 x 128 tiles with a 4-stage ring (the split BN = 128 variant)
  if (a.cout == 256) {
    const dim3 grid((unsigned)((rows + 223) / 224));
    if (a.cin == 64) hipLaunchKernelGGL((hmconv_kernel<256, 2, 0, 224, true, 64, 1, false, 8, 3>), grid, dim3(NT), 0, st, a);
    else hipLaunchKernelGGL((hmconv_kernel<256, 2, 0, 224, true, 256, 1, false, 8, 3>), grid, dim3(NT), 0, st, a);
  } else {
    const dim3 grid((unsigned)((rows + BM - 1) / BM));
    if (a.cin == 64) hipLaunchKernelGGL((hmconv_kernel<128, 4, 0, BM, true, 64, 1, false, 8, 3>), grid, dim3(NT), 0, st, a);
    else hipLaunchKernelGGL((hmconv_kernel<128, 4, 0, BM, true, 256, 1, false, 8, 3>), grid, dim3(NT), 0, st, a);
  }
  return hipGetLastError();
}

hipError_t launch_hmconv(const HmConvArgs& a0, hipStream_t st) {
  if (a0.R <= 0) return hipSuccess;
  if (a0.kh_ps) return launch_hmconv_kh(a0, st);
  if (a0.outf && !a0.out && !a0.fin_w) return launch_hmconv_linear(a0, st);
  const bool fin = a0.fin_w != nullptr, split = a0.split != 0;
  if (a0.cin % (split ? 32 : 64) || (fin ? a0.cout != 64 : a0.cout % 128) ||
      (fin && (!a0.slot || !a0.heat || !a0.fin_b)) || (!fin && !a0.out) ||
      (split && (!a0.hsc || a0.in_idx < 0 || a0.in_idx > 3 || a0.amax_idx > 3 || a0.out_idx > 3 ||
                 (!fin && a0.out_idx < 0))))
    return hipErrorInvalidValue;
  HmConvArgs a = a0;
  const long es = split ? 4 : 2;   // bytes per channel: bf16, or f16 hi + lo
  const long wt_bytes = (long)a.cout * 9 * a.cin * es, roi_bytes = (long)HPP * a.cin * es;
  if (wt_bytes > kMaxDesc) return hipErrorInvalidValue;
  a.wt_bytes = (int)wt_bytes;
  // one launch for all ROIs (the kernel's input descriptor is per tile, so
  // the 31-bit extent bounds a tile's window only); row indices stay 32-bit
  if ((long)a0.R * HPP >= 0x7fffffffL) return hipErrorInvalidValue;
  const int chunk = a0.R;
  for (int r0 = 0; r0 < a0.R; r0 += chunk) {
    const int nr = std::min(chunk, a0.R - r0);
    a.R = nr;
    a.r0 = a0.r0 + r0;
    a.in = static_cast<const char*>(a0.in) + (size_t)r0 * roi_bytes;
    if (!fin) a.out = static_cast<char*>(a0.out) + (size_t)r0 * HPP * a.cout * es;
    a.in_bytes = (int)std::min<long>((long)nr * roi_bytes, kMaxDesc);   // (unused: per-tile descriptors)
    const long rows = (long)nr * HPP - HP;
    // BN 256 with a 2-stage weight ring measured faster than BN 128 with 4
    // stages for conv 1 / 2 (89 / 233 us vs 92 / 256 us at 64 ROIs): the
    // wider tile halves the weight bytes per MFMA; conv 3 has 64 outputs
    const int bn = fin ? 64 : (a.cout % 256 == 0 ? 256 : 128);
    // BN 256: 224-row tiles when that packs the rounds of one workgroup per
    // CU better (64 ROIs: 961 tiles = 4 rounds of 224 rows instead of 841 =
    // 4 rounds of 256, the last one 29 % full)
    static int ncu = 0;
    if (!ncu) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
        ncu = 256;
    }
    static const int bm_env = kpd_diag_env("KPD_HMCONV_BM") ? atoi(kpd_diag_env("KPD_HMCONV_BM")) : 0;   // A/B
    auto cost = [&](long bm) { return ((rows + bm - 1) / bm * (a.cout / bn) + ncu - 1) / ncu * bm; };
    // conv 1 / 2 (cin 64 / 256) always take 224-row tiles: those are the
    // instances with the input channels as a compile-time constant (the
    // generic runtime-cin kernel ran conv 1 + 2 at 640 ROIs (C3) ~2x slower),
    // and conv 2's tail launch packs the last round
    const bool spec = a.cin == 64 || a.cin == 256;
    const int bm = fin || bn != 256 ? BM
                   : bm_env == 224 || bm_env == BM ? bm_env
                   : (spec || cost(224) < cost(BM)) ? 224 : BM;
    const dim3 grid((unsigned)(((rows + bm - 1) / bm) * (a.cout / bn)));
    static const int dbg = kpd_diag_env("KPD_HMCONV_DBG") ? atoi(kpd_diag_env("KPD_HMCONV_DBG")) : 0;   // ablations only
    static const int hm_tps = kpd_diag_env("KPD_HM3_TPS1") ? -1 : 0;   // A/B: conv 3 with one tap per K-step
    static const bool hm_db = kpd_diag_env("KPD_HM3_NODB") == nullptr;  // A/B: conv 3 single fragment set
    static const bool hm_stagger = kpd_diag_env("KPD_HM_NOSTAGGER") == nullptr;   // A/B: staggered DMA issue (split)
    a.stagger = hm_stagger ? 1 : 0;
#define HMK(...) hipLaunchKernelGGL((hmconv_kernel<__VA_ARGS__>), grid, dim3(NT), 0, st, a)
    // conv 3 (BN 64, one tile per CU round): the rounds after the last full
    // one would run a partial round of 256-row tiles (64 ROIs: 841 tiles =
    // 3.3 rounds, the 4th 29 % full).  Instead the full rounds take 256-row
    // tiles and the rest goes out as 128-row tiles in one extra launch
    // (146 at 64 ROIs: a half-length round).  Tile sizes never change the
    // arithmetic of a row (same K order), so results are unchanged.
    static const bool no_tail = kpd_diag_env("KPD_HM3_NOTAIL") != nullptr;   // A/B
    // A/B (KPD_HM3_NW4=1): conv 3 split as 4 waves of 64 x 64 -- 1.5x fewer LDS
    // bytes per MFMA, but one wave per SIMD hides no latency: 0.204 vs 0.173 ms
    static const bool hm3_nw4 = kpd_diag_env("KPD_HM3_NW4") != nullptr;
    a.m_off = 0;
    // one launch for the full rounds and the tail round, the first round
    // mixing both tile heights (hmconv_mixed_kernel).  Same-box A/B (round 4,
    // 64 ROIs): conv 1 178 / 180 vs 183 / 182 us (it had no tail launch, so
    // it also gains the tail tiles' packing), conv 2 502 / 504 vs 500 / 500,
    // conv 3 182 / 185 vs 178 / 174 -- on for conv 1 only (KPD_HM_MIX=0: off,
    // 2: conv 2 / conv 3 too)
    static const int mix_env = kpd_diag_env("KPD_HM_MIX") ? atoi(kpd_diag_env("KPD_HM_MIX")) : 1;
    const bool no_mix = mix_env == 0 || (mix_env == 1 && a.cin != 64);
    auto mix_ok = [&](long F, long H) { return !no_mix && ncu % 8 == 0 && F >= ncu && H > 0 && H <= ncu; };
    auto mix_set = [&](HmConvArgs& m, long F, long H, dim3& g) {
      m.mix_F = (int)F;
      m.mix_H = (int)((H + 7) / 8 * 8);   // a share per XCD; tiles past the rows return at once
      m.mix_lead = ncu / 16;              // half of each XCD's CUs start with a tail tile
      g = dim3((unsigned)(m.mix_F + m.mix_H));
    };
    if (fin && !dbg && !no_tail && !a.stamps && (!split || (a.cin == 256 && hm_db))) {
      const long nfull = rows / BM, F = nfull / ncu * ncu, rem = rows - F * BM, H = (rem + 127) / 128;
      if (split && mix_ok(F, H)) {
        HmConvArgs m = a;
        dim3 g;
        mix_set(m, F, H, g);
        hipLaunchKernelGGL((hmconv_mixed_kernel<64, 2, BM, 128, 256, 3, true, -1>), g, dim3(NT), 0, st, m);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        continue;
      }
      if (F > 0 && H > 0 && H <= ncu) {
        const dim3 g1((unsigned)F), g2((unsigned)H);
        HmConvArgs a2 = a;
        a2.m_off = (int)(F * BM);
        if (split && hm3_nw4) {
          hipLaunchKernelGGL((hmconv_kernel<64, 2, 0, BM, true, 256, 3, true, 4>), g1, dim3(256), 0, st, a);
          hipLaunchKernelGGL((hmconv_kernel<64, 2, 0, 128, true, 256, 3, true, 4>), g2, dim3(256), 0, st, a2);
        } else if (split) {
          hipLaunchKernelGGL((hmconv_kernel<64, 2, 0, BM, true, 256, 3, true>), g1, dim3(NT), 0, st, a);
          hipLaunchKernelGGL((hmconv_kernel<64, 2, 0, 128, true, 256, 3, true>), g2, dim3(NT), 0, st, a2);
        } else {
          hipLaunchKernelGGL((hmconv_kernel<64, 4>), g1, dim3(NT), 0, st, a);
          hipLaunchKernelGGL((hmconv_kernel<64, 4, 0, 128>), g2, dim3(NT), 0, st, a2);
        }
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        continue;
      }
    }
    // conv 2 (split, 224-row tiles): complete rounds of 224-row tiles, then
    // the remaining rows as 192-row tiles in a second launch when they fit
    // one round (64 ROIs: 768 + 225 tiles instead of 961, the last round
    // 0.86 as long): 0.528 -> 0.515 ms.  Conv 1 (18 K-steps a tile, so the
    // per-tile prologue / epilogue dominate) measured 2 % slower with it.
    // Same K order per row: results unchanged.
    static const bool no_tail12 = kpd_diag_env("KPD_HM12_NOTAIL") != nullptr;   // A/B
#if KPD_DIAG
    // A/B (KPD_HM_PERSIST=1): conv 1 / conv 2 persistent (hmconv_persist_kernel:
    // each tile's successor prologue issued under its epilogue).  Same-box
    // (round 4, 64 ROIs): conv 1 0.206 vs 0.174 ms, conv 2 0.503 vs 0.504 ms
    // -- not on by default
    static const int persist_env = kpd_diag_env("KPD_HM_PERSIST") ? atoi(kpd_diag_env("KPD_HM_PERSIST")) : 0;
    if (split && !fin && bn == 256 && bm == 224 && a.cout == 256 && (a.cin == 64 || a.cin == 256) && !dbg &&
        !a.stamps && persist_env) {
      const long F = rows / 224 / ncu * ncu, rem = rows - F * 224, H = (rem + 191) / 192;
      if (F > 0 && H <= ncu && F + H < 0x7fffffffL / 224) {
        HmConvArgs m = a;
        m.mix_F = (int)F;
        m.mix_H = (int)H;
        if (a.cin == 64) hipLaunchKernelGGL((hmconv_persist_kernel<64>), dim3((unsigned)ncu), dim3(NT), 0, st, m);
        else hipLaunchKernelGGL((hmconv_persist_kernel<256>), dim3((unsigned)ncu), dim3(NT), 0, st, m);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        continue;
      }
    }
#endif
    // tail tiles of conv 1 / conv 2: 160 rows when those fit one round (the
    // last round then runs 160-row instead of 192-row tiles), else 192
    const long F12 = rows / 224 / ncu * ncu, rem12 = rows - F12 * 224;
    const bool t160 = (rem12 + 159) / 160 <= ncu;
    const long H12 = t160 ? (rem12 + 159) / 160 : (rem12 + 191) / 192;
    if (split && !fin && bn == 256 && bm == 224 && (a.cin == 64 || a.cin == 256) && !dbg && !a.stamps) {
      if (mix_ok(F12, H12)) {   // conv 1 / conv 2
        HmConvArgs m = a;
        dim3 g;
        mix_set(m, F12, H12, g);
        if (a.cin == 64 && t160) hipLaunchKernelGGL((hmconv_mixed_kernel<256, 2, 224, 160, 64, 1, false, -1>), g, dim3(NT), 0, st, m);
        else if (a.cin == 64) hipLaunchKernelGGL((hmconv_mixed_kernel<256, 2, 224, 192, 64, 1, false, -1>), g, dim3(NT), 0, st, m);
        else if (t160) hipLaunchKernelGGL((hmconv_mixed_kernel<256, 2, 224, 160, 256, 1, false, -1>), g, dim3(NT), 0, st, m);
        else hipLaunchKernelGGL((hmconv_mixed_kernel<256, 2, 224, 192, 256, 1, false, -1>), g, dim3(NT), 0, st, m);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        continue;
      }
    }
    if (split && !fin && bn == 256 && bm == 224 && a.cin == 256 && !dbg && !no_tail12 && !a.stamps) {
      if (F12 > 0 && rem12 > 0 && H12 <= ncu) {
        const dim3 g1((unsigned)F12), g2((unsigned)H12);
        HmConvArgs a2 = a;
        a2.m_off = (int)(F12 * 224);
        hipLaunchKernelGGL((hmconv_kernel<256, 2, 0, 224, true, 256>), g1, dim3(NT), 0, st, a);
        if (t160) hipLaunchKernelGGL((hmconv_kernel<256, 2, 0, 160, true, 256>), g2, dim3(NT), 0, st, a2);
        else hipLaunchKernelGGL((hmconv_kernel<256, 2, 0, 192, true, 256>), g2, dim3(NT), 0, st, a2);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        continue;
      }
    }
#if KPD_DIAG
    if (split && dbg) {   // ablations (KPD_HMCONV_DBG=1: no MFMA, 2: no K-loop DMA); wrong results by design
      if (fin && dbg == 1) HMK(64, 2, 1, BM, true, 256, 3, true);   // the production conv 3 variant
      else if (fin) HMK(64, 2, 2, BM, true, 256, 3, true);
      else if (dbg == 1) HMK(256, 2, 1, 224, true, 256);
      else HMK(256, 2, 2, 224, true, 256);
    } else
#endif
    if (split) {
      if (fin && a.cin == 256 && hm_db && hm3_nw4)
        hipLaunchKernelGGL((hmconv_kernel<64, 2, 0, BM, true, 256, 3, true, 4>), grid, dim3(256), 0, st, a);
      else if (fin && a.cin == 256 && hm_db) HMK(64, 2, 0, BM, true, 256, 3, true);
      else if (fin && a.cin == 256 && !(hm_tps < 0)) HMK(64, 2, 0, BM, true, 256, 3);
      else if (fin && a.cin == 256) HMK(64, 4, 0, BM, true, 256);
      else if (fin) HMK(64, 4, 0, BM, true);
      else if (bn == 256 && bm == 224 && a.cin == 64) HMK(256, 2, 0, 224, true, 64);
      else if (bn == 256 && bm == 224 && a.cin == 256) HMK(256, 2, 0, 224, true, 256);
      else if (bn == 256 && bm == 224) HMK(256, 2, 0, 224, true);
      else if (bn == 256) HMK(256, 2, 0, BM, true);
      else HMK(128, 4, 0, BM, true);
    } else if (fin) hipLaunchKernelGGL((hmconv_kernel<64, 4>), grid, dim3(NT), 0, st, a);
    else if (bn == 256 && bm == 224 && dbg == 0 && a.cin == 64) HMK(256, 2, 0, 224, false, 64);
    else if (bn == 256 && bm == 224 && dbg == 0 && a.cin == 256) HMK(256, 2, 0, 224, false, 256);
    else if (bn == 256 && bm == 224 && dbg == 0) hipLaunchKernelGGL((hmconv_kernel<256, 2, 0, 224>), grid, dim3(NT), 0, st, a);
#if KPD_DIAG
    else if (bn == 256 && dbg == 1) hipLaunchKernelGGL((hmconv_kernel<256, 2, 1>), grid, dim3(NT), 0, st, a);
    else if (bn == 256 && dbg == 2) hipLaunchKernelGGL((hmconv_kernel<256, 2, 2>), grid, dim3(NT), 0, st, a);
#endif
    else if (bn == 256) hipLaunchKernelGGL((hmconv_kernel<256, 2>), grid, dim3(NT), 0, st, a);
    else hipLaunchKernelGGL((hmconv_kernel<128, 4>), grid, dim3(NT), 0, st, a);
#undef HMK
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_fpn0x(const Fpn0xArgs& a, hipStream_t st) {
  if (a.N <= 0) return hipSuccess;
  if (a.N > kFpn0xMaxImg || !a.sc || a.sc_n < a.N) return hipErrorInvalidValue;
  if (a.Hf != 4 * a.rh || a.Wf != 4 * a.rw || a.tpc != (a.rh * a.rw + BM - 1) / BM) return hipErrorInvalidValue;
  if ((long)a.tpc * BM >= 65536) return hipErrorInvalidValue;   // the kernel's float q / rw
  // 32-bit buffer offsets of the output and statistics stores
  if ((long)a.N * a.Hf * a.Wf * 512 >= (1L << 31) || (long)a.N * 16 * a.tpc * 1024 >= (1L << 31))
    return hipErrorInvalidValue;
  const long tiles = 16L * a.N * a.tpc;
  // persistent: one workgroup per CU (the kernel walks the tiles in rounds)
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
  }
  static const int grid_env = kpd_diag_env("KPD_FPN0X_GRID") ? atoi(kpd_diag_env("KPD_FPN0X_GRID")) : 0;   // A/B
  const long grid = std::min<long>(tiles, grid_env > 0 ? grid_env : ncu);
#if KPD_DIAG
  static const int dbg = kpd_diag_env("KPD_FPN0X_DBG") ? atoi(kpd_diag_env("KPD_FPN0X_DBG")) : 0;   // ablations only
#endif
  static const bool stagger = kpd_diag_env("KPD_FPN0X_NOSTAGGER") == nullptr;                   // A/B
  Fpn0xArgs b = a;
  b.stagger = stagger ? 1 : 0;
  // non-temporal output (KPD_FPN0X_NT=0: off): FETCH_SIZE 216 -> 162 MB per launch (the stores no longer
  // evict the weights and input rows from L2), -1 % time
  static const int out_nt = kpd_diag_env("KPD_FPN0X_NT") ? atoi(kpd_diag_env("KPD_FPN0X_NT")) : 1;
  b.out_nt = out_nt;
  // class-half tile order (the kernel's tile_at); KPD_FPN0X_ORDER=0: class-fastest rounds (A/B)
  static const int order = kpd_diag_env("KPD_FPN0X_ORDER") ? atoi(kpd_diag_env("KPD_FPN0X_ORDER")) : 1;
  // (every round must give each workgroup a tile until the last, so the
  // (image, row block) count must fill whole pairs of rounds: NJ a multiple
  // of grid / 8 and at least one pair)
  const long NJ = (long)a.N * a.tpc;
  b.order = (order && grid % 8 == 0 && NJ % (grid / 8) == 0 && NJ >= grid / 8) ? 1 : 0;
#if KPD_DIAG   // ablations (KPD_FPN0X_DBG=1: no MFMA, 2: no K-loop DMA, 4: one output piece); wrong results by design
  if (dbg == 1) hipLaunchKernelGGL(fpn0x_kernel<1>, dim3((unsigned)grid), dim3(NT), 0, st, b);
  else if (dbg == 2) hipLaunchKernelGGL(fpn0x_kernel<2>, dim3((unsigned)grid), dim3(NT), 0, st, b);
  else if (dbg == 4) hipLaunchKernelGGL(fpn0x_kernel<4>, dim3((unsigned)grid), dim3(NT), 0, st, b);
  else
#endif
  hipLaunchKernelGGL(fpn0x_kernel<0>, dim3((unsigned)grid), dim3(NT), 0, st, b);
  return hipGetLastError();
}

hipError_t launch_split_rows(const float* in, int N, long hw, int cin, const float* sc, int which, int w_exp0,
                             int w_expE, void* out, hipStream_t st) {
  if (cin != 16 && cin % 32 != 0) return hipErrorInvalidValue;
  const long n = (long)N * hw * (cin / 8);
  hipLaunchKernelGGL(split_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, in, N, hw, cin, sc,
                     which, w_exp0, w_expE, static_cast<_Float16*>(out));
  return hipGetLastError();
}

// ---------------------------------------------------------------- diagnostics
// Times conv16 variants on synthetic operands (DESIGN.md "K6b" measurements):
// split != 0 -> the FPN level-0 configuration (cin 128 as hi|lo, cout 128),
// else bf16 cin -> cout.  dbg selects the ablation (see DBG above).
template <int DBG>
static hipError_t bench_launch(const Conv16Args& a, int split, hipStream_t st) {
  if constexpr (DBG == 0) return launch_conv16(a, split, split ? 0 : 1, st);   // the production dispatch
  dim3 grid(((a.M + BM - 1) / BM) * (a.cout_p / 128));
  if (split) hipLaunchKernelGGL((conv16_kernel<true, float, 3, 128, 3, true, DBG>), grid, dim3(NT), 0, st, a);
  else hipLaunchKernelGGL((conv16_kernel<false, __bf16, 3, 128, 3, true, DBG>), grid, dim3(NT), 0, st, a);
  return hipGetLastError();
}

extern "C" int kpd_bench_conv16(int split, int N, int H, int W, int cin, int cout, int dbg, int iters, float* ms) {
  if (N <= 0 || H <= 0 || W <= 0 || cin % 64 || cout % 128 || iters <= 0 || !ms) return -1;
  if (split && (cin != 128 || cout != 128)) return -1;
  Conv16Args a{};
  const long M = (long)N * H * W;
  const int cin_e = split ? 2 * cin : cin;
  const long in_b = M * cin_e * 2, w_b = (long)cout * 9 * cin_e * 2, out_b = M * cout * 4;
  if (in_b > kMaxDesc) return -1;
  void *in = nullptr, *wt = nullptr, *out = nullptr, *bias = nullptr, *stats = nullptr;
  const bool with_stats = split && ((long)H * W) % BM == 0;   // as FPN0 runs: top-k statistics fused
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int rc = -2;
  if (hipMalloc(&in, in_b) != hipSuccess || hipMalloc(&wt, w_b) != hipSuccess || hipMalloc(&out, out_b) != hipSuccess ||
      hipMalloc(&bias, cout * 4) != hipSuccess ||
      (with_stats && hipMalloc(&stats, (size_t)N * (H * W / BM) * 2 * cout * 4) != hipSuccess))
    goto done;
  (void)hipMemset(in, 0x3C, in_b);
  (void)hipMemset(wt, 0x3A, w_b);
  (void)hipMemset(bias, 0, cout * 4);
  a.in = in; a.wt = wt; a.bias = (const float*)bias; a.out = out; a.N = N; a.H = H; a.W = W; a.cin_e = cin_e;
  a.cout_p = cout; a.in_cstride = cin_e; a.out_cstride = cout; a.act = ACT_RELU; a.M = (int)M;
  a.split_scale = 1.f;
  a.in_bytes = (int)in_b; a.wt_bytes = (int)w_b;
  if (with_stats) { a.stats = (float*)stats; a.tiles_per_img = H * W / BM; }
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) goto done;
  for (int it = -2; it < iters; ++it) {
    if (it == 0) (void)hipEventRecord(e0, 0);
    hipError_t e = hipSuccess;
    switch (dbg) {
      case 0: e = bench_launch<0>(a, split, 0); break;
#if KPD_DIAG   // ablation variants (wrong results by design): diagnostic builds only
      case 1: e = bench_launch<1>(a, split, 0); break;
      case 2: e = bench_launch<2>(a, split, 0); break;
      case 4: e = bench_launch<4>(a, split, 0); break;
      case 8: e = bench_launch<8>(a, split, 0); break;
      case 65536: e = bench_launch<65536>(a, split, 0); break;   // BN=128, S=3, PF (no ablation)
      case 16: e = bench_launch<16>(a, split, 0); break;
      case 24: e = bench_launch<24>(a, split, 0); break;
      case 128: e = bench_launch<128>(a, split, 0); break;
      case 4096: e = bench_launch<4096>(a, split, 0); break;
#endif
      default: e = hipErrorInvalidValue;
    }
    if (e != hipSuccess) goto done;
  }
  (void)hipEventRecord(e1, 0);
  if (hipEventSynchronize(e1) != hipSuccess) goto done;
  (void)hipEventElapsedTime(ms, e0, e1);
  *ms /= iters;
  rc = 0;
done:
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  (void)hipFree(in); (void)hipFree(wt); (void)hipFree(out); (void)hipFree(bias);
  (void)hipFree(stats);
  return rc;
}
