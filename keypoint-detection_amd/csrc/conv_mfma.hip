// Implicit-GEMM stride-1 "same" convolution (KSxKS, KS in {1,3}) on gfx950 MFMA.
//
//   out[m, co] = act( sum_k A[m, k] * Bw[co, k] + bias[co] ) (+ residual)
//   m = pixel (n, y, x) of an NHWC tensor, k = (tap, ci), tap = (ky, kx)
//
// Hot path users (reference file:line):
//   * FPN level-0 3x3 128->128 + BN + ReLU       dll/models/backbone.py:20-27,39
//   * FPN 1x1 laterals + nearest top-down add     dll/models/backbone.py:15-18,33-37
//   * MobileNetV3 pointwise expand/project 1x1    torchvision InvertedResidual (backbone.py:250)
//   * HeatmapHead 3x3 convs (+bias+BN+ReLU)       dll/models/heatmap_head.py:31-45,55-66
//   * KEYPOINT_HEAD convs                          dll/models/keypoint_head.py:21-44,64-90
//
// Design (MI355X-first, see DESIGN.md "K6"):
//   * 256-thread workgroups = 4 waves in a 2x2 grid; each wave owns a
//     (BM/2)x(BN/2) output tile built from 16x16 MFMA fragments.
//   * fp32 operands use v_mfma_f32_16x16x4_f32 (exact fp32 products, the
//     numerics the channel top-k needs); bf16 operands use
//     v_mfma_f32_16x16x32_bf16 with fp32 accumulation.
//   * Both read one 16-byte LDS chunk per lane per fragment: for bf16 that is
//     the native 8-element k-slice; for fp32 the k order inside a 16-wide
//     k-step is permuted (lane-group g holds k = 4g..4g+3 and feeds element s
//     to MFMA s) -- legal because A and B use the same permutation.
//   * Global->LDS is register-staged and double buffered: the next K-tile is
//     in flight while MFMAs run on the current one; one barrier per K-tile.
//     K order: channel chunks outer, taps inner (L2 reuse of the halo rows).
//   * Global loads are buffer loads with 32-bit per-lane offsets fixed over
//     K; the 3x3 halo and the M tail are zero-filled by the buffer
//     descriptor's range check (no predicated loads, no branches).
//   * Epilogue fuses bias (BN folded on the host), activation, residual add
//     with optional nearest-upsample indexing (FPN top-down), per-image
//     channel sum/max partials (ChannelAttention pooling), bf16/fp32 stores.
#include <algorithm>
#include "kpd_common.h"
#include "kpd_kernels.h"
#include "conv_epilogue.h"

namespace {

template <typename TA, typename TO, int KS, int BM, int BN, int BK, bool PF2 = false>
__global__ __launch_bounds__(256) void conv_mfma_kernel(const ConvArgs p) {
  constexpr int ES = sizeof(TA);
  constexpr int ROWB = BK * ES;           // bytes of one LDS row (one K-tile of one row)
  constexpr int CPR = ROWB / 16;          // 16-byte chunks per row
  constexpr int LDSROW = ROWB;            // unpadded; 16-B chunks XOR-swizzled (lds_chunk)
  constexpr int EPC = 16 / ES;            // elements per chunk
  constexpr int A_TOT = BM * CPR, B_TOT = BN * CPR;
  constexpr int NA = (A_TOT + 255) / 256, NB = (B_TOT + 255) / 256;
  constexpr int WM = BM / 2, WN = BN / 2, FM = WM / 16, FN = WN / 16;
  constexpr int KSTEPS = ROWB / 64;       // 4 lane groups x 16 B per k-step
  constexpr int BUF_A = BM * LDSROW, BUF_B = BN * LDSROW;
  constexpr unsigned OOB = 0x80000000u;   // out-of-range voffset: the buffer load returns 0
  static_assert(FM >= 1 && FN >= 1, "tile too small");
  static_assert(ROWB % 64 == 0, "BK must cover 64 bytes");

  constexpr int MAIN_LDS = 2 * (BUF_A + BUF_B);
  // BN = 128: the epilogue stages one 64-column half at a time (the two wave
  // columns in turn), halving its LDS -- the occupancy limiter of the
  // latency-bound small-K 1x1 convs
  constexpr int EBN = BN == 128 ? 64 : BN, HALVES = BN / EBN;
  constexpr int EPI_LDS = epi_lds_bytes<BM, EBN>();
  __shared__ __attribute__((aligned(16))) char lds[MAIN_LDS > EPI_LDS ? MAIN_LDS : EPI_LDS];
  char* As = lds;
  char* Bs = lds + 2 * BUF_A;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // 1-D grid: N-tile fastest (N-tiles of one M-tile share the A tile), XCD-aware order
  const int NT = (p.cout_p + BN - 1) / BN;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (L / NT) * BM, n0 = (L % NT) * BN;
  const int H = p.H, W = p.W, HW = H * W, M = p.M;
  const int cin_p = p.cin_p, cout_p = p.cout_p;

  // Buffer descriptors (wave-uniform kernargs): 32-bit offsets, hardware range
  // check -> halo / tail lanes get 0 without a branch (T8/T20 of the guide).
  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.in), (short)0,
                                                                       p.in_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rwt = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.wt), (short)0,
                                                                       p.wt_bytes, 0x00020000);

  // Per-thread staging geometry, fixed over K: byte offsets into the input /
  // weight buffers and the LDS slot of each 16-byte chunk this thread moves.
  unsigned a_off[NA];
  int a_scale_off[NA];
  unsigned a_taps[NA];                    // bit t: tap t of the KSxKS window is inside the image
  int a_lds[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int c = tid + 256 * i, row = c / CPR, col = c % CPR;
    const int m = m0 + row;
    a_lds[i] = row * LDSROW + lds_chunk<CPR>(row, col) * 16;
    a_taps[i] = 0;
    a_off[i] = 0;
    a_scale_off[i] = 0;
    if (c < A_TOT && m < M) {
      const int n = m / HW, r = m - n * HW, y = r / W, x = r - y * W;
      a_off[i] = (unsigned)(((n * H + y) * W + x) * p.in_cstride + col * EPC) * ES;
      a_scale_off[i] = n * cin_p + col * EPC;
#pragma unroll
      for (int t = 0; t < KS * KS; ++t) {
        const int yy = y + t / KS - KS / 2, xx = x + t % KS - KS / 2;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W) a_taps[i] |= 1u << t;
      }
    }
  }
  unsigned b_off[NB];
  int b_lds[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int c = tid + 256 * i, row = c / CPR, col = c % CPR;
    const int co = n0 + row;
    b_lds[i] = row * LDSROW + lds_chunk<CPR>(row, col) * 16;
    b_off[i] = (c < B_TOT && co < cout_p) ? (unsigned)((co * KS * KS * cin_p + col * EPC) * ES) : OOB;
  }

  const int kc_per_tap = cin_p / BK;
  // split-K (blockIdx.y = slice): this block runs K-tiles [kt0, kt0 + KT)
  const int KT_all = KS * KS * kc_per_tap, ks = blockIdx.y;
  const int kt0 = (int)((long)KT_all * ks / p.k_split);
  const int KT = (int)((long)KT_all * (ks + 1) / p.k_split) - kt0;
  // two register stage sets: with PF2 tile k+2 is in flight while tile k is computed
  uint4 ra0[NA], rb0[NB], ra1[NA], rb1[NB];

  auto load_tile = [&](int kk, uint4 (&ra)[NA], uint4 (&rb)[NB]) {
    const int kt = kt0 + kk;
    // taps inner, channel chunks outer (wave-uniform, SALU): the 9 shifted
    // reads of one chunk come in consecutive K-tiles and hit L2
    const int kc = kt / (KS * KS), tap = kt - kc * (KS * KS);
    const int ci0 = kc * BK;
    const int delta = (((tap / KS - KS / 2) * W + (tap % KS - KS / 2)) * p.in_cstride + ci0) * ES;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const unsigned voff = ((a_taps[i] >> tap) & 1u) ? a_off[i] + delta : OOB;
      uint4 v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rin, voff, 0, 0));
      if constexpr (sizeof(TA) == 4) {
        if (p.a_scale) {  // SE excitation folded into the project conv's A load
          const float4 s = *reinterpret_cast<const float4*>(p.a_scale + a_scale_off[i] + ci0);
          float4 f = __builtin_bit_cast(float4, v);
          f.x *= s.x; f.y *= s.y; f.z *= s.z; f.w *= s.w;
          v = __builtin_bit_cast(uint4, f);
        }
      }
      ra[i] = v;
    }
    const int soff = (tap * cin_p + ci0) * ES;              // scalar offset
#pragma unroll
    for (int i = 0; i < NB; ++i)
      rb[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rwt, b_off[i], soff, 0));
  };
  auto store_tile = [&](int buf, const uint4 (&ra)[NA], const uint4 (&rb)[NB]) {
#pragma unroll
    for (int i = 0; i < NA; ++i)
      if (A_TOT % 256 == 0 || tid + 256 * i < A_TOT) *reinterpret_cast<uint4*>(As + buf * BUF_A + a_lds[i]) = ra[i];
#pragma unroll
    for (int i = 0; i < NB; ++i)
      if (B_TOT % 256 == 0 || tid + 256 * i < B_TOT) *reinterpret_cast<uint4*>(Bs + buf * BUF_B + b_lds[i]) = rb[i];
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, r16 = lane & 15;
  const char* Abase = As + (wm * WM + r16) * LDSROW;
  const char* Bbase = Bs + (wn * WN + r16) * LDSROW;
  auto compute = [&](int cur) {
    const char* Ab = Abase + cur * BUF_A;
    const char* Bb = Bbase + cur * BUF_B;
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      const int ch = lds_chunk<CPR>(r16, ks * 4 + g) * 16;   // row & 7 == r16 & 7
      uint4 av[FM], bv[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) av[i] = *reinterpret_cast<const uint4*>(Ab + i * 16 * LDSROW + ch);
#pragma unroll
      for (int j = 0; j < FN; ++j) bv[j] = *reinterpret_cast<const uint4*>(Bb + j * 16 * LDSROW + ch);
      if constexpr (sizeof(TA) == 4) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) {
              const float a = __uint_as_float((&av[i].x)[s]);
              const float b = __uint_as_float((&bv[j].x)[s]);
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i][j], 0, 0, 0);
            }
      } else {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8, av[i]), __builtin_bit_cast(bf16x8, bv[j]), acc[i][j], 0, 0, 0);
      }
    }
  };

  // LDS buffer (k & 1) holds K-tile k.  One MFMA site in the loop keeps the
  // accumulators in a single AGPR home (a 2x-unrolled loop made the register
  // allocator rotate them through VGPRs every iteration).
  if constexpr (PF2) {   // latency-bound small GEMMs: two tiles in flight
    load_tile(0, ra0, rb0);
    store_tile(0, ra0, rb0);
    if (KT > 1) load_tile(1, ra1, rb1);
    __syncthreads();
    for (int kt = 0; kt < KT; ++kt) {
      const int cur = kt & 1;
      // ra0 holds tile kt+1 (odd kt) or is free (even kt) -- swap roles by parity
      if (cur == 0) {
        if (kt + 2 < KT) load_tile(kt + 2, ra0, rb0);
      } else {
        if (kt + 2 < KT) load_tile(kt + 2, ra1, rb1);
      }
      compute(cur);
      if (kt + 1 < KT) {
        if (cur == 0) store_tile(1, ra1, rb1);
        else store_tile(0, ra0, rb0);
      }
      __syncthreads();
    }
  } else {               // MFMA-bound convs: one register set keeps 2 waves/SIMD
    load_tile(0, ra0, rb0);
    store_tile(0, ra0, rb0);
    __syncthreads();
    for (int kt = 0; kt < KT; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < KT) load_tile(kt + 1, ra0, rb0);
      compute(cur);
      if (kt + 1 < KT) store_tile(cur ^ 1, ra0, rb0);
      __syncthreads();
    }
  }

  // ---------------- epilogue (LDS-staged, 16-byte row stores) ----------------
  float* tile = reinterpret_cast<float*>(lds);
  EpiArgs e{};
  e.bias = p.bias; e.out = p.out; e.res = p.res; e.stats = p.stats; e.amax = p.amax; e.scale = 1.f;
  e.M = M; e.H = H; e.W = W; e.cout_p = cout_p; e.out_cstride = p.out_cstride; e.rh = p.rh; e.rw = p.rw;
  e.act = p.act; e.tiles_per_img = p.tiles_per_img;
  e.post_scale = p.post_scale; e.post_shift = p.post_shift; e.act2 = p.act2; e.act3 = p.act3;
  for (int h = 0; h < HALVES; ++h) {
    if (h) __syncthreads();
    if constexpr (HALVES == 1) acc_to_lds<FM, FN, WM, WN, BN>(tile, acc, wm, wn, lane);
    else if (wn == h) acc_to_lds<FM, FN, WM, WN, EBN>(tile, acc, wm, 0, lane);
    const int nh = n0 + h * EBN;
    if (p.k_split > 1) {   // raw partial sums; splitk_reduce_kernel applies the epilogue
      constexpr int P = EBN + 4, C4 = EBN / 4;
      __syncthreads();
      float* dst = p.splitk_ws + (size_t)ks * M * cout_p;
      for (int idx = tid; idx < BM * C4; idx += 256) {
        const int row = idx / C4, c4 = idx - row * C4, m = m0 + row, co = nh + c4 * 4;
        if (m < M && co < cout_p)
          *reinterpret_cast<float4*>(dst + (size_t)m * cout_p + co) =
              *reinterpret_cast<const float4*>(tile + row * P + c4 * 4);
      }
      continue;
    }
    tile_store<TO, BM, EBN>(tile, e, m0, nh);
  }
}

// Split-K reduction + the conv epilogue (bias, act, second affine, residual
// with nearest upsample, act3, amax) -- partial slices summed in fixed order,
// so results do not depend on scheduling.  One thread per 4 output channels.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const ConvArgs p) {
  const int C4 = p.cout_p / 4;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx < (long)p.M * C4) {
    const int m = (int)(idx / C4), co = (int)(idx - (long)m * C4) * 4;
    const size_t slice = (size_t)p.M * p.cout_p, off = (size_t)m * p.cout_p + co;
    float4 x = *reinterpret_cast<const float4*>(p.splitk_ws + off);
    for (int k = 1; k < p.k_split; ++k) {
      const float4 q = *reinterpret_cast<const float4*>(p.splitk_ws + k * slice + off);
      x.x += q.x; x.y += q.y; x.z += q.z; x.w += q.w;
    }
    const float4 b = *reinterpret_cast<const float4*>(p.bias + co);
    x.x = kpd_act(x.x + b.x, p.act); x.y = kpd_act(x.y + b.y, p.act);
    x.z = kpd_act(x.z + b.z, p.act); x.w = kpd_act(x.w + b.w, p.act);
    if (p.post_scale) {
      const float4 s = *reinterpret_cast<const float4*>(p.post_scale + co);
      const float4 t = *reinterpret_cast<const float4*>(p.post_shift + co);
      x.x = kpd_act(x.x * s.x + t.x, p.act2); x.y = kpd_act(x.y * s.y + t.y, p.act2);
      x.z = kpd_act(x.z * s.z + t.z, p.act2); x.w = kpd_act(x.w * s.w + t.w, p.act2);
    }
    if (p.res) {
      const int HW = p.H * p.W, n = m / HW, r = m - n * HW, y = r / p.W, xx = r - y * p.W;
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
    *reinterpret_cast<float4*>(static_cast<float*>(p.out) + (size_t)m * p.out_cstride + co) = x;
    // per-image max|out| (split-K runs on maps of <= 256 pixels: few cells)
    if (p.amax)
      amax_publish_img(p.amax, m / (p.H * p.W), fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w))));
  }
}

constexpr long kMaxDesc = 0x7fffffffL;   // buffer descriptors take 31-bit extents

template <typename TA, typename TO, int KS, int BM, int BN, int BK, bool PF2 = false>
hipError_t launch(const ConvArgs& a0, hipStream_t st) {
  constexpr long ES = sizeof(TA), OS = sizeof(TO);
  ConvArgs a = a0;
  const long wt_bytes = (long)a.cout_p * KS * KS * a.cin_p * ES;
  const long img_bytes = (long)a.H * a.W * a.in_cstride * ES;
  if (wt_bytes > kMaxDesc || img_bytes > kMaxDesc) return hipErrorInvalidValue;
  a.wt_bytes = (int)wt_bytes;
  const long HW = (long)a.H * a.W;
  // split-K: a 1x1 fp32 GEMM on a coarse map (MobileNet projects at <= 16x12,
  // FPN lateral 3) has few output tiles and a long K -- one serial K loop per
  // block.  Slice K over blockIdx.y and reduce in fixed order.  The slice count
  // depends on the layer only (never on the batch), so an image's result does
  // not depend on what it is batched with.
  const int KT_all = KS * KS * (a.cin_p / BK);
  a.k_split = 1;
  if (KS == 1 && sizeof(TA) == 4 && sizeof(TO) == 4 && a.splitk_ws && !a.stats && HW <= 256 && KT_all >= 4 &&
      a.out_cstride == a.cout_p)
    a.k_split = std::min(KT_all / 2, 8);
  // images per launch: input descriptor below 2^31 bytes, partials within the scratch
  long chunk_l = std::min<long>(a.N, kMaxDesc / img_bytes);
  if (a.k_split > 1) chunk_l = std::min<long>(chunk_l, a.splitk_cap / (HW * a.cout_p * a.k_split));
  if (chunk_l < 1) a.k_split = 1, chunk_l = std::min<long>(a.N, kMaxDesc / img_bytes);
  const int chunk = (int)chunk_l;
  for (int n0 = 0; n0 < a0.N; n0 += chunk) {
    const int nb = std::min(chunk, a0.N - n0);
    a.N = nb;
    a.M = (int)(nb * HW);
    a.in = static_cast<const char*>(a0.in) + n0 * img_bytes;
    a.out = static_cast<char*>(a0.out) + n0 * HW * a.out_cstride * OS;
    a.res = a0.res ? a0.res + n0 * (long)a.rh * a.rw * a.cout_p : nullptr;
    a.a_scale = a0.a_scale ? a0.a_scale + (long)n0 * a.cin_p : nullptr;
    a.stats = a0.stats ? a0.stats + (long)n0 * a.tiles_per_img * 2 * a.cout_p : nullptr;
    a.in_bytes = (int)(nb * img_bytes);
    const int blocks = ((a.M + BM - 1) / BM) * ((a.cout_p + BN - 1) / BN);
    dim3 grid(blocks, a.k_split);
    hipLaunchKernelGGL((conv_mfma_kernel<TA, TO, KS, BM, BN, BK, PF2>), grid, dim3(256), 0, st, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (a.k_split > 1) {
      const long n4 = (long)a.M * (a.cout_p / 4);
      hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, a);
      e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
  }
  return hipSuccess;
}

}  // namespace

int conv_tile_m() { return 128; }

hipError_t launch_conv(const ConvArgs& a, ConvDType dt, int ks, hipStream_t st) {
  if (a.M <= 0) return hipSuccess;
  if (dt == CONV_F32) {
    const bool bk32 = (a.cin_p % 32) == 0;
    if (ks == 3) {
      if (!bk32) return hipErrorInvalidValue;
      if (a.cout_p <= 32) return launch<float, float, 3, 128, 32, 32>(a, st);
      if (a.cout_p <= 64) return launch<float, float, 3, 128, 64, 32>(a, st);
      return launch<float, float, 3, 128, 128, 32>(a, st);
    }
    if (ks != 1) return hipErrorInvalidValue;
    // small GEMMs (MobileNet body, coarse FPN laterals): halve the M tile so the
    // grid covers the 256 CUs at least twice
    const long blocks128 = (long)((a.M + 127) / 128) * ((a.cout_p + 127) / 128);
    if (blocks128 < 512 && a.stats == nullptr) {
      if (a.cout_p <= 32) return bk32 ? launch<float, float, 1, 64, 32, 32, true>(a, st)
                                      : launch<float, float, 1, 64, 32, 16, true>(a, st);
      if (a.cout_p <= 64) return bk32 ? launch<float, float, 1, 64, 64, 32, true>(a, st)
                                      : launch<float, float, 1, 64, 64, 16, true>(a, st);
      return bk32 ? launch<float, float, 1, 64, 128, 32, true>(a, st) : launch<float, float, 1, 64, 128, 16, true>(a, st);
    }
    if (a.cout_p <= 32) return bk32 ? launch<float, float, 1, 128, 32, 32>(a, st)
                                    : launch<float, float, 1, 128, 32, 16>(a, st);
    if (a.cout_p <= 64) return bk32 ? launch<float, float, 1, 128, 64, 32>(a, st)
                                    : launch<float, float, 1, 128, 64, 16>(a, st);
    return bk32 ? launch<float, float, 1, 128, 128, 32>(a, st)
                : launch<float, float, 1, 128, 128, 16>(a, st);
  }
  // bf16 operands (cin_p % 64 == 0 required), output bf16 or f32
  if (a.cin_p % 64 != 0) return hipErrorInvalidValue;
  if (ks == 3) {
    if (dt == CONV_BF16_OUT_BF16) {
      if (a.cout_p <= 64) return launch<__bf16, __bf16, 3, 128, 64, 64>(a, st);
      return launch<__bf16, __bf16, 3, 128, 128, 64>(a, st);
    }
    if (a.cout_p <= 64) return launch<__bf16, float, 3, 128, 64, 64>(a, st);
    return launch<__bf16, float, 3, 128, 128, 64>(a, st);
  }
  if (ks == 1) {
    if (dt == CONV_BF16_OUT_BF16) return launch<__bf16, __bf16, 1, 128, 64, 64>(a, st);
    return launch<__bf16, float, 1, 128, 64, 64>(a, st);
  }
  return hipErrorInvalidValue;
}
