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
//   * Zero padding of the 3x3 halo is done by predicating the A-tile loads.
//   * Epilogue fuses bias (BN folded on the host), activation, residual add
//     with optional nearest-upsample indexing (FPN top-down), per-image
//     channel sum/max partials (ChannelAttention pooling), bf16/fp32 stores.
#include "kpd_common.h"
#include "kpd_kernels.h"
#include "conv_epilogue.h"

namespace {

template <typename TA, typename TO, int KS, int BM, int BN, int BK>
__global__ __launch_bounds__(256) void conv_mfma_kernel(const ConvArgs p) {
  constexpr int ES = sizeof(TA);
  constexpr int ROWB = BK * ES;           // bytes of one LDS row (one K-tile of one row)
  constexpr int CPR = ROWB / 16;          // 16-byte chunks per row
  constexpr int LDSROW = ROWB + 16;       // padded row pitch (bank spread)
  constexpr int EPC = 16 / ES;            // elements per chunk
  constexpr int A_TOT = BM * CPR, B_TOT = BN * CPR;
  constexpr int NA = (A_TOT + 255) / 256, NB = (B_TOT + 255) / 256;
  constexpr int WM = BM / 2, WN = BN / 2, FM = WM / 16, FN = WN / 16;
  constexpr int KSTEPS = ROWB / 64;       // 4 lane groups x 16 B per k-step
  static_assert(FM >= 1 && FN >= 1, "tile too small");
  static_assert(ROWB % 64 == 0, "BK must cover 64 bytes");

  constexpr int MAIN_LDS = 2 * (BM + BN) * LDSROW;
  constexpr int EPI_LDS = epi_lds_bytes<BM, BN>();
  __shared__ __attribute__((aligned(16))) char lds[MAIN_LDS > EPI_LDS ? MAIN_LDS : EPI_LDS];
  char* As = lds;
  char* Bs = lds + 2 * BM * LDSROW;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int H = p.H, W = p.W, HW = H * W, M = p.M;
  const int cin_p = p.cin_p, cout_p = p.cout_p;
  const TA* __restrict__ in = reinterpret_cast<const TA*>(p.in);
  const TA* __restrict__ wt = reinterpret_cast<const TA*>(p.wt);

  // Pixel coordinates of the A rows this thread stages (fixed over K).
  int a_n[NA], a_y[NA], a_x[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int c = tid + 256 * i;
    const int m = m0 + c / CPR;
    if (c < A_TOT && m < M) {
      const int n = m / HW, r = m - n * HW, y = r / W;
      a_n[i] = n; a_y[i] = y; a_x[i] = r - y * W;
    } else {
      a_n[i] = -1; a_y[i] = 0; a_x[i] = 0;
    }
  }

  const int kc_per_tap = cin_p / BK;
  const int KT = KS * KS * kc_per_tap;
  uint4 ra[NA], rb[NB];

  auto load_tile = [&](int kt) {
    const int tap = kt / kc_per_tap;
    const int ci0 = (kt - tap * kc_per_tap) * BK;
    const int dy = tap / KS - KS / 2, dx = tap % KS - KS / 2;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int c = tid + 256 * i, col = c % CPR;
      const int yy = a_y[i] + dy, xx = a_x[i] + dx;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (a_n[i] >= 0 && yy >= 0 && yy < H && xx >= 0 && xx < W) {
        const int ci = ci0 + col * EPC;
        const TA* src = in + ((size_t)(a_n[i] * H + yy) * W + xx) * p.in_cstride + ci;
        v = *reinterpret_cast<const uint4*>(src);
        if constexpr (sizeof(TA) == 4) {
          if (p.a_scale) {  // SE excitation folded into the project conv's A load
            const float4 s = *reinterpret_cast<const float4*>(p.a_scale + (size_t)a_n[i] * cin_p + ci);
            float4 f = *reinterpret_cast<float4*>(&v);
            f.x *= s.x; f.y *= s.y; f.z *= s.z; f.w *= s.w;
            v = *reinterpret_cast<uint4*>(&f);
          }
        }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int c = tid + 256 * i, row = c / CPR, col = c % CPR;
      const int co = n0 + row;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (c < B_TOT && co < cout_p)
        v = *reinterpret_cast<const uint4*>(wt + ((size_t)co * KS * KS + tap) * cin_p + ci0 + col * EPC);
      rb[i] = v;
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int c = tid + 256 * i;
      if (c < A_TOT)
        *reinterpret_cast<uint4*>(As + (buf * BM + c / CPR) * LDSROW + (c % CPR) * 16) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int c = tid + 256 * i;
      if (c < B_TOT)
        *reinterpret_cast<uint4*>(Bs + (buf * BN + c / CPR) * LDSROW + (c % CPR) * 16) = rb[i];
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, r16 = lane & 15;
  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) load_tile(kt + 1);
    const char* Ab = As + (cur * BM + wm * WM + r16) * LDSROW;
    const char* Bb = Bs + (cur * BN + wn * WN + r16) * LDSROW;
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      uint4 av[FM], bv[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        av[i] = *reinterpret_cast<const uint4*>(Ab + i * 16 * LDSROW + (ks * 4 + g) * 16);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bv[j] = *reinterpret_cast<const uint4*>(Bb + j * 16 * LDSROW + (ks * 4 + g) * 16);
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
                *reinterpret_cast<const bf16x8*>(&av[i]), *reinterpret_cast<const bf16x8*>(&bv[j]),
                acc[i][j], 0, 0, 0);
      }
    }
    if (kt + 1 < KT) store_tile(cur ^ 1);
    __syncthreads();
  }

  // ---------------- epilogue (LDS-staged, 16-byte row stores) ----------------
  float* tile = reinterpret_cast<float*>(lds);
  acc_to_lds<FM, FN, WM, WN, BN>(tile, acc, wm, wn, lane);
  EpiArgs e;
  e.bias = p.bias; e.out = p.out; e.res = p.res; e.stats = p.stats; e.amax = p.amax; e.scale = 1.f;
  e.M = M; e.H = H; e.W = W; e.cout_p = cout_p; e.out_cstride = p.out_cstride; e.rh = p.rh; e.rw = p.rw;
  e.act = p.act; e.tiles_per_img = p.tiles_per_img;
  e.post_scale = p.post_scale; e.post_shift = p.post_shift; e.act2 = p.act2; e.act3 = p.act3;
  tile_store<TO, BM, BN>(tile, e, m0, n0);
}

template <typename TA, typename TO, int KS, int BM, int BN, int BK>
hipError_t launch(const ConvArgs& a, hipStream_t st) {
  dim3 grid((a.M + BM - 1) / BM, (a.cout_p + BN - 1) / BN);
  hipLaunchKernelGGL((conv_mfma_kernel<TA, TO, KS, BM, BN, BK>), grid, dim3(256), 0, st, a);
  return hipGetLastError();
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
      if (a.cout_p <= 32) return bk32 ? launch<float, float, 1, 64, 32, 32>(a, st)
                                      : launch<float, float, 1, 64, 32, 16>(a, st);
      if (a.cout_p <= 64) return bk32 ? launch<float, float, 1, 64, 64, 32>(a, st)
                                      : launch<float, float, 1, 64, 64, 16>(a, st);
      return bk32 ? launch<float, float, 1, 64, 128, 32>(a, st) : launch<float, float, 1, 64, 128, 16>(a, st);
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
