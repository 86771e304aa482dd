// FPN level-0 3x3 conv (128 -> 128, folded BN, ReLU) as an fp32-accurate
// implicit GEMM on the f16 MFMA pipe ("split16").
//
// Reference: LightweightFPN fpn_convs[0] (dll/models/backbone.py:20-27,39);
// its output feeds ChannelAttention + topk (keypoint_model.py:653-661), whose
// channel ORDER changes the rest of the network, so plain bf16/f16 is not
// allowed here (a bf16 conv changed the top-64 order on 16 of 24 images in
// the CPU emulation).
//
// Split: every fp32 operand x is carried as two f16 values, x*s = hi + lo,
// hi = f16(x*s), lo = f16(x*s - hi), with a power-of-two scale s chosen so
// max|x*s| < 2^15 (weights: on the host; activations: from the device-side
// max|lateral0| published by the lateral conv's epilogue).  Each 16x16x32
// k-step issues three v_mfma_f32_16x16x32_f16 (hi*lo, lo*hi, hi*hi) into one
// fp32 accumulator; f16 x f16 products are exact in fp32, the dropped lo*lo
// term is ~2^-22 relative, so the result matches an fp32 conv to fp32
// rounding -- at 3/16 of the fp32-MFMA cost.
#include "kpd_common.h"
#include "kpd_kernels.h"
#include "conv_epilogue.h"

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 128, BN = 128, BK = 32;   // BK in elements (one 16x16x32 k-step)
constexpr int ROWB = BK * 2;                  // 64 B per f16 row
constexpr int LDSROW = ROWB + 16;             // padded pitch
constexpr int PLANE_A = BM * LDSROW, PLANE_B = BN * LDSROW;
constexpr int BUF = 2 * PLANE_A + 2 * PLANE_B;   // hi/lo for A and B

__global__ __launch_bounds__(256) void conv3x3_split16_kernel(const Split16Args p) {
  static_assert(2 * BUF >= BM * (BN + 4) * 4, "epilogue tile must fit");
  __shared__ __attribute__((aligned(16))) char lds[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int H = p.H, W = p.W, HW = H * W, M = p.M, cin = p.cin, cout_p = p.cout_p;

  // activation scale from the published max|x| (power of two, exact)
  float sa = 1.f;
  int a_exp = 0;
  {
    const float amax = *p.amax;
    if (amax > 0.f && amax < INFINITY) {
      int e;
      frexpf(amax, &e);           // amax < 2^e
      a_exp = min(max(14 - e, -100), 100);
      sa = ldexpf(1.f, a_exp);
    }
  }
  const float out_scale = ldexpf(1.f, -(a_exp + p.w_exp));

  // A staging: 128 rows x 8 float4 chunks = 1024 chunks, 4 per thread
  int a_n[4], a_y[4], a_x[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i, m = m0 + c / 8;
    if (m < M) {
      const int n = m / HW, r = m - n * HW, y = r / W;
      a_n[i] = n; a_y[i] = y; a_x[i] = r - y * W;
    } else {
      a_n[i] = -1; a_y[i] = 0; a_x[i] = 0;
    }
  }
  const int kc_per_tap = cin / BK, KT = 9 * kc_per_tap;
  float4 ra[4];
  uint4 rb[4];

  auto load_tile = [&](int kt) {
    const int tap = kt / kc_per_tap, ci0 = (kt - tap * kc_per_tap) * BK;
    const int dy = tap / 3 - 1, dx = tap % 3 - 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + 256 * i, col = c % 8;
      const int yy = a_y[i] + dy, xx = a_x[i] + dx;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (a_n[i] >= 0 && yy >= 0 && yy < H && xx >= 0 && xx < W)
        v = *reinterpret_cast<const float4*>(p.in + ((size_t)(a_n[i] * H + yy) * W + xx) * cin + ci0 + col * 4);
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + 256 * i;           // 2 planes x 128 rows x 4 chunks
      const int plane = c >> 9, row = (c >> 2) & 127, col = c & 3;
      const int co = n0 + row;
      const _Float16* src = plane ? p.w_lo : p.w_hi;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (co < cout_p) v = *reinterpret_cast<const uint4*>(src + ((size_t)co * 9 + tap) * cin + ci0 + col * 8);
      rb[i] = v;
    }
  };
  auto store_tile = [&](int buf) {
    char* base = lds + buf * BUF;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + 256 * i, row = c / 8, col = c % 8;
      const float4 v = ra[i];
      const float x0 = v.x * sa, x1 = v.y * sa, x2 = v.z * sa, x3 = v.w * sa;
      f16x4 hi, lo;
      hi[0] = (_Float16)x0; hi[1] = (_Float16)x1; hi[2] = (_Float16)x2; hi[3] = (_Float16)x3;
      lo[0] = (_Float16)(x0 - (float)hi[0]); lo[1] = (_Float16)(x1 - (float)hi[1]);
      lo[2] = (_Float16)(x2 - (float)hi[2]); lo[3] = (_Float16)(x3 - (float)hi[3]);
      *reinterpret_cast<f16x4*>(base + row * LDSROW + col * 8) = hi;
      *reinterpret_cast<f16x4*>(base + PLANE_A + row * LDSROW + col * 8) = lo;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + 256 * i, plane = c >> 9, row = (c >> 2) & 127, col = c & 3;
      *reinterpret_cast<uint4*>(base + 2 * PLANE_A + plane * PLANE_B + row * LDSROW + col * 16) = rb[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, r16 = lane & 15;
  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) load_tile(kt + 1);
    const char* base = lds + cur * BUF;
    const char* Ah = base + (wm * 64 + r16) * LDSROW + g * 16;
    const char* Bh = base + 2 * PLANE_A + (wn * 64 + r16) * LDSROW + g * 16;
    f16x8 ah[4], al[4], bh[4], bl[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ah[i] = *reinterpret_cast<const f16x8*>(Ah + i * 16 * LDSROW);
      al[i] = *reinterpret_cast<const f16x8*>(Ah + PLANE_A + i * 16 * LDSROW);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bh[j] = *reinterpret_cast<const f16x8*>(Bh + j * 16 * LDSROW);
      bl[j] = *reinterpret_cast<const f16x8*>(Bh + PLANE_B + j * 16 * LDSROW);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
      }
    if (kt + 1 < KT) store_tile(cur ^ 1);
    __syncthreads();
  }

  // epilogue: unscale (exact power of two), bias (BN folded), ReLU, channel
  // sum/max partials -- LDS-staged full-row stores (conv_epilogue.h)
  float* tile = reinterpret_cast<float*>(lds);
  acc_to_lds<4, 4, 64, 64, BN>(tile, acc, wm, wn, lane);
  EpiArgs ep;
  ep.bias = p.bias; ep.out = p.out; ep.res = nullptr; ep.stats = p.stats; ep.amax = nullptr;
  ep.scale = out_scale; ep.M = M; ep.H = H; ep.W = W; ep.cout_p = cout_p; ep.out_cstride = cout_p;
  ep.rh = H; ep.rw = W; ep.act = p.act; ep.tiles_per_img = p.tiles_per_img;
  ep.post_scale = nullptr; ep.post_shift = nullptr; ep.act2 = 0; ep.act3 = 0;
  tile_store<float, BM, BN>(tile, ep, m0, n0);
}

}  // namespace

hipError_t launch_conv3x3_split16(const Split16Args& a, hipStream_t st) {
  if (a.M <= 0) return hipSuccess;
  if (a.cin % BK != 0) return hipErrorInvalidValue;
  dim3 grid((a.M + BM - 1) / BM, (a.cout_p + BN - 1) / BN);
  hipLaunchKernelGGL(conv3x3_split16_kernel, grid, dim3(256), 0, st, a);
  return hipGetLastError();
}
