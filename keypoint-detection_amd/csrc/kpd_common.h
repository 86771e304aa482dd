// Shared device/host helpers for the keypoint-detection HIP path (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <stdlib.h>

// Diagnostic switches -- A/B variants of measured changes, ablations that are
// wrong by design (KPD_*_DBG), phase stamps (KPD_STAMPS) -- are read from the
// environment only in a diagnostic build (make DIAG=1, -DKPD_DIAG=1).  The
// default libkpd.so never reads them: kpd_diag_env() is a constant null, the
// switches fold away and a stray variable on a serving box changes nothing.
#ifndef KPD_DIAG
#define KPD_DIAG 0
#endif
static inline const char* kpd_diag_env(const char* name) {
#if KPD_DIAG
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

// x / 6 without the IEEE division sequence (v_div_scale / fmas / fixup, ~10
// instructions): quotient by the rounded reciprocal, then one exact-residual
// correction, which returns the correctly rounded quotient.
__device__ __forceinline__ float kpd_div6(float x) {
  constexpr float r6 = 1.f / 6.f;
  const float q = x * r6;
  return fmaf(fmaf(-q, 6.f, x), r6, q);
}

enum KpdAct : int { ACT_NONE = 0, ACT_RELU = 1, ACT_RELU6 = 2, ACT_HSWISH = 3, ACT_SIGMOID = 4 };

// Activation formulas follow ATen's CPU kernels operation-for-operation
// (hardswish: x * min(max(x + 3, 0), 6) / 6) so rounding matches closely.
__device__ __forceinline__ float kpd_act(float v, int act) {
  switch (act) {
    case ACT_RELU: return v > 0.f ? v : 0.f;
    case ACT_RELU6: return fminf(fmaxf(v, 0.f), 6.f);
    case ACT_HSWISH: return kpd_div6(v * fminf(fmaxf(v + 3.f, 0.f), 6.f));
    case ACT_SIGMOID: return 1.f / (1.f + expf(-v));
    default: return v;
  }
}

__device__ __forceinline__ float kpd_sigmoid(float v) { return 1.f / (1.f + expf(-v)); }
__device__ __forceinline__ float kpd_hsigmoid(float v) { return kpd_div6(fminf(fmaxf(v + 3.f, 0.f), 6.f)); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// Sum over each 16-lane row of the wave, every lane of a row receiving it: the
// xor-1 / xor-2 / xor-4 / xor-8 butterfly on DPP lane moves (quad_perm, then
// row_half_mirror and row_mirror, which pair a lane with one of the other
// quad / half-row, whose lanes all hold the same partial by then), so the
// additions -- and the result, bit for bit -- are the __shfl_xor butterfly's,
// without its four LDS-crossbar (ds_bpermute) round trips.
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false));  // row_half_mirror
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, false));  // row_mirror
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Per-image max|x| of a tensor (the split FPN scale inputs): image n's
// maximum lives in its own 128-byte line, slots[n * kAmaxStride], so every
// scale derived from it depends on that image alone -- an image's result does
// not change with what it is batched or sharded with.  Writers publish with
// atomicMax on the float bits (values >= 0 order like unsigned ints); the
// caller zeroes the slots.
constexpr int kAmaxStride = 32;
// Output slot of an ROI: >= 0 = compacted position of a valid box; an
// all-zero box gets -1 - (pos | dummy << 16), pos = its padding position
// (after the image's valid boxes), dummy = the image has no valid box (the
// reference's dummy person, keypoint_model.py:171-199).
__host__ __device__ __forceinline__ int slot_empty(int pos, bool dummy) { return -1 - (pos | (dummy ? 0x10000 : 0)); }
__device__ __forceinline__ int slot_pos(int s) { return (-1 - s) & 0xFFFF; }
__device__ __forceinline__ bool slot_dummy(int s) { return ((-1 - s) >> 16) & 1; }

__device__ __forceinline__ void amax_publish_img(float* slots, int n, float v) {
  if (v > 0.f) atomicMax(reinterpret_cast<unsigned int*>(slots + (size_t)n * kAmaxStride), __float_as_uint(v));
}

// Split (fp32-accurate f16 hi + lo) FPN level 0 computed by linearity
// (conv_glds.hip, fpn0x_kernel): the stem tap and lateral 1 of image n are
// split with their own power-of-two scales 2^a_f, 2^a_l, chosen so that
// a_f + w_exp0 == a_l + w_expE == P (one unscale 2^-P for the summed
// products) and neither operand overflows f16: max|x * 2^a| < 2^14.
// f, l = max|tap0|, max|lateral 1| of the image (per-image slots).
__device__ __forceinline__ int split_exp_of(float amax) {
  const float u = amax * 1.0078125f;
  if (!(u > 0.f)) return 100;   // all-zero tensor: no constraint
  if (!(u < INFINITY)) return -100;
  int e;
  frexpf(u, &e);
  return min(max(14 - e, -100), 100);
}
__device__ __forceinline__ void fpn0x_exps(float f, float l, int w_exp0, int w_expE, int* a_f, int* a_l, int* P) {
  int pp = min(split_exp_of(f) + w_exp0, split_exp_of(l) + w_expE);
  pp = min(max(pp, -120), 120);
  *P = pp;
  *a_f = pp - w_exp0;
  *a_l = pp - w_expE;
}

#define KPD_CHECK_LAUNCH() (hipGetLastError())
