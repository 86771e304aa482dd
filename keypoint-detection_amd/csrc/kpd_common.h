// Shared device/host helpers for the keypoint-detection HIP path (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

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
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Device max|x| published by many workgroups: one float per 128-byte slot,
// kAmaxSlots slots (workgroup b uses slot b % kAmaxSlots), so the atomics of a
// whole grid spread over L2 channels instead of queueing on one address.
// Readers take the max over the slots.  The caller zeroes the slots.
constexpr int kAmaxSlots = 64, kAmaxStride = 32;
// Output slot of an ROI: >= 0 = compacted position of a valid box; an
// all-zero box gets -1 - (pos | dummy << 16), pos = its padding position
// (after the image's valid boxes), dummy = the image has no valid box (the
// reference's dummy person, keypoint_model.py:171-199).
__host__ __device__ __forceinline__ int slot_empty(int pos, bool dummy) { return -1 - (pos | (dummy ? 0x10000 : 0)); }
__device__ __forceinline__ int slot_pos(int s) { return (-1 - s) & 0xFFFF; }
__device__ __forceinline__ bool slot_dummy(int s) { return ((-1 - s) >> 16) & 1; }

__device__ __forceinline__ void amax_publish(float* slots, float v) {
  if (v > 0.f)
    atomicMax(reinterpret_cast<unsigned int*>(slots + (blockIdx.x % kAmaxSlots) * kAmaxStride), __float_as_uint(v));
}
// whole-wave call (all 64 lanes): returns the max over the slots in every lane
__device__ __forceinline__ float amax_read(const float* slots) {
  return wave_max(slots[(threadIdx.x & 63) * kAmaxStride]);
}

// Split (fp32-accurate f16 hi+lo) FPN level 0: power-of-two activation
// exponent from the device-side bound U >= max|lateral0| (producer and
// consumer evaluate the same expression on the same inputs, so they agree):
// U = (maxb + max|tap0| * maxs + max|lateral1|) * (1 + 2^-7), a_exp = 14 - e
// with U < 2^e, hence max|x * 2^a_exp| < 2^14 and the f16 hi part is finite.
// sc_in = two slotted maxima (amax_publish): [max|tap0|], [max|lateral1|].
// Whole-wave call.
__device__ __forceinline__ int split_a_exp(const float* sc_in, float maxb, float maxs) {
  const float a0 = amax_read(sc_in), l1 = amax_read(sc_in + kAmaxSlots * kAmaxStride);
  const float u = (maxb + a0 * maxs + l1) * 1.0078125f;
  if (!(u > 0.f) || !(u < INFINITY)) return 0;
  int e;
  frexpf(u, &e);
  return min(max(14 - e, -100), 100);
}

// Split FPN level 0 computed by linearity (conv_glds.hip, fpn0x_kernel): the
// stem tap and lateral 1 are split with their own power-of-two scales 2^a_f,
// 2^a_l, chosen so that a_f + w_exp0 == a_l + w_expE == P (one unscale 2^-P
// for the summed products) and neither operand overflows f16.  Whole-wave call.
__device__ __forceinline__ int split_exp_of(float amax) {
  const float u = amax * 1.0078125f;
  if (!(u > 0.f)) return 100;   // all-zero tensor: no constraint
  if (!(u < INFINITY)) return -100;
  int e;
  frexpf(u, &e);
  return min(max(14 - e, -100), 100);
}
// raw slot values of this lane (issue early, reduce late: fpn0x_exps_from)
__device__ __forceinline__ float2 fpn0x_slots(const float* sc_in) {
  const int i = (threadIdx.x & 63) * kAmaxStride;
  return make_float2(sc_in[i], sc_in[kAmaxSlots * kAmaxStride + i]);
}
__device__ __forceinline__ void fpn0x_exps_from(float2 sl, int w_exp0, int w_expE, int* a_f, int* a_l, int* P) {
  const int ef = split_exp_of(wave_max(sl.x)), el = split_exp_of(wave_max(sl.y));
  int pp = min(ef + w_exp0, el + w_expE);
  pp = min(max(pp, -120), 120);
  *P = pp;
  *a_f = pp - w_exp0;
  *a_l = pp - w_expE;
}
__device__ __forceinline__ void fpn0x_exps(const float* sc_in, int w_exp0, int w_expE, int* a_f, int* a_l, int* P) {
  const int ef = split_exp_of(amax_read(sc_in)), el = split_exp_of(amax_read(sc_in + kAmaxSlots * kAmaxStride));
  int pp = min(ef + w_exp0, el + w_expE);
  pp = min(max(pp, -120), 120);
  *P = pp;
  *a_f = pp - w_exp0;
  *a_l = pp - w_expE;
}

#define KPD_CHECK_LAUNCH() (hipGetLastError())
