// LDS-DMA helpers shared by the gfx950 kernels (buffer_load ... lds).
#pragma once
#include <hip/hip_runtime.h>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// raw buffer descriptor: base, stride 0, num_records = bytes (range-checked)
__device__ __forceinline__ i32x4 make_rsrc(const void* base, int bytes) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(base);
  return i32x4{(int)(unsigned)a, (int)((a >> 32) & 0xffffu), bytes, 0x00020000};
}

// One LDS-DMA wave-instruction: 16 bytes per lane from rsrc[voff + soff] to
// LDS byte address lds_dst + 16 * lane (lds_dst wave-uniform; an out-of-range
// offset loads zeros).  Inline asm on purpose: hipcc does not see these loads,
// so it neither drains them with vmcnt(0) before the next ds_read nor at a
// barrier -- the kernel counts them itself (wait_vmcnt).  M0 is written and
// restored inside the statement (guide §5.7).
__device__ __forceinline__ void glds16(i32x4 rsrc, unsigned lds_dst, unsigned voff, int soff) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(lds_dst), "v"(voff), "s"(rsrc), "s"(soff)
      : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wave-uniform LDS byte address of a __shared__ pointer
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  typedef __attribute__((address_space(3))) void lds_void_t;
  return __builtin_amdgcn_readfirstlane((unsigned)reinterpret_cast<unsigned long long>((lds_void_t*)p));
}
