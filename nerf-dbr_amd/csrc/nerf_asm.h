// Inline-asm building blocks shared by the MFMA kernels' weight streams.
//
// Why asm: when hipcc sees an LDS-DMA builtin (global_load_lds) in a function it
// stops counting LDS waits and emits lgkmcnt(0) before every fragment use.  The
// kernels issue the DMA from asm, which the compiler's waitcnt pass does not see (an
// asm vector-memory op only makes the compiler's own vmcnt waits stricter), and
// read LDS either with plain loads (default, below) or from asm with compile-time
// counted waits (NERF_ASM_LDS_READS, lab form).
#pragma once
#include <hip/hip_runtime.h>

namespace nerf {

typedef float asm_f32x4 __attribute__((ext_vector_type(4)));
typedef int asm_i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned asm_u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void compiler_fence() { asm volatile("" ::: "memory"); }

// LDS byte address of a __shared__ object (for asm operands)
template <typename T>
__device__ __forceinline__ unsigned lds_addr(T* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)(const char*)p;
}

// LDS fragment reads.  NERF_ASM_LDS_READS=1 issues them from asm with the counted waits
// below; that form is unsound in general: an asm output counts as written at the
// statement, so the register allocator may copy the destination (e.g. into an AGPR it
// prefers for the MFMA operand) before the wait that retires the read, and the copy then
// holds the register's old contents.  tools/lint_waits.py found exactly that in a
// split-fp16 build (a v_accvgpr_write of a fragment 2 instructions after its ds_read, the
// MFMA 200 instructions later reading the stale copy).  The default (0) is a plain LDS
// load the compiler sees: its waitcnt pass then counts the reads itself and a copy is
// placed after the data, correct by construction; wait_lgkm keeps only the scheduling
// barrier.  `make all` lints both forms (tools/lint_waits.py).
#ifndef NERF_ASM_LDS_READS
#define NERF_ASM_LDS_READS 0
#endif
template <typename V>
__device__ __forceinline__ const __attribute__((address_space(3))) V* lds_ptr(unsigned addr, int off) {
  return (const __attribute__((address_space(3))) V*)(uintptr_t)(addr + unsigned(off));
}

// 16-B LDS read; off must fold to a constant in [0, 65536) after unrolling
template <typename V>
__device__ __forceinline__ V ds_read_b128(unsigned addr, int off) {
  static_assert(sizeof(V) == 16, "16-byte fragment");
#if NERF_ASM_LDS_READS
  V v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(off));
  return v;
#else
  return *lds_ptr<V>(addr, off);
#endif
}
__device__ __forceinline__ asm_u32x2 ds_read_b64(unsigned addr, int off) {
#if NERF_ASM_LDS_READS
  asm_u32x2 v;
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(off));
  return v;
#else
  return *lds_ptr<asm_u32x2>(addr, off);
#endif
}

// s_waitcnt lgkmcnt(k), k a constant after unrolling, then a scheduling barrier
// so nothing that consumes the reads moves above it.  The field is 4 bits on
// gfx9: k > 15 waits at 15, i.e. for more reads than needed (safe).
__device__ __forceinline__ void wait_lgkm(int k) {
  if (!NERF_ASM_LDS_READS) {   // the compiler counts its own LDS reads
    __builtin_amdgcn_sched_barrier(0);
    return;
  }
#define NERF_LG(N) else if (k == N) asm volatile("s_waitcnt lgkmcnt(" #N ")" ::: "memory");
  if (k <= 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  NERF_LG(1) NERF_LG(2) NERF_LG(3) NERF_LG(4) NERF_LG(5) NERF_LG(6) NERF_LG(7) NERF_LG(8) NERF_LG(9)
  NERF_LG(10) NERF_LG(11) NERF_LG(12) NERF_LG(13) NERF_LG(14)
  else asm volatile("s_waitcnt lgkmcnt(15)" ::: "memory");
#undef NERF_LG
  __builtin_amdgcn_sched_barrier(0);
}

// s_waitcnt vmcnt(k) for a k that is a constant only after unrolling.
__device__ __forceinline__ void wait_vmcnt(int k) {
#define NERF_VM(N) else if (k == N) asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory");
  if (k <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  NERF_VM(1) NERF_VM(2) NERF_VM(3) NERF_VM(4) NERF_VM(5) NERF_VM(6) NERF_VM(7) NERF_VM(8)
  NERF_VM(10) NERF_VM(12) NERF_VM(14) NERF_VM(15) NERF_VM(16) NERF_VM(18) NERF_VM(20) NERF_VM(21)
  NERF_VM(24) NERF_VM(28) NERF_VM(30) NERF_VM(32)
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#undef NERF_VM
}

// s_waitcnt vmcnt(k) for every k in [0, 63] (the gfx9 field), k a constant after unrolling;
// wait_vmcnt above keeps its coarser table (values it lacks wait for everything).
__device__ __forceinline__ void wait_vmcnt_exact(int k) {
#define NERF_VX(N) else if (k == N) asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory");
  if (k <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  NERF_VX(1) NERF_VX(2) NERF_VX(3) NERF_VX(4) NERF_VX(5) NERF_VX(6) NERF_VX(7) NERF_VX(8)
  NERF_VX(9) NERF_VX(10) NERF_VX(11) NERF_VX(12) NERF_VX(13) NERF_VX(14) NERF_VX(15) NERF_VX(16)
  NERF_VX(17) NERF_VX(18) NERF_VX(19) NERF_VX(20) NERF_VX(21) NERF_VX(22) NERF_VX(23) NERF_VX(24)
  NERF_VX(25) NERF_VX(26) NERF_VX(27) NERF_VX(28) NERF_VX(29) NERF_VX(30) NERF_VX(31) NERF_VX(32)
  NERF_VX(33) NERF_VX(34) NERF_VX(35) NERF_VX(36) NERF_VX(37) NERF_VX(38) NERF_VX(39) NERF_VX(40)
  NERF_VX(41) NERF_VX(42) NERF_VX(43) NERF_VX(44) NERF_VX(45) NERF_VX(46) NERF_VX(47) NERF_VX(48)
  NERF_VX(49) NERF_VX(50) NERF_VX(51) NERF_VX(52) NERF_VX(53) NERF_VX(54) NERF_VX(55) NERF_VX(56)
  NERF_VX(57) NERF_VX(58) NERF_VX(59) NERF_VX(60) NERF_VX(61) NERF_VX(62)
  else asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
#undef NERF_VX
}

// One lane-linear 1 KiB LDS-DMA piece per wave, in saddr form: 16 B per lane
// from SGPR base (wave-uniform 64-bit) + a per-lane 32-bit VGPR offset to LDS
// byte address lds_base + lane*16 (wave-uniform base in M0), so advancing
// through a stream costs scalar adds instead of a 64-bit VALU add per piece.
// Completion is tracked with vmcnt.
// M0 is written without save/restore: hipcc treats M0 as reserved and ignores
// the clobber (-Winline-asm), so the library build checks that nothing else in
// the MFMA kernels reads or writes M0 (Makefile target check-m0, run by every
// build; it fails the build otherwise).
__device__ __forceinline__ void lds_dma_16_s(const void* sbase, unsigned voff, unsigned lds_base) {
  const unsigned base = __builtin_amdgcn_readfirstlane(lds_base);
  const unsigned long long sb = (unsigned long long)sbase;
  const unsigned lo = __builtin_amdgcn_readfirstlane(unsigned(sb)), hi = __builtin_amdgcn_readfirstlane(unsigned(sb >> 32));
  const unsigned long long s64 = (unsigned long long)lo | ((unsigned long long)hi << 32);
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
  asm volatile(
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %0, %1"
      :
      : "v"(voff), "s"(s64), "s"(base)
      : "memory", "m0");
#pragma clang diagnostic pop
}

}  // namespace nerf
