// nh_ldsdma.hpp -- LDS-DMA loads (gfx950 global_load_lds_*) for the config-5
// and closed-loop kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nh {

// LDS-DMA (global_load_lds_*): each active lane's bytes from gsrc land at the
// LDS byte address lds + lane * 16 for dwordx4, lds + lane * 4 for ushort (one
// zero-extended dword per lane; tools/ab/lds_dma_probe.hip); the LDS base travels in M0, which the
// compiler reserves, so it is saved and restored in the same statement.  As
// inline asm the load is invisible to the compiler's waitcnt bookkeeping: the
// caller retires it with an explicit vmcnt (wait_vm) -- the compiler's own
// counts are only made more conservative by it (in-order completion).
typedef __attribute__((address_space(3))) void lds_void_t;
__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)(lds_void_t*)(p); }
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory");
}
__device__ __forceinline__ void glds4(const void* gsrc, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory");
}
__device__ __forceinline__ void glds2(const void* gsrc, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_ushort %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory");
}
// The same with a uniform base in SGPRs and a 32-bit per-lane byte offset
// (global_load_lds_* v_off, s[base]): no 64-bit address arithmetic per lane.
__device__ __forceinline__ uint64_t sgpr_ptr(const void* p) {   // the (wave-uniform) pointer, in SGPRs
    const uint64_t v = (uint64_t)(uintptr_t)p;
    // (readfirstlane returns int: widen through uint32_t, or the low word's bit 31 would sign-extend)
    return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32);
}
__device__ __forceinline__ void glds16s(const void* sbase, uint32_t voff, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(sgpr_ptr(sbase)), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory");
}
__device__ __forceinline__ void glds2s(const void* sbase, uint32_t voff, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_ushort %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(sgpr_ptr(sbase)), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory"); }


}  // namespace nh
