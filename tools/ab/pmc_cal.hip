// Which SQ instruction counter counts which instruction (round 4, for the dynamic
// VALU mix of tools/valu_dyn.py).  Kernel variant K issues REP copies of ONE
// instruction in a straight line inside a fixed skeleton; variant 0 is the
// skeleton alone.  Under `rocprofv3 --pmc SQ_INSTS_*` the per-wave difference
// (variant K - variant 0) / REP says whether (1.0) or not (0.0) — or how many
// times — each counter counts that instruction.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ab/pmc_cal.hip -o tools/ab/_pmc_cal
// Run:   rocprofv3 --pmc <counters> -- tools/ab/_pmc_cal       (prints the variant table)
// Variants 0..40: the hand-written forms below; kop<OP> (kernel name "kop"):
// REP copies of every opcode of the probe's table (valu_ops.hpp), one chain.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "valu_ops.hpp"
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
#define REP "200"

template <int K>
__global__ void __launch_bounds__(256) kcal(int* g, int seed) {
    __shared__ int lds[256];
    lds[threadIdx.x] = seed;
    __syncthreads();
    unsigned a = seed + threadIdx.x, b = seed * 3;
    unsigned long long q = a;
    unsigned s = seed;
    f4 acc = {0, 0, 0, 0};
    h4 hv = {(_Float16)1, (_Float16)2, (_Float16)3, (_Float16)4};
    const unsigned lds_addr = (threadIdx.x & 63) * 4;
    if constexpr (K == 1) asm volatile(".rept " REP "\n v_add_u32 %0, %0, %1\n .endr" : "+v"(a) : "v"(b));
    else if constexpr (K == 2) asm volatile(".rept " REP "\n v_mov_b32 %0, %1\n .endr" : "+v"(a) : "v"(b));
    else if constexpr (K == 3) asm volatile(".rept " REP "\n v_pk_add_u16 %0, %0, %1\n .endr" : "+v"(a) : "v"(b));
    else if constexpr (K == 4) asm volatile(".rept " REP "\n v_dot2_i32_i16 %0, %1, %1, %0\n .endr" : "+v"(a) : "v"(b));
    else if constexpr (K == 5) asm volatile(".rept " REP "\n v_mad_i32_i24 %0, %1, %1, %0\n .endr" : "+v"(a) : "v"(b));
    else if constexpr (K == 6) asm volatile(".rept " REP "\n v_mul_lo_u32 %0, %0, %1\n .endr" : "+v"(a) : "v"(b));
    else if constexpr (K == 7) asm volatile(".rept " REP "\n v_mad_u64_u32 %0, vcc, %1, %1, %0\n .endr" : "+v"(q) : "v"(b) : "vcc");
    else if constexpr (K == 8) asm volatile(".rept " REP "\n v_lshlrev_b64 %0, 1, %0\n .endr" : "+v"(q));
    else if constexpr (K == 9) asm volatile(".rept " REP "\n v_cvt_f32_i32 %0, %0\n .endr" : "+v"(a));
    else if constexpr (K == 10) asm volatile(".rept " REP "\n v_add_f32 %0, %0, %1\n .endr" : "+v"(a) : "v"(b));
    else if constexpr (K == 11) asm volatile(".rept " REP "\n v_fma_f32 %0, %0, %1, %1\n .endr" : "+v"(a) : "v"(b));
    else if constexpr (K == 12) asm volatile(".rept " REP "\n v_mul_f32 %0, %0, %1\n .endr" : "+v"(a) : "v"(b));
    else if constexpr (K == 13) asm volatile(".rept " REP "\n v_cmp_gt_i32 vcc, %0, %1\n .endr" : : "v"(a), "v"(b) : "vcc");
    else if constexpr (K == 14) asm volatile(".rept " REP "\n v_cndmask_b32 %0, %0, %1, vcc\n .endr" : "+v"(a) : "v"(b));
    else if constexpr (K == 15) asm volatile(".rept " REP "\n v_readfirstlane_b32 %0, %1\n .endr" : "=s"(s) : "v"(a));
    else if constexpr (K == 16) asm volatile(".rept " REP "\n v_accvgpr_write_b32 a1, %0\n .endr" : : "v"(a) : "a1");
    else if constexpr (K == 17) asm volatile(".rept " REP "\n v_accvgpr_read_b32 %0, a1\n .endr" : "=v"(a) : : "a1");
    else if constexpr (K == 18) asm volatile(".rept " REP "\n v_mfma_f32_16x16x16_f16 %0, %1, %1, %0\n .endr" : "+v"(acc) : "v"(hv));
    else if constexpr (K == 19) asm volatile(".rept " REP "\n s_add_u32 %0, %0, 3\n .endr" : "+s"(s) : : "scc");
    else if constexpr (K == 20) asm volatile(".rept " REP "\n s_mov_b32 %0, %0\n .endr" : "+s"(s));
    else if constexpr (K == 21) asm volatile(".rept " REP "\n s_nop 0\n .endr");
    else if constexpr (K == 22) asm volatile(".rept " REP "\n s_waitcnt lgkmcnt(0)\n .endr");
    else if constexpr (K == 23) asm volatile(".rept " REP "\n s_cmp_eq_u32 %0, 7\n s_cbranch_scc1 1f\n 1:\n .endr" : : "s"(s) : "scc");
    else if constexpr (K == 24) asm volatile(".rept " REP "\n ds_read_b32 %0, %1\n .endr\n s_waitcnt lgkmcnt(0)" : "=v"(a) : "v"(lds_addr));
    else if constexpr (K == 25) asm volatile(".rept " REP "\n ds_write_b32 %0, %1\n .endr\n s_waitcnt lgkmcnt(0)" : : "v"(lds_addr), "v"(a));
    else if constexpr (K == 26) asm volatile(".rept " REP "\n ds_bpermute_b32 %0, %1, %0\n .endr\n s_waitcnt lgkmcnt(0)" : "+v"(a) : "v"(lds_addr));
    else if constexpr (K == 27) asm volatile(".rept " REP "\n global_load_dword %0, %1, off\n .endr\n s_waitcnt vmcnt(0)" : "=v"(a) : "v"(g + threadIdx.x));
    else if constexpr (K == 28) asm volatile(".rept " REP "\n v_perm_b32 %0, %0, %1, %1\n .endr" : "+v"(a) : "v"(b));
    else if constexpr (K == 29) asm volatile(".rept " REP "\n v_cvt_rpi_i32_f32 %0, %0\n .endr" : "+v"(a));
    else if constexpr (K == 30) asm volatile(".rept " REP "\n s_setprio 1\n .endr");
    else if constexpr (K == 31) asm volatile(".rept " REP "\n v_max_i32 %0, %0, %1\n .endr" : "+v"(a) : "v"(b));
    else if constexpr (K == 32) asm volatile(".rept " REP "\n v_readlane_b32 %0, %1, 3\n .endr" : "=s"(s) : "v"(a));
    else if constexpr (K == 33) asm volatile(".rept " REP "\n v_permlane32_swap_b32 %0, %1\n .endr" : "+v"(a), "+v"(b));
    else if constexpr (K == 34) asm volatile(".rept " REP "\n v_pk_mad_u16 %0, %0, %1, %0\n .endr" : "+v"(a) : "v"(b));
    else if constexpr (K == 35) asm volatile(".rept " REP "\n v_bfe_u32 %0, %0, 3, 5\n .endr" : "+v"(a));
    else if constexpr (K == 36) asm volatile(".rept " REP "\n s_load_dword %0, %1, 0x0\n .endr\n s_waitcnt lgkmcnt(0)" : "=s"(s) : "s"(g));
    else if constexpr (K == 37) asm volatile(".rept " REP "\n global_store_dword %0, %1, off\n .endr\n s_waitcnt vmcnt(0)" : : "v"(g + 1024 + threadIdx.x), "v"(a));
    else if constexpr (K == 38) asm volatile(".rept " REP "\n s_branch 1f\n 1:\n .endr");
    else if constexpr (K == 39) asm volatile(".rept " REP "\n v_floor_f32 %0, %0\n .endr" : "+v"(a));
    else if constexpr (K == 40) asm volatile(".rept " REP "\n v_add_co_u32 %0, vcc, %0, %1\n .endr" : "+v"(a) : "v"(b) : "vcc");
    const unsigned r = a ^ (unsigned)q ^ s ^ (unsigned)acc[0] ^ (unsigned)acc[3] ^ lds[(threadIdx.x + 1) & 255];
    if (r == 0x7fffffffu) g[threadIdx.x] = (int)r;
}
constexpr int NK = 41;
const char* const kVar[NK] = {
    "skeleton", "v_add_u32", "v_mov_b32", "v_pk_add_u16", "v_dot2_i32_i16", "v_mad_i32_i24", "v_mul_lo_u32",
    "v_mad_u64_u32", "v_lshlrev_b64", "v_cvt_f32_i32", "v_add_f32", "v_fma_f32", "v_mul_f32", "v_cmp_gt_i32",
    "v_cndmask_b32", "v_readfirstlane_b32", "v_accvgpr_write_b32", "v_accvgpr_read_b32", "v_mfma_f32_16x16x16_f16",
    "s_add_u32", "s_mov_b32", "s_nop", "s_waitcnt", "s_cmp+s_cbranch_scc1", "ds_read_b32", "ds_write_b32",
    "ds_bpermute_b32", "global_load_dword", "v_perm_b32", "v_cvt_rpi_i32_f32", "s_setprio", "v_max_i32",
    "v_readlane_b32", "v_permlane32_swap_b32", "v_pk_mad_u16", "v_bfe_u32", "s_load_dword", "global_store_dword",
    "s_branch", "v_floor_f32", "v_add_co_u32"};

template <int OP>
__global__ void __launch_bounds__(256) kop(int* g, int seed) {
    uint32_t a = seed + threadIdx.x, b = (uint32_t)(seed * 3) & 15u;
    uint64_t q = a * 0x9E3779B97F4A7C15ull, sc = 0;
    const uint64_t m = 0x5555555555555555ull ^ (uint64_t)seed;
    asm volatile("v_cmp_gt_u32_e32 vcc, %0, %1" :: "v"(a), "v"(b) : "vcc");
#pragma unroll
    for (int i = 0; i < 200; ++i) op<OP>(a, a, q, b, m, seed, sc);
    const uint32_t r = a ^ b ^ (uint32_t)q ^ (uint32_t)(q >> 32) ^ (uint32_t)sc;
    if (r == 0x7fffffffu) g[threadIdx.x] = (int)r;
}

template <int K>
static void launch_all(int* g) {
    kcal<K><<<256, 256>>>(g, K);   // 1,024 waves per variant
    if constexpr (K + 1 < NK) launch_all<K + 1>(g);
}
template <int OP>
static void launch_ops(int* g) {
    kop<OP><<<256, 256>>>(g, OP);
    if constexpr (OP + 1 < NOPS) launch_ops<OP + 1>(g);
}

int main() {
    int* g;
    if (hipMalloc(&g, 4096 * 4) != hipSuccess) return 1;
    if (hipMemset(g, 0, 4096 * 4) != hipSuccess) return 1;
    launch_all<0>(g);
    launch_ops<0>(g);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("{\"rep\": %s, \"waves_per_variant\": 1024, \"variants\": [", REP);
    for (int k = 0; k < NK; ++k) printf("%s\"%s\"", k ? ", " : "", kVar[k]);
    printf("], \"ops\": [");
    for (int k = 0; k < NOPS; ++k) printf("%s\"%s\"", k ? ", " : "", kNames[k]);
    printf("], \"insts_per_op\": [");
    for (int k = 0; k < NOPS; ++k) printf("%s%d", k ? ", " : "", insts_per_op(k));
    printf("]}\n");
    hipFree(g);
    return 0;
}
