// VALU issue-rate probe: chip-wide wave-instructions per second of one opcode at
// a time, 8 independent chains per lane, 8 waves per SIMD (enough to saturate
// issue), on the clock the chip holds under that load.  tools/valu_mix.py prices
// each kernel's static VALU mix with these rates to get its attainable VALU rate
// (the roofline peak of the VALU-bound configs).
// Build: hipcc --offload-arch=gfx950 -O3 tools/ab/valu_rate.hip -o tools/ab/_valu_rate
// Run:   tools/ab/_valu_rate > valu_rate.jsonl      (one JSON line per opcode)
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
typedef short v2s __attribute__((ext_vector_type(2)));
constexpr int ITERS = 2048;

// one opcode per OP; a[]: 32-bit chains, q[]: 64-bit chains
template <int OP>
__device__ __forceinline__ void op(uint32_t& a, uint64_t& q, uint32_t b, uint64_t m, int seed, uint64_t& sc) {
    if constexpr (OP == 0) a = (uint32_t)__builtin_amdgcn_sdot2(__builtin_bit_cast(v2s, b), (v2s){83, -36}, (int)a, false);
    else if constexpr (OP == 1) asm volatile("v_mad_i32_i24 %0, %1, %2, %0" : "+v"(a) : "v"(b), "s"(seed + 83));
    else if constexpr (OP == 2) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 3) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 4) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(a));
    else if constexpr (OP == 5) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a) : "v"(b), "s"(m));
    else if constexpr (OP == 6) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "s"(0x05040100));
    else if constexpr (OP == 7) asm volatile("v_bfe_i32 %0, %0, 5, 11" : "+v"(a));
    else if constexpr (OP == 8) asm volatile("v_ashrrev_i32 %0, 5, %0" : "+v"(a));
    else if constexpr (OP == 9) asm volatile("v_pk_mad_u16 %0, %0, %1, %0" : "+v"(a) : "v"(b));
    else if constexpr (OP == 10) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 11) asm volatile("v_mul_i32_i24 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 12) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 13) asm volatile("v_mov_b32 %0, %1" : "=v"(a) : "v"(b ^ a));
    else if constexpr (OP == 14) asm volatile("v_pk_sub_i16 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 15) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(q) : "v"(m));
    else if constexpr (OP == 16) asm volatile("v_cmp_gt_i32_e64 %0, %1, %2" : "=s"(sc) : "v"(a), "v"(b));
    else if constexpr (OP == 17) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 18) asm volatile("v_floor_f32 %0, %0" : "+v"(a));
    else if constexpr (OP == 19) asm volatile("v_cvt_i32_f32 %0, %0" : "+v"(a));
    else if constexpr (OP == 20) asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "s"(seed));
    else if constexpr (OP == 21) asm volatile("v_pk_lshrrev_b16 %0, 1, %0" : "+v"(a));
    else if constexpr (OP == 22) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(q), "=s"(sc) : "v"(a), "v"(b));
    else if constexpr (OP == 23) {
        uint32_t s;
        asm volatile("v_readlane_b32 %0, %1, 5" : "=s"(s) : "v"(a));
        sc = s;
    } else if constexpr (OP == 24) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 25) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 26) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(a));
    else if constexpr (OP == 27) asm volatile("v_dot2_i32_i16 %0, %1, %2, %0" : "+v"(a) : "v"(b), "s"(0x00530024));
    else if constexpr (OP == 28) asm volatile("v_lshl_or_b32 %0, %0, 2, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 29) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 30) asm volatile("v_cvt_f32_i32 %0, %0" : "+v"(a));
    else if constexpr (OP == 31) asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 32) asm volatile("v_max_i32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 33) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 34) asm volatile("v_mul_i32_i24_sdwa %0, sext(%0), sext(%1) dst_sel:DWORD src0_sel:WORD_0 src1_sel:WORD_1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 35) asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(a) : "v"(b));
}
constexpr int NOPS = 36;
const char* const kNames[NOPS] = {
    "v_dot2c_i32_i16", "v_mad_i32_i24", "v_pk_add_u16", "v_add_u32", "v_lshlrev_b32", "v_cndmask_b32",
    "v_perm_b32", "v_bfe_i32", "v_ashrrev_i32", "v_pk_mad_u16", "v_mul_lo_u32", "v_mul_i32_i24",
    "v_add3_u32", "v_mov_b32", "v_pk_sub_i16", "v_lshl_add_u64", "v_cmp_gt_i32", "v_add_f32",
    "v_floor_f32", "v_cvt_i32_f32", "v_med3_i32", "v_pk_lshrrev_b16", "v_mad_u64_u32", "v_readlane_b32",
    "v_xor_b32", "v_sub_u32", "v_lshrrev_b32", "v_dot2_i32_i16", "v_lshl_or_b32", "v_and_b32",
    "v_cvt_f32_i32", "v_pk_max_i16", "v_max_i32", "v_mul_u32_u24", "v_mul_i32_i24_sdwa", "v_lshl_add_u32"};

template <int OP>
__global__ void __launch_bounds__(256) k(int* out, int seed) {
    uint32_t a[8], b[8];
    uint64_t q[8], sc[8] = {};
    const uint64_t m = 0x5555555555555555ull ^ (uint64_t)seed;
    for (int i = 0; i < 8; ++i) {
        a[i] = seed + i + threadIdx.x;
        b[i] = (uint32_t)(seed * 3 + i);
        q[i] = a[i] * 0x9E3779B97F4A7C15ull;
    }
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) op<OP>(a[i], q[i], b[i], m, seed, sc[i]);
    }
    uint32_t s = 0;
    for (int i = 0; i < 8; ++i) s ^= a[i] ^ b[i] ^ (uint32_t)q[i] ^ (uint32_t)(q[i] >> 32) ^ (uint32_t)sc[i];
    if (s == 0x12345u) out[threadIdx.x] = (int)s;
}

template <int OP>
static float run(int blocks, int* d, int rep) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    k<OP><<<blocks, 256>>>(d, rep);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return ms;
}

template <int OP>
static void measure(int blocks, int* d, int cus, int clock_khz) {
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
        const float ms = run<OP>(blocks, d, rep);
        if (rep > 0 && ms < best) best = ms;   // rep 0 warms the clock / code
    }
    const double winst = (double)blocks * 4 * ITERS * 8;   // wave-instructions of the opcode
    const double per_s = winst / (best * 1e-3);
    printf("{\"op\": \"%s\", \"ms\": %.4f, \"chip_winst_per_s\": %.6e, \"wave_instr_per_simd_cycle_nominal\": %.4f, "
           "\"clock_khz_nominal\": %d, \"waves_per_simd\": 8}\n",
           kNames[OP], best, per_s, per_s / (cus * 4.0) / (clock_khz * 1e3), clock_khz);
    fflush(stdout);
    if constexpr (OP + 1 < NOPS) measure<OP + 1>(blocks, d, cus, clock_khz);
}

int main() {
    int* d;
    if (hipMalloc(&d, 1024 * 4) != hipSuccess) return 1;
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount, blocks = cus * 8;   // 8 workgroups x 4 waves per CU = 8 waves per SIMD
    measure<0>(blocks, d, cus, p.clockRate);
    hipFree(d);
    return 0;
}
