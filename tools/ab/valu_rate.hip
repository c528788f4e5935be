// VALU issue-rate probe (round 4): chip-wide wave-instructions per second of one
// opcode at a time AND the SIMD cycles each wave-instruction costs, measured
// with the shader clock inside the kernel (s_memtime), so a rate difference can
// be told apart from a clock difference.  tools/valu_mix.py / tools/valu_dyn.py
// price each kernel's VALU mix with these rates (the roofline peak of the
// VALU-bound configs).
//
// Round-3 probe errors fixed here:
//  * "v_mov_b32" issued a v_xor_b32 AND a v_mov_b32 per counted op; now one
//    v_mov_b32 per op (self move, and a rotation across the 8 chains);
//  * every opcode is measured in ROUNDS interleaved with all the others, best of
//    the rounds, so clock drift between opcodes cannot masquerade as a rate;
//  * each opcode sits beside its siblings of the same encoding (VOP2 shifts
//    with an inline constant or a VGPR amount, v_max/min signed/unsigned,
//    v_cndmask with VCC or an SGPR pair) so a half rate shows on a whole family
//    or on one member;
//  * the classes tools/valu_mix.py priced without a measurement
//    (v_lshlrev_b64, v_readfirstlane_b32, v_permlane32_swap, v_fma_f32) are
//    measured;
//  * the opcodes of interest are also swept over 1 / 2 / 4 / 8 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ab/valu_rate.hip -o tools/ab/_valu_rate
// Run:   tools/ab/_valu_rate > valu_rate.jsonl      (one JSON line per opcode and wave count)
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>
typedef short v2s __attribute__((ext_vector_type(2)));
constexpr int ITERS = 2048;

// one opcode per OP; a[]: 32-bit chains, q[]: 64-bit chains.  `n` is the next
// chain's value (for the rotation forms).
template <int OP>
__device__ __forceinline__ void op(uint32_t& a, uint32_t n, uint64_t& q, uint32_t b, uint64_t m, int seed, uint64_t& sc) {
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
    else if constexpr (OP == 13) asm volatile("v_mov_b32 %0, %0" : "+v"(a));
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
    // ---- round 4: siblings and the classes priced without a measurement before
    else if constexpr (OP == 36) asm volatile("v_mov_b32 %0, %1" : "=v"(a) : "v"(n));            // rotation: a_i = a_{i+1}
    else if constexpr (OP == 37) asm volatile("v_or_b32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 38) asm volatile("v_max_u32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 39) asm volatile("v_min_i32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 40) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(a) : "v"(b));   // VGPR amount
    else if constexpr (OP == 41) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(a) : "v"(b));
    else if constexpr (OP == 42) asm volatile("v_ashrrev_i32 %0, %1, %0" : "+v"(a) : "v"(b));
    else if constexpr (OP == 43) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a) : "v"(b));   // VOP2, VCC
    else if constexpr (OP == 44) asm volatile("v_not_b32 %0, %0" : "+v"(a));
    else if constexpr (OP == 45) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a) : "v"(b), "s"(seed));
    else if constexpr (OP == 46) asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(q));
    else if constexpr (OP == 47) {
        uint32_t s;
        asm volatile("v_readfirstlane_b32 %0, %1" : "=s"(s) : "v"(a));
        sc = s;
    } else if constexpr (OP == 48) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 49) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    else if constexpr (OP == 50) asm volatile("v_cvt_rpi_i32_f32 %0, %0" : "+v"(a));
    else if constexpr (OP == 51) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 52) asm volatile("v_lshlrev_b16 %0, 3, %0" : "+v"(a));
    else if constexpr (OP == 53) asm volatile("v_sub_i32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 54) asm volatile("v_max_f32 %0, %0, %1" : "+v"(a) : "v"(b));
    else if constexpr (OP == 55) asm volatile("v_accvgpr_write_b32 a0, %0\n v_accvgpr_read_b32 %0, a0" : "+v"(a) :: "a0");
}
constexpr int NOPS = 56;
const char* const kNames[NOPS] = {
    "v_dot2c_i32_i16", "v_mad_i32_i24", "v_pk_add_u16", "v_add_u32", "v_lshlrev_b32", "v_cndmask_b32",
    "v_perm_b32", "v_bfe_i32", "v_ashrrev_i32", "v_pk_mad_u16", "v_mul_lo_u32", "v_mul_i32_i24",
    "v_add3_u32", "v_mov_b32", "v_pk_sub_i16", "v_lshl_add_u64", "v_cmp_gt_i32", "v_add_f32",
    "v_floor_f32", "v_cvt_i32_f32", "v_med3_i32", "v_pk_lshrrev_b16", "v_mad_u64_u32", "v_readlane_b32",
    "v_xor_b32", "v_sub_u32", "v_lshrrev_b32", "v_dot2_i32_i16", "v_lshl_or_b32", "v_and_b32",
    "v_cvt_f32_i32", "v_pk_max_i16", "v_max_i32", "v_mul_u32_u24", "v_mul_i32_i24_sdwa", "v_lshl_add_u32",
    "v_mov_b32_rot", "v_or_b32", "v_max_u32", "v_min_i32", "v_lshlrev_b32_vamt", "v_lshrrev_b32_vamt",
    "v_ashrrev_i32_vamt", "v_cndmask_b32_vcc", "v_not_b32", "v_bfi_b32", "v_lshlrev_b64", "v_readfirstlane_b32",
    "v_fma_f32", "v_permlane32_swap", "v_cvt_rpi_i32_f32", "v_add_co_u32", "v_lshlrev_b16", "v_sub_i32",
    "v_max_f32", "v_accvgpr_write_read_pair"};
// instructions per counted op (the accvgpr pair issues two)
__host__ __device__ constexpr int insts_per_op(int opi) { return opi == 55 ? 2 : 1; }

// cyc[wave] = shader-clock cycles of the timed loop (lane 0 of each wave stores, vector store)
template <int OP>
__global__ void __launch_bounds__(256) k(int* out, unsigned long long* cyc, int seed) {
    uint32_t a[8], b[8];
    uint64_t q[8], sc[8] = {};
    const uint64_t m = 0x5555555555555555ull ^ (uint64_t)seed;
    for (int i = 0; i < 8; ++i) {
        a[i] = seed + i + threadIdx.x;
        b[i] = (uint32_t)(seed * 3 + i) & 15u;
        q[i] = a[i] * 0x9E3779B97F4A7C15ull;
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) op<OP>(a[i], a[(i + 1) & 7], q[i], b[i], m, seed, sc[i]);
    }
    uint32_t s = 0;
    for (int i = 0; i < 8; ++i) s ^= a[i] ^ b[i] ^ (uint32_t)q[i] ^ (uint32_t)(q[i] >> 32) ^ (uint32_t)sc[i];
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
    if (s == 0x12345u) out[threadIdx.x] = (int)s;
}

struct Res {
    float ms = 1e30f;
    double cyc = 0;   // mean per-wave loop cycles of the best run
};

template <int OP>
static void run_one(int blocks, int threads, int* d, unsigned long long* dc, int rep, Res& r) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    k<OP><<<blocks, threads>>>(d, dc, rep);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    if (ms < r.ms) {
        const int waves = blocks * threads / 64;
        std::vector<unsigned long long> h(waves);
        hipMemcpy(h.data(), dc, waves * sizeof(unsigned long long), hipMemcpyDeviceToHost);
        double s = 0;
        for (auto v : h) s += (double)v;
        r.ms = ms;
        r.cyc = s / waves;
    }
}

typedef void (*RunFn)(int, int, int*, unsigned long long*, int, Res&);
template <int OP>
static void fill(RunFn* t) {
    t[OP] = &run_one<OP>;
    if constexpr (OP + 1 < NOPS) fill<OP + 1>(t);
}

static void report(int opi, const Res& r, int blocks, int threads, int cus, int clock_khz, int waves_per_simd, int rounds) {
    const double winst = (double)blocks * (threads / 64) * ITERS * 8 * insts_per_op(opi);
    const double per_s = winst / (r.ms * 1e-3);
    // SIMD cycles per wave-instruction: every SIMD interleaves waves_per_simd waves,
    // each issuing 8*ITERS*k instructions inside its timed loop
    const double cpi = r.cyc / ((double)waves_per_simd * 8 * ITERS * insts_per_op(opi));
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"chip_winst_per_s\": %.6e, "
           "\"simd_cycles_per_winst\": %.4f, \"loop_cycles_per_wave\": %.0f, \"clock_GHz_implied\": %.4f, "
           "\"wave_instr_per_simd_cycle_nominal\": %.4f, \"clock_khz_nominal\": %d, \"rounds\": %d}\n",
           kNames[opi], waves_per_simd, r.ms, per_s, cpi, r.cyc, r.cyc / (r.ms * 1e6),
           per_s / (cus * 4.0) / (clock_khz * 1e3), clock_khz, rounds);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 5;
    int* d;
    unsigned long long* dc;
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    if (hipMalloc(&d, 1024 * 4) != hipSuccess) return 1;
    if (hipMalloc(&dc, (size_t)cus * 8 * 4 * sizeof(unsigned long long)) != hipSuccess) return 1;
    RunFn t[NOPS];
    fill<0>(t);
    // 1) every opcode at 8 waves/SIMD (8 workgroups x 4 waves per CU), interleaved rounds
    std::vector<Res> best(NOPS);
    for (int rd = 0; rd < rounds; ++rd)
        for (int o = 0; o < NOPS; ++o) t[o](cus * 8, 256, d, dc, rd, best[o]);
    for (int o = 0; o < NOPS; ++o) report(o, best[o], cus * 8, 256, cus, p.clockRate, 8, rounds);
    // 2) the families in question over 1/2/4/8 waves per SIMD (workgroups of 64 x 4 waves,
    //    one wave per SIMD per workgroup), interleaved
    const int sweep_ops[] = {3, 26, 4, 40, 8, 32, 38, 39, 5, 43, 13, 36, 24, 37, 17, 48, 27, 11};
    const int wps[] = {1, 2, 4, 8};
    for (int w : wps) {
        std::vector<Res> bs(NOPS);
        for (int rd = 0; rd < rounds; ++rd)
            for (int o : sweep_ops) t[o](cus * w, 256, d, dc, 100 + rd, bs[o]);
        for (int o : sweep_ops) report(o, bs[o], cus * w, 256, cus, p.clockRate, w, rounds);
    }
    hipFree(dc);
    hipFree(d);
    return 0;
}
