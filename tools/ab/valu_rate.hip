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
#include <algorithm>
#include <map>
#include <vector>
#include "valu_ops.hpp"
constexpr int ITERS = 2048;

// Per wave (lane 0, vector stores): shader-clock stamps around the timed loop
// (s_memtime), the same in the 100 MHz constant clock (s_memrealtime), and the
// wave's hardware place (HW_ID: SIMD / CU / SH / SE, and the XCC id), so the
// host can take each SIMD's issue span and the clock the chip held.
struct WaveRec {
    unsigned long long t0, t1, r0, r1, place;
};
template <int OP>
__global__ void __launch_bounds__(256) k(int* out, WaveRec* rec, int seed) {
    uint32_t a[8], b[8];
    uint64_t q[8], sc[8] = {};
    const uint64_t m = 0x5555555555555555ull ^ (uint64_t)seed;
    for (int i = 0; i < 8; ++i) {
        a[i] = seed + i + threadIdx.x;
        b[i] = (uint32_t)(seed * 3 + i) & 15u;
        q[i] = a[i] * 0x9E3779B97F4A7C15ull;
    }
    asm volatile("v_cmp_gt_u32_e32 vcc, %0, %1" :: "v"(a[0]), "v"(b[0]) : "vcc");   // a defined VCC for the VCC-mask forms
    uint32_t hwid, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) op<OP>(a[i], a[(i + 1) & 7], q[i], b[i], m, seed, sc[i]);
    }
    uint32_t s = 0;
    for (int i = 0; i < 8; ++i) s ^= a[i] ^ b[i] ^ (uint32_t)q[i] ^ (uint32_t)(q[i] >> 32) ^ (uint32_t)sc[i];
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0)
        rec[blockIdx.x * 4 + threadIdx.x / 64] = WaveRec{t0, t1, r0, r1, ((unsigned long long)xcc << 32) | hwid};
    if (s == 0x12345u) out[threadIdx.x] = (int)s;
}

struct Res {
    float ms = 1e30f;
    double cpi = 0;      // SIMD cycles per wave-instruction: per SIMD, its waves' issues over its span
    double clk = 0;      // GHz the chip held in the loops (memtime ticks / realtime)
    double cyc = 0;      // mean per-wave loop cycles
};

template <int OP>
static void run_one(int blocks, int threads, int* d, WaveRec* dr, int rep, Res& r) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    k<OP><<<blocks, threads>>>(d, dr, rep);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    if (ms < r.ms) {
        const int waves = blocks * threads / 64;
        std::vector<WaveRec> h(waves);
        hipMemcpy(h.data(), dr, waves * sizeof(WaveRec), hipMemcpyDeviceToHost);
        std::map<unsigned long long, std::pair<unsigned long long, unsigned long long>> span;   // SIMD -> [min t0, max t1]
        std::map<unsigned long long, int> nw;
        double cyc = 0, ticks = 0, real = 0;
        for (auto& w : h) {
            // HW_ID: simd [5:4], cu [11:8], sh [12], se [15:13]; + XCC
            const unsigned long long key = ((w.place >> 32) << 16) | (w.place & 0xFF30u) | 0;
            auto it = span.find(key);
            if (it == span.end()) span[key] = {w.t0, w.t1};
            else { it->second.first = std::min(it->second.first, w.t0); it->second.second = std::max(it->second.second, w.t1); }
            nw[key] += 1;
            cyc += (double)(w.t1 - w.t0);
            ticks += (double)(w.t1 - w.t0);
            real += (double)(w.r1 - w.r0);
        }
        double cpi = 0;
        for (auto& kv : span) cpi += (double)(kv.second.second - kv.second.first) / ((double)nw[kv.first] * 8 * ITERS);
        r.ms = ms;
        r.cyc = cyc / waves;
        r.cpi = cpi / span.size();
        r.clk = real > 0 ? ticks / (real * 10.0) : 0;   // realtime: 100 MHz
    }
}

typedef void (*RunFn)(int, int, int*, WaveRec*, int, Res&);
template <int OP>
static void fill(RunFn* t) {
    t[OP] = &run_one<OP>;
    if constexpr (OP + 1 < NOPS) fill<OP + 1>(t);
}

static void report(int opi, const Res& r, int blocks, int threads, int cus, int clock_khz, int waves_per_simd, int rounds) {
    const double winst = (double)blocks * (threads / 64) * ITERS * 8 * insts_per_op(opi);
    const double per_s = winst / (r.ms * 1e-3);
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"chip_winst_per_s\": %.6e, "
           "\"simd_cycles_per_winst\": %.4f, \"loop_cycles_per_wave\": %.0f, \"clock_GHz_held\": %.4f, "
           "\"wave_instr_per_simd_cycle_nominal\": %.4f, \"clock_khz_nominal\": %d, \"rounds\": %d}\n",
           kNames[opi], waves_per_simd, r.ms, per_s, r.cpi / insts_per_op(opi), r.cyc, r.clk,
           per_s / (cus * 4.0) / (clock_khz * 1e3), clock_khz, rounds);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 5;
    int* d;
    WaveRec* dc;
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    if (hipMalloc(&d, 1024 * 4) != hipSuccess) return 1;
    if (hipMalloc(&dc, (size_t)cus * 8 * 4 * sizeof(WaveRec)) != hipSuccess) return 1;
    RunFn t[NOPS];
    fill<0>(t);
    // 1) every opcode at 8 waves/SIMD (8 workgroups x 4 waves per CU), interleaved rounds
    std::vector<Res> best(NOPS);
    for (int rd = 0; rd < rounds; ++rd)
        for (int o = 0; o < NOPS; ++o) t[o](cus * 8, 256, d, dc, rd, best[o]);
    for (int o = 0; o < NOPS; ++o) report(o, best[o], cus * 8, 256, cus, p.clockRate, 8, rounds);
    // 2) the families in question over 1/2/4/8 waves per SIMD (workgroups of 64 x 4 waves,
    //    one wave per SIMD per workgroup), interleaved
    const int sweep_ops[] = {3, 26, 4, 40, 8, 32, 38, 39, 5, 43, 13, 36, 24, 37, 17, 48, 27, 11, 54, 93, 73};
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
