// VALU issue-rate probe (A/B record for DESIGN.md §4.4c): wave-instructions per
// SIMD-cycle of v_dot2c_i32_i16 (literal weights), v_mad_i32_i24, v_pk_add_u16
// and v_add_u32, 8 independent chains per lane, enough waves to fill the chip.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ab/valu_rate.hip -o tools/ab/_valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef short v2s __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096;

template <int OP>
__global__ void __launch_bounds__(256) k(int* out, int seed) {
    int a[8];
    uint32_t b[8];
    for (int i = 0; i < 8; ++i) { a[i] = seed + i + threadIdx.x; b[i] = (uint32_t)(seed * 3 + i); }
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (OP == 0) {
                a[i] = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2s, b[i]), (v2s){83, -36}, a[i], false);
            } else if constexpr (OP == 1) {
                asm volatile("v_mad_i32_i24 %0, %1, %2, %0" : "+v"(a[i]) : "v"(b[i]), "s"(seed + 83));
            } else if constexpr (OP == 2) {
                asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
            } else {
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
            }
        }
    }
    int s = 0;
    for (int i = 0; i < 8; ++i) s ^= a[i];
    if (s == 0x12345) out[threadIdx.x] = s;
}

int main() {
    int* d;
    hipMalloc(&d, 1024 * 4);
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount, blocks = cus * 8;   // 8 workgroups x 4 waves per CU = 8 waves per SIMD
    const char* names[4] = {"v_dot2c_i32_i16", "v_mad_i32_i24", "v_pk_add_u16", "v_add_u32"};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int op = 0; op < 4; ++op) {
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(e0);
            if (op == 0) k<0><<<blocks, 256>>>(d, rep);
            if (op == 1) k<1><<<blocks, 256>>>(d, rep);
            if (op == 2) k<2><<<blocks, 256>>>(d, rep);
            if (op == 3) k<3><<<blocks, 256>>>(d, rep);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double winst = (double)blocks * 4 * ITERS * 8;   // wave-instructions
            const double per_simd_cycle = winst / (cus * 4.0) / (ms * 1e-3 * p.clockRate * 1e3);
            if (rep == 2)
                printf("{\"op\": \"%s\", \"ms\": %.4f, \"wave_instr_per_simd_cycle\": %.4f, \"clock_khz\": %d}\n", names[op],
                       ms, per_simd_cycle, p.clockRate);
        }
    }
    return 0;
}
