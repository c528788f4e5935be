// LDS-DMA semantics probe (A/B tooling): where global_load_lds_dwordx4 /
// _ushort put each lane's bytes for a given M0, and what vmcnt retires them.
// Prints one JSON line: for each form, the LDS byte offsets each lane's data
// landed at (as found by the unique source pattern).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef __attribute__((address_space(3))) void lds_void_t;
__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)(lds_void_t*)(p); }

template <int FORM>
__global__ void k_probe(const uint16_t* src, uint16_t* out, int base_bytes) {
    __shared__ __attribute__((aligned(16))) uint16_t buf[4096];
    const int lane = threadIdx.x;
    for (int i = lane; i < 4096; i += 64) buf[i] = 0xEEEE;
    __syncthreads();
    const uint32_t m0v = __builtin_amdgcn_readfirstlane(lds_addr(buf) + base_bytes);
    uint32_t keep;
    if (FORM == 0) {   // 16 B per lane, source lane * 16 B
        const uint16_t* g = src + lane * 8;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(m0v) : "memory");
    } else if (FORM == 1) {   // 2 B per lane, source lane * 2 B * 37 (strided)
        const uint16_t* g = src + lane * 37;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_ushort %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(m0v) : "memory");
    } else {   // 16 B, lanes < 4 only
        const uint16_t* g = src + lane * 8;
        if (lane < 4)
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(g), "s"(m0v) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = lane; i < 4096; i += 64) out[i] = buf[i];
}

int main() {
    std::vector<uint16_t> h(65536);
    for (int i = 0; i < 65536; ++i) h[i] = (uint16_t)i;
    uint16_t *d, *o;
    hipMalloc(&d, 65536 * 2);
    hipMalloc(&o, 4096 * 2);
    hipMemcpy(d, h.data(), 65536 * 2, hipMemcpyHostToDevice);
    std::vector<uint16_t> r(4096);
    printf("{");
    for (int form = 0; form < 3; ++form) {
        for (int base : {0, 256}) {
            if (form == 0) k_probe<0><<<1, 64>>>(d, o, base);
            if (form == 1) k_probe<1><<<1, 64>>>(d, o, base);
            if (form == 2) k_probe<2><<<1, 64>>>(d, o, base);
            if (hipDeviceSynchronize() != hipSuccess) { printf("\"error\": 1}\n"); return 1; }
            hipMemcpy(r.data(), o, 4096 * 2, hipMemcpyDeviceToHost);
            printf("%s\"form%d_base%d\": [", form || base ? ", " : "", form, base);
            bool first = true;
            for (int i = 0; i < 4096; ++i)
                if (r[i] != 0xEEEE) {   // LDS halfword i holds source element r[i]
                    if (!first) printf(", ");
                    printf("[%d, %d]", 2 * i, r[i]);
                    first = false;
                }
            printf("]");
        }
    }
    printf("}\n");
    return 0;
}
