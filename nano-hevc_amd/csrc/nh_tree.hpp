// nh_tree.hpp -- the config-4 seeded TU quadtree, shared by
// the per-size TU kernels (nh_intraloop.hip) and the int8-MFMA 32x32 kernel
// (nh_tc32.hip).  Mirrors oh_tu_split in the CPU restatement bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace nh {

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
__device__ __forceinline__ bool tu_split(uint32_t seed, int plane_id, int x, int y, int size) {
    uint32_t k = mix32(seed ^ (0x9E3779B9U * (uint32_t)(plane_id + 1)));
    k = mix32(k ^ (uint32_t)x);
    k = mix32(k ^ ((uint32_t)y * 0x85ebca6bU));
    k = mix32(k ^ (uint32_t)size);
    return (k & 3u) < 2u;
}

// Leaf of the seeded quadtree containing sample (ux, uy):
// descend from the CTB root, at most 3 hash evaluations.  Returns its size.
__device__ __forceinline__ int tu_leaf(int w, int h, int ctb, int plane_id, uint32_t seed, int ux, int uy) {
    int s = ctb, x = (ux / ctb) * ctb, y = (uy / ctb) * ctb;
    while (s > 4 && ((x + s > w) || (y + s > h) || tu_split(seed, plane_id, x, y, s))) {
        s >>= 1;
        x += (ux >= x + s) ? s : 0;
        y += (uy >= y + s) ? s : 0;
    }
    return s;
}

enum { kAll = 0, kTree = 1 };
struct TreeArgs {
    int ctb, plane_id, y_base;   // y_base: first sample row of the band
    uint32_t seed;
    // batch of planes (blockIdx.y): plane p = g * ppg + c lives at
    // g * group_stride + c * plane_stride, has plane id plane_id + c and its
    // TU map at tu_log2 + p * tu_plane
    int ppg = 1;
    int64_t group_stride = 0, plane_stride = 0, tu_plane = 0;
};

}  // namespace nh
