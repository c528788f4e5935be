// nh_internal.hpp -- host-side plumbing shared by the C-ABI translation units:
// error reporting, A/B knobs and small helpers.  (The per-block call protocol
// and its per-device contexts live in nh_blocks.hip.)
#pragma once
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <mutex>
#include <string>
#include "../../include/nanohevc.h"

namespace nh {

void set_error(const std::string& msg);

#define NH_HIP(call)                                                               \
    do {                                                                           \
        hipError_t e_ = (call);                                                    \
        if (e_ != hipSuccess) {                                                    \
            ::nh::set_error(std::string(#call) + ": " + hipGetErrorString(e_));    \
            return NH_EHIP;                                                        \
        }                                                                          \
    } while (0)

// A/B knobs.  The product library (`make`) reads no environment: every knob is
// its default constant, the losing launch forms are not compiled in, and the
// knob names do not appear in the binary.  `make ab` builds
// libnanohevc_ab.so with -DNH_AB=1, where NH_KNOB reads the variable once
// (tools/ and the A/B parity tests load that library explicitly).
#ifndef NH_AB
#define NH_AB 0
#endif
#if NH_AB
#define NH_KNOB(name, dflt) ([] { const char* e_ = getenv(name); return e_ ? atoi(e_) : (dflt); }())
#else
#define NH_KNOB(name, dflt) (dflt)
#endif

// XCD-aware workgroup order of the streaming frame kernels (xcd_eighths,
// nh_common.hpp): on (A/B build: off with NH_XCD_ORDER=0).
inline bool xcd_order() {
    static const bool on = NH_KNOB("NH_XCD_ORDER", 1) != 0;
    return on;
}

// Dynamic LDS that caps `kern` at `wgs` resident workgroups per CU: the
// workgroup then reserves just over 1 / (wgs + 1) of the CU's LDS (static +
// this pad; the pad is never touched).  These kernels run faster with fewer
// resident workgroups.  Cached per kernel; 0 for wgs <= 0 or when
// the device reports no per-CU LDS figure.  A/B build: NH_OCC_CAP = 0 disables it.
template <class K>
inline unsigned lds_cap(K kern, int wgs) {
    static const int on = NH_KNOB("NH_OCC_CAP", 1);
    if (!on || wgs <= 0) return 0;
    struct Entry { const void* k; int wgs, dev; unsigned pad; };
    static Entry cache[32];
    static int used = 0;
    static std::mutex mu;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    std::lock_guard<std::mutex> g(mu);
    for (int i = 0; i < used; ++i)
        if (cache[i].k == (const void*)kern && cache[i].wgs == wgs && cache[i].dev == dev) return cache[i].pad;
    int lds_cu = 0;
    hipFuncAttributes fa{};
    if (hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess ||
        hipFuncGetAttributes(&fa, (const void*)kern) != hipSuccess) {
        (void)hipGetLastError();   // uncapped; keep the failed query out of the launch's error check
        return 0;
    }
    const long need = (long)lds_cu / (wgs + 1) + 1 - (long)fa.sharedSizeBytes;   // wgs + 1 must not fit
    const unsigned pad = need > 0 ? (unsigned)need : 0u;
    if (used < 32) cache[used++] = Entry{(const void*)kern, wgs, dev, pad};
    return pad;
}

#define NH_TRY(x)              \
    do {                       \
        int rc__ = (x);        \
        if (rc__) return rc__; \
    } while (0)

// Per-device one-time initialisation, thread-safe: init() runs at most once per
// device (again only if it failed), under a lock, on the calling thread with
// that device current.  init() must be host-synchronous (e.g. hipMemcpyToSymbol
// or a launch it synchronises), so work queued afterwards on ANY stream sees it.
struct PerDeviceOnce {
    std::mutex mu;
    bool done[64] = {};
    template <class F>
    int run(F init) {
        int dev = 0;
        NH_HIP(hipGetDevice(&dev));
        if (dev < 0 || dev >= 64) return NH_EARG;
        std::lock_guard<std::mutex> lk(mu);
        if (done[dev]) return NH_OK;
        const int rc = init();
        if (rc == NH_OK) done[dev] = true;
        return rc;
    }
};

// Compute units of the current device, cached per device (thread-safe).
inline int device_cus(int* out) {
    static std::mutex mu;
    static int cus[64] = {};
    int dev = 0;
    NH_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return NH_EARG;
    std::lock_guard<std::mutex> lk(mu);
    if (!cus[dev]) NH_HIP(hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev));
    *out = cus[dev];
    return NH_OK;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

}  // namespace nh
