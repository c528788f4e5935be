// nh_internal.hpp -- host-side plumbing shared by the C-ABI translation units:
// error reporting, the per-process staging context used by the synchronous
// per-block entry points, and argument checks.
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

// Per-process staging context for the per-block (host pointer) entry points.
// One device buffer + one pinned host buffer, grown on demand, one stream.
// Guarded by a mutex: per-block calls are reentrant but serialised.
struct Staging {
    std::mutex mu;
    int device = -1;
    hipStream_t stream = nullptr;
    void* dbuf = nullptr;
    void* hbuf = nullptr;
    size_t cap = 0;
    int* dstatus = nullptr;
};
Staging& staging();
// Ensure the context exists on the current device with >= bytes of buffer.
int staging_reserve(Staging& s, size_t bytes);
// Copy host->device for a region of the staging buffer.
int staging_upload(Staging& s, size_t off, const void* src, size_t bytes);
int staging_download(Staging& s, void* dst, size_t off, size_t bytes);
int staging_finish(Staging& s, int* status_out);  // sync + fetch kernel status word

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

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

}  // namespace nh
