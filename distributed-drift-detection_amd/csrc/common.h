// Shared helpers for the C-ABI entry points (error reporting, launch checks).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ddm_amd.h"

namespace ddm {

void set_error(const char* fmt, ...);

inline int hip_status(hipError_t e, const char* where) {
    if (e == hipSuccess) return 0;
    set_error("%s: %s", where, hipGetErrorString(e));
    return (int)e;
}

// Status of the last kernel launch on this thread.
inline int launch_status(const char* where) { return hip_status(hipGetLastError(), where); }

inline hipStream_t as_hip(ddm_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace ddm
