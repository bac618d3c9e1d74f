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

// A pointer into device (global) memory as the global address space: loads and stores
// through it are global_* instructions.  A pointer loaded from a job table is generic, so
// its accesses are flat_* instructions, which count on both vmcnt and lgkmcnt: every LDS
// wait of a kernel then also waits for its outstanding memory operations (and the other
// way round).  Keep the result typed as such down to the accesses (a cast back to generic
// is folded away).
template <typename T>
using gptr = __attribute__((address_space(1))) T*;
// ... and into LDS (ds_* instructions, counting on lgkmcnt only)
template <typename T>
using lptr = __attribute__((address_space(3))) T*;
template <typename T>
__device__ __forceinline__ gptr<T> as_global(T* p) {
    return (gptr<T>)p;
}
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ int4 ld_int4(gptr<const int32_t> p) {   // 16-byte aligned
    const i32x4 v = *(gptr<const i32x4>)p;
    return make_int4(v.x, v.y, v.z, v.w);
}
// Whole-struct copies to / from the global address space (no implicit operator= across
// address spaces): word-wise in the struct's own alignment, which the compiler merges.
template <typename T>
__device__ __forceinline__ void gput(gptr<T> p, const T& v) {
    static_assert(sizeof(T) % 4 == 0, "word-sized structs only");
    const uint32_t* s = reinterpret_cast<const uint32_t*>(&v);
    gptr<uint32_t> d = (gptr<uint32_t>)p;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); ++i) d[i] = s[i];
}
template <typename T>
__device__ __forceinline__ T gget(gptr<const T> p) {
    static_assert(sizeof(T) % 4 == 0, "word-sized structs only");
    T v;
    uint32_t* d = reinterpret_cast<uint32_t*>(&v);
    gptr<const uint32_t> s = (gptr<const uint32_t>)p;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); ++i) d[i] = s[i];
    return v;
}

// Cross-stream order by a sequence number in device memory (ddm_ctl_epoch.sync_flags):
// the producer's data are released (agent scope) before the number is stored; a poll ends
// when the number reaches v, or gives up and counts that in timeouts[0].  The give-up is a
// hang guard only: timeouts[1] (sync_flags[3]) is the join polls' limit in 10-ns ticks, 0 = 2 s (a
// group of epochs lasts ~0.5-2 ms; the limit must also outlast serialised dispatch under a
// profiler).  A give-up voids the phase and the runner redoes the run with event-ordered
// fork / join (ddm_amd/devctl.py FlagTimeout).  One thread each.
__device__ inline void flag_publish(uint32_t* flag, uint32_t v) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ inline void flag_poll(const uint32_t* flag, uint32_t v, uint32_t* timeouts) {
    const uint64_t t0 = wall_clock64();
    // the override applies to the join polls only: their consumers read perm bytes, every
    // one of which is a valid in-batch offset whenever it is read; the fork's consumers read
    // job tables, so the fork wait (flags[0], timeouts - 2) keeps the 2-s guard
    const uint32_t lim =
        flag == timeouts - 2 ? 0u : __hip_atomic_load(timeouts + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t limit = lim ? (uint64_t)lim : 200000000ull;   // 2 s at 100 MHz
    while ((int32_t)(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - v) < 0) {
        __builtin_amdgcn_s_sleep(1);
        if (wall_clock64() - t0 > limit) {
            atomicAdd(timeouts, 1u);
            break;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

}  // namespace ddm
