// C-ABI housekeeping: version and per-thread last-error string.
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace ddm {

static thread_local char g_last_error[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
    va_end(ap);
}

}  // namespace ddm

extern "C" int ddm_abi_version(void) { return DDM_AMD_ABI_VERSION; }

extern "C" const char* ddm_last_error(void) { return ddm::g_last_error; }

extern "C" int ddm_event_create(ddm_event_t* ev) {
    if (!ev) return DDM_E_ARG;
    hipEvent_t e;
    if (int rc = ddm::hip_status(hipEventCreate(&e), "ddm_event_create")) return rc;
    *ev = reinterpret_cast<ddm_event_t>(e);
    return 0;
}

// An event for stream ordering only (no timestamps): the epochs' fork / join events.
extern "C" int ddm_event_create_sync(ddm_event_t* ev) {
    if (!ev) return DDM_E_ARG;
    hipEvent_t e;
    if (int rc = ddm::hip_status(hipEventCreateWithFlags(&e, hipEventDisableTiming), "ddm_event_create_sync"))
        return rc;
    *ev = reinterpret_cast<ddm_event_t>(e);
    return 0;
}

extern "C" int ddm_event_destroy(ddm_event_t ev) {
    return ddm::hip_status(hipEventDestroy(reinterpret_cast<hipEvent_t>(ev)), "ddm_event_destroy");
}

extern "C" int ddm_event_record(ddm_event_t ev, ddm_stream_t stream) {
    return ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev), ddm::as_hip(stream)), "ddm_event_record");
}

extern "C" int ddm_event_synchronize(ddm_event_t ev) {
    return ddm::hip_status(hipEventSynchronize(reinterpret_cast<hipEvent_t>(ev)), "ddm_event_synchronize");
}

extern "C" int ddm_event_elapsed_ms(ddm_event_t begin, ddm_event_t end, float* ms) {
    if (!ms) return DDM_E_ARG;
    return ddm::hip_status(hipEventElapsedTime(ms, reinterpret_cast<hipEvent_t>(begin), reinterpret_cast<hipEvent_t>(end)),
                           "ddm_event_elapsed_ms");
}

// ABI 22: a stream whose kernels run on a subset of the device's CUs (hipExtStreamCreateWithCUMask):
// CU i is in the mask when i % stride == offset % stride (stride 1: every CU).  The runner's
// side stream takes the next windows' shuffles off the CUs the epoch stream's predict needs.
extern "C" int ddm_stream_create_cu_stride(int32_t stride, int32_t offset, ddm_stream_t* out, int32_t* n_cus) {
    if (!out || stride < 1) {
        ddm::set_error("ddm_stream_create_cu_stride: invalid argument");
        return DDM_E_ARG;
    }
    int dev = 0, cus = 0;
    if (int rc = ddm::hip_status(hipGetDevice(&dev), "ddm_stream_create_cu_stride")) return rc;
    if (int rc = ddm::hip_status(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev),
                                 "ddm_stream_create_cu_stride"))
        return rc;
    const int words = (cus + 31) / 32;
    uint32_t mask[64] = {0};
    if (words > 64) {
        ddm::set_error("ddm_stream_create_cu_stride: %d CUs", cus);
        return DDM_E_ARG;
    }
    int n = 0;
    for (int i = 0; i < cus; ++i)
        if (i % stride == offset % stride) {
            mask[i / 32] |= 1u << (i % 32);
            ++n;
        }
    hipStream_t st;
    if (int rc = ddm::hip_status(hipExtStreamCreateWithCUMask(&st, (uint32_t)words, mask), "hipExtStreamCreateWithCUMask"))
        return rc;
    *out = reinterpret_cast<ddm_stream_t>(st);
    if (n_cus) *n_cus = n;
    return 0;
}

// ABI 22: the CU mask a stream runs with (words of 32 CUs, n_words at most 64); *n_cus its CU count.
extern "C" int ddm_stream_cu_count(ddm_stream_t stream, int32_t* n_cus) {
    if (!n_cus) return DDM_E_ARG;
    uint32_t mask[64] = {0};
    if (int rc = ddm::hip_status(hipExtStreamGetCUMask(ddm::as_hip(stream), 64, mask), "hipExtStreamGetCUMask"))
        return rc;
    int n = 0;
    for (int k = 0; k < 64; ++k) n += __builtin_popcount(mask[k]);
    *n_cus = n;
    return 0;
}

extern "C" int ddm_stream_destroy(ddm_stream_t stream) {
    return ddm::hip_status(hipStreamDestroy(ddm::as_hip(stream)), "ddm_stream_destroy");
}
