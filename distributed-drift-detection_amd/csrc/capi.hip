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
