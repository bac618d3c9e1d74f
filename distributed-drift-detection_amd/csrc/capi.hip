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
