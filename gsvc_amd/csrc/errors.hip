// Error reporting of the C ABI: a per-thread message for gsvc_last_error().
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace gsvc {

static thread_local char g_last_error[512] = "";

int set_error(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
    va_end(ap);
    return code;
}

int check_launch(const char *what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(GSVC_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
    return GSVC_OK;
}

int g_knobs[kKnobs] = {};
void *g_debug_ptr = nullptr;

}  // namespace gsvc

extern "C" int gsvc_abi_version(void) { return 1; }

extern "C" int gsvc_debug_set(int key, int value) {
    if (key < 0 || key >= gsvc::kKnobs) return -1;
    const int old = gsvc::g_knobs[key];
    gsvc::g_knobs[key] = value;
    return old;
}

extern "C" void gsvc_debug_set_ptr(void *p) { gsvc::g_debug_ptr = p; }

extern "C" const char *gsvc_last_error(void) { return gsvc::g_last_error; }

extern "C" int gsvc_stream_sync(void *stream) {
    const hipError_t e = hipStreamSynchronize((hipStream_t)stream);
    if (e != hipSuccess)
        return gsvc::set_error(GSVC_ERR_HIP, "stream_sync: %s", hipGetErrorString(e));
    return GSVC_OK;
}
