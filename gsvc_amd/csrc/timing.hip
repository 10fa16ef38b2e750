// Launch timing of the composite kernel with HIP events (bench.py's roofline):
// when enabled, every ``every``-th sum-forward launch is timed by two events on
// the stream it is launched on.  Two ways (gsvc_timing_enable's ``how``):
//   0  marker events recorded before and after the launch (hipEventRecord):
//      includes the marker packets' latency and the kernel's dispatch, ~3 us
//   1  the launch itself carries the events (hipExtLaunchKernel): the
//      dispatch packet's own start / end timestamps, as rocprofv3's kernel trace
#include <mutex>
#include <vector>

#include "common.h"

namespace gsvc {

static std::mutex g_tmu;
static std::vector<hipEvent_t> g_tev;  // pairs
static int g_tevery = 1, g_tcalls = 0, g_tused = 0, g_thow = 0;

int timing_begin(hipStream_t s, hipEvent_t *dispatch_ev) {
    dispatch_ev[0] = dispatch_ev[1] = nullptr;
    std::lock_guard<std::mutex> lk(g_tmu);
    if (g_tev.empty()) return -1;
    if ((g_tcalls++) % g_tevery) return -1;
    if (2 * (g_tused + 1) > (int)g_tev.size()) return -1;
    const int slot = g_tused++;
    if (g_thow == 1) {
        dispatch_ev[0] = g_tev[2 * slot];
        dispatch_ev[1] = g_tev[2 * slot + 1];
    } else {
        hipEventRecord(g_tev[2 * slot], s);
    }
    return slot;
}

void timing_end(hipStream_t s, int slot) {
    if (slot < 0) return;
    std::lock_guard<std::mutex> lk(g_tmu);
    if (g_thow != 1) hipEventRecord(g_tev[2 * slot + 1], s);
}

static void timing_free() {
    for (hipEvent_t e : g_tev) hipEventDestroy(e);
    g_tev.clear();
    g_tcalls = g_tused = 0;
}

}  // namespace gsvc

using namespace gsvc;

extern "C" int gsvc_timing_enable(int max_launches, int every, int how) {
    std::lock_guard<std::mutex> lk(g_tmu);
    timing_free();
    if (max_launches <= 0) return GSVC_OK;
    if (how != 0 && how != 1) return set_error(GSVC_ERR_ARG, "timing_enable: how must be 0 or 1");
    g_tevery = every > 0 ? every : 1;
    g_thow = how;
    g_tev.resize(2 * (size_t)max_launches);
    for (hipEvent_t &e : g_tev)
        if (hipEventCreate(&e) != hipSuccess) {
            g_tev.clear();
            return set_error(GSVC_ERR_HIP, "timing_enable: hipEventCreate failed");
        }
    return GSVC_OK;
}

extern "C" int gsvc_timing_collect(float *ms, int max_out, int *count) {
    std::lock_guard<std::mutex> lk(g_tmu);
    int k = 0;
    for (int i = 0; i < g_tused && k < max_out; ++i) {
        if (hipEventSynchronize(g_tev[2 * i + 1]) != hipSuccess ||
            hipEventElapsedTime(&ms[k], g_tev[2 * i], g_tev[2 * i + 1]) != hipSuccess)
            return set_error(GSVC_ERR_HIP, "timing_collect: event query failed");
        ++k;
    }
    *count = k;
    return GSVC_OK;
}
