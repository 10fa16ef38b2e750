// Launch timing of the hot kernels with HIP events (bench.py's roofline): when
// a channel is enabled, every ``every``-th launch of that channel's kernel is
// timed by two events on the stream it is launched on.  Channels:
//   0  the sum-forward composite (every rasterizer entry point)
//   1  train_tile_kernel   (the fused training step's per-tile kernel)
//   2  frame_project_kernel (render and training projection + slab insertion)
//   3  train_splat_kernel  (projection VJP + Adan)
//   4  raster_sum_bwd_kernel (the op path's sum backward)
//   5  raster_alpha_fwd_kernel, 6 raster_alpha_bwd_kernel (the alpha path)
// Two ways (gsvc_timing_enable's ``how``):
//   0  marker events recorded before and after the launch (hipEventRecord):
//      includes the marker packets' latency and the kernel's dispatch, ~3 us
//   1  the launch itself carries the events (hipExtLaunchKernel): the
//      dispatch packet's own start / end timestamps, as rocprofv3's kernel trace
#include <mutex>
#include <vector>

#include "common.h"

namespace gsvc {

namespace {
struct Channel {
    std::vector<hipEvent_t> ev;  // pairs
    int every = 1, calls = 0, used = 0, how = 0;
};
std::mutex g_tmu;
Channel g_ch[kTimingChannels];

void channel_free(Channel &c) {
    for (hipEvent_t e : c.ev) hipEventDestroy(e);
    c.ev.clear();
    c.calls = c.used = 0;
}
}  // namespace

int timing_begin(hipStream_t s, hipEvent_t *dispatch_ev, int channel) {
    dispatch_ev[0] = dispatch_ev[1] = nullptr;
    if (channel < 0 || channel >= kTimingChannels) return -1;
    std::lock_guard<std::mutex> lk(g_tmu);
    Channel &c = g_ch[channel];
    if (c.ev.empty()) return -1;
    if ((c.calls++) % c.every) return -1;
    if (2 * (c.used + 1) > (int)c.ev.size()) return -1;
    const int slot = c.used++;
    if (c.how == 1) {
        dispatch_ev[0] = c.ev[2 * slot];
        dispatch_ev[1] = c.ev[2 * slot + 1];
    } else {
        hipEventRecord(c.ev[2 * slot], s);
    }
    return slot;
}

void timing_end(hipStream_t s, int slot, int channel) {
    if (slot < 0 || channel < 0 || channel >= kTimingChannels) return;
    std::lock_guard<std::mutex> lk(g_tmu);
    Channel &c = g_ch[channel];
    if (c.how != 1) hipEventRecord(c.ev[2 * slot + 1], s);
}

}  // namespace gsvc

using namespace gsvc;

extern "C" int gsvc_timing_enable_channel(int channel, int max_launches, int every, int how) {
    if (channel < 0 || channel >= kTimingChannels)
        return set_error(GSVC_ERR_ARG, "timing_enable: channel must be 0..%d", kTimingChannels - 1);
    std::lock_guard<std::mutex> lk(g_tmu);
    Channel &c = g_ch[channel];
    channel_free(c);
    if (max_launches <= 0) return GSVC_OK;
    if (how != 0 && how != 1) return set_error(GSVC_ERR_ARG, "timing_enable: how must be 0 or 1");
    c.every = every > 0 ? every : 1;
    c.how = how;
    c.ev.resize(2 * (size_t)max_launches);
    for (hipEvent_t &e : c.ev)
        if (hipEventCreate(&e) != hipSuccess) {
            c.ev.clear();
            return set_error(GSVC_ERR_HIP, "timing_enable: hipEventCreate failed");
        }
    return GSVC_OK;
}

extern "C" int gsvc_timing_collect_channel(int channel, float *ms, int max_out, int *count) {
    if (channel < 0 || channel >= kTimingChannels)
        return set_error(GSVC_ERR_ARG, "timing_collect: channel must be 0..%d", kTimingChannels - 1);
    std::lock_guard<std::mutex> lk(g_tmu);
    Channel &c = g_ch[channel];
    int k = 0;
    for (int i = 0; i < c.used && k < max_out; ++i) {
        if (hipEventSynchronize(c.ev[2 * i + 1]) != hipSuccess ||
            hipEventElapsedTime(&ms[k], c.ev[2 * i], c.ev[2 * i + 1]) != hipSuccess)
            return set_error(GSVC_ERR_HIP, "timing_collect: event query failed");
        ++k;
    }
    *count = k;
    return GSVC_OK;
}

extern "C" int gsvc_timing_enable(int max_launches, int every, int how) {
    return gsvc_timing_enable_channel(kTimingComposite, max_launches, every, how);
}

extern "C" int gsvc_timing_collect(float *ms, int max_out, int *count) {
    return gsvc_timing_collect_channel(kTimingComposite, ms, max_out, count);
}
