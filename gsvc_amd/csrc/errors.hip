// Error reporting of the C ABI: a per-thread message for gsvc_last_error().
#include <immintrin.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <chrono>

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

int refuse_capture(hipStream_t s, const char *what) {
    // the legacy default stream cannot capture; asking HIP about it costs a
    // device-wide wait (measured: op-path forward 77 -> 113 us)
    if (s == nullptr) return GSVC_OK;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    // (a failing query -- e.g. no device -- is left to the launches to report)
    if (hipStreamIsCapturing(s, &st) != hipSuccess || st == hipStreamCaptureStatusNone) return GSVC_OK;
    return set_error(GSVC_ERR_CAPTURE,
                     "%s cannot be captured in a graph: its workspace alternates parity slots indexed "
                     "by the host's call counter, which a replay would not advance", what);
}

namespace {
// 16-byte chunks where both ends allow it, bytes otherwise (grid-stride)
__global__ __launch_bounds__(256) void fill_kernel(unsigned char *__restrict__ dst,
                                                   const unsigned char *__restrict__ src,
                                                   size_t bytes) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const size_t t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool v16 = (((uintptr_t)dst | (uintptr_t)src) & 15u) == 0;
    const size_t n16 = v16 ? bytes / 16 : 0;
    for (size_t i = t0; i < n16; i += stride)
        reinterpret_cast<uint4 *>(dst)[i] =
            src ? reinterpret_cast<const uint4 *>(src)[i] : make_uint4(0u, 0u, 0u, 0u);
    for (size_t i = 16 * n16 + t0; i < bytes; i += stride) dst[i] = src ? src[i] : (unsigned char)0;
}

int fill_launch(void *dst, const void *src, size_t bytes, hipStream_t s, const char *what) {
    if (bytes == 0) return GSVC_OK;
    const size_t chunks = (bytes + 15) / 16;
    const unsigned grid = (unsigned)(chunks / 256 + 1 < 4096 ? chunks / 256 + 1 : 4096);
    hipLaunchKernelGGL(fill_kernel, dim3(grid), dim3(256), 0, s, (unsigned char *)dst,
                       (const unsigned char *)src, bytes);
    return check_launch(what);
}
}  // namespace

int dev_zero(void *p, size_t bytes, hipStream_t s) { return fill_launch(p, nullptr, bytes, s, "zero fill"); }
int dev_copy(void *dst, const void *src, size_t bytes, hipStream_t s) {
    return fill_launch(dst, src, bytes, s, "device copy");
}

#ifdef GSVC_DIAG
int g_knobs[kKnobs] = {};
void *g_debug_ptr = nullptr;
#endif

}  // namespace gsvc

extern "C" int gsvc_abi_version(void) { return GSVC_ABI_VERSION; }

#ifdef GSVC_DIAG
// include/gsvc_amd_diag.h: the diagnostic library only
extern "C" int gsvc_debug_set(int key, int value) {
    if (key < 0 || key >= gsvc::kKnobs) return -1;
    const int old = gsvc::g_knobs[key];
    gsvc::g_knobs[key] = value;
    return old;
}

extern "C" void gsvc_debug_set_ptr(void *p) { gsvc::g_debug_ptr = p; }
#endif

extern "C" const char *gsvc_last_error(void) { return gsvc::g_last_error; }

extern "C" int gsvc_stream_sync(void *stream) {
    const hipError_t e = hipStreamSynchronize((hipStream_t)stream);
    if (e != hipSuccess)
        return gsvc::set_error(GSVC_ERR_HIP, "stream_sync: %s", hipGetErrorString(e));
    return GSVC_OK;
}

extern "C" void *gsvc_host_alloc(size_t bytes) {
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocCoherent) != hipSuccess) {
        gsvc::set_error(GSVC_ERR_HIP, "host_alloc: hipHostMalloc(%zu) failed", bytes);
        return nullptr;
    }
    memset(p, 0, bytes);
    return p;
}

extern "C" int gsvc_host_free(void *p) {
    if (p && hipHostFree(p) != hipSuccess) return gsvc::set_error(GSVC_ERR_HIP, "host_free failed");
    return GSVC_OK;
}

// Spin on a word of coherent host memory until a kernel has stored ``seq``
// into it (system-scope release: everything the kernel stored before it is
// visible).  After ``spin_us`` without it, wait for the whole stream instead,
// which also reports a failed kernel; the word must then hold ``seq``.
extern "C" int gsvc_wait_host_seq(const unsigned *word, unsigned seq, void *stream, int spin_us) {
    if (!word) return gsvc::set_error(GSVC_ERR_ARG, "wait_host_seq: null word");
    const volatile unsigned *w = word;
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 1;; ++it) {
        if (*w == seq) {
            std::atomic_thread_fence(std::memory_order_acquire);
            return GSVC_OK;
        }
        _mm_pause();
        if ((it & 255u) == 0 &&
            std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us))
            break;
    }
    const int rc = gsvc_stream_sync(stream);
    if (rc) return rc;
    if (*w != seq)
        return gsvc::set_error(GSVC_ERR_HIP, "wait_host_seq: the stream finished without storing %u (word %u)",
                               seq, *w);
    std::atomic_thread_fence(std::memory_order_acquire);
    return GSVC_OK;
}
