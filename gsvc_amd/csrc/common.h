// Shared device helpers for the gfx950 kernels of gsvc_amd.
//
// Floating-point contract: the library is compiled with
// -ffp-contract=off, so every fused multiply-add below is an explicit fmaf();
// division and sqrt are IEEE; exp(-s) is v_exp_f32(s * -log2(e)).  The CPU
// oracle (oracle/oracle.c) follows the same op sequence.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gsvc_amd.h"

namespace gsvc {

constexpr int kTile = 16;          // BLOCK_X = BLOCK_Y (reference config.h:1-2)
constexpr int kTilePix = 256;      // BLOCK_SIZE (config.h:3): entries blended per tile
// The training step's carried candidate lists (GSVC_TRAIN_CARRY): slots per
// tile.  A tile of more than 256 candidates (dense content: the textured video
// stand-in passes 256 entries per tile after ~40 frames of training) sorts its
// members from this list; only past kCarryCap does it rebuild from every
// splat's bbox (tile_ids.h wave_brute_ids).
constexpr int kCarryCap = 1024;
// The training step's own carried lists hold kTrainCarryCap candidates per tile
// (134 MB at 1080p -- a few per mille of a 288 GB HBM stack): a tile of up to
// 4096 candidates, 16x the 256 entries the rasterizer blends, sorts its
// members from the list (cost by its candidates, not by every splat), so the
// bbox rebuild over all splats is left for tiles denser than that (VERDICT r5
// item 8: the textured stand-in had passed 1024 on its densest frames' way).
constexpr int kTrainCarryCap = 4096;
// The record slabs (frame path) keep a tile's slots [256, kCarryCap) as ids in
// an overflow area of kOvfSlots per tile: a tile of up to kCarryCap entries
// sorts its ids from the slab and the area instead of the bbox rebuild.
constexpr int kOvfSlots = kCarryCap - kTilePix;
static_assert(kCarryCap == GSVC_SLABS_WIDE_IDS, "include/gsvc_amd.h GSVC_SLABS_WIDE_IDS");
constexpr float kNegLog2e = -1.4426950408889634f;
constexpr float kAlphaMin = 1.0f / 255.0f;
// At unit opacity the reference's alpha cut (forward.cu:598-606:
// !(sigma < 0) && !(min(1, exp(-sigma)) < 1/255)) keeps exactly the sigma
// whose float bits lie in [0, kSigmaCutBits], and exp(-sigma) <= 1 there
// (alpha_cut.hip proves both on the device over every float; a NaN sigma is
// the exception -- see there).  The constant needs no runtime check: the
// library carries gfx950 code objects only (build.py: --offload-arch=gfx950,
// no other target), so its kernels cannot launch on a device whose exp was
// not the one scanned; the GPU suite re-runs the scan on every box.
constexpr unsigned kSigmaCutBits = 0x40b15208u;  // sigma 5.5412636 (gfx950 v_exp_f32, tests/test_alpha_cut.py)

// Host-side error plumbing -------------------------------------------------
int set_error(int code, const char *fmt, ...);
int check_launch(const char *what);
// GSVC_ERR_CAPTURE when stream s is capturing a graph (entries with host-indexed
// workspace parity; include/gsvc_amd.h conventions), else GSVC_OK
int refuse_capture(hipStream_t s, const char *what);
// hipMemsetAsync(p, 0, bytes, s) / a device-to-device hipMemcpyAsync as one
// kernel of this library (errors.hip): the HIP runtime torch loads (ROCm 7.0)
// replays graph-captured memset nodes wrongly once other work has run on the
// stream (tools/capture_debug.py), so the library's own zeroing and copies are
// kernels, which capture and replay like the rest.  Returns a gsvc status.
int dev_zero(void *p, size_t bytes, hipStream_t s);
int dev_copy(void *dst, const void *src, size_t bytes, hipStream_t s);
// A/B knobs and diagnostic kernel variants exist only in the diagnostic
// library (built with -DGSVC_DIAG: libgsvc_amd_diag.so, include/gsvc_amd_diag.h,
// for tools/ and the variant-comparison tests).  In the product library every
// knob is the constant 0 -- the production choice -- and the diagnostic
// variants are not compiled (``if constexpr (kDiag)`` around their launches).
constexpr int kKnobs = 40;
#ifdef GSVC_DIAG
constexpr bool kDiag = true;
extern int g_knobs[kKnobs];  // gsvc_debug_set(); knob 0 = sum-forward variant, 8 = training tile kernel
extern void *g_debug_ptr;    // gsvc_debug_set_ptr(): diagnostic output buffer
inline int knob(int k) { return g_knobs[k]; }
inline void *debug_ptr() { return g_debug_ptr; }
#else
constexpr bool kDiag = false;
constexpr int knob(int) { return 0; }
constexpr void *debug_ptr() { return nullptr; }
#endif
// timing.hip: slot, or -1 when not recording; dispatch_ev[2] = the events the
// launch must carry itself (hipExtLaunchKernel), both null otherwise
constexpr int kTimingComposite = 0, kTimingTrainTile = 1, kTimingProject = 2,
              kTimingTrainSplat = 3, kTimingSumBwd = 4, kTimingAlphaFwd = 5, kTimingAlphaBwd = 6,
              kTimingChannels = 7;
int timing_begin(hipStream_t s, hipEvent_t *dispatch_ev, int channel = kTimingComposite);
void timing_end(hipStream_t s, int slot, int channel = kTimingComposite);

// A launch that carries its timing events when tev[0] is set (timing.hip,
// how = 1), a plain launch otherwise.
template <typename K, typename... Args>
inline void launch_timed(K kernel, dim3 grid, dim3 block, size_t lds, hipStream_t s,
                         const hipEvent_t *tev, Args... args) {
    if (tev[0])
        hipExtLaunchKernelGGL(kernel, grid, block, lds, s, tev[0], tev[1], 0, args...);
    else
        hipLaunchKernelGGL(kernel, grid, block, lds, s, args...);
}

// XCD-aware block -> work-item remap.  Blocks b and b+8 share an XCD (they are
// dealt round-robin over the 8 XCDs), so give each XCD a contiguous range of
// tiles: neighbouring tiles share splats, which then hit the same L2.  Speed
// only; any placement gives the same results.  Bijective for any count
// (cdna_hip_programming.md §5, "XCD swizzle must be bijective").
__device__ __forceinline__ int xcd_remap(int orig, int count) {
    const int q = count >> 3, r = count & 7, xcd = orig & 7;
    const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + (orig >> 3);
}

// XCD-balanced variant: runs of kRun consecutive tiles (a strip of a tile row)
// dealt round-robin over the XCDs, so a dense region of the frame spreads over
// all eight while each run still shares its splats in one L2.  Blocks past the
// last whole round of 8 runs map to themselves (bijective for any count).
template <int kRun>
__device__ __forceinline__ int xcd_runs(int orig, int count) {
    constexpr int kGroup = 8 * kRun;
    const int full = (count / kGroup) * kGroup;
    if (orig >= full) return orig;
    const int xcd = orig & 7, s = orig >> 3;
    return ((s / kRun) * 8 + xcd) * kRun + (s % kRun);
}

// v_cvt_i32_f32 semantics: truncate, saturate, NaN -> 0.
// 16-byte write-through store (sc1: agent scope): the line leaves the XCD's L2
// as it is written, so the end-of-kernel release has no dirty line of it to
// write back; for data the NEXT kernel reads from other XCDs (MI355X_MICROARCH
// "publish-large").  A vector store; never a scalar-cache one.
__device__ __forceinline__ void store_wt(float4 *p, float4 v) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const f4 x = {v.x, v.y, v.z, v.w};
    // s_nop 1: the gfx940+ store-data hazard (raster_sum.hip st_f4)
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(x) : "memory");
}

__device__ __forceinline__ int cvt_i32(float f) {
    if (f != f) return 0;
    if (f >= 2147483648.0f) return 2147483647;
    if (f <= -2147483648.0f) return (-2147483647 - 1);
    return (int)f;
}

// helpers.cuh:11-43: tile bbox of a splat, [min, max) in tile units, clamped.
__device__ __forceinline__ void tile_bbox(float cx, float cy, float radius, int tbx, int tby,
                                          unsigned &x0, unsigned &y0, unsigned &x1, unsigned &y1) {
    const float tcx = cx / (float)kTile, tcy = cy / (float)kTile;
    const float tr = radius / (float)kTile;
    int a;
    a = cvt_i32(tcx - tr);          x0 = min((unsigned)max(a, 0), (unsigned)tbx);
    a = cvt_i32((tcx + tr) + 1.0f); x1 = min((unsigned)max(a, 0), (unsigned)tbx);
    a = cvt_i32(tcy - tr);          y0 = min((unsigned)max(a, 0), (unsigned)tby);
    a = cvt_i32((tcy + tr) + 1.0f); y1 = min((unsigned)max(a, 0), (unsigned)tby);
}

// sigma of forward.cu:595-597 in the build's fixed op order.
__device__ __forceinline__ float splat_sigma_h(float ha, float b, float hc, float dx, float dy) {
    const float cq = (hc * dy) * dy;
    const float bdy = b * dy;
    const float q = fmaf(ha, dx, bdy);
    return fmaf(q, dx, cq);
}

__device__ __forceinline__ float exp_neg(float s) {
    return __builtin_amdgcn_exp2f(s * kNegLog2e);
}

__host__ __device__ __forceinline__ int ceil_div(int a, int b) { return (a + b - 1) / b; }

}  // namespace gsvc
