// Frame-path pieces shared by frame.hip (the one-call render) and train.hip
// (the fused training step): the workspace layout and the projection kernel
// that fills the per-tile record slabs.
#pragma once

#include "common.h"

namespace gsvc {

inline size_t ws_align(size_t x) { return (x + 255) & ~(size_t)255; }

inline int tiles_of(unsigned h, unsigned w) {
    return ceil_div((int)w, kTile) * ceil_div((int)h, kTile);
}

// Workspace of one frame model (base NULL: sizes only).  The first ``zeroed``
// bytes (counts[2][T] and the two M slots) must be zero before the first call;
// every call leaves them zero.
struct FrameWs {
    unsigned *counts;  // [2][T]: this frame's and the next frame's
    int *m_slots;      // [2]
    float4 *slab;      // [T][256][3] splat records
    float2 *xys;       // [N]
    int *radii;        // [N]
    float4 *rec;       // [N][3] splat records
    size_t zeroed, bytes;
};
FrameWs frame_ws(char *base, int n, int ntiles);

// Frame f counts into parity f & 1 while its consumer clears the other parity.
struct FrameSlots {
    unsigned *counts, *counts_next;
    int *m_acc, *m_clear;
};
FrameSlots frame_slots(const FrameWs &w, int ntiles, int frame_index);

// Activations + projection of every splat, its 48-byte record
//   {x, y, a/2, b}, {c/2, opacity, r, g}, {b, id bits, a, c}
// and its insertion into the 256-slot slab of every tile it touches; this
// frame's M into f.m_acc.  grad_zero (optional): [N][4] float4 gradient
// records zeroed for the consumer's atomics.
int frame_project_launch(int n, const float *xyz, int xyz_tanh, const float *chol,
                         const float *chol_bound, const float *feat, const float *rgb_w,
                         const float *opac, unsigned img_h, unsigned img_w, const FrameWs &w,
                         const FrameSlots &f, float4 *grad_zero, hipStream_t s);

}  // namespace gsvc
