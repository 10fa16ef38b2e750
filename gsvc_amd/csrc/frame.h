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

// Per frame, the slab region is a dense head [T][kHeadSlots][3] float4 (the
// first slots of every tile: what the consumers load with the count -- 3 MB
// at 1080p, so a batch of frames touches few pages for them) followed by the
// body [T][256][3] (slots from kHeadSlots on, at their slot index).
constexpr int kHeadSlots = 8;
// (a render's id slabs use the same memory: kCarryCap ids per tile)
static_assert(4 * kCarryCap <= 16 * 3 * (kHeadSlots + kTilePix), "id slabs exceed the slab memory");
__host__ __device__ inline size_t slab_frame_f4(int ntiles) {
    return (size_t)3 * (kHeadSlots + kTilePix) * (size_t)ntiles;
}
// Record of slot s of tile t in a frame's slab region.
__host__ __device__ inline float4 *slab_rec(float4 *slab, int ntiles, int tile, int s) {
    return s < kHeadSlots ? slab + ((size_t)tile * kHeadSlots + s) * 3
                          : slab + (size_t)3 * kHeadSlots * ntiles + ((size_t)tile * kTilePix + s) * 3;
}
__host__ __device__ inline const float4 *slab_rec(const float4 *slab, int ntiles, int tile, int s) {
    return slab_rec(const_cast<float4 *>(slab), ntiles, tile, s);
}

// Workspace of F frame models rendered together (base NULL: sizes only).  The
// first ``zeroed`` bytes (counts and M slots) must be zero before the first
// call; every call leaves them zero.
struct FrameWs {
    unsigned *counts;  // [F][2][T]: per frame, this call's and the next call's
    int *m_slots;      // [F][2]
    float4 *slab;      // [F] x (head [T][kHeadSlots][3] + body [T][256][3]) splat records
    int *ovf;          // [F][T][kOvfSlots]: the ids of record-slab slots 256 .. kCarryCap - 1
    float2 *xys;       // [N] (N = splats of all F frames)
    int *radii;        // [N]
    float4 *rec;       // [N][3] splat records
    // single frame only (F = 1): the splat order (SplatOrder) -- strip keys and
    // ids written by a refreshing call's projection, radix-sorted into order
    unsigned *okey, *skey, *kbuf, *sort_counts, *sort_offsets;
    int *okey_id, *order, *vbuf;
    size_t zeroed, bytes;
};
FrameWs frame_ws(char *base, int n, int ntiles, int frames = 1);

// Call f counts into parity f & 1 while its consumer clears the other parity
// (pointers of frame 0; frame b's are counts_stride / m_stride further).
struct FrameSlots {
    unsigned *counts, *counts_next;
    int *m_acc, *m_clear;
    int counts_stride, m_stride;
};
FrameSlots frame_slots(const FrameWs &w, int ntiles, int frame_index);

// Activations + projection of every splat, its 48-byte record
//   {x, y, a/2, b}, {c/2, opacity, r, g}, {b, id bits, a, c}
// and its insertion into the 256-slot slab of every tile it touches; this
// frame's M into f.m_acc.  grad_zero (optional): [N][4] float4 gradient
// records zeroed for the consumer's atomics.
// frames > 1: the splats of frame b are [frame_off[b], frame_off[b + 1]) of
// the n (device array frame_off) and max_frame_n is the largest frame.
// ord (single frame only): lane t projects splat ord->order[t] (NULL:
// identity) and the workgroup aggregates its slot atomics per tile (the same
// entries per tile); ord->key / key_id (optional): every splat's strip key and
// id, the input of the next order's sort (frame.hip strip_key).
// carry_ids (optional, the training step's carried bins, train.hip): the
// insertion writes splat ids into carry_ids[T][256] counted in carry_counts
// instead of records into the slab, and every splat's tile box into
// carry_box and carry_hull.
struct SplatOrder {
    const int *order = nullptr;
    unsigned *key = nullptr;
    int *key_id = nullptr;
    int *carry_ids = nullptr;
    unsigned *carry_counts = nullptr;
    uint2 *carry_box = nullptr, *carry_hull = nullptr;
};
int frame_project_launch(int n, const float *xyz, int xyz_tanh, const float *chol,
                         const float *chol_bound, const float *feat, const float *rgb_w,
                         const float *opac, unsigned img_h, unsigned img_w, const FrameWs &w,
                         const FrameSlots &f, float4 *grad_zero, hipStream_t s, int frames = 1,
                         const int *frame_off = nullptr, int max_frame_n = 0,
                         const SplatOrder *ord = nullptr, int *id_slab = nullptr);
// Bits of the strip keys at this image size (invisible splats: the largest).
int strip_key_bits(int tbx, int tby);
// Sort the keys a refreshing projection wrote into w.order (F = 1 workspaces).
int splat_order_sort(const FrameWs &w, int n, int tbx, int tby, hipStream_t s);

}  // namespace gsvc
