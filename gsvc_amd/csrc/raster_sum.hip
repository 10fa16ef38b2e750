// Sum rasterizer of GSVC (rasterize_gaussians_sum), forward and backward, gfx950.
//
// Reference: gsplat/gsplat/cuda/csrc/forward.cu:512-627 (rasterize_forward_sum),
// backward.cu:696-862 (rasterize_backward_sum_kernel), bindings.cu:400-469,
// 706-779; Python glue rasterize_sum.py:92-254.
//
// Semantics kept from the reference: out = sum of
// colour * min(1, opacity * exp(-sigma)) over the FIRST <= 256 sorted entries
// of the pixel's tile (the reference breaks after one 256-entry batch,
// forward.cu:569-571,613), skipping sigma < 0 and alpha < 1/255; no
// transmittance, no background; final_idx = last contributing sorted index,
// 0 if none; final_Ts = 1.
//
// Forward layout: a 128-thread workgroup (2 waves) per 16x16
// tile, chosen per tile from its entry count n:
//   * sparse tile (n <= threshold, default 8): wave 0 blends the whole tile,
//     each lane owning 4 consecutive pixels of one row; entries are gathered
//     64 at a time into LDS (lane = entry) and broadcast to the wave; the row
//     terms of sigma are shared by the lane's 4 pixels; wave 1 exits;
//   * dense tile: each wave owns one 8-row band, 2 pixels per lane; per chunk
//     of 64 entries each lane gathers one entry and tests whether its
//     alpha >= 1/255 ellipse can reach the band at all (a conservative bbox
//     test); survivors are compacted (ballot + popcount) into LDS in sorted
//     order and blended with packed f32 math.  About half of the
//     (entry, band) pairs are culled at 50k splats; a culled pair contributes
//     nothing in the reference either, so results are identical.
// Output: RGB staged through LDS and written as whole 192-byte tile rows;
// final_idx as 16- or 8-byte groups.  The kernel is bound by the 16 B/pixel of
// output plus the VALU of the surviving (pixel, entry) pairs (see the
// timestamp and ablation measurements in DESIGN.md §5).
//
// Backward layout: one 256-thread workgroup per tile, ENTRY-parallel: with
// n entries (E = next pow2 >= n) thread t handles entry t % E against the
// pixels [E*(t/E), E*(t/E)+E) of the tile, so gradients accumulate in
// registers without a per-pixel reduction; the t/E groups are combined once
// per entry (shuffles + LDS), then one 64-byte-aligned 9-float record per
// (splat, tile) is added with 9 lanes of one atomic instruction (one memory
// request per entry instead of the reference's 9 per warp).
#include <hip/hip_ext.h>

#include <type_traits>

#include "cull.h"
#include "det.h"
#include "frame.h"
#include "frame_dev.h"
#include "raster_sum.h"
#include "rows.h"
#include "tile_ids.h"

namespace gsvc {

constexpr int kChunk = 64;
// Frame path: the first spec_slots (<= kHeadSlots) slab records are loaded in
// the count's round trip (speculatively: most tiles have that few); slot j of a
// tile is in its head (j < kHeadSlots) or at index j of its body.
__device__ __forceinline__ const float4 *slot_rec(const float4 *head, const float4 *body, int j) {
    return j < kHeadSlots ? head + 3 * j : body + 3 * j;
}
constexpr int kSlice = 220;  // float4s of LDS per wave (3.4 KB; sum_fwd_sparse's layout)

// Forward kernel modes.  Production: the launcher picks kModeSparse (one wave
// per tile) when the frame averages <= 8 entries per tile and kModeBanded
// (two waves per tile) above, from the intersection count the caller already
// holds (gsvc_rasterize_sum_forward_auto).  gsvc_debug_set(0, mode) forces a
// mode for tools/kbench.py:
//   1 sparse path only     2 banded path only
//   3 per-tile choice (2 waves per tile) with timestamps (diagnostic)
//   4 banded, no blending  5 banded, no stores   (ablations)
//   6 per-tile choice (2 waves per tile; threshold gsvc_debug_set(3, t))
//   7 sparse path with 4 timestamps per tile (start, staged, blended, stores
//     drained) into the buffer of gsvc_debug_set_ptr (diagnostic)
// A per-tile choice inside one launch was measured slower than either pure
// mode: a 128-thread workgroup whose second wave exits at once still halves
// the dispatch rate of sparse tiles.
enum { kModeAdaptive = 6, kModeSparse = 1, kModeBanded = 2, kModeStamp = 3, kModeNoBlend = 4,
       kModeNoStore = 5, kModeSparseStamp = 7, kModeSparsePrio = 8, kModeSparseIds = 9 };
// kModeSparseIds: kModeSparse over 4-byte id slabs (A.id_counts / A.ids_rw, the
// entries' records gathered by id from A.rec): the single-frame render -- its
// projection appends ids instead of 48-byte records (trained 1080p / 50k:
// projection 14.9 -> 10.5 us, composite 20.7 -> 21.4, frame 25.8k -> 28.8k fps;
// 10k equal; profiles/r04/id_slabs/).  A/B knob 24 = 1 restores the records.
// kModeSparsePrio: kModeSparse with the wave priority raised over the staging
// (s_setprio 3 until the blend; A/B knob 17 = 1 selects it for the sparse launches)
// Banded (two waves per tile) only past this many entries per tile on average.
// Measured with the lane-group lists (1080p, tools/fbench.py, profiles/r02/composite_modes/):
// sparse wins from 3 to 62 entries per tile (trained 50k, 28 per tile: 43.0 vs 48.0 us per
// frame; 62 per tile: 82.1 vs 93.8) and ties at 107 (138.4 vs 137.2).
constexpr int kDenseEntriesPerTile = 96;
// A sparse tile's chunk of at most this many entries is blended by every lane
// without the lane-group lists (A/B knob 15 = v > 0 sets it to v - 1).
constexpr int kGroupMinDefault = 24;

// Diagnostic only (kModeStamp): s_memrealtime (100 MHz) stamps per tile,
// written to the final_Ts slot reinterpreted as int64[ntiles][4].
__device__ __forceinline__ long long stamp() {
    long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

typedef float v2f __attribute__((ext_vector_type(2)));

// Diagnostic library only: the id-slab render's phases stamped per tile when
// A.stamps is set (knob 39 = 1 with gsvc_debug_set_ptr; int64[ntiles][8]: start,
// ids arrived, staged, blended, stores drained, entry count)
template <int kMode>
constexpr bool kIdStampMode = kDiag && kMode == kModeSparseIds;

// phase stamp k4 (kModeSparseStamp's 4-slot layout) or k8 (the id-slab 8-slot one)
template <int kMode>
__device__ __forceinline__ void phase_stamp(const SumFwdArgs &A, int tile, int k4, int k8) {
    if (kMode == kModeSparseStamp) {
        if ((threadIdx.x & 63) == 0) A.stamps[4 * (size_t)tile + k4] = stamp();
    } else if (kIdStampMode<kMode>) {
        if (A.stamps) {
            const long long t = stamp();
            if ((threadIdx.x & 63) == 0) A.stamps[8 * (size_t)tile + k8] = t;
        }
    }
}

// One splat against two pixels of a row (packed v_pk_fma / v_pk_mul): the
// reference's per-pixel op sequence (common.h splat_sigma_h, exp_neg) on both
// lanes of a v2f.  A pair that fails sigma >= 0 and alpha >= 1/255 keeps its
// accumulators bit for bit (the update is selected, not added as zero).
template <bool kIdx>
__device__ __forceinline__ void blend_pair(float gx, float ha, float b, float bdy, float cq,
                                           float opac, float cr, float cg, float cb, v2f px,
                                           int k, v2f &ar, v2f &ag, v2f &ab, int &l0, int &l1) {
    const v2f dx = gx - px;
    const v2f q = __builtin_elementwise_fma((v2f)ha, dx, (v2f)bdy);
    const v2f sg = __builtin_elementwise_fma(q, dx, (v2f)cq);
    const v2f x = sg * kNegLog2e;
    const v2f e = {__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)};
    const v2f al = opac * e;
    const v2f a = {fminf(1.0f, al.x), fminf(1.0f, al.y)};
    const bool v0 = !(sg.x < 0.0f) && !(a.x < kAlphaMin);
    const bool v1 = !(sg.y < 0.0f) && !(a.y < kAlphaMin);
    const v2f nr = __builtin_elementwise_fma((v2f)cr, a, ar);
    const v2f ng = __builtin_elementwise_fma((v2f)cg, a, ag);
    const v2f nb = __builtin_elementwise_fma((v2f)cb, a, ab);
    ar = (v2f){v0 ? nr.x : ar.x, v1 ? nr.y : ar.y};
    ag = (v2f){v0 ? ng.x : ag.x, v1 ? ng.y : ag.y};
    ab = (v2f){v0 ? nb.x : ab.x, v1 ? nb.y : ab.y};
    if (kIdx) {  // final_idx is written (the autograd forward)
        l0 = v0 ? k : l0;
        l1 = v1 ? k : l1;
    }
    (void)b;
}

// blend_pair for an entry of unit opacity, finite colour and bounded geometry
// (cull.h geo_bounded): the alpha cut as a sigma threshold (common.h
// kSigmaCutBits -- the same pairs pass, sigma is never NaN there, and
// alpha = exp(-sigma) <= 1 needs no min), and a failing pair adds colour * 0
// instead of selecting (+-0: an accumulator starts at +0 and is never -0).
// The same bits as blend_pair without the last-index tracking.  (An indexed
// variant -- final_idx from the same threshold test -- measured slower in the
// op path's composite: 28.3 vs 27.5 us at the trained 1080p / 50k frame, its
// extra loop bodies spilled 17 VGPRs around the chunk loop.)
__device__ __forceinline__ void blend_pair_cut(float gx, float ha, float bdy, float cq, float cr,
                                               float cg, float cb, v2f px, v2f &ar, v2f &ag,
                                               v2f &ab) {
    const v2f dx = gx - px;
    const v2f q = __builtin_elementwise_fma((v2f)ha, dx, (v2f)bdy);
    const v2f sg = __builtin_elementwise_fma(q, dx, (v2f)cq);
    const v2f x = sg * kNegLog2e;
    const v2f e = {__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)};
    const v2f av = {__float_as_uint(sg.x) <= kSigmaCutBits ? e.x : 0.0f,
                    __float_as_uint(sg.y) <= kSigmaCutBits ? e.y : 0.0f};
    ar = __builtin_elementwise_fma((v2f)cr, av, ar);
    ag = __builtin_elementwise_fma((v2f)cg, av, ag);
    ab = __builtin_elementwise_fma((v2f)cb, av, ab);
}

// A staged entry takes blend_pair_cut: unit opacity, finite colour, bounded geometry.
__device__ __forceinline__ bool entry_cut_ok(const float4 &geo, const float4 &col, float blu) {
    return col.y == 1.0f && __builtin_isfinite(col.z) && __builtin_isfinite(col.w) &&
           __builtin_isfinite(blu) && geo_bounded(geo.x, geo.y, geo.z, geo.w, col.x);
}

// Can splat (x, y, conic a b c, opacity o) reach alpha >= 1/255 on any pixel
// centre of [x0, x1] x [y0, y1]?  false only when provably not: alpha >= 1/255
// needs sigma <= ln(255 o), i.e. the point inside the ellipse
// d^T C d <= 2 ln(255 o), whose half-extents are sqrt(2 ln(255 o) c / det) and
// sqrt(2 ln(255 o) a / det); margins (0.1 % + 0.01) dwarf fp32 rounding.
__device__ __forceinline__ bool ellipse_hits_rect(float x, float y, float a, float b, float c,
                                                  float o, float x0, float x1, float y0, float y1) {
    if (!(o > 0.0f)) return !(o <= 0.0f);  // o <= 0: alpha <= 0 never valid; NaN: keep
    const float det = a * c - b * b;
    if (!cull_conditioned(a, c, det) || !(o < 3.0e38f) || !(fabsf(x) < 1e30f) || !(fabsf(y) < 1e30f))
        return true;  // not positive definite, ill-conditioned or non-finite: no culling
    const float lg = __logf(255.0f * o);
    if (lg < -0.01f) return false;  // o < e^-0.01 / 255: alpha < 1/255 everywhere
    const float S2 = 2.0f * (lg * 1.001f + 0.01f);
    const float ex = sqrtf(S2 * c / det) * 1.001f + 0.01f;
    const float ey = sqrtf(S2 * a / det) * 1.001f + 0.01f;
    return (x + ex >= x0) && (x - ex <= x1) && (y + ey >= y0) && (y - ey <= y1);
}

typedef float v4f __attribute__((ext_vector_type(4)));

// Plane stores of the render layout, by cache policy: streaming write-through
// (nt sc1, production: the lines leave L2 as they are written, so the
// end-of-kernel release has ~25 MB less to write back -- composite 10.6 ->
// 9.5 us at 1080p), plain (write-back L2), sc1, sc0 sc1, or nt alone.
//
// Every inline-asm store of more than 64 bits ends with ``s_nop 1``: the store
// reads its data VGPRs after it issues, and on gfx940+ a VALU write to one of
// them needs two wait states (LLVM GCNHazardRecognizer, VALU-after-VMEM-store
// data hazard).  The compiler pads its own stores, and inline-asm ones inside a
// basic block, but round 5's HWC write-through store ended an exec-masked block
// and the next block's first VALU overwrote data VGPR 0 one wait state later --
// one 16-lane pass of the wave stored the new value now and then (DESIGN.md
// §12, tools/store_hazard_scan.py, tests/test_store_hazard.py).  The trailing
// nop makes the asm safe wherever the compiler places it.
enum { kStoreNtSc1 = 0, kStorePlain = 1, kStoreSc1 = 2, kStoreSc01 = 3, kStoreNt = 4 };

__device__ __forceinline__ void st_f4(float *p, float a, float b, float c, float d, int policy) {
    const v4f v = {a, b, c, d};
    if (!kDiag) policy = kStoreNtSc1;  // the product's one policy
    switch (policy) {
    case kStoreNt: __builtin_nontemporal_store(v, reinterpret_cast<v4f *>(p)); break;
    case kStoreSc1: asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory"); break;
    case kStoreSc01:
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
        break;
    case kStoreNtSc1:
        asm volatile("global_store_dwordx4 %0, %1, off sc1 nt\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
        break;
    default: *reinterpret_cast<v4f *>(p) = v; break;
    }
}

__device__ __forceinline__ void st_f2(float *p, float a, float b, int policy) {
    const v2f v = {a, b};
    if (!kDiag) policy = kStoreNtSc1;  // the product's one policy
    switch (policy) {
    case kStoreNt: __builtin_nontemporal_store(v, reinterpret_cast<v2f *>(p)); break;
    case kStoreSc1: asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory"); break;
    case kStoreSc01:
        asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
        break;
    case kStoreNtSc1:
        asm volatile("global_store_dwordx2 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
        break;
    default: *reinterpret_cast<v2f *>(p) = v; break;
    }
}

__device__ __forceinline__ float clamp01(float x) {
    // torch.clamp(x, 0, 1): NaN stays NaN
    return x < 0.0f ? 0.0f : (x > 1.0f ? 1.0f : x);
}

// A plane value: clamped for the render's layout, as blended for the op path's
__device__ __forceinline__ float plane_val(const SumFwdArgs &A, float x) {
    return A.layout == kLayoutCHWClamped ? clamp01(x) : x;
}

// A tile's first pixel coordinate as a float, converted where it is used (the
// asm keeps the compiler from hoisting the conversion to the kernel entry and
// holding -- and, at 64 VGPRs, spilling -- the value across the blend loops).
__device__ __forceinline__ float tile_origin(int t) {
    int v = t * kTile;
    asm volatile("" : "+s"(v));
    return (float)v;
}

// Gather splat g: geo = {x, y, a/2, b}, col = {c/2, opacity, r, g}, blu = b.
__device__ __forceinline__ void load_splat(const SumFwdArgs &A, int g, float4 &geo, float4 &col,
                                           float &blu) {
    if (A.rec) {
        geo = A.rec[3 * g];
        col = A.rec[3 * g + 1];
        blu = A.rec[3 * g + 2].x;
        return;
    }
    const float2 xy = A.xys[g];
    const float a = A.conics[3 * g], b = A.conics[3 * g + 1], c = A.conics[3 * g + 2];
    geo = make_float4(xy.x, xy.y, 0.5f * a, b);
    col = make_float4(0.5f * c, A.opac[g], A.colors[3 * g], A.colors[3 * g + 1]);
    blu = A.colors[3 * g + 2];
}

// Scalar store of one pixel in either layout.
__device__ __forceinline__ void store_pixel(const SumFwdArgs &A, size_t p, float r, float g, float b,
                                            int l) {
    if (layout_planes(A.layout)) {
        const size_t hw = (size_t)A.img_w * (size_t)A.img_h;
        A.out[p] = plane_val(A, r);
        A.out[hw + p] = plane_val(A, g);
        A.out[2 * hw + p] = plane_val(A, b);
    } else {
        A.out[3 * p] = r;
        A.out[3 * p + 1] = g;
        A.out[3 * p + 2] = b;
    }
    if (A.final_idx) A.final_idx[p] = l;
    if (A.final_Ts) A.final_Ts[p] = 1.0f;
}

// A tile with more than 256 entries on the frame path (its slab kept an
// arbitrary 256): its first 256 ids are rebuilt from every splat's tile bbox.
__device__ __forceinline__ int wave_brute_tile_ids(const SumFwdArgs &A, int tile, int *s_ids) {
    return wave_brute_ids(A.cull_xys, A.cull_radii, A.splat_begin, A.num_points, A.tbx,
                          (A.img_h + kTile - 1) / kTile, tile, s_ids);
}

// Sparse path: one wave blends the whole 16x16 tile, 4 pixels per lane.
template <int kMode, bool kIdx, bool kSplit = false>
__device__ __forceinline__ void sum_fwd_sparse(const SumFwdArgs &A, int tile, int2 range, int n,
                                               float4 *s_slice, float3 init, bool ids_in_lds,
                                               const int *s_ids, const float4 *seg_rec,
                                               const float4 *seg_head, float4 spec0, float4 spec1,
                                               float4 spec2, int spec_slots, int spec_id) {
    // staged entries (slot kChunk: the grouped loop's no-op sentinel), their
    // blocks, and the lane groups' lists [64 iterations][16 groups]
    constexpr int kS = kChunk + 1, kS4 = (kS + 3) / 4;
    float4 *s_geo = s_slice;                           // x, y, 0.5a, b
    float4 *s_col = s_slice + kS;                      // 0.5c, opacity, r, g
    float *s_blu = (float *)(s_slice + 2 * kS);        // b
    unsigned short *s_gm = reinterpret_cast<unsigned short *>(s_slice + 2 * kS + kS4);
    unsigned char *s_list = reinterpret_cast<unsigned char *>(s_slice + 2 * kS + kS4 + kChunk / 8);
    static_assert(2 * kS + kS4 + kChunk / 8 + kChunk <= kSlice, "sparse LDS layout");
    const int lane = threadIdx.x & 63;
    if (lane == 0) {
        // sigma = +inf at every pixel: alpha = 0 fails the test, no change
        s_geo[kChunk] = make_float4(0.0f, 1e30f, 0.0f, 0.0f);
        s_col[kChunk] = make_float4(1e30f, 1.0f, 0.0f, 0.0f);
        s_blu[kChunk] = 0.0f;
    }
    const int kGroupMin = A.group_min;
    const int ty = tile / A.tbx, tx = tile - ty * A.tbx;
    const int pi = ty * kTile + (lane >> 2);
    const int pj = tx * kTile + ((lane & 3) << 2);
    const float py = (float)pi;
    const float px0 = (float)pj, px1 = (float)(pj + 1), px2 = (float)(pj + 2), px3 = (float)(pj + 3);
    v2f ar01 = {init.x, init.x}, ag01 = {init.y, init.y}, ab01 = {init.z, init.z};
    v2f ar23 = ar01, ag23 = ag01, ab23 = ab01;
    const v2f px01 = {px0, px1}, px23 = {px2, px3};
    int l0 = 0, l1 = 0, l2 = 0, l3 = 0;
    // the chunk's entries all take blend_pair_cut (render paths only: the
    // cut variant tracks no last index)
    bool cut = false;
    if (seg_rec) {
        // <= 64 slab records in fill order: staged at their rank by id, before
        // the chunk loop (the speculative records die here)
        const int cnt = n;
            // <= 64 slab records in fill order: staged at their rank by id
        float4 geo = spec0, col = spec1, bx = spec2;
        if (kIdStampMode<kMode> && A.stamps) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            phase_stamp<kMode>(A, tile, 0, 1);
        }
        if (lane >= spec_slots && lane < cnt && !(kDiag && (A.ablate & 4))) {
            if (seg_head || A.rec) {
                // slab records at their slot, or (id slabs, no head) the record of
                // the lane's id gathered from A.rec -- the same 48 bytes
                const float4 *r = seg_head ? slot_rec(seg_head, seg_rec, lane) : A.rec + 3 * (size_t)spec_id;
                geo = r[0];
                col = r[1];
                bx = r[2];
            } else {  // the op path: the lane's id's inputs
                load_splat(A, spec_id, geo, col, bx.x);
                bx.y = __int_as_float(spec_id);
            }
        }
        const int id = lane < cnt ? __float_as_int(bx.y) : 0x7fffffff;
        // rank by id: the ids through LDS (the lists' bytes, free until the
        // chunk loop), 4 per broadcast read -- 2 VALU per entry instead of the
        // 3 of a readlane loop; padding lanes hold 0x7fffffff, below no id
        int *s_rid = reinterpret_cast<int *>(s_list);
        s_rid[lane] = id;
        wave_lds_sync();
        // (staging in slot order instead was measured, round 5: -3-5 %, at the
        // cost of bit-identity with the op path and run-to-run determinism)
        int rank = 0;
        if (kDiag && (A.ablate & 8)) rank = lane;
        else
        for (int k = 0; k < cnt; k += 4) {
            const int4 q = *reinterpret_cast<const int4 *>(s_rid + k);
            rank += (q.x < id ? 1 : 0) + (q.y < id ? 1 : 0) + (q.z < id ? 1 : 0) + (q.w < id ? 1 : 0);
        }
        wave_lds_sync();
        if (A.bins_out) {  // the op path: the tile's ids in id order and its bins, for the backward
            if (lane < cnt) A.ids_rw[(size_t)tile * A.ids_cap + rank] = id;
            if (lane == 0) A.bins_out[tile] = make_int2(range.x, range.x + cnt);
        }
        if (!kIdx) cut = A.cut && __ballot(lane < cnt && !entry_cut_ok(geo, col, bx.x)) == 0ull;
        if (lane < cnt) {
            s_geo[rank] = geo;
            s_col[rank] = col;
            s_blu[rank] = bx.x;
            if (n > kGroupMin)
                s_gm[rank] = (unsigned short)ellipse_blocks<16>(
                    geo.x, geo.y, 2.0f * geo.z, geo.w, 2.0f * col.x, col.y, tile_origin(tx), tile_origin(ty));
        }
    }
    for (int base = 0; base < n; base += kChunk) {
        const int cnt = min(kChunk, n - base);
        if (!seg_rec) {  // (seg_rec: staged above, n <= 64: one chunk)
            bool ok = true;
            float4 geo = make_float4(0.f, 0.f, 0.f, 0.f), col = geo;
            float blu = 0.f;
            if (lane < cnt) {
                const int j = base + lane;
                load_splat(A, ids_in_lds ? s_ids[j] : A.ids[range.x + j], geo, col, blu);
                if (!kIdx) ok = entry_cut_ok(geo, col, blu);
            }
            if (!kIdx) cut = A.cut && __ballot(!ok) == 0ull;
            if (lane < cnt) {
                s_geo[lane] = geo;
                s_col[lane] = col;
                s_blu[lane] = blu;
                if (cnt > kGroupMin)
                    s_gm[lane] = (unsigned short)ellipse_blocks<16>(
                        geo.x, geo.y, 2.0f * geo.z, geo.w, 2.0f * col.x, col.y, tile_origin(tx), tile_origin(ty));
            }
        }
        wave_lds_sync();
        const int k0 = range.x + base;
        // entry t of the chunk into the lane's 4 pixels
        auto blend = [&](int t, auto cutc) {
            const float4 G = s_geo[t];
            const float4 C = s_col[t];
            const float dy = G.y - py;
            const float cq = (C.x * dy) * dy;
            const float bdy = G.w * dy;
            if constexpr (decltype(cutc)::value) {
                const float bl = s_blu[t];
                blend_pair_cut(G.x, G.z, bdy, cq, C.z, C.w, bl, px01, ar01, ag01, ab01);
                blend_pair_cut(G.x, G.z, bdy, cq, C.z, C.w, bl, px23, ar23, ag23, ab23);
            } else {
                const float bl = s_blu[t];
                const int k = k0 + t;
                blend_pair<kIdx>(G.x, G.z, G.w, bdy, cq, C.y, C.z, C.w, bl, px01, k, ar01, ag01, ab01, l0, l1);
                blend_pair<kIdx>(G.x, G.z, G.w, bdy, cq, C.y, C.z, C.w, bl, px23, k, ar23, ag23, ab23, l2, l3);
            }
        };
        if (cnt <= kGroupMin) {
            if (kMode == kModeSparsePrio) __builtin_amdgcn_s_setprio(0);
            // a few entries: every lane walks them all (the lists would cost
            // more than the pairs they skip)
            if (base == 0) phase_stamp<kMode>(A, tile, 1, 2);
            for (int t = 0; t < cnt && !(kDiag && (A.ablate & 1)); ++t) {
                if (!kIdx && cut)
                    blend(t, std::true_type{});
                else
                    blend(t, std::false_type{});
            }
            wave_lds_sync();
            continue;
        }
        const unsigned gmt = lane < cnt ? s_gm[lane] : 0u;
        const unsigned long long lt = (1ull << lane) - 1ull;
        *reinterpret_cast<uint4 *>(s_list + 16 * lane) =
            make_uint4(0x40404040u, 0x40404040u, 0x40404040u, 0x40404040u);
        __builtin_amdgcn_wave_barrier();
        int maxlen = 0;
#pragma unroll 1
        for (int g = 0; g < 16; ++g) {
            const bool in = (gmt >> g) & 1u;
            const unsigned long long mg = __ballot(in);
            if (in) s_list[16 * __popcll(mg & lt) + g] = (unsigned char)lane;
            maxlen = max(maxlen, __popcll(mg));
        }
        wave_lds_sync();
        if (kMode == kModeSparsePrio) __builtin_amdgcn_s_setprio(0);
        if (base == 0) phase_stamp<kMode>(A, tile, 1, 2);
        // the lane's 4x4 block of the tile
        const unsigned char *ml = s_list + (((lane >> 4) << 2) | (lane & 3));
        if constexpr (kSplit) {
            // one loop per variant: no accumulator moves between the two bodies'
            // registers each trip (6 v_mov_b64 of ~40 VALU), at the cost of a
            // few spilled registers around the loops -- the dense render's
            // instance (raster_render_ids_kernel<W, true>, chosen by the density
            // hint): trained 1080p / 50k composite 20.3 -> 19.2 us, 10k frames
            // keep the single loop (7.9 vs 8.1 us; profiles/r06/render_split/)
            if (!kIdx && cut) {
#pragma unroll 1
                for (int it = 0; it < maxlen; ++it) blend(ml[16 * it], std::true_type{});
            } else {
#pragma unroll 1
                for (int it = 0; it < maxlen; ++it) blend(ml[16 * it], std::false_type{});
            }
        } else {
            for (int it = 0; it < maxlen; ++it) {
                if (!kIdx && cut)
                    blend(ml[16 * it], std::true_type{});
                else
                    blend(ml[16 * it], std::false_type{});
            }
        }
        wave_lds_sync();
    }
    phase_stamp<kMode>(A, tile, 2, 3);
    const float r0 = ar01.x, r1 = ar01.y, r2 = ar23.x, r3 = ar23.y;
    const float g0 = ag01.x, g1 = ag01.y, g2 = ag23.x, g3 = ag23.y;
    const float b0 = ab01.x, b1 = ab01.y, b2 = ab23.x, b3 = ab23.y;
    if (layout_planes(A.layout) && A.vec_chw && (tx + 1) * kTile <= A.img_w) {
        // 4 lanes write a 64-byte row segment of each plane
        if (pi < A.img_h && !(kDiag && (A.ablate & 2))) {
            const size_t hw = (size_t)A.img_w * (size_t)A.img_h;
            float *o = A.out + (size_t)pi * (size_t)A.img_w + (size_t)pj;
            st_f4(o, plane_val(A, r0), plane_val(A, r1), plane_val(A, r2), plane_val(A, r3), A.store_policy);
            st_f4(o + hw, plane_val(A, g0), plane_val(A, g1), plane_val(A, g2), plane_val(A, g3),
                  A.store_policy);
            st_f4(o + 2 * hw, plane_val(A, b0), plane_val(A, b1), plane_val(A, b2), plane_val(A, b3),
                  A.store_policy);
            if (A.final_idx)
                *reinterpret_cast<int4 *>(A.final_idx + (o - A.out)) = make_int4(l0, l1, l2, l3);
        }
        if (kMode == kModeSparseStamp || (kIdStampMode<kMode> && A.stamps)) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            phase_stamp<kMode>(A, tile, 3, 4);
        }
        return;
    }
    if (A.layout == kLayoutHWC && A.vec && (tx + 1) * kTile <= A.img_w) {
        // stage the tile's 3 KB of RGB (lane l owns floats 12l..12l+11, a
        // conflict-free 48-byte stride), then write 16-byte chunk c = 64j + lane
        // = row c / 12, column chunk c % 12: whole 192-byte rows per instruction
        s_slice[3 * lane] = make_float4(r0, g0, b0, r1);
        s_slice[3 * lane + 1] = make_float4(g1, b1, r2, g2);
        s_slice[3 * lane + 2] = make_float4(b2, r3, g3, b3);
        wave_lds_sync();
        const size_t tile_base = ((size_t)(ty * kTile) * (size_t)A.img_w + (size_t)(tx * kTile)) * 3;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int c = j * 64 + lane;
            const int row = c / 12, cc = c - row * 12;
            // written through like the planes (the op composite 20.0 -> 18.6 us
            // over 10k + 50k frames, tools/hwc_store_ab.py, profiles/r06/hwc_store/);
            // round 5's unpadded asm form lost 16 floats in 1-4 % of the tiles
            // (the store-data hazard above, tests/analysis/store_hazard_repro.py)
            if (ty * kTile + row < A.img_h) {
                float *o = A.out + tile_base + (size_t)row * A.img_w * 3 + cc * 4;
                const float4 q = s_slice[c];
                st_f4(o, q.x, q.y, q.z, q.w, A.store_policy);
            }
        }
        if (pi < A.img_h && A.final_idx) {
            const size_t p0 = (size_t)pi * (size_t)A.img_w + (size_t)pj;
            *reinterpret_cast<int4 *>(A.final_idx + p0) = make_int4(l0, l1, l2, l3);
            if (A.final_Ts)
                *reinterpret_cast<float4 *>(A.final_Ts + p0) = make_float4(1.f, 1.f, 1.f, 1.f);
        }
        return;
    }
    if (pi >= A.img_h) return;
    const float rr[4] = {r0, r1, r2, r3}, gg[4] = {g0, g1, g2, g3}, bb[4] = {b0, b1, b2, b3};
    const int ll[4] = {l0, l1, l2, l3};
#pragma unroll
    for (int q = 0; q < 4; ++q)
        if (pj + q < A.img_w)
            store_pixel(A, (size_t)pi * (size_t)A.img_w + (size_t)(pj + q), rr[q], gg[q], bb[q], ll[q]);
}

// Dense path: this wave blends one 8-row band, 2 pixels per lane.
template <int kMode, bool kIdx>
__device__ __forceinline__ void sum_fwd_band(const SumFwdArgs &A, int tile, int band, int2 range,
                                             int n, float4 *s_slice, float3 init, bool ids_in_lds,
                                             const int *s_ids, const float4 *seg_rec,
                                             const float4 *seg_head, float4 spec0, float4 spec1,
                                             float4 spec2) {
    // staged entries (slot kChunk: the grouped loop's no-op sentinel), their
    // blocks, and the lane groups' lists [64 iterations][8 groups]
    constexpr int kS = kChunk + 1, kS4 = (kS + 3) / 4;
    float4 *s_geo = s_slice;                                      // x, y, 0.5a, b
    float4 *s_col = s_slice + kS;                                 // 0.5c, opacity, r, g
    float *s_blu = reinterpret_cast<float *>(s_slice + 2 * kS);
    int *s_k = reinterpret_cast<int *>(s_slice + 2 * kS + kS4);
    unsigned char *s_gm = reinterpret_cast<unsigned char *>(s_slice + 2 * kS + 2 * kS4);
    unsigned char *s_list = s_gm + kChunk;
    static_assert(2 * kS + 2 * kS4 + (kChunk + 8 * kChunk) / 16 <= kSlice, "band LDS layout");
    const int lane = threadIdx.x & 63;
    if (lane == 0) {
        // sigma = +inf at every pixel: alpha = 0 fails the test, no change
        s_geo[kChunk] = make_float4(0.0f, 1e30f, 0.0f, 0.0f);
        s_col[kChunk] = make_float4(1e30f, 1.0f, 0.0f, 0.0f);
        s_blu[kChunk] = 0.0f;
        s_k[kChunk] = 0;
    }
    const int grp = ((lane >> 5) << 2) | ((lane & 7) >> 1);  // the lane's 4x4 block
    const int ty = tile / A.tbx, tx = tile - ty * A.tbx;
    const int row0 = ty * kTile + band * 8;
    const int pi = row0 + (lane >> 3);
    const int pj = tx * kTile + ((lane & 7) << 1);
    const float py = (float)pi;
    const v2f pxv = {(float)pj, (float)(pj + 1)};
    const float bx0 = (float)(tx * kTile), by0 = (float)row0;
    if (kMode == kModeNoBlend) n = 0;
    v2f ar = {init.x, init.x}, ag = {init.y, init.y}, ab = {init.z, init.z};
    int l0 = 0, l1 = 0;
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (int base = 0; base < n; base += kChunk) {
        const int j = base + lane;
        bool keep = false;
        unsigned gm = 0u;
        float4 geo = make_float4(0.f, 0.f, 0.f, 0.f), col = geo;
        float blu = 0.f;
        int id = 0x7fffffff;
        if (j < n) {
            if (seg_rec) {  // <= 64 slab records in fill order
                float4 bx = spec2;
                geo = spec0;
                col = spec1;
                if (lane >= A.spec_slots) {
                    const float4 *r = slot_rec(seg_head, seg_rec, j);
                    geo = r[0];
                    col = r[1];
                    bx = r[2];
                }
                blu = bx.x;
                id = __float_as_int(bx.y);
            } else {
                load_splat(A, ids_in_lds ? s_ids[j] : A.ids[range.x + j], geo, col, blu);
            }
            // 2 * (a/2) == a except for subnormal a, where culling is off anyway
            gm = ellipse_blocks<8>(geo.x, geo.y, 2.0f * geo.z, geo.w, 2.0f * col.x, col.y, bx0, by0);
            keep = gm != 0u;
        }
        const unsigned long long m = __ballot(keep);
        if (seg_rec) {
            // kept records in id order; k = rank among all entries (sorted index)
            int pos = 0, rank = 0;
            for (int k = 0; k < n; ++k) {
                const int below = __builtin_amdgcn_readlane(id, k) < id ? 1 : 0;
                rank += below;
                pos += below & (int)((m >> k) & 1ull);
            }
            if (keep) {
                s_geo[pos] = geo;
                s_col[pos] = col;
                s_blu[pos] = blu;
                s_k[pos] = range.x + rank;
                s_gm[pos] = (unsigned char)gm;
            }
        } else if (keep) {
            const int pos = __popcll(m & lt);
            s_geo[pos] = geo;
            s_col[pos] = col;
            s_blu[pos] = blu;
            s_k[pos] = range.x + j;
            s_gm[pos] = (unsigned char)gm;
        }
        const int cnt = __popcll(m);
        wave_lds_sync();
        // each group walks, in order, only the staged entries reaching its
        // block; its list is padded with the sentinel to the longest
        const unsigned gmt = lane < cnt ? s_gm[lane] : 0u;
        *reinterpret_cast<unsigned long long *>(s_list + 8 * lane) = 0x4040404040404040ull;
        __builtin_amdgcn_wave_barrier();
        int maxlen = 0;
#pragma unroll 1
        for (int g = 0; g < 8; ++g) {
            const bool in = (gmt >> g) & 1u;
            const unsigned long long mg = __ballot(in);
            if (in) s_list[8 * __popcll(mg & lt) + g] = (unsigned char)lane;
            maxlen = max(maxlen, __popcll(mg));
        }
        wave_lds_sync();
        const unsigned char *ml = s_list + grp;
        for (int it = 0; it < maxlen; ++it) {
            const int t = ml[8 * it];
            const float4 G = s_geo[t];
            const float4 C = s_col[t];
            const float bl = s_blu[t];
            const int k = kIdx ? s_k[t] : 0;
            const float dy = G.y - py;
            const float cq = (C.x * dy) * dy;
            const float bdy = G.w * dy;
            blend_pair<kIdx>(G.x, G.z, G.w, bdy, cq, C.y, C.z, C.w, bl, pxv, k, ar, ag, ab, l0, l1);
        }
        wave_lds_sync();
    }
    if (kMode == kModeNoStore) {
        asm volatile("" ::"v"(ar.x), "v"(ar.y), "v"(ag.x), "v"(ag.y), "v"(ab.x), "v"(ab.y), "v"(l0),
                     "v"(l1));
        return;
    }
    if (layout_planes(A.layout) && A.vec_chw && (tx + 1) * kTile <= A.img_w) {
        if (pi < A.img_h) {
            const size_t hw = (size_t)A.img_w * (size_t)A.img_h;
            float *o = A.out + (size_t)pi * (size_t)A.img_w + (size_t)pj;
            st_f2(o, plane_val(A, ar.x), plane_val(A, ar.y), A.store_policy);
            st_f2(o + hw, plane_val(A, ag.x), plane_val(A, ag.y), A.store_policy);
            st_f2(o + 2 * hw, plane_val(A, ab.x), plane_val(A, ab.y), A.store_policy);
            if (A.final_idx) *reinterpret_cast<int2 *>(A.final_idx + (o - A.out)) = make_int2(l0, l1);
        }
        return;
    }
    if (A.layout == kLayoutHWC && A.vec && (tx + 1) * kTile <= A.img_w) {
        // stage 8 rows x 16 px x 12 B = 1536 B (lane l owns floats 6l..6l+5),
        // then 96 16-byte chunks as whole 192-byte rows; final_idx as pairs
        float2 *so2 = reinterpret_cast<float2 *>(s_slice);
        so2[3 * lane] = make_float2(ar.x, ag.x);
        so2[3 * lane + 1] = make_float2(ab.x, ar.y);
        so2[3 * lane + 2] = make_float2(ag.y, ab.y);
        wave_lds_sync();
        const size_t base_off = ((size_t)row0 * (size_t)A.img_w + (size_t)(tx * kTile)) * 3;
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
            const int c = jj * 64 + lane;
            if (c < 96) {
                const int row = c / 12, cc = c - row * 12;
                if (row0 + row < A.img_h) {
                    const float4 q = s_slice[c];
                    st_f4(A.out + base_off + (size_t)row * A.img_w * 3 + cc * 4, q.x, q.y, q.z, q.w,
                          A.store_policy);
                }
            }
        }
        if (pi < A.img_h && A.final_idx) {
            const size_t p0 = (size_t)pi * (size_t)A.img_w + (size_t)pj;
            *reinterpret_cast<int2 *>(A.final_idx + p0) = make_int2(l0, l1);
            if (A.final_Ts)
                *reinterpret_cast<float2 *>(A.final_Ts + p0) = make_float2(1.f, 1.f);
        }
        return;
    }
    if (pi >= A.img_h) return;
    const float rr[2] = {ar.x, ar.y}, gg[2] = {ag.x, ag.y}, bb[2] = {ab.x, ab.y};
    const int ll[2] = {l0, l1};
#pragma unroll
    for (int q = 0; q < 2; ++q)
        if (pj + q < A.img_w)
            store_pixel(A, (size_t)pi * (size_t)A.img_w + (size_t)(pj + q), rr[q], gg[q], bb[q], ll[q]);
}

// Op path with id slabs: the tile's sorted ids back in place (the backward's
// gaussian_ids_sorted) and its bins row [begin, begin + n).
__device__ __forceinline__ void write_sorted_ids(const SumFwdArgs &A, int tile, int begin, int n,
                                                 const int *s_ids) {
    const int lane = threadIdx.x & 63;
    for (int j = lane; j < n; j += 64) A.ids_rw[(size_t)tile * A.ids_cap + j] = s_ids[j];
    if (lane == 0) A.bins_out[tile] = make_int2(begin, begin + n);
}

// kModeSparse launches 64-thread workgroups (one wave per tile); every other
// mode 128-thread workgroups (two waves per tile).  (Two one-tile waves per
// workgroup, as raster_render_ids_kernel, measured for the op path's
// kModeSparseIds, round 6: 24.6-25.1 vs 24.3-24.5 us; not kept,
// profiles/r06/generic_w2/.)
// kIdx: final_idx is written (the autograd forward); the render paths launch
// the kIdx = false instance, which tracks no indices.
// (2 and 4 one-tile waves per workgroup were measured, round 5: within +-2 %,
// not kept)
template <int kMode, bool kIdx>
__global__ __launch_bounds__(kMode == kModeSparse || kMode == kModeSparseStamp || kMode == kModeSparsePrio ||
                              kMode == kModeSparseIds ? 64 : 128, 8) void
raster_sum_fwd_kernel(SumFwdArgs A) {
    constexpr bool kOneWave = kMode == kModeSparse || kMode == kModeSparseStamp || kMode == kModeSparsePrio ||
                              kMode == kModeSparseIds;
    // id slabs: the op path's autograd forward (kIdx, or sparse / banded
    // without final_idx) and the single-frame render
    constexpr bool kIds = kIdx || kMode == kModeSparseIds || kMode == kModeBanded;
    __shared__ float4 s_buf[kOneWave ? 1 : 2][kSlice];
    __shared__ int s_ids[1][kTilePix];  // the tile's sorted ids
    // raised wave priority over the staging (loads, ranking, lists): the
    // arbiter favours older waves, so a young wave would otherwise wait behind
    // its elders' blending to issue its round trips (train.hip, same reason)
    if (kMode == kModeSparsePrio) __builtin_amdgcn_s_setprio(3);
    const int w = kOneWave ? 0 : (threadIdx.x >> 6);
    constexpr int sub = 0;
    // runs of 16 tiles dealt over the XCDs, as the training tile kernel
    // (fbench: 10k frame 17.0 vs 17.3-17.4 us, the textured video's dense
    // frame 116 at M = 894k 251.5-252.6 vs 263.9-264.6, trained 50k equal;
    // A/B knob 37: 1 dispatch order, 4 contiguous XCD ranges)
    int tile = !(kDiag && A.xcd_off) ? xcd_runs<16>(blockIdx.x, A.ntiles * A.frames)
                     : A.xcd_off == 1      ? (int)blockIdx.x
                                           : xcd_remap(blockIdx.x, A.ntiles * A.frames);
    if (A.frames > 1) {  // batched frames: this block's frame and tile
        const int b = tile / A.ntiles;
        tile -= b * A.ntiles;
        if (A.slab) {  // (an offset null pointer would read as a slab)
            A.slab += b * A.slab_stride;
            if (A.slab_ovf) A.slab_ovf += (size_t)b * kOvfSlots * (size_t)A.ntiles;
            A.slab_counts += (size_t)b * A.counts_stride;
            A.slab_counts_clear += (size_t)b * A.counts_stride;
        }
        if (kMode == kModeSparseIds) {  // id slabs in each frame's slab memory
            A.ids_rw += 4 * b * A.slab_stride;
            A.id_counts += (size_t)b * A.counts_stride;
            A.id_counts_clear += (size_t)b * A.counts_stride;
        }
        A.m_dev += (size_t)b * A.m_stride;
        A.meta_out += (size_t)b * A.m_stride;
        A.out += b * A.out_stride;
        A.splat_begin = A.frame_off[b];
        A.num_points = A.frame_off[b + 1];
    }
    // M in the first round trip, before any store: read after the counts'
    // clearing store it could not be a scalar load and waited a round trip of
    // its own between the count and the records
    const int m_val = A.m_dev ? *A.m_dev : 1;
    long long t0 = 0;
    if (kMode == kModeStamp || kMode == kModeSparseStamp || (kIdStampMode<kMode> && A.stamps)) t0 = stamp();
    int2 range;
    SegIds seg;  // the tile's ids (unsorted when A.sort_ids)
    int n_all;
    const float4 *seg_rec = nullptr;  // slab records, when the fast path applies
    float4 spec0 = make_float4(0.f, 0.f, 0.f, 0.f), spec1 = spec0, spec2 = spec0;
    int spec_id = 0;  // id slabs (render): the lane's slot, loaded with the count
    if (kMode != kModeSparseIds && A.slab) {  // (mode 9 renders over id slabs only)
        // this frame's count, and the first kSpecSlots records loaded in the
        // same round trip (speculatively: most tiles have that few)
        const int lane = threadIdx.x & 63;
        // slots >= kHeadSlots at their index from recs; the first ones in the head
        const float4 *recs = slab_rec(A.slab, A.ntiles, tile, kHeadSlots) - 3 * kHeadSlots;
        n_all = (int)__builtin_amdgcn_readfirstlane(A.slab_counts[tile]);
        if (lane < A.spec_slots) {
            const float4 *h = slab_rec(A.slab, A.ntiles, tile, lane);
            spec0 = h[0];
            spec1 = h[1];
            spec2 = h[2];
        }
        if ((threadIdx.x & 63) == 0) {
            A.slab_counts_clear[tile] = 0u;  // the next frame's counts
            if (tile == 0) {
                A.meta_out[0] = m_val;
                A.meta_out[1] = 0;
            }
        }
        range = make_int2(0, n_all);
        seg.ids = nullptr;
        seg.recs = recs;
        seg.head = slab_rec(A.slab, A.ntiles, tile, 0);
        seg.ovf = A.slab_ovf ? A.slab_ovf + (size_t)tile * kOvfSlots : nullptr;
        if (n_all <= kChunk) seg_rec = recs;  // slots past the head, at their index
    } else if (kIds && A.id_counts) {
        // op path, unsorted id slabs (its autograd forward: kIdx instances
        // only): this call's count (M from the insertion)
        n_all = (int)__builtin_amdgcn_readfirstlane(A.id_counts[tile]);
        // render over id slabs: slot `lane` in the same round trip as the count
        // (all 256 slots of every tile exist; past the count it is not used)
        // (measured for the op path's indexed instance too, its <= 64 ids ranked
        // from these: slower, 44.3 vs 42.4 us per tools/slabbench.py call at
        // the trained 1080p / 50k frame -- its ids stay read after the count)
        if (kMode == kModeSparseIds)
            spec_id = A.ids_rw[(size_t)tile * A.ids_cap + (threadIdx.x & 63)];
        if ((threadIdx.x & 63) == 0) {
            A.id_counts_clear[tile] = 0u;  // the next call's counts
            if (tile == 0) {
                A.meta_out[0] = m_val;
                A.meta_out[1] = 0;
            }
        }
        range = make_int2(tile * A.ids_cap, tile * A.ids_cap + (n_all < kTilePix ? n_all : kTilePix));
        seg.ids = A.ids_rw + (size_t)tile * A.ids_cap;
        seg.cap_ids = A.ids_cap;
        seg.recs = nullptr;
        seg.head = nullptr;
        // <= 64 entries: records gathered by id and ranked straight into the
        // staging, as the slab records are (sum_fwd_sparse) -- the render's
        // packed records (A.rec), or the op path's inputs (seg_rec then only
        // flags the path: sum_fwd_sparse gathers from xys / conics / colours)
        if (kMode == kModeSparseIds && n_all <= kChunk)
            seg_rec = A.rec ? A.rec : reinterpret_cast<const float4 *>(A.xys);
    } else {
        range = A.bins[tile];
        n_all = range.y - range.x;
        n_all = n_all < 0 ? 0 : n_all;
        seg.ids = A.ids + range.x;
        seg.recs = nullptr;
        seg.head = nullptr;
    }
    int n = n_all > kTilePix ? kTilePix : n_all;
    // rasterize_sum.py:121-127: a frame without intersections is the background
    float3 init = make_float3(0.f, 0.f, 0.f);
    if (m_val < 1) {
        n = n_all = 0;
        init = make_float3(A.bg[0], A.bg[1], A.bg[2]);
    }
    const int ty = tile / A.tbx;
    if (kMode == kModeSparseStamp && (threadIdx.x & 63) == 0) A.stamps[4 * (size_t)tile] = t0;
    if (kIdStampMode<kMode> && A.stamps && (threadIdx.x & 63) == 0) {
        A.stamps[8 * (size_t)tile] = t0;
        A.stamps[8 * (size_t)tile + 5] = n_all;
    }
    const bool sparse = kMode == kModeSparse || kMode == kModeSparseStamp || kMode == kModeSparsePrio ||
                        kMode == kModeSparseIds ||
                        ((kMode == kModeAdaptive || kMode == kModeStamp) && n <= A.sparse_max);
    if (n == 0) seg_rec = nullptr;
    const bool by_ids = A.sort_ids && !seg_rec;  // ids sorted into s_ids first
    if (sparse) {
        if (w != 0) return;
        if (by_ids)
            n = ((A.slab || (kIds && A.id_counts)) && n_all > seg.cap())
                    ? wave_brute_tile_ids(A, tile, s_ids[sub])
                    : wave_sorted_tile_ids(seg, n_all, s_ids[sub], reinterpret_cast<unsigned *>(s_buf[sub]));
        // the op path: the tile's sorted ids and bins for the backward (a tile
        // staged straight from its id slab writes them in sum_fwd_sparse)
        if (A.bins_out && A.id_counts && !seg_rec) write_sorted_ids(A, tile, range.x, n, s_ids[sub]);
        sum_fwd_sparse<kMode, kIdx>(A, tile, range, n, s_buf[sub], init, by_ids, s_ids[sub], seg_rec,
                                    seg.head, spec0, spec1, spec2, seg.head ? A.spec_slots : 0,
                                    spec_id);
    } else {
        if (by_ids) {
            // ONE sort per tile, by wave 0, shared by both waves through LDS:
            // with id slabs wave 0 writes the sorted ids back over the very
            // slots a second sorting wave would still be reading
            __shared__ int s_n;
            if (w == 0) {
                const int ns = ((A.slab || (kIds && A.id_counts)) && n_all > seg.cap())
                                   ? wave_brute_tile_ids(A, tile, s_ids[sub])
                                   : wave_sorted_tile_ids(seg, n_all, s_ids[sub],
                                                          reinterpret_cast<unsigned *>(s_buf[sub]));
                if ((threadIdx.x & 63) == 0) s_n = ns;
            }
            __syncthreads();
            n = s_n;
            if (A.bins_out && A.id_counts && w == 0) write_sorted_ids(A, tile, range.x, n, s_ids[sub]);
        }
        if (ty * kTile + w * 8 >= A.img_h) return;  // band below the image
        sum_fwd_band<kMode, kIdx>(A, tile, w, range, n, s_buf[w], init, by_ids, s_ids[sub], seg_rec,
                                  seg.head, spec0, spec1, spec2);
    }
    if (kMode == kModeStamp && (threadIdx.x & 63) == 0) {
        long long *st = A.stamps + 4 * (size_t)tile;
        st[w == 0 ? 0 : 2] = t0;
        st[w == 0 ? 1 : 3] = stamp();
    }
}

// The single-frame render over id slabs (render_frames with one frame: CHW
// clamped planes, no final_idx, 1024-id slabs) -- the configs[1] render and
// the frame render of configs[2] -- as W one-tile waves per workgroup
// (production W = 2: workgroup b takes tiles 2b, 2b + 1) with a prologue of
// its own.  raster_sum_fwd_kernel<kModeSparseIds>'s tile: the same device
// functions (sum_fwd_sparse, wave_sorted_tile_ids, wave_brute_tile_ids) in the
// same order, so the same bits (tools/fbench.py checks every A/B pass's image
// against the first).  Measured against the generic kernel, interleaved on
// three boxes (profiles/r06/render_ids/): one wave per workgroup -0.65 us at
// 1080p / 10k; two -1.1 us at 10k (-9 %) and -1.2 to -1.5 us at the trained
// 50k frame (-6 %), frame time -1.0 to -1.3 us; four: the composite -1.5 us
// but 4.3 us between the projection's end and its start (the frame no
// faster); two with XCD runs of 16 tiles instead of pairs: equal.  K tiles
// per wave with every tile's loads issued before the first blends (K = 2, 4):
// slower (12.7 vs 12.0 us; 4: 26 vs 20 us per frame).  A/B knob 38 = 1: the
// generic kernel.
template <int W, bool kSplit>
__global__ __launch_bounds__(64 * W, 8) void raster_render_ids_kernel(SumFwdArgs A) {
    __shared__ float4 s_bufw[W][kSlice];
    __shared__ int s_idsw[W][kTilePix];
    const int lane = threadIdx.x & 63, w = W > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;
    float4 *s_buf = s_bufw[w];
    int *s_ids = s_idsw[w];
    // W one-tile waves per workgroup: workgroup b (XCD b % 8) takes tiles W b .. W b + W - 1
    const int tile = W == 1 ? xcd_runs<16>(blockIdx.x, A.ntiles) : (int)blockIdx.x * W + w;
    if (tile >= A.ntiles) return;
    // M, the count and slot `lane` in one round trip
    const bool no_loads = kDiag && (A.ablate & 16);  // diagnostic: the stores alone
    const int m_val = no_loads ? 1 : *A.m_dev;
    const int n_all = no_loads ? 0 : (int)__builtin_amdgcn_readfirstlane(A.id_counts[tile]);
    const int spec_id = no_loads ? 0 : A.ids_rw[(size_t)tile * kCarryCap + lane];
    long long t0 = 0;
    if (kIdStampMode<kModeSparseIds> && A.stamps) t0 = stamp();
    if (lane == 0) {
        A.id_counts_clear[tile] = 0u;  // the next frame's counts
        if (tile == 0 && A.meta_out) {
            A.meta_out[0] = m_val;
            A.meta_out[1] = 0;
        }
    }
    int n = n_all < kTilePix ? n_all : kTilePix;
    // rasterize_sum.py:121-127: a frame without intersections is the background
    float3 init = make_float3(0.f, 0.f, 0.f);
    if (m_val < 1) {
        n = 0;
        init = make_float3(A.bg[0], A.bg[1], A.bg[2]);
    }
    if (kIdStampMode<kModeSparseIds> && A.stamps && lane == 0) {
        A.stamps[8 * (size_t)tile] = t0;
        A.stamps[8 * (size_t)tile + 5] = m_val < 1 ? 0 : n_all;
    }
    const int2 range = make_int2(tile * kCarryCap, tile * kCarryCap + n);
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    if (n <= kChunk) {
        // <= 64 entries: the records gathered by id and ranked into the staging
        sum_fwd_sparse<kModeSparseIds, false, kSplit>(A, tile, range, n, s_buf, init, false, s_ids,
                                              n > 0 ? A.rec : nullptr, nullptr, z, z, z, 0, spec_id);
        return;
    }
    SegIds seg;
    seg.ids = A.ids_rw + (size_t)tile * kCarryCap;
    seg.cap_ids = kCarryCap;
    seg.recs = nullptr;
    seg.head = nullptr;
    n = n_all > kCarryCap ? wave_brute_tile_ids(A, tile, s_ids)
                          : wave_sorted_tile_ids(seg, n_all, s_ids, reinterpret_cast<unsigned *>(s_buf));
    sum_fwd_sparse<kModeSparseIds, false, kSplit>(A, tile, range, n, s_buf, init, true, s_ids, nullptr, nullptr, z,
                                          z, z, 0, spec_id);
}

__device__ __forceinline__ int ceil_log2(int n) { return n <= 1 ? 0 : 32 - __clz(n - 1); }

// v_out element (row i, column j, channel c) at v_out[i * h + j * w + c * c_]
// (in floats): the HWC layout is {3 W, 3, 1}; the op path also takes the
// autograd engine's strided gradients as they come (e.g. channel planes after
// the caller's permute), without a copy.
struct VStrides {
    long long h, w, c;
};
__host__ __device__ inline VStrides hwc_strides(unsigned img_w) {
    return VStrides{3ll * (long long)img_w, 3ll, 1ll};
}

// det_off (deterministic backward, det.h): each (splat, tile) sum goes to
// det_part[9 * slot ...] instead of the record's atomics (slots past det_cap:
// atomics); det_radii: the splats' radii for the slot's bbox.
//
// Backward (backward.cu:696-862), round 5: a 128-thread workgroup (two waves)
// per tile, each wave over the rectangle rows of its own 8-row band -- the
// training tile kernel's per-row work items (rows.h).  Per chunk of 64 of the
// tile's first <= 256 sorted entries: the entries' records gathered by id
// with their alpha >= 1/255 rectangle of tile pixels (ellipse_rect: a pair
// outside contributes nothing in the reference either); work items = one
// rectangle row of an entry in the band, laid out longest first; each lane
// walks its item's pixels accumulating the row sums S_k = sum v_sigma dx^k
// (k = 0, 1, 2: v_xy and v_conic factor by the row's constant dy), the colour
// sums alpha * v_out and v_opacity = sum vis * v_alpha; a DPP segmented scan
// adds an entry's items in a fixed tree order and the run's last lane adds the
// run into the entry's LDS sums (fixed order, no LDS atomics); the two bands'
// sums go to the splat's record with one 9-lane atomic request per (splat,
// tile).  final_idx (kFinal, when the caller passes one): the reference's
// per-pixel skip of entries k > final_idx[p] (backward.cu:783-786), the pixel's
// bound staged in LDS beside its v_out; without one (the op path's C++ Function,
// whose forward writes none) the bound is the one this library's own forward
// implies -- an entry past a pixel's last contributor fails the alpha test
// there in the same op sequence -- so nothing is read.  Entries past the tile's
// 256th are skipped as there (final_idx < range.x + 256).
// Round 4's entry-per-thread kernel (each thread looping over E pixels with
// the skip, 9 block reductions per entry) is raster_sum_bwd_kernel_r4 below,
// in the diagnostic library only (A/B knob 29 = 1).
constexpr int kSBChunk = 64;
constexpr int kSBThreads = 128;
struct SumBwdLds {
    float v[3][kTile * kVRow];          // v_out planes (rows padded to kVRow words)
    float4 geo[kSBChunk];               // x, y, a/2, b
    float4 col[kSBChunk];               // c/2, opacity, r, g
    float blu[kSBChunk];                // b
    unsigned short ro[kSBChunk];        // alpha >= 1/255 rectangle (ellipse_rect)
    int gid[kSBChunk];                  // splat id
    float part[2][9][kSBChunk];         // per wave: the entries' 9 sums of its band
    signed char own[kSBThreads];        // per wave: the entry of the round's first items
    signed char perm[kSBThreads];       // per wave: the chunk's entries by item length
};
struct SumBwdLdsFinal : SumBwdLds {
    int fi[kTile * kVRow];              // final_idx (kFinal), rows as v's
};

// kOpac false (GSVC_BWD_NO_OPACITY: the caller's opacity takes no gradient, as
// GSVC's constant ones): the v_opacity sum is neither formed nor stored, so a
// (splat, tile) request covers the record's first 32 bytes only.
template <bool kFinal, bool kOpac>
__global__ __launch_bounds__(kSBThreads, 8) void raster_sum_bwd_kernel(
    int tbx, int img_w, int img_h, int ntiles, const int *__restrict__ ids,
    const int2 *__restrict__ bins, const float2 *__restrict__ xys, const float *__restrict__ conics,
    const float *__restrict__ colors, const float *__restrict__ opac,
    const int *__restrict__ final_idx, const float *__restrict__ v_out, VStrides vs,
    float *__restrict__ grad, const int *__restrict__ det_off, const int *__restrict__ det_radii,
    float *__restrict__ det_part, long long det_cap) {
    __shared__ std::conditional_t<kFinal, SumBwdLdsFinal, SumBwdLds> S;
    const int tile = xcd_remap(blockIdx.x, ntiles);
    const int ty = tile / tbx, tx = tile - ty * tbx;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const float tx0 = (float)(tx * kTile), ty0 = (float)(ty * kTile);
    const int2 range = bins[tile];
    const int n = min(max(range.y - range.x, 0), kTilePix);
    // the lane's pixel pair of its band: v_out into the planes (0 outside the
    // image, where no item reaches)
    {
        const int prow = 8 * w + (lane >> 3), pcol = (lane & 7) << 1;
        const int pi = ty * kTile + prow, pj = tx * kTile + pcol;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            float a = 0.f, b = 0.f, c = 0.f;
            if (n > 0 && pi < img_h && pj + q < img_w) {
                const float *v = v_out + (long long)pi * vs.h + (long long)(pj + q) * vs.w;
                a = v[0];
                b = v[vs.c];
                c = v[2 * vs.c];
            }
            S.v[0][prow * kVRow + pcol + q] = a;
            S.v[1][prow * kVRow + pcol + q] = b;
            S.v[2][prow * kVRow + pcol + q] = c;
            if constexpr (kFinal)
                S.fi[prow * kVRow + pcol + q] =
                    n > 0 && pi < img_h && pj + q < img_w ? final_idx[(size_t)pi * img_w + pj + q] : 0;
        }
    }
    if (n == 0) return;  // (block-uniform)
    const int y_lo = 8 * w, y_hi = 8 * w + 7;
    float *eacc = &S.part[w][0][0];
    signed char *wown = S.own + w * 64;
    signed char *wperm = S.perm + w * 64;
    const int tby = (img_h + kTile - 1) / kTile;
    for (int c0 = 0; c0 < n; c0 += kSBChunk) {
        const int gn = min(kSBChunk, n - c0);
        __syncthreads();  // the previous chunk's flush has read the staging
        if (tid < gn) {
            const int g = ids[range.x + c0 + tid];
            const float2 xy = xys[g];
            const float a = conics[3 * g], b = conics[3 * g + 1], c = conics[3 * g + 2];
            const float o = opac[g];
            S.geo[tid] = make_float4(xy.x, xy.y, 0.5f * a, b);
            S.col[tid] = make_float4(0.5f * c, o, colors[3 * g], colors[3 * g + 1]);
            S.blu[tid] = colors[3 * g + 2];
            S.gid[tid] = g;
            S.ro[tid] = (unsigned short)ellipse_rect(xy.x, xy.y, a, b, c, o, tx0, ty0);
        }
        __syncthreads();
        // work items of entry `lane` in this band: one per rectangle row
        int items = 0, ilen = 0;
        unsigned rc = kNoRect;
        if (lane < gn) {
            rc = S.ro[lane];
            if (rc != kNoRect) {
                const int ry0 = max((int)((rc >> 8) & 15u), y_lo), ry1 = min((int)((rc >> 12) & 15u), y_hi);
                if (ry0 <= ry1) {
                    items = ry1 - ry0 + 1;
                    ilen = (int)((rc >> 4) & 15u) - (int)(rc & 15u) + 1;
                }
            }
        }
        // the entries' items laid out longest first (four length classes, entry
        // order within a class): a round's 64 items have similar pixel loops;
        // each entry's items stay together, in row order
        {
            const unsigned long long below = (1ull << lane) - 1ull;
            int rank = 0, seen = 0;
            unsigned long long left = __ballot(true);
            const int cls = ilen >= 9 ? 3 : (ilen >= 7 ? 2 : (ilen >= 5 ? 1 : 0));
            for (int L = 3; L >= 0 && left; --L) {
                const unsigned long long m = __ballot(cls == L);
                if (cls == L) rank = seen + __popcll(m & below);
                seen += __popcll(m);
                left &= ~m;
            }
            wperm[rank] = (signed char)lane;
        }
        __builtin_amdgcn_wave_barrier();
        // unit opacity and bounded geometry for the whole chunk (GSVC's frames):
        // the alpha cut as the sigma threshold (common.h kSigmaCutBits)
        bool ok = true;
        if (lane < gn) {
            const float4 G = S.geo[lane], C = S.col[lane];
            ok = C.y == 1.0f && geo_bounded(G.x, G.y, G.z, G.w, C.x);
        }
        const bool bcut = __ballot(!ok) == 0ull;
        const int ent = wperm[lane];  // the entry in sorted slot `lane`
        const int sitems = __shfl(items, ent, 64);
        const int incl = wave_scan_dpp<false>(sitems, 0);
        const int off = incl - sitems;  // sorted slot `lane`'s first item
        const int total = __builtin_amdgcn_readlane(incl, 63);
#pragma unroll
        for (int c = 0; c < 9; ++c) eacc[c * kSBChunk + lane] = 0.0f;
        for (int base = 0; base < total; base += 64) {
            // the entry of item base + lane: the last entry whose first item is <= it
            wown[lane] = -1;
            __builtin_amdgcn_wave_barrier();
            if (sitems > 0 && off >= base && off < base + 64) wown[off - base] = (signed char)lane;
            const int straddle = __popcll(__ballot(lane < gn && off <= base)) - 1;
            __builtin_amdgcn_wave_barrier();
            int slot = max((int)wown[lane], straddle);
            slot = wave_scan_dpp<true>(slot, -2147483647 - 1);  // sorted slot of item base + lane
            const int item = base + lane;
            const int own = __shfl(ent, slot, 64);
            const int eoff = __shfl(off, slot, 64);
            const unsigned ro = (unsigned)__shfl((int)rc, own, 64);
            float g[9];
#pragma unroll
            for (int c = 0; c < 9; ++c) g[c] = 0.0f;
            if (item < total) {
                const float4 G = S.geo[own], C = S.col[own];
                const float bl = S.blu[own];
                const int row = max((int)((ro >> 8) & 15u), y_lo) + (item - eoff);
                const int cs = (int)(ro & 15u);
                const int ce = min((int)((ro >> 4) & 15u), img_w - 1 - (int)tx0);
                const float pyf = ty0 + (float)row;
                if ((int)pyf < img_h) {
                    const float dy = G.y - pyf;
                    const float cq = (C.x * dy) * dy;  // splat_sigma_h's row terms
                    const float bdy = G.w * dy;
                    // dy is constant along the row, so the per-pixel sums of
                    // backward.cu:822-848 factor: v_conic = 1/2 (S2, dy S1, dy^2 S0),
                    // v_xy = (a S1 + b dy S0, b S1 + c dy S0), S_k = sum v_sigma dx^k
                    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
                    const float *vp = &S.v[0][0] + row * kVRow + cs;
                    const float *const ve = &S.v[0][0] + row * kVRow + ce;
                    float px = tx0 + (float)cs;
                    // kFinal: the entry's sorted index against each pixel's bound
                    const int kk = range.x + c0 + own;
                    const int *fp = nullptr;
                    if constexpr (kFinal) fp = &S.fi[0] + row * kVRow + cs;
                    auto walk = [&](auto kcut) {
                        for (; vp <= ve; ++vp, px += 1.0f) {
                            if constexpr (kFinal) {
                                if (kk > *fp++) continue;
                            }
                            const float Px = vp[0], Py = vp[kTile * kVRow], Pz = vp[2 * kTile * kVRow];
                            const float dx = G.x - px;  // the forward's own dx
                            const float sgm = fmaf(fmaf(G.z, dx, bdy), dx, cq);
                            const float vis = exp_neg(sgm);
                            float al;
                            if constexpr (decltype(kcut)::value) {
                                // (the training tile kernel's select in place of this
                                // branch was measured here, round 6: 41.8-42.3 vs
                                // 41.2-41.3 us, profiles/r06/select_cut/op_*; not kept)
                                if (__float_as_uint(sgm) > kSigmaCutBits) continue;
                                al = vis;  // opacity 1
                            } else {
                                al = fminf(1.0f, C.y * vis);
                                if (sgm < 0.0f || al < kAlphaMin) continue;
                            }
                            const float v_alpha = fmaf(bl, Pz, fmaf(C.w, Py, C.z * Px));
                            const float v_sigma = (-C.y * vis) * v_alpha;
                            g[5] = fmaf(al, Px, g[5]);
                            g[6] = fmaf(al, Py, g[6]);
                            g[7] = fmaf(al, Pz, g[7]);
                            if constexpr (kOpac) g[8] = fmaf(vis, v_alpha, g[8]);
                            s0 += v_sigma;
                            const float vdx = v_sigma * dx;
                            s1 += vdx;
                            s2 = fmaf(vdx, dx, s2);
                        }
                    };
                    if (bcut)
                        walk(std::true_type{});
                    else
                        walk(std::false_type{});
                    const float hdy = 0.5f * dy;
                    g[0] = fmaf(2.0f * G.z, s1, bdy * s0);
                    g[1] = fmaf(G.w, s1, ((2.0f * C.x) * dy) * s0);
                    g[2] = 0.5f * s2;
                    g[3] = hdy * s1;
                    g[4] = (hdy * dy) * s0;
                }
            }
            // an entry has at most 8 rows in a band: runs of <= 8 lanes
            if constexpr (kOpac)
                wave_seg_sums<9, false>(g, own);
            else
                wave_seg_sums<8, false>(*reinterpret_cast<float(*)[8]>(&g[0]), own);
            const int own_next = __shfl_down(own, 1, 64);
            if (item < total && (lane == 63 || item + 1 == total || own_next != own)) {
#pragma unroll
                for (int c = 0; c < (kOpac ? 9 : 8); ++c) eacc[c * kSBChunk + own] += g[c];
            }
            __builtin_amdgcn_wave_barrier();
        }
        __syncthreads();
        // 16 lanes per entry, 9 of them add band 0 + band 1 of one sum into the
        // splat's 64-byte record: one memory request per (splat, tile)
        for (int q = tid; q < gn * 16; q += kSBThreads) {
            const int e = q >> 4, c = q & 15;
            if (c >= (kOpac ? 9 : 8)) continue;
            const float v = S.part[0][c][e] + S.part[1][c][e];
            if (det_off) {
                const long long slot = det_slot(det_off, xys, det_radii, S.gid[e], tx, ty, tbx, tby);
                if (slot < det_cap) {
                    det_part[9 * slot + c] = v;
                    continue;
                }
            }
            unsafeAtomicAdd(grad + (size_t)S.gid[e] * 16 + c, v);
        }
    }
}

#ifdef GSVC_DIAG
// Round 4's op-path backward (diagnostic library, A/B knob 29 = 1): one
// 256-thread workgroup per tile, entry-parallel (below).
__global__ __launch_bounds__(256) void raster_sum_bwd_kernel_r4(
    int tbx, int img_w, int img_h, int ntiles, const int *__restrict__ ids,
    const int2 *__restrict__ bins, const float2 *__restrict__ xys, const float *__restrict__ conics,
    const float *__restrict__ colors, const float *__restrict__ opac,
    const int *__restrict__ final_idx, const float *__restrict__ v_out, VStrides vs,
    float *__restrict__ grad, const int *__restrict__ det_off, const int *__restrict__ det_radii,
    float *__restrict__ det_part, long long det_cap) {
    __shared__ float4 s_pix[kTilePix];  // v_out rgb, final_idx bits
    __shared__ float4 s_geo[kTilePix];  // x, y, a, b
    __shared__ float4 s_col[kTilePix];  // c, opacity, r, g
    __shared__ float s_blu[kTilePix];
    __shared__ int s_gid[kTilePix];
    __shared__ float s_red[9][kTilePix];
    __shared__ int s_max[4];
    const int tile = xcd_remap(blockIdx.x, ntiles);
    const int ty = tile / tbx, tx = tile - ty * tbx;
    const int tid = threadIdx.x;
    const int pi = ty * kTile + (tid >> 4), pj = tx * kTile + (tid & 15);
    const bool inside = pi < img_h && pj < img_w;
    float4 pd = make_float4(0.f, 0.f, 0.f, __int_as_float(-2147483647 - 1));
    if (inside) {
        const size_t p = (size_t)pi * (size_t)img_w + (size_t)pj;
        const float *v = v_out + (long long)pi * vs.h + (long long)pj * vs.w;
        pd = make_float4(v[0], v[vs.c], v[2 * vs.c], __int_as_float(final_idx[p]));
    }
    s_pix[tid] = pd;
    int f = __float_as_int(pd.w);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) f = max(f, __shfl_xor(f, off, 64));
    if ((tid & 63) == 0) s_max[tid >> 6] = f;
    __syncthreads();
    const int maxf = max(max(s_max[0], s_max[1]), max(s_max[2], s_max[3]));
    const int2 range = bins[tile];
    const int kend = min(range.y, maxf == (-2147483647 - 1) ? maxf : maxf + 1);
    const float tx0 = (float)(tx * kTile), ty0 = (float)(ty * kTile);

    for (int cs = range.x; cs < kend; cs += kTilePix) {
        const int n = min(kTilePix, kend - cs);
        if (tid < n) {
            const int g = ids[cs + tid];
            s_gid[tid] = g;
            const float2 xy = xys[g];
            s_geo[tid] = make_float4(xy.x, xy.y, conics[3 * g], conics[3 * g + 1]);
            s_col[tid] = make_float4(conics[3 * g + 2], opac[g], colors[3 * g], colors[3 * g + 1]);
            s_blu[tid] = colors[3 * g + 2];
        }
        __syncthreads();
        const int lg = ceil_log2(n);
        const int E = 1 << lg;
        const int e = tid & (E - 1);
        const int p_begin = (tid >> lg) << lg;  // E pixels per group
        float a_r = 0.f, a_g = 0.f, a_b = 0.f, a_c0 = 0.f, a_c1 = 0.f, a_c2 = 0.f;
        float a_x = 0.f, a_y = 0.f, a_o = 0.f;
        if (e < n) {
            const int k = cs + e;
            const float4 G = s_geo[e];
            const float4 C = s_col[e];
            const float bl = s_blu[e];
            const float ha = 0.5f * G.z, hc = 0.5f * C.x;
            for (int pp = 0; pp < E; ++pp) {
                const int p = p_begin + pp;
                const float4 P = s_pix[p];
                if (k > __float_as_int(P.w)) continue;
                const float dx = G.x - (tx0 + (float)(p & 15));
                const float dy = G.y - (ty0 + (float)(p >> 4));
                const float s = splat_sigma_h(ha, G.w, hc, dx, dy);
                const float vis = exp_neg(s);
                const float al = fminf(1.0f, C.y * vis);
                if (s < 0.0f || al < kAlphaMin) continue;
                const float v_alpha = fmaf(bl, P.z, fmaf(C.w, P.y, C.z * P.x));
                const float v_sigma = (-C.y * vis) * v_alpha;
                a_r = fmaf(al, P.x, a_r);
                a_g = fmaf(al, P.y, a_g);
                a_b = fmaf(al, P.z, a_b);
                const float hs = 0.5f * v_sigma;
                const float hsdx = hs * dx;
                a_c0 = fmaf(hsdx, dx, a_c0);
                a_c1 = fmaf(hsdx, dy, a_c1);
                a_c2 = fmaf(hs * dy, dy, a_c2);
                a_x = fmaf(v_sigma, fmaf(G.z, dx, G.w * dy), a_x);
                a_y = fmaf(v_sigma, fmaf(G.w, dx, C.x * dy), a_y);
                a_o = fmaf(vis, v_alpha, a_o);
            }
        }
        // combine the 256/E pixel groups of each entry
        if (E < 64) {
            for (int off = 32; off >= E; off >>= 1) {
                a_r += __shfl_xor(a_r, off, 64);
                a_g += __shfl_xor(a_g, off, 64);
                a_b += __shfl_xor(a_b, off, 64);
                a_c0 += __shfl_xor(a_c0, off, 64);
                a_c1 += __shfl_xor(a_c1, off, 64);
                a_c2 += __shfl_xor(a_c2, off, 64);
                a_x += __shfl_xor(a_x, off, 64);
                a_y += __shfl_xor(a_y, off, 64);
                a_o += __shfl_xor(a_o, off, 64);
            }
        }
        const int S = E < 64 ? 64 : E;
        if (E >= 64 || (tid & 63) < E) {
            s_red[0][tid] = a_x;
            s_red[1][tid] = a_y;
            s_red[2][tid] = a_c0;
            s_red[3][tid] = a_c1;
            s_red[4][tid] = a_c2;
            s_red[5][tid] = a_r;
            s_red[6][tid] = a_g;
            s_red[7][tid] = a_b;
            s_red[8][tid] = a_o;
        }
        __syncthreads();
        if (tid < n) {
            const int reps = kTilePix / S;
#pragma unroll
            for (int c = 0; c < 9; ++c) {
                float v = s_red[c][tid];
                for (int j = 1; j < reps; ++j) v += s_red[c][tid + j * S];
                s_red[c][tid] = v;
            }
        }
        __syncthreads();
        // 16 lanes per entry, 9 of them add one float each into the splat's
        // 64-byte gradient record: one memory request per (splat, tile).
        for (int q = tid; q < n * 16; q += kTilePix) {
            const int e2 = q >> 4, c = q & 15;
            if (c >= 9) continue;
            if (det_off) {
                const int tby = (img_h + kTile - 1) / kTile;
                const long long slot = det_slot(det_off, xys, det_radii, s_gid[e2], tx, ty, tbx, tby);
                if (slot < det_cap) {
                    det_part[9 * slot + c] = s_red[c][e2];
                    continue;
                }
            }
            unsafeAtomicAdd(grad + (size_t)s_gid[e2] * 16 + c, s_red[c][e2]);
        }
        __syncthreads();
    }
}

#endif

// Deterministic backward: splat i's record = its slots summed in bbox order +
// the atomics of slots past det_cap (zero unless the capacity was short).
__global__ __launch_bounds__(256) void det_gather_kernel(int n, const int *__restrict__ off,
                                                         const float *__restrict__ part,
                                                         long long cap, float *__restrict__ grad) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const long long b = off[i], e = min((long long)off[i + 1], cap);
    float s[9];
#pragma unroll
    for (int c = 0; c < 9; ++c) s[c] = 0.0f;
    for (long long k = b; k < e; ++k) {
#pragma unroll
        for (int c = 0; c < 9; ++c) s[c] += part[9 * k + c];
    }
    float *g = grad + 16 * (size_t)i;
#pragma unroll
    for (int c = 0; c < 9; ++c) g[c] = s[c] + g[c];
}

static int check_tiles(const char *what, int bx, int by, int tbx, int tby, unsigned w, unsigned h) {
    if (bx != kTile || by != kTile)
        return set_error(GSVC_ERR_ARG, "%s: only 16x16 tiles are supported (got %dx%d)", what, bx, by);
    if (tbx != ceil_div((int)w, kTile) || tby != ceil_div((int)h, kTile))
        return set_error(GSVC_ERR_ARG, "%s: tile_bounds (%d,%d) do not match image %ux%u", what, tbx,
                         tby, w, h);
    return GSVC_OK;
}

// Op path binning in one kernel (gsvc_rasterize_sum_forward_slabs): every
// visible splat appends its id to the 256-slot id slab of each tile of its
// bbox (slot = device atomic count, paired for adjacent tiles; ids past 256
// dropped, the composite rebuilds such a tile), the block's hit total goes
// into this call's M, and -- optionally -- the splat's gradient record is
// zeroed for the backward's atomics.  Replaces utils.py:99-167's cumsum,
// map, sort and bin edges (and this library's count / scan / fill /
// segment-sort kernels): the composite sorts each tile's <= 256 ids in LDS.
__global__ __launch_bounds__(kProjThreads) void tile_insert_ids_kernel(
    int n, const float2 *__restrict__ xys, const int *__restrict__ radii, int tbx, int tby,
    unsigned *__restrict__ counts, int *__restrict__ ids, int *__restrict__ m_acc,
    int *__restrict__ m_clear, float4 *__restrict__ rec_zero, int ids_cap) {
    __shared__ int s_hits[kProjThreads / 64];
    const int i = blockIdx.x * kProjThreads + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x == 0) *m_clear = 0;  // the next call's M
    int hits = 0;
    if (i < n) {
        if (rec_zero) {
            const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int q = 0; q < 4; ++q) rec_zero[4 * (size_t)i + q] = z;
        }
        const int r = radii[i];
        if (r > 0) {
            const float2 c = xys[i];
            const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
            hits = slab_insert_pairs<8>(c.x, c.y, r, tbx, tby, z, z,
                                        make_float4(0.f, __int_as_float(i), 0.f, 0.f), counts,
                                        nullptr, 0, ids, ids_cap);
        }
    }
    add_hits(hits, s_hits, m_acc);
}

// Splat i's 48-byte record for the composite's gather (the frame path's
// layout: {x, y, a/2, b}, {c/2, opacity, r, g}, {b, id, a, c}): one record per
// entry instead of eight scattered loads.
__device__ __forceinline__ void pack_record(int i, const float2 *__restrict__ xys,
                                            const float *__restrict__ conics,
                                            const float *__restrict__ colors,
                                            const float *__restrict__ opac, float4 *__restrict__ rec) {
    const float2 c = xys[i];
    const float a = conics[3 * (size_t)i], b = conics[3 * (size_t)i + 1], cc = conics[3 * (size_t)i + 2];
    rec[3 * (size_t)i] = make_float4(c.x, c.y, 0.5f * a, b);
    rec[3 * (size_t)i + 1] = make_float4(0.5f * cc, opac[i], colors[3 * (size_t)i], colors[3 * (size_t)i + 1]);
    rec[3 * (size_t)i + 2] = make_float4(colors[3 * (size_t)i + 2], __int_as_float(i), a, cc);
}

// The same insertion with a splat order (gsvc_rasterize_sum_forward_slabs_ordered):
// lane t inserts splat order[t] (NULL: t), and the workgroup -- spatially
// coherent once ``order`` sorts the splats by their centre's tile strip --
// takes its slots window-wise (frame_dev.h slab_insert_window: one device
// atomic per touched tile of the block's window instead of one per (splat,
// tile)).  The slabs hold the same ids per tile either way; the composite
// sorts them.  ``key`` (the refresh call): each splat's strip key and id for
// the next order.
template <int kThr>
__global__ __launch_bounds__(kThr) void tile_insert_ids_ordered_kernel(
    int n, const int *__restrict__ order, const float2 *__restrict__ xys,
    const int *__restrict__ radii, int tbx, int tby, unsigned *__restrict__ counts,
    int *__restrict__ ids, int *__restrict__ m_acc, int *__restrict__ m_clear,
    float4 *__restrict__ rec_zero, unsigned *__restrict__ key, int *__restrict__ key_id,
    unsigned key_invisible, const float *__restrict__ conics, const float *__restrict__ colors,
    const float *__restrict__ opac, float4 *__restrict__ rec, int scatter, int ids_cap) {
    __shared__ int s_hits[kThr / 64];
    __shared__ unsigned s_cnt[kAggWin];
    __shared__ int s_box[4][kThr / 64];
    const int t = blockIdx.x * kThr + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x == 0) *m_clear = 0;  // the next call's M
    const int i = t < n ? (order ? order[t] : t) : n;
    const bool have = (unsigned)i < (unsigned)n;  // (an unsorted order buffer: nothing)
    SplatOut S;
    S.P.xy = make_float2(0.f, 0.f);
    S.P.rad = 0;
    S.r0 = S.r1 = make_float4(0.f, 0.f, 0.f, 0.f);
    S.r2 = make_float4(0.f, __int_as_float(i), 0.f, 0.f);  // the id (slab_insert_window's ids)
    unsigned x0 = 0, y0 = 0, x1 = 0, y1 = 0;
    // the gradient records' zeroing, the 48-byte records and the strip keys go
    // by position t, not by the ordered id i: every id in [0, n) is some t's,
    // and the stores are coalesced (A/B knob 32 = 1: at i, scattered)
    const bool by_pos = !(kDiag && scatter);
    if (by_pos && t < n) {
        if (rec_zero) {
            const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int q = 0; q < 4; ++q) rec_zero[4 * (size_t)t + q] = z;
        }
        if (rec) pack_record(t, xys, conics, colors, opac, rec);
        if (key) {
            const float2 c = xys[t];
            key[t] = strip_key(c.x, c.y, radii[t], tbx, tby, key_invisible);
            key_id[t] = t;
        }
    }
    if (have) {
        if (!by_pos && rec_zero) {
            const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int q = 0; q < 4; ++q) rec_zero[4 * (size_t)i + q] = z;
        }
        const int r = radii[i];
        const float2 c = xys[i];
        S.P.xy = c;
        S.P.rad = r;
        if (r > 0) tile_bbox(c.x, c.y, (float)r, tbx, tby, x0, y0, x1, y1);
        if (!by_pos && rec) pack_record(i, xys, conics, colors, opac, rec);
        if (!by_pos && key) {
            key[i] = strip_key(c.x, c.y, r, tbx, tby, key_invisible);
            key_id[i] = i;
        }
    }
    // every lane of the block (block-uniform control flow inside)
    const int hits = slab_insert_window<kThr>(S, x0, y0, x1, y1, tbx, tby, counts, nullptr, s_cnt,
                                              s_box, nullptr, ids, ids_cap);
    add_hits<kThr>(hits, s_hits, m_acc);
}

// The op path's splat-order buffers (n-sized): strip keys and ids, the sorted
// keys and the order, the sort's scratch and counters.
struct OpOrderWs {
    unsigned *okey, *skey, *kbuf;
    int *okey_id, *order, *vbuf;
    float4 *rec;  // the splats' 48-byte records (the ordered insertion writes them)
    unsigned *sort_counts, *sort_offsets;
    size_t bytes;
};
static OpOrderWs op_order_ws(char *base, int n) {
    OpOrderWs w;
    size_t off = 0;
    const size_t nn = (size_t)(n > 0 ? n : 1);
    auto take = [&](size_t b) {
        char *p = base ? base + off : nullptr;
        off += ws_align(b);
        return p;
    };
    w.okey = (unsigned *)take(sizeof(unsigned) * nn);
    w.skey = (unsigned *)take(sizeof(unsigned) * nn);
    w.kbuf = (unsigned *)take(sizeof(unsigned) * nn);
    w.okey_id = (int *)take(sizeof(int) * nn);
    w.order = (int *)take(sizeof(int) * nn);
    w.vbuf = (int *)take(sizeof(int) * nn);
    const size_t cb = sort_u32_counts_bytes(n > 0 ? n : 1);
    w.sort_counts = (unsigned *)take(cb);
    w.sort_offsets = (unsigned *)take(cb);
    w.rec = (float4 *)take(sizeof(float4) * 3 * nn);
    w.bytes = off;
    return w;
}

bool sum_forward_dense(int density_hint, int ntiles, int frames) {
    if (knob(0) != 0) return knob(0) != kModeSparse;  // a forced kernel mode (A/B): no id slabs
    return (long long)density_hint > (long long)kDenseEntriesPerTile * ntiles * frames;
}

void sum_fwd_args_init(SumFwdArgs &A) {
    A = SumFwdArgs{};
    A.sparse_max = knob(3) > 0 ? knob(3) : 8;
    // A/B knob 10: speculative slab records per tile (default all kHeadSlots)
    A.spec_slots = knob(10) > 0 && knob(10) < kHeadSlots ? knob(10) : kHeadSlots;
    A.group_min = knob(15) > 0 ? knob(15) - 1 : kGroupMinDefault;
    A.cut = knob(19) != 1;
    A.ids_cap = kTilePix;
    A.xcd_off = knob(37);
    A.ablate = knob(36);
    A.layout = kLayoutHWC;
    A.frames = 1;
}

// A timed launch carries its HIP events in the dispatch (timing.hip, how = 1);
// every other launch is a plain one.
template <typename K>
static void launch_fwd(K kernel, dim3 grid, dim3 block, hipStream_t s, const hipEvent_t *tev,
                       const SumFwdArgs &A) {
    if (tev[0])
        hipExtLaunchKernelGGL(kernel, grid, block, 0, s, tev[0], tev[1], 0, A);
    else
        hipLaunchKernelGGL(kernel, grid, block, 0, s, A);
}

int sum_forward_launch(SumFwdArgs &A, int density_hint, hipStream_t s) {
    A.vec = (A.img_w % 4 == 0) && (((uintptr_t)A.out & 15) == 0) &&
            (((uintptr_t)A.final_idx & 15) == 0) && (((uintptr_t)A.final_Ts & 15) == 0);
    A.vec_chw = A.vec && (((size_t)A.img_w * (size_t)A.img_h) % 4 == 0);
    A.store_policy = knob(7);  // kStoreNtSc1 unless an A/B run selects another (knob 7)
    const int ntiles = A.ntiles;
    int mode = knob(0);
    if (mode == 0) mode = sum_forward_dense(density_hint, ntiles, A.frames) ? kModeBanded : kModeSparse;
    if (knob(17) == 1 && mode == kModeSparse) mode = kModeSparsePrio;  // A/B knob 17
    // id slabs without final_idx (the render; the op path's forward, whose
    // backward needs no final_idx): the one-wave id-slab instance, or the
    // banded kernel for a dense op-path frame
    if (A.id_counts && !A.final_idx && mode != kModeBanded) mode = kModeSparseIds;
    if (mode == kModeStamp && A.layout != kLayoutHWC)
        return set_error(GSVC_ERR_ARG, "rasterize_sum_forward: stamp mode needs the HWC layout");
    if (A.frames > 1 && (mode == kModeStamp || mode == kModeSparseStamp))
        return set_error(GSVC_ERR_ARG, "rasterize_sum_forward: stamp modes render one frame");
    hipEvent_t tev[2];
    const int tslot = timing_begin(s, tev);
    const dim3 grid(ntiles * A.frames);
    if (mode == kModeSparse) {
        launch_fwd(A.final_idx ? raster_sum_fwd_kernel<kModeSparse, true>
                               : raster_sum_fwd_kernel<kModeSparse, false>,
                   grid, dim3(64), s, tev, A);
    } else if (mode == kModeBanded) {
        launch_fwd(A.final_idx ? raster_sum_fwd_kernel<kModeBanded, true>
                               : raster_sum_fwd_kernel<kModeBanded, false>,
                   grid, dim3(128), s, tev, A);
    } else if (mode == kModeSparseIds) {
        if (kDiag && knob(39) == 1 && A.frames == 1) A.stamps = reinterpret_cast<long long *>(debug_ptr());
        // the single-frame render: two one-tile waves per workgroup (A/B knob 38 = 1:
        // the generic kernel)
        const bool render = A.frames == 1 && !A.bins_out && !A.final_idx && A.m_dev &&
                            A.ids_cap == kCarryCap && A.layout == kLayoutCHWClamped && A.rec && A.sort_ids;
        if (render && knob(38) != 1) {
            // more than 8 entries per tile on average: the split-loop instance
            if ((long long)density_hint > 8ll * A.ntiles)
                launch_fwd(raster_render_ids_kernel<2, true>, dim3((A.ntiles + 1) / 2), dim3(128), s, tev, A);
            else
                launch_fwd(raster_render_ids_kernel<2, false>, dim3((A.ntiles + 1) / 2), dim3(128), s, tev, A);
        }
        else
            launch_fwd(raster_sum_fwd_kernel<kModeSparseIds, false>, grid, dim3(64), s, tev, A);
    } else if constexpr (kDiag) {
        // diagnostic variants (libgsvc_amd_diag.so only)
        switch (mode) {
            case kModeStamp:
                A.stamps = reinterpret_cast<long long *>(A.final_Ts);
                A.final_Ts = nullptr;
                launch_fwd(A.final_idx ? raster_sum_fwd_kernel<kModeStamp, true> : raster_sum_fwd_kernel<kModeStamp, false>, grid,
                           dim3(128), s, tev, A);
                break;
            case kModeNoBlend:
                launch_fwd(A.final_idx ? raster_sum_fwd_kernel<kModeNoBlend, true> : raster_sum_fwd_kernel<kModeNoBlend, false>, grid,
                           dim3(128), s, tev, A);
                break;
            case kModeNoStore:
                launch_fwd(A.final_idx ? raster_sum_fwd_kernel<kModeNoStore, true> : raster_sum_fwd_kernel<kModeNoStore, false>, grid,
                           dim3(128), s, tev, A);
                break;
            case kModeAdaptive:
                launch_fwd(A.final_idx ? raster_sum_fwd_kernel<kModeAdaptive, true> : raster_sum_fwd_kernel<kModeAdaptive, false>, grid,
                           dim3(128), s, tev, A);
                break;
            case kModeSparseStamp:
                if (!debug_ptr())
                    return set_error(GSVC_ERR_ARG, "rasterize_sum_forward: mode 7 needs gsvc_debug_set_ptr");
                A.stamps = reinterpret_cast<long long *>(debug_ptr());
                launch_fwd(A.final_idx ? raster_sum_fwd_kernel<kModeSparseStamp, true> : raster_sum_fwd_kernel<kModeSparseStamp, false>, grid,
                           dim3(64), s, tev, A);
                break;
            case kModeSparsePrio:
                launch_fwd(A.final_idx ? raster_sum_fwd_kernel<kModeSparsePrio, true>
                                       : raster_sum_fwd_kernel<kModeSparsePrio, false>,
                           grid, dim3(64), s, tev, A);
                break;
            default:
                return set_error(GSVC_ERR_ARG, "rasterize_sum_forward: unknown kernel mode %d", mode);
        }
    }
    timing_end(s, tslot);
    return check_launch("rasterize_sum_forward");
}

}  // namespace gsvc

using namespace gsvc;

extern "C" int gsvc_rasterize_sum_forward_ex(
    int tbx, int tby, int tbz, int block_x, int block_y, int block_z, unsigned img_width,
    unsigned img_height, unsigned img_depth, const int *gaussian_ids_sorted, const int *tile_bins,
    const float *xys, const float *conics, const float *colors, const float *opacities,
    const float *background, const int *num_intersects_dev, int density_hint, int out_layout,
    float *out_img, float *final_Ts, int *final_idx, void *stream) {
    (void)tbz; (void)block_z; (void)img_depth;
    int rc = check_tiles("rasterize_sum_forward", block_x, block_y, tbx, tby, img_width, img_height);
    if (rc) return rc;
    if (out_layout != kLayoutHWC && !layout_planes(out_layout))
        return set_error(GSVC_ERR_ARG, "rasterize_sum_forward: unknown output layout %d", out_layout);
    if (num_intersects_dev && !background)
        return set_error(GSVC_ERR_ARG, "rasterize_sum_forward: background required with a device count");
    const int ntiles = tbx * tby;
    if (ntiles == 0) return GSVC_OK;
    SumFwdArgs A;
    sum_fwd_args_init(A);
    A.tbx = tbx;
    A.img_w = (int)img_width;
    A.img_h = (int)img_height;
    A.ntiles = ntiles;
    A.layout = out_layout;
    A.m_dev = num_intersects_dev;
    A.bg = background;
    A.ids = gaussian_ids_sorted;
    A.bins = (const int2 *)tile_bins;
    A.xys = (const float2 *)xys;
    A.conics = conics;
    A.colors = colors;
    A.opac = opacities;
    A.out = out_img;
    A.final_idx = final_idx;
    A.final_Ts = final_Ts;
    return sum_forward_launch(A, density_hint, (hipStream_t)stream);
}

extern "C" int gsvc_rasterize_sum_forward(int tbx, int tby, int tbz, int block_x, int block_y,
                                          int block_z, unsigned img_width, unsigned img_height,
                                          unsigned img_depth, const int *gaussian_ids_sorted,
                                          const int *tile_bins, const float *xys, const float *conics,
                                          const float *colors, const float *opacities,
                                          const float *background, float *out_img, float *final_Ts,
                                          int *final_idx, void *stream) {
    // without the intersection count the sparse path is the safe default
    return gsvc_rasterize_sum_forward_ex(tbx, tby, tbz, block_x, block_y, block_z, img_width,
                                         img_height, img_depth, gaussian_ids_sorted, tile_bins, xys,
                                         conics, colors, opacities, background, nullptr, 0, kLayoutHWC,
                                         out_img, final_Ts, final_idx, stream);
}

extern "C" size_t gsvc_rasterize_sum_slabs_workspace_bytes(int num_tiles) {
    // counts [2][T] and the M slots [2]: two parities, used on alternate calls
    return sizeof(unsigned) * (2 * (size_t)(num_tiles > 0 ? num_tiles : 0) + 2);
}

static int forward_slabs_impl(
    int num_points, const float *xys, const int *radii, const float *conics, const float *colors,
    const float *opacities, const float *background, unsigned img_height, unsigned img_width,
    int call_index, int density_hint, void *workspace, size_t workspace_bytes,
    int *gaussian_ids, int *tile_bins, int *meta, float *grad_records_zero, float *out_img,
    int *final_idx, void *stream, void *order_ws, size_t order_ws_bytes, int order_flags) {
    if (num_points < 0 || img_height == 0 || img_width == 0)
        return set_error(GSVC_ERR_ARG, "rasterize_sum_forward_slabs: bad sizes");
    const int tbx = ceil_div((int)img_width, kTile), tby = ceil_div((int)img_height, kTile);
    const int ntiles = tbx * tby;
    if (!workspace || workspace_bytes < gsvc_rasterize_sum_slabs_workspace_bytes(ntiles))
        return set_error(GSVC_ERR_WORKSPACE, "rasterize_sum_forward_slabs: workspace too small");
    if (!gaussian_ids || !tile_bins || !meta || !out_img || !background ||
        (num_points > 0 && (!xys || !radii || !conics || !colors || !opacities)))
        return set_error(GSVC_ERR_ARG, "rasterize_sum_forward_slabs: missing input");
    hipStream_t s = (hipStream_t)stream;
    if (const int rc = refuse_capture(s, "rasterize_sum_forward_slabs")) return rc;
    const int par = call_index & 1;
    unsigned *counts = (unsigned *)workspace;
    int *m_slots = (int *)(counts + 2 * (size_t)ntiles);
    const bool ordered = order_ws && (order_flags & (GSVC_TRAIN_ORDER | GSVC_TRAIN_ORDER_REFRESH));
    // GSVC_SLABS_WIDE: gaussian_ids holds kCarryCap ids per tile (a tile of up
    // to 1024 entries sorts its first 256 from them; past that, the bbox rebuild)
    const int ids_cap = (order_flags & GSVC_SLABS_WIDE) ? kCarryCap : kTilePix;
    OpOrderWs ow{};
    if (ordered) {
        ow = op_order_ws((char *)order_ws, num_points);
        if (order_ws_bytes < ow.bytes)
            return set_error(GSVC_ERR_WORKSPACE, "rasterize_sum_forward_slabs_ordered: order workspace too small");
    }
    if (num_points > 0 && ordered) {
        const bool refresh = (order_flags & GSVC_TRAIN_ORDER_REFRESH) != 0;
        // (128 and 512 threads per workgroup measured, round 5: no gain)
        constexpr int thr = kProjThreads;
        auto kfn = tile_insert_ids_ordered_kernel<kProjThreads>;
        hipLaunchKernelGGL(kfn, dim3(ceil_div(num_points, thr)), dim3(thr), 0, s, num_points,
                           (order_flags & GSVC_TRAIN_ORDER) ? (const int *)ow.order : nullptr,
                           (const float2 *)xys, radii, tbx, tby, counts + (size_t)par * ntiles,
                           gaussian_ids, m_slots + par, m_slots + (par ^ 1),
                           (float4 *)grad_records_zero, refresh ? ow.okey : nullptr,
                           refresh ? ow.okey_id : nullptr, strip_key_invisible(tbx, tby), conics,
                           colors, opacities, ow.rec, knob(32), ids_cap);
    } else if (num_points > 0) {
        hipLaunchKernelGGL(tile_insert_ids_kernel, dim3(ceil_div(num_points, kProjThreads)),
                           dim3(kProjThreads), 0, s, num_points, (const float2 *)xys, radii, tbx,
                           tby, counts + (size_t)par * ntiles, gaussian_ids, m_slots + par,
                           m_slots + (par ^ 1), (float4 *)grad_records_zero, ids_cap);
    } else if (dev_zero(m_slots, 2 * sizeof(int), s) != GSVC_OK) {
        return set_error(GSVC_ERR_HIP, "rasterize_sum_forward_slabs: memset failed");
    }
    SumFwdArgs A;
    sum_fwd_args_init(A);
    A.tbx = tbx;
    A.img_w = (int)img_width;
    A.img_h = (int)img_height;
    A.ntiles = ntiles;
    A.layout = (order_flags & GSVC_SLABS_PLANES) ? kLayoutCHW : kLayoutHWC;
    A.m_dev = m_slots + par;
    A.meta_out = meta;
    A.bg = background;
    A.sort_ids = true;
    A.id_counts = counts + (size_t)par * ntiles;
    A.id_counts_clear = counts + (size_t)(par ^ 1) * ntiles;
    A.ids_rw = gaussian_ids;
    A.ids_cap = ids_cap;
    A.bins_out = (int2 *)tile_bins;
    A.cull_xys = (const float2 *)xys;
    A.cull_radii = radii;
    A.num_points = num_points;
    A.xys = (const float2 *)xys;
    A.conics = conics;
    A.colors = colors;
    A.opac = opacities;
    // the ordered insertion packs each splat's record: the composite gathers one
    // 48-byte record per entry, as the frame render does
    A.rec = (ordered && num_points > 0) ? ow.rec : nullptr;
    A.out = out_img;
    A.final_idx = final_idx;
    const int rc = sum_forward_launch(A, density_hint, s);
    if (rc || !ordered || !(order_flags & GSVC_TRAIN_ORDER_REFRESH) || num_points <= 0) return rc;
    // the next calls' order: splat ids by strip key (stable)
    return sort_u32_pairs(num_points, ow.okey, ow.okey_id, ow.skey, ow.order, ow.kbuf, ow.vbuf,
                          strip_key_bits(tbx, tby), ow.sort_counts, ow.sort_offsets, s);
}

extern "C" int gsvc_rasterize_sum_forward_slabs(
    int num_points, const float *xys, const int *radii, const float *conics, const float *colors,
    const float *opacities, const float *background, unsigned img_height, unsigned img_width,
    int call_index, int density_hint, void *workspace, size_t workspace_bytes,
    int *gaussian_ids, int *tile_bins, int *meta, float *grad_records_zero, float *out_img,
    int *final_idx, void *stream) {
    return forward_slabs_impl(num_points, xys, radii, conics, colors, opacities, background,
                              img_height, img_width, call_index, density_hint, workspace,
                              workspace_bytes, gaussian_ids, tile_bins, meta, grad_records_zero,
                              out_img, final_idx, stream, nullptr, 0, 0);
}

extern "C" size_t gsvc_rasterize_sum_order_workspace_bytes(int num_points) {
    return op_order_ws(nullptr, num_points).bytes;
}

extern "C" int gsvc_rasterize_sum_forward_slabs_ordered(
    int num_points, const float *xys, const int *radii, const float *conics, const float *colors,
    const float *opacities, const float *background, unsigned img_height, unsigned img_width,
    int call_index, int density_hint, void *workspace, size_t workspace_bytes,
    int *gaussian_ids, int *tile_bins, int *meta, float *grad_records_zero, float *out_img,
    int *final_idx, void *stream, void *order_workspace, size_t order_workspace_bytes,
    int order_flags) {
    if (order_flags & ~(GSVC_TRAIN_ORDER | GSVC_TRAIN_ORDER_REFRESH | GSVC_SLABS_WIDE | GSVC_SLABS_PLANES))
        return set_error(GSVC_ERR_ARG, "rasterize_sum_forward_slabs_ordered: unknown flags");
    if ((order_flags & (GSVC_TRAIN_ORDER | GSVC_TRAIN_ORDER_REFRESH)) && !order_workspace)
        return set_error(GSVC_ERR_WORKSPACE, "rasterize_sum_forward_slabs_ordered: no order workspace");
    return forward_slabs_impl(num_points, xys, radii, conics, colors, opacities, background,
                              img_height, img_width, call_index, density_hint, workspace,
                              workspace_bytes, gaussian_ids, tile_bins, meta, grad_records_zero,
                              out_img, final_idx, stream, order_workspace, order_workspace_bytes,
                              order_flags);
}

// The op-path backward's launch (every backward entry point): the row-item
// kernel, timed on channel kTimingSumBwd; the diagnostic library's knob 29 = 1
// launches round 4's kernel instead (A/B).
static void sum_bwd_launch(hipStream_t s, int tbx, int img_w, int img_h, int ntiles,
                           const int *ids, const int2 *bins, const float2 *xys, const float *conics,
                           const float *colors, const float *opac, const int *final_idx,
                           const float *v_out, VStrides vs, float *grad, const int *det_off,
                           const int *det_radii, float *det_part, long long det_cap, int flags = 0) {
    hipEvent_t tev[2];
    const int tslot = timing_begin(s, tev, kTimingSumBwd);
#ifdef GSVC_DIAG
    if (knob(29) == 1) {
        launch_timed(raster_sum_bwd_kernel_r4, dim3(ntiles), dim3(256), 0, s, tev, tbx, img_w, img_h,
                     ntiles, ids, bins, xys, conics, colors, opac, final_idx, v_out, vs, grad, det_off,
                     det_radii, det_part, det_cap);
        timing_end(s, tslot, kTimingSumBwd);
        return;
    }
#endif
    // the deterministic slots always carry all 9 sums (det_gather reads them)
    const bool opac_grad = !(flags & GSVC_BWD_NO_OPACITY) || det_off;
    auto k = final_idx ? (opac_grad ? raster_sum_bwd_kernel<true, true> : raster_sum_bwd_kernel<true, false>)
                       : (opac_grad ? raster_sum_bwd_kernel<false, true> : raster_sum_bwd_kernel<false, false>);
    launch_timed(k, dim3(ntiles), dim3(kSBThreads), 0, s, tev, tbx, img_w, img_h, ntiles, ids, bins, xys,
                 conics, colors, opac, final_idx, v_out, vs, grad, det_off, det_radii, det_part, det_cap);
    timing_end(s, tslot, kTimingSumBwd);
}

extern "C" int gsvc_rasterize_sum_backward_zeroed_strided_ex(
    unsigned img_height, unsigned img_width, int num_points, const int *gaussian_ids_sorted,
    const int *tile_bins, const float *xys, const float *conics, const float *colors,
    const float *opacities, const int *final_idx, const float *v_output, long long v_stride_h,
    long long v_stride_w, long long v_stride_c, float *grad_records, void *stream, int flags) {
    const VStrides vs{v_stride_h, v_stride_w, v_stride_c};
    const int tbx = ceil_div((int)img_width, kTile), tby = ceil_div((int)img_height, kTile);
    if (num_points < 0)
        return set_error(GSVC_ERR_ARG, "rasterize_sum_backward_zeroed_strided: bad num_points");
    const int ntiles = tbx * tby;
    if (ntiles == 0 || num_points == 0) return GSVC_OK;
    sum_bwd_launch((hipStream_t)stream, tbx, (int)img_width, (int)img_height, ntiles,
                   gaussian_ids_sorted, (const int2 *)tile_bins, (const float2 *)xys, conics, colors,
                   opacities, final_idx, v_output, vs, grad_records, nullptr, nullptr, nullptr, 0ll, flags);
    return check_launch("rasterize_sum_backward_zeroed_strided");
}

extern "C" int gsvc_rasterize_sum_backward_zeroed_strided(
    unsigned img_height, unsigned img_width, int num_points, const int *gaussian_ids_sorted,
    const int *tile_bins, const float *xys, const float *conics, const float *colors,
    const float *opacities, const int *final_idx, const float *v_output, long long v_stride_h,
    long long v_stride_w, long long v_stride_c, float *grad_records, void *stream) {
    return gsvc_rasterize_sum_backward_zeroed_strided_ex(
        img_height, img_width, num_points, gaussian_ids_sorted, tile_bins, xys, conics, colors,
        opacities, final_idx, v_output, v_stride_h, v_stride_w, v_stride_c, grad_records, stream, 0);
}

extern "C" int gsvc_rasterize_sum_backward_zeroed(
    unsigned img_height, unsigned img_width, int num_points, const int *gaussian_ids_sorted,
    const int *tile_bins, const float *xys, const float *conics, const float *colors,
    const float *opacities, const int *final_idx, const float *v_output, float *grad_records,
    void *stream) {
    const VStrides vs = hwc_strides(img_width);
    return gsvc_rasterize_sum_backward_zeroed_strided(
        img_height, img_width, num_points, gaussian_ids_sorted, tile_bins, xys, conics, colors,
        opacities, final_idx, v_output, vs.h, vs.w, vs.c, grad_records, stream);
}

extern "C" int gsvc_rasterize_sum_backward(unsigned img_height, unsigned img_width, unsigned block_h,
                                           unsigned block_w, int num_points,
                                           const int *gaussian_ids_sorted, const int *tile_bins,
                                           const float *xys, const float *conics, const float *colors,
                                           const float *opacities, const float *background,
                                           const float *final_Ts, const int *final_idx,
                                           const float *v_output, const float *v_output_alpha,
                                           float *grad_records, void *stream) {
    (void)background; (void)final_Ts; (void)v_output_alpha;
    const int tbx = ceil_div((int)img_width, (int)block_w), tby = ceil_div((int)img_height, (int)block_h);
    int rc = check_tiles("rasterize_sum_backward", (int)block_w, (int)block_h, tbx, tby, img_width,
                         img_height);
    if (rc) return rc;
    if (num_points < 0) return set_error(GSVC_ERR_ARG, "rasterize_sum_backward: bad num_points");
    hipStream_t s = (hipStream_t)stream;
    if (num_points > 0 &&
        dev_zero(grad_records, sizeof(float) * 16 * (size_t)num_points, s) != GSVC_OK)
        return set_error(GSVC_ERR_HIP, "rasterize_sum_backward: memset failed");
    const int ntiles = tbx * tby;
    if (ntiles == 0 || num_points == 0) return GSVC_OK;
    sum_bwd_launch(s, tbx, (int)img_width, (int)img_height, ntiles, gaussian_ids_sorted,
                   (const int2 *)tile_bins, (const float2 *)xys, conics, colors, opacities, final_idx,
                   v_output, hwc_strides(img_width), grad_records, nullptr, nullptr, nullptr, 0ll);
    return check_launch("rasterize_sum_backward");
}

extern "C" size_t gsvc_rasterize_sum_backward_det_workspace_bytes(int num_points,
                                                                  long long det_capacity) {
    const size_t nn = (size_t)(num_points > 0 ? num_points : 0);
    const size_t cap = (size_t)(det_capacity > 0 ? det_capacity : 0);
    return 256 * ((sizeof(int) * (nn + 1) + 255) / 256) + sizeof(float) * 9 * cap;
}

extern "C" int gsvc_rasterize_sum_backward_det(
    unsigned img_height, unsigned img_width, unsigned block_h, unsigned block_w, int num_points,
    const int *gaussian_ids_sorted, const int *tile_bins, const float *xys, const float *conics,
    const float *colors, const float *opacities, const int *radii, const int *final_idx,
    const float *v_output, float *grad_records, void *det_workspace, size_t det_workspace_bytes,
    long long det_capacity, int *pairs_out, void *stream) {
    const int tbx = ceil_div((int)img_width, (int)block_w), tby = ceil_div((int)img_height, (int)block_h);
    int rc = check_tiles("rasterize_sum_backward_det", (int)block_w, (int)block_h, tbx, tby,
                         img_width, img_height);
    if (rc) return rc;
    if (num_points < 0 || det_capacity < 0)
        return set_error(GSVC_ERR_ARG, "rasterize_sum_backward_det: bad sizes");
    if (!radii || !det_workspace ||
        det_workspace_bytes < gsvc_rasterize_sum_backward_det_workspace_bytes(num_points, det_capacity))
        return set_error(GSVC_ERR_WORKSPACE, "rasterize_sum_backward_det: missing radii or workspace");
    hipStream_t s = (hipStream_t)stream;
    if (num_points > 0 &&
        dev_zero(grad_records, sizeof(float) * 16 * (size_t)num_points, s) != GSVC_OK)
        return set_error(GSVC_ERR_HIP, "rasterize_sum_backward_det: memset failed");
    const int ntiles = tbx * tby;
    if (ntiles == 0 || num_points == 0) return GSVC_OK;
    int *off = (int *)det_workspace;
    float *part = (float *)((char *)det_workspace + 256 * ((sizeof(int) * ((size_t)num_points + 1) + 255) / 256));
    // (the block totals live in part until its memset below)
    det_offsets_launch(num_points, (const float2 *)xys, radii, tbx, tby, off, (int *)part,
                       9 * (size_t)det_capacity, s);
    if (det_capacity > 0 &&
        dev_zero(part, sizeof(float) * 9 * (size_t)det_capacity, s) != GSVC_OK)
        return set_error(GSVC_ERR_HIP, "rasterize_sum_backward_det: memset failed");
    sum_bwd_launch(s, tbx, (int)img_width, (int)img_height, ntiles, gaussian_ids_sorted,
                   (const int2 *)tile_bins, (const float2 *)xys, conics, colors, opacities, final_idx,
                   v_output, hwc_strides(img_width), grad_records, off, radii, part, det_capacity);
    hipLaunchKernelGGL(det_gather_kernel, dim3(ceil_div(num_points, 256)), dim3(256), 0, s,
                       num_points, off, part, det_capacity, grad_records);
    if (pairs_out &&
        dev_copy(pairs_out, off + num_points, sizeof(int), s) != GSVC_OK)
        return set_error(GSVC_ERR_HIP, "rasterize_sum_backward_det: copy failed");
    return check_launch("rasterize_sum_backward_det");
}
