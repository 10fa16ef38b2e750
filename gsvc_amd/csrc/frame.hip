// Whole-frame render of GSVC's per-frame model, one C call, two kernels (gfx950).
//
// Reference: GaussianSplats_Represent.py:57-90 (parameter activations and
// forward), i.e. for each frame
//     means2d = tanh(_xyz); L = _cholesky + cholesky_bound;
//     colors = _features_dc * rgb_W; opacity = 1
//     project_gaussians_2d -> rasterize_gaussians_sum -> clamp -> NCHW
// (foward2d.cu:12-69, utils.py:99-167, forward.cu:512-627).
//
// The rasterizer reads only the first <= 256 entries of each tile in splat-id
// order (forward.cu:569-571,613), so the frame path needs no global sort and
// no scan:
//   frame_project_kernel  activations + projection (project2d.h, the op's own
//                         op sequence) + a 48-byte record per splat (its id
//                         in a spare lane); each visible splat appends its
//                         record to a fixed 256-slot slab per tile it touches
//                         (slot = atomic count; records past 256 dropped) and
//                         the block-reduced tile count goes into this frame's M;
//   raster_sum_fwd_kernel loads a tile's count and first 8 records in one
//                         round trip, ranks <= 64 records by id straight into
//                         its LDS staging (longer slabs: LDS bitmap sort of
//                         the ids; more than 256 entries: the first 256 ids
//                         rebuilt by scanning every splat's bbox in id order),
//                         blends, and writes the clamped [3,H,W] planes.
// Counts and M live in two parity slots used on alternate frames
// (frame_index & 1): each frame clears the other parity, which the previous
// frame has finished with.  Nothing is read back to the host.
#include "frame_dev.h"
#include "raster_sum.h"

namespace gsvc {

// Append splat i's record to the slab of tiles sub, sub + K, ... of its bbox
// (row-major), one of the K lanes of the splat; the slot atomics are issued in
// batches of 8 before their results are waited for.
template <int K>
__device__ __forceinline__ int slab_insert(float cx, float cy, int r, int tbx, int tby, int sub,
                                           float4 r0, float4 r1, float4 r2,
                                           unsigned *__restrict__ counts,
                                           float4 *__restrict__ slab, int wt,
                                           int *__restrict__ ovf) {
    unsigned x0, y0, x1, y1;
    tile_bbox(cx, cy, (float)r, tbx, tby, x0, y0, x1, y1);
    if (x1 <= x0 || y1 <= y0) return 0;
    const int ntiles = tbx * tby;
    const unsigned bw = x1 - x0;
    constexpr int kBatch = 8;
    unsigned tl[kBatch];
    int cnt = 0, hits = 0;
    auto flush = [&]() {
        unsigned sl[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; ++k)
            if (k < cnt) sl[k] = atomicAdd(counts + tl[k], 1u);
#pragma unroll
        for (int k = 0; k < kBatch; ++k)
            if (k < cnt && sl[k] >= (unsigned)kTilePix && sl[k] < (unsigned)kCarryCap && ovf) {
                ovf[(size_t)tl[k] * kOvfSlots + (sl[k] - kTilePix)] = __float_as_int(r2.y);
            } else if (k < cnt && sl[k] < (unsigned)kTilePix) {
                float4 *d = slab_rec(slab, ntiles, (int)tl[k], (int)sl[k]);
                if (kDiag && (wt & 1)) {
                    store_wt(d, r0);
                    store_wt(d + 1, r1);
                    store_wt(d + 2, r2);
                } else {
                    d[0] = r0;
                    d[1] = r1;
                    d[2] = r2;
                }
            }
        hits += cnt;
        cnt = 0;
    };
    unsigned y = y0 + (unsigned)sub / bw, x = x0 + (unsigned)sub % bw;
    while (y < y1) {
        tl[cnt < kBatch ? cnt : 0] = y * (unsigned)tbx + x;
        if (++cnt == kBatch) flush();
        x += K;
        while (x >= x1) {
            x -= bw;
            ++y;
        }
    }
    if (cnt) flush();
    return hits;
}

// K lanes per splat: each computes the (cheap) projection, lane s writes part
// of the splat's outputs and inserts every K-th tile of its bbox (K = 1 in
// production: more lanes did not shorten the insertion, see the launcher).


// Diagnostic only (gsvc_debug_set(5, 1) with gsvc_debug_set_ptr): s_memrealtime
// (100 MHz) stamps per wave -- start, projected, inserted, end -- as int64[4].
__device__ __forceinline__ long long proj_stamp() {
    long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

template <int K, bool kStamp>
__global__ __launch_bounds__(kProjThreads) void frame_project_kernel(
    int n, const float *__restrict__ xyz, int xyz_tanh, const float *__restrict__ chol,
    const float *__restrict__ chol_bound, const float *__restrict__ feat,
    const float *__restrict__ rgb_w, const float *__restrict__ opac, float hw, float hh, int tbx,
    int tby, float2 *__restrict__ xys, int *__restrict__ radii, float4 *__restrict__ rec,
    unsigned *__restrict__ counts, float4 *__restrict__ slab, int *__restrict__ m_acc,
    int *__restrict__ m_clear, float4 *__restrict__ grad_zero, long long *stamps,
    const int *__restrict__ frame_off, int counts_stride, int m_stride, size_t slab_stride,
    int wt, int *__restrict__ ids, int *__restrict__ ovf) {
    __shared__ int s_hits[kProjThreads / 64];
    // batched frames (grid.y): this block's frame owns splats [begin, end)
    int begin = 0, end = n;
    if (frame_off) {
        const int b = blockIdx.y;
        begin = frame_off[b];
        end = frame_off[b + 1];
        counts += (size_t)b * counts_stride;
        slab += b * slab_stride;
        if (ids) ids += 4 * b * slab_stride;  // id slabs in the frame's slab memory
        if (ovf) ovf += (size_t)b * kOvfSlots * (size_t)(tbx * tby);
        m_acc += (size_t)b * m_stride;
        m_clear += (size_t)b * m_stride;
    }
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    long long *st = kStamp ? stamps + 4 * (size_t)(t >> 6) : nullptr;
    if (kStamp && (threadIdx.x & 63) == 0) st[0] = proj_stamp();
    const int i = begin + t / K, sub = t % K;
    if (blockIdx.x == 0 && threadIdx.x == 0) *m_clear = 0;  // the next frame's slot
    int hits = 0;
    if (i < end) {
        const SplatOut S = load_project(i, xyz, xyz_tanh, chol, chol_bound, feat, rgb_w, opac, hw,
                                        hh, tbx, tby);
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int q = sub; q < 4; q += K) {
            if (q < 3) {
                const float4 rq = q == 0 ? S.r0 : (q == 1 ? S.r1 : S.r2);
                if (kDiag && (wt & 1))
                    store_wt(rec + 3 * i + q, rq);
                else
                    rec[3 * i + q] = rq;
            }
            if (q == 3) {
                xys[i] = S.P.xy;
                radii[i] = S.P.rad;
            }
            if (grad_zero) grad_zero[4 * i + q] = z;
        }
        if (kStamp && (threadIdx.x & 63) == 0) st[1] = proj_stamp();
        if (S.P.rad > 0) {
            if (K == 1 && !(kDiag && (wt & 3)))  // paired atomics unless write-through / A/B knob 2 = 4
                hits = slab_insert_pairs<8>(S.P.xy.x, S.P.xy.y, S.P.rad, tbx, tby, S.r0, S.r1,
                                            S.r2, counts, slab, wt, ids, kCarryCap,
                                            ids ? nullptr : ovf);
            else
                hits = slab_insert<K>(S.P.xy.x, S.P.xy.y, S.P.rad, tbx, tby, sub, S.r0, S.r1,
                                      S.r2, counts, slab, wt, ovf);
        }
    }
    if (kStamp) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if ((threadIdx.x & 63) == 0) st[2] = proj_stamp();
    }
    add_hits(hits, s_hits, m_acc);
    if (kStamp) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if ((threadIdx.x & 63) == 0) st[3] = proj_stamp();
    }
}

// Ordered projection (single frame): lane t projects splat order[t], and the
// workgroup -- spatially coherent when ``order`` sorts splats by their
// centre's tile strip -- takes its slots window-wise: the bboxes of its small
// splats (<= kAggArea tiles) span a window of <= kAggWin tiles; it counts
// them per tile in LDS, takes ONE device-scope atomic per touched tile for
// the base, and hands out base + LDS cursor.  Large splats, and workgroups
// whose window is too large, insert directly as frame_project_kernel does.
// The slab then holds the same set of entries per tile (the order of slots
// within a tile is arbitrary either way: the consumers rank by id).
// ``key`` (optional): each splat's strip key and id, for the next order.
template <bool kStamp>
__global__ __launch_bounds__(kProjThreads) void frame_project_ordered_kernel(
    int n, const int *__restrict__ order, const float *__restrict__ xyz, int xyz_tanh,
    const float *__restrict__ chol, const float *__restrict__ chol_bound,
    const float *__restrict__ feat, const float *__restrict__ rgb_w,
    const float *__restrict__ opac, float hw, float hh, int tbx, int tby,
    float2 *__restrict__ xys, int *__restrict__ radii, float4 *__restrict__ rec,
    unsigned *__restrict__ counts, float4 *__restrict__ slab, int *__restrict__ m_acc,
    int *__restrict__ m_clear, float4 *__restrict__ grad_zero, unsigned *__restrict__ key,
    int *__restrict__ key_id, unsigned key_invisible, long long *stamps,
    int *__restrict__ carry_ids, uint2 *__restrict__ carry_box, uint2 *__restrict__ carry_hull,
    int *__restrict__ id_slab, int *__restrict__ ovf) {
    __shared__ int s_hits[kProjThreads / 64];
    __shared__ unsigned s_cnt[kAggWin];
    __shared__ int s_box[4][kProjThreads / 64];
    const int tid = threadIdx.x, lane = tid & 63;
    const int t = blockIdx.x * blockDim.x + tid;
    long long *st = kStamp ? stamps + 8 * (size_t)((blockIdx.x * blockDim.x + tid) >> 6) : nullptr;
    if (kStamp && lane == 0) st[0] = proj_stamp();
    if (blockIdx.x == 0 && tid == 0) *m_clear = 0;  // the next frame's slot
    const int i = t < n ? (order ? order[t] : t) : n;  // order NULL: identity
    // unsigned: an order entry outside [0, n) (a buffer never sorted) projects
    // nothing instead of indexing before the arrays (round-4 fault)
    const bool have = (unsigned)i < (unsigned)n;
    SplatOut S;
    S.P.rad = 0;
    unsigned x0 = 0, y0 = 0, x1 = 0, y1 = 0;
    if (have) {
        S = load_project(i, xyz, xyz_tanh, chol, chol_bound, feat, rgb_w, opac, hw, hh, tbx, tby);
        rec[3 * i] = S.r0;
        rec[3 * i + 1] = S.r1;
        rec[3 * i + 2] = S.r2;
        xys[i] = S.P.xy;
        radii[i] = S.P.rad;
        if (grad_zero) {
            const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int q = 0; q < 4; ++q) grad_zero[4 * i + q] = z;
        }
        if (key) {
            key[i] = strip_key(S.P.xy.x, S.P.xy.y, S.P.rad, tbx, tby, key_invisible);
            key_id[i] = i;
        }
        if (S.P.rad > 0) tile_bbox(S.P.xy.x, S.P.xy.y, (float)S.P.rad, tbx, tby, x0, y0, x1, y1);
        if (carry_ids) carry_box[i] = carry_hull[i] = pack_box(x0, y0, x1, y1);
    }
    if (kStamp && lane == 0) st[1] = proj_stamp();
    // ids in place of records: the carried bins' candidate lists, or the
    // render's id slabs (both 256 slots per tile)
    const int hits = slab_insert_window(S, x0, y0, x1, y1, tbx, tby, counts, slab, s_cnt, s_box, st,
                                        carry_ids ? carry_ids : id_slab,
                                        carry_ids ? kTrainCarryCap : kCarryCap,
                                        carry_ids || id_slab ? nullptr : ovf);
    if (kStamp) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) st[2] = proj_stamp();
    }
    add_hits(hits, s_hits, m_acc);
    if (kStamp) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) st[3] = proj_stamp();
    }
}

int strip_key_bits(int tbx, int tby) {
    const unsigned top = strip_key_invisible(tbx, tby);
    int b = 1;
    while (b < 32 && (top >> b) != 0u) ++b;
    return b;
}

FrameWs frame_ws(char *base, int n, int ntiles, int frames) {
    FrameWs w;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char *p = base ? base + off : nullptr;
        off += ws_align(bytes);
        return p;
    };
    const size_t nn = (size_t)(n > 0 ? n : 1), nt = (size_t)(ntiles > 0 ? ntiles : 1);
    const size_t nf = (size_t)(frames > 0 ? frames : 1);
    // first: counts[F][2][T] and the M slots [F][2], zeroed by the caller once;
    // call f counts into parity f & 1 while its rasterizer clears the other
    w.counts = (unsigned *)take(sizeof(unsigned) * 2 * nt * nf + 2 * nf * sizeof(int));
    w.m_slots = (int *)(w.counts + 2 * nt * nf);
    w.zeroed = sizeof(unsigned) * 2 * nt * nf + 2 * nf * sizeof(int);
    w.slab = (float4 *)take(sizeof(float4) * slab_frame_f4((int)nt) * nf);
    w.ovf = (int *)take(sizeof(int) * (size_t)kOvfSlots * nt * nf);
    w.xys = (float2 *)take(sizeof(float2) * nn);
    w.radii = (int *)take(sizeof(int) * nn);
    w.rec = (float4 *)take(sizeof(float4) * 3 * nn);
    w.okey = w.skey = w.kbuf = w.sort_counts = w.sort_offsets = nullptr;
    w.okey_id = w.order = w.vbuf = nullptr;
    if (nf == 1) {
        w.okey = (unsigned *)take(sizeof(unsigned) * nn);
        w.skey = (unsigned *)take(sizeof(unsigned) * nn);
        w.kbuf = (unsigned *)take(sizeof(unsigned) * nn);
        w.okey_id = (int *)take(sizeof(int) * nn);
        w.order = (int *)take(sizeof(int) * nn);
        w.vbuf = (int *)take(sizeof(int) * nn);
        const size_t cb = sort_u32_counts_bytes(n > 0 ? n : 1);
        w.sort_counts = (unsigned *)take(cb);
        w.sort_offsets = (unsigned *)take(cb);
    }
    w.bytes = off;
    return w;
}

int splat_order_sort(const FrameWs &w, int n, int tbx, int tby, hipStream_t s) {
    if (n <= 0) return GSVC_OK;
    if (!w.order) return set_error(GSVC_ERR_ARG, "splat order: a multi-frame workspace has none");
    // ids by strip key (stable: ties in id order)
    return sort_u32_pairs(n, w.okey, w.okey_id, w.skey, w.order, w.kbuf, w.vbuf,
                          strip_key_bits(tbx, tby), w.sort_counts, w.sort_offsets, s);
}

FrameSlots frame_slots(const FrameWs &w, int ntiles, int frame_index) {
    const int par = frame_index & 1;
    FrameSlots f;
    f.counts_stride = 2 * ntiles;
    f.m_stride = 2;
    f.m_acc = w.m_slots + par;
    f.m_clear = w.m_slots + (par ^ 1);
    f.counts = w.counts + (size_t)par * ntiles;
    f.counts_next = w.counts + (size_t)(par ^ 1) * ntiles;
    return f;
}

int frame_project_launch(int n, const float *xyz, int xyz_tanh, const float *chol,
                         const float *chol_bound, const float *feat, const float *rgb_w,
                         const float *opac, unsigned img_h, unsigned img_w, const FrameWs &w,
                         const FrameSlots &f, float4 *grad_zero, hipStream_t s, int frames,
                         const int *frame_off, int max_frame_n, const SplatOrder *ord,
                         int *id_slab) {
    const int tbx = ceil_div((int)img_w, kTile), tby = ceil_div((int)img_h, kTile);
    const float hw = 0.5f * (float)img_w, hh = 0.5f * (float)img_h;
    if (ord && frames == 1 && n > 0) {
        const dim3 grid(ceil_div(n, kProjThreads));
        if constexpr (kDiag) if (knob(5) == 1 && debug_ptr()) {  // diagnostic: per-wave stamps
            hipLaunchKernelGGL(frame_project_ordered_kernel<true>, grid, dim3(kProjThreads), 0, s, n,
                               ord->order, xyz, xyz_tanh, chol, chol_bound, feat, rgb_w, opac, hw,
                               hh, tbx, tby, w.xys, w.radii, w.rec,
                               ord->carry_ids ? ord->carry_counts : f.counts, w.slab, f.m_acc,
                               f.m_clear, grad_zero, ord->key, ord->key_id, strip_key_invisible(tbx, tby),
                               reinterpret_cast<long long *>(debug_ptr()), ord->carry_ids,
                               ord->carry_box, ord->carry_hull, id_slab, w.ovf);
            return check_launch("frame projection (ordered)");
        }
        hipEvent_t tev[2];
        const int tslot = timing_begin(s, tev, kTimingProject);
        launch_timed(frame_project_ordered_kernel<false>, grid, dim3(kProjThreads), 0, s, tev, n,
                     ord->order, xyz, xyz_tanh, chol, chol_bound, feat, rgb_w, opac, hw, hh, tbx,
                     tby, w.xys, w.radii, w.rec, ord->carry_ids ? ord->carry_counts : f.counts,
                     w.slab, f.m_acc, f.m_clear, grad_zero, ord->key, ord->key_id,
                     strip_key_invisible(tbx, tby), (long long *)nullptr, ord->carry_ids,
                     ord->carry_box, ord->carry_hull, id_slab, w.ovf);
        timing_end(s, tslot, kTimingProject);
        return check_launch("frame projection (ordered)");
    }
    // lanes per splat: 1 unless gsvc_debug_set(4, k) picks 2, 4 or 8 (A/B knob;
    // measured at 1080p: equal at 10k splats, 1 lane fastest at 50k)
    // id_slab (A/B knob 24): 4-byte ids instead of the 48-byte records, paired atomics
    const int k = !id_slab && (knob(4) == 2 || knob(4) == 4 || knob(4) == 8) ? knob(4) : 1;
    const size_t slab_stride = slab_frame_f4(tbx * tby);
    // plain record stores; A/B knob 6 = 1 writes them through (sc1): measured
    // slower (projection 7.1 -> 9.8 us at 10k: each scattered 16-byte sc1 store
    // is its own fabric write) and no faster for the composite's loads
    // bit 0: write-through record stores (A/B knob 6 = 1); bit 1: one 32-bit
    // slot atomic per tile instead of the pairs (A/B knob 2 = 4).  Measured
    // with the isolation runs of profiles/r01/paired_atomics/NOTES.md.
    const int wt = id_slab ? 0 : (knob(6) == 1 ? 1 : 0) | (knob(2) == 4 ? 2 : 0);
    if (frames > 1 && !frame_off) return set_error(GSVC_ERR_ARG, "frame projection: frame offsets");
    const int per = frames > 1 ? max_frame_n : n;
    if (frames > 1 && per <= 0) {
        // no splats anywhere: only the M slots (memset of the whole [F][2] block)
        if (dev_zero(f.m_acc < f.m_clear ? f.m_acc : f.m_clear, sizeof(int) * 2 * (size_t)frames, s) != GSVC_OK)
            return set_error(GSVC_ERR_HIP, "frame projection: memset failed");
        return check_launch("frame projection");
    }
    if (per > 0) {
        // workgroup size: 256 unless A/B knob 1 picks 64 or 128
        const int bs = knob(1) == 64 || knob(1) == 128 ? knob(1) : kProjThreads;
        const dim3 grid(ceil_div(per, bs / k), frames > 1 ? frames : 1);
#define GSVC_FRAME_PROJECT(K)                                                                    \
    {                                                                                            \
        hipEvent_t tev[2];                                                                       \
        const int tslot = timing_begin(s, tev, kTimingProject);                                  \
        launch_timed(frame_project_kernel<K, false>, grid, dim3(bs), 0, s, tev, n, xyz,          \
                     xyz_tanh, chol, chol_bound, feat, rgb_w, opac, hw, hh, tbx, tby, w.xys,     \
                     w.radii, w.rec, f.counts, w.slab, f.m_acc, f.m_clear, grad_zero,            \
                     (long long *)nullptr, frames > 1 ? frame_off : (const int *)nullptr,        \
                     f.counts_stride, f.m_stride, slab_stride, wt, id_slab, w.ovf);              \
        timing_end(s, tslot, kTimingProject);                                                    \
    }
        if constexpr (kDiag) if (knob(5) == 1 && debug_ptr()) {  // diagnostic: per-wave stamps
            auto kfn = frame_project_kernel<1, true>;
            hipLaunchKernelGGL(kfn, grid, dim3(bs), 0, s, n, xyz, xyz_tanh, chol,
                               chol_bound, feat, rgb_w, opac, hw, hh, tbx, tby, w.xys, w.radii,
                               w.rec, f.counts, w.slab, f.m_acc, f.m_clear, grad_zero,
                               reinterpret_cast<long long *>(debug_ptr()),
                               frames > 1 ? frame_off : nullptr, f.counts_stride, f.m_stride,
                               slab_stride, wt, id_slab, w.ovf);
            return check_launch("frame projection");
        }
        if constexpr (kDiag) {
            switch (k) {
                case 2: GSVC_FRAME_PROJECT(2); break;
                case 8: GSVC_FRAME_PROJECT(8); break;
                case 4: GSVC_FRAME_PROJECT(4); break;
                default: GSVC_FRAME_PROJECT(1); break;
            }
        } else {
            GSVC_FRAME_PROJECT(1);
        }
#undef GSVC_FRAME_PROJECT
    } else if (dev_zero(f.m_acc, sizeof(int), s) != GSVC_OK)
        return set_error(GSVC_ERR_HIP, "frame projection: memset failed");
    return check_launch("frame projection");
}

}  // namespace gsvc

using namespace gsvc;

namespace gsvc {

constexpr int kPlainProjMaxPerTile = 8;

// The one-call render of ``frames`` frames (frame b: splats [frame_off[b],
// frame_off[b + 1]), image out + b * 3HW); frames == 1: splats [0, n).
static int render_frames(int frames, const int *frame_off_host, const int *frame_off_dev,
                         int num_points, const float *xyz, int xyz_tanh, const float *cholesky,
                         const float *cholesky_bound, const float *features, const float *rgb_w,
                         const float *opacity, const float *background, unsigned img_height,
                         unsigned img_width, int frame_index, int density_hint, int *meta,
                         void *workspace, size_t workspace_bytes, float *out, hipStream_t s,
                         int flags = 0) {
    const int tbx = ceil_div((int)img_width, kTile), tby = ceil_div((int)img_height, kTile);
    const int ntiles = tbx * tby;
    const FrameWs w = frame_ws((char *)workspace, num_points, ntiles, frames);
    if (!workspace || workspace_bytes < w.bytes)
        return set_error(GSVC_ERR_WORKSPACE, "render_frame_sum: workspace too small (%zu < %zu)",
                         workspace_bytes, w.bytes);
    if (const int rc = refuse_capture(s, frames > 1 ? "render_frames_sum" : "render_frame_sum")) return rc;
    int max_n = num_points;
    if (frames > 1) {
        max_n = 0;
        for (int b = 0; b < frames; ++b) {
            const int nb = frame_off_host[b + 1] - frame_off_host[b];
            if (nb < 0 || frame_off_host[b] < 0 || frame_off_host[b + 1] > num_points)
                return set_error(GSVC_ERR_ARG, "render_frames_sum: bad frame offsets");
            max_n = nb > max_n ? nb : max_n;
        }
    }
    const FrameSlots f = frame_slots(w, ntiles, frame_index);
    // GSVC_TRAIN_ORDER / _REFRESH (single frame): the training path's splat order
    const bool use_order = frames == 1 && (flags & GSVC_TRAIN_ORDER) != 0;
    const bool refresh = frames == 1 && (flags & GSVC_TRAIN_ORDER_REFRESH) != 0 && num_points > 0;
    SplatOrder ord;
    ord.order = use_order ? w.order : nullptr;
    if (refresh) {
        ord.key = w.okey;
        ord.key_id = w.okey_id;
    }
    // A single sparse frame renders over id slabs: the projection appends each
    // splat's id (4 B) in place of its 48-byte record and the composite gathers
    // the records by id from w.rec (the slab memory holds T x kCarryCap ids: a
    // tile of up to 1024 entries sorts its first 256 from them).
    // Batched frames and dense frames (the banded kernel) keep the records;
    // A/B knob 24 = 1 (diagnostic library) too.
    int *id_slab = nullptr;
    if (!sum_forward_dense(density_hint, ntiles, frames) && knob(24) != 1 &&
        (frames == 1 || knob(25) == 1))  // A/B knob 25 = 1: batched frames too
        id_slab = reinterpret_cast<int *>(w.slab);
    // A sparse single frame (<= kPlainProjMaxPerTile entries per tile by the
    // hint) projects in id order with plain paired atomics: the windowed
    // atomics pay only where tiles are dense (fbench at 1080p / 10k: 6.7 vs
    // 7.9-8.4 us).  A refresh call still takes the ordered kernel, which writes
    // the strip keys its sort reads -- a refresh whose projection skipped them
    // sorted uninitialised keys and ids into the order, and the next ordered
    // call gathered splats through it (the round-4 fault).  Knob 27
    // = 1 keeps the order at any density (A/B).
    const bool plain = use_order && !refresh && knob(27) != 1 &&
                       (long long)density_hint <= (long long)kPlainProjMaxPerTile * ntiles;
    int rc = frame_project_launch(num_points, xyz, xyz_tanh, cholesky, cholesky_bound, features,
                                  rgb_w, opacity, img_height, img_width, w, f, nullptr, s, frames,
                                  frame_off_dev, max_n,
                                  ((use_order && !plain) || refresh) ? &ord : nullptr, id_slab);
    if (rc) return rc;
    SumFwdArgs A;
    sum_fwd_args_init(A);
    A.tbx = tbx;
    A.img_w = (int)img_width;
    A.img_h = (int)img_height;
    A.ntiles = ntiles;
    A.layout = kLayoutCHWClamped;
    A.m_dev = f.m_acc;
    A.meta_out = meta;
    A.bg = background;
    A.sort_ids = true;
    if (id_slab) {
        A.id_counts = f.counts;
        A.id_counts_clear = f.counts_next;
        A.ids_rw = id_slab;
        A.ids_cap = kCarryCap;  // 1024 ids per tile fit the tile's 12.4 KB of slab memory
    } else {
        A.slab = w.slab;
        A.slab_ovf = w.ovf;
        A.slab_counts = f.counts;
        A.slab_counts_clear = f.counts_next;
    }
    A.cull_xys = w.xys;
    A.cull_radii = w.radii;
    A.num_points = num_points;
    A.rec = w.rec;
    A.out = out;
    if (frames > 1) {
        A.frames = frames;
        A.frame_off = frame_off_dev;
        A.counts_stride = f.counts_stride;
        A.m_stride = f.m_stride;
        A.slab_stride = slab_frame_f4(ntiles);
        A.out_stride = (size_t)3 * img_width * img_height;
    }
    rc = sum_forward_launch(A, density_hint, s);
    if (rc || !refresh) return rc;
    return splat_order_sort(w, num_points, tbx, tby, s);
}

}  // namespace gsvc

extern "C" size_t gsvc_render_frames_workspace_bytes(int frames, int num_points,
                                                     unsigned img_height, unsigned img_width) {
    return frame_ws(nullptr, num_points, tiles_of(img_height, img_width), frames).bytes;
}

extern "C" size_t gsvc_render_frames_zeroed_bytes(int frames, unsigned img_height,
                                                  unsigned img_width) {
    return frame_ws(nullptr, 1, tiles_of(img_height, img_width), frames).zeroed;
}

extern "C" int gsvc_render_frames_sum(int frames, const int *frame_offsets_host,
                                      const int *frame_offsets_dev, const float *xyz, int xyz_tanh,
                                      const float *cholesky, const float *cholesky_bound,
                                      const float *features, const float *rgb_w,
                                      const float *opacity, const float *background,
                                      unsigned img_height, unsigned img_width, int call_index,
                                      int density_hint, int *meta, void *workspace,
                                      size_t workspace_bytes, float *out, void *stream) {
    if (frames < 1 || frames > 4096 || img_height == 0 || img_width == 0)
        return set_error(GSVC_ERR_ARG, "render_frames_sum: bad sizes");
    if (!frame_offsets_host || !frame_offsets_dev || !background || !meta || !out)
        return set_error(GSVC_ERR_ARG, "render_frames_sum: missing input");
    if (frame_offsets_host[0] != 0)
        return set_error(GSVC_ERR_ARG, "render_frames_sum: frame offsets must start at 0");
    const int n = frame_offsets_host[frames];
    if (n > 0 && (!xyz || !cholesky || !features))
        return set_error(GSVC_ERR_ARG, "render_frames_sum: missing input");
    return render_frames(frames, frame_offsets_host, frame_offsets_dev, n, xyz, xyz_tanh, cholesky,
                         cholesky_bound, features, rgb_w, opacity, background, img_height,
                         img_width, call_index, density_hint, meta, workspace, workspace_bytes, out,
                         (hipStream_t)stream);
}

extern "C" size_t gsvc_render_frame_workspace_bytes(int num_points, unsigned img_height,
                                                    unsigned img_width) {
    return frame_ws(nullptr, num_points, tiles_of(img_height, img_width)).bytes;
}

extern "C" size_t gsvc_render_frame_zeroed_bytes(unsigned img_height, unsigned img_width) {
    return frame_ws(nullptr, 1, tiles_of(img_height, img_width)).zeroed;
}

extern "C" int gsvc_render_frame_sum_ex(int num_points, const float *xyz, int xyz_tanh,
                                        const float *cholesky, const float *cholesky_bound,
                                        const float *features, const float *rgb_w,
                                        const float *opacity, const float *background,
                                        unsigned img_height, unsigned img_width, int frame_index,
                                        int density_hint, int *meta, void *workspace,
                                        size_t workspace_bytes, float *out, void *stream,
                                        int flags) {
    if (num_points < 0 || img_height == 0 || img_width == 0)
        return set_error(GSVC_ERR_ARG, "render_frame_sum: bad sizes");
    if ((num_points > 0 && (!xyz || !cholesky || !features)) || !background || !meta || !out)
        return set_error(GSVC_ERR_ARG, "render_frame_sum: missing input");
    if (flags & ~(GSVC_TRAIN_ORDER | GSVC_TRAIN_ORDER_REFRESH))
        return set_error(GSVC_ERR_ARG, "render_frame_sum_ex: unknown flags");
    return render_frames(1, nullptr, nullptr, num_points, xyz, xyz_tanh, cholesky, cholesky_bound,
                         features, rgb_w, opacity, background, img_height, img_width, frame_index,
                         density_hint, meta, workspace, workspace_bytes, out, (hipStream_t)stream,
                         flags);
}

extern "C" int gsvc_render_frame_sum(int num_points, const float *xyz, int xyz_tanh,
                                     const float *cholesky, const float *cholesky_bound,
                                     const float *features, const float *rgb_w,
                                     const float *opacity, const float *background,
                                     unsigned img_height, unsigned img_width, int frame_index,
                                     int density_hint, int *meta, void *workspace,
                                     size_t workspace_bytes, float *out, void *stream) {
    if (num_points < 0 || img_height == 0 || img_width == 0)
        return set_error(GSVC_ERR_ARG, "render_frame_sum: bad sizes");
    if ((num_points > 0 && (!xyz || !cholesky || !features)) || !background || !meta || !out)
        return set_error(GSVC_ERR_ARG, "render_frame_sum: missing input");
    return render_frames(1, nullptr, nullptr, num_points, xyz, xyz_tanh, cholesky, cholesky_bound,
                         features, rgb_w, opacity, background, img_height, img_width, frame_index,
                         density_hint, meta, workspace, workspace_bytes, out, (hipStream_t)stream);
}
