// Torch binding of the drop-in operator path (the ops GSVC's own files call).
//
// GSVC's GaussianSplats_Represent.py:83-90 calls, per frame and iteration,
// gsplat.project_gaussians_2d and gsplat.rasterize_sum.rasterize_gaussians_sum
// -- two autograd Functions in the reference (project_gaussians_2d.py:59-141,
// rasterize_sum.py:89-254), each a Python wrapper around the extension's ops.
// Here the same two Functions are C++ torch::autograd::Functions over the C
// ABI of libgsvc_amd.so (include/gsvc_amd.h): one Python -> C++ call per op in
// the forward, none in the backward (the autograd engine calls the C++ node),
// outputs from the PyTorch caching allocator, launches on the current stream.
// The Python wrappers (gsvc_amd/project_gaussians_2d.py, rasterize_sum.py)
// keep the reference's argument checks and route here; the general paths
// (sorted binning for non-zero depths, the deterministic backward) stay in
// their Python Functions.  Semantics are those of the Python Functions:
//   project: saves (L, radii, conics); radii and num_tiles_hit are
//            not differentiable; backward = the projection VJP (backward2d.cu).
//   rasterize_sum: two kernels (gsvc_rasterize_sum_forward_slabs): id slabs
//            per tile by device atomics, then the composite sorting each
//            tile's ids in LDS (its first 256 in (tile, splat id) order, M on
//            the device, the M < 1 background branch in the kernel) and
//            writing them back for the backward = backward.cu:696-862 into one
//            [N, 16] record zeroed by the forward (the returned gradients are
//            its views, which the projection backward reads in place).
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>
#include <torch/extension.h>

#include <algorithm>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <vector>

#include "../../include/gsvc_amd.h"

using at::Tensor;
using torch::autograd::AutogradContext;
using torch::autograd::variable_list;

namespace {

void check(int rc, const char *what) {
    TORCH_CHECK(rc == 0, what, " failed (status ", rc, "): ", gsvc_last_error());
}

void *stream_of(const Tensor &t) {
    return (void *)c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

Tensor dev_f32(const Tensor &t, const char *name) {
    TORCH_CHECK(t.is_cuda(), name, " must be a CUDA tensor (gsvc_amd has no CPU path)");
    TORCH_CHECK(t.scalar_type() == at::kFloat, name, ": expected scalar type Float but found ",
                t.scalar_type());
    return t.contiguous();
}

Tensor dev_i32(const Tensor &t, const char *name) {
    TORCH_CHECK(t.is_cuda(), name, " must be a CUDA tensor (gsvc_amd has no CPU path)");
    TORCH_CHECK(t.scalar_type() == at::kInt, name, ": expected scalar type Int but found ",
                t.scalar_type());
    return t.contiguous();
}

float *fp(const Tensor &t) { return t.defined() ? t.data_ptr<float>() : nullptr; }
int *ip(const Tensor &t) { return t.defined() ? t.data_ptr<int>() : nullptr; }

// The intersection count of a recent frame on this device, for the kernel
// choice only (sparse / banded composite): every 16th call copies M to pinned
// memory without waiting; a stale value only costs speed (utils._LazyCount).
struct LazyCount {
    int *pinned = nullptr;
    hipEvent_t ev = nullptr;
    bool pending = false;
    int value = 0;
    unsigned calls = 0;
};
LazyCount g_counts[64];
std::mutex g_count_lock;

// The last value read, without polling the event (graph capture).
int hint_cached(int d) {
    if (d < 0 || d >= 64) return 0;
    std::lock_guard<std::mutex> g(g_count_lock);
    return g_counts[d].value;
}

int hint_value(int d) {
    if (d < 0 || d >= 64) return 0;
    std::lock_guard<std::mutex> g(g_count_lock);
    LazyCount &c = g_counts[d];
    if (c.pending && hipEventQuery(c.ev) == hipSuccess) {
        c.value = *c.pinned;
        c.pending = false;
    }
    return c.value;
}

// After the call that wrote m_dev: every 16th call copies it (no wait).
void hint_refresh(const Tensor &m_dev, void *stream) {
    const int d = m_dev.device().index();
    if (d < 0 || d >= 64) return;
    std::lock_guard<std::mutex> g(g_count_lock);
    LazyCount &c = g_counts[d];
    if ((c.calls++ & 15u) != 0 || c.pending) return;
    if (!c.pinned) {
        if (hipHostMalloc((void **)&c.pinned, sizeof(int), hipHostMallocDefault) != hipSuccess ||
            hipEventCreateWithFlags(&c.ev, hipEventDisableTiming) != hipSuccess) {
            c.pinned = nullptr;
            return;
        }
    }
    if (hipMemcpyAsync(c.pinned, m_dev.data_ptr<int>(), sizeof(int), hipMemcpyDeviceToHost,
                       (hipStream_t)stream) == hipSuccess &&
        hipEventRecord(c.ev, (hipStream_t)stream) == hipSuccess)
        c.pending = true;
}

// A [N, C] float gradient as (pointer, row stride in floats): rows may be
// strided views of the rasterizer backward's [N, 16] records (no copy).
const float *rows(Tensor &g, int64_t cols, int &stride, const char *name) {
    if (!(g.dim() == 2 && g.size(1) == cols && g.stride(1) == 1 && g.stride(0) >= cols &&
          g.is_cuda() && g.scalar_type() == at::kFloat))
        g = dev_f32(g, name);
    stride = (int)g.stride(0);
    return g.data_ptr<float>();
}

// project_gaussians_2d.py:59-141 (bindings.cu:781-839, 902-949).
struct ProjectFn : public torch::autograd::Function<ProjectFn> {
    static variable_list forward(AutogradContext *ctx, Tensor means2d, Tensor L, int64_t H,
                                 int64_t W, int64_t tbx, int64_t tby, int64_t tbz, double clip) {
        means2d = dev_f32(means2d, "means2d");
        L = dev_f32(L, "L_elements");
        const int64_t n = means2d.size(-2);
        const auto f = means2d.options();
        const auto i = f.dtype(at::kInt);
        Tensor xys = at::empty({n, 2}, f), depths = at::empty({n}, f), radii = at::empty({n}, i);
        Tensor conics = at::empty({n, 3}, f), nth = at::empty({n}, i);
        check(gsvc_project_gaussians_2d_forward((int)n, fp(means2d), fp(L), (unsigned)H, (unsigned)W,
                                                (int)tbx, (int)tby, (int)tbz, (float)clip, fp(xys),
                                                fp(depths), ip(radii), fp(conics), ip(nth),
                                                stream_of(means2d)),
              "gsvc_project_gaussians_2d_forward");
        ctx->save_for_backward({L, radii, conics});
        // no zero-filled gradients for depths / radii / num_tiles_hit (three
        // fill launches per backward): an undefined gradient stays undefined
        ctx->set_materialize_grads(false);
        ctx->saved_data["H"] = H;
        ctx->saved_data["W"] = W;
        ctx->mark_non_differentiable({radii, nth});
        return {xys, depths, radii, conics, nth};
    }

    static variable_list backward(AutogradContext *ctx, variable_list g) {
        const auto s = ctx->get_saved_variables();
        const Tensor &L = s[0], &radii = s[1], &conics = s[2];
        const int64_t n = L.size(0);
        const auto f = L.options();
        Tensor v_xy = g[0].defined() ? g[0] : at::zeros({n, 2}, f);
        Tensor v_conic = g[3].defined() ? g[3] : at::zeros({n, 3}, f);
        int sxy = 2, sc = 3;
        const float *pxy = rows(v_xy, 2, sxy, "v_xy");
        const float *pc = rows(v_conic, 3, sc, "v_conic");
        Tensor v_cov2d = at::empty({n, 3}, f), v_mean = at::empty({n, 2}, f), v_L = at::empty({n, 3}, f);
        check(gsvc_project_gaussians_2d_backward_strided(
                  (int)n, fp(L), (unsigned)ctx->saved_data["H"].toInt(),
                  (unsigned)ctx->saved_data["W"].toInt(), ip(radii), fp(conics), pxy, sxy, pc, sc,
                  fp(v_cov2d), fp(v_mean), fp(v_L), stream_of(L)),
              "gsvc_project_gaussians_2d_backward_strided");
        return {v_mean, v_L, Tensor(), Tensor(), Tensor(), Tensor(), Tensor(), Tensor()};
    }
};

constexpr int kTileKeep = 256;  // entries per tile the sum rasterizer blends (config.h BLOCK_SIZE)

// The id-slab counters of gsvc_rasterize_sum_forward_slabs, per device and
// stream (zeroed once; each call leaves them ready for the next).  A call
// holds the workspace's lock from its flags to its launches; the workspaces
// live behind unique_ptrs, so registering another (device, stream) never
// moves one a call is using.
struct SlabWs {
    std::mutex lock;
    Tensor buf;
    int tiles = -1;  // -1: (re)zero before use -- new, or a failed call left it dirty
    int calls = 0;
    // the splat order of the id insertion (speed only): sorted by a refresh
    // call for order_n splats, re-sorted every kOrderRefresh calls
    Tensor order;
    int order_n = -1, order_age = 0;
};
constexpr int kOrderRefresh = 64;  // as the training path's ORDER_REFRESH_EVERY

// GSVC_OP_ORDER=0 turns the op path's splat order off (A/B)
bool op_order_enabled() {
    static const bool on = [] {
        const char *e = std::getenv("GSVC_OP_ORDER");
        return !(e && e[0] == '0');
    }();
    return on;
}

// GSVC_TRAIN_ORDER when ws holds an order for n splats, GSVC_TRAIN_ORDER_REFRESH
// when it has none or it is kOrderRefresh calls old (train.py order_flags).
// Nothing is recorded here: order_commit() does that once the call has
// succeeded, so a failed call never leaves an order marked valid that was not
// written (an unsorted order buffer is what faulted in round 4).
int order_flags(SlabWs &ws, int n, const Tensor &like) {
    if (!op_order_enabled() || n <= 0) return 0;
    int flags = 0;
    if (ws.order_n == n) flags |= GSVC_TRAIN_ORDER;
    if (ws.order_n != n || ws.order_age + 1 >= kOrderRefresh) {
        flags |= GSVC_TRAIN_ORDER_REFRESH;
        const size_t bytes = gsvc_rasterize_sum_order_workspace_bytes(n);
        if (!ws.order.defined() || (size_t)ws.order.numel() < bytes)
            ws.order = at::empty({(int64_t)bytes}, like.options().dtype(at::kByte));
    }
    return flags;
}

void order_commit(SlabWs &ws, int n, int flags) {
    if (flags & GSVC_TRAIN_ORDER_REFRESH) {
        ws.order_n = n;
        ws.order_age = 0;
    } else if (flags & GSVC_TRAIN_ORDER) {
        ++ws.order_age;
    }
}

std::mutex g_ws_lock;
std::vector<std::pair<std::pair<int, void *>, std::unique_ptr<SlabWs>>> g_ws;

// The (device, stream) workspace, created on first use (stable address).
SlabWs &slab_ws(const Tensor &like, void *stream) {
    std::lock_guard<std::mutex> g(g_ws_lock);
    const std::pair<int, void *> key(like.device().index(), stream);
    for (auto &kv : g_ws)
        if (kv.first == key) return *kv.second;
    g_ws.emplace_back(key, std::make_unique<SlabWs>());
    return *g_ws.back().second;
}

// Counters for ntiles tiles, zeroed when the workspace is new, resized or dirty
// (caller holds ws.lock).
void slab_ws_ready(SlabWs &w, const Tensor &like, int ntiles) {
    if (w.tiles != ntiles) {
        const size_t bytes = gsvc_rasterize_sum_slabs_workspace_bytes(ntiles);
        w.buf = at::zeros({(int64_t)((bytes + 3) / 4)}, like.options().dtype(at::kInt));
        w.tiles = ntiles;
        w.calls = 0;
        w.order_n = -1;
    }
}

// The op path's image as channel planes (GSVC_SLABS_PLANES): out_img is the
// [H, W, 3] image with strides (W, 1, H*W).  GSVC's epilogue -- clamp, view(-1,
// H, W, 3), permute(0, 3, 1, 2), contiguous (GaussianSplats_Represent.py:88-89,
// GaussianSplats_Compress.py:68,82,162,177) -- then finds its NCHW result
// already contiguous (no 25 MB copy per 1080p forward), and the backward's
// gradient arrives in the same planes.  Values are the reference's; only the
// strides differ, so a caller that views the image as (-1, 3) needs
// .contiguous() first.  GSVC_OP_PLANAR=0 returns the contiguous [H, W, 3]
// (read per call, so a process can switch).
bool op_planar_enabled() {
    const char *e = std::getenv("GSVC_OP_PLANAR");
    return !(e && e[0] == '0');
}

bool capturing(void *stream) {
    if (stream == nullptr) return false;  // the legacy default stream never captures (errors.hip)
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing((hipStream_t)stream, &cs) == hipSuccess &&
           cs != hipStreamCaptureStatusNone;
}

// rasterize_sum.py:89-254 with the binning of gsvc_rasterize_sum_forward_slabs
// (two kernels, no host sync; the caller checked that the depths are zero).
// Returns (out_img [H,W,3], M [1] on the device).  need_grad: the gradient
// records are allocated (and zeroed by the forward) for the backward.
struct RasterSumFn : public torch::autograd::Function<RasterSumFn> {
    static variable_list forward(AutogradContext *ctx, Tensor xys, Tensor radii, Tensor conics,
                                 Tensor colors, Tensor opacity, Tensor background, int64_t H,
                                 int64_t W, bool need_grad) {
        xys = dev_f32(xys, "xys");
        radii = dev_i32(radii, "radii");
        conics = dev_f32(conics, "conics");
        colors = dev_f32(colors, "colors");
        opacity = dev_f32(opacity, "opacities");
        background = dev_f32(background, "background");
        TORCH_CHECK(colors.dim() == 2 && colors.size(1) == 3, "colors must have shape (N, 3)");
        TORCH_CHECK(xys.dim() == 2 && xys.size(1) == 2, "xys must have dimensions (num_points, 2)");
        const int64_t n = xys.size(0);
        const int tbx = (int)((W + 15) / 16), tby = (int)((H + 15) / 16), nt = tbx * tby;
        const auto f = xys.options();
        const auto i = f.dtype(at::kInt);
        void *st = stream_of(xys);
        // the slab route's ids: GSVC_SLABS_WIDE_IDS per tile (a tile of up to 1024
        // entries sorts its first 256 from its slab; the capture route's
        // counted binning keeps 256)
        const bool capture = capturing(st);
        Tensor gids = at::empty({(int64_t)nt * (capture ? kTileKeep : GSVC_SLABS_WIDE_IDS)}, i);
        Tensor bins = at::empty({nt, 2}, i);
        // no final_idx: the backward (raster_sum_bwd_kernel) does not read it --
        // an entry past a pixel's final index fails the alpha test there anyway
        const bool planar = op_planar_enabled();
        Tensor meta = at::empty({2}, i);
        Tensor out = planar ? at::empty({3, H, W}, f).permute({1, 2, 0}) : at::empty({H, W, 3}, f);
        Tensor rec;
        if (capture) {
            // Graph capture: the slab workspace's parity is host state a replay
            // would freeze, so the capturable route -- the counted binning (its
            // scratch allocated per call, from the graph's pool) and the
            // composite over its bins; the same ids, order and bits.  The
            // backward adds into records zeroed here (the insertion zeroes them
            // on the slab route).
            rec = need_grad ? at::zeros({n, 16}, f) : Tensor();
            const int64_t cap = (int64_t)nt * std::min<int64_t>(n, kTileKeep);
            Tensor scratch = at::empty({std::max<int64_t>(cap, 1)}, i);
            Tensor cws = at::empty(
                {(int64_t)(gsvc_bin_tiles_counted_workspace_bytes(nt) / 4 + 1)}, i);
            check(gsvc_bin_tiles_counted((int)n, fp(xys), ip(radii), tbx, tby, cap, kTileKeep,
                                         ip(scratch), ip(gids), ip(bins), ip(meta), cws.data_ptr(),
                                         4 * (size_t)cws.numel(), st),
                  "gsvc_bin_tiles_counted");
            check(gsvc_rasterize_sum_forward_ex(tbx, tby, 1, 16, 16, 1, (unsigned)W, (unsigned)H, 1,
                                                ip(gids), ip(bins), fp(xys), fp(conics), fp(colors),
                                                fp(opacity), fp(background), ip(meta),
                                                hint_cached(xys.device().index()), planar ? 2 : 0,
                                                fp(out),
                                                nullptr, nullptr, st),
                  "gsvc_rasterize_sum_forward_ex");
        } else {
            rec = need_grad ? at::empty({n, 16}, f) : Tensor();
            SlabWs &ws = slab_ws(xys, st);
            std::lock_guard<std::mutex> wl(ws.lock);
            slab_ws_ready(ws, xys, nt);
            const int hint = hint_value(xys.device().index());  // M of an earlier call
            const int oflags = order_flags(ws, (int)n, xys);
            const int rc = gsvc_rasterize_sum_forward_slabs_ordered(
                (int)n, fp(xys), ip(radii), fp(conics), fp(colors), fp(opacity), fp(background),
                (unsigned)H, (unsigned)W, ws.calls, hint, ws.buf.data_ptr(),
                4 * (size_t)ws.buf.numel(), ip(gids), ip(bins), ip(meta), fp(rec), fp(out), nullptr,
                st, oflags ? ws.order.data_ptr() : nullptr, oflags ? (size_t)ws.order.numel() : 0,
                oflags | GSVC_SLABS_WIDE | (planar ? GSVC_SLABS_PLANES : 0));
            if (rc != 0) ws.tiles = -1;  // counters and order in an unknown state: rebuild
            check(rc, "gsvc_rasterize_sum_forward_slabs_ordered");
            ++ws.calls;
            order_commit(ws, (int)n, oflags);
            hint_refresh(meta, st);
        }
        Tensor m_dev = meta.narrow(0, 0, 1);
        ctx->save_for_backward({gids, bins, xys, conics, colors, opacity});
        ctx->set_materialize_grads(false);  // M's gradient (always undefined): no fill
        ctx->saved_data["rec"] = rec;  // zeroed: the first backward adds into it
        ctx->saved_data["H"] = H;
        ctx->saved_data["W"] = W;
        ctx->mark_non_differentiable({m_dev});
        return {out, m_dev};
    }

    static variable_list backward(AutogradContext *ctx, variable_list g) {
        const auto s = ctx->get_saved_variables();
        const Tensor &gids = s[0], &bins = s[1], &xys = s[2], &conics = s[3], &colors = s[4];
        const Tensor &opacity = s[5];
        const int64_t H = ctx->saved_data["H"].toInt(), W = ctx->saved_data["W"].toInt();
        const int64_t n = xys.size(0);
        // the gradient at its own strides (after GSVC's clamp + permute it
        // arrives as channel planes; .contiguous() would copy the frame)
        Tensor v_out = g[0];
        if (!v_out.defined()) {
            v_out = at::zeros({H, W, 3}, xys.options());
        } else if (!(v_out.is_cuda() && v_out.scalar_type() == at::kFloat && v_out.dim() == 3 &&
                     v_out.size(0) == H && v_out.size(1) == W && v_out.size(2) == 3)) {
            v_out = dev_f32(v_out, "v_output");
        }
        Tensor rec = ctx->saved_data["rec"].toTensor();
        if (rec.defined()) {
            ctx->saved_data["rec"] = Tensor();  // a second backward (retain_graph) zeroes its own
        } else {
            rec = at::zeros({n, 16}, xys.options());
        }
        // GSVC's opacity is a constant (GaussianSplats_Represent.py:84): no
        // v_opacity sum, 32-byte gradient requests instead of 64
        const bool opac_grad = ctx->needs_input_grad(4);
        check(gsvc_rasterize_sum_backward_zeroed_strided_ex(
                  (unsigned)H, (unsigned)W, (int)n, ip(gids), ip(bins), fp(xys), fp(conics),
                  fp(colors), fp(opacity), nullptr, v_out.data_ptr<float>(), v_out.stride(0),
                  v_out.stride(1), v_out.stride(2), fp(rec), stream_of(xys),
                  opac_grad ? 0 : GSVC_BWD_NO_OPACITY),
              "gsvc_rasterize_sum_backward_zeroed_strided_ex");
        Tensor v_opac;
        if (opac_grad) {
            v_opac = rec.narrow(1, 8, 1);
            if (opacity.dim() != 2) v_opac = v_opac.reshape(opacity.sizes());
        }
        return {rec.narrow(1, 0, 2), Tensor(), rec.narrow(1, 2, 3), rec.narrow(1, 5, 3), v_opac,
                Tensor(), Tensor(), Tensor(), Tensor()};
    }
};

std::vector<Tensor> project_gaussians_2d(Tensor means2d, Tensor L, int64_t H, int64_t W,
                                         int64_t tbx, int64_t tby, int64_t tbz, double clip) {
    return ProjectFn::apply(means2d, L, H, W, tbx, tby, tbz, clip);
}

std::vector<Tensor> rasterize_sum(Tensor xys, Tensor radii, Tensor conics, Tensor colors,
                                  Tensor opacity, Tensor background, int64_t H, int64_t W) {
    const bool need_grad = at::GradMode::is_enabled() &&
                           (xys.requires_grad() || conics.requires_grad() ||
                            colors.requires_grad() || opacity.requires_grad());
    return RasterSumFn::apply(xys, radii, conics, colors, opacity, background, H, W, need_grad);
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
    m.doc() = "gsvc_amd: C++ autograd Functions of the drop-in operators over libgsvc_amd.so";
    m.def("project_gaussians_2d", &project_gaussians_2d,
          "project_gaussians_2d.py:59-141 (forward + backward through the C ABI)");
    m.def("rasterize_sum", &rasterize_sum,
          "rasterize_sum.py:89-254 on the sync-free binning: (out_img, M on the device)");
    m.def("abi_version", []() { return gsvc_abi_version(); });
}
