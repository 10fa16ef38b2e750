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
//   project: saves (means2d, L, radii, conics); radii and num_tiles_hit are
//            not differentiable; backward = the projection VJP (backward2d.cu).
//   rasterize_sum: the sync-free binning (each tile's first 256 entries in
//            (tile, splat id) order, M on the device) + the sum composite with
//            final_idx; the M < 1 background branch in the kernel; backward =
//            backward.cu:696-862 into one [N, 16] record (the returned
//            gradients are its views).
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>
#include <torch/extension.h>

#include <algorithm>
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

int density_hint(const Tensor &m_dev, void *stream) {
    const int d = m_dev.device().index();
    if (d < 0 || d >= 64) return 0;
    std::lock_guard<std::mutex> g(g_count_lock);
    LazyCount &c = g_counts[d];
    if ((c.calls++ & 15u) != 0) return c.value;
    if (c.pending && hipEventQuery(c.ev) == hipSuccess) {
        c.value = *c.pinned;
        c.pending = false;
    }
    if (!c.pending) {
        if (!c.pinned) {
            if (hipHostMalloc((void **)&c.pinned, sizeof(int), hipHostMallocDefault) != hipSuccess ||
                hipEventCreateWithFlags(&c.ev, hipEventDisableTiming) != hipSuccess) {
                c.pinned = nullptr;
                return c.value;
            }
        }
        if (hipMemcpyAsync(c.pinned, m_dev.data_ptr<int>(), sizeof(int), hipMemcpyDeviceToHost,
                           (hipStream_t)stream) == hipSuccess &&
            hipEventRecord(c.ev, (hipStream_t)stream) == hipSuccess)
            c.pending = true;
    }
    return c.value;
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
        ctx->save_for_backward({means2d, L, radii, conics});
        ctx->saved_data["H"] = H;
        ctx->saved_data["W"] = W;
        ctx->mark_non_differentiable({radii, nth});
        return {xys, depths, radii, conics, nth};
    }

    static variable_list backward(AutogradContext *ctx, variable_list g) {
        const auto s = ctx->get_saved_variables();
        const Tensor &means2d = s[0], &L = s[1], &radii = s[2], &conics = s[3];
        const int64_t n = means2d.size(-2);
        const auto f = L.options();
        Tensor v_xy = g[0].defined() ? dev_f32(g[0], "v_xy") : at::zeros({n, 2}, f);
        Tensor v_conic = g[3].defined() ? dev_f32(g[3], "v_conic") : at::zeros({n, 3}, f);
        Tensor v_cov2d = at::empty({n, 3}, f), v_mean = at::empty({n, 2}, f), v_L = at::empty({n, 3}, f);
        check(gsvc_project_gaussians_2d_backward(
                  (int)n, fp(means2d), fp(L), (unsigned)ctx->saved_data["H"].toInt(),
                  (unsigned)ctx->saved_data["W"].toInt(), ip(radii), fp(conics), fp(v_xy), nullptr,
                  fp(v_conic), fp(v_cov2d), fp(v_mean), fp(v_L), stream_of(L)),
              "gsvc_project_gaussians_2d_backward");
        return {v_mean, v_L, Tensor(), Tensor(), Tensor(), Tensor(), Tensor(), Tensor()};
    }
};

constexpr int kTileKeep = 256;  // entries per tile the sum rasterizer blends (config.h BLOCK_SIZE)

// rasterize_sum.py:89-254 on the sync-free binning (utils.bin_for_raster's
// counted path; the caller checked that it applies).  Returns (out_img [H,W,3],
// M [1] on the device).
struct RasterSumFn : public torch::autograd::Function<RasterSumFn> {
    static variable_list forward(AutogradContext *ctx, Tensor xys, Tensor radii, Tensor conics,
                                 Tensor colors, Tensor opacity, Tensor background, int64_t H,
                                 int64_t W) {
        xys = dev_f32(xys, "xys");
        radii = dev_i32(radii, "radii");
        conics = dev_f32(conics, "conics");
        colors = dev_f32(colors, "colors");
        opacity = dev_f32(opacity, "opacities");
        background = dev_f32(background, "background");
        TORCH_CHECK(colors.dim() == 2 && colors.size(1) == 3, "colors must have shape (N, 3)");
        const int64_t n = xys.size(0);
        const int tbx = (int)((W + 15) / 16), tby = (int)((H + 15) / 16), nt = tbx * tby;
        const long long cap = (long long)std::min<int64_t>(n, kTileKeep) * nt;
        const auto f = xys.options();
        const auto i = f.dtype(at::kInt);
        void *st = stream_of(xys);
        Tensor scratch = at::empty({cap}, i), gids = at::empty({cap}, i);
        Tensor bins = at::empty({nt, 2}, i), meta = at::empty({2}, i);
        const size_t wsb = gsvc_bin_tiles_counted_workspace_bytes(nt);
        Tensor ws = at::empty({(int64_t)(wsb / 4 + 1)}, i);
        check(gsvc_bin_tiles_counted((int)n, fp(xys), ip(radii), tbx, tby, cap,
                                     n > kTileKeep ? kTileKeep : 0, ip(scratch), ip(gids), ip(bins),
                                     ip(meta), ws.data_ptr(), 4 * (size_t)ws.numel(), st),
              "gsvc_bin_tiles_counted");
        const int hint = density_hint(meta, st);
        Tensor out = at::empty({H, W, 3}, f), idx = at::empty({H, W}, i);
        check(gsvc_rasterize_sum_forward_ex(tbx, tby, 1, 16, 16, 1, (unsigned)W, (unsigned)H, 1,
                                            ip(gids), ip(bins), fp(xys), fp(conics), fp(colors),
                                            fp(opacity), fp(background), ip(meta), hint, 0,
                                            fp(out), nullptr, ip(idx), st),
              "gsvc_rasterize_sum_forward_ex");
        Tensor m_dev = meta.narrow(0, 0, 1);
        ctx->save_for_backward({gids, bins, xys, conics, colors, opacity, background, idx});
        ctx->saved_data["H"] = H;
        ctx->saved_data["W"] = W;
        ctx->mark_non_differentiable({m_dev});
        return {out, m_dev};
    }

    static variable_list backward(AutogradContext *ctx, variable_list g) {
        const auto s = ctx->get_saved_variables();
        const Tensor &gids = s[0], &bins = s[1], &xys = s[2], &conics = s[3], &colors = s[4];
        const Tensor &opacity = s[5], &background = s[6], &idx = s[7];
        const int64_t H = ctx->saved_data["H"].toInt(), W = ctx->saved_data["W"].toInt();
        const int64_t n = xys.size(0);
        Tensor v_out = g[0].defined() ? dev_f32(g[0], "v_output") : at::zeros({H, W, 3}, xys.options());
        Tensor rec = at::empty({n, 16}, xys.options());
        check(gsvc_rasterize_sum_backward((unsigned)H, (unsigned)W, 16, 16, (int)n, ip(gids),
                                          ip(bins), fp(xys), fp(conics), fp(colors), fp(opacity),
                                          fp(background), nullptr, ip(idx), fp(v_out), nullptr,
                                          fp(rec), stream_of(xys)),
              "gsvc_rasterize_sum_backward");
        Tensor v_opac = rec.narrow(1, 8, 1);
        if (opacity.dim() != 2) v_opac = v_opac.reshape(opacity.sizes());
        return {rec.narrow(1, 0, 2), Tensor(), rec.narrow(1, 2, 3), rec.narrow(1, 5, 3), v_opac,
                Tensor(), Tensor(), Tensor()};
    }
};

std::vector<Tensor> project_gaussians_2d(Tensor means2d, Tensor L, int64_t H, int64_t W,
                                         int64_t tbx, int64_t tby, int64_t tbz, double clip) {
    return ProjectFn::apply(means2d, L, H, W, tbx, tby, tbz, clip);
}

std::vector<Tensor> rasterize_sum(Tensor xys, Tensor radii, Tensor conics, Tensor colors,
                                  Tensor opacity, Tensor background, int64_t H, int64_t W) {
    return RasterSumFn::apply(xys, radii, conics, colors, opacity, background, H, W);
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
