// 2D projection of Gaussian splats, forward and backward (gfx950).
//
// Reference: gsplat/gsplat/cuda/csrc/foward2d.cu:12-69 (forward),
// backward2d.cu:8-51 (backward), helpers.cuh:45-82 (cov2d bounds and
// conic VJP), bindings.cu:21-60,781-839,902-949 (bindings).
//
// One lane per splat; the kernels are HBM/launch bound (52N bytes forward,
// 92N backward).  Unlike the reference binding, which zero-fills
// five outputs with torch::zeros before the launch, the kernel writes every
// output element itself, so a call is exactly one kernel.
#include "project2d.h"

namespace gsvc {

__global__ __launch_bounds__(256) void project2d_fwd_kernel(
    int n, const float2 *__restrict__ means2d, const float *__restrict__ L,
    float hw, float hh, int tbx, int tby,
    float2 *__restrict__ xys, float *__restrict__ depths, int *__restrict__ radii,
    float *__restrict__ conics, int *__restrict__ num_tiles_hit) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float2 m = means2d[i];
    const SplatProj P = project_splat(m.x, m.y, L[3 * i], L[3 * i + 1], L[3 * i + 2], hw, hh, tbx, tby);
    const float2 xy = P.xy;
    const float c0 = P.c0, c1 = P.c1, c2 = P.c2;
    const int rad = P.rad, hit = P.hit;
    xys[i] = xy;
    depths[i] = 0.0f;
    radii[i] = rad;
    conics[3 * i] = c0;
    conics[3 * i + 1] = c1;
    conics[3 * i + 2] = c2;
    num_tiles_hit[i] = hit;
}

// backward2d.cu:8-51; cov2d_to_conic_vjp (helpers.cuh:71-82) expanded in glm's
// column-major mat2 product order: V = ((-X) * G) * X.
__global__ __launch_bounds__(256) void project2d_bwd_kernel(
    int n, const float *__restrict__ L, float hw, float hh,
    const int *__restrict__ radii, const float *__restrict__ conics,
    const float *__restrict__ v_xy, int sxy, const float *__restrict__ v_conic, int sc,
    float *__restrict__ v_cov2d, float2 *__restrict__ v_mean2d, float *__restrict__ v_L) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float g11 = 0.0f, g12 = 0.0f, g22 = 0.0f, vl0 = 0.0f, vl1 = 0.0f, vl2 = 0.0f;
    float2 vm = make_float2(0.0f, 0.0f);
    if (radii[i] > 0) {
        const float X00 = conics[3 * i], X01 = conics[3 * i + 1], X10 = X01, X11 = conics[3 * i + 2];
        const float *vc = v_conic + (size_t)sc * i;  // row i (row stride sc floats)
        const float G00 = vc[0], G01 = vc[1], G10 = G01, G11 = vc[2];
        const float N00 = -X00, N01 = -X01, N10 = -X10, N11 = -X11;
        const float P00 = N00 * G00 + N10 * G01;
        const float P01 = N01 * G00 + N11 * G01;
        const float P10 = N00 * G10 + N10 * G11;
        const float P11 = N01 * G10 + N11 * G11;
        const float V00 = P00 * X00 + P10 * X01;
        const float V01 = P01 * X00 + P11 * X01;
        const float V10 = P00 * X10 + P10 * X11;
        const float V11 = P01 * X10 + P11 * X11;
        g11 = V00;
        g12 = V10 + V01;
        g22 = V11;
        const float l11 = L[3 * i], l21 = L[3 * i + 1], l22 = L[3 * i + 2];
        vl0 = 2.0f * l11 * g11 + 2.0f * g12 * l21;  // doubled cross term: backward2d.cu:39
        vl1 = 2.0f * l11 * g12 + 2.0f * l21 * g22;
        vl2 = 2.0f * l22 * g22;
        const float *vx = v_xy + (size_t)sxy * i;
        vm = make_float2(vx[0] * hw, vx[1] * hh);
    }
    v_cov2d[3 * i] = g11;
    v_cov2d[3 * i + 1] = g12;
    v_cov2d[3 * i + 2] = g22;
    v_mean2d[i] = vm;
    v_L[3 * i] = vl0;
    v_L[3 * i + 1] = vl1;
    v_L[3 * i + 2] = vl2;
}

// bindings.cu:21-39 (degenerate covariances give zeros here; the reference
// wrote uninitialised registers).
__global__ __launch_bounds__(256) void cov2d_bounds_kernel(
    int n, const float *__restrict__ covs, float *__restrict__ conics, float *__restrict__ radii) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float c0 = 0.0f, c1 = 0.0f, c2 = 0.0f, r = 0.0f;
    if (!cov2d_bounds(covs[3 * i], covs[3 * i + 1], covs[3 * i + 2], c0, c1, c2, r)) {
        c0 = c1 = c2 = r = 0.0f;
    }
    conics[3 * i] = c0;
    conics[3 * i + 1] = c1;
    conics[3 * i + 2] = c2;
    radii[i] = r;
}

}  // namespace gsvc

using namespace gsvc;

extern "C" int gsvc_project_gaussians_2d_forward(
    int num_points, const float *means2d, const float *L_elements, unsigned img_height,
    unsigned img_width, int tbx, int tby, int tbz, float clip_thresh, float *xys, float *depths,
    int *radii, float *conics, int *num_tiles_hit, void *stream) {
    (void)tbz;
    (void)clip_thresh;
    if (num_points < 0 || tbx < 0 || tby < 0)
        return set_error(GSVC_ERR_ARG, "project_gaussians_2d_forward: bad sizes");
    if (num_points == 0) return GSVC_OK;
    const float hw = 0.5f * (float)img_width, hh = 0.5f * (float)img_height;
    hipLaunchKernelGGL(project2d_fwd_kernel, dim3(ceil_div(num_points, 256)), dim3(256), 0,
                       (hipStream_t)stream, num_points, (const float2 *)means2d, L_elements, hw, hh,
                       tbx, tby, (float2 *)xys, depths, radii, conics, num_tiles_hit);
    return check_launch("project_gaussians_2d_forward");
}

extern "C" int gsvc_project_gaussians_2d_backward_strided(
    int num_points, const float *L_elements, unsigned img_height, unsigned img_width,
    const int *radii, const float *conics, const float *v_xy, int v_xy_stride,
    const float *v_conic, int v_conic_stride, float *v_cov2d, float *v_mean2d,
    float *v_L_elements, void *stream) {
    if (num_points < 0 || v_xy_stride < 2 || v_conic_stride < 3)
        return set_error(GSVC_ERR_ARG, "project_gaussians_2d_backward: bad size or stride");
    if (num_points == 0) return GSVC_OK;
    const float hw = 0.5f * (float)img_width, hh = 0.5f * (float)img_height;
    hipLaunchKernelGGL(project2d_bwd_kernel, dim3(ceil_div(num_points, 256)), dim3(256), 0,
                       (hipStream_t)stream, num_points, L_elements, hw, hh, radii, conics, v_xy,
                       v_xy_stride, v_conic, v_conic_stride, v_cov2d, (float2 *)v_mean2d,
                       v_L_elements);
    return check_launch("project_gaussians_2d_backward");
}

extern "C" int gsvc_project_gaussians_2d_backward(
    int num_points, const float *means2d, const float *L_elements, unsigned img_height,
    unsigned img_width, const int *radii, const float *conics, const float *v_xy,
    const float *v_depth, const float *v_conic, float *v_cov2d, float *v_mean2d,
    float *v_L_elements, void *stream) {
    (void)means2d;
    (void)v_depth;
    return gsvc_project_gaussians_2d_backward_strided(num_points, L_elements, img_height,
                                                      img_width, radii, conics, v_xy, 2, v_conic,
                                                      3, v_cov2d, v_mean2d, v_L_elements, stream);
}

extern "C" int gsvc_compute_cov2d_bounds(int num_pts, const float *covs2d, float *conics,
                                         float *radii, void *stream) {
    if (num_pts < 0) return set_error(GSVC_ERR_ARG, "compute_cov2d_bounds: bad size");
    if (num_pts == 0) return GSVC_OK;
    hipLaunchKernelGGL(cov2d_bounds_kernel, dim3(ceil_div(num_pts, 256)), dim3(256), 0,
                       (hipStream_t)stream, num_pts, covs2d, conics, radii);
    return check_launch("compute_cov2d_bounds");
}
