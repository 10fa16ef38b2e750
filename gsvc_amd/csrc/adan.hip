// Fused Adan step (gfx950): GSVC's optimizer update in one kernel.
//
// Reference: optimizer.py:296-362 (_multi_tensor_adan) with the bias
// corrections of :171-173,211 computed by the host.  Per element, the foreach
// sequence
//     g = grad * clip;  d = npg + g
//     m    = m * b1 + (1 - b1) * g                          (exp_avg)
//     diff = diff * b2 + (1 - b2) * d                       (exp_avg_diff)
//     t    = d * b2 + g
//     v    = v * b3 + (1 - b3) * t * t                      (exp_avg_sq)
//     den  = sqrt(v) / bc3_sqrt + eps
//     p    = [p * (1 - lr wd)] - step * m / den - step_diff * diff / den [/ (1 + lr wd)]
//     npg  = -g
// is done in registers: 6 loads + 5 stores (44 B) per element, HBM-bound,
// instead of ~17 foreach launches each streaming the tensors.  The gradient
// itself is not written back (the reference scales p.grad in place, but
// train_iter clears it right after the step).  fp32 throughout; results
// agree with the foreach path to rounding (tests/test_adan.py).
#include "adan.h"

namespace gsvc {

constexpr int kAdanMaxTensors = 8;

struct AdanArgs {
    int ntensors;
    long long offset[kAdanMaxTensors + 1];  // prefix of element counts
    float *p[kAdanMaxTensors];
    const float *g[kAdanMaxTensors];
    float *m[kAdanMaxTensors], *v[kAdanMaxTensors], *diff[kAdanMaxTensors], *npg[kAdanMaxTensors];
    AdanScalars S;
};

__device__ __forceinline__ void adan_elem(const AdanArgs &A, int t, long long j) {
    float m = A.m[t][j], v = A.v[t][j], df = A.diff[t][j], npg = A.npg[t][j];
    A.p[t][j] = adan_update(A.S, A.p[t][j], A.g[t][j], m, v, df, npg);
    A.m[t][j] = m;
    A.diff[t][j] = df;
    A.v[t][j] = v;
    A.npg[t][j] = npg;
}

__global__ __launch_bounds__(256) void adan_kernel(AdanArgs A) {
    const long long total = A.offset[A.ntensors];
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        int t = 0;
        while (t + 1 < A.ntensors && i >= A.offset[t + 1]) ++t;
        adan_elem(A, t, i - A.offset[t]);
    }
}

}  // namespace gsvc

using namespace gsvc;

extern "C" int gsvc_adan_step(int ntensors, const long long *numels, float *const *params,
                              const float *const *grads, float *const *exp_avgs,
                              float *const *exp_avg_sqs, float *const *exp_avg_diffs,
                              float *const *neg_pre_grads, double beta1, double beta2,
                              double beta3, double bias_correction1, double bias_correction2,
                              double bias_correction3_sqrt, double lr, double weight_decay,
                              double eps, int no_prox, double clip_global_grad_norm, void *stream) {
    if (ntensors < 0 || (ntensors > 0 && (!numels || !params || !grads || !exp_avgs ||
                                          !exp_avg_sqs || !exp_avg_diffs || !neg_pre_grads)))
        return set_error(GSVC_ERR_ARG, "adan_step: bad arguments");
    AdanArgs A{};
    A.S = adan_scalars(beta1, beta2, beta3, bias_correction1, bias_correction2,
                       bias_correction3_sqrt, lr, weight_decay, eps, no_prox, clip_global_grad_norm);
    hipStream_t s = (hipStream_t)stream;
    for (int base = 0; base < ntensors; base += kAdanMaxTensors) {
        const int k = min(kAdanMaxTensors, ntensors - base);
        A.ntensors = k;
        A.offset[0] = 0;
        for (int t = 0; t < k; ++t) {
            if (numels[base + t] < 0) return set_error(GSVC_ERR_ARG, "adan_step: negative numel");
            A.offset[t + 1] = A.offset[t] + numels[base + t];
            A.p[t] = params[base + t];
            A.g[t] = grads[base + t];
            A.m[t] = exp_avgs[base + t];
            A.v[t] = exp_avg_sqs[base + t];
            A.diff[t] = exp_avg_diffs[base + t];
            A.npg[t] = neg_pre_grads[base + t];
        }
        const long long total = A.offset[k];
        if (total == 0) continue;
        const int grid = (int)std::min<long long>((total + 255) / 256, 4096);
        hipLaunchKernelGGL(adan_kernel, dim3(grid), dim3(256), 0, s, A);
        const int rc = check_launch("adan_step");
        if (rc) return rc;
    }
    return GSVC_OK;
}
