// Per-element Adan update shared by adan.hip (the optimizer op) and train.hip
// (the fused training step): one op sequence, so both give identical bits.
//
// Reference: optimizer.py:296-362 (_multi_tensor_adan), bias corrections
// :171-173,211 computed by the host.  Per element the foreach sequence is
//     g = grad * clip;  d = npg + g
//     m    = m * b1 + (1 - b1) * g                          (exp_avg)
//     diff = diff * b2 + (1 - b2) * d                       (exp_avg_diff)
//     t    = d * b2 + g
//     v    = v * b3 + (1 - b3) * t * t                      (exp_avg_sq)
//     den  = sqrt(v) / bc3_sqrt + eps
//     p    = [p * (1 - lr wd)] - step * m / den - step_diff * diff / den [/ (1 + lr wd)]
//     npg  = -g
// On a parameter's first step the reference initialises npg = grad * -clip
// (optimizer.py:187-189), so d = -g + g = 0 exactly.
#pragma once

#include "common.h"

namespace gsvc {

struct AdanScalars {
    float b1, b2, b3, one_m_b1, one_m_b2, one_m_b3, bc3_sqrt, eps, step, step_diff, clip;
    float decay_mul, decay_div;  // no_prox: p *= decay_mul first; else p /= decay_div after
    int no_prox;
};

// torch's foreach ops take Python-float scalars as fp32 for fp32 tensors.
inline AdanScalars adan_scalars(double beta1, double beta2, double beta3, double bias_correction1,
                                double bias_correction2, double bias_correction3_sqrt, double lr,
                                double weight_decay, double eps, int no_prox, double clip) {
    AdanScalars S;
    S.b1 = (float)beta1;
    S.b2 = (float)beta2;
    S.b3 = (float)beta3;
    S.one_m_b1 = (float)(1.0 - beta1);
    S.one_m_b2 = (float)(1.0 - beta2);
    S.one_m_b3 = (float)(1.0 - beta3);
    S.bc3_sqrt = (float)bias_correction3_sqrt;
    S.eps = (float)eps;
    S.step = (float)(lr / bias_correction1);
    S.step_diff = (float)(lr * beta2 / bias_correction2);
    S.clip = (float)clip;
    S.decay_mul = (float)(1.0 - lr * weight_decay);
    S.decay_div = (float)(1.0 + lr * weight_decay);
    S.no_prox = no_prox;
    return S;
}

// One element: returns the new parameter; m, v, df, npg updated in place.
__device__ __forceinline__ float adan_update(const AdanScalars &S, float p, float grad, float &m,
                                             float &v, float &df, float &npg) {
    const float g = grad * S.clip;
    const float d = npg + g;
    m = m * S.b1 + S.one_m_b1 * g;
    df = df * S.b2 + S.one_m_b2 * d;
    const float tt = d * S.b2 + g;
    v = v * S.b3 + S.one_m_b3 * (tt * tt);
    const float den = sqrtf(v) / S.bc3_sqrt + S.eps;
    if (S.no_prox) p = p * S.decay_mul;
    p = p + (-S.step) * (m / den);
    p = p + (-S.step_diff) * (df / den);
    if (!S.no_prox) p = p / S.decay_div;
    npg = -g;
    return p;
}

}  // namespace gsvc
