// The alpha cut of the sum rasterizer at unit opacity as one threshold on
// sigma, verified over every float on the device it runs on.
//
// forward.cu:598-606 (and backward.cu:822-828) keep a (splat, pixel) pair when
//     !(sigma < 0) && !(min(1, opacity * exp(-sigma)) < 1/255).
// GSVC's frame model has opacity 1, where this is a predicate of sigma alone:
// exp(-sigma) is v_exp_f32(sigma * -log2 e) here (common.h exp_neg), and both
// the rounded multiply and v_exp_f32 are non-decreasing, so the pairs kept are
// exactly the sigma whose bits lie in [+0, kSigmaCutBits] (common.h).  This
// scan proves it for the hardware at hand: over all 2^31 non-negative float
// bit patterns (+0 .. +inf, and the NaNs above) it records the largest kept
// pattern, the smallest dropped one and how many kept patterns have
// exp_neg(sigma) > 1 (where dropping the min(1, .) would change alpha).  The
// cut is exact iff smallest dropped == largest kept + 1 below the NaNs and
// that count is 0 (tests/test_alpha_cut.py).  A NaN sigma -- impossible for
// finite splat geometry -- is kept by the reference predicate (min(1, NaN) = 1)
// and dropped by the threshold: the kernels take the threshold only for chunks
// whose entries' geometry is finite.
#include "common.h"

namespace gsvc {

__device__ __forceinline__ bool alpha_kept_unit(float sigma, float &alpha) {
    const float e = exp_neg(sigma);
    alpha = fminf(1.0f, e);
    return !(sigma < 0.0f) && !(alpha < kAlphaMin);
}

constexpr unsigned kCutScanPerThread = 64;

// out: [0] largest kept pattern, [1] smallest dropped pattern (both among the
// non-NaN patterns 0 .. 0x7f800000), [2] kept patterns with exp_neg > 1,
// [3] kept NaN patterns (the reference keeps NaN sigma)
__global__ __launch_bounds__(256) void alpha_cut_scan_kernel(unsigned *out) {
    const unsigned base = (blockIdx.x * 256u + threadIdx.x) * kCutScanPerThread;
    unsigned kept_max = 0u, drop_min = 0xffffffffu, over = 0u, nan_kept = 0u;
    for (unsigned k = 0; k < kCutScanPerThread; ++k) {
        const unsigned b = base + k;
        if (b > 0x7fffffffu) break;
        float a;
        const bool kept = alpha_kept_unit(__uint_as_float(b), a);
        if (b <= 0x7f800000u) {
            if (kept) {
                kept_max = max(kept_max, b);
                over += exp_neg(__uint_as_float(b)) > 1.0f ? 1u : 0u;
            } else {
                drop_min = min(drop_min, b);
            }
        } else {
            nan_kept += kept ? 1u : 0u;
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        kept_max = max(kept_max, (unsigned)__shfl_xor((int)kept_max, off, 64));
        drop_min = min(drop_min, (unsigned)__shfl_xor((int)drop_min, off, 64));
        over += (unsigned)__shfl_xor((int)over, off, 64);
        nan_kept += (unsigned)__shfl_xor((int)nan_kept, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(out, kept_max);
        atomicMin(out + 1, drop_min);
        if (over) atomicAdd(out + 2, over);
        if (nan_kept) atomicAdd(out + 3, nan_kept);
    }
}

__global__ void alpha_cut_init_kernel(unsigned *out) {
    out[0] = 0u;
    out[1] = 0xffffffffu;
    out[2] = 0u;
    out[3] = 0u;
}

}  // namespace gsvc

using namespace gsvc;

extern "C" int gsvc_alpha_cut_scan(unsigned *out, void *stream) {
    if (!out) return set_error(GSVC_ERR_ARG, "alpha_cut_scan: null output");
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(alpha_cut_init_kernel, dim3(1), dim3(1), 0, s, out);
    const unsigned blocks = (0x80000000u / kCutScanPerThread) / 256u;
    hipLaunchKernelGGL(alpha_cut_scan_kernel, dim3(blocks), dim3(256), 0, s, out);
    return check_launch("alpha_cut_scan");
}

extern "C" unsigned gsvc_alpha_cut_bits(void) { return kSigmaCutBits; }
