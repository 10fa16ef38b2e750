// Video frame input of GSVC's driver (gfx950): planar I420 (YUV 4:2:0, 8 bit)
// to the float RGB image the trainer fits, [3, H, W] in [0, 1].
//
// Reference: utils.py:134-156 (process_yuv_video: cv2.cvtColor(yuv,
// COLOR_YUV2RGB_I420) per frame) followed by train_video_Represent.py:204-207
// (torchvision ToTensor: uint8 HWC -> float CHW / 255).  The conversion
// restates OpenCV's fixed-point ITU-R BT.601 limited-range formula
// (Y' = max(0, Y - 16) * 1.164, 20-bit fixed point, round half up,
// saturate to [0, 255]); OpenCV is not installed here, so this arithmetic is
// parity-unpinned against cv2.  One lane per pixel pair of a
// row; HBM-bound (1.5 B read + 12 B written per pixel).
#include "common.h"

namespace gsvc {

constexpr int kCY = 1220542, kCUB = 2116026, kCUG = -409993, kCVG = -852492, kCVR = 1673527;
constexpr int kShift = 20;

__device__ __forceinline__ float chan(int y, int uv) {
    int x = (y + uv) >> kShift;
    x = x < 0 ? 0 : (x > 255 ? 255 : x);
    return (float)x / 255.0f;
}

__global__ __launch_bounds__(256) void i420_to_rgb_kernel(const unsigned char *__restrict__ yuv,
                                                          int h, int w, float *__restrict__ out) {
    const int hw2 = (w + 1) / 2;
    const long long pairs = (long long)h * hw2;
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= pairs) return;
    const int i = (int)(t / hw2), jp = (int)(t - (long long)i * hw2);
    const size_t plane = (size_t)w * h, cplane = (size_t)hw2 * ((h + 1) / 2);
    const size_t c = (size_t)(i >> 1) * hw2 + jp;
    const int u = (int)yuv[plane + c] - 128, v = (int)yuv[plane + cplane + c] - 128;
    const int ruv = (1 << (kShift - 1)) + kCVR * v;
    const int guv = (1 << (kShift - 1)) + kCVG * v + kCUG * u;
    const int buv = (1 << (kShift - 1)) + kCUB * u;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int j = 2 * jp + k;
        if (j >= w) break;
        const size_t p = (size_t)i * w + j;
        const int y = max(0, (int)yuv[p] - 16) * kCY;
        out[p] = chan(y, ruv);
        out[plane + p] = chan(y, guv);
        out[2 * plane + p] = chan(y, buv);
    }
}

}  // namespace gsvc

using namespace gsvc;

extern "C" int gsvc_i420_to_rgb(const unsigned char *yuv, int height, int width, float *out,
                                void *stream) {
    if (height <= 0 || width <= 0 || (height & 1) || (width & 1))
        return set_error(GSVC_ERR_ARG, "i420_to_rgb: height and width must be positive and even");
    if (!yuv || !out) return set_error(GSVC_ERR_ARG, "i420_to_rgb: missing buffer");
    const long long pairs = (long long)height * (width / 2);
    hipLaunchKernelGGL(i420_to_rgb_kernel, dim3((unsigned)((pairs + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, yuv, height, width, out);
    return check_launch("i420_to_rgb");
}
