// SSIM and MS-SSIM of GSVC's SSIM-family losses and MS-SSIM metric (gfx950),
// forward and backward.
//
// Reference call sites: utils.py:29-40 (loss_fn 'SSIM', 'Fusion1', 'Fusion2',
// 'Fusion4', 'Fusion_hinerv') and train_video_Represent.py:145 (per-frame
// MS-SSIM).  The arithmetic is pytorch_msssim's published algorithm
// (ssim/ms_ssim/_ssim/gaussian_filter; the package is unpinned in
// requirements.txt:5 and not installed here, so parity is against our own
// restatement: oracle/oracle.py ssim/ms_ssim):
//   w      = normalised 1-D Gaussian (win_size taps, win_sigma), applied along
//            H then W as VALID correlations; a dimension shorter than the
//            window is not filtered;
//   mu1 = w*X, mu2 = w*Y, s1 = w*(X X) - mu1^2, s2 = w*(Y Y) - mu2^2,
//   s12 = w*(X Y) - mu1 mu2, C1 = (K1 R)^2, C2 = (K2 R)^2,
//   cs  = (2 s12 + C2) / (s1 + s2 + C2),
//   ssim_map = ((2 mu1 mu2 + C1) / (mu1^2 + mu2^2 + C1)) * cs,
//   per (batch, channel): the means of ssim_map and cs over the valid window;
//   MS-SSIM: 5 levels joined by 2x2 average pooling (padding H%2, W%2, pads
//   counted), prod_i relu(cs_i)^w_i (i < 4) * relu(ssim_4)^w_4.
//
// Layout: planes [P = B*C][H][W] fp32.  Every level is one LDS-tiled launch
// over (W tiles, H tiles, planes): the 5 windowed moments of a 16x64 output
// tile from a 26x74 input tile (vertical pass, then horizontal), per-block
// partial sums of ssim_map and cs (reduced in double, in a fixed order, by
// ssim_reduce_kernel, then ssim_combine_kernel forms the values and the
// per-plane upstream factors the backward needs -- nothing goes to the host).
// Backward (w.r.t. X; w.r.t. Y by symmetry with X and Y swapped): per level
//   dX = w^T*g_mu1 + 2 X (w^T*g_E11) + Y (w^T*g_E12)
// with the per-output coefficients g recomputed in LDS from a (16+20)x(64+20)
// input tile, plus the coarser level's gradient through the average pool.
// HBM: forward 8 B per pixel and level, backward 12 B (+4 B per coarse pixel).
#include "common.h"

namespace gsvc {

constexpr int kSsimMaxWin = 11;
constexpr int kSsimTH = 16, kSsimTW = 64;
constexpr int kSsimMaxLevels = 8;

struct SsimWin {
    float wv[kSsimMaxWin];  // vertical taps (kv of them; kv = 1: identity)
    float wh[kSsimMaxWin];  // horizontal taps
    int kv, kh;
};

// ---------------------------------------------------------------- forward

__global__ __launch_bounds__(256) void ssim_fwd_kernel(const float *__restrict__ X,
                                                       const float *__restrict__ Y, int H, int W,
                                                       int Ho, int Wo, SsimWin w, float C1,
                                                       float C2, float2 *__restrict__ partial) {
    constexpr int kInH = kSsimTH + kSsimMaxWin - 1, kInW = kSsimTW + kSsimMaxWin - 1;
    __shared__ float s_x[kInH][kInW], s_y[kInH][kInW];
    __shared__ float s_v[5][kSsimTH][kInW];
    __shared__ float2 s_red[4];
    const int tid = threadIdx.x;
    const int plane = blockIdx.z;
    const int r0 = blockIdx.y * kSsimTH, c0 = blockIdx.x * kSsimTW;
    const size_t hw = (size_t)H * (size_t)W;
    const float *x = X + plane * hw, *y = Y + plane * hw;
    const int inh = kSsimTH + w.kv - 1, inw = kSsimTW + w.kh - 1;
    for (int k = tid; k < inh * inw; k += 256) {
        const int rr = k / inw, cc = k - rr * inw;
        const int gr = r0 + rr, gc = c0 + cc;
        float a = 0.f, b = 0.f;
        if (gr < H && gc < W) {
            a = x[(size_t)gr * W + gc];
            b = y[(size_t)gr * W + gc];
        }
        s_x[rr][cc] = a;
        s_y[rr][cc] = b;
    }
    __syncthreads();
    // vertical pass: the 5 moments of rows r0..r0+15 over columns of the tile
    for (int k = tid; k < kSsimTH * inw; k += 256) {
        const int rr = k / inw, cc = k - rr * inw;
        float m1 = 0.f, m2 = 0.f, e11 = 0.f, e22 = 0.f, e12 = 0.f;
#pragma unroll
        for (int t = 0; t < kSsimMaxWin; ++t) {
            if (t < w.kv) {
                const float a = s_x[rr + t][cc], b = s_y[rr + t][cc], q = w.wv[t];
                m1 = fmaf(q, a, m1);
                m2 = fmaf(q, b, m2);
                e11 = fmaf(q, a * a, e11);
                e22 = fmaf(q, b * b, e22);
                e12 = fmaf(q, a * b, e12);
            }
        }
        s_v[0][rr][cc] = m1;
        s_v[1][rr][cc] = m2;
        s_v[2][rr][cc] = e11;
        s_v[3][rr][cc] = e22;
        s_v[4][rr][cc] = e12;
    }
    __syncthreads();
    float acc_s = 0.f, acc_c = 0.f;
#pragma unroll
    for (int j = 0; j < kSsimTH * kSsimTW / 256; ++j) {
        const int k = tid + 256 * j;
        const int rr = k / kSsimTW, cc = k - rr * kSsimTW;
        if (r0 + rr >= Ho || c0 + cc >= Wo) continue;
        float m[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < kSsimMaxWin; ++t) {
            if (t < w.kh) {
#pragma unroll
                for (int q = 0; q < 5; ++q) m[q] = fmaf(w.wh[t], s_v[q][rr][cc + t], m[q]);
            }
        }
        const float mu1_sq = m[0] * m[0], mu2_sq = m[1] * m[1], mu12 = m[0] * m[1];
        const float s1 = m[2] - mu1_sq, s2 = m[3] - mu2_sq, s12 = m[4] - mu12;
        const float cs = (2.0f * s12 + C2) / ((s1 + s2) + C2);
        const float ss = ((2.0f * mu12 + C1) / ((mu1_sq + mu2_sq) + C1)) * cs;
        acc_s += ss;
        acc_c += cs;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        acc_s += __shfl_xor(acc_s, off, 64);
        acc_c += __shfl_xor(acc_c, off, 64);
    }
    if ((tid & 63) == 0) s_red[tid >> 6] = make_float2(acc_s, acc_c);
    __syncthreads();
    if (tid == 0) {
        const float2 a = s_red[0], b = s_red[1], c = s_red[2], d = s_red[3];
        partial[((size_t)plane * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x] =
            make_float2((a.x + b.x) + (c.x + d.x), (a.y + b.y) + (c.y + d.y));
    }
}

// 2x2 average pool, stride 2, padding (pr, pc), pads counted (F.avg_pool2d
// defaults): the sum in window order, then / 4.
__global__ __launch_bounds__(256) void ssim_pool_kernel(const float *__restrict__ in, int H, int W,
                                                        float *__restrict__ out, int Hc, int Wc,
                                                        int pr, int pc, int planes) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long per = (long long)Hc * Wc;
    if (t >= per * planes) return;
    const int plane = (int)(t / per);
    const int o = (int)(t - (long long)plane * per);
    const int orow = o / Wc, ocol = o - orow * Wc;
    const float *p = in + (size_t)plane * H * W;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r = 2 * orow - pr + i;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int c = 2 * ocol - pc + j;
            if (r >= 0 && r < H && c >= 0 && c < W) s += p[(size_t)r * W + c];
        }
    }
    out[(size_t)plane * per + o] = s / 4.0f;
}

// Per (plane, level): the means of ssim_map and cs in double, fixed order.
struct SsimLevels {
    int n;
    int Ho[kSsimMaxLevels], Wo[kSsimMaxLevels];
    int nblk[kSsimMaxLevels];
    long long part_off[kSsimMaxLevels];  // float2 offset of level l's partials
    float weight[kSsimMaxLevels];
};

__global__ __launch_bounds__(256) void ssim_reduce_kernel(const float2 *__restrict__ partial,
                                                          SsimLevels L, int planes,
                                                          double2 *__restrict__ stats) {
    __shared__ double s_a[256], s_b[256];
    const int plane = blockIdx.x, lvl = blockIdx.y;
    const int nb = L.nblk[lvl];
    const float2 *p = partial + L.part_off[lvl] + (size_t)plane * nb;
    double a = 0.0, b = 0.0;
    for (int k = threadIdx.x; k < nb; k += 256) {
        a += (double)p[k].x;
        b += (double)p[k].y;
    }
    s_a[threadIdx.x] = a;
    s_b[threadIdx.x] = b;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            s_a[threadIdx.x] += s_a[threadIdx.x + s];
            s_b[threadIdx.x] += s_b[threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const double cnt = (double)L.Ho[lvl] * (double)L.Wo[lvl];
        stats[(size_t)lvl * planes + plane] = make_double2(s_a[0] / cnt, s_b[0] / cnt);
    }
}

// Values (out[1] when size_average, else out[B]) and per-(level, plane)
// upstream factors {d value / d ssim_map pixel, d value / d cs pixel} per unit
// of the caller's output gradient.  flags: bit0 size_average, bit1
// nonnegative_ssim (single level).  One thread: planes are few (B*C).
__global__ void ssim_combine_kernel(const double2 *__restrict__ stats, SsimLevels L, int batch,
                                    int channels, int flags, float *__restrict__ out,
                                    float2 *__restrict__ fac) {
    if (threadIdx.x != 0) return;
    const int planes = batch * channels;
    const bool avg = flags & 1, nonneg = flags & 2;
    const double scale = avg ? 1.0 / (double)planes : 1.0 / (double)channels;
    double total = 0.0;
    for (int b = 0; b < batch; ++b) {
        double sum_b = 0.0;
        for (int c = 0; c < channels; ++c) {
            const int p = b * channels + c;
            double val;
            if (L.n == 1) {
                const double s = stats[p].x;
                val = (nonneg && s < 0.0) ? 0.0 : s;
                const double d = (nonneg && s <= 0.0) ? 0.0 : scale;
                const double cnt = (double)L.Ho[0] * (double)L.Wo[0];
                fac[p] = make_float2((float)(d / cnt), 0.0f);
            } else {
                double term[kSsimMaxLevels], base[kSsimMaxLevels];
                val = 1.0;
                for (int l = 0; l < L.n; ++l) {
                    const double raw = l < L.n - 1 ? stats[(size_t)l * planes + p].y
                                                   : stats[(size_t)l * planes + p].x;
                    base[l] = raw > 0.0 ? raw : 0.0;  // relu
                    term[l] = pow(base[l], (double)L.weight[l]);
                    val *= term[l];
                }
                for (int l = 0; l < L.n; ++l) {
                    double d = 0.0;
                    if (base[l] > 0.0) {
                        double others = 1.0;
                        for (int j = 0; j < L.n; ++j)
                            if (j != l) others *= term[j];
                        d = scale * (double)L.weight[l] * pow(base[l], (double)L.weight[l] - 1.0) *
                            others;
                    }
                    const double cnt = (double)L.Ho[l] * (double)L.Wo[l];
                    const float f = (float)(d / cnt);
                    fac[(size_t)l * planes + p] =
                        l < L.n - 1 ? make_float2(0.0f, f) : make_float2(f, 0.0f);
                }
            }
            sum_b += val;
        }
        if (!avg) out[b] = (float)(sum_b / (double)channels);
        total += sum_b;
    }
    if (avg) out[0] = (float)(total / (double)planes);
}

// ---------------------------------------------------------------- backward

constexpr int kBInH = kSsimTH + 2 * kSsimMaxWin - 2;   // 36 input rows
constexpr int kBInW = kSsimTW + 2 * kSsimMaxWin - 2;   // 84 input columns
constexpr int kBCoH = kSsimTH + kSsimMaxWin - 1;       // 26 coefficient rows
constexpr int kBCoW = kSsimTW + kSsimMaxWin - 1;       // 74 coefficient columns

__global__ __launch_bounds__(256) void ssim_bwd_kernel(
    const float *__restrict__ X, const float *__restrict__ Y, int H, int W, int Ho, int Wo,
    SsimWin w, float C1, float C2, const float2 *__restrict__ fac, const float *__restrict__ gout,
    int gdiv, const float *__restrict__ dcoarse, int Hc, int Wc, int pr, int pc,
    float *__restrict__ dX) {
    // phase buffers: inputs [2][36][84] then coefficients [3][26][74];
    // vertical moments [5][26][84] then transposed partials [3][16][74]
    __shared__ float s_a[2 * kBInH * kBInW];
    __shared__ float s_b[5 * kBCoH * kBInW];
    const int tid = threadIdx.x;
    const int plane = blockIdx.z;
    const int r0 = blockIdx.y * kSsimTH, c0 = blockIdx.x * kSsimTW;
    const size_t hw = (size_t)H * (size_t)W;
    const float *x = X + plane * hw, *y = Y + plane * hw;
    const int kv = w.kv, kh = w.kh;
    const int ir0 = r0 - (kv - 1), ic0 = c0 - (kh - 1);
    const int inh = kSsimTH + 2 * (kv - 1), inw = kSsimTW + 2 * (kh - 1);
    const int coh = kSsimTH + kv - 1, cow = kSsimTW + kh - 1;
    const float g = gout[gdiv > 0 ? plane / gdiv : 0];
    const float2 f = fac[plane];
    const float us = f.x * g, uc = f.y * g;
    float *in_x = s_a, *in_y = s_a + kBInH * kBInW;  // [36][84] each
    for (int k = tid; k < inh * inw; k += 256) {
        const int rr = k / inw, cc = k - rr * inw;
        const int gr = ir0 + rr, gc = ic0 + cc;
        float a = 0.f, b = 0.f;
        if (gr >= 0 && gr < H && gc >= 0 && gc < W) {
            a = x[(size_t)gr * W + gc];
            b = y[(size_t)gr * W + gc];
        }
        in_x[rr * kBInW + cc] = a;
        in_y[rr * kBInW + cc] = b;
    }
    __syncthreads();
    // vertical moments at coefficient rows, all input columns
    for (int k = tid; k < coh * inw; k += 256) {
        const int rr = k / inw, cc = k - rr * inw;
        float m1 = 0.f, m2 = 0.f, e11 = 0.f, e22 = 0.f, e12 = 0.f;
#pragma unroll
        for (int t = 0; t < kSsimMaxWin; ++t) {
            if (t < kv) {
                const float a = in_x[(rr + t) * kBInW + cc], b = in_y[(rr + t) * kBInW + cc];
                const float q = w.wv[t];
                m1 = fmaf(q, a, m1);
                m2 = fmaf(q, b, m2);
                e11 = fmaf(q, a * a, e11);
                e22 = fmaf(q, b * b, e22);
                e12 = fmaf(q, a * b, e12);
            }
        }
        const int o = rr * kBInW + cc;
        s_b[o] = m1;
        s_b[kBCoH * kBInW + o] = m2;
        s_b[2 * kBCoH * kBInW + o] = e11;
        s_b[3 * kBCoH * kBInW + o] = e22;
        s_b[4 * kBCoH * kBInW + o] = e12;
    }
    __syncthreads();
    // coefficients at every output p of the region (zero outside [0,Ho)x[0,Wo))
    float *co = s_a;  // [3][26][74]
    for (int k = tid; k < coh * cow; k += 256) {
        const int rr = k / cow, cc = k - rr * cow;
        const int pr_ = ir0 + rr, pc_ = ic0 + cc;
        float ga = 0.f, gb = 0.f, gc = 0.f;
        if (pr_ >= 0 && pr_ < Ho && pc_ >= 0 && pc_ < Wo) {
            float m[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int t = 0; t < kSsimMaxWin; ++t) {
                if (t < kh) {
#pragma unroll
                    for (int q = 0; q < 5; ++q)
                        m[q] = fmaf(w.wh[t], s_b[q * kBCoH * kBInW + rr * kBInW + cc + t], m[q]);
                }
            }
            const float mu1_sq = m[0] * m[0], mu2_sq = m[1] * m[1], mu12 = m[0] * m[1];
            const float s1 = m[2] - mu1_sq, s2 = m[3] - mu2_sq, s12 = m[4] - mu12;
            const float B1 = (mu1_sq + mu2_sq) + C1, B2 = (s1 + s2) + C2;
            const float l = (2.0f * mu12 + C1) / B1;
            const float cs = (2.0f * s12 + C2) / B2;
            const float dl_dm1 = (2.0f * m[1] - 2.0f * m[0] * l) / B1;
            const float dcs_dm1 = (2.0f * m[0] * cs - 2.0f * m[1]) / B2;
            const float k_cs = us * l + uc;  // d loss / d cs through both routes
            ga = us * (dl_dm1 * cs) + k_cs * dcs_dm1;
            gb = k_cs * (-cs / B2);
            gc = k_cs * (2.0f / B2);
        }
        co[rr * kBCoW + cc] = ga;
        co[kBCoH * kBCoW + rr * kBCoW + cc] = gb;
        co[2 * kBCoH * kBCoW + rr * kBCoW + cc] = gc;
    }
    __syncthreads();
    // transposed vertical: tile rows x coefficient columns
    float *tv = s_b;  // [3][16][74]
    for (int k = tid; k < kSsimTH * cow; k += 256) {
        const int rr = k / cow, cc = k - rr * cow;
        float a = 0.f, b = 0.f, c = 0.f;
#pragma unroll
        for (int t = 0; t < kSsimMaxWin; ++t) {
            if (t < kv) {
                const int src = (rr + kv - 1 - t) * kBCoW + cc;
                const float q = w.wv[t];
                a = fmaf(q, co[src], a);
                b = fmaf(q, co[kBCoH * kBCoW + src], b);
                c = fmaf(q, co[2 * kBCoH * kBCoW + src], c);
            }
        }
        tv[rr * kBCoW + cc] = a;
        tv[kSsimTH * kBCoW + rr * kBCoW + cc] = b;
        tv[2 * kSsimTH * kBCoW + rr * kBCoW + cc] = c;
    }
    __syncthreads();
    float *dx = dX + plane * hw;
    const float *dc = dcoarse ? dcoarse + (size_t)plane * Hc * Wc : nullptr;
#pragma unroll
    for (int j = 0; j < kSsimTH * kSsimTW / 256; ++j) {
        const int k = tid + 256 * j;
        const int rr = k / kSsimTW, cc = k - rr * kSsimTW;
        const int qr = r0 + rr, qc = c0 + cc;
        if (qr >= H || qc >= W) continue;
        float a = 0.f, b = 0.f, c = 0.f;
#pragma unroll
        for (int t = 0; t < kSsimMaxWin; ++t) {
            if (t < kh) {
                const int src = rr * kBCoW + cc + kh - 1 - t;
                const float q = w.wh[t];
                a = fmaf(q, tv[src], a);
                b = fmaf(q, tv[kSsimTH * kBCoW + src], b);
                c = fmaf(q, tv[2 * kSsimTH * kBCoW + src], c);
            }
        }
        const size_t qi = (size_t)qr * W + qc;
        float v = a + 2.0f * x[qi] * b + y[qi] * c;
        if (dc) {
            const int orow = (qr + pr) >> 1, ocol = (qc + pc) >> 1;
            if (orow < Hc && ocol < Wc) v += 0.25f * dc[(size_t)orow * Wc + ocol];
        }
        dx[qi] = v;
    }
}

}  // namespace gsvc

using namespace gsvc;

namespace {

struct SsimPlan {
    int levels, H[kSsimMaxLevels], W[kSsimMaxLevels], pr[kSsimMaxLevels], pc[kSsimMaxLevels];
    SsimWin win[kSsimMaxLevels];
    SsimLevels L;
    // workspace
    size_t pyr_off[kSsimMaxLevels];  // floats: X_l at pyr_off[l], Y_l right after (l >= 1)
    size_t dx_off[kSsimMaxLevels];   // floats: dX_l (l >= 1)
    size_t part_off, stats_off, fac_off, bytes;
};

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

int make_plan(int planes, int H, int W, int win_size, float sigma, int levels,
              const double *weights, SsimPlan &P) {
    if (planes <= 0 || H <= 0 || W <= 0) return set_error(GSVC_ERR_ARG, "ssim: empty input");
    if (win_size < 1 || win_size > kSsimMaxWin || !(win_size & 1))
        return set_error(GSVC_ERR_ARG, "ssim: window size must be odd and at most %d", kSsimMaxWin);
    if (levels < 1 || levels > kSsimMaxLevels) return set_error(GSVC_ERR_ARG, "ssim: levels");
    // _fspecial_gauss_1d: coords - size//2, exp(-(c^2) / (2 sigma^2)), normalised (fp32)
    float g[kSsimMaxWin], sum = 0.f;
    for (int t = 0; t < win_size; ++t) {
        const float c = (float)(t - win_size / 2);
        g[t] = expf(-(c * c) / (2.0f * sigma * sigma));
        sum += g[t];
    }
    for (int t = 0; t < win_size; ++t) g[t] /= sum;
    P.levels = levels;
    P.L.n = levels;
    size_t off = 0;  // bytes
    int h = H, w = W;
    long long part = 0;
    for (int l = 0; l < levels; ++l) {
        P.H[l] = h;
        P.W[l] = w;
        SsimWin &wn = P.win[l];
        wn.kv = h >= win_size ? win_size : 1;
        wn.kh = w >= win_size ? win_size : 1;
        for (int t = 0; t < kSsimMaxWin; ++t) {
            wn.wv[t] = wn.kv == 1 ? (t == 0 ? 1.0f : 0.0f) : (t < win_size ? g[t] : 0.0f);
            wn.wh[t] = wn.kh == 1 ? (t == 0 ? 1.0f : 0.0f) : (t < win_size ? g[t] : 0.0f);
        }
        P.L.Ho[l] = h - wn.kv + 1;
        P.L.Wo[l] = w - wn.kh + 1;
        P.L.nblk[l] = ceil_div(P.L.Wo[l], kSsimTW) * ceil_div(P.L.Ho[l], kSsimTH);
        P.L.part_off[l] = part;
        part += (long long)P.L.nblk[l] * planes;
        P.L.weight[l] = weights ? (float)weights[l] : 1.0f;
        if (l >= 1) {
            P.pyr_off[l] = off / sizeof(float);
            off += align256(sizeof(float) * 2 * (size_t)planes * h * w);
            P.dx_off[l] = off / sizeof(float);
            off += align256(sizeof(float) * (size_t)planes * h * w);
        }
        P.pr[l] = h % 2;
        P.pc[l] = w % 2;
        // F.avg_pool2d(kernel 2, stride 2, padding p): (n + 2p - 2) / 2 + 1
        h = (h + 2 * P.pr[l] - 2) / 2 + 1;
        w = (w + 2 * P.pc[l] - 2) / 2 + 1;
    }
    P.part_off = off;
    off += align256(sizeof(float2) * (size_t)part);
    P.stats_off = off;
    off += align256(sizeof(double2) * (size_t)levels * planes);
    P.fac_off = off;
    off += align256(sizeof(float2) * (size_t)levels * planes);
    P.bytes = off;
    return 0;
}

const float *level_x(const SsimPlan &P, int l, const float *X0, char *ws, int planes) {
    if (l == 0) return X0;
    return reinterpret_cast<float *>(ws) + P.pyr_off[l];
}
const float *level_y(const SsimPlan &P, int l, const float *Y0, char *ws, int planes) {
    if (l == 0) return Y0;
    return reinterpret_cast<float *>(ws) + P.pyr_off[l] + (size_t)planes * P.H[l] * P.W[l];
}

}  // namespace

extern "C" size_t gsvc_ssim_workspace_bytes(int planes, int height, int width, int win_size,
                                            int levels) {
    SsimPlan P;
    if (make_plan(planes, height, width, win_size, 1.5f, levels, nullptr, P) != 0) return 0;
    return P.bytes;
}

extern "C" int gsvc_ssim_forward(int batch, int channels, int height, int width, const float *X,
                                 const float *Y, int win_size, float win_sigma, float C1, float C2,
                                 int levels, const double *weights, int flags, float *out,
                                 void *ws, size_t ws_bytes, void *stream) {
    const int planes = batch * channels;
    SsimPlan P;
    if (int rc = make_plan(planes, height, width, win_size, win_sigma, levels, weights, P)) return rc;
    if (!X || !Y || !out || !ws) return set_error(GSVC_ERR_ARG, "ssim: missing buffer");
    if (ws_bytes < P.bytes) return set_error(GSVC_ERR_WORKSPACE, "ssim: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    char *w = (char *)ws;
    float2 *part = reinterpret_cast<float2 *>(w + P.part_off);
    for (int l = 0; l < levels; ++l) {
        const float *xl = level_x(P, l, X, w, planes), *yl = level_y(P, l, Y, w, planes);
        if (l >= 1) {
            const float *xp = level_x(P, l - 1, X, w, planes), *yp = level_y(P, l - 1, Y, w, planes);
            const long long n = (long long)planes * P.H[l] * P.W[l];
            const unsigned blocks = (unsigned)((n + 255) / 256);
            hipLaunchKernelGGL(ssim_pool_kernel, dim3(blocks), dim3(256), 0, s, xp, P.H[l - 1],
                               P.W[l - 1], const_cast<float *>(xl), P.H[l], P.W[l], P.pr[l - 1],
                               P.pc[l - 1], planes);
            hipLaunchKernelGGL(ssim_pool_kernel, dim3(blocks), dim3(256), 0, s, yp, P.H[l - 1],
                               P.W[l - 1], const_cast<float *>(yl), P.H[l], P.W[l], P.pr[l - 1],
                               P.pc[l - 1], planes);
        }
        const dim3 grid(ceil_div(P.L.Wo[l], kSsimTW), ceil_div(P.L.Ho[l], kSsimTH), planes);
        hipLaunchKernelGGL(ssim_fwd_kernel, grid, dim3(256), 0, s, xl, yl, P.H[l], P.W[l],
                           P.L.Ho[l], P.L.Wo[l], P.win[l], C1, C2, part + P.L.part_off[l]);
    }
    double2 *stats = reinterpret_cast<double2 *>(w + P.stats_off);
    hipLaunchKernelGGL(ssim_reduce_kernel, dim3(planes, levels), dim3(256), 0, s, part, P.L,
                       planes, stats);
    hipLaunchKernelGGL(ssim_combine_kernel, dim3(1), dim3(64), 0, s, stats, P.L, batch, channels,
                       flags, out, reinterpret_cast<float2 *>(w + P.fac_off));
    return check_launch("ssim forward");
}

extern "C" int gsvc_ssim_backward(int batch, int channels, int height, int width, const float *X,
                                  const float *Y, int win_size, float win_sigma, float C1,
                                  float C2, int levels, int flags, const float *grad_out,
                                  float *dX, float *dY, void *ws, size_t ws_bytes, void *stream) {
    const int planes = batch * channels;
    SsimPlan P;
    if (int rc = make_plan(planes, height, width, win_size, win_sigma, levels, nullptr, P)) return rc;
    if (!X || !Y || !grad_out || !ws) return set_error(GSVC_ERR_ARG, "ssim: missing buffer");
    if (ws_bytes < P.bytes) return set_error(GSVC_ERR_WORKSPACE, "ssim: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    char *w = (char *)ws;
    const float2 *fac = reinterpret_cast<const float2 *>(w + P.fac_off);
    const int gdiv = (flags & 1) ? 0 : channels;
    for (int side = 0; side < 2; ++side) {
        float *dst0 = side == 0 ? dX : dY;
        if (!dst0) continue;
        // SSIM is symmetric in X and Y: d/dY is d/dX with the two swapped
        for (int l = levels - 1; l >= 0; --l) {
            const float *xl = level_x(P, l, X, w, planes), *yl = level_y(P, l, Y, w, planes);
            if (side == 1) {
                const float *t = xl;
                xl = yl;
                yl = t;
            }
            float *dst = l == 0 ? dst0 : reinterpret_cast<float *>(w) + P.dx_off[l];
            const float *dc = l + 1 < levels ? reinterpret_cast<float *>(w) + P.dx_off[l + 1] : nullptr;
            const dim3 grid(ceil_div(P.W[l], kSsimTW), ceil_div(P.H[l], kSsimTH), planes);
            hipLaunchKernelGGL(ssim_bwd_kernel, grid, dim3(256), 0, s, xl, yl, P.H[l], P.W[l],
                               P.L.Ho[l], P.L.Wo[l], P.win[l], C1, C2, fac + (size_t)l * planes,
                               grad_out, gdiv, dc, l + 1 < levels ? P.H[l + 1] : 0,
                               l + 1 < levels ? P.W[l + 1] : 0, P.pr[l], P.pc[l], dst);
        }
    }
    return check_launch("ssim backward");
}
