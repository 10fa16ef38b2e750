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
// over (W tiles, H tiles, planes) of ssim_moments_kernel: the 5 windowed
// moments of a 16x64 output tile from its 26x74 input region (every load
// issued before the first LDS store; vertical pass over 4-row runs, horizontal
// over 4-column runs read as conflict-free ds_read_b128), then per-block sums
// of ssim_map and cs, reduced in double in a fixed order (ssim_reduce_kernel);
// ssim_combine_kernel forms the values and the per-plane upstream factors the
// backward needs -- nothing goes to the host.
// Backward (w.r.t. X; w.r.t. Y by symmetry with X and Y swapped), per level
// from the coarsest: ssim_moments_kernel<true> writes the per-output
// coefficients (g_mu1, g_E11, g_E12) as 3 maps, ssim_grad_kernel applies the
// transposed filter,
//   dX = w^T*g_mu1 + 2 X (w^T*g_E11) + Y (w^T*g_E12),
// and adds the coarser level's gradient through the average pool.
// 1080p x 3: forward 82 us (SSIM) / 162 us (MS-SSIM), forward + backward
// 250 / 444 us (tools/ssimbench.py; torch conv2d restatement: 3.9 / 6.9 ms
// and 6.6 / 11.7 ms).  The level-0 moments launch is latency/LDS-issue bound
// (73 us for 50 MB of input).
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

// ---------------------------------------------------------------- moments

constexpr int kRegH = kSsimTH + kSsimMaxWin - 1;  // 26 input rows of a tile
constexpr int kRegW = kSsimTW + kSsimMaxWin - 1;  // 74 input columns
constexpr int kRowP = 76;                          // padded row of the float4-read buffers
constexpr int kRun = 4;                            // rows / columns per thread per pass
constexpr int kSpan = kRun + kSsimMaxWin - 1;      // 14 values a 4-run reads

// Column run of a thread in the 4-column passes: 16 lanes cover one 64-column
// row, and the lane -> run map differs by row parity so that every 16-lane
// group of a ds_read_b128 (two rows, 76-float stride = 3 chunks of bank shift)
// reads 16 distinct 4-bank chunks: no bank conflicts.
__device__ __forceinline__ int run_of_lane(int tid) {
    const int l = tid & 15;
    if ((tid >> 4) & 1) return (l + 1) & 15;
    return l < 4 ? l : (l < 12 ? l + 4 : l - 8);
}

// All four floats of an LDS float4 (one ds_read_b128 even when the caller
// uses only some of them).
__device__ __forceinline__ float4 lds_f4(const float *p) {
    float4 f = *reinterpret_cast<const float4 *>(p);
    asm volatile("" : "+v"(f.x), "+v"(f.y), "+v"(f.z), "+v"(f.w));
    return f;
}

// Per output of the plane: the SSIM terms at one window position.
struct SsimTerms {
    float mu1, mu2, B1, B2, l, cs;
};
__device__ __forceinline__ SsimTerms ssim_terms(const float m[5], float C1, float C2) {
    SsimTerms T;
    const float mu1_sq = m[0] * m[0], mu2_sq = m[1] * m[1], mu12 = m[0] * m[1];
    const float s1 = m[2] - mu1_sq, s2 = m[3] - mu2_sq, s12 = m[4] - mu12;
    T.mu1 = m[0];
    T.mu2 = m[1];
    T.B1 = (mu1_sq + mu2_sq) + C1;
    T.B2 = (s1 + s2) + C2;
    T.cs = (2.0f * s12 + C2) / T.B2;            // cs_map
    T.l = (2.0f * mu12 + C1) / T.B1;            // ssim_map = l * cs
    return T;
}

// One 16x64 output tile of a plane: the 5 windowed moments (vertical pass over
// 4-row runs, horizontal pass over 4-column runs read as float4s), then
//   kCoef = false: the tile's sums of ssim_map and cs -> partial[plane][tile];
//   kCoef = true : the backward coefficients of every output,
//     g_mu1 = us (dl/dmu1 cs + l dcs/dmu1) + uc dcs/dmu1,
//     g_E11 = (us l + uc) dcs/dE11,  g_E12 = (us l + uc) dcs/dE12,
//     with us, uc = the plane's upstream factors times the output gradient,
//   -> coef[plane][3][Ho][Wo].
template <bool kCoef>
__global__ __launch_bounds__(256) void ssim_moments_kernel(
    const float *__restrict__ X, const float *__restrict__ Y, int H, int W, int Ho, int Wo,
    SsimWin w, float C1, float C2, float2 *__restrict__ partial, const float2 *__restrict__ fac,
    const float *__restrict__ gout, int gdiv, float *__restrict__ coef) {
    __shared__ float s_x[kRegH][kRegW], s_y[kRegH][kRegW];
    __shared__ __attribute__((aligned(16))) float s_v[5][kSsimTH][kRowP];
    __shared__ float2 s_red[4];
    const int tid = threadIdx.x;
    const int plane = blockIdx.z;
    const int r0 = blockIdx.y * kSsimTH, c0 = blockIdx.x * kSsimTW;
    const size_t hw = (size_t)H * (size_t)W;
    const float *x = X + plane * hw, *y = Y + plane * hw;
    const int kv = w.kv, kh = w.kh;
    const int inw = kSsimTW + kh - 1;
    {  // the whole 26x74 region, every load issued before the first LDS store
        constexpr int kN = (kRegH * kRegW + 255) / 256;
        float a[kN], b[kN];
#pragma unroll
        for (int j = 0; j < kN; ++j) {
            const int k = tid + 256 * j;
            const int rr = k / kRegW, cc = k - rr * kRegW;
            const int gr = r0 + rr, gc = c0 + cc;
            a[j] = 0.f;
            b[j] = 0.f;
            if (k < kRegH * kRegW && gr < H && gc < W) {
                a[j] = x[(size_t)gr * W + gc];
                b[j] = y[(size_t)gr * W + gc];
            }
        }
#pragma unroll
        for (int j = 0; j < kN; ++j) {
            const int k = tid + 256 * j;
            if (k < kRegH * kRegW) {
                const int rr = k / kRegW, cc = k - rr * kRegW;
                s_x[rr][cc] = a[j];
                s_y[rr][cc] = b[j];
            }
        }
    }
    __syncthreads();
    {  // vertical: lane = column, wave = a run of 4 rows
        const int tx = tid & 63, rb = (tid >> 6) * kRun;
        for (int cc = tx; cc < inw; cc += 64) {
            float a[kSpan], b[kSpan];
#pragma unroll
            for (int j = 0; j < kSpan; ++j) {
                if (j < kRun + kv - 1) {
                    a[j] = s_x[rb + j][cc];
                    b[j] = s_y[rb + j][cc];
                }
            }
#pragma unroll
            for (int r = 0; r < kRun; ++r) {
                float m1 = 0.f, m2 = 0.f, e11 = 0.f, e22 = 0.f, e12 = 0.f;
#pragma unroll
                for (int t = 0; t < kSsimMaxWin; ++t) {
                    if (t < kv) {
                        const float av = a[r + t], bv = b[r + t], q = w.wv[t];
                        m1 = fmaf(q, av, m1);
                        m2 = fmaf(q, bv, m2);
                        e11 = fmaf(q, av * av, e11);
                        e22 = fmaf(q, bv * bv, e22);
                        e12 = fmaf(q, av * bv, e12);
                    }
                }
                s_v[0][rb + r][cc] = m1;
                s_v[1][rb + r][cc] = m2;
                s_v[2][rb + r][cc] = e11;
                s_v[3][rb + r][cc] = e22;
                s_v[4][rb + r][cc] = e12;
            }
        }
    }
    __syncthreads();
    // horizontal: a thread owns 4 consecutive outputs of one row
    const int rr = tid >> 4, cb = run_of_lane(tid) * kRun;
    float m[kRun][5];
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        float v[16];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float4 f = lds_f4(&s_v[q][rr][cb + 4 * j]);
            v[4 * j] = f.x;
            v[4 * j + 1] = f.y;
            v[4 * j + 2] = f.z;
            v[4 * j + 3] = f.w;
        }
#pragma unroll
        for (int c = 0; c < kRun; ++c) {
            float acc = 0.f;
#pragma unroll
            for (int t = 0; t < kSsimMaxWin; ++t)
                if (t < kh) acc = fmaf(w.wh[t], v[c + t], acc);
            m[c][q] = acc;
        }
    }
    const int orow = r0 + rr;
    if (!kCoef) {
        float acc_s = 0.f, acc_c = 0.f;
#pragma unroll
        for (int c = 0; c < kRun; ++c) {
            if (orow < Ho && c0 + cb + c < Wo) {
                const SsimTerms T = ssim_terms(m[c], C1, C2);
                acc_s += T.l * T.cs;
                acc_c += T.cs;
            }
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
    } else {
        const float g = gout[gdiv > 0 ? plane / gdiv : 0];
        const float2 f = fac[plane];
        const float us = f.x * g, uc = f.y * g;
        const size_t ohw = (size_t)Ho * (size_t)Wo;
        float *co = coef + (size_t)plane * 3 * ohw;
#pragma unroll
        for (int c = 0; c < kRun; ++c) {
            const int ocol = c0 + cb + c;
            if (orow < Ho && ocol < Wo) {
                const SsimTerms T = ssim_terms(m[c], C1, C2);
                const float dl_dm1 = (2.0f * T.mu2 - 2.0f * T.mu1 * T.l) / T.B1;
                const float dcs_dm1 = (2.0f * T.mu1 * T.cs - 2.0f * T.mu2) / T.B2;
                const float k_cs = us * T.l + uc;  // d loss / d cs through both routes
                const size_t o = (size_t)orow * Wo + ocol;
                co[o] = us * (dl_dm1 * T.cs) + k_cs * dcs_dm1;
                co[ohw + o] = k_cs * (-T.cs / T.B2);
                co[2 * ohw + o] = k_cs * (2.0f / T.B2);
            }
        }
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
// nonnegative_ssim (single level).  A thread per plane forms its value in fp32
// as the package does (relu, ** weights, product); thread 0 then takes the
// means over planes in double, in plane order.
__global__ __launch_bounds__(256) void ssim_combine_kernel(const double2 *__restrict__ stats,
                                                           SsimLevels L, int batch, int channels,
                                                           int flags, float *__restrict__ out,
                                                           float2 *__restrict__ fac,
                                                           float *__restrict__ vals) {
    const int planes = batch * channels;
    const bool avg = flags & 1, nonneg = flags & 2;
    const float scale = avg ? 1.0f / (float)planes : 1.0f / (float)channels;
    for (int p = threadIdx.x; p < planes; p += blockDim.x) {
        float val;
        if (L.n == 1) {
            const float s = (float)stats[p].x;
            val = (nonneg && s < 0.0f) ? 0.0f : s;
            const float d = (nonneg && s <= 0.0f) ? 0.0f : scale;
            fac[p] = make_float2(d / ((float)L.Ho[0] * (float)L.Wo[0]), 0.0f);
        } else {
            float term[kSsimMaxLevels], base[kSsimMaxLevels];
            val = 1.0f;
            for (int l = 0; l < L.n; ++l) {
                const float raw = (float)(l < L.n - 1 ? stats[(size_t)l * planes + p].y
                                                      : stats[(size_t)l * planes + p].x);
                base[l] = raw > 0.0f ? raw : 0.0f;  // relu
                term[l] = powf(base[l], L.weight[l]);
                val *= term[l];
            }
            for (int l = 0; l < L.n; ++l) {
                float d = 0.0f;
                if (base[l] > 0.0f) {  // relu'(0) = 0
                    float others = 1.0f;
                    for (int j = 0; j < L.n; ++j)
                        if (j != l) others *= term[j];
                    d = scale * L.weight[l] * powf(base[l], L.weight[l] - 1.0f) * others;
                }
                const float f = d / ((float)L.Ho[l] * (float)L.Wo[l]);
                fac[(size_t)l * planes + p] = l < L.n - 1 ? make_float2(0.0f, f) : make_float2(f, 0.0f);
            }
        }
        vals[p] = val;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    double total = 0.0;
    for (int b = 0; b < batch; ++b) {
        double sum_b = 0.0;
        for (int c = 0; c < channels; ++c) sum_b += (double)vals[b * channels + c];
        if (!avg) out[b] = (float)(sum_b / (double)channels);
        total += sum_b;
    }
    if (avg) out[0] = (float)(total / (double)planes);
}

// ---------------------------------------------------------------- backward

// Input gradient of one 16x64 tile of a plane from the coefficient maps:
//   dX = w^T * g_mu1 + 2 X (w^T * g_E11) + Y (w^T * g_E12)
// (transposed separable filter: vertical 4-row runs, horizontal 4-column runs),
// plus the coarser level's gradient through the 2x2 average pool (1/4 each).
__global__ __launch_bounds__(256) void ssim_grad_kernel(
    const float *__restrict__ coef, int Ho, int Wo, const float *__restrict__ X,
    const float *__restrict__ Y, int H, int W, SsimWin w, const float *__restrict__ dcoarse,
    int Hc, int Wc, int pr, int pc, float *__restrict__ dX) {
    __shared__ float s_co[3][kRegH][kRegW];
    __shared__ __attribute__((aligned(16))) float s_t[3][kSsimTH][kRowP];
    const int tid = threadIdx.x;
    const int plane = blockIdx.z;
    const int r0 = blockIdx.y * kSsimTH, c0 = blockIdx.x * kSsimTW;
    const int kv = w.kv, kh = w.kh;
    const int ir0 = r0 - (kv - 1), ic0 = c0 - (kh - 1);
    const int coh = kSsimTH + kv - 1, cow = kSsimTW + kh - 1;
    const size_t ohw = (size_t)Ho * (size_t)Wo;
    const float *co = coef + (size_t)plane * 3 * ohw;
    {  // the 26x74 coefficient region, every load issued before the first LDS store
        constexpr int kN = (kRegH * kRegW + 255) / 256;
        float a[kN], b[kN], c[kN];
#pragma unroll
        for (int j = 0; j < kN; ++j) {
            const int k = tid + 256 * j;
            const int rr = k / kRegW, cc = k - rr * kRegW;
            const int p_r = ir0 + rr, p_c = ic0 + cc;
            a[j] = 0.f;
            b[j] = 0.f;
            c[j] = 0.f;
            if (k < kRegH * kRegW && rr < coh && cc < cow && p_r >= 0 && p_r < Ho && p_c >= 0 &&
                p_c < Wo) {
                const size_t o = (size_t)p_r * Wo + p_c;
                a[j] = co[o];
                b[j] = co[ohw + o];
                c[j] = co[2 * ohw + o];
            }
        }
#pragma unroll
        for (int j = 0; j < kN; ++j) {
            const int k = tid + 256 * j;
            if (k < kRegH * kRegW) {
                const int rr = k / kRegW, cc = k - rr * kRegW;
                s_co[0][rr][cc] = a[j];
                s_co[1][rr][cc] = b[j];
                s_co[2][rr][cc] = c[j];
            }
        }
    }
    __syncthreads();
    {  // transposed vertical: row rb + r gathers coefficient rows rb + r + kv-1-t
        const int tx = tid & 63, rb = (tid >> 6) * kRun;
        for (int cc = tx; cc < cow; cc += 64) {
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                float v[kSpan];
#pragma unroll
                for (int j = 0; j < kSpan; ++j)
                    if (j < kRun + kv - 1) v[j] = s_co[q][rb + j][cc];
#pragma unroll
                for (int r = 0; r < kRun; ++r) {
                    float acc = 0.f;
#pragma unroll
                    for (int t = 0; t < kSsimMaxWin; ++t)
                        if (t < kv) acc = fmaf(w.wv[t], v[r + kv - 1 - t], acc);
                    s_t[q][rb + r][cc] = acc;
                }
            }
        }
    }
    __syncthreads();
    const int rr = tid >> 4, cb = run_of_lane(tid) * kRun;
    float G[3][kRun];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        float v[16];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float4 f = lds_f4(&s_t[q][rr][cb + 4 * j]);
            v[4 * j] = f.x;
            v[4 * j + 1] = f.y;
            v[4 * j + 2] = f.z;
            v[4 * j + 3] = f.w;
        }
#pragma unroll
        for (int c = 0; c < kRun; ++c) {
            float acc = 0.f;
#pragma unroll
            for (int t = 0; t < kSsimMaxWin; ++t)
                if (t < kh) acc = fmaf(w.wh[t], v[c + kh - 1 - t], acc);
            G[q][c] = acc;
        }
    }
    const int qr = r0 + rr;
    if (qr >= H) return;
    const size_t hw = (size_t)H * (size_t)W;
    const float *x = X + plane * hw, *y = Y + plane * hw;
    float *dx = dX + plane * hw;
    const float *dc = dcoarse ? dcoarse + (size_t)plane * Hc * Wc : nullptr;
    const int orow = (qr + pr) >> 1;
#pragma unroll
    for (int c = 0; c < kRun; ++c) {
        const int qc = c0 + cb + c;
        if (qc >= W) break;
        const size_t qi = (size_t)qr * W + qc;
        float v = G[0][c] + 2.0f * x[qi] * G[1][c] + y[qi] * G[2][c];
        if (dc) {
            const int ocol = (qc + pc) >> 1;
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
    // forward workspace (kept for the backward): pyramid, partials, stats, factors
    size_t part_off, stats_off, fac_off, vals_off, bytes;
    // backward scratch: the coefficient maps of level 0's size, dX_l (l >= 1)
    size_t dx_off[kSsimMaxLevels];   // floats
    size_t coef_off, scratch_bytes;
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
    size_t off = 0, soff = 0;  // bytes: workspace, scratch
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
            P.dx_off[l] = soff / sizeof(float);
            soff += align256(sizeof(float) * (size_t)planes * h * w);
        }
        P.pr[l] = h % 2;
        P.pc[l] = w % 2;
        // F.avg_pool2d(kernel 2, stride 2, padding p): (n + 2p - 2) / 2 + 1
        h = (h + 2 * P.pr[l] - 2) / 2 + 1;
        w = (w + 2 * P.pc[l] - 2) / 2 + 1;
    }
    P.part_off = off;
    off += align256(sizeof(float2) * (size_t)part);
    P.coef_off = soff;  // [P][3][Ho][Wo] of level 0
    soff += align256(sizeof(float) * 3 * (size_t)planes * P.L.Ho[0] * P.L.Wo[0]);
    P.scratch_bytes = soff;
    P.stats_off = off;
    off += align256(sizeof(double2) * (size_t)levels * planes);
    P.fac_off = off;
    off += align256(sizeof(float2) * (size_t)levels * planes);
    P.vals_off = off;
    off += align256(sizeof(float) * (size_t)planes);
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

extern "C" size_t gsvc_ssim_backward_scratch_bytes(int planes, int height, int width,
                                                   int win_size, int levels) {
    SsimPlan P;
    if (make_plan(planes, height, width, win_size, 1.5f, levels, nullptr, P) != 0) return 0;
    return P.scratch_bytes;
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
        auto kfn = ssim_moments_kernel<false>;
        hipLaunchKernelGGL(kfn, grid, dim3(256), 0, s, xl, yl, P.H[l], P.W[l], P.L.Ho[l],
                           P.L.Wo[l], P.win[l], C1, C2, part + P.L.part_off[l], nullptr, nullptr,
                           0, nullptr);
    }
    double2 *stats = reinterpret_cast<double2 *>(w + P.stats_off);
    hipLaunchKernelGGL(ssim_reduce_kernel, dim3(planes, levels), dim3(256), 0, s, part, P.L,
                       planes, stats);
    hipLaunchKernelGGL(ssim_combine_kernel, dim3(1), dim3(256), 0, s, stats, P.L, batch, channels,
                       flags, out, reinterpret_cast<float2 *>(w + P.fac_off),
                       reinterpret_cast<float *>(w + P.vals_off));
    return check_launch("ssim forward");
}

extern "C" int gsvc_ssim_backward(int batch, int channels, int height, int width, const float *X,
                                  const float *Y, int win_size, float win_sigma, float C1,
                                  float C2, int levels, int flags, const float *grad_out,
                                  float *dX, float *dY, void *ws, size_t ws_bytes, void *scratch,
                                  size_t scratch_bytes, void *stream) {
    const int planes = batch * channels;
    SsimPlan P;
    if (int rc = make_plan(planes, height, width, win_size, win_sigma, levels, nullptr, P)) return rc;
    if (!X || !Y || !grad_out || !ws || !scratch)
        return set_error(GSVC_ERR_ARG, "ssim: missing buffer");
    if (ws_bytes < P.bytes || scratch_bytes < P.scratch_bytes)
        return set_error(GSVC_ERR_WORKSPACE, "ssim: workspace or scratch too small");
    hipStream_t s = (hipStream_t)stream;
    char *w = (char *)ws;
    float *sc = reinterpret_cast<float *>(scratch);
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
            float *dst = l == 0 ? dst0 : sc + P.dx_off[l];
            const float *dc = l + 1 < levels ? sc + P.dx_off[l + 1] : nullptr;
            float *coef = sc + P.coef_off / sizeof(float);
            const dim3 ogrid(ceil_div(P.L.Wo[l], kSsimTW), ceil_div(P.L.Ho[l], kSsimTH), planes);
            auto kfn = ssim_moments_kernel<true>;
            hipLaunchKernelGGL(kfn, ogrid, dim3(256), 0, s, xl, yl, P.H[l], P.W[l], P.L.Ho[l],
                               P.L.Wo[l], P.win[l], C1, C2, nullptr, fac + (size_t)l * planes,
                               grad_out, gdiv, coef);
            const dim3 igrid(ceil_div(P.W[l], kSsimTW), ceil_div(P.H[l], kSsimTH), planes);
            hipLaunchKernelGGL(ssim_grad_kernel, igrid, dim3(256), 0, s, coef, P.L.Ho[l], P.L.Wo[l],
                               xl, yl, P.H[l], P.W[l], P.win[l], dc,
                               l + 1 < levels ? P.H[l + 1] : 0, l + 1 < levels ? P.W[l + 1] : 0,
                               P.pr[l], P.pc[l], dst);
        }
    }
    return check_launch("ssim backward");
}
