// VALU issue rate of one MI355X (gfx950) SIMD, measured: wave64 instructions
// per cycle per SIMD for independent v_fma_f32, v_pk_fma_f32, v_exp_f32 and a
// blend-like mix, at 1, 2, 4 and 8 waves per SIMD -- the peak the tile
// kernels' VALU fraction is priced against (bench.py VALU roofline).
//
//   hipcc -O3 --offload-arch=gfx950 tools/micro/valu_rate.hip -o /tmp/valu_rate && /tmp/valu_rate
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float v2f __attribute__((ext_vector_type(2)));

constexpr int kIters = 4096;

// 8 independent chains per lane, so a wave never waits on its own results
template <int kKind>
__global__ __launch_bounds__(256) void valu_kernel(float *out, float s) {
    float a[8];
    v2f p[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        a[k] = (float)(threadIdx.x + k) * 1e-3f;
        p[k] = (v2f){a[k], a[k] + 0.5f};
    }
    const v2f m = {s, s};
    unsigned long long mask = __builtin_amdgcn_read_exec() & 0x5555555555555555ull, cm;
    // one instruction per chain and step, written out (the compiler would
    // otherwise pack independent scalar FMAs into v_pk_fma_f32)
    // a defined VCC for kinds 3 and 10 (the kernel's own lane mask)
    if (kKind == 3 || kKind == 10) asm volatile("s_mov_b64 vcc, %0" : : "s"(mask) : "vcc");
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (kKind == 0) asm volatile("v_fma_f32 %0, %0, %1, 0.5" : "+v"(a[k]) : "v"(s));
            if (kKind == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(p[k]) : "v"(m));
            if (kKind == 2) asm volatile("v_exp_f32 %0, %0" : "+v"(a[k]));
            if (kKind == 3) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[k]) : "v"(s));
            // the same select with a mask the kernel wrote itself (VOP3, SGPR pair)
            if (kKind == 4) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[k]) : "v"(s), "s"(mask));
            // compare + select, as the blend loops use it
            if (kKind == 5)
                asm volatile("v_cmp_gt_f32_e64 %1, %0, %2\n\tv_cndmask_b32_e64 %0, %0, %2, %1"
                             : "+v"(a[k]), "=&s"(cm) : "v"(s));
            // VOP2 compare into VCC + VOP2 select on it, the compiler's usual pair
            if (kKind == 9)
                asm volatile("v_cmp_gt_f32_e32 vcc, %0, %1\n\tv_cndmask_b32_e32 %0, %0, %1, vcc"
                             : "+v"(a[k]) : "v"(s) : "vcc");
            // VOP3 select with VCC named as its mask
            if (kKind == 10) asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(a[k]) : "v"(s));
            if (kKind == 6) asm volatile("v_max_f32 %0, %0, %1" : "+v"(a[k]) : "v"(s));
            if (kKind == 7) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[k]) : "v"(s));
            if (kKind == 8) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[k]) : "v"(s));
        }
    }
    float r = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) r += a[k] + p[k].x + p[k].y;
    if (r == 12345.0f) out[threadIdx.x] = r;  // keep the work
}

template <int kKind>
static void run(const char *name, int waves_per_simd) {
    // 256 CUs x 4 SIMDs; 256-thread workgroups = 4 waves = one per SIMD
    const int blocks = 256 * waves_per_simd;
    float *out;
    (void)hipMalloc(&out, 1024);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    valu_kernel<kKind><<<blocks, 256>>>(out, 0.999f);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) valu_kernel<kKind><<<blocks, 256>>>(out, 0.999f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double insts = 5.0 * blocks * 4.0 * kIters * 8.0 * (kKind == 5 || kKind == 9 ? 2 : 1);
    const double per_s = insts / (ms * 1e-3);
    // per SIMD per cycle at 2.4 GHz (kinds 5 and 9 count both instructions)
    printf("{\"kind\": \"%s\", \"waves_per_simd\": %d, \"G_wave_inst_per_s\": %.1f, "
           "\"inst_per_simd_cycle_at_2.4GHz\": %.3f}\n",
           name, waves_per_simd, per_s / 1e9, per_s / (1024.0 * 2.4e9));
    (void)hipFree(out);
}

int main() {
    for (int w : {1, 8}) {
        run<0>("v_fma_f32", w);
        run<1>("v_pk_fma_f32", w);
        run<2>("v_exp_f32", w);
        run<3>("v_cndmask_b32", w);
        run<4>("v_cndmask_b32_e64_sgpr", w);
        run<5>("v_cmp_gt_f32+v_cndmask_b32 (2 inst)", w);
        run<9>("v_cmp_gt_f32_e32 vcc+v_cndmask_b32_e32 (2 inst)", w);
        run<10>("v_cndmask_b32_e64_vcc", w);
        run<6>("v_max_f32", w);
        run<7>("v_mul_f32", w);
        run<8>("v_add_u32", w);
    }
    return 0;
}
