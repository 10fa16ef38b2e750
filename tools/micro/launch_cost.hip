// Host cost of enqueueing three dependent kernels: three hipLaunchKernelGGL
// vs one hipGraphLaunch of the captured three (with and without a per-launch
// kernel-node parameter update), each followed by a stream sync, as the
// fused training step does per iteration.  Build + run:
//   hipcc --offload-arch=gfx950 -O2 tools/micro/launch_cost.hip -o /tmp/lc && /tmp/lc
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

struct Args { float *p; int n; float s; };

__global__ void k_small(Args a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < a.n) a.p[i] = a.p[i] * a.s + 1.0f;
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    float *p;
    const int n = 1 << 16;
    hipMalloc(&p, n * sizeof(float));
    hipMemset(p, 0, n * sizeof(float));
    Args a{p, n, 0.5f};
    const int iters = 2000;
    auto three = [&]() {
        for (int k = 0; k < 3; ++k) hipLaunchKernelGGL(k_small, dim3(n / 256), dim3(256), 0, s, a);
    };
    for (int i = 0; i < 100; ++i) { three(); hipStreamSynchronize(s); }
    double t0 = now_us(), tl = 0;
    for (int i = 0; i < iters; ++i) {
        const double a0 = now_us();
        three();
        tl += now_us() - a0;
        hipStreamSynchronize(s);
    }
    const double plain = (now_us() - t0) / iters;
    printf("{\"three_launches_us_per_iter\": %.2f, \"enqueue_us\": %.2f}\n", plain, tl / iters);

    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    three();
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int i = 0; i < 100; ++i) { hipGraphLaunch(ge, s); hipStreamSynchronize(s); }
    t0 = now_us(); tl = 0;
    for (int i = 0; i < iters; ++i) {
        const double a0 = now_us();
        hipGraphLaunch(ge, s);
        tl += now_us() - a0;
        hipStreamSynchronize(s);
    }
    printf("{\"graph_us_per_iter\": %.2f, \"enqueue_us\": %.2f}\n", (now_us() - t0) / iters, tl / iters);

    // per-launch update of the last node's arguments
    size_t nn = 0;
    hipGraphGetNodes(g, nullptr, &nn);
    hipGraphNode_t nodes[8];
    hipGraphGetNodes(g, nodes, &nn);
    hipKernelNodeParams kp;
    hipGraphKernelNodeGetParams(nodes[nn - 1], &kp);
    t0 = now_us(); tl = 0;
    for (int i = 0; i < iters; ++i) {
        const double a0 = now_us();
        a.s = 0.5f + 1e-6f * (float)(i & 7);
        void *args[] = {&a};
        kp.kernelParams = args;
        hipGraphExecKernelNodeSetParams(ge, nodes[nn - 1], &kp);
        hipGraphLaunch(ge, s);
        tl += now_us() - a0;
        hipStreamSynchronize(s);
    }
    printf("{\"graph_update_us_per_iter\": %.2f, \"enqueue_us\": %.2f}\n", (now_us() - t0) / iters, tl / iters);

    // one kernel + sync: the floor
    t0 = now_us();
    for (int i = 0; i < iters; ++i) {
        hipLaunchKernelGGL(k_small, dim3(n / 256), dim3(256), 0, s, a);
        hipStreamSynchronize(s);
    }
    printf("{\"one_launch_us_per_iter\": %.2f}\n", (now_us() - t0) / iters);
    return 0;
}
