// Host cost of queueing a kernel launch on gfx950 (ROCm 7.2): empty kernels
// with small and with ~1.2 KB arguments, plain and hipExtLaunchKernelGGL, and
// a captured graph of the same 17 launches replayed -- what an epoch's ~17-25
// launches cost the host (tools/micro/launch_cost.hip; bench DVCC_HOST_PROF).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>

struct Big { unsigned long long w[150]; };  // ~1.2 KB, as the probe / kill's table descriptors
__global__ void k_small(int *p, int v) { if (p && threadIdx.x == 0 && blockIdx.x == 0 && v < 0) p[0] = v; }
__global__ void k_big(int *p, Big b) { if (p && threadIdx.x == 0 && blockIdx.x == 0 && b.w[3] == 7) p[0] = 1; }

int main() {
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    Big b{};
    auto us = [](auto t0) { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count(); };
    const int N = 2000;
    for (int rep = 0; rep < 2; rep++) {
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < N; i++) hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, s, nullptr, i);
        const double a = us(t0) / N;
        (void)hipStreamSynchronize(s);
        t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < N; i++) hipExtLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, s, nullptr, nullptr, 0, nullptr, i);
        const double a2 = us(t0) / N;
        (void)hipStreamSynchronize(s);
        t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < N; i++) hipLaunchKernelGGL(k_big, dim3(256), dim3(256), 0, s, nullptr, b);
        const double c = us(t0) / N;
        (void)hipStreamSynchronize(s);
        // a graph of 17 launches, replayed
        hipGraph_t g;
        hipGraphExec_t ge;
        (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
        for (int i = 0; i < 17; i++) hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, s, nullptr, i);
        (void)hipStreamEndCapture(s, &g);
        (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < N / 17; i++) (void)hipGraphLaunch(ge, s);
        const double d = us(t0) / (N / 17);
        (void)hipStreamSynchronize(s);
        std::printf("host us per launch: small %.2f, ext %.2f, 1.2 KB args %.2f; 17-launch graph replay %.2f us\n", a, a2,
                    c, d);
        (void)hipGraphExecDestroy(ge);
        (void)hipGraphDestroy(g);
    }
    return 0;
}
