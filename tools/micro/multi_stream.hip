// Dispatch throughput across CU-masked streams (as the decision lanes use
// them): N back-to-back launches spread round-robin over S streams, each
// stream masked to CUs i with i mod S = l -- the wall time per launch for
// empty kernels and for kernels of a few microseconds, 1 / 2 / 4 streams.
// Does one queue's dispatch, or the command processor, bound the lanes?
// tools/micro/multi_stream.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void k_empty() {}
__global__ void k_spin(unsigned *p, unsigned iters) {  // ~iters x 1 us-ish of per-block work
    unsigned v = threadIdx.x;
    for (unsigned i = 0; i < iters; i++) v = v * 1664525u + 1013904223u;
    if (v == 0x12345678u) p[0] = v;
}
__global__ void k_touch(unsigned *p, unsigned n) {
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] += 1;
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned *d = nullptr;
    if (hipMalloc(&d, 64 << 20) != hipSuccess) return 1;
    for (int S : {1, 2, 4}) {
        std::vector<hipStream_t> st(S);
        for (int l = 0; l < S; l++) {
            std::vector<uint32_t> mask((cus + 31) / 32, 0u);
            for (int i = 0; i < cus; i++)
                if (S == 1 || i % S == l) mask[i / 32] |= 1u << (i % 32);
            if (hipExtStreamCreateWithCUMask(&st[l], (uint32_t)mask.size(), mask.data()) != hipSuccess) return 2;
        }
        auto run = [&](const char *name, auto launch) {
            for (int i = 0; i < 100; i++) launch(st[i % S]);
            (void)hipDeviceSynchronize();
            const int N = 1000;
            const auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < N; i++) launch(st[i % S]);
            (void)hipDeviceSynchronize();
            const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / N;
            std::printf("streams %d  %-34s %.2f us per launch\n", S, name, us);
            std::fflush(stdout);
        };
        run("empty 256x256", [&](hipStream_t s) { hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s); });
        run("empty 64x1024", [&](hipStream_t s) { hipLaunchKernelGGL(k_empty, dim3(64), dim3(1024), 0, s); });
        run("spin 256x256 (2000 it)", [&](hipStream_t s) { hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, s, d, 2000u); });
        run("touch 1M words 256x256", [&](hipStream_t s) { hipLaunchKernelGGL(k_touch, dim3(256), dim3(256), 0, s, d, 1u << 20); });
        for (auto s : st) (void)hipStreamDestroy(s);
    }
    (void)hipFree(d);
    return 0;
}
