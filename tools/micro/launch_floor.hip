// Launch-floor microbenchmark: back-to-back launches of trivial kernels on one
// stream (rocprofv3 --kernel-trace gives their durations; the host clock the
// per-launch wall time).  tools/micro/launch_floor.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_empty() {}
__global__ void k_one(unsigned *p) {
    if (blockIdx.x == 0 && threadIdx.x == 0) p[0] = 1;
}
__global__ void k_fill(unsigned *p, unsigned n) {
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = i;
}

int main() {
    unsigned *d = nullptr;
    if (hipMalloc(&d, 64 << 20) != hipSuccess) return 1;
    hipStream_t s;
    (void)hipStreamCreate(&s);
    auto run = [&](const char *name, auto launch) {
        for (int i = 0; i < 50; i++) launch();
        (void)hipStreamSynchronize(s);
        const auto t0 = std::chrono::steady_clock::now();
        const int N = 2000;
        for (int i = 0; i < N; i++) launch();
        (void)hipStreamSynchronize(s);
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / N;
        std::printf("%-28s %.2f us per launch\n", name, us);
    };
    run("empty 1x64", [&] { k_empty<<<1, 64, 0, s>>>(); });
    run("empty 256x256", [&] { k_empty<<<256, 256, 0, s>>>(); });
    run("empty 2048x256", [&] { k_empty<<<2048, 256, 0, s>>>(); });
    run("empty 256x1024", [&] { k_empty<<<256, 1024, 0, s>>>(); });
    run("one-word 256x256", [&] { k_one<<<256, 256, 0, s>>>(d); });
    run("fill 64K words 256x256", [&] { k_fill<<<256, 256, 0, s>>>(d, 1u << 16); });
    run("fill 1M words 1024x256", [&] { k_fill<<<1024, 256, 0, s>>>(d, 1u << 20); });
    run("fill 4M words 2048x256", [&] { k_fill<<<2048, 256, 0, s>>>(d, 1u << 22); });
    (void)hipFree(d);
    return 0;
}
