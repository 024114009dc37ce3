// Do two HIP streams share a hardware queue?  (ordered lanes at
// N > 1.)  A kernel on stream A spins -- bounded: it gives up after ~50 ms --
// until a kernel launched AFTER it on stream B sets a flag.  If A and B feed
// one AQL queue, B's kernel sits behind A's and A times out; on queues of
// their own, B runs beside A and A sees the flag.  Run for plain streams and
// for CU-masked streams (hipExtStreamCreateWithCUMask, the decision lanes'),
// more streams than GPU_MAX_HW_QUEUES.   tools/micro/queue_share.hip
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void k_wait(unsigned *flag, unsigned *seen) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = wall_clock64();
    unsigned v = 0;
    while ((v = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0u &&
           wall_clock64() - t0 < 5000000ull)  // 50 ms at the 100 MHz constant clock
        __builtin_amdgcn_s_sleep(4);
    *seen = v;
}
__global__ void k_set(unsigned *flag) {
    if (threadIdx.x == 0) __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

static int pairs(const char *what, std::vector<hipStream_t> &st, unsigned *d) {
    int shared = 0;
    for (size_t k = 1; k < st.size(); k++) {
        (void)hipMemset(d, 0, 8);
        (void)hipDeviceSynchronize();
        k_wait<<<1, 64, 0, st[0]>>>(d, d + 1);
        k_set<<<1, 64, 0, st[k]>>>(d);
        (void)hipDeviceSynchronize();
        unsigned seen = 0;
        (void)hipMemcpy(&seen, d + 1, 4, hipMemcpyDeviceToHost);
        std::printf("%s: stream 0 and stream %zu: %s\n", what, k, seen ? "own queues" : "SHARED queue");
        shared += seen ? 0 : 1;
    }
    return shared;
}

int main() {
    const char *q = std::getenv("GPU_MAX_HW_QUEUES");
    std::printf("GPU_MAX_HW_QUEUES=%s\n", q ? q : "(unset)");
    unsigned *d = nullptr;
    if (hipMalloc(&d, 64) != hipSuccess) return 1;
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int N = 8;
    std::vector<hipStream_t> plain(N), masked(N), mixed;
    for (int i = 0; i < N; i++) (void)hipStreamCreateWithFlags(&plain[i], hipStreamNonBlocking);
    int sp = pairs("plain", plain, d);
    for (int l = 0; l < N; l++) {
        std::vector<uint32_t> mask((cus + 31) / 32, 0u);
        for (int i = 0; i < cus; i++)
            if (i % 4 == l % 4) mask[i / 32] |= 1u << (i % 32);  // lane l of 4 (two lanes per share)
        (void)hipExtStreamCreateWithCUMask(&masked[l], (uint32_t)mask.size(), mask.data());
    }
    int sm = pairs("cu-masked", masked, d);
    // masked lanes beside the plain streams already holding the queues
    mixed.push_back(masked[0]);
    for (int i = 0; i < N; i++) mixed.push_back(plain[i]);
    int sx = pairs("masked[0] vs plain", mixed, d);
    std::printf("shared pairs: plain %d, cu-masked %d, masked-vs-plain %d\n", sp, sm, sx);
    (void)hipFree(d);
    return 0;
}
