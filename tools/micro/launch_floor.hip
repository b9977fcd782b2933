// Launch-floor microbenchmark: what a chain of dependent launches costs on one stream (the
// depth sort is 12 such launches).  Prints us per launch for empty / small / 600-block kernels,
// plain and captured in a hipGraph, and the cost of a "last block done" scan tail (device-scope
// release fence + ticket atomic per block).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            return 1;                                                             \
        }                                                                         \
    } while (0)

__global__ void k_empty(int *p) {
    if (p && threadIdx.x == 1023 && blockIdx.x == 1u << 30) p[0] = 1;
}

__global__ __launch_bounds__(256) void k_touch(const uint4 *in, uint4 *out, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = in[i];
}

// every block stores 256 words, then takes a ticket; the last block sums all stored words
__global__ __launch_bounds__(256) void k_lastblock(uint32_t *hist, uint32_t *ticket,
                                                   uint32_t *total) {
    __shared__ bool last;
    hist[blockIdx.x * 256 + threadIdx.x] = blockIdx.x + threadIdx.x;
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(ticket, 1u) == gridDim.x - 1;
    __syncthreads();
    if (!last) return;
    __threadfence();
    uint32_t s = 0;
    for (unsigned b = 0; b < gridDim.x; ++b) s += hist[b * 256 + threadIdx.x];
    total[threadIdx.x] = s;
    if (threadIdx.x == 0) *ticket = 0;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int n = 600 * 256;
    uint4 *x, *y;
    uint32_t *hist, *ticket, *total;
    CK(hipMalloc(&x, n * 16));
    CK(hipMalloc(&y, n * 16));
    CK(hipMalloc(&hist, 1024 * 256 * 4));
    CK(hipMalloc(&ticket, 4));
    CK(hipMalloc(&total, 1024));
    CK(hipMemset(ticket, 0, 4));
    const int N = 200;
    auto chain = [&](int kind) {
        for (int i = 0; i < N; ++i) {
            if (kind == 0) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, nullptr);
            if (kind == 1) hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s, nullptr);
            if (kind == 2) hipLaunchKernelGGL(k_touch, dim3(600), dim3(256), 0, s, x, y, n);
            if (kind == 3) hipLaunchKernelGGL(k_lastblock, dim3(600), dim3(256), 0, s, hist, ticket, total);
            if (kind == 4) hipLaunchKernelGGL(k_lastblock, dim3(150), dim3(256), 0, s, hist, ticket, total);
        }
    };
    const char *names[] = {"empty 1x64", "empty 256x256", "copy 600x256 (2.4 MB)",
                           "last-block 600 blocks", "last-block 150 blocks"};
    for (int kind = 0; kind < 5; ++kind) {
        chain(kind);
        CK(hipStreamSynchronize(s));
        float best = 1e9f;
        for (int rep = 0; rep < 5; ++rep) {
            CK(hipEventRecord(a, s));
            chain(kind);
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            best = std::min(best, ms);
        }
        // graph
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        chain(kind);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        float bestg = 1e9f;
        for (int rep = 0; rep < 5; ++rep) {
            CK(hipEventRecord(a, s));
            CK(hipGraphLaunch(ge, s));
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            bestg = std::min(bestg, ms);
        }
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
        std::printf("%-26s stream %.2f us/launch   graph %.2f us/launch\n", names[kind],
                    1e3f * best / N, 1e3f * bestg / N);
    }
    return 0;
}
