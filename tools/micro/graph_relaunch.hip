// Does hipGraphLaunch block the host while an earlier launch of the same executable graph is
// still running on the GPU?  A 3-kernel linear graph whose kernels each spin ~100 us: launch it
// 10 times back to back (one exec), then alternating between two execs of the same graph, then
// with direct launches, timing the host's submission loop.  Also: a graph holding a kernel with
// > 64 KiB of dynamic LDS (like k_color / k_tile_diff).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t err_ = (x);                                                      \
        if (err_ != hipSuccess) {                                                   \
            std::printf("HIP error %s at %d\n", hipGetErrorString(err_), __LINE__); \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

__global__ void k_spin(long long cycles, int *p) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {
    }
    if (p && threadIdx.x == 1023 && blockIdx.x == 1u << 30) p[0] = 1;
}

__global__ void k_lds(int *p) {
    extern __shared__ int s[];
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (p && s[threadIdx.x] == -1) p[0] = 1;
}

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) {
    return std::chrono::duration<double, std::micro>(b - a).count();
}

static long long g_cycles = 100000;  // ~100 us at 1 GHz shader clock counter (clock64)
static int g_lds = 0;

static void chain(hipStream_t s) {
    for (int i = 0; i < 3; ++i)
        hipLaunchKernelGGL(k_spin, dim3(64), dim3(64), 0, s, g_cycles, nullptr);
    if (g_lds) hipLaunchKernelGGL(k_lds, dim3(64), dim3(256), g_lds, s, nullptr);
}

static hipGraphExec_t record(hipStream_t cs) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
    chain(cs);
    CK(hipStreamEndCapture(cs, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphDestroy(g));
    return ge;
}

int main() {
    hipStream_t s, cs;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_lds),
                           hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024));
    // calibrate: one direct chain
    CK(hipDeviceSynchronize());
    auto t0 = clk::now();
    chain(s);
    CK(hipStreamSynchronize(s));
    std::printf("one chain on the GPU: %.1f us\n", us(t0, clk::now()));
    for (int lds = 0; lds <= 1; ++lds) {
        g_lds = lds ? 100 * 1024 : 0;
        hipGraphExec_t a = record(cs), b = record(cs);
        for (int mode = 0; mode < 3; ++mode) {
            CK(hipDeviceSynchronize());
            const int N = 10;
            t0 = clk::now();
            for (int i = 0; i < N; ++i) {
                if (mode == 0) CK(hipGraphLaunch(a, s));
                if (mode == 1) CK(hipGraphLaunch(i & 1 ? b : a, s));
                if (mode == 2) chain(s);
            }
            const auto t1 = clk::now();
            CK(hipStreamSynchronize(s));
            const auto t2 = clk::now();
            std::printf("%s%-26s host %.1f us per launch, total %.1f us per chain\n",
                        lds ? "[+100 KiB LDS kernel] " : "",
                        mode == 0 ? "one exec relaunched:" : mode == 1 ? "two execs alternating:"
                                                                       : "direct launches:",
                        us(t0, t1) / N, us(t0, t2) / N);
        }
        CK(hipGraphExecDestroy(a));
        CK(hipGraphExecDestroy(b));
    }
    return 0;
}
