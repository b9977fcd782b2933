// Host-side cost of the calls a frame makes (what bounds small frames: the C ABI's forward
// spends ~100 us of host time per frame).  Prints us of host time per call for
// hipLaunchKernel (small args / a 400-B argument struct), hipEventRecord, hipStreamWaitEvent
// across two streams, and hipGraphLaunch of a captured 20-kernel chain (per graph).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t err_ = (x);                                                       \
        if (err_ != hipSuccess) {                                                 \
            std::printf("HIP error %s at %d\n", hipGetErrorString(err_), __LINE__); \
            return 1;                                                             \
        }                                                                         \
    } while (0)

struct Big {
    float v[100];
};

__global__ void k_empty(int *p) {
    if (p && threadIdx.x == 1023 && blockIdx.x == 1u << 30) p[0] = 1;
}
__global__ void k_big(Big b, int *p) {
    if (p && threadIdx.x == 1023 && blockIdx.x == 1u << 30) p[0] = (int)b.v[3];
}

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) {
    return std::chrono::duration<double, std::micro>(b - a).count();
}

int main() {
    hipStream_t s, s2;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t e, et, e2, e3;
    CK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventReleaseToDevice));
    CK(hipEventCreate(&et));
    CK(hipEventCreateWithFlags(&e2, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&e3, hipEventDisableTiming | hipEventDisableSystemFence));
    Big big{};
    const int N = 20, R = 200;
    auto chain = [&](int kind) {
        for (int i = 0; i < N; ++i) {
            if (kind == 0) hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s, nullptr);
            if (kind == 1) hipLaunchKernelGGL(k_big, dim3(256), dim3(256), 0, s, big, nullptr);
            if (kind == 2) hipEventRecord(e, s);
            if (kind == 3) hipEventRecord(et, s);
            if (kind == 4) {
                hipEventRecord(e, s);
                hipStreamWaitEvent(s2, e, 0);
            }
            if (kind == 5) hipEventRecord(e2, s);
            if (kind == 6) hipEventRecord(e3, s);
            if (kind == 7) {
                hipEventRecord(e3, s);
                hipStreamWaitEvent(s2, e3, 0);
            }
            if (kind == 8) {
                hipEventRecord(et, s);
                hipStreamWaitEvent(s2, et, 0);
            }
        }
    };
    const char *names[] = {"hipLaunchKernel (8-B args)", "hipLaunchKernel (400-B args)",
                           "hipEventRecord (no timing)", "hipEventRecord (timing)",
                           "record + hipStreamWaitEvent", "hipEventRecord (DisableTiming)",
                           "hipEventRecord (no timing/sysfence)", "record+wait (no timing/sysfence)",
                           "record+wait (timing event)"};
    for (int kind = 0; kind < 9; ++kind) {
        double best = 1e30;
        for (int r = 0; r < R; ++r) {
            CK(hipStreamSynchronize(s));
            CK(hipStreamSynchronize(s2));
            const auto t0 = clk::now();
            chain(kind);
            const auto t1 = clk::now();
            best = std::min(best, us(t0, t1));
        }
        double med = 0;
        {  // mean over back-to-back frames without syncing in between (queue keeps filling)
            CK(hipStreamSynchronize(s));
            const auto t0 = clk::now();
            for (int r = 0; r < 50; ++r) chain(kind);
            const auto t1 = clk::now();
            med = us(t0, t1) / 50;
        }
        std::printf("%-30s best %.2f us/call, back-to-back %.2f us/call\n", names[kind],
                    best / N, med / N);
    }
    for (int kind = 0; kind < 2; ++kind) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        chain(kind);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        double best = 1e30;
        for (int r = 0; r < R; ++r) {
            CK(hipStreamSynchronize(s));
            const auto t0 = clk::now();
            CK(hipGraphLaunch(ge, s));
            const auto t1 = clk::now();
            best = std::min(best, us(t0, t1));
        }
        CK(hipStreamSynchronize(s));
        const auto t0 = clk::now();
        for (int r = 0; r < 50; ++r) CK(hipGraphLaunch(ge, s));
        const auto t1 = clk::now();
        CK(hipStreamSynchronize(s));
        const auto t2 = clk::now();
        std::printf("hipGraphLaunch of %d %s kernels: best %.2f us, back-to-back %.2f us host, "
                    "%.2f us GPU per graph\n",
                    N, kind ? "400-B-arg" : "8-B-arg", best, us(t0, t1) / 50, us(t0, t2) / 50);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    // fork / join topology: 15 kernels on s, 5 on s2 between a fork and a join
    for (int variant = 0; variant < 2; ++variant) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k_big, dim3(256), dim3(256), 0, s, big, nullptr);
        if (variant == 1) {
            CK(hipEventRecord(e, s));
            CK(hipStreamWaitEvent(s2, e, 0));
            for (int i = 0; i < 5; ++i)
                hipLaunchKernelGGL(k_big, dim3(256), dim3(256), 0, s2, big, nullptr);
            CK(hipEventRecord(e2, s2));
        } else {
            for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k_big, dim3(256), dim3(256), 0, s, big, nullptr);
        }
        for (int i = 0; i < 12; ++i) hipLaunchKernelGGL(k_big, dim3(256), dim3(256), 0, s, big, nullptr);
        if (variant == 1) CK(hipStreamWaitEvent(s, e2, 0));
        CK(hipStreamEndCapture(s, &g));
        size_t nn = 0;
        CK(hipGraphGetNodes(g, nullptr, &nn));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        double best = 1e30, sum = 0;
        for (int r = 0; r < R; ++r) {
            CK(hipStreamSynchronize(s));
            const auto t0 = clk::now();
            CK(hipGraphLaunch(ge, s));
            const auto t1 = clk::now();
            best = std::min(best, us(t0, t1));
            sum += us(t0, t1);
        }
        CK(hipStreamSynchronize(s));
        const auto t0 = clk::now();
        for (int r = 0; r < 50; ++r) CK(hipGraphLaunch(ge, s));
        const auto t1 = clk::now();
        CK(hipStreamSynchronize(s));
        const auto t2 = clk::now();
        std::printf("%s graph (%zu nodes): launch best %.2f us, mean %.2f us, back-to-back %.2f us "
                    "host, %.2f us GPU per graph\n",
                    variant ? "fork/join" : "linear", nn, best, sum / R, us(t0, t1) / 50,
                    us(t0, t2) / 50);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    return 0;
}
