// Host cost of one frame's submission in three shapes (what bounds small frames):
//   direct   -- today's forward: 1 launch, fork event, 11 launches on the frame stream and 4 on
//               the second stream, join, 1 launch (17 launches, 2 records, 2 waits);
//   graphs   -- the same work with the two chains recorded as two LINEAR graphs (one per
//               stream; ROCm launches a linear graph as one pre-built packet batch), the fork /
//               join and the first / last kernel still direct;
//   threads  -- two host threads each submitting the direct frame on their own stream pair
//               (does HIP's launch path scale across threads?).
// Prints host us per frame (back-to-back frames) and GPU us per frame.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <thread>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t err_ = (x);                                                      \
        if (err_ != hipSuccess) {                                                   \
            std::printf("HIP error %s at %d\n", hipGetErrorString(err_), __LINE__); \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

struct Big {
    float v[64];
};

__global__ void k_big(Big b, int *p) {
    if (p && threadIdx.x == 1023 && blockIdx.x == 1u << 30) p[0] = (int)b.v[3];
}

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) {
    return std::chrono::duration<double, std::micro>(b - a).count();
}

struct Slot {
    hipStream_t s, a;
    hipEvent_t fork, join;
    hipGraphExec_t gm = nullptr, ga = nullptr;
};

static const Big kBig{};
static void launch(hipStream_t s) { hipLaunchKernelGGL(k_big, dim3(512), dim3(256), 0, s, kBig, nullptr); }
static void main_chain(hipStream_t s) { for (int i = 0; i < 11; ++i) launch(s); }
static void aux_chain(hipStream_t s) { for (int i = 0; i < 4; ++i) launch(s); }

static void frame_direct(Slot &q) {
    launch(q.s);
    hipEventRecord(q.fork, q.s);
    main_chain(q.s);
    hipStreamWaitEvent(q.a, q.fork, 0);
    aux_chain(q.a);
    hipEventRecord(q.join, q.a);
    hipStreamWaitEvent(q.s, q.join, 0);
    launch(q.s);
}

static void frame_graphs(Slot &q) {
    launch(q.s);
    hipEventRecord(q.fork, q.s);
    hipGraphLaunch(q.gm, q.s);
    hipStreamWaitEvent(q.a, q.fork, 0);
    hipGraphLaunch(q.ga, q.a);
    hipEventRecord(q.join, q.a);
    hipStreamWaitEvent(q.s, q.join, 0);
    launch(q.s);
}

static hipGraphExec_t record(hipStream_t s, void (*chain)(hipStream_t)) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    chain(s);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphDestroy(g));
    return ge;
}

static void make_slot(Slot &q) {
    CK(hipStreamCreateWithFlags(&q.s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&q.a, hipStreamNonBlocking));
    CK(hipEventCreateWithFlags(&q.fork, hipEventDisableTiming | hipEventReleaseToDevice));
    CK(hipEventCreateWithFlags(&q.join, hipEventDisableTiming | hipEventReleaseToDevice));
    q.gm = record(q.s, main_chain);
    q.ga = record(q.a, aux_chain);
}

int main() {
    Slot q[2];
    make_slot(q[0]);
    make_slot(q[1]);
    const int F = 400;
    for (int shape = 0; shape < 2; ++shape) {
        for (int depth = 1; depth <= 2; ++depth) {
            for (int rep = 0; rep < 2; ++rep) {
                CK(hipDeviceSynchronize());
                const auto t0 = clk::now();
                for (int f = 0; f < F; ++f) {
                    Slot &s = q[f % depth];
                    if (shape == 0) frame_direct(s);
                    else frame_graphs(s);
                }
                const auto t1 = clk::now();
                CK(hipDeviceSynchronize());
                const auto t2 = clk::now();
                if (rep == 1)
                    std::printf("%-7s depth %d: host %.2f us/frame, host+GPU %.2f us/frame\n",
                                shape ? "graphs" : "direct", depth, us(t0, t1) / F, us(t0, t2) / F);
            }
        }
    }
    // two host threads, one slot each, direct frames
    for (int shape = 0; shape < 2; ++shape) {
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipDeviceSynchronize());
            const auto t0 = clk::now();
            auto work = [&](int t) {
                for (int f = 0; f < F / 2; ++f) {
                    if (shape == 0) frame_direct(q[t]);
                    else frame_graphs(q[t]);
                }
            };
            std::thread th(work, 1);
            work(0);
            th.join();
            const auto t1 = clk::now();
            CK(hipDeviceSynchronize());
            const auto t2 = clk::now();
            if (rep == 1)
                std::printf("2 threads %-7s: host %.2f us/frame, host+GPU %.2f us/frame\n",
                            shape ? "graphs" : "direct", us(t0, t1) / F, us(t0, t2) / F);
        }
    }
    return 0;
}
