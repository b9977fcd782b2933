// Depth-sort probe: times each kernel of gsr_depth_sort on 1M synthetic depth keys (60% kept,
// depths in [2, 6) like C3) with events around every launch.  Built three ways by
// tools/micro/build_probe.sh (full / no output stores / no second sub-pass).
#include "../../gaussiansplattingviewer_amd/csrc/depth_sort.hip"

#include <cstdio>
#include <vector>

int main() {
    const int64_t n = 1000000;
    std::vector<uint32_t> h(n);
    uint64_t x = 88172645463325252ull;
    for (int64_t i = 0; i < n; ++i) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        const float d = 2.0f + 4.0f * (float)((x >> 11) & 0xFFFFFF) / 16777216.0f;
        h[i] = ((x >> 40) % 10) < 6 ? __builtin_bit_cast(uint32_t, d) : 0xFFFFFFFFu;
    }
    uint32_t *keys, *perm, *hist, *dt, *ctl;
    uint2 *pa, *pb;
    hipMalloc(&keys, n * 4); hipMalloc(&pa, n * 8); hipMalloc(&pb, n * 8); hipMalloc(&perm, n * 4);
    hipMalloc(&hist, gsr_depth_sort_hist_words(n) * 4);
    hipMalloc(&dt, 4096 * 4);
    hipMalloc(&ctl, gsr_depth_sort_ctl_words(n) * 4);
    hipMemcpy(keys, h.data(), n * 4, hipMemcpyHostToDevice);
    hipStream_t s;
    hipStreamCreate(&s);
    // warm up (sets the LDS attribute)
    for (int i = 0; i < 5; ++i) gsr_depth_sort(keys, n, 1, pa, pb, perm, hist, dt, ctl, 0, 2, s);
    hipStreamSynchronize(s);
    // whole sort
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const int R = 50;
    hipEventRecord(a, s);
    for (int i = 0; i < R; ++i) gsr_depth_sort(keys, n, 1, pa, pb, perm, hist, dt, ctl, 0, 2, s);
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    uint32_t c[2];
    hipMemcpy(c, ctl, 8, hipMemcpyDeviceToHost);
    std::printf("depth sort: %.2f us/sort (kept %u, D %u)\n", 1e3f * ms / R, c[0], c[1]);
    // per kernel: replay the launches one at a time with events between them
    const unsigned nt = (unsigned)((n + kDT - 1) / kDT);
    hipEvent_t ev[10];
    for (auto &e : ev) hipEventCreate(&e);
    double acc[9] = {};
    for (int r = 0; r < R; ++r) {
        const void *in[3] = {keys, pa, pb};
        uint2 *out[3] = {pa, pb, nullptr};
        int q = 0;
        hipEventRecord(ev[q++], s);
        for (int p = 0; p < 3; ++p) {  // pass 2 exits at once (D = 24)
            const int shift = p * 12;
            if (p == 0) {
                hipLaunchKernelGGL(k_ds_upsweep<true>, dim3(nt), dim3(kDThreads), 0, s, in[p], n, 1, ctl, shift, hist, nullptr);
                hipEventRecord(ev[q++], s);
                hipLaunchKernelGGL(k_ds_scan<true>, dim3(kDBins / kScanDigits), dim3(256), 0, s, hist, n, ctl, shift, dt, nullptr, nullptr, 0u);
                hipEventRecord(ev[q++], s);
                hipLaunchKernelGGL(k_ds_downsweep<true>, dim3(nt), dim3(kDThreads), 0, s, in[p], out[p], perm, n, 1, ctl, shift, hist, dt, nullptr, nullptr);
            } else {
                hipLaunchKernelGGL(k_ds_upsweep<false>, dim3(nt), dim3(kDThreads), 0, s, in[p], n, 0, ctl, shift, hist, nullptr);
                hipEventRecord(ev[q++], s);
                hipLaunchKernelGGL(k_ds_scan<false>, dim3(kDBins / kScanDigits), dim3(256), 0, s, hist, n, ctl, shift, dt, nullptr, nullptr, 0u);
                hipEventRecord(ev[q++], s);
                hipLaunchKernelGGL(k_ds_downsweep<false>, dim3(nt), dim3(kDThreads), 0, s, in[p], out[p], perm, n, 0, ctl, shift, hist, dt, nullptr, nullptr);
            }
            hipEventRecord(ev[q++], s);
        }
        hipEventSynchronize(ev[9]);
        for (int i = 0; i < 9; ++i) {
            hipEventElapsedTime(&ms, ev[i], ev[i + 1]);
            acc[i] += ms;
        }
    }
    const char *nm[3] = {"up", "scan", "down"};
    for (int i = 0; i < 9; ++i) std::printf("  pass %d %-5s %7.2f us\n", i / 3, nm[i % 3], 1e3 * acc[i] / R);
    return 0;
}
