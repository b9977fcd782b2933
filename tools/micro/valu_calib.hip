// SQ counter calibration: a kernel whose VALU instruction count is known exactly.  Each of
// `blocks` 64-thread blocks (one wave, like the blend's quadrant waves) runs `iters` x 16
// v_fma_f32 (inline asm, so none is folded) plus a fixed prologue / epilogue.  Run under
// rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE to
// read how the counters scale (tools/micro/valu_calib.sh).
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ __launch_bounds__(64) void k_valu(float *out, int iters) {
    float a = threadIdx.x * 1e-3f, b = 1.0001f, c = 0.5f;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 16; ++u) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a) : "v"(b), "v"(c));
    }
    if (a == 12345.f) out[blockIdx.x * 64 + threadIdx.x] = a;
}

int main() {
    float *out;
    hipMalloc(&out, 64 * 32640 * 4);
    const int blocks = 32640, iters = 200;
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(64), 0, 0, out, iters);
    hipDeviceSynchronize();
    std::printf("launched 3 x %d waves x %d v_fma_f32 (+ loop overhead) = %.1f M fma wave-instr per launch\n",
                blocks, iters * 16, blocks * (double)iters * 16 / 1e6);
    return 0;
}
