// Calibration kernels: the bf16 MFMA rate and the shader clock this box sustains (SURVEY.md §8(d) C2 "measure the
// achievable peak on the box"; MI355X_MICROARCH.md "DVFS give-back" items 1, 6, 7).  Diagnostics only: no training
// path calls them.
//
// scd_calib_mfma_peak: every wave keeps 4 A and 4 B fragments of random bf16 in registers and issues, per iteration,
// 16 v_mfma_f32_16x16x32_bf16 on 16 independent accumulators, each with a different (A, B) pair (the operand inputs
// toggle as in a GEMM main loop, so the chip's power/clock response is that of real data, not of zeros).  One wave per
// SIMD per 256-thread workgroup; grid = CUs x k gives k waves per SIMD.  Lane 0 of each wave stamps s_memtime (shader
// clock) and s_memrealtime (100 MHz) around the loop, so clock = d(memtime) / d(realtime) x 100 MHz per wave.
//
// scd_calib_set_stamps: the buffer the GEMM kernels of a stamped diagnostic build (make variant VFLAGS=-DSCD_STAMP=1)
// write their per-workgroup main-loop stamps to: [workgroup][4] = {memtime at loop start, at loop end, realtime at
// loop start, at loop end}.  The product build never writes it.
#include "scd_common.h"

namespace {

__global__ __launch_bounds__(256) void mfma_peak_kernel(const bf16x8* src, int iters, float* out,
                                                        unsigned long long* stamps) {
    const int lane = threadIdx.x & 63;
    const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int slot = gw & 255;
    bf16x8 a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        a[i] = src[(slot * 8 + i) * 64 + lane];
        b[i] = src[(slot * 8 + 4 + i) * 64 + lane];
    }
    f32x4 acc[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[k] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 16; ++k) acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[k & 3], b[k >> 2], acc[k], 0, 0, 0);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
    out[gw * 64 + lane] = s;
    if (lane == 0 && stamps) {
        stamps[gw * 4 + 0] = t0;
        stamps[gw * 4 + 1] = t1;
        stamps[gw * 4 + 2] = r0;
        stamps[gw * 4 + 3] = r1;
    }
}

}  // namespace

unsigned long long* scd_calib_stamp_buffer = nullptr;   // read by conv_gemm.hip's fill_params

extern "C" int scd_calib_mfma_peak(const void* src, int grid, int iters, float* out, unsigned long long* stamps,
                                   void* stream) {
    if (!src || !out || grid <= 0 || iters <= 0) return SCD_ERR_ARG;
    hipLaunchKernelGGL(mfma_peak_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const bf16x8*)src, iters, out,
                       stamps);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_calib_set_stamps(unsigned long long* stamps) {
    scd_calib_stamp_buffer = stamps;
    return 0;
}

extern "C" int scd_calib_stamped_build(void) {
#if defined(SCD_STAMP) && SCD_STAMP
    return 1;
#else
    return 0;
#endif
}
