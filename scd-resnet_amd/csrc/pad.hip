// Channel padding for narrow convolutions (the `*h` / `*q` plugins: 16- and 32-channel layers, e.g.
// trainer/model/centerOffsetRes10q.py dims [16, 16, 32, 64, ...]).  The gather-GEMM's K-stage spans BK channels
// of one tap (64 bf16 / 32 fp32), so a layer whose input width is not a multiple of BK runs on a copy of its
// input -- and of its packed weight operand -- zero-extended per pixel / per tap to the next multiple of BK.
// dst[r][c] = c < C ? src[r][c] : 0 for r < rows, c < Cp; 16-byte vectors (C and Cp multiples of the vector).
#include "scd_common.h"

namespace {
SCD_KERNEL_NS_BEGIN

__global__ __launch_bounds__(256) void pad_channels_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                           long rows, int cv, int cpv) {
    const long n = rows * cpv;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        long r = i / cpv;
        int c = (int)(i - r * cpv);
        dst[i] = c < cv ? src[r * cv + c] : make_uint4(0u, 0u, 0u, 0u);
    }
}

SCD_KERNEL_NS_END
}  // namespace

extern "C" int scd_pad_channels(int dtype, const void* src, long rows, int C, int Cp, void* dst, void* stream) {
    SCD_F16_FWD(scd_pad_channels, src, rows, C, Cp, dst, stream);
    const int esz = dtype == SCD_DT_BF16 ? 2 : 4;
    const int vec = 16 / esz;
    if (rows < 1 || C < 1 || Cp < C || C % vec || Cp % vec || src == dst) return SCD_ERR_ARG;
    const long n = rows * (Cp / vec);
    const long blocks = (n + 255) / 256;
    hipLaunchKernelGGL(pad_channels_kernel, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256), 0,
                       (hipStream_t)stream, (const uint4*)src, (uint4*)dst, rows, C / vec, Cp / vec);
    SCD_RETURN_LAUNCH();
}
