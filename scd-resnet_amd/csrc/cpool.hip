// Directional corner pooling (models/backbones/cornerPooling/source/{top,bottom,left,right}Pool.cpp)
// on NHWC activations.  The reference issues ~H sequential ATen launches forward and ~5H
// backward per pool; here one launch per direction: each thread owns a (n, line, channel-chunk)
// and scans the line in registers (coalesced across channels).  Backward routes each dy to the
// running argmax of the same scan; ties keep the first-scanned position (strict '>' update,
// topPool.cpp:61-65), every position is written exactly once (no memset, deterministic).
#include <algorithm>

#include "scd_common.h"

namespace {

// dir: 0 top (scan h descending), 1 bottom (h ascending), 2 left (w descending), 3 right (w ascending)
template <typename T>
__global__ void cpool_fwd_kernel(int dir, const T* x, const T* addend, T* y, int N, int H, int W, int C) {
    constexpr int E = Vec16<T>::N;
    const int cpp = C / E;
    const bool vert = dir < 2;
    const int L = vert ? H : W;                // scan length
    const int O = vert ? W : H;                // other spatial dim
    const long lines = (long)N * O * cpp;
    const long step = vert ? (long)W * C : (long)C;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < lines; i += (long)gridDim.x * blockDim.x) {
        const int ch = (int)(i % cpp);
        const long r = i / cpp;
        const int o = (int)(r % O);
        const int n = (int)(r / O);
        const long base = vert ? (((long)n * H) * W + o) * C + ch * E : (((long)n * H + o) * W) * C + ch * E;
        const bool desc = (dir == 0 || dir == 2);
        float m[E];
        for (int k = 0; k < L; ++k) {
            const int pos = desc ? (L - 1 - k) : k;
            float v[E];
            Vec16<T>::load(x + base + pos * step, v);
#pragma unroll
            for (int e = 0; e < E; ++e) m[e] = (k == 0) ? v[e] : fmaxf(m[e], v[e]);
            if (addend) {
                float a[E], o[E];
                Vec16<T>::load(addend + base + pos * step, a);
#pragma unroll
                for (int e = 0; e < E; ++e) o[e] = m[e] + a[e];
                Vec16<T>::store(y + base + pos * step, o);
            } else {
                Vec16<T>::store(y + base + pos * step, m);
            }
        }
    }
}

template <typename T>
__global__ void cpool_bwd_kernel(int dir, const T* x, const T* dy, T* dx, int N, int H, int W, int C) {
    constexpr int E = Vec16<T>::N;
    const int cpp = C / E;
    const bool vert = dir < 2;
    const int L = vert ? H : W;
    const int O = vert ? W : H;
    const long lines = (long)N * O * cpp;
    const long step = vert ? (long)W * C : (long)C;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < lines; i += (long)gridDim.x * blockDim.x) {
        const int ch = (int)(i % cpp);
        const long r = i / cpp;
        const int o = (int)(r % O);
        const int n = (int)(r / O);
        const long base = vert ? (((long)n * H) * W + o) * C + ch * E : (((long)n * H + o) * W) * C + ch * E;
        const bool desc = (dir == 0 || dir == 2);
        float mv[E], acc[E];
        int mi[E];
        for (int k = 0; k < L; ++k) {
            const int pos = desc ? (L - 1 - k) : k;
            float v[E], g[E];
            Vec16<T>::load(x + base + pos * step, v);
            Vec16<T>::load(dy + base + pos * step, g);
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const bool upd = (k == 0) || (v[e] > mv[e]);
                // a replaced argmax is final: flush its accumulated gradient
                if (upd && k > 0) dx[base + mi[e] * step + e] = from_f<T>(acc[e]);
                if (upd) { mv[e] = v[e]; mi[e] = pos; acc[e] = 0.f; }
                acc[e] += g[e];
                // a position that is not the running argmax now can never become one later
                if (!upd) dx[base + pos * step + e] = from_f<T>(0.f);
            }
        }
#pragma unroll
        for (int e = 0; e < E; ++e) dx[base + mi[e] * step + e] = from_f<T>(acc[e]);
    }
}

inline int ew_blocks(long n) { return (int)std::min<long>(4096, std::max<long>(1, (n + 255) / 256)); }

}  // namespace

extern "C" int scd_cpool_fwd(int dtype, int dir, const void* x, const void* addend, void* y, int N, int H, int W, int C,
                             void* stream) {
    if (dir < 0 || dir > 3) return SCD_ERR_ARG;
    const int E = dtype == SCD_DT_BF16 ? 8 : 4;
    if (C % E) return SCD_ERR_ARG;
    const long lines = (long)N * (dir < 2 ? W : H) * (C / E);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == SCD_DT_BF16)
        hipLaunchKernelGGL((cpool_fwd_kernel<__bf16>), dim3(ew_blocks(lines)), dim3(256), 0, st, dir, (const __bf16*)x,
                           (const __bf16*)addend, (__bf16*)y, N, H, W, C);
    else if (dtype == SCD_DT_F32)
        hipLaunchKernelGGL((cpool_fwd_kernel<float>), dim3(ew_blocks(lines)), dim3(256), 0, st, dir, (const float*)x,
                           (const float*)addend, (float*)y, N, H, W, C);
    else
        return SCD_ERR_ARG;
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_cpool_bwd(int dtype, int dir, const void* x, const void* dy, void* dx, int N, int H, int W, int C,
                             void* stream) {
    if (dir < 0 || dir > 3) return SCD_ERR_ARG;
    const int E = dtype == SCD_DT_BF16 ? 8 : 4;
    if (C % E) return SCD_ERR_ARG;
    const long lines = (long)N * (dir < 2 ? W : H) * (C / E);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == SCD_DT_BF16)
        hipLaunchKernelGGL((cpool_bwd_kernel<__bf16>), dim3(ew_blocks(lines)), dim3(256), 0, st, dir, (const __bf16*)x,
                           (const __bf16*)dy, (__bf16*)dx, N, H, W, C);
    else if (dtype == SCD_DT_F32)
        hipLaunchKernelGGL((cpool_bwd_kernel<float>), dim3(ew_blocks(lines)), dim3(256), 0, st, dir, (const float*)x,
                           (const float*)dy, (float*)dx, N, H, W, C);
    else
        return SCD_ERR_ARG;
    SCD_RETURN_LAUNCH();
}

extern "C" const char* scd_version(void) { return "libscdhip 0.1 gfx950"; }
