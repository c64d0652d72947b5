// Shared device helpers for libscdhip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/scdhip.h"

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

#define SCD_RETURN_LAUNCH() return (int)hipGetLastError()

template <typename T> __device__ __forceinline__ float to_f(T v);
template <> __device__ __forceinline__ float to_f<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f<__bf16>(__bf16 v) { return (float)v; }

template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ __bf16 from_f<__bf16>(float v) { return (__bf16)v; }

// 16-byte vector of T <-> floats
template <typename T> struct Vec16;
template <> struct Vec16<float> {
    static constexpr int N = 4;
    __device__ static void load(const void* p, float* f) {
        float4 v = *(const float4*)p;
        f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
    }
    __device__ static void store(void* p, const float* f) {
        *(float4*)p = make_float4(f[0], f[1], f[2], f[3]);
    }
};
template <> struct Vec16<__bf16> {
    static constexpr int N = 8;
    __device__ static void load(const void* p, float* f) {
        bf16x8 v = *(const bf16x8*)p;
#pragma unroll
        for (int i = 0; i < 8; ++i) f[i] = (float)v[i];
    }
    __device__ static void store(void* p, const float* f) {
        bf16x8 v;
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = (__bf16)f[i];
        *(bf16x8*)p = v;
    }
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// fp64 atomic add (global_atomic_add_f64 on gfx950)
__device__ __forceinline__ void atomic_add_f64(double* p, double v) { unsafeAtomicAdd(p, v); }
__device__ __forceinline__ void atomic_add_f32(float* p, float v) { unsafeAtomicAdd(p, v); }

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// Workgroups of `kernel` (blockDim `threads`, no dynamic LDS) resident on the whole device at once:
// grid-stride HBM kernels launch exactly this many, so every workgroup runs in the first (only) round
// and the grid never has a partial second round.
static inline int resident_grid(const void* kernel, int threads) {
    int dev = 0, cus = 256, per = 1;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, threads, 0) != hipSuccess || per < 1) per = 1;
    return per * cus;
}
