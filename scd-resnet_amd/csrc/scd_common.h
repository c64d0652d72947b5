// Shared device helpers for libscdhip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

// fp16 compute mode (SCD_DT_F16).  The type-generic sources (conv_gemm, bn, layers, stem, pad) are compiled twice:
// once as written (16-bit storage type h16 = __bf16, v_mfma_f32_16x16x32_bf16) and once with SCD_F16_BUILD, where h16
// is _Float16, the MFMA is v_mfma_f32_16x16x32_f16 and every entry point gets the suffix __f16.  Those sources name
// the 16-bit type h16 (and h16x8 / mfma_16x16x32_h16) wherever it is the build's type; __bf16 in them is always a real
// bf16, whichever build.  A call with
// dtype SCD_DT_F16 is forwarded by the first build to the second with dtype SCD_DT_BF16 ("the 16-bit type"), so
// every kernel, tile shape and dispatch rule is shared and the C-ABI takes SCD_DT_F16 like any other dtype.
#ifdef SCD_F16_BUILD
#define scd_conv_gemm scd_conv_gemm__f16
#define scd_conv_gemm_bnbwd scd_conv_gemm_bnbwd__f16
#define scd_conv_gemm_heads scd_conv_gemm_heads__f16
#define scd_conv_gemm_heads_keep scd_conv_gemm_heads_keep__f16
#define scd_conv_wgrad_workspace scd_conv_wgrad_workspace__f16
#define scd_conv_wgrad_nsplit2 scd_conv_wgrad_nsplit2__f16
#define scd_conv_wgrad_nsplit scd_conv_wgrad_nsplit__f16
#define scd_conv_wgrad scd_conv_wgrad__f16
#define scd_wgrad_reduce scd_wgrad_reduce__f16
#define scd_wgrad_reduce_rows scd_wgrad_reduce_rows__f16
#define scd_stats_collapse scd_stats_collapse__f16
#define scd_stats_collapse_to scd_stats_collapse_to__f16
#define scd_bn_finalize scd_bn_finalize__f16
#define scd_bn_finalize_n scd_bn_finalize_n__f16
#define scd_bn_bwd_finalize_n scd_bn_bwd_finalize_n__f16
#define scd_bn_apply scd_bn_apply__f16
#define scd_bn_bwd_reduce scd_bn_bwd_reduce__f16
#define scd_bn_bwd_finalize scd_bn_bwd_finalize__f16
#define scd_bn_bwd_apply scd_bn_bwd_apply__f16
#define scd_bn_bwd_reduce2 scd_bn_bwd_reduce2__f16
#define scd_bn_bwd_apply2 scd_bn_bwd_apply2__f16
#define scd_pack_weights_batched scd_pack_weights_batched__f16
#define scd_pack_weight scd_pack_weight__f16
#define scd_im2col_stem scd_im2col_stem__f16
#define scd_stem_pool_fwd scd_stem_pool_fwd__f16
#define scd_stem_pool_bwd scd_stem_pool_bwd__f16
#define scd_stem_pool_bwd_bn scd_stem_pool_bwd_bn__f16
#define scd_heads_fwd scd_heads_fwd__f16
#define scd_heads_bwd_accsize scd_heads_bwd_accsize__f16
#define scd_heads_bwd scd_heads_bwd__f16
#define scd_heads_bwd_packed scd_heads_bwd_packed__f16
#define scd_heads_bwd_packed_split scd_heads_bwd_packed_split__f16
#define scd_heads_sparse_bwd scd_heads_sparse_bwd__f16
#define scd_heads_sparse_fixup scd_heads_sparse_fixup__f16
#define scd_heads_bwd_weight_finalize scd_heads_bwd_weight_finalize__f16
#define scd_adam_step scd_adam_step__f16
#define scd_adam_step_dev scd_adam_step_dev__f16
#define scd_sgd_step_dev scd_sgd_step_dev__f16
#define scd_stem_conv_fwd scd_stem_conv_fwd__f16
#define scd_stem_conv_wgrad_nsplit scd_stem_conv_wgrad_nsplit__f16
#define scd_stem_conv_wgrad scd_stem_conv_wgrad__f16
#define scd_stem_bwd_nsplit scd_stem_bwd_nsplit__f16
#define scd_conv_dgrad_s2 scd_conv_dgrad_s2__f16
#define scd_stem_bwd_fused scd_stem_bwd_fused__f16
#define scd_stem_bwd_combine scd_stem_bwd_combine__f16
#define scd_pad_channels scd_pad_channels__f16
#endif

#include "../../include/scdhip.h"

// The fp16 build's kernels sit in an inline namespace `f16` inside each file's anonymous namespace, so their symbol
// names (and the rocprofv3 kernel names) differ from the bf16 build's even where a kernel is not templated on the
// 16-bit type (tools/prof_summary.py labels them by it).
#ifdef SCD_F16_BUILD
#define SCD_KERNEL_NS_BEGIN inline namespace f16 {
#define SCD_KERNEL_NS_END }
#else
#define SCD_KERNEL_NS_BEGIN
#define SCD_KERNEL_NS_END
#endif

#ifdef SCD_F16_BUILD
#define SCD_F16_FWD(fn, ...) ((void)0)
#else
#define SCD_F16_DECL(fn) extern "C" decltype(fn) fn##__f16;
SCD_F16_DECL(scd_conv_gemm)
SCD_F16_DECL(scd_conv_gemm_bnbwd)
SCD_F16_DECL(scd_conv_gemm_heads)
SCD_F16_DECL(scd_conv_gemm_heads_keep)
SCD_F16_DECL(scd_conv_wgrad_nsplit2)
SCD_F16_DECL(scd_conv_wgrad_nsplit)
SCD_F16_DECL(scd_conv_wgrad)
SCD_F16_DECL(scd_bn_apply)
SCD_F16_DECL(scd_bn_bwd_reduce)
SCD_F16_DECL(scd_bn_bwd_apply)
SCD_F16_DECL(scd_bn_bwd_reduce2)
SCD_F16_DECL(scd_bn_bwd_apply2)
SCD_F16_DECL(scd_pack_weights_batched)
SCD_F16_DECL(scd_pack_weight)
SCD_F16_DECL(scd_im2col_stem)
SCD_F16_DECL(scd_stem_pool_fwd)
SCD_F16_DECL(scd_stem_pool_bwd)
SCD_F16_DECL(scd_stem_pool_bwd_bn)
SCD_F16_DECL(scd_heads_fwd)
SCD_F16_DECL(scd_heads_bwd)
SCD_F16_DECL(scd_heads_bwd_packed)
SCD_F16_DECL(scd_heads_bwd_packed_split)
SCD_F16_DECL(scd_heads_sparse_bwd)
SCD_F16_DECL(scd_heads_sparse_fixup)
SCD_F16_DECL(scd_stem_conv_fwd)
SCD_F16_DECL(scd_stem_conv_wgrad)
SCD_F16_DECL(scd_stem_bwd_fused)
SCD_F16_DECL(scd_conv_dgrad_s2)
SCD_F16_DECL(scd_stem_bwd_combine)
SCD_F16_DECL(scd_pad_channels)
#define SCD_F16_FWD(fn, ...) \
    do { if (dtype == SCD_DT_F16) return fn##__f16(SCD_DT_BF16, __VA_ARGS__); } while (0)
#endif

// half `hi` of a 32-bit word holding two 16-bit values, as float
__device__ __forceinline__ float h16_word_half(unsigned w, int hi) {
#ifdef SCD_F16_BUILD
    return (float)__builtin_bit_cast(_Float16, (unsigned short)(hi ? w >> 16 : w & 0xffffu));
#else
    return __uint_as_float(hi ? (w & 0xffff0000u) : (w << 16));
#endif
}

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;     // a real bf16 vector in either build
#ifdef SCD_F16_BUILD
typedef _Float16 h16;                                           // the build's 16-bit compute type
#else
typedef __bf16 h16;
#endif
typedef __attribute__((ext_vector_type(8))) h16 h16x8;
typedef __attribute__((ext_vector_type(4))) h16 h16x4;
// v_mfma_f32_16x16x32_{bf16,f16} on the build's 16-bit type
__device__ __forceinline__ f32x4 mfma_16x16x32_h16(h16x8 a, h16x8 b, f32x4 c) {
#ifdef SCD_F16_BUILD
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
#else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
#endif
}
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

#define SCD_RETURN_LAUNCH() return (int)hipGetLastError()

template <typename T> __device__ __forceinline__ float to_f(T v);
template <> __device__ __forceinline__ float to_f<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f<h16>(h16 v) { return (float)v; }

template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ h16 from_f<h16>(float v) { return (h16)v; }

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
template <> struct Vec16<h16> {
    static constexpr int N = 8;
    __device__ static void load(const void* p, float* f) {
        h16x8 v = *(const h16x8*)p;
#pragma unroll
        for (int i = 0; i < 8; ++i) f[i] = (float)v[i];
    }
    __device__ static void store(void* p, const float* f) {
        h16x8 v;
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = (h16)f[i];
        *(h16x8*)p = v;
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
static inline int resident_grid(const void* kernel, int threads, size_t dyn_lds = 0) {
    int dev = 0, cus = 256, per = 1;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, threads, dyn_lds) != hipSuccess || per < 1) per = 1;
    return per * cus;
}
