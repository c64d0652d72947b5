// Shared device helpers for libscdhip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

// fp16 compute mode (SCD_DT_F16).  The type-generic sources (conv_gemm, bn, layers, stem, pad) are compiled twice:
// once as written (16-bit type __bf16, v_mfma_f32_16x16x32_bf16) and once with SCD_F16_BUILD, where the 16-bit type
// is _Float16, the MFMA is v_mfma_f32_16x16x32_f16 and every entry point gets the suffix __f16.  A call with
// dtype SCD_DT_F16 is forwarded by the first build to the second with dtype SCD_DT_BF16 ("the 16-bit type"), so
// every kernel, tile shape and dispatch rule is shared and the C-ABI takes SCD_DT_F16 like any other dtype.
#ifdef SCD_F16_BUILD
#define scd_conv_gemm scd_conv_gemm__f16
#define scd_conv_gemm_bnbwd scd_conv_gemm_bnbwd__f16
#define scd_conv_gemm_fin scd_conv_gemm_fin__f16
#define scd_conv_gemm_bnbwd_fin scd_conv_gemm_bnbwd_fin__f16
#define scd_stem_conv_fwd_fin scd_stem_conv_fwd_fin__f16
#define scd_bn_bwd_reduce_fin scd_bn_bwd_reduce_fin__f16
#define scd_bn_bwd_reduce2_fin scd_bn_bwd_reduce2_fin__f16
#define scd_bn_fin_standalone scd_bn_fin_standalone__f16
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
#define scd_stem_bwd_fused_pooled scd_stem_bwd_fused_pooled__f16
#define scd_stem_conv_pool_fwd scd_stem_conv_pool_fwd__f16
#define scd_stem_bwd_combine scd_stem_bwd_combine__f16
#define scd_pad_channels scd_pad_channels__f16
#define __bf16 _Float16
#define __builtin_amdgcn_mfma_f32_16x16x32_bf16 __builtin_amdgcn_mfma_f32_16x16x32_f16
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
SCD_F16_DECL(scd_conv_gemm_fin)
SCD_F16_DECL(scd_conv_gemm_bnbwd_fin)
SCD_F16_DECL(scd_stem_conv_fwd_fin)
SCD_F16_DECL(scd_bn_bwd_reduce_fin)
SCD_F16_DECL(scd_bn_bwd_reduce2_fin)
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
SCD_F16_DECL(scd_stem_bwd_fused_pooled)
SCD_F16_DECL(scd_stem_conv_pool_fwd)
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

// ---- BN finalize fused into the statistics producer (scd_bn_fin, include/scdhip.h) ----
// The descriptor lives in device memory (written once by the caller); the kernels take its pointer plus the
// statistics buffer they add into, and read the descriptor only in the tail -- so it costs the kernel body one
// pointer argument, not twenty (kernel arguments are loaded into SGPRs up front: the by-value form spilled SGPRs in
// the ping-pong GEMM and VGPRs in the BN reduce).
// SCD_FIN_ABL (timing-only ablation builds, `make variant`; never the product): 1 = the last workgroup skips the
// finalize arithmetic, 2 = no vmcnt drain before the arrival count
#ifndef SCD_FIN_ABL
#define SCD_FIN_ABL 0
#endif
struct BnFinDev {
    const scd_bn_fin* f;      // device memory; NULL: the launch does not finalize
    double* stats;            // the producer's statistics, [rep][2][ld]
    int ld;
};
// replica a workgroup adds its statistics into: the first SCD_FIN_REPLICAS when the launch finalizes them itself
__device__ __forceinline__ int stat_rep(const BnFinDev& d, int bid) {
    return d.f ? bid % SCD_FIN_REPLICAS : bid % SCD_STAT_REPLICAS;
}
// Called by every remaining thread of every workgroup at its end: true in the last workgroup to arrive, once every
// other workgroup's statistics atomics are visible.  The hand-off is "8-byte agent atomics on both sides": the
// statistics are fp64 atomic adds (performed at the memory side, never dirty in an L2) and the last workgroup reads
// them with agent-scope (sc1) loads, so no fence is needed -- only every wave's own atomics drained (vmcnt) before
// the one counter add that signals them.  An agent-scope release/acquire here (a `__threadfence()` per workgroup)
// writes back the XCD's whole L2 every time and made the producers 1.2-10x slower.
// flag: one int of the kernel's own LDS (free once the workgroup's epilogue has passed the first barrier here): a
// second `__shared__` object in an LDS-DMA kernel makes the compiler's wait counting drain every DMA prefetch
// (s_waitcnt vmcnt(0) before the fragment reads: the ring kernel lost 20-35 % per call)
__device__ __forceinline__ bool bn_fin_arrive(int* counter, int* flag) {
    // two levels, so no counter word takes more than ~1/64 of the launch's arrivals (one word serialises its returning
    // atomics at ~90 per us: a resident-grid launch of 2048 workgroups, all finishing together, waited ~20 us on one):
    // workgroup b counts in on shard b % 64, the last of a shard counts the shard in on counter[SCD_FIN_SHARDS]
#if SCD_FIN_ABL != 2
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    __syncthreads();
    if (threadIdx.x == 0) {
        const int nblk = (int)(gridDim.x * gridDim.y * gridDim.z);
        const int bid = (int)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z));
        const int sh = bid % SCD_FIN_SHARDS;
        const int nsh = nblk < SCD_FIN_SHARDS ? nblk : SCD_FIN_SHARDS;
        const int members = (nblk - sh + SCD_FIN_SHARDS - 1) / SCD_FIN_SHARDS;
        int last = __hip_atomic_fetch_add(counter + sh, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == members - 1;
        if (last)
            last = __hip_atomic_fetch_add(counter + SCD_FIN_SHARDS, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                   nsh - 1;
        *flag = last;
    }
    __syncthreads();
    return *flag != 0;
}
// global-address-space view of a pointer read from a descriptor (plain `global_` accesses instead of `flat_`)
template <typename T> __device__ __forceinline__ __attribute__((address_space(1))) T* gptr(T* p) {
    return (__attribute__((address_space(1))) T*)p;
}
// The finalize of one layer by threads 0 .. nact-1 of the last workgroup: the replicas summed in a fixed order
// (agent-scope loads: they were written by other XCDs' atomics) and re-zeroed, then bn_finalize_kernel's /
// bn_bwd_finalize_kernel's arithmetic.  This runs after every other workgroup has left, so its latency is the
// launch's: the descriptor is copied to registers once (its fields would otherwise be re-read after every store
// through one of its pointers) and every per-channel operand is loaded before the first wait.
template <int NREP = SCD_FIN_REPLICAS>
__device__ __forceinline__ void bn_fin_compute(const scd_bn_fin* fp, double* stats, int ld, int nact) {
    const scd_bn_fin f = *fp;
    const int C = f.C;
    const double count = f.count;
    // CH replicas (2 CH loads) in flight at a time: within the register budget of the BN kernels (BN_EW_WAVES)
    constexpr int CH = NREP < 4 ? NREP : 4;
    static_assert(NREP % CH == 0, "replica count");
    for (int c = threadIdx.x; c < C; c += nact) {
        float g = 1.f, b = 0.f, rm = 0.f, rv = 0.f, is = 0.f, mu = 0.f, dg = 0.f, db = 0.f;
        if (f.gamma) g = gptr(f.gamma)[c];
        if (!f.backward) {
            if (f.beta) b = gptr(f.beta)[c];
            if (f.running_mean) { rm = gptr(f.running_mean)[c]; rv = gptr(f.running_var)[c]; }
        } else {
            is = gptr(f.invstd)[c];
            mu = gptr(f.mean)[c];
            if (f.dgamma) dg = gptr(f.dgamma)[c];
            if (f.dbeta) db = gptr(f.dbeta)[c];
        }
        __attribute__((address_space(1))) double* p0 = gptr(stats) + c;
        double s = 0.0, q = 0.0;
        for (int r0 = 0; r0 < NREP; r0 += CH) {
            double vs[CH], vq[CH];
#pragma unroll
            for (int r = 0; r < CH; ++r) {
                vs[r] = __hip_atomic_load(p0 + (long)(2 * (r0 + r)) * ld, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                vq[r] = __hip_atomic_load(p0 + (long)(2 * (r0 + r) + 1) * ld, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
            }
#pragma unroll
            for (int r = 0; r < CH; ++r) { s += vs[r]; q += vq[r]; }
        }
#pragma unroll
        for (int r = 0; r < NREP; ++r) {
            p0[(long)(2 * r) * ld] = 0.0;
            p0[(long)(2 * r + 1) * ld] = 0.0;
        }
        if (!f.backward) {
            const double mean = s / count;
            double var = q / count - mean * mean;
            if (var < 0.0) var = 0.0;
            const float invstd = (float)(1.0 / sqrt(var + (double)f.eps));
            const float sc = g * invstd;
            gptr(f.mean)[c] = (float)mean;
            gptr(f.invstd)[c] = invstd;
            gptr(f.scale)[c] = sc;
            gptr(f.shift)[c] = b - (float)mean * sc;
            if (f.running_mean) {
                const float m = f.momentum;
                const double unbiased = count > 1.0 ? var * count / (count - 1.0) : var;
                gptr(f.running_mean)[c] = (1.f - m) * rm + m * (float)mean;
                gptr(f.running_var)[c] = (1.f - m) * rv + m * (float)unbiased;
            }
        } else {
            if (f.dgamma) gptr(f.dgamma)[c] = dg + f.gscale * (float)q;
            if (f.dbeta) gptr(f.dbeta)[c] = db + f.gscale * (float)s;
            const float sc = g * is;
            const float k1 = (float)(s / count);
            const float k2 = (float)(q / count);
            gptr(f.coef)[c] = sc;
            gptr(f.coef)[C + c] = -sc * is * k2;
            gptr(f.coef)[2 * C + c] = -sc * k1 + sc * is * k2 * mu;
        }
    }
    if (threadIdx.x == 0 && !f.backward && f.num_batches) *gptr(f.num_batches) += 1;
}
// the tail of a producer (one layer; d1 != NULL: a second layer whose statistics the launch produced too, counted on
// d0's counter); every remaining thread calls it at the kernel's end
__device__ __forceinline__ void bn_fin_tail2(const BnFinDev& d0, const BnFinDev* d1, int nact, void* lds) {
    if (!d0.f) return;
    int* counter = d0.f->counter;
    if (!bn_fin_arrive(counter, (int*)lds)) return;
#if SCD_FIN_ABL != 1
    bn_fin_compute(d0.f, d0.stats, d0.ld, nact);
    if (d1 && d1->f) bn_fin_compute(d1->f, d1->stats, d1->ld, nact);
#endif
    for (int i = threadIdx.x; i < SCD_FIN_COUNTERS; i += nact)
        __hip_atomic_store(counter + i, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void bn_fin_tail(const BnFinDev& d, int nact, void* lds) { bn_fin_tail2(d, nullptr, nact, lds); }
// host: the kernels' view of a `_fin` entry point's argument (off when fin == NULL)
static inline BnFinDev bn_fin_dev(const scd_bn_fin* fin_dev, double* stats, int ld) {
    BnFinDev d;
    d.f = (fin_dev && stats) ? fin_dev : nullptr;
    d.stats = stats;
    d.ld = ld;
    return d;
}

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
