// Training-mode BatchNorm2d pieces for NHWC activations (residuals.py:92,95,212,262,306).
// Statistics are accumulated in fp64 into SCD_STAT_REPLICAS replicas (spreads the atomics),
// finalised per channel; apply / backward passes are 16-byte-vectorised elementwise kernels.
#include <algorithm>
#include <type_traits>

#include "scd_common.h"

#ifndef BN_BWD_U
#define BN_BWD_U 1
#endif
// Elementwise BN kernels are budgeted for 6 waves per SIMD (<= 80 VGPRs): the weight-gradient stream's ping-pong
// kernel holds 2 x 216 of the 512 VGPRs per SIMD lane (one 8-wave workgroup per CU), so a wave that needs 88 could
// not start on any CU until those workgroups retire (in the step the deconv2 BN backward apply then waited out the
// whole deconv3 weight gradient)
// vectors in flight per thread in bn_bwd_apply_kernel (80 VGPRs at 2, no spill): beside the weight-gradient stream's
// one-workgroup-per-CU GEMM a CU holds one or two of its waves per SIMD, so the bytes each wave keeps in flight set
// its bandwidth there (75 VGPRs at 2 in both 16-bit builds since the loop is specialised per mask kind)
#ifndef BN_APPLY_U
#define BN_APPLY_U 2
#endif
#ifndef BN_EW_WAVES
#define BN_EW_WAVES 6
#endif

namespace {
SCD_KERNEL_NS_BEGIN

// sum replicas into replica 0 and zero the others (buffers are persistent: the consumer re-zeroes)
__global__ void stats_collapse_kernel(double* stats, int nrep, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double s = 0.0;
    for (int r = 0; r < nrep; ++r) {
        s += stats[(long)r * n + i];
        if (r) stats[(long)r * n + i] = 0.0;
    }
    stats[i] = s;
}

// SyncBN staging: out[i] = sum of the replicas, every replica zeroed (two layers' sums side by side in one buffer,
// so one collective reduces both)
__global__ void stats_collapse_to_kernel(double* stats, int nrep, int n, double* out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double s = 0.0;
    for (int r = 0; r < nrep; ++r) {
        s += stats[(long)r * n + i];
        stats[(long)r * n + i] = 0.0;
    }
    out[i] = s;
}

// one wave per channel: lane r sums replica r (and zeroes it: persistent, consumer-cleared buffers)
__device__ __forceinline__ void wave_collect(double* stats, int nrep, int C, int c, double& s, double& q) {
    const int lane = threadIdx.x & 63;
    double a = 0.0, b = 0.0;
    for (int r = lane; r < nrep; r += 64) {
        double* p = stats + (long)r * 2 * C;
        a += p[c];
        b += p[C + c];
        p[c] = 0.0;
        p[C + c] = 0.0;
    }
    s = wave_sum_d(a);
    q = wave_sum_d(b);
}

__device__ __forceinline__ void bn_finalize_channel(int c, double* stats, int nrep, int C, double count,
                                                    const float* gamma, const float* beta, float* rmean, float* rvar,
                                                    float momentum, float eps, float* mean_o, float* invstd_o,
                                                    float* scale_o, float* shift_o, int64_t* nbt) {
    double mean, var;
    if (stats) {
        double s, q;
        wave_collect(stats, nrep, C, c, s, q);
        mean = s / count;
        var = q / count - mean * mean;
        if (var < 0.0) var = 0.0;
    } else {                       // eval mode: normalise with the running statistics
        mean = rmean[c];
        var = rvar[c];
    }
    if ((threadIdx.x & 63) != 0) return;
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    const float g = gamma ? gamma[c] : 1.f;
    const float b = beta ? beta[c] : 0.f;
    const float sc = g * invstd;
    mean_o[c] = (float)mean;
    invstd_o[c] = invstd;
    scale_o[c] = sc;
    shift_o[c] = b - (float)mean * sc;
    // (statistics that are NaN -- a failed peer-memory SyncBN all-reduce poisons its result, scdhip/peer.py -- leave the
    // running statistics AND num_batches_tracked as they were, so a checkpoint written after the failure still carries
    // the last good, mutually consistent ones; channel 0's lane counts the batch)
    if (c == 0 && nbt && stats && mean == mean && var == var) *nbt += 1;
    if (stats && rmean && mean == mean && var == var) {
        const double unbiased = count > 1.0 ? var * count / (count - 1.0) : var;
        rmean[c] = (1.f - momentum) * rmean[c] + momentum * (float)mean;
        rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)unbiased;
    }
}

__global__ void bn_finalize_kernel(double* stats, int nrep, int C, double count, const float* gamma,
                                   const float* beta, float* rmean, float* rvar, int64_t* nbt, float momentum,
                                   float eps, float* mean_o, float* invstd_o, float* scale_o, float* shift_o) {
    const int c = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (c >= C) return;
    bn_finalize_channel(c, stats, nrep, C, count, gamma, beta, rmean, rvar, momentum, eps, mean_o, invstd_o, scale_o,
                        shift_o, nbt);
}

// up to SCD_BN_FIN_MAX layers in one launch (scd_bn_finalize_n): layer i owns blocks [b0[i], b0[i + 1])
struct FinN {
    scd_bn_fin_args l[SCD_BN_FIN_MAX];
    int b0[SCD_BN_FIN_MAX + 1];
    int n;
};
__global__ void bn_finalize_n_kernel(FinN f) {
    int i = 0;
#pragma unroll
    for (int k = 1; k < SCD_BN_FIN_MAX; ++k)
        if (k < f.n && (int)blockIdx.x >= f.b0[k]) i = k;
    const scd_bn_fin_args& a = f.l[i];
    const int blk = blockIdx.x - f.b0[i];
    const int c = blk * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (c >= a.C) return;
    bn_finalize_channel(c, a.stats, a.nrep, a.C, a.count, a.gamma, a.beta, a.running_mean, a.running_var, a.momentum,
                        a.eps, a.mean, a.invstd, a.scale, a.shift, a.num_batches);
}

// E consecutive per-channel floats (E = 4 or 8, 16-B aligned) as float4 loads
template <int E>
__device__ __forceinline__ void load_params(const float* p, float* v) {
#pragma unroll
    for (int k = 0; k < E / 4; ++k) {
        const float4 f = *(const float4*)(p + 4 * k);
        v[4 * k] = f.x; v[4 * k + 1] = f.y; v[4 * k + 2] = f.z; v[4 * k + 3] = f.w;
    }
}

// Per-channel parameters of the backward kernels live in LDS and are re-read per vector instead of held in
// registers (5-6 x E floats per thread otherwise): with <= 80 VGPRs (BN_EW_WAVES) the waves fit beside the
// weight-gradient stream's one-workgroup-per-CU GEMMs.  The offset is made opaque so the reads stay in the loop.
// Only the channels a block touches are staged (chan_window): at most 256 chunks of E channels, so the dynamic LDS is
// bounded (<= 6 x 2048 x 4 B for bf16) whatever C is, and the host sizes the grid with that LDS in the occupancy query.
__device__ __forceinline__ void stage_params(float* sp, const float* const* src, int nsrc, int cb, int W) {
    for (int i = threadIdx.x; i < nsrc * W; i += blockDim.x) {
        const int k = i / W;
        sp[i] = src[k] ? src[k][cb + i - k * W] : 0.f;
    }
    __syncthreads();
}
// first channel and width of the channel window of this block's threads in the elementwise kernels (one fixed chunk
// of E channels per thread, grid stride a multiple of the C/E chunks per row, ew_rows_ok): the whole row when it has
// <= 256 chunks, else the block's own 256-chunk window
__device__ __forceinline__ void chan_window(int C, int E, int& cb, int& W) {
    const unsigned cpr = (unsigned)C / E;
    cb = cpr > 256u ? (int)((blockIdx.x * 256u) % cpr) * E : 0;
    W = cpr > 256u ? 256 * E : C;
}
template <int E>
__device__ __forceinline__ void lds_params(const float* sp, int off, float* v) {
    asm volatile("" : "+v"(off));
#pragma unroll
    for (int k = 0; k < E / 4; ++k) {
        const float4 f = *(const float4*)(sp + off + 4 * k);
        v[4 * k] = f.x; v[4 * k + 1] = f.y; v[4 * k + 2] = f.z; v[4 * k + 3] = f.w;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void bn_apply_kernel(const T* y, T* out, int C, unsigned nvec, const float* scale,
                                                       const float* shift, const T* res, const float* rscale,
                                                       const float* rshift, int relu) {
    constexpr int E = Vec16<T>::N;
    constexpr int U = 4;
    // the grid stride is a multiple of the chunks per row (C/E divides 256): a thread always owns the same
    // E channels, so the per-channel parameters live in registers (no LDS, no bank conflicts).  U vectors
    // per thread are loaded before any is used (U x 16 B, x2 with a residual, in flight per thread).
    const unsigned cpr = (unsigned)C / E;
    const unsigned v0 = blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned stride = gridDim.x * blockDim.x;
    const int c0 = (int)(v0 % cpr) * E;
    float sc[E], sh[E], rs[E], rh[E];
    load_params<E>(scale + c0, sc);
    load_params<E>(shift + c0, sh);
    if (rscale) { load_params<E>(rscale + c0, rs); load_params<E>(rshift + c0, rh); }
    else {
#pragma unroll
        for (int e = 0; e < E; ++e) { rs[e] = 0.f; rh[e] = 0.f; }
    }
    auto body = [&](float* a, const float* r) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
            float o = a[e] * sc[e] + sh[e];
            if (res) o += rscale ? (r[e] * rs[e] + rh[e]) : r[e];
            if (relu) o = fmaxf(o, 0.f);
            a[e] = o;
        }
    };
    unsigned v = v0;
    for (; v + (U - 1) * stride < nvec; v += U * stride) {
        float a[U][E], r[U][E];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            Vec16<T>::load(y + (size_t)(v + u * stride) * E, a[u]);
            if (res) Vec16<T>::load(res + (size_t)(v + u * stride) * E, r[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            body(a[u], r[u]);
            Vec16<T>::store(out + (size_t)(v + u * stride) * E, a[u]);
        }
    }
    for (; v < nvec; v += stride) {
        float a[E], r[E];
        Vec16<T>::load(y + (size_t)v * E, a);
        if (res) Vec16<T>::load(res + (size_t)v * E, r);
        body(a, r);
        Vec16<T>::store(out + (size_t)v * E, a);
    }
}

// Per-channel Σdz and Σdz·x̂ over rows (dz = dout masked by relu(mask) > 0).  A 256-thread block owns
// rows [r0, r1): thread = (row lane rsub, 16-B channel chunk ch); 4 rows per step are loaded before
// any is used (4 x 3 independent 16-B loads in flight per thread); the block's partials are folded
// over row lanes in LDS by all threads and added to one fp64 replica slot per channel.
template <typename T>
__global__ __launch_bounds__(256, BN_EW_WAVES) void bn_bwd_reduce_kernel(const T* dout, const T* mask, const T* y,
                                                            const float* rsc, const float* rsh,
                                                            const float* mean, const float* invstd, int C, int ld,
                                                            unsigned rows, unsigned rows_per_block, double* stats) {
    constexpr int E = Vec16<T>::N;
    constexpr int U = BN_BWD_U;
    constexpr int nt = 256;
    const int cpr = C / E;                     // chunks per row of this channel slice (divides 256)
    const int rpi = nt / cpr;                  // row lanes
    const int tid = threadIdx.x;
    const int ch = tid % cpr;
    const int rsub = tid / cpr;
    const unsigned r0 = blockIdx.x * rows_per_block;
    const unsigned r1 = min(rows, r0 + rows_per_block);
    __shared__ float red[2 * nt * E];
    extern __shared__ __attribute__((aligned(16))) float sp[];        // 4 x C floats (dynamic LDS)     // mean, invstd, rsc, rsh
    {
        const float* src[4] = {mean, invstd, rsc, rsh};
        stage_params(sp, src, 4, 0, C);
    }
    float s[E], q[E];
#pragma unroll
    for (int e = 0; e < E; ++e) { s[e] = 0.f; q[e] = 0.f; }
    // one loop per mask kind (0: none, 1: the stored activation, 2: BN+ReLU recomputed from y), as in
    // bn_bwd_apply_kernel: no per-element branch regions
    auto run = [&](auto kind) {
        constexpr int MK = decltype(kind)::value;
        auto acc_raw = [&](const uint4& rd, const uint4& ry, const uint4& rm) {
            float d[E], yv[E], mk[E], mu[E], is[E], ka[E], kb[E];
            Vec16<T>::load(&rd, d);
            Vec16<T>::load(&ry, yv);
            if constexpr (MK == 1) Vec16<T>::load(&rm, mk);
            lds_params<E>(sp, ch * E, mu);
            lds_params<E>(sp, C + ch * E, is);
            if constexpr (MK == 2) { lds_params<E>(sp, 2 * C + ch * E, ka); lds_params<E>(sp, 3 * C + ch * E, kb); }
#pragma unroll
            for (int e = 0; e < E; ++e) {
                bool off = false;
                if constexpr (MK == 1) off = !(mk[e] > 0.f);
                if constexpr (MK == 2) off = !(yv[e] * ka[e] + kb[e] > 0.f);
                const float dz = off ? 0.f : d[e];
                s[e] += dz;
                q[e] += dz * (yv[e] - mu[e]) * is[e];
            }
        };
        unsigned r = r0 + rsub;
        for (; r + (U - 1) * rpi < r1; r += U * rpi) {
            uint4 rd[U], ry[U], rm[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const unsigned i = (r + u * rpi) * (unsigned)ld + ch * E;
                rd[u] = *(const uint4*)(dout + i);
                ry[u] = *(const uint4*)(y + i);
                rm[u] = MK == 1 ? *(const uint4*)(mask + i) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) acc_raw(rd[u], ry[u], rm[u]);
        }
        for (; r < r1; r += rpi) {
            const unsigned i = r * (unsigned)ld + ch * E;
            const uint4 rd = *(const uint4*)(dout + i), ry = *(const uint4*)(y + i);
            const uint4 rm = MK == 1 ? *(const uint4*)(mask + i) : make_uint4(0, 0, 0, 0);
            acc_raw(rd, ry, rm);
        }
    };
    if (mask) run(std::integral_constant<int, 1>{});
    else if (rsc) run(std::integral_constant<int, 2>{});
    else run(std::integral_constant<int, 0>{});
    // red[stat][rsub][channel]
#pragma unroll
    for (int e = 0; e < E; ++e) {
        red[rsub * C + ch * E + e] = s[e];
        red[nt * E + rsub * C + ch * E + e] = q[e];
    }
    __syncthreads();
    const int rep = (int)(blockIdx.x % SCD_STAT_REPLICAS);
    for (int c = tid; c < C; c += nt) {
        double ss = 0.0, qq = 0.0;
        for (int k = 0; k < rpi; ++k) {
            ss += red[k * C + c];
            qq += red[nt * E + k * C + c];
        }
        atomic_add_f64(stats + ((long)rep * 2 + 0) * ld + c, ss);
        atomic_add_f64(stats + ((long)rep * 2 + 1) * ld + c, qq);
    }
}

__device__ __forceinline__ void bn_bwd_finalize_channel(int c, double* stats, int nrep, int C, double count,
                                                        const float* gamma, const float* mean, const float* invstd,
                                                        float* dgamma, float* dbeta, float gscale, float* coef) {
    double s, q;
    wave_collect(stats, nrep, C, c, s, q);
    if ((threadIdx.x & 63) != 0) return;
    if (dgamma) dgamma[c] += gscale * (float)q;
    if (dbeta) dbeta[c] += gscale * (float)s;
    const float g = gamma ? gamma[c] : 1.f;
    const float is = invstd[c];
    const float sc = g * is;
    const float k1 = (float)(s / count);
    const float k2 = (float)(q / count);
    // dy = sc*(dz - k1 - xhat*k2), xhat = (y-mean)*is
    coef[c] = sc;
    coef[C + c] = -sc * is * k2;
    coef[2 * C + c] = -sc * k1 + sc * is * k2 * mean[c];
}

__global__ void bn_bwd_finalize_kernel(double* stats, int nrep, int C, double count, const float* gamma,
                                       const float* mean, const float* invstd, float* dgamma, float* dbeta,
                                       float gscale, float* coef) {
    const int c = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (c >= C) return;
    bn_bwd_finalize_channel(c, stats, nrep, C, count, gamma, mean, invstd, dgamma, dbeta, gscale, coef);
}

struct BwdFinN {
    scd_bn_bwd_fin_args l[SCD_BN_FIN_MAX];
    int b0[SCD_BN_FIN_MAX + 1];
    int n;
};
__global__ void bn_bwd_finalize_n_kernel(BwdFinN f) {
    int i = 0;
#pragma unroll
    for (int k = 1; k < SCD_BN_FIN_MAX; ++k)
        if (k < f.n && (int)blockIdx.x >= f.b0[k]) i = k;
    const scd_bn_bwd_fin_args& a = f.l[i];
    const int c = (blockIdx.x - f.b0[i]) * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (c >= a.C) return;
    bn_bwd_finalize_channel(c, a.stats, a.nrep, a.C, a.count, a.gamma, a.mean, a.invstd, a.dgamma, a.dbeta, a.gscale,
                            a.coef);
}

template <typename T>
__global__ __launch_bounds__(256, BN_EW_WAVES) void bn_bwd_apply_kernel(const T* dout, const T* mask, const T* y, const float* rsc,
                                                           const float* rsh, const float* coef, int C, unsigned nvec,
                                                           T* dy, T* dz_out) {
    constexpr int E = Vec16<T>::N;
    // BN_APPLY_U vectors in flight, kept packed (16 B each) until used: <= 80 VGPRs, so the kernel's waves fit beside
    // a one-workgroup-per-CU GEMM of the weight-gradient stream (2 x 216 of the 512 VGPRs per lane) instead of
    // waiting for its workgroups to retire
    constexpr int U = BN_APPLY_U;
    // fixed channel chunk per thread (see bn_apply_kernel): coefficients in registers
    const unsigned cpr = (unsigned)C / E;
    const unsigned v0 = blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned stride = gridDim.x * blockDim.x;
    const int c0 = (int)(v0 % cpr) * E;
    extern __shared__ __attribute__((aligned(16))) float sp[];        // 5 x W floats (dynamic LDS): coef a, b, c, rsc, rsh
    int cb, W;
    chan_window(C, E, cb, W);
    {
        const float* src[5] = {coef, coef + C, coef + 2 * C, rsc, rsh};
        stage_params(sp, src, 5, cb, W);
    }
    const int cl = c0 - cb;
    // raw 16-B vectors -> dz (masked gradient) and dy, stored.  One loop per mask kind (0: none, 1: the stored
    // activation, 2: BN+ReLU recomputed from y): with the kind a runtime test inside the element loop the compiler
    // built the loop from per-element branch regions (8 per vector)
    auto run = [&](auto kind) {
        constexpr int MK = decltype(kind)::value;
        auto body = [&](size_t i, const uint4& rd, const uint4& ry, const uint4& rm) {
            float d[E], yv[E], mk[E], ca[E], cq[E], cc[E], ka[E], kb[E];
            Vec16<T>::load(&rd, d);
            Vec16<T>::load(&ry, yv);
            if constexpr (MK == 1) Vec16<T>::load(&rm, mk);
            lds_params<E>(sp, cl, ca);
            lds_params<E>(sp, W + cl, cq);
            lds_params<E>(sp, 2 * W + cl, cc);
            if constexpr (MK == 2) { lds_params<E>(sp, 3 * W + cl, ka); lds_params<E>(sp, 4 * W + cl, kb); }
#pragma unroll
            for (int e = 0; e < E; ++e) {
                bool off = false;
                if constexpr (MK == 1) off = !(mk[e] > 0.f);
                if constexpr (MK == 2) off = !(yv[e] * ka[e] + kb[e] > 0.f);
                const float dz = off ? 0.f : d[e];
                d[e] = dz;
                yv[e] = ca[e] * dz + cq[e] * yv[e] + cc[e];
            }
            Vec16<T>::store(dy + i, yv);
            if (dz_out) Vec16<T>::store(dz_out + i, d);
        };
        unsigned v = v0;
        for (; v + (U - 1) * stride < nvec; v += U * stride) {
            uint4 rd[U], ry[U], rm[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const size_t i = (size_t)(v + u * stride) * E;
                rd[u] = *(const uint4*)(dout + i);
                ry[u] = *(const uint4*)(y + i);
                rm[u] = MK == 1 ? *(const uint4*)(mask + i) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) body((size_t)(v + u * stride) * E, rd[u], ry[u], rm[u]);
        }
        for (; v < nvec; v += stride) {
            const size_t i = (size_t)v * E;
            const uint4 rd = *(const uint4*)(dout + i), ry = *(const uint4*)(y + i);
            const uint4 rm = MK == 1 ? *(const uint4*)(mask + i) : make_uint4(0, 0, 0, 0);
            body(i, rd, ry, rm);
        }
    };
    if (mask) run(std::integral_constant<int, 1>{});
    else if (rsc) run(std::integral_constant<int, 2>{});
    else run(std::integral_constant<int, 0>{});
}

// ---- two BN layers behind one residual join (BasicBlock / Bottleneck bn2|bn3 + downsample BN, residuals.py:
// 110-120, 158-165; CornerPool branchMergeBn + shortcutBn, cornerNetCPool.py:117-122): both take the same gradient
// dout through the same ReLU mask, so one pass reads dout and the mask once for both.  Per element and per thread the
// arithmetic is that of bn_bwd_reduce_kernel / bn_bwd_apply_kernel with a mask (no BN+ReLU recompute).
template <typename T>
__global__ __launch_bounds__(256, BN_EW_WAVES) void bn_bwd_reduce2_kernel(const T* dout, const T* mask, const T* ya, const T* yb,
                                                             const float* mean_a, const float* invstd_a,
                                                             const float* mean_b, const float* invstd_b, int C, int ld,
                                                             unsigned rows, unsigned rows_per_block, double* stats_a,
                                                             double* stats_b) {
    constexpr int E = Vec16<T>::N;
    constexpr int U = BN_BWD_U;
    constexpr int nt = 256;
    const int cpr = C / E;
    const int rpi = nt / cpr;
    const int tid = threadIdx.x;
    const int ch = tid % cpr;
    const int rsub = tid / cpr;
    const unsigned r0 = blockIdx.x * rows_per_block;
    const unsigned r1 = min(rows, r0 + rows_per_block);
    __shared__ float red[2 * nt * E];
    extern __shared__ __attribute__((aligned(16))) float sp[];        // 4 x C floats (dynamic LDS)     // mean_a, invstd_a, mean_b, invstd_b
    {
        const float* src[4] = {mean_a, invstd_a, mean_b, invstd_b};
        stage_params(sp, src, 4, 0, C);
    }
    float s[E], qa[E], qb[E];
#pragma unroll
    for (int e = 0; e < E; ++e) { s[e] = 0.f; qa[e] = 0.f; qb[e] = 0.f; }
    auto acc_raw = [&](const uint4& rd, const uint4& rm, const uint4& ra, const uint4& rb) {
        float d[E], mk[E], va[E], vb[E], mu[E], is[E];
        Vec16<T>::load(&rd, d);
        Vec16<T>::load(&rm, mk);
        Vec16<T>::load(&ra, va);
        Vec16<T>::load(&rb, vb);
#pragma unroll
        for (int e = 0; e < E; ++e) d[e] = !(mk[e] > 0.f) ? 0.f : d[e];
        lds_params<E>(sp, ch * E, mu);
        lds_params<E>(sp, C + ch * E, is);
#pragma unroll
        for (int e = 0; e < E; ++e) {
            s[e] += d[e];
            qa[e] += d[e] * (va[e] - mu[e]) * is[e];
        }
        lds_params<E>(sp, 2 * C + ch * E, mu);
        lds_params<E>(sp, 3 * C + ch * E, is);
#pragma unroll
        for (int e = 0; e < E; ++e) qb[e] += d[e] * (vb[e] - mu[e]) * is[e];
    };
    unsigned r = r0 + rsub;
    for (; r + (U - 1) * rpi < r1; r += U * rpi) {
        uint4 rd[U], rm[U], ra[U], rb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned i = (r + u * rpi) * (unsigned)ld + ch * E;
            rd[u] = *(const uint4*)(dout + i);
            rm[u] = *(const uint4*)(mask + i);
            ra[u] = *(const uint4*)(ya + i);
            rb[u] = *(const uint4*)(yb + i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc_raw(rd[u], rm[u], ra[u], rb[u]);
    }
    for (; r < r1; r += rpi) {
        const unsigned i = r * (unsigned)ld + ch * E;
        acc_raw(*(const uint4*)(dout + i), *(const uint4*)(mask + i), *(const uint4*)(ya + i), *(const uint4*)(yb + i));
    }
    const int rep = (int)(blockIdx.x % SCD_STAT_REPLICAS);
    // pass 1: sum dz (both layers) and layer a's sum dz*xhat; pass 2: layer b's
#pragma unroll
    for (int e = 0; e < E; ++e) {
        red[rsub * C + ch * E + e] = s[e];
        red[nt * E + rsub * C + ch * E + e] = qa[e];
    }
    __syncthreads();
    for (int c = tid; c < C; c += nt) {
        double ss = 0.0, qq = 0.0;
        for (int k = 0; k < rpi; ++k) {
            ss += red[k * C + c];
            qq += red[nt * E + k * C + c];
        }
        atomic_add_f64(stats_a + ((long)rep * 2 + 0) * ld + c, ss);
        atomic_add_f64(stats_a + ((long)rep * 2 + 1) * ld + c, qq);
        atomic_add_f64(stats_b + ((long)rep * 2 + 0) * ld + c, ss);
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; ++e) red[nt * E + rsub * C + ch * E + e] = qb[e];
    __syncthreads();
    for (int c = tid; c < C; c += nt) {
        double qq = 0.0;
        for (int k = 0; k < rpi; ++k) qq += red[nt * E + k * C + c];
        atomic_add_f64(stats_b + ((long)rep * 2 + 1) * ld + c, qq);
    }
}

template <typename T>
__global__ __launch_bounds__(256, BN_EW_WAVES) void bn_bwd_apply2_kernel(const T* dout, const T* mask, const T* ya, const T* yb,
                                                            const float* coef_a, const float* coef_b, int C,
                                                            unsigned nvec, T* dya, T* dyb) {
    constexpr int E = Vec16<T>::N;
    constexpr int U = BN_BWD_U;
    const unsigned cpr = (unsigned)C / E;
    const unsigned v0 = blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned stride = gridDim.x * blockDim.x;
    const int c0 = (int)(v0 % cpr) * E;
    extern __shared__ __attribute__((aligned(16))) float sp[];        // 6 x W floats (dynamic LDS): coef_a a, b, c, coef_b a, b, c
    int cb, W;
    chan_window(C, E, cb, W);
    {
        const float* src[6] = {coef_a, coef_a + C, coef_a + 2 * C, coef_b, coef_b + C, coef_b + 2 * C};
        stage_params(sp, src, 6, cb, W);
    }
    const int cl = c0 - cb;
    auto body = [&](size_t i, const uint4& rd, const uint4& rm, const uint4& ra, const uint4& rb) {
        float d[E], mk[E], va[E], vb[E], k0[E], k1[E], k2[E];
        Vec16<T>::load(&rd, d);
        Vec16<T>::load(&rm, mk);
        Vec16<T>::load(&ra, va);
        Vec16<T>::load(&rb, vb);
#pragma unroll
        for (int e = 0; e < E; ++e) d[e] = !(mk[e] > 0.f) ? 0.f : d[e];
        lds_params<E>(sp, cl, k0);
        lds_params<E>(sp, W + cl, k1);
        lds_params<E>(sp, 2 * W + cl, k2);
#pragma unroll
        for (int e = 0; e < E; ++e) va[e] = k0[e] * d[e] + k1[e] * va[e] + k2[e];
        lds_params<E>(sp, 3 * W + cl, k0);
        lds_params<E>(sp, 4 * W + cl, k1);
        lds_params<E>(sp, 5 * W + cl, k2);
#pragma unroll
        for (int e = 0; e < E; ++e) vb[e] = k0[e] * d[e] + k1[e] * vb[e] + k2[e];
        Vec16<T>::store(dya + i, va);
        Vec16<T>::store(dyb + i, vb);
    };
    unsigned v = v0;
    for (; v + (U - 1) * stride < nvec; v += U * stride) {
        uint4 rd[U], rm[U], ra[U], rb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = (size_t)(v + u * stride) * E;
            rd[u] = *(const uint4*)(dout + i);
            rm[u] = *(const uint4*)(mask + i);
            ra[u] = *(const uint4*)(ya + i);
            rb[u] = *(const uint4*)(yb + i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) body((size_t)(v + u * stride) * E, rd[u], rm[u], ra[u], rb[u]);
    }
    for (; v < nvec; v += stride) {
        const size_t i = (size_t)v * E;
        body(i, *(const uint4*)(dout + i), *(const uint4*)(mask + i), *(const uint4*)(ya + i), *(const uint4*)(yb + i));
    }
}

// elementwise BN kernels keep one channel chunk per thread: the grid stride (grid * 256 threads) must be a
// multiple of the chunks per row cpr, i.e. cpr divides 256 or is a multiple of it (grid a multiple of cpr/256)
inline bool ew_rows_ok(int cpr) { return cpr > 0 && (256 % cpr == 0 || cpr % 256 == 0); }
inline int ew_grid(int resident, long nvec, int cpr) {
    const long m = cpr > 256 ? cpr / 256 : 1;
    long g = std::min<long>(resident, (nvec + 255) / 256);
    g = std::max<long>(m, g / m * m);
    return (int)g;
}
inline int fin_blocks(int C) { return (C + 3) / 4; }   // 4 waves (channels) per 256-thread block
// dynamic LDS of an elementwise backward kernel staging nsrc per-channel arrays over its channel window (chan_window)
inline size_t ew_param_lds(int nsrc, int C, int E) { return (size_t)nsrc * std::min(C, 256 * E) * sizeof(float); }
constexpr size_t EW_LDS_MAX = 64 * 1024;
// resident blocks of `kernel` with `lds` bytes of dynamic LDS, cached per (kernel slot, window width)
template <int SLOT>
inline int ew_resident(const void* kernel, size_t lds) {
    static int cache[EW_LDS_MAX / 16 + 1] = {0};        // lds is a multiple of 16 B (E >= 4 floats per chunk)
    const size_t k = std::min<size_t>(lds / 16, EW_LDS_MAX / 16);
    if (!cache[k]) cache[k] = resident_grid(kernel, 256, lds);
    return cache[k];
}

SCD_KERNEL_NS_END
}  // namespace

extern "C" int scd_stats_collapse(double* stats, int nrep, int C, void* stream) {
    const int n = 2 * C;
    hipLaunchKernelGGL(stats_collapse_kernel, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, stats, nrep, n);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_stats_collapse_to(double* stats, int nrep, int C, double* out, void* stream) {
    const int n = 2 * C;
    if (!stats || !out || nrep < 1) return SCD_ERR_ARG;
    hipLaunchKernelGGL(stats_collapse_to_kernel, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, stats, nrep, n,
                       out);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_bn_finalize(double* stats, int nrep, int C, double count, const float* gamma,
                               const float* beta, float* running_mean, float* running_var, int64_t* num_batches,
                               float momentum, float eps, float* mean, float* invstd, float* scale, float* shift,
                               void* stream) {
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(fin_blocks(C)), dim3(256), 0, (hipStream_t)stream, stats, nrep, C,
                       count, gamma, beta, running_mean, running_var, num_batches, momentum, eps, mean, invstd, scale,
                       shift);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_bn_finalize_n(const scd_bn_fin_args* layers, int n, void* stream) {
    if (!layers || n < 1 || n > SCD_BN_FIN_MAX) return SCD_ERR_ARG;
    FinN f;
    memset(&f, 0, sizeof(f));
    f.n = n;
    int blocks = 0;
    for (int i = 0; i < n; ++i) {
        if (layers[i].C <= 0) return SCD_ERR_ARG;
        f.l[i] = layers[i];
        f.b0[i] = blocks;
        blocks += fin_blocks(layers[i].C);
    }
    f.b0[n] = blocks;
    hipLaunchKernelGGL(bn_finalize_n_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, f);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_bn_bwd_finalize_n(const scd_bn_bwd_fin_args* layers, int n, void* stream) {
    if (!layers || n < 1 || n > SCD_BN_FIN_MAX) return SCD_ERR_ARG;
    BwdFinN f;
    memset(&f, 0, sizeof(f));
    f.n = n;
    int blocks = 0;
    for (int i = 0; i < n; ++i) {
        if (layers[i].C <= 0 || !layers[i].stats || !layers[i].invstd || !layers[i].mean || !layers[i].coef)
            return SCD_ERR_ARG;
        f.l[i] = layers[i];
        f.b0[i] = blocks;
        blocks += fin_blocks(layers[i].C);
    }
    f.b0[n] = blocks;
    hipLaunchKernelGGL(bn_bwd_finalize_n_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, f);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_bn_apply(int dtype, const void* y, void* out, int C, long total, const float* scale,
                            const float* shift, const void* res, const float* rscale, const float* rshift, int relu,
                            void* stream) {
    SCD_F16_FWD(scd_bn_apply, y, out, C, total, scale, shift, res, rscale, rshift, relu, stream);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == SCD_DT_BF16) {
        if (C % 8 || !ew_rows_ok(C / 8)) return SCD_ERR_ARG;
        long nvec = total / 8;
        static const int g = resident_grid((const void*)bn_apply_kernel<h16>, 256);
        hipLaunchKernelGGL((bn_apply_kernel<h16>), dim3(ew_grid(g, nvec, C / 8)), dim3(256), 0, st, (const h16*)y,
                           (h16*)out, C, (unsigned)nvec, scale, shift, (const h16*)res, rscale, rshift, relu);
    } else if (dtype == SCD_DT_F32) {
        if (C % 4 || !ew_rows_ok(C / 4)) return SCD_ERR_ARG;
        long nvec = total / 4;
        static const int g = resident_grid((const void*)bn_apply_kernel<float>, 256);
        hipLaunchKernelGGL((bn_apply_kernel<float>), dim3(ew_grid(g, nvec, C / 4)), dim3(256), 0, st, (const float*)y,
                           (float*)out, C, (unsigned)nvec, scale, shift, (const float*)res, rscale, rshift, relu);
    } else {
        return SCD_ERR_ARG;
    }
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_bn_bwd_reduce(int dtype, const void* dout, const void* mask, const void* y, const float* relu_scale,
                                 const float* relu_shift, const float* mean,
                                 const float* invstd, int C, long total, double* stats, void* stream) {
    SCD_F16_FWD(scd_bn_bwd_reduce, dout, mask, y, relu_scale, relu_shift, mean, invstd, C, total, stats, stream);
    hipStream_t st = (hipStream_t)stream;
    const int E = dtype == SCD_DT_BF16 ? 8 : 4;
    if (C % E) return SCD_ERR_ARG;
    const long rows = total / C;
    const int cpr = C / E;
    // rows wider than 256 chunks run as channel slices of 256 chunks (ld = the full row)
    if (!ew_rows_ok(cpr) || total >= (1L << 31)) return SCD_ERR_ARG;
    const int scpr = std::min(cpr, 256), sC = scpr * E;
    // one round of resident blocks (at most), at least 8 rows per row lane
    const size_t lds = (size_t)4 * sC * sizeof(float);
    const long nb = dtype == SCD_DT_BF16 ? ew_resident<4>((const void*)bn_bwd_reduce_kernel<h16>, lds)
                                         : ew_resident<5>((const void*)bn_bwd_reduce_kernel<float>, lds);
    const long rpi = 256 / scpr;
    const long rpb = std::max<long>(8 * rpi, (rows + nb - 1) / nb + rpi - 1) / rpi * rpi;
    const int blocks = cdiv(rows, rpb);
    const int esz = dtype == SCD_DT_BF16 ? 2 : 4;
    for (int c0 = 0; c0 < C; c0 += sC) {
        const char* dz = (const char*)dout + (size_t)c0 * esz;
        const char* mk = mask ? (const char*)mask + (size_t)c0 * esz : nullptr;
        const char* yy = (const char*)y + (size_t)c0 * esz;
        const float* rs = relu_scale ? relu_scale + c0 : nullptr;
        const float* rh = relu_shift ? relu_shift + c0 : nullptr;
        if (dtype == SCD_DT_BF16)
            hipLaunchKernelGGL((bn_bwd_reduce_kernel<h16>), dim3(blocks), dim3(256), 4 * sC * 4, st, (const h16*)dz,
                               (const h16*)mk, (const h16*)yy, rs, rh, mean + c0, invstd + c0, sC, C,
                               (unsigned)rows, (unsigned)rpb, stats + c0);
        else if (dtype == SCD_DT_F32)
            hipLaunchKernelGGL((bn_bwd_reduce_kernel<float>), dim3(blocks), dim3(256), 4 * sC * 4, st, (const float*)dz,
                               (const float*)mk, (const float*)yy, rs, rh, mean + c0, invstd + c0, sC, C,
                               (unsigned)rows, (unsigned)rpb, stats + c0);
        else
            return SCD_ERR_ARG;
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return (int)e;
    }
    return 0;
}

extern "C" int scd_bn_bwd_reduce2(int dtype, const void* dout, const void* mask, const void* ya, const void* yb,
                                  const float* mean_a, const float* invstd_a, const float* mean_b,
                                  const float* invstd_b, int C, long total, double* stats_a, double* stats_b,
                                  void* stream) {
    SCD_F16_FWD(scd_bn_bwd_reduce2, dout, mask, ya, yb, mean_a, invstd_a, mean_b, invstd_b, C, total, stats_a, stats_b,
                stream);
    hipStream_t st = (hipStream_t)stream;
    const int E = dtype == SCD_DT_BF16 ? 8 : 4;
    if (!dout || !mask || !ya || !yb || C % E) return SCD_ERR_ARG;
    const long rows = total / C;
    const int cpr = C / E;
    if (!ew_rows_ok(cpr) || total >= (1L << 31)) return SCD_ERR_ARG;
    const int scpr = std::min(cpr, 256), sC = scpr * E;
    // the same row partition as scd_bn_bwd_reduce (per-thread partial sums identical to two separate passes)
    const size_t lds = (size_t)4 * sC * sizeof(float);
    const long nb = dtype == SCD_DT_BF16 ? ew_resident<4>((const void*)bn_bwd_reduce_kernel<h16>, lds)
                                         : ew_resident<5>((const void*)bn_bwd_reduce_kernel<float>, lds);
    const long rpi = 256 / scpr;
    const long rpb = std::max<long>(8 * rpi, (rows + nb - 1) / nb + rpi - 1) / rpi * rpi;
    const int blocks = cdiv(rows, rpb);
    const int esz = dtype == SCD_DT_BF16 ? 2 : 4;
    for (int c0 = 0; c0 < C; c0 += sC) {
        const size_t o = (size_t)c0 * esz;
        const char *d = (const char*)dout + o, *m = (const char*)mask + o, *a = (const char*)ya + o,
                   *b = (const char*)yb + o;
        if (dtype == SCD_DT_BF16)
            hipLaunchKernelGGL((bn_bwd_reduce2_kernel<h16>), dim3(blocks), dim3(256), 4 * sC * 4, st, (const h16*)d,
                               (const h16*)m, (const h16*)a, (const h16*)b, mean_a + c0, invstd_a + c0,
                               mean_b + c0, invstd_b + c0, sC, C, (unsigned)rows, (unsigned)rpb, stats_a + c0,
                               stats_b + c0);
        else if (dtype == SCD_DT_F32)
            hipLaunchKernelGGL((bn_bwd_reduce2_kernel<float>), dim3(blocks), dim3(256), 4 * sC * 4, st, (const float*)d,
                               (const float*)m, (const float*)a, (const float*)b, mean_a + c0, invstd_a + c0,
                               mean_b + c0, invstd_b + c0, sC, C, (unsigned)rows, (unsigned)rpb, stats_a + c0,
                               stats_b + c0);
        else
            return SCD_ERR_ARG;
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return (int)e;
    }
    return 0;
}

extern "C" int scd_bn_bwd_apply2(int dtype, const void* dout, const void* mask, const void* ya, const void* yb,
                                 const float* coef_a, const float* coef_b, int C, long total, void* dya, void* dyb,
                                 void* stream) {
    SCD_F16_FWD(scd_bn_bwd_apply2, dout, mask, ya, yb, coef_a, coef_b, C, total, dya, dyb, stream);
    hipStream_t st = (hipStream_t)stream;
    const int E = dtype == SCD_DT_BF16 ? 8 : 4;
    if (!dout || !mask || !ya || !yb || !dya || !dyb || C % E || !ew_rows_ok(C / E) || total / E >= (1L << 32))
        return SCD_ERR_ARG;
    const long nvec = total / E;
    if (dtype == SCD_DT_BF16) {
        const size_t lds = ew_param_lds(6, C, 8);
        if (lds > EW_LDS_MAX) return SCD_ERR_ARG;
        const int g = ew_resident<0>((const void*)bn_bwd_apply2_kernel<h16>, lds);
        hipLaunchKernelGGL((bn_bwd_apply2_kernel<h16>), dim3(ew_grid(g, nvec, C / 8)), dim3(256), lds, st,
                           (const h16*)dout, (const h16*)mask, (const h16*)ya, (const h16*)yb, coef_a,
                           coef_b, C, (unsigned)nvec, (h16*)dya, (h16*)dyb);
    } else if (dtype == SCD_DT_F32) {
        const size_t lds = ew_param_lds(6, C, 4);
        if (lds > EW_LDS_MAX) return SCD_ERR_ARG;
        const int g = ew_resident<1>((const void*)bn_bwd_apply2_kernel<float>, lds);
        hipLaunchKernelGGL((bn_bwd_apply2_kernel<float>), dim3(ew_grid(g, nvec, C / 4)), dim3(256), lds, st,
                           (const float*)dout, (const float*)mask, (const float*)ya, (const float*)yb, coef_a, coef_b,
                           C, (unsigned)nvec, (float*)dya, (float*)dyb);
    } else {
        return SCD_ERR_ARG;
    }
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_bn_bwd_finalize(double* stats, int nrep, int C, double count, const float* gamma,
                                   const float* mean, const float* invstd, float* dgamma, float* dbeta, float gscale,
                                   float* coef, void* stream) {
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(fin_blocks(C)), dim3(256), 0, (hipStream_t)stream, stats, nrep, C,
                       count, gamma, mean, invstd, dgamma, dbeta, gscale, coef);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_bn_bwd_apply(int dtype, const void* dout, const void* mask, const void* y, const float* relu_scale,
                                const float* relu_shift, const float* coef, int C, long total, void* dy, void* dz,
                                void* stream) {
    SCD_F16_FWD(scd_bn_bwd_apply, dout, mask, y, relu_scale, relu_shift, coef, C, total, dy, dz, stream);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == SCD_DT_BF16) {
        if (C % 8 || !ew_rows_ok(C / 8)) return SCD_ERR_ARG;
        long nvec = total / 8;
        const size_t lds = ew_param_lds(5, C, 8);
        if (lds > EW_LDS_MAX) return SCD_ERR_ARG;
        const int g = ew_resident<2>((const void*)bn_bwd_apply_kernel<h16>, lds);
        hipLaunchKernelGGL((bn_bwd_apply_kernel<h16>), dim3(ew_grid(g, nvec, C / 8)), dim3(256), lds, st,
                           (const h16*)dout, (const h16*)mask, (const h16*)y, relu_scale, relu_shift, coef, C,
                           (unsigned)nvec, (h16*)dy, (h16*)dz);
    } else if (dtype == SCD_DT_F32) {
        if (C % 4 || !ew_rows_ok(C / 4)) return SCD_ERR_ARG;
        long nvec = total / 4;
        const size_t lds = ew_param_lds(5, C, 4);
        if (lds > EW_LDS_MAX) return SCD_ERR_ARG;
        const int g = ew_resident<3>((const void*)bn_bwd_apply_kernel<float>, lds);
        hipLaunchKernelGGL((bn_bwd_apply_kernel<float>), dim3(ew_grid(g, nvec, C / 4)), dim3(256), lds, st, (const float*)dout,
                           (const float*)mask, (const float*)y, relu_scale, relu_shift, coef, C, (unsigned)nvec, (float*)dy,
                           (float*)dz);
    } else {
        return SCD_ERR_ARG;
    }
    SCD_RETURN_LAUNCH();
}
