// Layer glue kernels: weight packing, stem im2col, stem BN+ReLU+MaxPool (fwd/bwd),
// fused CenterNet head tails (1x1 convs), Adam.  All HBM-bound; 16-B vectorised where the
// layout allows.
#include <algorithm>

#include "scd_common.h"

namespace {
SCD_KERNEL_NS_BEGIN

// ---------------------------------------------------------------- weight packing
// mode 3 (a 3x3 stride-2 conv's input gradient as a 2x2-tap forward GEMM with the four output phases as channels,
// scd_conv_dgrad_s2): out[(2 rh + rw) B + b][(2 dq + dp) A + a] = w[a][b][rh + 1 - 2 dq][rw + 1 - 2 dp], 0 where the
// tap index leaves 0..2
__device__ __forceinline__ float s2_phase_weight(const float* w, unsigned A, unsigned B, unsigned r, unsigned k) {
    const unsigned ph = r / B, b = r - ph * B, t = k / A, a = k - t * A;
    const int kr = (int)(ph >> 1) + 1 - 2 * (int)(t >> 1), ks = (int)(ph & 1) + 1 - 2 * (int)(t & 1);
    return (kr >= 0 && kr < 3 && ks >= 0 && ks < 3) ? w[(a * B + b) * 9 + kr * 3 + ks] : 0.f;
}

template <typename T>
__global__ void pack_weight_kernel(const float* w, T* out, int A, int B, int Tt, int mode, int ldp, int row_off) {
    if (mode == 3) {
        const unsigned total = 4u * B * ldp;
        for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
            const unsigned r = i / (unsigned)ldp, k = i - r * (unsigned)ldp;
            out[(long)(row_off + r) * ldp + k] = from_f<T>(k < 4u * A ? s2_phase_weight(w, A, B, r, k) : 0.f);
        }
        return;
    }
    const int rows = mode == 0 ? A : mode == 1 ? B : Tt * B;
    const unsigned total = (unsigned)rows * ldp;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const int r = (int)(i / (unsigned)ldp);
        const int k = (int)(i - (unsigned)r * ldp);
        float v = 0.f;
        if (mode == 0) {        // out[a][t*B+b] = w[a][b][t]
            const int t = k / B, b = k - (k / B) * B;
            if (t < Tt) v = w[((long)r * B + b) * Tt + t];
        } else if (mode == 1) { // out[b][t*A+a] = w[a][b][t]
            const int t = k / A, a = k - (k / A) * A;
            if (t < Tt) v = w[((long)a * B + r) * Tt + t];
        } else {                // out[t*B+b][a] = w[a][b][t]: columns k >= A belong to other operands (row_off = a offset)
            if (k >= A) continue;
            const int t = r / B, b = r - (r / B) * B;
            out[(long)r * ldp + row_off + k] = from_f<T>(w[((long)k * B + b) * Tt + t]);
            continue;
        }
        out[(long)(row_off + r) * ldp + k] = from_f<T>(v);
    }
}

// ---------------------------------------------------------------- batched pack (one launch per step)
// Every conv/deconv weight operand of a training step in one launch.  Descriptor starts are multiples of
// PACK_UNIT elements (host side), so each workgroup handles one unit of ONE descriptor, found by a
// workgroup-uniform binary search (scalar loads).
constexpr int PACK_UNIT = 4096;

__global__ __launch_bounds__(256) void pack_weights_batched_kernel(const scd_pack_desc* __restrict__ d, int n, int bf16) {
    const long e0 = (long)blockIdx.x * PACK_UNIT;
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (d[mid].start <= e0) lo = mid; else hi = mid - 1;
    }
    const scd_pack_desc q = d[lo];
    if (q.mode == 1) {
        // [B][taps][A] (input-gradient operand): a transpose of every tap's A x B plane.  Unit u of the
        // descriptor is one tile of 64 a x BB b (BB*T <= 64 elements of a contiguous input row segment): the
        // tile's rows are read coalesced into LDS and written as runs of <= 64 consecutive a per (b, tap).
        __shared__ float tile[64 * 65];
        const int T = q.T, BB = max(1, 64 / T);
        const int nbb = (q.B + BB - 1) / BB;
        const int u = (int)((e0 - q.start) / PACK_UNIT);
        const int ta = u / nbb, tb = u - (u / nbb) * nbb;
        const int a0 = ta * 64, b0 = tb * BB;
        if (a0 >= q.A) return;
        const int na = min(64, q.A - a0), nb = min(BB, q.B - b0);
        const int rowl = nb * T, pitch = rowl | 1;         // odd pitch: the column reads below hit distinct banks
        for (int i = threadIdx.x; i < na * rowl; i += 256) {
            const int a = i / rowl, k = i - a * rowl;
            tile[a * pitch + k] = q.w[((unsigned)(a0 + a) * q.B + b0) * T + k];
        }
        __syncthreads();
        if (bf16 && na % 8 == 0 && q.ldp % 8 == 0 && q.a_tot % 8 == 0 && q.a_off % 8 == 0) {
            // 8 consecutive a per thread: one 16-B store instead of eight 2-byte ones
            const int na8 = na / 8;
            for (int i = threadIdx.x; i < na8 * rowl; i += 256) {
                const int bt = i / na8, a = (i - bt * na8) * 8;
                const int b = bt / T, t = bt - b * T;
                typedef __attribute__((ext_vector_type(8))) h16 bf8;
                bf8 v;
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = (h16)tile[(a + e) * pitch + b * T + t];
                const unsigned o = (unsigned)(b0 + b) * q.ldp + t * q.a_tot + q.a_off + a0 + a;
                *(bf8*)((h16*)q.out + o) = v;
            }
            return;
        }
        for (int i = threadIdx.x; i < na * rowl; i += 256) {
            const int bt = i / na, a = i - bt * na;
            const int b = bt / T, t = bt - b * T;
            const float v = tile[a * pitch + b * T + t];
            const unsigned o = (unsigned)(b0 + b) * q.ldp + t * q.a_tot + q.a_off + a0 + a;
            if (bf16) ((h16*)q.out)[o] = (h16)v;
            else ((float*)q.out)[o] = v;
        }
        return;
    }
    // 32-bit index math (a descriptor holds < 2^31 elements; 64-bit divides dominated this kernel)
    if (q.mode == 3) {                // out[row_off + r][k], 4B x ldp elements (ldp = 4A)
        const unsigned count3 = 4u * q.B * q.ldp, base3 = (unsigned)(e0 - q.start);
#pragma unroll 4
        for (int j = 0; j < PACK_UNIT / 256; ++j) {
            const unsigned i = base3 + threadIdx.x + 256 * j;
            if (i >= count3) break;
            const unsigned r = i / (unsigned)q.ldp, k = i - r * (unsigned)q.ldp;
            const float v = s2_phase_weight(q.w, q.A, q.B, r, k);
            const unsigned o = (q.row_off + r) * (unsigned)q.ldp + k;
            if (bf16) ((h16*)q.out)[o] = (h16)v;
            else ((float*)q.out)[o] = v;
        }
        return;
    }
    const unsigned count = q.mode == 0 ? (unsigned)q.A * q.ldp : (unsigned)q.B * q.T * q.A;   // mode 1 / 2: B x T x A
    const unsigned base = (unsigned)(e0 - q.start);
    const unsigned ldp = q.ldp, B = q.B, Tt = q.T, A = q.A, TA = Tt * A;
    if (q.mode == 0 && bf16 && ldp % 8 == 0 && B % 8 == 0 && q.row_off >= 0) {
        // 8 consecutive k of one row share their tap (B % 8 == 0): one 16-B store per thread and chunk (staging the
        // source rows through LDS for coalesced reads measured slower: 62 vs 48 us per step)
        typedef __attribute__((ext_vector_type(8))) h16 bf8;
#pragma unroll
        for (int j = 0; j < PACK_UNIT / 256 / 8; ++j) {
            const unsigned i = base + 8 * (threadIdx.x + 256 * j);
            if (i >= count) break;
            const unsigned r = i / ldp, k = i - r * ldp;
            const unsigned t = k / B, b = k - t * B;
            bf8 v;
            // unconditional loads (the padding columns t >= T read tap T-1 and are zeroed): a load under the test
            // would be a branch the compiler waits on
            const float* src = q.w + (r * B + b) * Tt + min(t, Tt - 1);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float x = src[e * Tt];
                v[e] = (h16)(t < Tt ? x : 0.f);
            }
            *(bf8*)((h16*)q.out + (q.row_off + r) * ldp + k) = v;
        }
        return;
    }
#pragma unroll 4
    for (int j = 0; j < PACK_UNIT / 256; ++j) {
        const unsigned i = base + threadIdx.x + 256 * j;
        if (i >= count) break;
        float v;
        unsigned o;
        if (q.mode == 0) {            // out[row_off + a][t*B + b] = w[a][b][t]   (A x ldp elements, padding zeroed)
            const unsigned r = i / ldp, k = i - r * ldp;
            const unsigned t = k / B, b = k - t * B;
            v = t < Tt ? q.w[(r * B + b) * Tt + t] : 0.f;
            o = (q.row_off + r) * ldp + k;
        } else if (q.mode == 1) {     // out[b][t*a_tot + a_off + a] = w[a][b][t]  (B x T x A elements)
            const unsigned r = i / TA, rem = i - r * TA;
            const unsigned t = rem / A, a = rem - t * A;
            v = q.w[(a * B + r) * Tt + t];
            o = r * ldp + t * q.a_tot + q.a_off + a;
        } else {                      // out[t*B + b][a_off + a] = w[a][b][t]  (T x B x A elements, ldp = a_tot)
            const unsigned BA = B * A;
            const unsigned t = i / BA, rem = i - t * BA;
            const unsigned b = rem / A, a = rem - b * A;
            v = q.w[(a * B + b) * Tt + t];
            o = (t * B + b) * ldp + q.a_off + a;
        }
        if (bf16) ((h16*)q.out)[o] = (h16)v;
        else ((float*)q.out)[o] = v;
    }
}

extern "C" int scd_pack_weights_batched(int dtype, const scd_pack_desc* descs, int n, long total, void* stream) {
    SCD_F16_FWD(scd_pack_weights_batched, descs, n, total, stream);
    if (n < 1 || total < 1 || total >= (1L << 31) || total % PACK_UNIT || (dtype != SCD_DT_BF16 && dtype != SCD_DT_F32)) return SCD_ERR_ARG;
    hipLaunchKernelGGL(pack_weights_batched_kernel, dim3((unsigned)(total / PACK_UNIT)), dim3(256), 0, (hipStream_t)stream,
                       descs, n, dtype == SCD_DT_BF16 ? 1 : 0);
    SCD_RETURN_LAUNCH();
}

// ---------------------------------------------------------------- stem im2col
template <typename T>
__global__ void im2col_stem_kernel(const float* x, T* cols, int N, int H, int W, int Ho, int Wo, int kh, int kw,
                                   int stride, int pad, int Kpad) {
    constexpr int E = Vec16<T>::N;
    const unsigned cpp = Kpad / E;
    const unsigned total = (unsigned)N * Ho * Wo * cpp;
    const unsigned HoWo = (unsigned)Ho * Wo;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const unsigned pix = i / cpp;
        const int ch = (int)(i - pix * cpp);
        const int n = (int)(pix / HoWo);
        const int rem = (int)(pix - (unsigned)n * HoWo);
        const int oh = rem / Wo, ow = rem - (rem / Wo) * Wo;
        float v[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int k = ch * E + e;
            float val = 0.f;
            if (k < kh * kw) {
                const int r = k / kw, s = k - (k / kw) * kw;
                const int ih = oh * stride - pad + r, iw = ow * stride - pad + s;
                if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) val = x[((long)n * H + ih) * W + iw];
            }
            v[e] = val;
        }
        Vec16<T>::store(cols + (size_t)pix * Kpad + ch * E, v);
    }
}

// ---------------------------------------------------------------- stem BN+ReLU+MaxPool(3,2,1)
// One thread = one 16-B channel chunk of SPR consecutive pooled rows at one pooled column: it loads the 2 SPR + 1 conv
// rows x 3 conv columns of those windows at once (clamped addresses; taps outside the image never win).  Conv row
// 2 oh + 1 is the bottom of window oh and the top of window oh + 1, so one row per thread fetches 1.5x the conv output
// (PMC, round 4) and four rows per thread 9/8 -- but in the step the conv output was just written and is read back
// from the Infinity Cache, and the four-row build (203 VGPRs, 2 waves per SIMD) measured 99 us against 82 us for one
// row per thread (round 5, tools/gpu_abn.sh): one row per thread stays.
// workgroups of 256 per CU the pool is compiled for (registers: the window loads in flight per thread)
#ifndef STEM_POOL_OCC
#define STEM_POOL_OCC 4
#endif
#ifndef STEM_SPR
#define STEM_SPR 1
#endif
constexpr int SPR = STEM_SPR;                       // pooled rows per thread
template <typename T>
__global__ __launch_bounds__(256, STEM_POOL_OCC) void stem_pool_fwd_kernel(const T* y, const float* scale, const float* shift, T* out, uint8_t* argmax,
                                     int N, int H, int W, int C, int Ho, int Wo) {
    constexpr int E = Vec16<T>::N;
    constexpr int NR = 2 * SPR + 1;
    const unsigned cpp = C / E;
    const unsigned G = (unsigned)(Ho + SPR - 1) / SPR;
    const unsigned GW = G * (unsigned)Wo;
    const unsigned total = (unsigned)N * GW * cpp;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const unsigned item = i / cpp;
        const int ch = (int)(i - item * cpp);
        const int n = (int)(item / GW);
        const unsigned rem = item - (unsigned)n * GW;
        const int g = (int)(rem / (unsigned)Wo), ow = (int)(rem - (unsigned)g * Wo);
        const int oh0 = g * SPR;
        float sc[E], sh[E];
#pragma unroll
        for (int e = 0; e < E; ++e) { sc[e] = scale[ch * E + e]; sh[e] = shift[ch * E + e]; }
        uint4 raw[NR][3];
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const int h = min(max(2 * oh0 - 1 + r, 0), H - 1), w = min(max(2 * ow - 1 + c, 0), W - 1);
                raw[r][c] = *(const uint4*)(y + (((long)n * H + h) * W + w) * C + ch * E);
            }
#pragma unroll
        for (int j = 0; j < SPR; ++j) {
            const int oh = oh0 + j;
            float best[E];
            int arg[E];
#pragma unroll
            for (int e = 0; e < E; ++e) { best[e] = -INFINITY; arg[e] = 0; }
            // the window in window order (first maximum wins, as before)
#pragma unroll
            for (int d = 0; d < 9; ++d) {
                const bool in = (unsigned)(2 * oh - 1 + d / 3) < (unsigned)H && (unsigned)(2 * ow - 1 + d % 3) < (unsigned)W;
                float v[E];
                Vec16<T>::load(&raw[2 * j + d / 3][d % 3], v);
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const float z = in ? fmaxf(v[e] * sc[e] + sh[e], 0.f) : -INFINITY;
                    if (z > best[e]) { best[e] = z; arg[e] = d; }
                }
            }
            if (oh < Ho) {
                const size_t pix = ((size_t)n * Ho + oh) * Wo + ow;
                Vec16<T>::store(out + pix * C + ch * E, best);
                // the E argmax bytes of this chunk in one store
                unsigned lo = 0, hi = 0;
#pragma unroll
                for (int e = 0; e < E && e < 4; ++e) lo |= (unsigned)arg[e] << (8 * e);
#pragma unroll
                for (int e = 4; e < E; ++e) hi |= (unsigned)arg[e] << (8 * (e - 4));
                if constexpr (E == 8) *(uint2*)(argmax + pix * C + ch * E) = make_uint2(lo, hi);
                else *(unsigned*)(argmax + pix * C + ch * E) = lo;
            }
        }
    }
}

template <typename T>
__global__ void stem_pool_bwd_kernel(const T* dout, const uint8_t* argmax, const T* y, const float* scale,
                                     const float* shift, T* dz, int N, int H, int W, int C, int Ho, int Wo) {
    constexpr int E = Vec16<T>::N;
    const unsigned cpp = C / E;
    const unsigned total = (unsigned)N * H * W * cpp;
    const unsigned HW = (unsigned)H * W;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const size_t pix = i / cpp;
        const int ch = (int)(i - (unsigned)pix * cpp);
        const int n = (int)((unsigned)pix / HW);
        const int rem = (int)((unsigned)pix - (unsigned)n * HW);
        const int h = rem / W, w = rem - (rem / W) * W;
        float acc[E];
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] = 0.f;
        const int oh0 = h / 2, oh1 = min(Ho - 1, (h + 1) / 2);
        const int ow0 = w / 2, ow1 = min(Wo - 1, (w + 1) / 2);
        for (int oh = oh0; oh <= oh1; ++oh) {
            const int di = h - (2 * oh - 1);
            if (di < 0 || di > 2) continue;
            for (int ow = ow0; ow <= ow1; ++ow) {
                const int dj = w - (2 * ow - 1);
                if (dj < 0 || dj > 2) continue;
                const long o = (((long)n * Ho + oh) * Wo + ow) * C + ch * E;
                float d[E];
                Vec16<T>::load(dout + o, d);
#pragma unroll
                for (int e = 0; e < E; ++e)
                    if (argmax[o + e] == di * 3 + dj) acc[e] += d[e];
            }
        }
        float v[E];
        Vec16<T>::load(y + pix * C + ch * E, v);
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const float z = v[e] * scale[ch * E + e] + shift[ch * E + e];
            acc[e] = z > 0.f ? acc[e] : 0.f;
        }
        Vec16<T>::store(dz + pix * C + ch * E, acc);
    }
}

// Stem MaxPool backward + ReLU mask (as stem_pool_bwd_kernel) fused with the stem BN backward reduction:
// the same pass accumulates sum dz and sum dz*(y-mean)*invstd per channel (fp64 replica slots), so the
// separate reduce pass over dz and y is gone.  The grid stride is a multiple of the chunks per pixel, so a
// thread always owns the same 8 (bf16) channels.
template <typename T>
__global__ __launch_bounds__(256) void stem_pool_bwd_bn_kernel(const T* dout, const uint8_t* argmax, const T* y,
                                                               const float* scale, const float* shift, const float* mean,
                                                               const float* invstd, T* dz, double* stats, int N, int H,
                                                               int W, int C, int Ho, int Wo) {
    constexpr int E = Vec16<T>::N;
    const unsigned cpp = C / E;
    const unsigned total = (unsigned)N * H * W * cpp;
    const unsigned HW = (unsigned)H * W;
    const int ch = (int)(threadIdx.x % cpp);
    float sc[E], sh[E], mu[E], is[E], s1[E], s2[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        sc[e] = scale[ch * E + e]; sh[e] = shift[ch * E + e]; mu[e] = mean[ch * E + e]; is[e] = invstd[ch * E + e];
        s1[e] = 0.f; s2[e] = 0.f;
    }
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const size_t pix = i / cpp;
        const int n = (int)((unsigned)pix / HW);
        const int rem = (int)((unsigned)pix - (unsigned)n * HW);
        const int h = rem / W, w = rem - (rem / W) * W;
        float acc[E];
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] = 0.f;
        const int oh0 = h / 2, oh1 = min(Ho - 1, (h + 1) / 2);
        const int ow0 = w / 2, ow1 = min(Wo - 1, (w + 1) / 2);
        for (int oh = oh0; oh <= oh1; ++oh) {
            const int di = h - (2 * oh - 1);
            if (di < 0 || di > 2) continue;
            for (int ow = ow0; ow <= ow1; ++ow) {
                const int dj = w - (2 * ow - 1);
                if (dj < 0 || dj > 2) continue;
                const long o = (((long)n * Ho + oh) * Wo + ow) * C + ch * E;
                float d[E];
                Vec16<T>::load(dout + o, d);
                uint8_t am[E];
                if constexpr (E == 8) *(uint2*)am = *(const uint2*)(argmax + o);
                else *(uint32_t*)am = *(const uint32_t*)(argmax + o);
                const int sel = di * 3 + dj;
#pragma unroll
                for (int e = 0; e < E; ++e)
                    if (am[e] == sel) acc[e] += d[e];
            }
        }
        float v[E];
        Vec16<T>::load(y + pix * C + ch * E, v);
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const float z = v[e] * sc[e] + sh[e];
            acc[e] = z > 0.f ? acc[e] : 0.f;
        }
        Vec16<T>::store(dz + pix * C + ch * E, acc);
        // BN backward sums of the value the apply pass will see (the stored, rounded dz)
        float r[E];
#pragma unroll
        for (int e = 0; e < E; ++e) r[e] = to_f<T>(from_f<T>(acc[e]));
#pragma unroll
        for (int e = 0; e < E; ++e) {
            s1[e] += r[e];
            s2[e] += r[e] * (v[e] - mu[e]) * is[e];
        }
    }
    __shared__ float red[2][256][E + 1];
#pragma unroll
    for (int e = 0; e < E; ++e) { red[0][threadIdx.x][e] = s1[e]; red[1][threadIdx.x][e] = s2[e]; }
    __syncthreads();
    // channel c = ch*E + e is held by threads t with t % cpp == ch
    for (int k = threadIdx.x; k < 2 * C; k += blockDim.x) {
        const int stat = k / C, c = k - (k / C) * C;
        const int cc = c / E, e = c - (c / E) * E;
        double a = 0.0;
        for (int t = cc; t < (int)blockDim.x; t += cpp) a += red[stat][t][e];
        atomic_add_f64(stats + ((long)(blockIdx.x % SCD_STAT_REPLICAS) * 2 + stat) * C + c, a);
    }
}

// The same pass for even inputs (H = 2 Ho, W = 2 Wo), one thread per 2x2 input block and 16-B channel chunk:
// input rows {2oh, 2oh+1} x cols {2ow, 2ow+1} are covered only by pooled outputs (oh..oh+1, ow..ow+1), so the
// thread issues its 4 gradient vectors, 4 argmax words and 4 activation vectors together (no data-dependent
// branches around loads) and each pooled gradient is read ~once per 4 inputs.  Window position of input
// (2oh+a, 2ow+b) in output (oh+i, ow+j): di = a - 2i + 1, dj = b - 2j + 1; sums run over outputs in
// (oh, ow) order as the generic kernel's loops do.
template <typename T>
__global__ __launch_bounds__(256) void stem_pool_bwd_bn_2x2_kernel(const T* dout, const uint8_t* argmax, const T* y,
                                                                   const float* scale, const float* shift,
                                                                   const float* mean, const float* invstd, T* dz,
                                                                   double* stats, int N, int C, int Ho, int Wo) {
    constexpr int E = Vec16<T>::N;
    const unsigned cpp = C / E;
    const unsigned total = (unsigned)N * Ho * Wo * cpp;
    const unsigned HWo = (unsigned)Ho * Wo;
    const int W = 2 * Wo;
    const int ch = (int)(threadIdx.x % cpp);
    float sc[E], sh[E], mu[E], is[E], s1[E], s2[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        sc[e] = scale[ch * E + e]; sh[e] = shift[ch * E + e]; mu[e] = mean[ch * E + e]; is[e] = invstd[ch * E + e];
        s1[e] = 0.f; s2[e] = 0.f;
    }
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const unsigned blk = i / cpp;
        const unsigned n = blk / HWo;
        const unsigned rem = blk - n * HWo;
        const int oh = (int)(rem / Wo), ow = (int)(rem - (rem / Wo) * Wo);
        const bool okh = oh + 1 < Ho, okw = ow + 1 < Wo;
        // pooled outputs O[i][j] = (oh+i, ow+j); out-of-range ones read O[0][0] and are ignored
        float d[2][2][E];
        uint8_t am[2][2][E];
        float v[2][2][E];
#pragma unroll
        for (int oi = 0; oi < 2; ++oi)
#pragma unroll
            for (int oj = 0; oj < 2; ++oj) {
                const bool ok = (oi == 0 || okh) && (oj == 0 || okw);
                const unsigned o = ((n * Ho + oh + (ok ? oi : 0)) * Wo + ow + (ok ? oj : 0)) * C + ch * E;
                Vec16<T>::load(dout + o, d[oi][oj]);
                if constexpr (E == 8) *(uint2*)am[oi][oj] = *(const uint2*)(argmax + o);
                else *(uint32_t*)am[oi][oj] = *(const uint32_t*)(argmax + o);
                if (!ok)
#pragma unroll
                    for (int e = 0; e < E; ++e) am[oi][oj][e] = 0xff;
            }
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
                Vec16<T>::load(y + ((n * (2 * Ho) + 2 * oh + a) * W + 2 * ow + b) * (unsigned)C + ch * E, v[a][b]);
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                float acc[E];
#pragma unroll
                for (int e = 0; e < E; ++e) acc[e] = 0.f;
#pragma unroll
                for (int oi = 0; oi < 2; ++oi)
#pragma unroll
                    for (int oj = 0; oj < 2; ++oj) {
                        if (oi > a || oj > b) continue;                // (a=0 -> only i=0; a=1 -> i=0,1)
                        const int sel = (a - 2 * oi + 1) * 3 + (b - 2 * oj + 1);
#pragma unroll
                        for (int e = 0; e < E; ++e)
                            if (am[oi][oj][e] == sel) acc[e] += d[oi][oj][e];
                    }
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const float z = v[a][b][e] * sc[e] + sh[e];
                    acc[e] = z > 0.f ? acc[e] : 0.f;
                }
                Vec16<T>::store(dz + ((n * (2 * Ho) + 2 * oh + a) * W + 2 * ow + b) * (unsigned)C + ch * E, acc);
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const float r = to_f<T>(from_f<T>(acc[e]));
                    s1[e] += r;
                    s2[e] += r * (v[a][b][e] - mu[e]) * is[e];
                }
            }
    }
    __shared__ float red[2][256][E + 1];
#pragma unroll
    for (int e = 0; e < E; ++e) { red[0][threadIdx.x][e] = s1[e]; red[1][threadIdx.x][e] = s2[e]; }
    __syncthreads();
    for (int k = threadIdx.x; k < 2 * C; k += blockDim.x) {
        const int stat = k / C, c = k - (k / C) * C;
        const int cc = c / E, e = c - (c / E) * E;
        double a = 0.0;
        for (int t = cc; t < (int)blockDim.x; t += cpp) a += red[stat][t][e];
        atomic_add_f64(stats + ((long)(blockIdx.x % SCD_STAT_REPLICAS) * 2 + stat) * C + c, a);
    }
}

// ---------------------------------------------------------------- CenterNet head tails
struct HeadsDesc {
    int nh, Hd, od[4], orow[4], nout;
    int nd;                 // the tail backward covers heads [0, nd) (the rest: scd_heads_sparse_bwd)
    int hstride, dstride;   // row strides (elements) of the hidden activation and of the written dhid
    const float* w1[4];
    const float* b1[4];
    const float* dout[4];
    float* out[4];
    const float* pk;        // packed head-output gradients [pixel][nh][4] (scd_heads_bwd_packed), or null
};

// the head-output gradients (NCHW fp32, od[h] channels each) repacked pixel-major, 4 floats per head (zero padded)
// and multiplied by `scale` (the fp16 loss scale): the tail backward then reads one 16-B vector per pixel and head
__global__ void heads_pack_kernel(int N, int HW, HeadsDesc d, float scale, float* pk) {
    const long P = (long)N * HW;
    for (long px = blockIdx.x * (long)blockDim.x + threadIdx.x; px < P; px += (long)gridDim.x * blockDim.x) {
        const long n = px / HW, q = px - n * HW;
        for (int h = 0; h < d.nd; ++h) {
            float v[4];
#pragma unroll
            for (int o = 0; o < 4; ++o) v[o] = o < d.od[h] ? d.dout[h][(n * d.od[h] + o) * HW + q] * scale : 0.f;
            *(float4*)(pk + (px * d.nd + h) * 4) = make_float4(v[0], v[1], v[2], v[3]);
        }
    }
}

// thread = (pixel, 16-B channel chunk): coalesced hidden reads; per-head partial dot products
// reduced over the head's Hd/E chunk-lanes with xor-shuffles (aligned groups: Hd/E | 64).
template <typename T>
__global__ void heads_fwd_kernel(const T* hid, int N, int HW, HeadsDesc d) {
    constexpr int E = Vec16<T>::N;
    const int cph = d.Hd / E;                       // chunk-lanes per head (power of two <= 64)
    const unsigned cpp = (unsigned)(d.nh * cph);     // chunks per pixel
    const unsigned total = (unsigned)N * HW * cpp;
    // grid-stride loop must keep whole waves inside the range for the shuffles
    for (unsigned base = blockIdx.x * blockDim.x; base < total; base += gridDim.x * blockDim.x) {
        const unsigned i = base + threadIdx.x;
        const bool ok = i < total;
        const unsigned px = ok ? i / cpp : 0;
        const int ch = ok ? (int)(i - px * cpp) : 0;
        const int h = ch / cph;
        const int cl = (ch - h * cph) * E;
        float v[E];
        if (ok) Vec16<T>::load(hid + (size_t)i * E, v);
        else
#pragma unroll
            for (int e = 0; e < E; ++e) v[e] = 0.f;
        float acc[4];
#pragma unroll
        for (int o = 0; o < 4; ++o) {
            float a = 0.f;
            if (ok && o < d.od[h]) {
                const float* w = d.w1[h] + o * d.Hd + cl;
#pragma unroll
                for (int e = 0; e < E; ++e) a += v[e] * w[e];
            }
            for (int m = cph >> 1; m > 0; m >>= 1) a += __shfl_xor(a, m, 64);
            acc[o] = a;
        }
        if (ok && (ch - h * cph) == 0) {
            const int n = (int)(px / (unsigned)HW);
            const int q = (int)(px - (unsigned)n * HW);
            for (int o = 0; o < d.od[h]; ++o)
                d.out[h][((size_t)n * d.od[h] + o) * HW + q] = acc[o] + d.b1[h][o];
        }
    }
}

// fused backward of the head tails: dhid = relu'(hid) * (W1^T dout) and, in the same pass,
// dW1 = sum_px dout x hid, db1 = sum_px dout, db0 (3x3 conv bias) = sum_px dhid.
// Block = PXB pixels, blockDim = G pixel-lanes x cpp chunk-lanes; each thread streams its chunk over
// every G-th pixel, 4 pixels per step with all loads issued before use; block partials are folded in
// LDS by all threads and added to fp64 replicas (SCD_STAT_REPLICAS).
template <typename T, int U, bool PK = false>
__global__ __launch_bounds__(512) void heads_bwd_kernel(const T* hid, int N, int HW, HeadsDesc d, T* dhid,
                                                        double* acc, int accsz, int PXB) {
    constexpr int E = Vec16<T>::N;
    constexpr int NA = 4 * E + E + 4;               // dW1 partials, db0 partials, db1 partials
    const int cph = d.Hd / E;
    const int cpp = d.nd * cph;
    const int G = blockDim.x / cpp;
    const int tid = threadIdx.x;
    const int c = tid % cpp;
    const int g = tid / cpp;
    const int h = c / cph;
    const int cl = (c - h * cph) * E;
    const int ct = h * d.Hd + cl;                   // channel of this chunk in the hidden tensor
    const int od = d.od[h];
    const float* dout = d.dout[h];
    float w[4][E];
#pragma unroll
    for (int o = 0; o < 4; ++o)
#pragma unroll
        for (int e = 0; e < E; ++e) w[o][e] = o < od ? d.w1[h][o * d.Hd + cl + e] : 0.f;
    float a[NA];
#pragma unroll
    for (int k = 0; k < NA; ++k) a[k] = 0.f;
    const unsigned P = (unsigned)N * HW;
    const unsigned p0 = blockIdx.x * (unsigned)PXB;
    const unsigned p1 = min(P, p0 + PXB);
    const unsigned Ctot = d.hstride, Dtot = d.dstride;
    auto body = [&](unsigned px, const float* gd, float* v) {
        float r[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const float s = gd[0] * w[0][e] + gd[1] * w[1][e] + gd[2] * w[2][e] + gd[3] * w[3][e];
            r[e] = v[e] > 0.f ? s : 0.f;
#pragma unroll
            for (int o = 0; o < 4; ++o) a[o * E + e] += gd[o] * v[e];
            a[4 * E + e] += r[e];
        }
#pragma unroll
        for (int o = 0; o < 4; ++o) a[5 * E + o] += gd[o];
        Vec16<T>::store(dhid + px * Dtot + ct, r);
    };
    auto load_gd = [&](unsigned px, float* gd) {
        if constexpr (PK) {
            const float4 v = *(const float4*)(d.pk + ((size_t)px * d.nd + h) * 4);
            gd[0] = v.x; gd[1] = v.y; gd[2] = v.z; gd[3] = v.w;
        } else {
            const unsigned n = px / (unsigned)HW;
            const unsigned q = px - n * HW;
#pragma unroll
            for (int o = 0; o < 4; ++o) gd[o] = o < od ? dout[(n * od + o) * (unsigned)HW + q] : 0.f;
        }
    };
    if (g < G) {
        unsigned px = p0 + g;
        for (; px + (U - 1) * G < p1; px += U * G) {
            float gd[U][4], v[U][E];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                load_gd(px + u * G, gd[u]);
                Vec16<T>::load(hid + (px + u * G) * Ctot + ct, v[u]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) body(px + u * G, gd[u], v[u]);
        }
        for (; px < p1; px += G) {
            float gd[4], v[E];
            load_gd(px, gd);
            Vec16<T>::load(hid + px * Ctot + ct, v);
            body(px, gd, v);
        }
    }
    // fold the G pixel-lanes in LDS, KR partials per round (red[k][g][c]), all threads busy
    constexpr int KR = (NA + 3) / 4;
    __shared__ float red[KR * 512];
    double* dst = acc + (size_t)(blockIdx.x % SCD_STAT_REPLICAS) * accsz;
#pragma unroll
    for (int k0 = 0; k0 < NA; k0 += KR) {
        if (k0) __syncthreads();
        if (g < G)
#pragma unroll
            for (int k = 0; k < KR; ++k)
                if (k0 + k < NA) red[(k * G + g) * cpp + c] = a[k0 + k];
        __syncthreads();
        for (int i = tid; i < KR * cpp; i += blockDim.x) {
            const int kk = i / cpp, cc = i - (i / cpp) * cpp;
            const int k = k0 + kk;
            if (k >= NA) continue;
            float s = 0.f;
            for (int j = 0; j < G; ++j) s += red[(kk * G + j) * cpp + cc];
            const int hh = cc / cph;
            const int cll = (cc - hh * cph) * E;
            const int odh = d.od[hh];
            if (k < 4 * E) {                        // dW1[o][cl + e]
                const int o = k / E, e = k - (k / E) * E;
                if (o < odh) atomic_add_f64(dst + (d.orow[hh] + o) * d.Hd + cll + e, (double)s);
            } else if (k < 5 * E) {                 // db0[ct + e]
                atomic_add_f64(dst + d.nout * d.Hd + d.nout + hh * d.Hd + cll + (k - 4 * E), (double)s);
            } else {                                // db1[o]: one chunk-lane per head
                const int o = k - 5 * E;
                if (o < odh && cll == 0) atomic_add_f64(dst + d.nout * d.Hd + d.orow[hh] + o, (double)s);
            }
        }
    }
}

struct HeadsGrad {
    float* dw1[4];
    float* db1[4];
    float* db0[4];
};

__global__ void heads_bwd_weight_finalize_kernel(double* acc, int accsz, HeadsDesc d, HeadsGrad g, int accumulate,
                                                 double alpha) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < accsz; i += gridDim.x * blockDim.x) {
        double s = 0.0;
        for (int r = 0; r < SCD_STAT_REPLICAS; ++r) {
            s += acc[(long)r * accsz + i];
            acc[(long)r * accsz + i] = 0.0;
        }
        float* dst;
        if (i < d.nout * d.Hd) {
            const int row = i / d.Hd, cl = i - (i / d.Hd) * d.Hd;
            int h = 0;
            while (h + 1 < d.nh && row >= d.orow[h + 1]) ++h;
            dst = g.dw1[h] + (row - d.orow[h]) * d.Hd + cl;
        } else if (i < d.nout * d.Hd + d.nout) {
            const int row = i - d.nout * d.Hd;
            int h = 0;
            while (h + 1 < d.nh && row >= d.orow[h + 1]) ++h;
            dst = g.db1[h] + (row - d.orow[h]);
        } else {
            const int c = i - d.nout * d.Hd - d.nout;
            const int h = c / d.Hd;
            dst = g.db0[h] + (c - h * d.Hd);
        }
        s *= alpha;
        *dst = accumulate ? (*dst + (float)s) : (float)s;
    }
}

bool make_desc(HeadsDesc& d, int nh, int Hd, const int* od) {
    if (nh < 1 || nh > 4 || Hd % 8 != 0) return false;
    d.nh = nh; d.Hd = Hd; d.nout = 0;
    d.nd = nh; d.hstride = d.dstride = nh * Hd;
    for (int h = 0; h < 4; ++h) {
        d.od[h] = h < nh ? od[h] : 0;
        if (d.od[h] > 4) return false;
        d.orow[h] = d.nout;
        d.nout += d.od[h];
        d.w1[h] = nullptr; d.b1[h] = nullptr; d.dout[h] = nullptr; d.out[h] = nullptr;
        d.pk = nullptr;
    }
    return d.nout * Hd <= 8 * 512;
}

// ---------------------------------------------------------------- Adam (torch.optim.Adam, foreach form)
__global__ void adam_kernel(float* p, const float* g, float* m, float* v, long n, float lr, float b1, float b2,
                            float eps, float bc1, float bc2_sqrt, float gscale) {
    const float step = lr / bc1;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const float gi = g[i] * gscale;
        float mi = m[i];
        mi = mi + (1.f - b1) * (gi - mi);                 // exp_avg.lerp_(grad, 1-beta1)
        float vi = v[i] * b2 + (1.f - b2) * gi * gi;      // exp_avg_sq.mul_(b2).addcmul_(g,g,1-b2)
        const float denom = sqrtf(vi) / bc2_sqrt + eps;
        p[i] = p[i] - step * (mi / denom);
        m[i] = mi;
        v[i] = vi;
    }
}

// Device-resident step state (hyper = {lr, step}, fp64) so a captured step graph replays with the current learning
// rate and bias corrections: the tick advances the step, the update kernel derives the corrections exactly as
// the host path does (fp64 powers rounded to fp32, torch/optim/adam.py _single_tensor_adam).
// skip (optional): a device word (the peer-memory SyncBN error word, scdhip/peer.py); non-zero = this step's gradients
// were formed from unreduced (NaN-poisoned) statistics: neither the step count nor any parameter or moment changes.
__global__ void adam_tick_kernel(double* hyper, const unsigned long long* skip) {
    if (skip && *skip) return;
    if (threadIdx.x == 0) hyper[1] = hyper[1] + 1.0;
}

__global__ void adam_dev_kernel(float* p, const float* g, float* m, float* v, long n, const double* hyper, float b1,
                                float b2, float eps, float gscale, const unsigned long long* skip) {
    if (skip && *skip) return;
    const double s = hyper[1];
    const float lr = (float)hyper[0];
    const float bc1 = (float)(1.0 - pow((double)b1, s));
    const float bc2 = (float)(1.0 - pow((double)b2, s));
    const float step = lr / bc1;
    const float bc2_sqrt = sqrtf(bc2);
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const float gi = g[i] * gscale;
        float mi = m[i];
        mi = mi + (1.f - b1) * (gi - mi);
        float vi = v[i] * b2 + (1.f - b2) * gi * gi;
        const float denom = sqrtf(vi) / bc2_sqrt + eps;
        p[i] = p[i] - step * (mi / denom);
        m[i] = mi;
        v[i] = vi;
    }
}

// ---------------------------------------------------------------- SGD (torch.optim.SGD, single-tensor form)
// networkFactory.py:84-89: SGD(lr, momentum 0.9, weight_decay 1e-4).  d = g + wd*p; the momentum buffer starts as a
// copy of d on the buffer's first step, then buf = mom*buf + (1-dampening)*d; the update uses d + mom*buf (nesterov) or
// buf.  hyper = {lr, step, initialised, snapshot} fp64 in device memory: the tick advances the step and moves the
// buffer's "initialised" flag into the snapshot the update reads (set to 1 for the next step), so a buffer re-created
// mid-training (flag cleared by the host) starts as torch's does, not from the global step count.
__global__ void sgd_tick_kernel(double* hyper, const unsigned long long* skip) {
    if (skip && *skip) return;
    if (threadIdx.x == 0) {
        hyper[1] = hyper[1] + 1.0;
        hyper[3] = hyper[2];
        hyper[2] = 1.0;
    }
}

__global__ void sgd_dev_kernel(float* p, const float* g, float* buf, long n, const double* hyper, float mom, float damp,
                               float wd, int nesterov, float gscale, const unsigned long long* skip) {
    if (skip && *skip) return;
    const float lr = (float)hyper[0];
    const bool first = hyper[3] == 0.0;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const float pi = p[i];
        float d = g[i] * gscale;
        if (wd != 0.f) d = d + wd * pi;
        if (mom != 0.f) {
            const float b = first ? d : buf[i] * mom + (1.f - damp) * d;
            buf[i] = b;
            d = nesterov ? d + mom * b : b;
        }
        p[i] = pi - lr * d;
    }
}

inline int ew_blocks(long n) { return (int)std::min<long>(8192, std::max<long>(1, (n + 255) / 256)); }

SCD_KERNEL_NS_END
}  // namespace

extern "C" int scd_pack_weight(int dtype, const float* w, void* out, int A, int B, int T, int mode, int ldp, int row_off,
                               void* stream) {
    SCD_F16_FWD(scd_pack_weight, w, out, A, B, T, mode, ldp, row_off, stream);
    if (mode == 3 && (T != 9 || ldp < 4 * A)) return SCD_ERR_ARG;
    const long total = (long)(mode == 0 ? A : mode == 3 ? 4 * B : B) * ldp;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == SCD_DT_BF16)
        hipLaunchKernelGGL((pack_weight_kernel<h16>), dim3(ew_blocks(total)), dim3(256), 0, st, w, (h16*)out, A, B,
                           T, mode, ldp, row_off);
    else if (dtype == SCD_DT_F32)
        hipLaunchKernelGGL((pack_weight_kernel<float>), dim3(ew_blocks(total)), dim3(256), 0, st, w, (float*)out, A, B, T,
                           mode, ldp, row_off);
    else
        return SCD_ERR_ARG;
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_im2col_stem(int dtype, const float* x, void* cols, int N, int H, int W, int Ho, int Wo, int kh,
                               int kw, int stride, int pad, int Kpad, void* stream) {
    SCD_F16_FWD(scd_im2col_stem, x, cols, N, H, W, Ho, Wo, kh, kw, stride, pad, Kpad, stream);
    hipStream_t st = (hipStream_t)stream;
    if (Kpad % 8 || Kpad < kh * kw) return SCD_ERR_ARG;
    const long total = (long)N * Ho * Wo * (Kpad / (dtype == SCD_DT_BF16 ? 8 : 4));
    if (dtype == SCD_DT_BF16)
        hipLaunchKernelGGL((im2col_stem_kernel<h16>), dim3(ew_blocks(total)), dim3(256), 0, st, x, (h16*)cols, N, H,
                           W, Ho, Wo, kh, kw, stride, pad, Kpad);
    else if (dtype == SCD_DT_F32)
        hipLaunchKernelGGL((im2col_stem_kernel<float>), dim3(ew_blocks(total)), dim3(256), 0, st, x, (float*)cols, N, H,
                           W, Ho, Wo, kh, kw, stride, pad, Kpad);
    else
        return SCD_ERR_ARG;
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_stem_pool_fwd(int dtype, const void* y, const float* scale, const float* shift, void* out,
                                 uint8_t* argmax, int N, int H, int W, int C, int Ho, int Wo, void* stream) {
    SCD_F16_FWD(scd_stem_pool_fwd, y, scale, shift, out, argmax, N, H, W, C, Ho, Wo, stream);
    hipStream_t st = (hipStream_t)stream;
    const int E = dtype == SCD_DT_BF16 ? 8 : 4;
    if (C % E) return SCD_ERR_ARG;
    const long total = (long)N * ((Ho + SPR - 1) / SPR) * Wo * (C / E);
    if (total >= (1L << 32)) return SCD_ERR_ARG;
    if (dtype == SCD_DT_BF16)
        hipLaunchKernelGGL((stem_pool_fwd_kernel<h16>), dim3(ew_blocks(total)), dim3(256), 0, st, (const h16*)y,
                           scale, shift, (h16*)out, argmax, N, H, W, C, Ho, Wo);
    else if (dtype == SCD_DT_F32)
        hipLaunchKernelGGL((stem_pool_fwd_kernel<float>), dim3(ew_blocks(total)), dim3(256), 0, st, (const float*)y,
                           scale, shift, (float*)out, argmax, N, H, W, C, Ho, Wo);
    else
        return SCD_ERR_ARG;
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_stem_pool_bwd(int dtype, const void* dout, const uint8_t* argmax, const void* y, const float* scale,
                                 const float* shift, void* dz, int N, int H, int W, int C, int Ho, int Wo, void* stream) {
    SCD_F16_FWD(scd_stem_pool_bwd, dout, argmax, y, scale, shift, dz, N, H, W, C, Ho, Wo, stream);
    hipStream_t st = (hipStream_t)stream;
    const int E = dtype == SCD_DT_BF16 ? 8 : 4;
    if (C % E) return SCD_ERR_ARG;
    const long total = (long)N * H * W * (C / E);
    if (dtype == SCD_DT_BF16)
        hipLaunchKernelGGL((stem_pool_bwd_kernel<h16>), dim3(ew_blocks(total)), dim3(256), 0, st,
                           (const h16*)dout, argmax, (const h16*)y, scale, shift, (h16*)dz, N, H, W, C, Ho, Wo);
    else if (dtype == SCD_DT_F32)
        hipLaunchKernelGGL((stem_pool_bwd_kernel<float>), dim3(ew_blocks(total)), dim3(256), 0, st, (const float*)dout,
                           argmax, (const float*)y, scale, shift, (float*)dz, N, H, W, C, Ho, Wo);
    else
        return SCD_ERR_ARG;
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_stem_pool_bwd_bn(int dtype, const void* dout, const uint8_t* argmax, const void* y, const float* scale,
                                    const float* shift, const float* mean, const float* invstd, void* dz, double* stats,
                                    int N, int H, int W, int C, int Ho, int Wo, void* stream) {
    SCD_F16_FWD(scd_stem_pool_bwd_bn, dout, argmax, y, scale, shift, mean, invstd, dz, stats, N, H, W, C, Ho, Wo, stream);
    hipStream_t st = (hipStream_t)stream;
    const int E = dtype == SCD_DT_BF16 ? 8 : 4;
    if (C % E || 256 % (C / E)) return SCD_ERR_ARG;
    const long total = (long)N * H * W * (C / E);
    static int mode = -1;
    if (mode < 0) { const char* e = getenv("SCD_POOL_2X2"); mode = e ? atoi(e) : 1; }
    if (mode && H == 2 * Ho && W == 2 * Wo && (long)N * H * W * C < (1L << 31)) {
        static const int g2b = resident_grid((const void*)stem_pool_bwd_bn_2x2_kernel<h16>, 256);
        static const int g2f = resident_grid((const void*)stem_pool_bwd_bn_2x2_kernel<float>, 256);
        const long blocks2 = (long)N * Ho * Wo * (C / E);
        const int grid = (int)std::min<long>(dtype == SCD_DT_BF16 ? g2b : g2f, (blocks2 + 255) / 256);
        if (dtype == SCD_DT_BF16)
            hipLaunchKernelGGL((stem_pool_bwd_bn_2x2_kernel<h16>), dim3(grid), dim3(256), 0, st, (const h16*)dout,
                               argmax, (const h16*)y, scale, shift, mean, invstd, (h16*)dz, stats, N, C, Ho, Wo);
        else if (dtype == SCD_DT_F32)
            hipLaunchKernelGGL((stem_pool_bwd_bn_2x2_kernel<float>), dim3(grid), dim3(256), 0, st, (const float*)dout,
                               argmax, (const float*)y, scale, shift, mean, invstd, (float*)dz, stats, N, C, Ho, Wo);
        else
            return SCD_ERR_ARG;
        SCD_RETURN_LAUNCH();
    }
    static const int gb = resident_grid((const void*)stem_pool_bwd_bn_kernel<h16>, 256);
    static const int gf = resident_grid((const void*)stem_pool_bwd_bn_kernel<float>, 256);
    const int blocks = (int)std::min<long>(dtype == SCD_DT_BF16 ? gb : gf, (total + 255) / 256);
    if (dtype == SCD_DT_BF16)
        hipLaunchKernelGGL((stem_pool_bwd_bn_kernel<h16>), dim3(blocks), dim3(256), 0, st, (const h16*)dout, argmax,
                           (const h16*)y, scale, shift, mean, invstd, (h16*)dz, stats, N, H, W, C, Ho, Wo);
    else if (dtype == SCD_DT_F32)
        hipLaunchKernelGGL((stem_pool_bwd_bn_kernel<float>), dim3(blocks), dim3(256), 0, st, (const float*)dout, argmax,
                           (const float*)y, scale, shift, mean, invstd, (float*)dz, stats, N, H, W, C, Ho, Wo);
    else
        return SCD_ERR_ARG;
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_heads_fwd(int dtype, const void* hid, int N, int HW, int nh, int Hd, const int* od,
                             const float* const* w1, const float* const* b1, float* const* outs, void* stream) {
    SCD_F16_FWD(scd_heads_fwd, hid, N, HW, nh, Hd, od, w1, b1, outs, stream);
    HeadsDesc d;
    if (!make_desc(d, nh, Hd, od)) return SCD_ERR_ARG;
    const int E = dtype == SCD_DT_BF16 ? 8 : 4;
    const int cph = Hd / E;
    if (cph > 64 || (cph & (cph - 1))) return SCD_ERR_ARG;
    for (int h = 0; h < nh; ++h) { d.w1[h] = w1[h]; d.b1[h] = b1[h]; d.out[h] = outs[h]; }
    hipStream_t st = (hipStream_t)stream;
    const long total = (long)N * HW * nh * cph;
    const int blocks = (int)std::min<long>(16384, (total + 255) / 256);
    if (dtype == SCD_DT_BF16)
        hipLaunchKernelGGL((heads_fwd_kernel<h16>), dim3(blocks), dim3(256), 0, st, (const h16*)hid, N, HW, d);
    else if (dtype == SCD_DT_F32)
        hipLaunchKernelGGL((heads_fwd_kernel<float>), dim3(blocks), dim3(256), 0, st, (const float*)hid, N, HW, d);
    else
        return SCD_ERR_ARG;
    SCD_RETURN_LAUNCH();
}

extern "C" size_t scd_heads_bwd_accsize(int nh, int Hd, const int* od) {
    int nout = 0;
    for (int h = 0; h < nh; ++h) nout += od[h];
    return (size_t)SCD_STAT_REPLICAS * (nout * Hd + nout + nh * Hd) * sizeof(double);
}

extern "C" int scd_heads_bwd(int dtype, const void* hid, int N, int HW, int nh, int Hd, const int* od,
                             const float* const* w1, const float* const* douts, void* dhid, double* acc,
                             void* stream) {
    SCD_F16_FWD(scd_heads_bwd, hid, N, HW, nh, Hd, od, w1, douts, dhid, acc, stream);
    HeadsDesc d;
    if (!make_desc(d, nh, Hd, od)) return SCD_ERR_ARG;
    const int E = dtype == SCD_DT_BF16 ? 8 : 4;
    const int cpp = nh * Hd / E;
    if (cpp > 256 || (Hd % E)) return SCD_ERR_ARG;
    for (int h = 0; h < nh; ++h) { d.w1[h] = w1[h]; d.dout[h] = douts[h]; }
    const int accsz = d.nout * Hd + d.nout + nh * Hd;
    const long P = (long)N * HW;
    if (P * nh * Hd >= (1L << 31)) return SCD_ERR_ARG;     // 32-bit element offsets
    const int G = 512 / cpp;                                // pixel lanes (cpp <= 256 -> G >= 2)
    const int threads = G * cpp;
    static int pxb_env = -1;
    if (pxb_env < 0) { const char* e = getenv("SCD_HEADS_PXB"); pxb_env = e ? atoi(e) : 0; }
    const int PXB = pxb_env > 0 ? pxb_env : 2048;      // one 1-per-CU round at B=32, 128x128
    const int blocks = cdiv(P, PXB);
    hipStream_t st = (hipStream_t)stream;
    static int u_env = -1;
    if (u_env < 0) { const char* e = getenv("SCD_HEADS_U"); u_env = e ? atoi(e) : 8; }
    if (dtype == SCD_DT_BF16 && u_env == 8)
        hipLaunchKernelGGL((heads_bwd_kernel<h16, 8>), dim3(blocks), dim3(threads), 0, st, (const h16*)hid, N,
                           HW, d, (h16*)dhid, acc, accsz, PXB);
    else if (dtype == SCD_DT_BF16)
        hipLaunchKernelGGL((heads_bwd_kernel<h16, 4>), dim3(blocks), dim3(threads), 0, st, (const h16*)hid, N,
                           HW, d, (h16*)dhid, acc, accsz, PXB);
    else if (dtype == SCD_DT_F32)
        hipLaunchKernelGGL((heads_bwd_kernel<float, 4>), dim3(blocks), dim3(threads), 0, st, (const float*)hid, N, HW,
                           d, (float*)dhid, acc, accsz, PXB);
    else
        return SCD_ERR_ARG;
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_heads_bwd_weight_finalize(double* acc, int nh, int Hd, const int* od, float* const* dw1,
                                             float* const* db1, float* const* db0, int accumulate, float alpha, void* stream) {
    HeadsDesc d;
    if (!make_desc(d, nh, Hd, od)) return SCD_ERR_ARG;
    HeadsGrad g;
    for (int h = 0; h < 4; ++h) {
        g.dw1[h] = h < nh ? dw1[h] : nullptr;
        g.db1[h] = h < nh ? db1[h] : nullptr;
        g.db0[h] = h < nh ? db0[h] : nullptr;
    }
    const int accsz = d.nout * Hd + d.nout + nh * Hd;
    hipLaunchKernelGGL(heads_bwd_weight_finalize_kernel, dim3(cdiv(accsz, 256)), dim3(256), 0, (hipStream_t)stream, acc,
                       accsz, d, g, accumulate, (double)alpha);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_adam_step(float* p, const float* g, float* m, float* v, long n, float lr, float beta1, float beta2,
                             float eps, float bc1, float bc2, float gscale, void* stream) {
    hipLaunchKernelGGL(adam_kernel, dim3(ew_blocks(n)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, lr, beta1,
                       beta2, eps, bc1, sqrtf(bc2), gscale);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_adam_step_dev(float* p, const float* g, float* m, float* v, long n, double* hyper, float beta1,
                                 float beta2, float eps, float gscale, const unsigned long long* skip, void* stream) {
    if (!hyper) return SCD_ERR_ARG;
    hipLaunchKernelGGL(adam_tick_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, hyper, skip);
    hipLaunchKernelGGL(adam_dev_kernel, dim3(ew_blocks(n)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n,
                       (const double*)hyper, beta1, beta2, eps, gscale, skip);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_sgd_step_dev(float* p, const float* g, float* buf, long n, double* hyper, float momentum,
                                float dampening, float weight_decay, int nesterov, float gscale,
                                const unsigned long long* skip, void* stream) {
    if (!hyper || (momentum != 0.f && !buf)) return SCD_ERR_ARG;
    hipLaunchKernelGGL(sgd_tick_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, hyper, skip);
    hipLaunchKernelGGL(sgd_dev_kernel, dim3(ew_blocks(n)), dim3(256), 0, (hipStream_t)stream, p, g, buf, n,
                       (const double*)hyper, momentum, dampening, weight_decay, nesterov, gscale, skip);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_heads_bwd_packed(int dtype, const void* hid, int N, int HW, int nh, int Hd, const int* od,
                                    const float* const* w1, const float* const* douts, float dscale, float* packed,
                                    void* dhid, double* acc, void* stream) {
    return scd_heads_bwd_packed_split(dtype, hid, N, HW, nh, Hd, od, nh, w1, douts, dscale, packed, dhid, acc, stream);
}

extern "C" int scd_heads_bwd_packed_split(int dtype, const void* hid, int N, int HW, int nh, int Hd, const int* od,
                                          int nd, const float* const* w1, const float* const* douts, float dscale,
                                          float* packed, void* dhid, double* acc, void* stream) {
    SCD_F16_FWD(scd_heads_bwd_packed_split, hid, N, HW, nh, Hd, od, nd, w1, douts, dscale, packed, dhid, acc, stream);
    HeadsDesc d;
    if (!make_desc(d, nh, Hd, od) || !packed || nd < 1 || nd > nh) return SCD_ERR_ARG;
    d.nd = nd;
    d.dstride = nd * Hd;
    const int E = dtype == SCD_DT_BF16 ? 8 : 4;
    const int cpp = nd * Hd / E;
    if (cpp > 256 || (Hd % E)) return SCD_ERR_ARG;
    for (int h = 0; h < nh; ++h) { d.w1[h] = w1[h]; d.dout[h] = douts[h]; }
    const int accsz = d.nout * Hd + d.nout + nh * Hd;
    const long P = (long)N * HW;
    if (P * nh * Hd >= (1L << 31)) return SCD_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(heads_pack_kernel, dim3(ew_blocks(P)), dim3(256), 0, st, N, HW, d, dscale, packed);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    d.pk = packed;
    const int G = 512 / cpp;
    const int threads = G * cpp;
    static int pxb_env = -1;
    if (pxb_env < 0) { const char* ev = getenv("SCD_HEADS_PXB"); pxb_env = ev ? atoi(ev) : 0; }
    const int PXB = pxb_env > 0 ? pxb_env : 2048;
    const int blocks = cdiv(P, PXB);
    if (dtype == SCD_DT_BF16)
        hipLaunchKernelGGL((heads_bwd_kernel<h16, 8, true>), dim3(blocks), dim3(threads), 0, st, (const h16*)hid,
                           N, HW, d, (h16*)dhid, acc, accsz, PXB);
    else if (dtype == SCD_DT_F32)
        hipLaunchKernelGGL((heads_bwd_kernel<float, 4, true>), dim3(blocks), dim3(threads), 0, st, (const float*)hid,
                           N, HW, d, (float*)dhid, acc, accsz, PXB);
    else
        return SCD_ERR_ARG;
    SCD_RETURN_LAUNCH();
}

// ---------------------------------------------------------------- CenterNet heads: sparse-gradient backward
// The regression / offset heads (centerNetOffset.py:106-110) are trained only through L1LossMask on
// gather(head, inds) (centerNetOffset.py:199-214, regression.py:37-44): their output gradient is zero except at
// the <= K gathered pixels per image.  For those heads the tail backward, the 3x3 weight gradient and the 3x3
// input gradient reduce to sums over that pixel set (slots s = b*K + k; the first slot naming a pixel carries it,
// repeats carry nothing, so a pixel named twice is counted once with its summed gradient):
//   dhid_s[s][c]         = relu'(hid) * sum_o W1[o][c] g[o]           (heads [nd, nh), c over their channels)
//   xcol[s][t*Cin + ci]  = feat[p + d_t][ci]                           (im2col of the slot's pixel, tap-major)
//   dW0 = dhid_s^T xcol, and dX[q] += sum_{t : q - d_t active} C[slot(q - d_t)][t*Cin + ci], C = dhid_s W0^T
// The dense heads [0, nd) keep the dense tail (scd_heads_bwd_packed_split) and GEMMs over their channels only.
// slotmap (pixel -> slot, -1 elsewhere) and ownermap (q -> first (slot, tap) reaching q, INT_MAX elsewhere) are
// persistent int32 maps over the N*H*W pixels; the kernels below leave them as they found them.
namespace {
SCD_KERNEL_NS_BEGIN
constexpr int SP_SPB = 2;                   // slots per workgroup of the sparse tail

template <typename T>
__global__ __launch_bounds__(256) void heads_sparse_bwd_kernel(const T* hid, const T* feat, int N, int H, int W, int Cin,
                                                               HeadsDesc d, float dscale, const long* inds, int K,
                                                               T* dhid_s, T* xcol, double* acc, int accsz,
                                                               int* slotmap, int* ownermap) {
    const int HW = H * W;
    const int Cs = (d.nh - d.nd) * d.Hd;
    const int tid = threadIdx.x;
    const int c = tid;                                  // sparse-head channel of this thread
    const bool cok = c < Cs;
    const int h = cok ? d.nd + c / d.Hd : d.nd;
    const int j = cok ? c - (h - d.nd) * d.Hd : 0;
    const int od = d.od[h];
    float w[4];
#pragma unroll
    for (int o = 0; o < 4; ++o) w[o] = (cok && o < od) ? d.w1[h][o * d.Hd + j] : 0.f;
    float a_dw1[4] = {0.f, 0.f, 0.f, 0.f}, a_db1[4] = {0.f, 0.f, 0.f, 0.f}, a_db0 = 0.f;
    const int S = N * K;
    const int s0 = blockIdx.x * SP_SPB;
    const int ns = min(S, s0 + SP_SPB) - s0;
    // which of the workgroup's slots repeat an earlier slot's pixel of the same image (all pairs in parallel)
    __shared__ int dup[SP_SPB];
    if (tid < SP_SPB) dup[tid] = 0;
    __syncthreads();
    for (int i = tid; i < ns * K; i += blockDim.x) {
        const int jj = i / K, k2 = i - (i / K) * K;
        const int s = s0 + jj, k = s - (s / K) * K;
        if (k2 < k && inds[s - k + k2] == inds[s]) dup[jj] = 1;
    }
    __syncthreads();
    for (int jj = 0; jj < ns; ++jj) {
        const int s = s0 + jj;
        const int b = s / K;
        const long ind = inds[s];
        const bool active = ind >= 0 && ind < HW && !dup[jj];
        const int q0 = active ? (int)ind : 0;
        const int y = q0 / W, x = q0 - (q0 / W) * W;
        const long p = (long)b * HW + q0;
        float r = 0.f;
        if (active && cok) {
            const float hv = to_f<T>(hid[p * d.hstride + d.nd * d.Hd + c]);
            float g[4];
#pragma unroll
            for (int o = 0; o < 4; ++o) g[o] = o < od ? d.dout[h][((long)b * od + o) * HW + q0] * dscale : 0.f;
            const float sacc = g[0] * w[0] + g[1] * w[1] + g[2] * w[2] + g[3] * w[3];
            r = hv > 0.f ? sacc : 0.f;
#pragma unroll
            for (int o = 0; o < 4; ++o) { a_dw1[o] += g[o] * hv; a_db1[o] += g[o]; }
            a_db0 += r;
        }
        if (cok) dhid_s[(long)s * Cs + c] = from_f<T>(r);
        if (active && tid < 9) {
            if (tid == 0) slotmap[p] = s;
            const int qy = y + tid / 3 - 1, qx = x + tid % 3 - 1;
            if ((unsigned)qy < (unsigned)H && (unsigned)qx < (unsigned)W)
                atomicMin(ownermap + (long)b * HW + qy * W + qx, s * 9 + tid);
        }
        // im2col row of the slot, tap-major (xcol[s][t*Cin + ci]; zeros outside the image): coalesced rows of feat
        for (int ci = tid; ci < Cin; ci += blockDim.x) {
            T v[9];
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const int iy = y + t / 3 - 1, ix = x + t % 3 - 1;
                const bool in = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
                v[t] = in ? feat[(((long)b * H + iy) * W + ix) * Cin + ci] : from_f<T>(0.f);
            }
#pragma unroll
            for (int t = 0; t < 9; ++t) xcol[(long)s * 9 * Cin + t * Cin + ci] = v[t];
        }
    }
    // weight / bias partials of the sparse heads (same accumulator layout as heads_bwd_kernel)
    if (cok) {
        double* dst = acc + (size_t)(blockIdx.x % SCD_STAT_REPLICAS) * accsz;
#pragma unroll
        for (int o = 0; o < 4; ++o)
            if (o < od) atomic_add_f64(dst + (d.orow[h] + o) * d.Hd + j, (double)a_dw1[o]);
        atomic_add_f64(dst + d.nout * d.Hd + d.nout + h * d.Hd + j, (double)a_db0);
        if (j == 0)
#pragma unroll
            for (int o = 0; o < 4; ++o)
                if (o < od) atomic_add_f64(dst + d.nout * d.Hd + d.orow[h] + o, (double)a_db1[o]);
    }
}

// dX[q] += the sparse heads' input-gradient at the pixels q their slots reach; one workgroup per slot, one
// thread per input channel; q is handled by the first (slot, tap) reaching it (ownermap), which sums the
// contributions of every active neighbour in tap order (cols[s][t*Cin + ci], tap-major).  The slot maps of the
// 5x5 neighbourhood and the owners of the 3x3 reach are read once into LDS.  With bn_y: the following BN+ReLU
// layer's backward sums (scd_conv_gemm_bnbwd's epilogue over the dense part) get the change of each rewritten value.
template <typename T>
__global__ __launch_bounds__(256) void heads_sparse_fixup_kernel(T* dx, const T* cols, int N, int H, int W, int Cin,
                                                                 const long* inds, int K, const int* slotmap,
                                                                 int* ownermap, const T* bny, const float* mean,
                                                                 const float* invstd, const float* rsc,
                                                                 const float* rsh, double* stats) {
    const int HW = H * W;
    const int s = blockIdx.x;
    const int b = s / K;
    const long ind = inds[s];
    if (ind < 0 || ind >= HW) return;
    const long p = (long)b * HW + ind;
    if (slotmap[p] != s) return;                       // a repeat of an earlier slot's pixel
    const int y = (int)ind / W, x = (int)ind - ((int)ind / W) * W;
    const int tid = threadIdx.x;
    __shared__ int nb[25], own[9];
    if (tid < 25) {
        const int py = y + tid / 5 - 2, px = x + tid % 5 - 2;
        nb[tid] = ((unsigned)py < (unsigned)H && (unsigned)px < (unsigned)W) ? slotmap[(long)b * HW + py * W + px] : -1;
    } else if (tid >= 32 && tid < 41) {
        const int t = tid - 32;
        const int qy = y + t / 3 - 1, qx = x + t % 3 - 1;
        own[t] = ((unsigned)qy < (unsigned)H && (unsigned)qx < (unsigned)W) ? ownermap[(long)b * HW + qy * W + qx] : -1;
    }
    __syncthreads();
    if (tid < 9 && own[tid] == s * 9 + tid)          // restore the owner map (every read above is done)
        ownermap[(long)b * HW + (y + tid / 3 - 1) * W + x + tid % 3 - 1] = 0x7fffffff;
    const long KC = 9L * Cin;
    for (int ci = tid; ci < Cin; ci += blockDim.x) {
        float bm = 0.f, bi = 0.f, bs = 0.f, bh = 0.f;
        if (bny) { bm = mean[ci]; bi = invstd[ci]; bs = rsc[ci]; bh = rsh[ci]; }
        float dsum = 0.f, dsq = 0.f;
        for (int t = 0; t < 9; ++t) {
            if (own[t] != s * 9 + t) continue;
            const int oy = t / 3 - 1, ox = t % 3 - 1;    // q - p
            float corr = 0.f;
#pragma unroll
            for (int t2 = 0; t2 < 9; ++t2) {
                const int s2 = nb[(oy - (t2 / 3 - 1) + 2) * 5 + ox - (t2 % 3 - 1) + 2];
                if (s2 >= 0) corr += to_f<T>(cols[(long)s2 * KC + t2 * Cin + ci]);
            }
            const long qi = p + oy * W + ox;
            T* dp = dx + qi * Cin + ci;
            const T old = *dp;
            const T nv = from_f<T>(to_f<T>(old) + corr);
            *dp = nv;
            if (bny) {
                const float yv = to_f<T>(bny[qi * Cin + ci]);
                const float dd = yv * bs + bh > 0.f ? to_f<T>(nv) - to_f<T>(old) : 0.f;
                dsum += dd;
                dsq += dd * (yv - bm) * bi;
            }
        }
        if (bny) {
            const int rep = s % SCD_STAT_REPLICAS;
            atomic_add_f64(stats + ((long)rep * 2 + 0) * Cin + ci, (double)dsum);
            atomic_add_f64(stats + ((long)rep * 2 + 1) * Cin + ci, (double)dsq);
        }
    }
}

__global__ void heads_sparse_reset_kernel(const long* inds, int S, int K, int HW, int* slotmap) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    const long ind = inds[s];
    if (ind < 0 || ind >= HW) return;
    const long p = (long)(s / K) * HW + ind;
    if (slotmap[p] == s) slotmap[p] = -1;
}

SCD_KERNEL_NS_END
}  // namespace

extern "C" int scd_heads_sparse_bwd(int dtype, const void* hid, const void* feat, int N, int H, int W, int Cin, int nh,
                                    int Hd, const int* od, int nd, const float* const* w1, const float* const* douts,
                                    float dscale, const long* inds, int K, void* dhid_s, void* xcol, double* acc,
                                    int* slotmap, int* ownermap, void* stream) {
    SCD_F16_FWD(scd_heads_sparse_bwd, hid, feat, N, H, W, Cin, nh, Hd, od, nd, w1, douts, dscale, inds, K, dhid_s, xcol,
                acc, slotmap, ownermap, stream);
    HeadsDesc d;
    if (!make_desc(d, nh, Hd, od) || nd < 0 || nd >= nh || K < 1 || (nh - nd) * Hd > 256) return SCD_ERR_ARG;
    if ((long)N * K * 9 * 9 >= (1L << 31) || (long)N * H * W * nh * Hd >= (1L << 31)) return SCD_ERR_ARG;
    d.nd = nd;
    for (int h = 0; h < nh; ++h) { d.w1[h] = w1[h]; d.dout[h] = douts[h]; }
    const int accsz = d.nout * Hd + d.nout + nh * Hd;
    const int blocks = cdiv((long)N * K, SP_SPB);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == SCD_DT_BF16)
        hipLaunchKernelGGL(heads_sparse_bwd_kernel<h16>, dim3(blocks), dim3(256), 0, st, (const h16*)hid,
                           (const h16*)feat, N, H, W, Cin, d, dscale, inds, K, (h16*)dhid_s, (h16*)xcol, acc,
                           accsz, slotmap, ownermap);
    else if (dtype == SCD_DT_F32)
        hipLaunchKernelGGL(heads_sparse_bwd_kernel<float>, dim3(blocks), dim3(256), 0, st, (const float*)hid,
                           (const float*)feat, N, H, W, Cin, d, dscale, inds, K, (float*)dhid_s, (float*)xcol, acc,
                           accsz, slotmap, ownermap);
    else
        return SCD_ERR_ARG;
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_heads_sparse_fixup(int dtype, void* dx, const void* cols, int N, int H, int W, int Cin,
                                      const long* inds, int K, int* slotmap, int* ownermap, const void* bn_y,
                                      const float* mean, const float* invstd, const float* relu_scale,
                                      const float* relu_shift, double* bn_stats, void* stream) {
    SCD_F16_FWD(scd_heads_sparse_fixup, dx, cols, N, H, W, Cin, inds, K, slotmap, ownermap, bn_y, mean, invstd,
                relu_scale, relu_shift, bn_stats, stream);
    if (Cin < 1 || K < 1) return SCD_ERR_ARG;
    if (bn_y && !(mean && invstd && relu_scale && relu_shift && bn_stats)) return SCD_ERR_ARG;
    const int S = N * K;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == SCD_DT_BF16)
        hipLaunchKernelGGL(heads_sparse_fixup_kernel<h16>, dim3(S), dim3(256), 0, st, (h16*)dx,
                           (const h16*)cols, N, H, W, Cin, inds, K, slotmap, ownermap, (const h16*)bn_y, mean,
                           invstd, relu_scale, relu_shift, bn_stats);
    else if (dtype == SCD_DT_F32)
        hipLaunchKernelGGL(heads_sparse_fixup_kernel<float>, dim3(S), dim3(256), 0, st, (float*)dx, (const float*)cols,
                           N, H, W, Cin, inds, K, slotmap, ownermap, (const float*)bn_y, mean, invstd, relu_scale,
                           relu_shift, bn_stats);
    else
        return SCD_ERR_ARG;
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(heads_sparse_reset_kernel, dim3(cdiv(S, 256)), dim3(256), 0, st, inds, S, K, H * W, slotmap);
    SCD_RETURN_LAUNCH();
}
