// Direct stem convolution Conv2d(1, 64, 7, stride 2, pad 3, no bias) (residuals.py:209-216) on MFMA, bf16.
//
// The im2col path (scd_im2col_stem + a 1x1 GEMM over 64 padded taps) writes and re-reads a 64-tap column
// tensor as large as the conv output (B x 256 x 256 x 64 bf16 = 268 MB at B = 32).  Here each workgroup
// stages the fp32 input patch its output tile needs (a few KB), builds the [pixel][tap] tile in LDS and
// multiplies it with the [64 co][64 tap] weight tile: HBM traffic is the input image plus the output.
// The weight gradient does the same with a [tap][pixel] tile against the output gradient and writes one
// fp32 64 x 64 partial per split (reduced by scd_wgrad_reduce, T = 1, Ci = 64, cvalid = 49).
#include <algorithm>

#include "scd_common.h"

namespace {
SCD_KERNEL_NS_BEGIN

constexpr int KS = 7, KK = 49, SP = 2, PD = 3, CO = 64;

__device__ __forceinline__ int swz128(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

// ---- forward: one workgroup = 2 output rows x 128 output columns (256 pixels) of one image
constexpr int FTW = 128, FTH = 2;
constexpr int PROWS = SP * (FTH - 1) + KS;          // 9 input rows
constexpr int PCOLS = SP * (FTW - 1) + KS + 1;      // 262 -> padded to an even count

__global__ __launch_bounds__(256) void stem_conv_fwd_kernel(const float* __restrict__ x, const __bf16* __restrict__ wpk,
                                                            __bf16* __restrict__ y, double* __restrict__ stats,
                                                            int H, int W, int Ho, int Wo) {
    constexpr int AT = FTH * FTW * 128;             // A tile [256 px][64 taps] bf16, 128-B rows
    constexpr int BT = CO * 128;                    // B tile [64 co][64 taps]
    constexpr int EROW = CO * 2 + 16;
    __shared__ __attribute__((aligned(16))) char smem[AT + BT + PROWS * PCOLS * 4];
    char* As = smem;
    char* Bs = smem + AT;
    float* patch = (float*)(smem + AT + BT);

    const int tid = threadIdx.x;
    const int tiles_w = Wo / FTW;
    const int bid = blockIdx.x;
    const int n = bid / ((Ho / FTH) * tiles_w);
    const int rem = bid - n * (Ho / FTH) * tiles_w;
    const int oh0 = (rem / tiles_w) * FTH, ow0 = (rem - (rem / tiles_w) * tiles_w) * FTW;
    const int ih0 = oh0 * SP - PD, iw0 = ow0 * SP - PD;

    // weights: 64 rows x 8 chunks of 16 B
    for (int i = tid; i < CO * 8; i += 256) {
        const int r = i >> 3, c = i & 7;
        *(uint4*)(Bs + swz128(r, c)) = *(const uint4*)(wpk + r * 64 + c * 8);
    }
    // input patch (zero outside the image)
    const float* xn = x + (size_t)n * H * W;
    for (int i = tid; i < PROWS * PCOLS; i += 256) {
        const int r = i / PCOLS, c = i - (i / PCOLS) * PCOLS;
        const int ih = ih0 + r, iw = iw0 + c;
        patch[i] = ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) ? xn[(size_t)ih * W + iw] : 0.f;
    }
    __syncthreads();
    // im2col tile: thread -> pixel p = tid, all 64 taps (8 chunks of 8)
    {
        const int pr = tid / FTW, pc = tid - (tid / FTW) * FTW;
        const float* pp = patch + (SP * pr) * PCOLS + SP * pc;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            bf16x8 v;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int k = c * 8 + e;
                v[e] = (__bf16)(k < KK ? pp[(k / KS) * PCOLS + (k % KS)] : 0.f);
            }
            *(bf16x8*)(As + swz128(tid, c)) = v;
        }
    }
    __syncthreads();

    // MFMA: wave w owns pixels 64w .. 64w+63 (4 blocks) x all 64 channels (4 blocks), K = 64 (2 steps)
    const int lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, lg = lane >> 4, l7 = l16 & 7;
    f32x4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const int co = ((s * 4 + lg) ^ l7) << 4;
        bf16x8 af[4], bfr[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) af[a] = *(const bf16x8*)(As + (wave * 64 + a * 16 + l16) * 128 + co);
#pragma unroll
        for (int b = 0; b < 4; ++b) bfr[b] = *(const bf16x8*)(Bs + (b * 16 + l16) * 128 + co);
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b)
                acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[b], af[a], acc[a][b], 0, 0, 0);
    }
    __syncthreads();          // A tile no longer read: reuse it for the output staging

    // epilogue: lane holds pixel a*16+l16 (of its wave) and channels b*16+4lg .. +3
    float csum[4][4], csq[4][4];
    char* ep = smem + wave * 64 * EROW;
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) { csum[b][r] = 0.f; csq[b][r] = 0.f; }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
            bf16x4 o;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float v = acc[a][b][r];
                o[r] = (__bf16)v;
                csum[b][r] += v;
                csq[b][r] += v * v;
            }
            *(bf16x4*)(ep + (a * 16 + l16) * EROW + (b * 16 + lg * 4) * 2) = o;
        }
    __syncthreads();
    // the 2 x 128 output pixels are two contiguous 16-KB runs of NHWC
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int idx = tid + 256 * j;            // 16-B chunk of the 256 x 128-B tile
        const int p = idx >> 3, c = idx & 7;
        const int w = p >> 6, pl = p & 63;
        const uint4 v = *(const uint4*)(smem + w * 64 * EROW + pl * EROW + c * 16);
        const int pr = p / FTW, pc = p - (p / FTW) * FTW;
        *(uint4*)(y + (((size_t)n * Ho + oh0 + pr) * Wo + ow0 + pc) * CO + c * 8) = v;
    }
    if (stats) {
        float* red = (float*)(smem + 4 * 64 * EROW);        // [4 waves][64 ch][2]
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float s = csum[b][r], q = csq[b][r];
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) { s += __shfl_xor(s, o, 64); q += __shfl_xor(q, o, 64); }
                if (l16 == 0) {
                    const int c = b * 16 + lg * 4 + r;
                    red[(wave * CO + c) * 2] = s;
                    red[(wave * CO + c) * 2 + 1] = q;
                }
            }
        __syncthreads();
        if (tid < CO) {
            double s = 0.0, q = 0.0;
#pragma unroll
            for (int w = 0; w < 4; ++w) { s += red[(w * CO + tid) * 2]; q += red[(w * CO + tid) * 2 + 1]; }
            const int rep = bid % SCD_STAT_REPLICAS;
            atomic_add_f64(stats + ((long)rep * 2 + 0) * CO + tid, s);
            atomic_add_f64(stats + ((long)rep * 2 + 1) * CO + tid, q);
        }
    }
}

// ---- weight gradient: ws[z][co][k] = sum over the split's pixels of dy[pix][co] * col[pix][k]
// stage = 64 output pixels of one row; the dy stage is read with ds_read_b64_tr_b16 (co-major fragments),
// the [tap][pixel] tile is built transposed so its fragments are plain 16-B reads.
constexpr int WPX = 64;
constexpr int WPCOLS = SP * (WPX - 1) + KS + 1;     // 134
constexpr int DROW = 288;                           // dy stage row stride (128 B of data): conflict-free tr reads

__device__ __forceinline__ int dswz(int row, int byte) { return row * DROW + (byte ^ (((row >> 3) & 1) << 7)); }

__global__ __launch_bounds__(256) void stem_conv_wgrad_kernel(const __bf16* __restrict__ dy, const __bf16* __restrict__ ybn,
                                                              const float* __restrict__ coef, const float* __restrict__ x,
                                                              float* __restrict__ ws, int H, int W, int Ho, int Wo,
                                                              long M, int chunk) {
    constexpr int DT = WPX * DROW;                  // dy stage
    constexpr int CT = KK < 64 ? 64 * 128 : 0;      // [64 taps][64 px] bf16
    __shared__ __attribute__((aligned(16))) char smem[DT + CT + KS * WPCOLS * 4];
    char* Ds = smem;
    char* Cs = smem + DT;
    float* patch = (float*)(smem + DT + CT);

    const int tid = threadIdx.x;
    const int z = blockIdx.x;
    const long p0 = (long)z * chunk;
    const long p1 = min(M, p0 + chunk);
    const int lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, lg = lane >> 4;
    const int q4 = l16 >> 2, pp = l16 & 3;
    // wave (wm, wn): output channels 32wm .. +31 (M side), taps 32wn .. +31 (N side)
    const int wm = wave >> 1, wn = wave & 1;
    f32x4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
    typedef __attribute__((ext_vector_type(8))) short s16x8;

    for (long ps = p0; ps < p1; ps += WPX) {
        // stage position: WPX pixels of one output row (Wo % WPX == 0, chunk % WPX == 0)
        const int n = (int)(ps / ((long)Ho * Wo));
        const int rem = (int)(ps - (long)n * Ho * Wo);
        const int oh = rem / Wo, ow0 = rem - (rem / Wo) * Wo;
        const int ih0 = oh * SP - PD, iw0 = ow0 * SP - PD;
        const float* xn = x + (size_t)n * H * W;
        __syncthreads();                              // previous stage's reads are done
        // dy stage: 64 px x 128 B = 512 chunks of 16 B.  With coef (fused BN backward apply): dy is the masked
        // dz and the BN input y of the stem, and the stage holds a*dz + b*y + c rounded to bf16 (as the apply pass)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int idx = tid + 256 * j;
            const int r = idx >> 3, c = idx & 7;
            uint4 v = *(const uint4*)(dy + (ps + r) * CO + c * 8);
            if (coef) {
                const uint4 yv = *(const uint4*)(ybn + (ps + r) * CO + c * 8);
                const bf16x8 d8 = __builtin_bit_cast(bf16x8, v), y8 = __builtin_bit_cast(bf16x8, yv);
                bf16x8 o8;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const int ch = c * 8 + e;
                    o8[e] = (__bf16)(coef[ch] * (float)d8[e] + coef[CO + ch] * (float)y8[e] + coef[2 * CO + ch]);
                }
                v = __builtin_bit_cast(uint4, o8);
            }
            *(uint4*)(Ds + dswz(r, c * 16)) = v;
        }
        for (int i = tid; i < KS * WPCOLS; i += 256) {
            const int r = i / WPCOLS, c = i - (i / WPCOLS) * WPCOLS;
            const int ih = ih0 + r, iw = iw0 + c;
            patch[i] = ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) ? xn[(size_t)ih * W + iw] : 0.f;
        }
        __syncthreads();
        // transposed im2col tile: thread -> tap k = tid / 4, pixels 16 * (tid % 4) .. +15 (two 16-B chunks)
        {
            const int k = tid >> 2, pq = tid & 3;
            const int kh = k / KS, kw = k - (k / KS) * KS;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                bf16x8 v;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const int px = pq * 16 + h * 8 + e;
                    v[e] = (__bf16)(k < KK ? patch[kh * WPCOLS + SP * px + kw] : 0.f);
                }
                *(bf16x8*)(Cs + swz128(k, pq * 2 + h)) = v;
            }
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            // A (taps, 8 consecutive pixels) from the [tap][px] tile; B (channels, 8 consecutive pixels) by tr reads
            const int r0 = 32 * s + 8 * lg + q4;
            bf16x8 tf[2], df[2];
#pragma unroll
            for (int b = 0; b < 2; ++b)
                tf[b] = *(const bf16x8*)(Cs + swz128(wn * 32 + b * 16 + l16, s * 4 + lg));
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                const int cb = (wm * 32 + a * 16 + 4 * pp) * 2;
                s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Ds + dswz(r0, cb)));
                s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Ds + dswz(r0 + 4, cb)));
                s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                df[a] = __builtin_bit_cast(bf16x8, v);
            }
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tf[b], df[a], acc[a][b], 0, 0, 0);
        }
    }
    // lane holds taps wn*32 + b*16 + 4lg .. +3 of channel wm*32 + a*16 + l16
    float* wz = ws + (size_t)z * CO * 64;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
            *(f32x4*)(wz + (wm * 32 + a * 16 + l16) * 64 + wn * 32 + b * 16 + lg * 4) = acc[a][b];
}


// ================================================================ stem without the full-resolution activation
//
// BASELINE's stem (residuals.py:209-216): y = conv7x7/s2(x) (N,256,256,64 at 512^2), BN (batch statistics), ReLU,
// MaxPool(3,2,1).  y is 4x the pooled output; the kernels above write it once, read it for the pool, and the
// backward reads it twice more and writes/reads its gradient.  Everything the step needs follows from the input,
// the pooled side and one 64 x 64 matrix:
//   * Gram matrix of the im2col rows, G = sum_p col[p] col[p]^T (49 taps + a ones column at tap 49, so G[k][49] =
//     sum_p col[p][k] = s[k] and G[49][49] = M): the BN batch statistics are sum_p y = W s and
//     sum_p y^2 = diag(W G W^T) -- exact algebra on the bf16 operands the conv multiplies (stem_gram_kernel,
//     stem_gram_stats_kernel);
//   * forward: conv + BN apply + ReLU + max-pool in one pass over an input patch (stem_fused_fwd_kernel); y is
//     rounded to bf16 in LDS exactly where the unfused kernel stored it, so pooled values / argmax are identical;
//     the pre-BN value at each argmax (bf16) is kept at pooled size for the backward;
//   * backward: dz (the pool + ReLU gradient) is non-zero only at argmax positions, so the weight-gradient stage
//     builds dz for its 64 conv pixels from the pooled gradient / argmax / y-at-argmax (L2-resident, 1/4 size) and
//     accumulates the BN backward sums on the way (stem_wgrad_pooled_kernel); with dy = a*dz + b*y + c (the BN
//     backward apply, scd_bn_bwd_finalize's coefficients) the weight gradient is
//     dW = a * sum dz col^T + b * W G + c * s^T  (stem_wgrad_combine_kernel).
constexpr int GONE = KK;                               // tap index of the ones column

// The tap operand of a 64-pixel stage (conv row oh, pixels ow0 .. ow0+63) without an im2col tile: 8 copies of the
// stage's 7 input rows in bf16, copy (par, u) holding x[row][2 (j + u) + par] at j = 0..63 (tile-relative input
// columns), so the 8 pixels px0 .. px0+7 of tap (kh, kw) -- input columns 2 px + kw -- are copy (kw & 1, kw >> 1),
// row kh, j = px0 .. px0+7: one aligned 16-B LDS read per MFMA fragment.
constexpr int TCOPY = 128;                             // bytes per copy row (64 bf16)
constexpr int TSZ = 8 * KS * TCOPY;                    // 7168 B per stage buffer
constexpr int TPL = (KS * WPCOLS + 255) / 256;         // patch elements per thread (4)

__device__ __forceinline__ void tap_load(float (&pv)[TPL], const float* __restrict__ x, int H, int W, int Ho, int Wo,
                                         long ps, int tid) {
    const int n = (int)(ps / ((long)Ho * Wo));
    const int rem = (int)(ps - (long)n * Ho * Wo);
    const int oh = rem / Wo, ow0 = rem - (rem / Wo) * Wo;
    const int ih0 = oh * SP - PD, iw0 = ow0 * SP - PD;
    const float* xn = x + (size_t)n * H * W;
#pragma unroll
    for (int q = 0; q < TPL; ++q) {
        const int i = tid + 256 * q;
        const int r = i / WPCOLS, c = i - (i / WPCOLS) * WPCOLS;
        const int ih = ih0 + r, iw = iw0 + c;
        pv[q] = (i < KS * WPCOLS && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) ? xn[(size_t)ih * W + iw] : 0.f;
    }
}

__device__ __forceinline__ void tap_store(char* Ts, const float (&pv)[TPL], int tid) {
#pragma unroll
    for (int q = 0; q < TPL; ++q) {
        const int i = tid + 256 * q;
        if (i >= KS * WPCOLS) break;
        const int r = i / WPCOLS, c = i - (i / WPCOLS) * WPCOLS;
        const __bf16 v = (__bf16)pv[q];
        const int par = c & 1, j = c >> 1;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int jj = j - u;
            if (jj >= 0 && jj < WPX) *(__bf16*)(Ts + ((par * 4 + u) * KS + r) * TCOPY + jj * 2) = v;
        }
    }
}

// fragment of tap k (MFMA row), pixels 8*chunk .. +7; tap 49 = ones when `ones`, taps > 49 zero
__device__ __forceinline__ bf16x8 tap_frag(const char* Ts, int k, int chunk, bool ones) {
    if (k < KK) {
        const int kh = k / KS, kw = k - (k / KS) * KS;
        return *(const bf16x8*)(Ts + (((kw & 1) * 4 + (kw >> 1)) * KS + kh) * TCOPY + chunk * 16);
    }
    const __bf16 v = (__bf16)((ones && k == GONE) ? 1.f : 0.f);
    return (bf16x8){v, v, v, v, v, v, v, v};
}

__global__ __launch_bounds__(256) void stem_gram_kernel(const float* __restrict__ x, float* __restrict__ ws, int H,
                                                        int W, int Ho, int Wo, long M, int chunk) {
    __shared__ __attribute__((aligned(16))) char smem[2 * TSZ];
    const int tid = threadIdx.x;
    const int z = blockIdx.x;
    const long p0 = (long)z * chunk;
    const long p1 = min(M, p0 + chunk);
    const int lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, lg = lane >> 4;
    const int wm = wave >> 1, wn = wave & 1;
    f32x4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
    float pv[TPL];
    if (p0 < p1) tap_load(pv, x, H, W, Ho, Wo, p0, tid);
    int buf = 0;
    for (long ps = p0; ps < p1; ps += WPX, buf ^= 1) {
        char* Ts = smem + buf * TSZ;
        tap_store(Ts, pv, tid);                       // (double buffer: the last readers of Ts passed the previous barrier)
        if (ps + WPX < p1) tap_load(pv, x, H, W, Ho, Wo, ps + WPX, tid);
        __syncthreads();
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            bf16x8 ta[2], tb[2];
#pragma unroll
            for (int a = 0; a < 2; ++a) ta[a] = tap_frag(Ts, wm * 32 + a * 16 + l16, s * 4 + lg, true);
#pragma unroll
            for (int b = 0; b < 2; ++b) tb[b] = tap_frag(Ts, wn * 32 + b * 16 + l16, s * 4 + lg, true);
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tb[b], ta[a], acc[a][b], 0, 0, 0);
        }
    }
    // lane holds G[wm*32 + a*16 + l16][wn*32 + b*16 + 4lg .. +3]
    float* wz = ws + (size_t)z * 64 * 64;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
            *(f32x4*)(wz + (wm * 32 + a * 16 + l16) * 64 + wn * 32 + b * 16 + lg * 4) = acc[a][b];
}

// stats[0][0][co] += sum_p y = W[co] . s,  stats[0][1][co] += sum_p y^2 = W[co] G W[co]^T (fp64); one workgroup
// (one wave) per channel, lane k < 49 forms (G W[co]^T)[k]
__global__ __launch_bounds__(64) void stem_gram_stats_kernel(const float* __restrict__ G, const __bf16* __restrict__ wpk,
                                                             double* __restrict__ stats) {
    __shared__ double Ws[KK];
    const int co = blockIdx.x, k = threadIdx.x;
    if (k < KK) Ws[k] = (double)(float)wpk[co * 64 + k];
    __syncthreads();
    double s1 = 0.0, s2 = 0.0;
    if (k < KK) {
        double t = 0.0;
        for (int l = 0; l < KK; ++l) t += Ws[l] * (double)G[k * 64 + l];
        s2 = Ws[k] * t;
        s1 = Ws[k] * (double)G[k * 64 + GONE];
    }
    s1 = wave_sum_d(s1);
    s2 = wave_sum_d(s2);
    if (k == 0) {
        stats[co] += s1;
        stats[CO + co] += s2;
    }
}

// ---- fused forward: one workgroup = 2 pooled rows x 32 pooled cols; conv region 5 rows x 65 cols (+ the pool's
// top/left halo), MFMA over the 325 conv pixels as a flat list of 21 16-pixel blocks
constexpr int FPR = 2, FPC = 32;                        // pooled tile
constexpr int FCR = 2 * FPR + 1, FCC = 2 * FPC + 1;     // conv region 5 x 65
constexpr int FNP = FCR * FCC;                          // 325
constexpr int FNB = (FNP + 15) / 16;                    // 21 blocks
constexpr int FIR = SP * (FCR - 1) + KS;                // 15 input rows
constexpr int FIC = SP * (FCC - 1) + KS + 1;            // 136 input cols (135 used)
constexpr int FYROW = 144;                              // staged y row stride (128 B + 16): conflict-free 16-B reads

__global__ __launch_bounds__(256) void stem_fused_fwd_kernel(const float* __restrict__ x, const __bf16* __restrict__ wpk,
                                                             const float* __restrict__ scale,
                                                             const float* __restrict__ shift, __bf16* __restrict__ out,
                                                             uint8_t* __restrict__ argmax, __bf16* __restrict__ yam,
                                                             int H, int W, int Ho, int Wo, int Hp, int Wp) {
    // No im2col tile: with K ordered (kh, kw) and kw padded to 8, the A fragment of pixel (r, c) for K chunk kh is
    // the 8 consecutive bf16 patch[2r + kh][2c .. 2c + 7] (the 8th meets a zero weight).  The patch is kept as 4
    // copies shifted by 0/2/4/6 elements, so every fragment is one aligned 16-B LDS read.
    constexpr int PROW = FIC * 2;                       // 272 B per bf16 patch row
    constexpr int PT = 4 * FIR * PROW;                  // 16320 B
    constexpr int YT = FNP * FYROW;                     // 46800 B staged y (aliases patch + weights after the MFMAs)
    constexpr int U = YT > PT + CO * 128 ? YT : PT + CO * 128;
    __shared__ __attribute__((aligned(16))) char smem[U];
    char* Ps = smem;
    char* Bs = smem + PT;
    char* Ys = smem;

    const int tid = threadIdx.x;
    const int tiles_w = Wp / FPC, tiles_h = Hp / FPR;
    const int bid = blockIdx.x;
    const int n = bid / (tiles_h * tiles_w);
    const int rem = bid - n * tiles_h * tiles_w;
    const int pi0 = (rem / tiles_w) * FPR, pj0 = (rem - (rem / tiles_w) * tiles_w) * FPC;
    const int cr0 = 2 * pi0 - 1, cc0 = 2 * pj0 - 1;     // conv region origin (may be -1)
    const int ih0 = cr0 * SP - PD, iw0 = cc0 * SP - PD;

    // weights re-laid [co][kh*8 + kw] (kw = 7 and kh = 7 zero), 128-B swizzled rows
    for (int i = tid; i < CO * 64; i += 256) {
        const int co = i >> 6, kk = i & 63, kh = kk >> 3, kw = kk & 7;
        const __bf16 v = (kh < KS && kw < KS) ? wpk[co * 64 + kh * KS + kw] : (__bf16)0.f;
        *(__bf16*)(Bs + swz128(co, kk >> 3) + (kk & 7) * 2) = v;
    }
    {
        const float* xn = x + (size_t)n * H * W;
        for (int i = tid; i < FIR * FIC; i += 256) {
            const int r = i / FIC, c = i - (i / FIC) * FIC;
            const int ih = ih0 + r, iw = iw0 + c;
            const __bf16 v = (__bf16)(((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) ? xn[(size_t)ih * W + iw] : 0.f);
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (c - 2 * t >= 0) *(__bf16*)(Ps + (t * FIR + r) * PROW + (c - 2 * t) * 2) = v;
        }
    }
    __syncthreads();

    const int lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, lg = lane >> 4, l7 = l16 & 7;
    bf16x8 bfr[2][4];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int b = 0; b < 4; ++b) bfr[s][b] = *(const bf16x8*)(Bs + (b * 16 + l16) * 128 + (((s * 4 + lg) ^ l7) << 4));
    f32x4 acc[6][4];
    int nblk = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const int blk = wave + 4 * i;
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[i][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
        if (blk < FNB) {
            nblk = i + 1;
            const int p = min(blk * 16 + l16, FNP - 1);
            const int r = p / FCC, c = p - (p / FCC) * FCC;
            const char* pb = Ps + ((c & 3) * FIR + 2 * r) * PROW + (c >> 2) * 16;
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int kh = s * 4 + lg;
                const bf16x8 af = kh < KS ? *(const bf16x8*)(pb + kh * PROW) : (bf16x8){};
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    acc[i][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[s][b], af, acc[i][b], 0, 0, 0);
            }
        }
    }
    __syncthreads();                                    // patch dead: stage y (bf16, as the unfused kernel stores it)
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        if (i >= nblk) break;
        const int p = (wave + 4 * i) * 16 + l16;
        if (p < FNP) {
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
                bf16x4 o;
#pragma unroll
                for (int r = 0; r < 4; ++r) o[r] = (__bf16)acc[i][b][r];
                *(bf16x4*)(Ys + p * FYROW + (b * 16 + lg * 4) * 2) = o;
            }
        }
    }
    __syncthreads();
    // BN apply + ReLU + 3x3/s2 max-pool (stem_pool_fwd_kernel's rule: first strictly greater window position wins)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int item = tid + 256 * j;                 // 64 pooled px x 8 channel chunks
        const int pp = item >> 3, c = item & 7;
        const int pi = pp / FPC, pj = pp - (pp / FPC) * FPC;
        float sc[8], sh[8], best[8], yb[8];
        int arg[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            sc[e] = scale[c * 8 + e]; sh[e] = shift[c * 8 + e];
            best[e] = -INFINITY; arg[e] = 0; yb[e] = 0.f;
        }
#pragma unroll
        for (int di = 0; di < 3; ++di) {
            const int tr = 2 * pi + di, gr = cr0 + tr;
            if ((unsigned)gr >= (unsigned)Ho) continue;
#pragma unroll
            for (int dj = 0; dj < 3; ++dj) {
                const int tc = 2 * pj + dj, gc = cc0 + tc;
                if ((unsigned)gc >= (unsigned)Wo) continue;
                const bf16x8 v = *(const bf16x8*)(Ys + (tr * FCC + tc) * FYROW + c * 16);
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float yv = (float)v[e];
                    const float zz = fmaxf(yv * sc[e] + sh[e], 0.f);
                    if (zz > best[e]) { best[e] = zz; arg[e] = di * 3 + dj; yb[e] = yv; }
                }
            }
        }
        const size_t o = (((size_t)n * Hp + pi0 + pi) * Wp + pj0 + pj) * CO + c * 8;
        bf16x8 ov, yv8;
        uint8_t a8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) { ov[e] = (__bf16)best[e]; yv8[e] = (__bf16)yb[e]; a8[e] = (uint8_t)arg[e]; }
        *(bf16x8*)(out + o) = ov;
        *(bf16x8*)(yam + o) = yv8;
        *(uint2*)(argmax + o) = *(const uint2*)a8;
    }
}

// ---- backward weight gradient from the pooled side: stage = 64 conv pixels of one row; dz (pool + ReLU gradient)
// built from the pooled gradient / argmax / y-at-argmax, BN backward sums accumulated (stats, fp64 replicas).
// The stage's pooled neighbourhood (1 or 2 pooled rows x 33 columns: gradient, y-at-argmax, argmax) is read with
// coalesced 16-B loads into LDS (prefetched into registers one stage ahead, like the input patch), then every
// conv pixel gathers its <= 4 window candidates from LDS.
constexpr int PNC = WPX / 2 + 1;                       // 33 pooled columns
constexpr int PNCH = PNC * 20;                         // 16-B chunks per pooled row: 8 gradient + 8 y + 4 argmax per px
constexpr int PNL = (2 * PNCH + 255) / 256;            // chunks per thread (6)
constexpr int PN_D = 0, PN_Y = 2 * PNC * 128, PN_A = 4 * PNC * 128, PNSZ = PN_A + 2 * PNC * 64;   // 21120 B

struct PooledStage {
    int n, oh, ow0, nrows, ja0;
};

__device__ __forceinline__ PooledStage pooled_stage(long ps, int Ho, int Wo, int Hp) {
    PooledStage st;
    st.n = (int)(ps / ((long)Ho * Wo));
    const int rem = (int)(ps - (long)st.n * Ho * Wo);
    st.oh = rem / Wo;
    st.ow0 = rem - (rem / Wo) * Wo;
    st.nrows = ((st.oh & 1) && (st.oh >> 1) + 1 < Hp) ? 2 : 1;
    st.ja0 = st.ow0 >> 1;
    return st;
}

__device__ __forceinline__ void pooled_load(uint4 (&pr)[PNL], const __bf16* __restrict__ dout,
                                            const __bf16* __restrict__ yam, const uint8_t* __restrict__ argmax,
                                            const PooledStage& st, int Hp, int Wp, int tid) {
#pragma unroll
    for (int q = 0; q < PNL; ++q) {
        const int i = tid + 256 * q;
        const int ri = i / PNCH, k = i - (i / PNCH) * PNCH;
        int jl, off;
        const char* base;
        if (k < 2 * PNC * 8) {                         // gradient / y chunks: [kind][jl][8]
            const int kind = k / (PNC * 8), kk = k - kind * PNC * 8;
            jl = kk >> 3;
            off = (kk & 7) * 16;
            base = kind ? (const char*)yam : (const char*)dout;
            off += jl * 128;
            const long row = ((long)st.n * Hp + (st.oh >> 1) + ri) * Wp + st.ja0;
            base += row * 128;
        } else {                                       // argmax chunks: [jl][4]
            const int kk = k - 2 * PNC * 8;
            jl = kk >> 2;
            off = jl * 64 + (kk & 3) * 16;
            const long row = ((long)st.n * Hp + (st.oh >> 1) + ri) * Wp + st.ja0;
            base = (const char*)argmax + row * 64;
        }
        const bool ok = ri < st.nrows && st.ja0 + jl < Wp;
        pr[q] = ok ? *(const uint4*)(base + off) : make_uint4(0, 0, 0, 0);
    }
}

__device__ __forceinline__ void pooled_store(char* Pn, const uint4 (&pr)[PNL], int tid) {
#pragma unroll
    for (int q = 0; q < PNL; ++q) {
        const int i = tid + 256 * q;
        if (i >= 2 * PNCH) break;
        const int ri = i / PNCH, k = i - (i / PNCH) * PNCH;
        int dst;
        if (k < 2 * PNC * 8) {
            const int kind = k / (PNC * 8), kk = k - kind * PNC * 8;
            dst = (kind ? PN_Y : PN_D) + (ri * PNC + (kk >> 3)) * 128 + (kk & 7) * 16;
        } else {
            const int kk = k - 2 * PNC * 8;
            dst = PN_A + (ri * PNC + (kk >> 2)) * 64 + (kk & 3) * 16;
        }
        *(uint4*)(Pn + dst) = pr[q];
    }
}

__global__ __launch_bounds__(256) void stem_wgrad_pooled_kernel(const __bf16* __restrict__ dout, const uint8_t* __restrict__ argmax,
                                                                const __bf16* __restrict__ yam, const float* __restrict__ scale,
                                                                const float* __restrict__ shift, const float* __restrict__ mean,
                                                                const float* __restrict__ invstd, const float* __restrict__ x,
                                                                float* __restrict__ ws, double* __restrict__ stats, int H,
                                                                int W, int Ho, int Wo, int Hp, int Wp, long M, int chunk) {
    constexpr int DT = WPX * DROW;                     // 18432 B dz stage
    __shared__ __attribute__((aligned(16))) char smem[DT + 2 * TSZ + PNSZ];
    char* Ds = smem;
    char* Tb = smem + DT;
    char* Pn = smem + DT + 2 * TSZ;
    __shared__ float red[2][4][CO];
    __shared__ float bnp[4][CO];                        // scale, shift, mean, invstd (kept out of registers)

    const int tid = threadIdx.x;
    const int z = blockIdx.x;
    const long p0 = (long)z * chunk;
    const long p1 = min(M, p0 + chunk);
    const int lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, lg = lane >> 4;
    const int q4 = l16 >> 2, qq = l16 & 3;
    const int wm = wave >> 1, wn = wave & 1;
    const int cch = tid & 7;                            // this thread's channel chunk in every stage
    if (tid < CO) {
        bnp[0][tid] = scale[tid]; bnp[1][tid] = shift[tid]; bnp[2][tid] = mean[tid]; bnp[3][tid] = invstd[tid];
    }
    float s1[8], s2[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
    f32x4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
    typedef __attribute__((ext_vector_type(8))) short s16x8;

    float pv[TPL];
    uint4 pr[PNL];
    PooledStage st = pooled_stage(p0, Ho, Wo, Hp);
    if (p0 < p1) {
        tap_load(pv, x, H, W, Ho, Wo, p0, tid);
        pooled_load(pr, dout, yam, argmax, st, Hp, Wp, tid);
    }
    int buf = 0;
    for (long ps = p0; ps < p1; ps += WPX, buf ^= 1) {
        char* Ts = Tb + buf * TSZ;
        tap_store(Ts, pv, tid);
        pooled_store(Pn, pr, tid);
        const PooledStage cur = st;
        if (ps + WPX < p1) {
            st = pooled_stage(ps + WPX, Ho, Wo, Hp);
            tap_load(pv, x, H, W, Ho, Wo, ps + WPX, tid);
            pooled_load(pr, dout, yam, argmax, st, Hp, Wp, tid);
        }
        __syncthreads();
        // dz for (pixel r, chunk cch): window candidates (row slot, column) in (row, col) order; an even conv row /
        // column has one pooled row / column (window position 1), an odd one two (positions 2 then 0)
        const int dia = cur.oh & 1 ? 2 : 1;
#pragma unroll 1
        for (int j = 0; j < 2; ++j) {
            const int r = (tid + 256 * j) >> 3;
            const int ow = cur.ow0 + r;
            const int dja = ow & 1 ? 2 : 1;
            const bool hasb = cur.nrows == 2;
            const bool hasbj = (ow & 1) && (ow >> 1) + 1 < Wp;
            float accv[8], yv[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) { accv[e] = 0.f; yv[e] = 0.f; }
#pragma unroll
            for (int ci = 0; ci < 2; ++ci)
#pragma unroll
                for (int cj = 0; cj < 2; ++cj) {
                    const bool ok = (ci == 0 || hasb) && (cj == 0 || hasbj);
                    const int slot = ok ? ci * PNC + (r >> 1) + cj : (r >> 1);
                    const int sel = ok ? (ci ? 0 : dia) * 3 + (cj ? 0 : dja) : 255;
                    const bf16x8 d8 = *(const bf16x8*)(Pn + PN_D + slot * 128 + cch * 16);
                    const bf16x8 y8 = *(const bf16x8*)(Pn + PN_Y + slot * 128 + cch * 16);
                    uint8_t a8[8];
                    *(uint2*)a8 = *(const uint2*)(Pn + PN_A + slot * 64 + cch * 8);
#pragma unroll
                    for (int e = 0; e < 8; ++e)
                        if (a8[e] == sel) { accv[e] += (float)d8[e]; yv[e] = (float)y8[e]; }
                }
            bf16x8 stv;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int c = cch * 8 + e;
                const float dz = (yv[e] * bnp[0][c] + bnp[1][c] > 0.f) ? accv[e] : 0.f;
                stv[e] = (__bf16)dz;
                const float rr = (float)stv[e];
                s1[e] += rr;
                s2[e] += rr * (yv[e] - bnp[2][c]) * bnp[3][c];
            }
            *(bf16x8*)(Ds + dswz(r, cch * 16)) = stv;
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int r0 = 32 * s + 8 * lg + q4;
            bf16x8 tf[2], df[2];
#pragma unroll
            for (int b = 0; b < 2; ++b) tf[b] = tap_frag(Ts, wn * 32 + b * 16 + l16, s * 4 + lg, false);
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                const int cb = (wm * 32 + a * 16 + 4 * qq) * 2;
                s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Ds + dswz(r0, cb)));
                s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Ds + dswz(r0 + 4, cb)));
                s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                df[a] = __builtin_bit_cast(bf16x8, v);
            }
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tf[b], df[a], acc[a][b], 0, 0, 0);
        }
    }
    float* wz = ws + (size_t)z * CO * 64;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
            *(f32x4*)(wz + (wm * 32 + a * 16 + l16) * 64 + wn * 32 + b * 16 + lg * 4) = acc[a][b];
    // BN backward sums: lanes with equal (lane & 7) share channels; then the 4 waves through LDS
#pragma unroll
    for (int e = 0; e < 8; ++e) {
#pragma unroll
        for (int o = 8; o < 64; o <<= 1) { s1[e] += __shfl_xor(s1[e], o, 64); s2[e] += __shfl_xor(s2[e], o, 64); }
    }
    if (lane < 8) {
#pragma unroll
        for (int e = 0; e < 8; ++e) { red[0][wave][lane * 8 + e] = s1[e]; red[1][wave][lane * 8 + e] = s2[e]; }
    }
    __syncthreads();
    if (tid < 2 * CO) {
        const int sti = tid / CO, c = tid - (tid / CO) * CO;
        double a = 0.0;
#pragma unroll
        for (int w = 0; w < 4; ++w) a += red[sti][w][c];
        atomic_add_f64(stats + ((long)(z % SCD_STAT_REPLICAS) * 2 + sti) * CO + c, a);
    }
}

// dW[co][k] (+)= a[co] * sum_z ws[z][co][k] + b[co] * (W G)[co][k] + c[co] * s[k]   (k < 49; one workgroup per co)
__global__ __launch_bounds__(256) void stem_wgrad_combine_kernel(const float* __restrict__ ws, int nsplit,
                                                                 const float* __restrict__ coef,
                                                                 const float* __restrict__ G,
                                                                 const __bf16* __restrict__ wpk, float* __restrict__ dst,
                                                                 int accumulate) {
    __shared__ float part[4][64];
    const int co = blockIdx.x, tid = threadIdx.x;
    const int k = tid & 63, g = tid >> 6;
    float t = 0.f;
    for (int z = g; z < nsplit; z += 4) t += ws[((size_t)z * CO + co) * 64 + k];
    part[g][k] = t;
    __syncthreads();
    if (tid < KK) {
        const float t1 = part[0][k] + part[1][k] + part[2][k] + part[3][k];
        double wg = 0.0;
        for (int l = 0; l < KK; ++l) wg += (double)(float)wpk[co * 64 + l] * (double)G[l * 64 + k];
        const float v = (float)((double)coef[co] * t1 + (double)coef[CO + co] * wg + (double)coef[2 * CO + co] * G[k * 64 + GONE]);
        float* d = dst + co * KK + k;
        *d = accumulate ? *d + v : v;
    }
}

SCD_KERNEL_NS_END
}  // namespace

extern "C" int scd_stem_conv_fwd(int dtype, const float* x, const void* wpk, void* y, double* stats, int N, int H,
                                 int W, int Ho, int Wo, void* stream) {
    SCD_F16_FWD(scd_stem_conv_fwd, x, wpk, y, stats, N, H, W, Ho, Wo, stream);
    if (dtype != SCD_DT_BF16 || N <= 0 || Ho != (H + 2 * PD - KS) / SP + 1 || Wo != (W + 2 * PD - KS) / SP + 1 ||
        Wo % FTW || Ho % FTH)
        return SCD_ERR_ARG;
    const int blocks = N * (Ho / FTH) * (Wo / FTW);
    hipLaunchKernelGGL(stem_conv_fwd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, (const __bf16*)wpk,
                       (__bf16*)y, stats, H, W, Ho, Wo);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_stem_conv_wgrad_nsplit(long M) {
    // ~4 resident workgroups per CU, whole 64-pixel stages per split
    long ns = std::min(2048L, std::max(1L, M / (4 * WPX)));
    return (int)ns;
}

extern "C" int scd_stem_conv_wgrad(int dtype, const void* dy, const void* ybn, const float* coef, const float* x,
                                   float* ws, int nsplit, int N, int H, int W, int Ho, int Wo, void* stream) {
    SCD_F16_FWD(scd_stem_conv_wgrad, dy, ybn, coef, x, ws, nsplit, N, H, W, Ho, Wo, stream);
    if (dtype != SCD_DT_BF16 || nsplit < 1 || Wo % WPX || Ho != (H + 2 * PD - KS) / SP + 1 ||
        Wo != (W + 2 * PD - KS) / SP + 1)
        return SCD_ERR_ARG;
    const long M = (long)N * Ho * Wo;
    long chunk = (M + nsplit - 1) / nsplit;
    chunk = (chunk + WPX - 1) / WPX * WPX;
    if (chunk >= (1L << 31)) return SCD_ERR_ARG;
    if (coef && !ybn) return SCD_ERR_ARG;
    hipLaunchKernelGGL(stem_conv_wgrad_kernel, dim3(nsplit), dim3(256), 0, (hipStream_t)stream, (const __bf16*)dy,
                       (const __bf16*)ybn, coef, x, ws, H, W, Ho, Wo, M, (int)chunk);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_stem_gram(const float* x, float* ws, int nsplit, int N, int H, int W, int Ho, int Wo, void* stream) {
    if (nsplit < 1 || N <= 0 || Wo % WPX || Ho != (H + 2 * PD - KS) / SP + 1 || Wo != (W + 2 * PD - KS) / SP + 1)
        return SCD_ERR_ARG;
    const long M = (long)N * Ho * Wo;
    long chunk = (M + nsplit - 1) / nsplit;
    chunk = (chunk + WPX - 1) / WPX * WPX;
    if (chunk >= (1L << 31)) return SCD_ERR_ARG;
    hipLaunchKernelGGL(stem_gram_kernel, dim3(nsplit), dim3(256), 0, (hipStream_t)stream, x, ws, H, W, Ho, Wo, M,
                       (int)chunk);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_stem_gram_stats(const float* G, const void* wpk, double* stats, void* stream) {
    hipLaunchKernelGGL(stem_gram_stats_kernel, dim3(CO), dim3(64), 0, (hipStream_t)stream, G, (const __bf16*)wpk, stats);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_stem_fused_fwd(const float* x, const void* wpk, const float* scale, const float* shift, void* out,
                                  uint8_t* argmax, void* yam, int N, int H, int W, int Ho, int Wo, int Hp, int Wp,
                                  void* stream) {
    if (N <= 0 || Ho != (H + 2 * PD - KS) / SP + 1 || Wo != (W + 2 * PD - KS) / SP + 1 || Hp != (Ho - 1) / 2 + 1 ||
        Wp != (Wo - 1) / 2 + 1 || Hp % FPR || Wp % FPC)
        return SCD_ERR_ARG;
    const int blocks = N * (Hp / FPR) * (Wp / FPC);
    hipLaunchKernelGGL(stem_fused_fwd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, (const __bf16*)wpk,
                       scale, shift, (__bf16*)out, argmax, (__bf16*)yam, H, W, Ho, Wo, Hp, Wp);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_stem_wgrad_pooled(const void* dout, const uint8_t* argmax, const void* yam, const float* scale,
                                     const float* shift, const float* mean, const float* invstd, const float* x,
                                     float* ws, double* stats, int nsplit, int N, int H, int W, int Ho, int Wo, int Hp,
                                     int Wp, void* stream) {
    if (nsplit < 1 || N <= 0 || Wo % WPX || Ho != (H + 2 * PD - KS) / SP + 1 || Wo != (W + 2 * PD - KS) / SP + 1 ||
        Hp != (Ho - 1) / 2 + 1 || Wp != (Wo - 1) / 2 + 1)
        return SCD_ERR_ARG;
    const long M = (long)N * Ho * Wo;
    long chunk = (M + nsplit - 1) / nsplit;
    chunk = (chunk + WPX - 1) / WPX * WPX;
    if (chunk >= (1L << 31)) return SCD_ERR_ARG;
    hipLaunchKernelGGL(stem_wgrad_pooled_kernel, dim3(nsplit), dim3(256), 0, (hipStream_t)stream, (const __bf16*)dout,
                       argmax, (const __bf16*)yam, scale, shift, mean, invstd, x, ws, stats, H, W, Ho, Wo, Hp, Wp, M,
                       (int)chunk);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_stem_wgrad_combine(const float* ws, int nsplit, const float* coef, const float* G, const void* wpk,
                                      float* dst, int accumulate, void* stream) {
    if (nsplit < 1) return SCD_ERR_ARG;
    hipLaunchKernelGGL(stem_wgrad_combine_kernel, dim3(CO), dim3(256), 0, (hipStream_t)stream, ws, nsplit, coef, G,
                       (const __bf16*)wpk, dst, accumulate);
    SCD_RETURN_LAUNCH();
}
