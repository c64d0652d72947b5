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
