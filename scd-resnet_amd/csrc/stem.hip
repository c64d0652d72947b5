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

// sum over the 16 lanes of a DPP row (quad butterflies, then the half-row and row mirrors): VALU only, where
// __shfl_xor costs an LDS permute per step
__device__ __forceinline__ float stem_row16_sum(float v) {
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, true));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, true));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, true));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, true));
    return v;
}

// ---- forward: one workgroup = 2 output rows x 128 output columns (256 pixels) of one image
constexpr int FTW = 128, FTH = 2;
// workgroups per CU the forward conv is compiled for (registers); its LDS (49 KB) admits 3
#ifndef STEM_FWD_OCC
#define STEM_FWD_OCC 3
#endif
constexpr int PROWS = SP * (FTH - 1) + KS;          // 9 input rows
constexpr int PCOLS = SP * (FTW - 1) + KS + 1;      // 262 -> padded to an even count
// the forward's input patch in LDS with each row split by column parity (as the backward's, bpatch_idx): the 64 lanes
// of a wave (64 consecutive pixels) then read 64 consecutive floats per tap instead of every other one (2-way bank
// conflicts on every tap read of the im2col build)
constexpr int FPAR = 132;                            // >= 131 columns per parity
constexpr int FROW = 2 * FPAR;

__global__ __launch_bounds__(256, STEM_FWD_OCC) void stem_conv_fwd_kernel(const float* __restrict__ x, const h16* __restrict__ wpk,
                                                            h16* __restrict__ y, double* __restrict__ stats,
                                                            int H, int W, int Ho, int Wo) {
    constexpr int AT = FTH * FTW * 128;             // A tile [256 px][64 taps] bf16, 128-B rows
    constexpr int BT = CO * 128;                    // B tile [64 co][64 taps]
    constexpr int EROW = CO * 2 + 16;
    __shared__ __attribute__((aligned(16))) char smem[AT + BT + PROWS * FROW * 4];
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
    // input patch (zero outside the image): a fixed number of loads per thread from clamped addresses, all in flight
    // at once (a bounds branch around each load made the compiler wait for every one before the next)
    const float* xn = x + (size_t)n * H * W;
    constexpr int PN = (PROWS * PCOLS + 255) / 256;
    float pv[PN];
#pragma unroll
    for (int j = 0; j < PN; ++j) {
        const int i = min(tid + 256 * j, PROWS * PCOLS - 1);
        const int r = i / PCOLS, c = i - (i / PCOLS) * PCOLS;
        const int ih = min(max(ih0 + r, 0), H - 1), iw = min(max(iw0 + c, 0), W - 1);
        pv[j] = xn[(size_t)ih * W + iw];
    }
#pragma unroll
    for (int j = 0; j < PN; ++j) {
        const int i = tid + 256 * j;
        if (i < PROWS * PCOLS) {
            const int r = i / PCOLS, c = i - (i / PCOLS) * PCOLS;
            const int ih = ih0 + r, iw = iw0 + c;
            patch[r * FROW + (c & 1) * FPAR + (c >> 1)] =
                ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) ? pv[j] : 0.f;
        }
    }
    __syncthreads();
    // im2col tile: thread -> pixel p = tid, all 64 taps (8 chunks of 8)
    {
        const int pr = tid / FTW, pc = tid - (tid / FTW) * FTW;
        const float* pp = patch + (SP * pr) * FROW + pc;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            h16x8 v;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int k = c * 8 + e;
                v[e] = (h16)(k < KK ? pp[(k / KS) * FROW + ((k % KS) & 1) * FPAR + ((k % KS) >> 1)] : 0.f);
            }
            *(h16x8*)(As + swz128(tid, c)) = v;
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
        h16x8 af[4], bfr[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) af[a] = *(const h16x8*)(As + (wave * 64 + a * 16 + l16) * 128 + co);
#pragma unroll
        for (int b = 0; b < 4; ++b) bfr[b] = *(const h16x8*)(Bs + (b * 16 + l16) * 128 + co);
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b)
                acc[a][b] = mfma_16x16x32_h16(bfr[b], af[a], acc[a][b]);
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
            typedef __attribute__((ext_vector_type(4))) h16 bf16x4;
            bf16x4 o;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float v = acc[a][b][r];
                o[r] = (h16)v;
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
                const float s = stem_row16_sum(csum[b][r]), q = stem_row16_sum(csq[b][r]);
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

__global__ __launch_bounds__(256) void stem_conv_wgrad_kernel(const h16* __restrict__ dy, const h16* __restrict__ ybn,
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
                const h16x8 d8 = __builtin_bit_cast(h16x8, v), y8 = __builtin_bit_cast(h16x8, yv);
                h16x8 o8;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const int ch = c * 8 + e;
                    o8[e] = (h16)(coef[ch] * (float)d8[e] + coef[CO + ch] * (float)y8[e] + coef[2 * CO + ch]);
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
                h16x8 v;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const int px = pq * 16 + h * 8 + e;
                    v[e] = (h16)(k < KK ? patch[kh * WPCOLS + SP * px + kw] : 0.f);
                }
                *(h16x8*)(Cs + swz128(k, pq * 2 + h)) = v;
            }
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            // A (taps, 8 consecutive pixels) from the [tap][px] tile; B (channels, 8 consecutive pixels) by tr reads
            const int r0 = 32 * s + 8 * lg + q4;
            h16x8 tf[2], df[2];
#pragma unroll
            for (int b = 0; b < 2; ++b)
                tf[b] = *(const h16x8*)(Cs + swz128(wn * 32 + b * 16 + l16, s * 4 + lg));
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                const int cb = (wm * 32 + a * 16 + 4 * pp) * 2;
                s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Ds + dswz(r0, cb)));
                s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Ds + dswz(r0 + 4, cb)));
                s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                df[a] = __builtin_bit_cast(h16x8, v);
            }
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    acc[a][b] = mfma_16x16x32_h16(tf[b], df[a], acc[a][b]);
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


// ---- stem backward in one pass over the pooled gradient (residuals.py:209-216 backward; BN layer :212)
// With dz = the MaxPool + ReLU gradient at the conv output and the BN backward apply dy = a*dz + b*y + c
// (scd_bn_bwd_finalize's coefficients, which need the batch sums of dz and dz*xhat first), the weight gradient is
//     dW = sum_p dy[p] col[p]^T = a * T1 + b * W G + c * s,   T1 = sum_p dz[p] col[p]^T,  G = sum_p col[p] col[p]^T,
// s = sum_p col[p] (tap 49 of col is 1, so s = G[.][49]).  One pass therefore rebuilds dz per 2x2 conv block from
// the pooled gradient / argmax / y (as stem_pool_bwd_bn_2x2_kernel), accumulates the BN backward sums, and runs the
// T1 and G MFMAs on an LDS tile of dz and the [tap][pixel] input columns: dz is never written to HBM and y is read
// once (the unfused backward wrote dz and read it, and y, again).  Tile = 2 conv rows x 64 columns (32 2x2 blocks
// x 8 channel chunks = one item per thread).  W G uses the conv's bf16 weights in fp32 (the forward multiplied
// the same operands), so dW matches the unfused path up to the bf16 rounding of y and dy that it no longer has.
constexpr int BTW = 64;                              // conv columns per tile (two conv rows per tile)
// The backward's input patch in LDS with each row split by column parity (even columns at 0.., odd at PPAR..) and rows
// PROW floats apart: tap (kh, kw) of pixel px reads row kh at parity kw & 1, index px + kw / 2, so the 16 taps x 4
// pixel groups of a wave's column-build read hit 64 distinct banks but for a few taps of a third kernel row (row
// offsets 4 (mod 16) apart, parities 8 apart); the plain layout (column 2 px + kw, rows 134 apart) averaged ~4
// bank-conflict cycles per LDS instruction in this kernel (profiles/r4_sq_stem.txt)
constexpr int PPAR = 72;                             // >= 67 columns per parity, = 8 (mod 16)
constexpr int PROW = 148;                            // >= PPAR + 67, = 4 (mod 16)
__device__ __forceinline__ int bpatch_idx(int r, int c) { return r * PROW + (c & 1) * PPAR + (c >> 1); }
constexpr int BPROWS = 9;                            // input rows of a tile: conv rows 2bo, 2bo+1 -> 4bo-3 .. 4bo+5
constexpr int ONE_TAP = KK;                          // col tap 49 = 1

__global__ __launch_bounds__(256, 2) void stem_bwd_fused_kernel(
    const h16* __restrict__ dout, const uint8_t* __restrict__ argmax, const h16* __restrict__ y,
    const float* __restrict__ scale, const float* __restrict__ shift, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ x, double* __restrict__ stats, float* __restrict__ ws,
    int H, int W, int Ho, int Wo, int ntiles, int chunk) {
    constexpr int DT = WPX * DROW;                   // one conv row of dz: [64 px][DROW]
    constexpr int CT = 64 * 128;                     // one conv row of columns: [64 taps][64 px] bf16
    __shared__ __attribute__((aligned(16))) char smem[2 * DT + 2 * CT + BPROWS * PROW * 4];
    // the BN parameters in LDS ([scale | shift | mean | invstd][64]), read per 2x2 block: 32 VGPRs fewer than holding
    // each thread's 8 channels of all four in registers (the kernel sits at its 256-VGPR bound)
    __shared__ __attribute__((aligned(16))) float prm[4 * CO];
    char* Ds = smem;
    char* Cs = smem + 2 * DT;
    float* patch = (float*)(smem + 2 * DT + 2 * CT);

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, lg = lane >> 4;
    const int q4 = l16 >> 2, pp = l16 & 3;
    const int wm = wave >> 1, wn = wave & 1;
    const int Hp = Ho / 2, Wp = Wo / 2;
    const int gpr = Wo / BTW;                        // column groups per conv row pair
    const int tpi = Hp * gpr;
    const int bl = tid >> 3, ch = tid & 7;           // this thread's 2x2 block of the tile and channel chunk
    typedef __attribute__((ext_vector_type(8))) short s16x8;

    float s1[8], s2[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
    if (tid < CO) {
        prm[tid] = scale[tid]; prm[CO + tid] = shift[tid]; prm[2 * CO + tid] = mean[tid]; prm[3 * CO + tid] = invstd[tid];
    }
    __syncthreads();
    f32x4 acc1[2][2], acc2[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) { acc1[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f}; acc2[a][b] = acc1[a][b]; }

    const int t0 = blockIdx.x * chunk, t1 = min(ntiles, t0 + chunk);
    // raw operands of one tile, loaded one tile ahead (issued as soon as the previous tile's are consumed).  Tiles run
    // down a column group (t = (n, column group jc, pooled row bo), bo fastest), so the pooled row bo + 1 of a tile is
    // row bo of the next one: carried in registers instead of fetched again (each pooled row was read by two tiles:
    // PMC 1.34x the algorithmic bytes of this kernel; ~1.1x with the carry)
    uint4 rd[2][2], ry[2][2];
    uint2 ra[2][2];
    float rp[(BPROWS * WPCOLS + 255) / 256];
    auto load_tile = [&](int t, bool carry) {
        const int n = t / tpi, rem = t - (t / tpi) * tpi;
        const int jc = rem / Hp, bo = rem - (rem / Hp) * Hp;
        const int w0 = jc * BTW, bc = jc * (BTW / 2) + bl;
        const bool okh = bo + 1 < Hp, okw = bc + 1 < Wp;
        if (carry) {                                      // workgroup-uniform
#pragma unroll
            for (int oj = 0; oj < 2; ++oj) { rd[0][oj] = rd[1][oj]; ra[0][oj] = ra[1][oj]; }
        }
#pragma unroll
        for (int oi = 0; oi < 2; ++oi)
#pragma unroll
            for (int oj = 0; oj < 2; ++oj) {
                if (oi == 0 && carry) continue;
                const bool ok = (oi == 0 || okh) && (oj == 0 || okw);
                const long o = (((long)n * Hp + bo + (ok ? oi : 0)) * Wp + bc + (ok ? oj : 0)) * CO + ch * 8;
                rd[oi][oj] = *(const uint4*)(dout + o);
                const uint2 av = *(const uint2*)(argmax + o);        // o is in range either way: no branch
                ra[oi][oj] = ok ? av : make_uint2(0xffffffffu, 0xffffffffu);
            }
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
                ry[a][b] = *(const uint4*)(y + (((long)n * Ho + 2 * bo + a) * Wo + 2 * bc + b) * CO + ch * 8);
        const float* xn = x + (size_t)n * H * W;
        const int ih0 = 4 * bo - PD, iw0 = 2 * w0 - PD;
#pragma unroll
        for (int q = 0; q < (BPROWS * WPCOLS + 255) / 256; ++q) {
            const int i = tid + 256 * q;
            const int ic = min(i, BPROWS * WPCOLS - 1);
            const int r = ic / WPCOLS, c = ic - (ic / WPCOLS) * WPCOLS;
            const int ih = ih0 + r, iw = iw0 + c;
            // unconditional load from a clamped address, then the select (a load under the bounds test would be a
            // branch, and the compiler then waits for it before the next one)
            const float v = xn[(size_t)min(max(ih, 0), H - 1) * W + min(max(iw, 0), W - 1)];
            rp[q] = (i < BPROWS * WPCOLS && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) ? v : 0.f;
        }
    };
    if (t0 < t1) load_tile(t0, false);
    for (int t = t0; t < t1; ++t) {
        // ---- dz of the 2x2 conv block (2bo + a, 2bc + b), channels 8ch .. 8ch+7
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                float g[8], v[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) g[e] = 0.f;
                const uint4 yb = ry[a][b];
#pragma unroll
                for (int oi = 0; oi < 2; ++oi)
#pragma unroll
                    for (int oj = 0; oj < 2; ++oj) {
                        if (oi > a || oj > b) continue;
                        const unsigned sel = (a - 2 * oi + 1) * 3 + (b - 2 * oj + 1);
                        float d[8];
                        Vec16<h16>::load(&rd[oi][oj], d);
                        const unsigned aw[2] = {ra[oi][oj].x, ra[oi][oj].y};
#pragma unroll
                        for (int e = 0; e < 8; ++e) {
                            const bool hit = ((aw[e >> 2] >> (8 * (e & 3))) & 0xffu) == sel;
                            // a select, not a branch (as `if (hit) g += d` the compiler emitted 63 exec-masked
                            // branch regions per tile); g is never -0, so adding +0 leaves it unchanged
                            g[e] += hit ? d[e] : 0.f;
                        }
                    }
                Vec16<h16>::load(&yb, v);
                float sc[8], sh[8], mu[8], is[8];
                *(float4*)sc = *(const float4*)(prm + ch * 8); *(float4*)(sc + 4) = *(const float4*)(prm + ch * 8 + 4);
                *(float4*)sh = *(const float4*)(prm + CO + ch * 8);
                *(float4*)(sh + 4) = *(const float4*)(prm + CO + ch * 8 + 4);
                *(float4*)mu = *(const float4*)(prm + 2 * CO + ch * 8);
                *(float4*)(mu + 4) = *(const float4*)(prm + 2 * CO + ch * 8 + 4);
                *(float4*)is = *(const float4*)(prm + 3 * CO + ch * 8);
                *(float4*)(is + 4) = *(const float4*)(prm + 3 * CO + ch * 8 + 4);
                h16x8 o8;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    o8[e] = (h16)(v[e] * sc[e] + sh[e] > 0.f ? g[e] : 0.f);
                    const float r = (float)o8[e];
                    s1[e] += r;
                    s2[e] += r * (v[e] - mu[e]) * is[e];
                }
                *(h16x8*)(Ds + a * DT + dswz(2 * bl + b, ch * 16)) = o8;
            }
#pragma unroll
        for (int q = 0; q < (BPROWS * WPCOLS + 255) / 256; ++q) {
            const int i = tid + 256 * q;
            if ((q + 1) * 256 <= BPROWS * WPCOLS || i < BPROWS * WPCOLS) {   // (only the last q can be partial)
                const int r = i / WPCOLS, c = i - (i / WPCOLS) * WPCOLS;
                patch[bpatch_idx(r, c)] = rp[q];
            }
        }
        if (t + 1 < t1) load_tile(t + 1, (t + 1) % Hp != 0);      // in flight during this tile's column build and MFMAs
        __syncthreads();
        // ---- transposed column tiles of both conv rows: thread -> tap k = tid / 4, pixels 16 (tid % 4) .. +15
        {
            const int k = tid >> 2, pq = tid & 3;
            // taps >= KK read tap KK-1's address and drop it: an LDS read under `k < KK` became an exec-masked
            // branch per read (32 per tile)
            const int kc = min(k, KK - 1);
            const int kh = kc / KS, kw = kc - (kc / KS) * KS;
            const float kfill = k == ONE_TAP ? 1.f : 0.f;
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    h16x8 v;
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const int px = pq * 16 + h * 8 + e;
                        const float pv = patch[(2 * a + kh) * PROW + (kw & 1) * PPAR + px + (kw >> 1)];
                        v[e] = (h16)(k < KK ? pv : kfill);
                    }
                    *(h16x8*)(Cs + a * CT + swz128(k, pq * 2 + h)) = v;
                }
        }
        __syncthreads();
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            const char* D = Ds + a * DT;
            const char* C = Cs + a * CT;
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int r0 = 32 * s + 8 * lg + q4;
                h16x8 tf[2], df[2], gf[2];
#pragma unroll
                for (int b = 0; b < 2; ++b) tf[b] = *(const h16x8*)(C + swz128(wn * 32 + b * 16 + l16, s * 4 + lg));
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    gf[i] = *(const h16x8*)(C + swz128(wm * 32 + i * 16 + l16, s * 4 + lg));
                    const int cb = (wm * 32 + i * 16 + 4 * pp) * 2;
                    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(D + dswz(r0, cb)));
                    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(D + dswz(r0 + 4, cb)));
                    s16x8 v8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                    df[i] = __builtin_bit_cast(h16x8, v8);
                }
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int b = 0; b < 2; ++b) {
                        acc1[i][b] = mfma_16x16x32_h16(tf[b], df[i], acc1[i][b]);
                        acc2[i][b] = mfma_16x16x32_h16(tf[b], gf[i], acc2[i][b]);
                    }
            }
        }
        __syncthreads();                             // tiles read before the next tile overwrites them
    }
    // ---- partial T1 (channel rows) and G (tap rows) of this split; lane holds columns (taps) wn*32 + b*16 + 4lg ..
    float* wz = ws + (size_t)blockIdx.x * 2 * CO * 64;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            *(f32x4*)(wz + (wm * 32 + i * 16 + l16) * 64 + wn * 32 + b * 16 + lg * 4) = acc1[i][b];
            *(f32x4*)(wz + CO * 64 + (wm * 32 + i * 16 + l16) * 64 + wn * 32 + b * 16 + lg * 4) = acc2[i][b];
        }
    // ---- BN backward sums: threads with equal tid % 8 hold the same channels
    float* red = (float*)smem;                        // [2][256][9]
#pragma unroll
    for (int e = 0; e < 8; ++e) { red[tid * 9 + e] = s1[e]; red[(256 + tid) * 9 + e] = s2[e]; }
    __syncthreads();
    if (tid < 2 * CO) {
        const int stat = tid / CO, c = tid - (tid / CO) * CO;
        const int cc = c / 8, e = c - (c / 8) * 8;
        double acc = 0.0;
        for (int t = cc; t < 256; t += 8) acc += red[(stat * 256 + t) * 9 + e];
        atomic_add_f64(stats + ((long)(blockIdx.x % SCD_STAT_REPLICAS) * 2 + stat) * CO + c, acc);
    }
}

// sum of the per-split [T1 | G] slabs in a fixed order: workgroup = 32 consecutive elements x 8 split lanes (each
// summing every 8th split in order), the 8 partials combined in order in fp64
__global__ __launch_bounds__(256) void stem_bwd_reduce_kernel(const float* __restrict__ ws, int nsplit,
                                                              float* __restrict__ out) {
    const int col = threadIdx.x & 31, lane8 = threadIdx.x >> 5;
    const int i = blockIdx.x * 32 + col;
    double a = 0.0;
    int z = lane8;
    for (; z + 56 < nsplit; z += 64) {               // 8 independent loads in flight, summed in split order
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = ws[(size_t)(z + 8 * u) * 2 * CO * 64 + i];
#pragma unroll
        for (int u = 0; u < 8; ++u) a += v[u];
    }
    for (; z < nsplit; z += 8) a += ws[(size_t)z * 2 * CO * 64 + i];
    __shared__ double part[8][32];
    part[lane8][col] = a;
    __syncthreads();
    if (lane8 == 0) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k) t += part[k][col];
        out[i] = (float)t;
    }
}

// dst[co][k] (+)= alpha (a[co] T1[co][k] + b[co] (W G)[co][k] + c[co] G[k][49]) for the 49 taps, W = the conv's bf16
// weights (wpk rows [co][64], taps >= 49 zero); one workgroup per output channel
__global__ __launch_bounds__(64) void stem_bwd_combine_kernel(const float* __restrict__ tg, const h16* __restrict__ wpk,
                                                              const float* __restrict__ coef, float* __restrict__ dst,
                                                              int accumulate, float alpha) {
    const int co = blockIdx.x, k = threadIdx.x;
    const float* T1 = tg;
    const float* G = tg + CO * 64;
    __shared__ float wrow[64];
    wrow[k] = k < KK ? (float)wpk[co * 64 + k] : 0.f;
    __syncthreads();
    if (k >= KK) return;
    double wg = 0.0;
    for (int l = 0; l < KK; ++l) wg += (double)wrow[l] * (double)G[l * 64 + k];
    const double v = (double)coef[co] * T1[co * 64 + k] + (double)coef[CO + co] * wg + (double)coef[2 * CO + co] * G[k * 64 + ONE_TAP];
    float* d = dst + co * KK + k;
    *d = (accumulate ? *d : 0.f) + alpha * (float)v;
}


SCD_KERNEL_NS_END
}  // namespace

extern "C" int scd_stem_conv_fwd(int dtype, const float* x, const void* wpk, void* y, double* stats, int N, int H,
                                 int W, int Ho, int Wo, void* stream) {
    SCD_F16_FWD(scd_stem_conv_fwd, x, wpk, y, stats, N, H, W, Ho, Wo, stream);
    if (dtype != SCD_DT_BF16 || N <= 0 || Ho != (H + 2 * PD - KS) / SP + 1 || Wo != (W + 2 * PD - KS) / SP + 1 ||
        Wo % FTW || Ho % FTH || !y)
        return SCD_ERR_ARG;
    // one workgroup per tile (a resident-grid walk with the next tile's patch in flight and the weights in registers
    // measured slower, 121 vs 106 us: the kernel is bound by its LDS / VALU tile build, not by load latency)
    const int blocks = N * (Ho / FTH) * (Wo / FTW);
    hipLaunchKernelGGL(stem_conv_fwd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, (const h16*)wpk,
                       (h16*)y, stats, H, W, Ho, Wo);
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
    hipLaunchKernelGGL(stem_conv_wgrad_kernel, dim3(nsplit), dim3(256), 0, (hipStream_t)stream, (const h16*)dy,
                       (const h16*)ybn, coef, x, ws, H, W, Ho, Wo, M, (int)chunk);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_stem_bwd_nsplit(void) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    return 2 * cus;
}

extern "C" int scd_stem_bwd_fused(int dtype, const void* dout, const uint8_t* argmax, const void* y, const float* scale,
                                  const float* shift, const float* mean, const float* invstd, const float* x,
                                  double* stats, float* ws, int nsplit, float* tg, int N, int H, int W, int Ho, int Wo,
                                  void* stream) {
    SCD_F16_FWD(scd_stem_bwd_fused, dout, argmax, y, scale, shift, mean, invstd, x, stats, ws, nsplit, tg, N, H, W, Ho,
                Wo, stream);
    if (dtype != SCD_DT_BF16 || nsplit < 1 || Wo % BTW || Ho % 2 || Ho != (H + 2 * PD - KS) / SP + 1 ||
        Wo != (W + 2 * PD - KS) / SP + 1 || (long)N * Ho * Wo * CO >= (1L << 31))
        return SCD_ERR_ARG;
    const int ntiles = N * (Ho / 2) * (Wo / BTW);
    const int chunk = (ntiles + nsplit - 1) / nsplit;
    const int grid = (ntiles + chunk - 1) / chunk;
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(stem_bwd_fused_kernel, dim3(grid), dim3(256), 0, st, (const h16*)dout, argmax,
                       (const h16*)y, scale, shift, mean, invstd, x, stats, ws, H, W, Ho, Wo, ntiles, chunk);
    hipLaunchKernelGGL(stem_bwd_reduce_kernel, dim3(2 * CO * 64 / 32), dim3(256), 0, st, (const float*)ws, grid, tg);
    SCD_RETURN_LAUNCH();
}


extern "C" int scd_stem_bwd_combine(int dtype, const float* tg, const void* wpk, const float* coef, float* dst,
                                    int accumulate, float alpha, void* stream) {
    SCD_F16_FWD(scd_stem_bwd_combine, tg, wpk, coef, dst, accumulate, alpha, stream);
    if (dtype != SCD_DT_BF16) return SCD_ERR_ARG;
    hipLaunchKernelGGL(stem_bwd_combine_kernel, dim3(CO), dim3(64), 0, (hipStream_t)stream, tg, (const h16*)wpk,
                       coef, dst, accumulate, alpha);
    SCD_RETURN_LAUNCH();
}
