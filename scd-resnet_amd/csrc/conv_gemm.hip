// Implicit-GEMM convolution family on CDNA4 MFMA (gfx950).
//
// One gather-GEMM covers Conv2d fwd, Conv2d dgrad (sub-pixel phases for stride 2),
// ConvTranspose2d fwd (4 phases) and ConvTranspose2d dgrad.  Activations are NHWC, the
// weight operand is a packed [Co][taps][Ci] matrix (K contiguous), so both operands are
// K-contiguous rows: 16-byte loads per lane, LDS tiles of 128-byte rows (+16 B pad),
// bf16 v_mfma_f32_16x16x32_bf16 (64 K per stage) or exact-f32 v_mfma_f32_16x16x4_f32
// (32 K per stage, K permuted identically on both operands).
// The weight gradient is a separate split-K kernel whose operands are M-contiguous, read
// from LDS with ds_read_b64_tr_b16 (bf16) so the MFMA A/B fragments come out K-major.
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "scd_common.h"

// Compile-time ablations of the LDS-DMA GEMM kernels (make ABLATE=N builds a separate library; never in the
// product build): 1 = no MFMA, 2 = loop DMAs read nothing, 3 = no loop DMA instructions, 4 = no loop
// fragment reads, 5 = no loop barriers; halo kernel: 6 = weight DMAs read nothing, 7 = halo DMAs read nothing,
// 8 = no vmcnt waits in the loop.  Runtime switches would put branches in the main loop and change
// its code (the waitcnt pass falls back to full drains around branched loads).
#ifndef SCD_ABLATE
#define SCD_ABLATE 0
#endif
#ifndef L1P_SWAP
#define L1P_SWAP 1      // conv_gemm_l1p_kernel, 256-pixel rows: 16-B stores of channel-block pairs (A/B option)
#endif
#ifndef S1X1_FULLROW
#define S1X1_FULLROW 1  // conv1x1_stream_kernel: stores of whole 128-B row pieces (A/B option)
#endif
#ifndef S1X1_STG
#define S1X1_STG 1    // conv1x1_stream_kernel: waves that share pixels take the operand from one LDS-DMA copy (A/B option)
#endif
#ifndef S1X1_UA2
#define S1X1_UA2 1    // conv1x1_stream_kernel: 32-pixel units where K = 64 (A/B build option)
#endif
#ifndef WGRAD_OCC
#define WGRAD_OCC 2   // register-staged weight-gradient kernel: workgroups per CU the registers are budgeted for
#endif

extern unsigned long long* scd_calib_stamp_buffer;   // calib.hip (stamped diagnostic builds)

namespace {
SCD_KERNEL_NS_BEGIN

struct GemmParams {
    const char* x;
    const char* w;
    char* y;
    const float* bias;
    double* stats;
    int N, Hi, Wi, Ci, Ho, Wo, Co;
    int is, os, wrow, relu, accumulate, nphase, ntn;
    int xbytes, wbytes;
    int ybytes;        // ping-pong BN-backward epilogue: bytes of the pre-BN activation (bny), its buffer range
    int tile_start[SCD_MAX_PHASES + 1];
    scd_gemm_phase ph[SCD_MAX_PHASES];
    // optional fused CenterNet head tails (n-tile t == head t, BN == head hidden width)
    int head_on;
    int debug;      // ablation (SCD_GEMM_DEBUG): 1 = no MFMA, 2 = no DMA after the prologue
    int head_od[4];
    const float* head_w[4];
    const float* head_b[4];
    float* head_out[4];
    // BN-backward sums in the epilogue (ping-pong kernel; scd_conv_gemm_bnbwd): the GEMM output is the gradient
    // dout of a following BN+ReLU layer whose pre-BN activation is bny; stats accumulates sum dz and
    // sum dz*(y-mean)*invstd with dz = dout (as stored) where y*rsc + rsh > 0
    int bnbwd;
    const char* bny;
    const float* bn_mean;
    const float* bn_invstd;
    const float* bn_rsc;
    const float* bn_rsh;
    // heads384 (scd_conv_gemm_heads_keep): hidden channels >= hid_cols stored only where hid_keep[pixel] != 0
    const unsigned char* hid_keep;
    int hid_cols;
    // scd_conv_dgrad_s2 (ping-pong kernel): GEMM column c = phase * Co/4 + channel is stored at output pixel
    // (2 oh + phase / 2, 2 ow + phase % 2) of a (2 Ho, 2 Wo, Co/4) tensor
    int shuf;
    // heads384: K-stage order reversed on every other round of 256 workgroups (kserp = 1; SCD_HEADS_SERP)
    int kserp;
    // stamped diagnostic build only (SCD_STAMP, calib.hip): per-workgroup main-loop clock stamps
    unsigned long long* stamps;
    // duo kernel: workgroups [duo_ncu, 2 duo_ncu) sleep duo_delay x 8K cycles before their first tile
    int duo_ncu, duo_delay;
};

#ifndef SCD_STAMP
#define SCD_STAMP 0
#endif
// SCD_STAMP builds: thread 0 of each workgroup records s_memtime / s_memrealtime at the start and the end of the
// main loop into p.stamps[blockIdx.x][4] (tools/clock_probe.py; MI355X_MICROARCH.md "DVFS give-back" item 6)
#define SCD_STAMP_BEGIN()                                                             \
    unsigned long long stamp_t0 = 0, stamp_r0 = 0;                                    \
    if constexpr (SCD_STAMP) {                                                        \
        stamp_t0 = __builtin_amdgcn_s_memtime();                                      \
        stamp_r0 = __builtin_amdgcn_s_memrealtime();                                  \
    }
#define SCD_STAMP_END()                                                               \
    if constexpr (SCD_STAMP) {                                                        \
        const unsigned long long stamp_t1 = __builtin_amdgcn_s_memtime();             \
        const unsigned long long stamp_r1 = __builtin_amdgcn_s_memrealtime();         \
        if (threadIdx.x == 0 && p.stamps) {                                           \
            unsigned long long* sp = p.stamps + (long)blockIdx.x * 4;                 \
            sp[0] = stamp_t0; sp[1] = stamp_t1; sp[2] = stamp_r0; sp[3] = stamp_r1;  \
        }                                                                             \
    }

// LDS image of one operand stage: rows of 128 B (BK elements), 16-B chunk c of row r stored at
// chunk c ^ (r & 7).  ds_read_b128 fragment reads (16 consecutive rows, one chunk) and the
// ds_write_b128 staging stores (8 chunks of one row) are then bank-conflict free.
// 16x16x16 MFMA on 4-element 16-bit vectors (the 16-bit type is h16, or _Float16 in the SCD_F16_BUILD pass)
typedef __attribute__((ext_vector_type(4))) h16 hx4;
__device__ __forceinline__ f32x4 mfma_16x16x16(hx4 a, hx4 b, f32x4 c) {
#ifdef SCD_F16_BUILD
    return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0);
#else
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, a), __builtin_bit_cast(s16x4, b), c, 0, 0, 0);
#endif
}

#ifndef PP_PRIO
// ping-pong kernels (conv_gemm_pp, heads384, wgrad_pp2): 1 = s_setprio 1 around every MFMA segment (the round-1
// form), 2 = static priority for the second-dispatched group for the whole main loop, no per-segment flips
// (MI355X_MICROARCH.md "Two waves per SIMD" item 4), 0 = none (A/B build option)
#define PP_PRIO 1
#endif
#ifndef PP_YPF
#define PP_YPF 1      // ping-pong BN-backward epilogue: the pre-BN rows loaded before the accumulators are staged
#endif
#ifndef PP_DPP
#define PP_DPP 1      // ping-pong epilogue: BN sums over the 16 pixel lanes with DPP row ops instead of ds_bpermute
#endif

// sum over the 16 lanes of a DPP row (every lane gets it): quad butterflies, then the half-row and row mirrors
__device__ __forceinline__ float row16_sum(float v) {
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, true));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, true));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, true));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, true));
    return v;
}

__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

// Buffer-load offset or an out-of-range one (the load then returns zeros).  The offset is made
// opaque before the select so the compiler cannot sink its arithmetic into an exec-masked branch:
// branches around loads make its waitcnt pass fall back to vmcnt(0) and drain the prefetch.
__device__ __forceinline__ int sel_off(bool ok, int off) {
    asm volatile("" : "+v"(off));
    return ok ? off : -16;
}
__device__ __forceinline__ uint4 bload(__amdgpu_buffer_rsrc_t r, int off) {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// Shared GEMM epilogue (NT = 2*BM threads, waves of 64x64 outputs, WN waves along N): bias / ReLU in
// registers, the wave's tile staged in LDS, coalesced 16-B NHWC stores (+= when accumulating), BN
// channel sums into fp64 replicas, and optionally the fused 1x1 head tails (n-tile t == head t).
template <typename T, int BM, int BN, int WN, bool HEADS, bool BNB = false>
__device__ __forceinline__ void gemm_epilogue(const GemmParams& p, f32x4 (&acc)[4][4], char* smem, int tid, int bid,
                                              int mt, int nt, int M, int QQ, const scd_gemm_phase& ph) {
    constexpr int ESZ = sizeof(T);
    constexpr int EPC = 16 / ESZ;
    constexpr int EROW = 64 * ESZ + 16; // epilogue staging row (64 channels + pad)
    constexpr int EPI = (BM / 64) * WN * 64 * EROW;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / WN, wn = wave - (wave / WN) * WN;
    const int l16 = lane & 15, lg = lane >> 4;
    // the LDS-DMA ring kernel (256 x 128) takes its loads from clamped addresses with the values selected after and its
    // statistics by select (no branch regions); the register-staged kernels keep the branches (at their 256-VGPR bound
    // the selects' live values spill)
    constexpr bool SELF = BM == 256 && BN == 128;
    // ---- epilogue 1: bias / relu in registers, BN partial sums, stage the wave's 64x64 tile in LDS
    char* ep = smem + wave * 64 * EROW;
    float csum[4][4], csq[4][4];
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) { csum[b][r] = 0.f; csq[b][r] = 0.f; }
    // BN-backward mode (BNB: 16-bit types, scd_conv_gemm_bnbwd): output pixel of each of the lane's 4 rows
    // (-1 past the end); a separate instantiation, so the other kernels keep their register allocation
    int pix[4];
    if constexpr (BNB) {
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            const int m = mt * BM + wm * 64 + a * 16 + l16;
            const int n = m / QQ;
            const int rem = m - n * QQ;
            const int qh = rem / ph.Qw, qw = rem - (rem / ph.Qw) * ph.Qw;
            pix[a] = m < M ? (n * p.Ho + p.os * qh + ph.rho_h) * p.Wo + p.os * qw + ph.rho_w : -1;
        }
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int col0 = nt * BN + wn * 64 + b * 16 + lg * 4;
        float bias[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) bias[r] = (p.bias && col0 + r < p.Co) ? p.bias[col0 + r] : 0.f;
        float bmu[4], bis[4], bsc[4], bsh[4];
        uint2 yq[4];
        if constexpr (BNB) {
            // every load from a valid address (channel 0 / pixel 0 when masked off) and the value selected after:
            // a load under the test is a branch region the compiler waits on before the next load
            const bool okc = col0 < p.Co;
            const int cl = okc ? col0 : 0;
            const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
            float4 f0, f1, f2, f3;
            if constexpr (SELF) {
                const float4 l0 = *(const float4*)(p.bn_mean + cl), l1 = *(const float4*)(p.bn_invstd + cl);
                const float4 l2 = *(const float4*)(p.bn_rsc + cl), l3 = *(const float4*)(p.bn_rsh + cl);
                f0 = okc ? l0 : z4; f1 = okc ? l1 : z4; f2 = okc ? l2 : z4; f3 = okc ? l3 : z4;
            } else {
                f0 = okc ? *(const float4*)(p.bn_mean + col0) : z4;
                f1 = okc ? *(const float4*)(p.bn_invstd + col0) : z4;
                f2 = okc ? *(const float4*)(p.bn_rsc + col0) : z4;
                f3 = okc ? *(const float4*)(p.bn_rsh + col0) : z4;
            }
            bmu[0] = f0.x; bmu[1] = f0.y; bmu[2] = f0.z; bmu[3] = f0.w;
            bis[0] = f1.x; bis[1] = f1.y; bis[2] = f1.z; bis[3] = f1.w;
            bsc[0] = f2.x; bsc[1] = f2.y; bsc[2] = f2.z; bsc[3] = f2.w;
            bsh[0] = f3.x; bsh[1] = f3.y; bsh[2] = f3.z; bsh[3] = f3.w;
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                const bool ok = pix[a] >= 0 && okc;
                if constexpr (SELF) {
                    const uint2 raw = *(const uint2*)(p.bny + ((long)(ok ? pix[a] : 0) * p.Co + cl) * 2);
                    yq[a] = ok ? raw : make_uint2(0, 0);
                } else {
                    yq[a] = ok ? *(const uint2*)(p.bny + ((long)pix[a] * p.Co + col0) * 2) : make_uint2(0, 0);
                }
            }
        }
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            const int m = mt * BM + wm * 64 + a * 16 + l16;
            float v[4];
            if constexpr (!BNB) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[r] = acc[a][b][r] + bias[r];
                    if (p.relu) v[r] = fmaxf(v[r], 0.f);
                    if constexpr (SELF) {
                        // a select, not a branch region (the sums never hold -0: adding +0 past M leaves them unchanged)
                        const float t = m < M ? v[r] : 0.f;
                        csum[b][r] += t;
                        csq[b][r] += t * t;
                    } else {
                        if (m < M) { csum[b][r] += v[r]; csq[b][r] += v[r] * v[r]; }
                    }
                }
            } else {
                // the following BN+ReLU layer's backward sums over the gradient as stored (16-bit)
                const unsigned yw[2] = {yq[a].x, yq[a].y};
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[r] = acc[a][b][r];
                    const float yv = h16_word_half(yw[r >> 1], r & 1);
                    const float d = (float)(T)v[r];
                    const float dz = yv * bsc[r] + bsh[r] > 0.f ? d : 0.f;
                    csum[b][r] += dz;
                    csq[b][r] += dz * (yv - bmu[r]) * bis[r];
                }
            }
            char* dst = ep + (a * 16 + l16) * EROW + (b * 16 + lg * 4) * ESZ;
            if constexpr (ESZ == 2) {
                typedef __attribute__((ext_vector_type(4))) h16 bf16x4;
                bf16x4 o = {(h16)v[0], (h16)v[1], (h16)v[2], (h16)v[3]};
                *(bf16x4*)dst = o;
            } else {
                *(float4*)dst = make_float4(v[0], v[1], v[2], v[3]);
            }
        }
    }
    __syncthreads();
    // ---- epilogue 2: coalesced 16-B NHWC stores (+= for accumulate) of the staged tile
    {
        constexpr int CPR = 64 * ESZ / 16;        // 16-B chunks per staged row
        constexpr int RPI = 64 / CPR;             // rows per wave instruction
        const int ch = lane % CPR;
        const int col = nt * BN + wn * 64 + ch * EPC;
#pragma unroll
        for (int j = 0; j < 64 / RPI; ++j) {
            const int row = lane / CPR + RPI * j;
            const int mr = mt * BM + wm * 64 + row;
            // ring kernel: rows past M / columns past Co address pixel 0 / channel 0 and skip only the store (no branch
            // around the accumulate load)
            const bool ok = mr < M && col < p.Co;
            if constexpr (!SELF) {
                if (!ok) continue;
            }
            const int m = SELF ? (ok ? mr : 0) : mr;
            const int n = m / QQ;
            const int rem = m - n * QQ;
            const int qh = rem / ph.Qw;
            const int qw = rem - qh * ph.Qw;
            const int oh = p.os * qh + ph.rho_h, ow = p.os * qw + ph.rho_w;
            T* dst = (T*)(p.y) + ((long)(n * p.Ho + oh) * p.Wo + ow) * p.Co + (SELF ? (ok ? col : 0) : col);
            uint4 v = *(const uint4*)(ep + row * EROW + ch * 16);
            if (p.accumulate) {
                float a[EPC], o[EPC];
                Vec16<T>::load(&v, a);
                Vec16<T>::load(dst, o);
#pragma unroll
                for (int e = 0; e < EPC; ++e) a[e] += o[e];
                Vec16<T>::store(&v, a);
            }
            if (!SELF || ok) *(uint4*)dst = v;
        }
    }
    if (p.stats) {
        // channel sums: over the 16 pixel-lanes (xor 1..8), then over the waves sharing the columns
        float* red = (float*)(smem + EPI);   // [BM/64][BN][2] floats  (<= 2 KB)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float s = row16_sum(csum[b][r]), q = row16_sum(csq[b][r]);   // DPP, no LDS permutes
                if (l16 == 0) {
                    const int c = wn * 64 + b * 16 + lg * 4 + r;
                    red[(wm * BN + c) * 2 + 0] = s;
                    red[(wm * BN + c) * 2 + 1] = q;
                }
            }
        __syncthreads();
        if (tid < BN) {
            const int col = nt * BN + tid;
            if (col < p.Co) {
                double s = 0.0, q = 0.0;
#pragma unroll
                for (int w = 0; w < BM / 64; ++w) { s += red[(w * BN + tid) * 2]; q += red[(w * BN + tid) * 2 + 1]; }
                const int rep = bid % SCD_STAT_REPLICAS;
                atomic_add_f64(p.stats + ((long)rep * 2 + 0) * p.Co + col, s);
                atomic_add_f64(p.stats + ((long)rep * 2 + 1) * p.Co + col, q);
            }
        }
    }
    if constexpr (HEADS && BN == 128) {
        {
            // fused terminal 1x1 (centerNetOffset.py:108-110): head = n-tile, hidden = staged tile.
            // thread -> (row = tid/2, half = tid&1): 64-channel partial dots, combined across the pair.
            const int h = nt;
            const int od = p.head_od[h];
            float* ws = (float*)(smem + EPI);   // w1 of this head, [od][128]
            __syncthreads();
            for (int i = tid; i < od * 128; i += 256) ws[i] = p.head_w[h][i];
            __syncthreads();
            const int row = tid >> 1, half = tid & 1;
            const int wv = (row >> 6) * WN + half;          // wave that staged this (row, half)
            const char* src = smem + wv * 64 * EROW + (row & 63) * EROW;
            float o4[4] = {0.f, 0.f, 0.f, 0.f};
            for (int c = 0; c < 64; c += EPC) {
                float v[EPC];
                Vec16<T>::load(src + c * ESZ, v);
#pragma unroll
                for (int o = 0; o < 4; ++o)
                    if (o < od) {
#pragma unroll
                        for (int e = 0; e < EPC; ++e) o4[o] += v[e] * ws[o * 128 + half * 64 + c + e];
                    }
            }
#pragma unroll
            for (int o = 0; o < 4; ++o) o4[o] += __shfl_xor(o4[o], 1, 64);
            const int m = mt * BM + row;
            if (half == 0 && m < M) {
                const int n = m / QQ;
                const int rem = m - n * QQ;
                const int qh = rem / ph.Qw;
                const int qw = rem - qh * ph.Qw;
                const int oh = p.os * qh + ph.rho_h, ow = p.os * qw + ph.rho_w;
                for (int o = 0; o < od; ++o)
                    p.head_out[h][((long)n * od + o) * p.Ho * p.Wo + oh * p.Wo + ow] = o4[o] + p.head_b[h][o];
            }
        }
    }
}

// KS = 2: intra-workgroup split K for grids of about one tile per CU (layer4 at 512 px, long K): two groups of
// four waves each run the 128x128 tile over one half of the K stages in their own double-buffered LDS
// stages (8 waves per CU instead of 4, no partial sums through HBM); group 1 hands its accumulators to group
// 0 through LDS and exits (S_BARRIER then waits on the surviving waves only), group 0 runs the epilogue.
template <typename T, int BM, int BN, bool HEADS, bool BNB = false, int KS = 1>
__global__ __launch_bounds__(256 * KS, 2 / KS) void conv_gemm_kernel(GemmParams p) {
    static_assert(KS == 1 || KS == 2, "split K by 1 or 2");
    constexpr int ESZ = sizeof(T);
    constexpr int EPC = 16 / ESZ;       // elements per 16-B chunk
    constexpr int BK = 128 / ESZ;       // K elements per stage
    constexpr int ACH = BM / 32;        // A chunks per thread
    constexpr int BCH = BN / 32;
    constexpr int WN = BN / 64;         // waves along N (each wave: 64x64)
    constexpr int STAGE = (BM + BN) * 128;
    constexpr int EROW = 64 * ESZ + 16; // epilogue staging row (64 channels + pad)
    constexpr int EPI = 4 * 64 * EROW;
    constexpr int SMEM1 = (KS * 2 * STAGE > EPI + 2048) ? KS * 2 * STAGE : EPI + 2048;
    constexpr int SMEM = (KS > 1 && SMEM1 < 4 * 64 * 64 * 4) ? 4 * 64 * 64 * 4 : SMEM1;
    __shared__ __attribute__((aligned(16))) char smem[SMEM];

    const int grp = KS == 1 ? 0 : (int)(threadIdx.x >> 8);
    const int tid = threadIdx.x & 255;
    char* const gsm = smem + grp * 2 * STAGE;     // this group's two operand stages
    // XCD-aware bijective remap: blocks that share an A (pixel) tile run on one XCD's L2
    int bid;
    {
        const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7, xcd = blockIdx.x & 7;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (blockIdx.x >> 3);
    }
    int phase = 0;
#pragma unroll
    for (int i = 1; i < SCD_MAX_PHASES; ++i)
        if (i < p.nphase && bid >= p.tile_start[i]) phase = i;
    const scd_gemm_phase& ph = p.ph[phase];
    const int local = bid - p.tile_start[phase];
    const int mt = local / p.ntn;
    const int nt = local - mt * p.ntn;
    const int QQ = ph.Qh * ph.Qw;
    const int M = p.N * QQ;

    // ---- per-thread gather rows (fixed across the K loop)
    const int cch = tid & 7;
    const int srow = tid >> 3;                        // staging row (mod 32)
    int a_pix[ACH], a_ih[ACH], a_iw[ACH];
    bool a_ok[ACH];
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
        int m = mt * BM + srow + 32 * i;
        a_ok[i] = m < M;
        int mm = a_ok[i] ? m : 0;
        int n = mm / QQ;
        int rem = mm - n * QQ;
        int qh = rem / ph.Qw;
        int qw = rem - qh * ph.Qw;
        a_pix[i] = n * p.Hi * p.Wi;
        a_ih[i] = p.is * qh;
        a_iw[i] = p.is * qw;
    }
    int b_row[BCH];
    bool b_ok[BCH];
#pragma unroll
    for (int j = 0; j < BCH; ++j) {
        int nn = nt * BN + srow + 32 * j;
        b_ok[j] = nn < p.Co;
        b_row[j] = b_ok[j] ? nn : 0;
    }
    const int cpt = p.Ci / BK;            // K stages per tap
    const int KT = ph.ntaps * cpt;
    const int KTg = (KT + KS - 1) / KS;   // stages per group (both groups run KTg, so barriers pair up)
    const int kb = grp * KTg;
    const int ke = min(KT, kb + KTg);
    const int st_off = swz(srow, cch);    // (srow + 32i) & 7 == srow & 7

    // raw buffer loads: out-of-range lanes use an offset past num_records and read zeros
    // (no exec-mask branches around the loads, so the compiler can count vmcnt per stage)
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.xbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, p.wbytes, 0x00020000);
    auto gload = [&](int kt_req, uint4 (&ra)[ACH], uint4 (&rb)[BCH]) {
        // stages past the end are issued with out-of-range offsets (no traffic, no branch)
        const bool live = kb + kt_req < ke;
        const int kt = max(0, min(kb + kt_req, ke - 1));
        const int chunk = kt / ph.ntaps, tap = kt - chunk * ph.ntaps;   // channel chunk outer, taps inner
        int c0 = chunk * BK + cch * EPC;
        int dh = ph.dh[tap], dw = ph.dw[tap], wt = ph.wt[tap];
#pragma unroll
        for (int i = 0; i < ACH; ++i) {
            int ih = a_ih[i] + dh, iw = a_iw[i] + dw;
            bool ok = live && a_ok[i] && (unsigned)ih < (unsigned)p.Hi && (unsigned)iw < (unsigned)p.Wi;
            ra[i] = bload(xrs, sel_off(ok, ((a_pix[i] + ih * p.Wi + iw) * p.Ci + c0) * ESZ));
        }
#pragma unroll
        for (int j = 0; j < BCH; ++j) {
            rb[j] = bload(wrs, sel_off(live && b_ok[j], (b_row[j] * p.wrow + wt * p.Ci + c0) * ESZ));
        }
    };
    auto lstore = [&](int buf, const uint4 (&ra)[ACH], const uint4 (&rb)[BCH]) {
        char* As = gsm + buf * STAGE;
        char* Bs = As + BM * 128;
#pragma unroll
        for (int i = 0; i < ACH; ++i) *(uint4*)(As + st_off + 32 * 128 * i) = ra[i];
#pragma unroll
        for (int j = 0; j < BCH; ++j) *(uint4*)(Bs + st_off + 32 * 128 * j) = rb[j];
    };

    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / WN, wn = wave - (wave / WN) * WN;
    const int l16 = lane & 15, lg = lane >> 4;
    const int l7 = l16 & 7;

    // acc[a][b] = D[n][m] with the weight fragment as the MFMA "A" operand: lane holds pixel
    // m = a*16 + l16 and the 4 consecutive channels n = b*16 + 4*lg + r (r = register).
    f32x4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};

    auto compute = [&](int buf) {
        const char* As = gsm + buf * STAGE;
        const char* Bs = As + BM * 128;
        if constexpr (ESZ == 2) {
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                h16x8 af[4], bfr[4];
                const int co = ((s * 4 + lg) ^ l7) << 4;
#pragma unroll
                for (int a = 0; a < 4; ++a) af[a] = *(const h16x8*)(As + (wm * 64 + a * 16 + l16) * 128 + co);
#pragma unroll
                for (int b = 0; b < 4; ++b) bfr[b] = *(const h16x8*)(Bs + (wn * 64 + b * 16 + l16) * 128 + co);
#pragma unroll
                for (int a = 0; a < 4; ++a)
#pragma unroll
                    for (int b = 0; b < 4; ++b)
                        acc[a][b] = mfma_16x16x32_h16(bfr[b], af[a], acc[a][b]);
            }
        } else {
            // exact-f32 MFMA: lane group lg owns K elements [8lg, 8lg+8) of the 32-wide stage;
            // step j multiplies element 8lg+j of A and B (same permutation on both operands).
            const int c0 = ((2 * lg) ^ l7) << 4, c1 = ((2 * lg + 1) ^ l7) << 4;
            float4 af[4][2], bfr[4][2];
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                const char* pa = As + (wm * 64 + a * 16 + l16) * 128;
                af[a][0] = *(const float4*)(pa + c0);
                af[a][1] = *(const float4*)(pa + c1);
            }
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const char* pb = Bs + (wn * 64 + b * 16 + l16) * 128;
                bfr[b][0] = *(const float4*)(pb + c0);
                bfr[b][1] = *(const float4*)(pb + c1);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    float av = (j < 4) ? af[a][0][j & 3] : af[a][1][j & 3];
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        float bv = (j < 4) ? bfr[b][0][j & 3] : bfr[b][1][j & 3];
                        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(bv, av, acc[a][b], 0, 0, 0);
                    }
                }
            }
        }
    };

    if (KT > 0) {
        // two stages of global loads in flight: stage k+1 lands while stage k is computed and
        // stage k+2 is issued; LDS is double-buffered, one barrier per stage
        uint4 ra0[ACH], rb0[BCH], ra1[ACH], rb1[BCH];
        gload(0, ra0, rb0);
        gload(1, ra1, rb1);
        lstore(0, ra0, rb0);
        __syncthreads();
        for (int kt = 0; kt < KTg; kt += 2) {
            gload(kt + 2, ra0, rb0);
            compute(0);
            lstore(1, ra1, rb1);
            __syncthreads();
            if (kt + 1 >= KTg) break;
            gload(kt + 3, ra1, rb1);
            compute(1);
            lstore(0, ra0, rb0);
            __syncthreads();
        }
    }
    if constexpr (KS == 2) {
        // group 1's accumulators -> group 0 through LDS ([wave][register][lane] floats: conflict-free)
        float* xs = (float*)smem + (wave * 64) * 64 + lane;
        if (grp == 1) {
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b)
#pragma unroll
                    for (int r = 0; r < 4; ++r) xs[(a * 16 + b * 4 + r) * 64] = acc[a][b][r];
        }
        __syncthreads();
        if (grp == 1) return;
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[a][b][r] += xs[(a * 16 + b * 4 + r) * 64];
        __syncthreads();
    }

    gemm_epilogue<T, BM, BN, WN, HEADS, BNB>(p, acc, smem, tid, bid, mt, nt, M, QQ, ph);
}

// -------------------------------------------------------------------------------------
// Large-shape bf16 gather-GEMM: 256x128 tile, 8 waves (4 along M x 2 along N, 64x64 each), one
// workgroup per CU.  Both operands are staged by LDS-DMA (buffer_load_dwordx4 ... lds) into a
// 3-slot LDS ring: two K-stages stay in flight across the single raw s_barrier of each K-step
// (counted vmcnt, never 0 in the loop), so the MFMAs of stage k overlap the HBM/L2 latency of
// stages k+1 and k+2.  The 16-B chunk c of LDS row r lives in slot c ^ (r & 7): the DMA writes
// each wave-instruction's 1 KiB lane-linearly, so the swizzle is applied to the SOURCE chunk.
// Out-of-image taps and stages past the end use out-of-range buffer offsets (zeros, no traffic).
typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds_wave_base, int off) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)lds_wave_base, 16, off, 0, 0, 0);
}

// The same LDS-DMA as inline asm: hipcc does not track it, so it emits no conservative vmcnt(0) in front of
// the ds_read_b64_tr_b16 builtins that follow (it does for its own LDS-DMA).  Completion is counted by hand
// (s_waitcnt vmcnt(N) + barrier).  M0 is saved and restored inside the statement (it is compiler-reserved).
__device__ __forceinline__ void dma16_asm(__amdgpu_buffer_rsrc_t r, const char* lds_dst, int off) {
    const unsigned lds = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_ptr_t)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(off), "s"(lds), "s"(r)
                 : "memory");
}

// -------------------------------------------------------------------------------------
// 3x3 / stride 1 / pad 1 convolution with 64 input and 64 output channels on whole image rows (ResNet layer1,
// residuals.py:84-120; forward and input gradient).  A tile is 256 output pixels = TR = 256 / WO rows of one image;
// the input rows with their one-pixel halo sit in LDS (columns padded to WH = WO + 8 pixel slots, 16-B chunk c of
// slot q at c ^ (q & 7), the swizzle applied to the DMA's source chunk), so every tap reads its A fragments at a
// constant displacement from 6 per-lane base addresses: no address arithmetic in the loop (the register-staged
// 256 x 64 kernel spends ~9 VALU per MFMA on it), and the MFMA order per output is that kernel's (tap-major, two
// K halves per tap), so the results are bit-identical.  A workgroup runs `run` consecutive tiles of one image
// (TR output rows each) down the image, so consecutive tiles share two input rows.  LDS holds a ring of 2 TR + 2 input rows: the TR + 2 rows of the current tile and the TR new rows of the
// next tile, which are DMA'd while the current tile is computed (HBM reads ~1x the input instead of 2x, and the
// load latency hides behind the MFMAs).  8 waves: wave w computes tile pixels 64 (w & 3) .. +63 x channels
// 32 (w >> 2) .. +31, its 32 x 576 weight slice held in registers for the whole run (144 VGPRs, loaded once).
// Epilogue per tile: the accumulators are staged in LDS and the tile -- TR whole rows, one contiguous NHWC block
// -- leaves as linear 16-B stores (+= when accumulating); BN sums (forward: fp32 accumulators, as the shared
// epilogue; BNB: the stored gradient against the BN input) are carried in registers across the run and added to
// the fp64 replicas once per workgroup.
// Rows of 256 pixels (Res50 layer1 at 1024^2 input, residuals.py:122-165, 357): a tile is one row, and the four ring
// rows (132 KiB) leave no room for the staging buffer, so the tile is stored straight from the accumulators (16-B
// stores of 8 channels after v_permlane16_swap pairs the lane's two channel blocks; L2 merges a pixel's 128 B):
// outputs bit-identical.  The BN-backward-sum variant
// is not built for them (its operand loads in this layout spill registers): scd_conv_gemm_bnbwd then runs this
// kernel's plain input gradient and the separate scd_bn_bwd_reduce.
template <int WO, bool FLIP, bool BNB>
__global__ __launch_bounds__(512, 1) void conv_gemm_l1p_kernel(GemmParams p, int run) {
    typedef h16 T;
    constexpr int TR = WO >= 256 ? 1 : 256 / WO;  // output rows per tile
    constexpr bool DIRECT = WO == 256;            // no staging buffer: stores from the accumulators
    static_assert(!(DIRECT && BNB), "256-pixel rows: BN-backward sums by the separate reduction");
    constexpr int WH = WO + 8;                    // pixel slots per ring row (slot = input column + 1)
    constexpr int ROWB = WH * 128;
    constexpr int RING = 2 * TR + 2;
    constexpr int SROW = 64 * 2 + 16;             // staging row: 64 channels + 16 B pad
    constexpr int STG = DIRECT ? 0 : 256 * SROW;
    static_assert(WO * TR == 256 && WH % 8 == 0, "tile geometry");
    __shared__ __attribute__((aligned(16))) char smem[RING * ROWB + (STG ? STG : 16)];
    char* const stg = smem + RING * ROWB;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, lg = lane >> 4;
    const int pw = wave & 3, chh = wave >> 2;
    const int wr = (64 * pw) / WO, wc = (64 * pw) % WO;
    const int tpi = p.Ho / TR;                    // tiles per image
    const int t0 = blockIdx.x * run;
    const int n = t0 / tpi, r0 = (t0 - n * tpi) * TR;

    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.xbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, p.wbytes, 0x00020000);

    // ---- input rows -> ring slot (row + 1) % RING; one 1-KB DMA per 8 pixel slots (lane: slot lane/8, chunk lane%8)
    const int hq = lane >> 3, csrc = (lane & 7) ^ hq;
    auto dma_rows = [&](int ir0, int nrows) {
        for (int j = wave; j < nrows * (WH / 8); j += 8) {
            const int hr = j / (WH / 8), g = j - (j / (WH / 8)) * (WH / 8);
            const int ir = ir0 + hr, ic = g * 8 + hq - 1;
            const bool ok = (unsigned)ir < (unsigned)p.Hi && (unsigned)ic < (unsigned)p.Wi;
            dma16(xrs, smem + ((ir + 1) % RING) * ROWB + g * 8 * 128,
                  sel_off(ok, (((n * p.Hi + ir) * p.Wi + ic) * 64 + csrc * 8) * 2));
        }
    };
    dma_rows(r0 - 1, TR + 2);

    // ---- this wave's weight slice: co = 32 chh + 16 b + l16, K chunk lg of each (tap, half)
    uint4 wreg[9][2][2];
    {
        const int wl = ((32 * chh + l16) * p.wrow + lg * 8) * 2;
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    wreg[t][s][b] = bload(wrs, wl + (b * 16 * p.wrow + t * 64 + s * 32) * 2);
    }
    // BN-backward epilogue parameters in LDS (the store phase owns fixed 8-channel chunks)
    __shared__ __attribute__((aligned(16))) float bnpar[BNB ? 4 * 64 : 4];
    if constexpr (BNB) {
        if (tid < 256) {
            const int k = tid >> 6, c = tid & 63;
            const float* src = k == 0 ? p.bn_mean : k == 1 ? p.bn_invstd : k == 2 ? p.bn_rsc : p.bn_rsh;
            bnpar[tid] = src[c];
        }
    }
    int abase[3][2];
#pragma unroll
    for (int d = 0; d < 3; ++d)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int q = wc + l16 + d;
            abase[d][s] = q * 128 + (((s * 4 + lg) ^ (q & 7)) << 4);
        }
    // the workgroup's BN sums: per tile the waves' partials go to fixed LDS slots ([wave][channel][2]) and threads
    // 0..127 (channel tid & 63, sum tid >> 6) add them in a fixed order, so the sums are deterministic
    __shared__ float bnred[8 * 64 * 2];
    float bnsum = 0.f;
    const bool fwd_stats = !BNB && p.stats;
    const int cc = tid & 7;                       // store phase: this thread's 8-channel chunk

    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    for (int i = 0; i < run; ++i) {
        const int r = r0 + i * TR;
        if (i + 1 < run) dma_rows(r + TR + 1, TR);            // the next tile's new rows, into free ring slots
        f32x4 acc[4][2];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
        int rowoff[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) rowoff[d] = ((r + wr + d) % RING) * ROWB;   // input row r + wr + d - 1
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int kr = t / 3, kc = t - (t / 3) * 3;
            const int dhi = FLIP ? 2 - kr : kr, dwi = FLIP ? 2 - kc : kc;
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                h16x8 af[4];
#pragma unroll
                for (int a = 0; a < 4; ++a) af[a] = *(const h16x8*)(smem + rowoff[dhi] + abase[dwi][s] + a * 16 * 128);
#pragma unroll
                for (int a = 0; a < 4; ++a)
#pragma unroll
                    for (int b = 0; b < 2; ++b)
                        acc[a][b] = mfma_16x16x32_h16(__builtin_bit_cast(h16x8, wreg[t][s][b]),
                                                                            af[a], acc[a][b]);
            }
        }
        if constexpr (DIRECT && L1P_SWAP) {
            // the tile is row r of image n: lane's pixel 64pw + 16a + l16 is its column.  The two channel blocks
            // paired by v_permlane16_swap: the lane then holds 8 consecutive channels 32chh + 4lg + 12(lg & 1) ..,
            // one 16-B store per pixel block (16 pixels x 64 B per instruction instead of 16 x 32 B)
            const long base = ((long)(n * p.Ho + r) * p.Wo) * 64;
            typedef __attribute__((ext_vector_type(4))) h16 bf16x4;
            typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
            const int cst = 32 * chh + 4 * lg + 12 * (lg & 1);
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                const long off = base + (long)(64 * pw + 16 * a + l16) * 64 + cst;
                bf16x4 h0, h1;
#pragma unroll
                for (int q = 0; q < 4; ++q) { h0[q] = (h16)acc[a][0][q]; h1[q] = (h16)acc[a][1][q]; }
                const u32x2 xv = __builtin_bit_cast(u32x2, h0), yv = __builtin_bit_cast(u32x2, h1);
                const auto s0 = __builtin_amdgcn_permlane16_swap(xv[0], yv[0], false, false);
                const auto s1 = __builtin_amdgcn_permlane16_swap(xv[1], yv[1], false, false);
                uint4 v;
                v.x = s0[0]; v.y = s1[0]; v.z = s0[1]; v.w = s1[1];
                if (p.accumulate) {
                    float a8[8], o8[8];
                    Vec16<T>::load(&v, a8);
                    Vec16<T>::load((const T*)p.y + off, o8);
#pragma unroll
                    for (int e = 0; e < 8; ++e) a8[e] += o8[e];
                    Vec16<T>::store(&v, a8);
                }
                *(uint4*)((T*)p.y + off) = v;
            }
        } else if constexpr (DIRECT) {
            // the tile is row r of image n: lane's pixel 64pw + 16a + l16 is its column; channels 32chh + 16b + 4lg
            const long base = ((long)(n * p.Ho + r) * p.Wo) * 64;
            typedef __attribute__((ext_vector_type(4))) h16 bf16x4;
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    const long off = base + (long)(64 * pw + 16 * a + l16) * 64 + 32 * chh + 16 * b + 4 * lg;
                    bf16x4 o;
#pragma unroll
                    for (int q = 0; q < 4; ++q) o[q] = (h16)acc[a][b][q];
                    if (p.accumulate) {
                        const bf16x4 old4 = *(const bf16x4*)((const T*)p.y + off);
#pragma unroll
                        for (int q = 0; q < 4; ++q) o[q] = (h16)((float)o[q] + (float)old4[q]);
                    }
                    *(bf16x4*)((T*)p.y + off) = o;
                }
        } else {
        // stage: lane holds pixel 64pw + 16a + l16, channels 32chh + 16b + 4lg + (0..3)
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                typedef __attribute__((ext_vector_type(4))) h16 bf16x4;
                bf16x4 o;
#pragma unroll
                for (int q = 0; q < 4; ++q) o[q] = (h16)acc[a][b][q];
                *(bf16x4*)(stg + (64 * pw + 16 * a + l16) * SROW + (32 * chh + 16 * b + 4 * lg) * 2) = o;
            }
        }
        if (fwd_stats) {
            // forward BN sums of the fp32 accumulators (as the shared epilogue): over the wave's 4 pixel blocks,
            // the 16 pixel lanes (DPP row sums), then the 4 pixel-group waves through LDS
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    float sv = 0.f, qv = 0.f;
#pragma unroll
                    for (int a = 0; a < 4; ++a) { sv += acc[a][b][q]; qv += acc[a][b][q] * acc[a][b][q]; }
                    sv = row16_sum(sv);
                    qv = row16_sum(qv);
                    if (l16 == 0) {
                        const int c = 32 * chh + 16 * b + 4 * lg + q;
                        bnred[(pw * 64 + c) * 2] = sv;
                        bnred[(pw * 64 + c) * 2 + 1] = qv;
                    }
                }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");        // next tile's rows (and the previous stores)
        __syncthreads();
        if (fwd_stats && tid < 128) {
#pragma unroll
            for (int w = 0; w < 4; ++w) bnsum += bnred[(w * 64 + (tid & 63)) * 2 + (tid >> 6)];
        }
        if constexpr (DIRECT) {
            __syncthreads();                                     // bnred read before the next tile writes it
            continue;
        }
        // ---- store phase: the tile is rows r .. r+TR-1 of image n, one contiguous 32-KB NHWC block
        {
            const long base = ((long)(n * p.Ho + r) * p.Wo) * 64;
            float bs[8], bq[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) { bs[e] = 0.f; bq[e] = 0.f; }
#pragma unroll(BNB ? 1 : 4)
            for (int k = 0; k < 4; ++k) {
                const int j = tid + 512 * k;                    // 16-B chunk of the tile (pixel j / 8, chunk cc)
                const int px = j >> 3;
                uint4 v = *(const uint4*)(stg + px * SROW + cc * 16);
                T* dst = (T*)p.y + base + px * 64 + cc * 8;
                if (p.accumulate) {
                    float a8[8], o8[8];
                    Vec16<T>::load(&v, a8);
                    Vec16<T>::load(dst, o8);
#pragma unroll
                    for (int e = 0; e < 8; ++e) a8[e] += o8[e];
                    Vec16<T>::store(&v, a8);
                }
                if constexpr (BNB) {
                    float d8[8], y8[8];
                    Vec16<T>::load(&v, d8);
                    Vec16<T>::load((const T*)p.bny + base + px * 64 + cc * 8, y8);
                    // parameters re-read from LDS per chunk (an opaque offset keeps them out of the live registers)
                    int po = cc * 8;
                    asm volatile("" : "+v"(po));
#pragma unroll
                    for (int e = 0; e < 8; ++e) d8[e] = y8[e] * bnpar[128 + po + e] + bnpar[192 + po + e] > 0.f ? d8[e] : 0.f;
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        bs[e] += d8[e];
                        bq[e] += d8[e] * (y8[e] - bnpar[po + e]) * bnpar[64 + po + e];
                    }
                }
                *(uint4*)dst = v;
            }
            if constexpr (BNB) {
                // lanes with equal lane % 8 hold the same channels: fold lane bits 3..5, then the 8 waves via LDS
#pragma unroll
                for (int e = 0; e < 8; ++e) {
#pragma unroll
                    for (int o = 8; o < 64; o <<= 1) { bs[e] += __shfl_xor(bs[e], o, 64); bq[e] += __shfl_xor(bq[e], o, 64); }
                }
                if (lane < 8) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        bnred[(wave * 64 + cc * 8 + e) * 2] = bs[e];
                        bnred[(wave * 64 + cc * 8 + e) * 2 + 1] = bq[e];
                    }
                }
            }
        }
        __syncthreads();                                         // staging read before the next tile writes it
        if (BNB && tid < 128) {
#pragma unroll
            for (int w = 0; w < 8; ++w) bnsum += bnred[(w * 64 + (tid & 63)) * 2 + (tid >> 6)];
        }
    }

    // ---- BN sums: once per workgroup into replica blockIdx % SCD_STAT_REPLICAS
    if ((BNB || p.stats) && tid < 128) {
        const int rep = blockIdx.x % SCD_STAT_REPLICAS;
        atomic_add_f64(p.stats + ((long)rep * 2 + (tid >> 6)) * p.Co + (tid & 63), (double)bnsum);
    }
}

template <bool HEADS, bool BNB = false>
__global__ __launch_bounds__(512, 1) void conv_gemm_ring_kernel(GemmParams p) {
    typedef h16 T;
    constexpr int BM = 256, BN = 128, WN = 2, BK = 64, EPC = 8;
    constexpr int STAGE = (BM + BN) * 128;          // 48 KiB
    constexpr int NSLOT = 3;
    __shared__ __attribute__((aligned(16))) char smem[NSLOT * STAGE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int bid;
    {
        const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7, xcd = blockIdx.x & 7;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (blockIdx.x >> 3);
    }
    int phase = 0;
#pragma unroll
    for (int i = 1; i < SCD_MAX_PHASES; ++i)
        if (i < p.nphase && bid >= p.tile_start[i]) phase = i;
    const scd_gemm_phase& ph = p.ph[phase];
    const int local = bid - p.tile_start[phase];
    const int mt = local / p.ntn;
    const int nt = local - mt * p.ntn;
    const int QQ = ph.Qh * ph.Qw;
    const int M = p.N * QQ;

    // DMA rows of this lane: A rows 32*wave + 8*i + lane/8 (i < 4), B rows 16*wave + 8*j + lane/8 (j < 2);
    // the lane fetches logical chunk (lane & 7) ^ (row & 7) so that LDS slot (lane & 7) holds it.
    const int lrow = lane >> 3;
    const int cch = (lane & 7) ^ (lrow & 7);
    int a_pix[4], a_ih[4], a_iw[4];
    bool a_ok[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = mt * BM + 32 * wave + 8 * i + lrow;
        a_ok[i] = m < M;
        const int mm = a_ok[i] ? m : 0;
        const int n = mm / QQ;
        const int rem = mm - n * QQ;
        const int qh = rem / ph.Qw;
        const int qw = rem - qh * ph.Qw;
        a_pix[i] = n * p.Hi * p.Wi;
        a_ih[i] = p.is * qh;
        a_iw[i] = p.is * qw;
    }
    int b_row[2];
    bool b_ok[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int nn = nt * BN + 16 * wave + 8 * j + lrow;
        b_ok[j] = nn < p.Co;
        b_row[j] = b_ok[j] ? nn : 0;
    }
    const int cpt = p.Ci / BK;
    const int KT = ph.ntaps * cpt;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.xbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, p.wbytes, 0x00020000);

    // per-stage tap parameters (scalar loads from the phase table), fetched one step ahead so their
    // latency is not exposed after the barrier
    struct StageArgs { int live, c0, dh, dw, wt; };
    auto stage_args = [&](int kt_req) {
        StageArgs a;
        a.live = kt_req < KT;
        const int kt = min(kt_req, KT - 1);
        const int chunk = kt / ph.ntaps, tap = kt - chunk * ph.ntaps;   // channel chunk outer, taps inner
        a.c0 = chunk * BK + cch * EPC;
        a.dh = ph.dh[tap]; a.dw = ph.dw[tap]; a.wt = ph.wt[tap];
        return a;
    };
    // the 6 DMA instructions of one K-stage into ring slot `slot` (always 6: the vmcnt counts are static)
    auto issue = [&](const StageArgs& g, int slot) {
        char* As = smem + slot * STAGE;
        char* Bs = As + BM * 128;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int ih = a_ih[i] + g.dh, iw = a_iw[i] + g.dw;
            const bool ok = g.live && a_ok[i] && (unsigned)ih < (unsigned)p.Hi && (unsigned)iw < (unsigned)p.Wi;
            dma16(xrs, As + (32 * wave + 8 * i) * 128, sel_off(ok, ((a_pix[i] + ih * p.Wi + iw) * p.Ci + g.c0) * 2));
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
            dma16(wrs, Bs + (16 * wave + 8 * j) * 128,
                  sel_off(g.live && b_ok[j], (b_row[j] * p.wrow + g.wt * p.Ci + g.c0) * 2));
    };

    const int wm = wave / WN, wn = wave - (wave / WN) * WN;
    const int l16 = lane & 15, lg = lane >> 4;
    const int l7 = l16 & 7;
    f32x4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};

    issue(stage_args(0), 0);
    issue(stage_args(1), 1);
    int slot = 0;
    for (int kt = 0; kt < KT; ++kt) {
        const StageArgs nxt = stage_args(kt + 2);
        // this wave's DMAs of stage kt have landed (stage kt+1's 6 stay in flight); after the barrier
        // every wave's have, and every wave is done reading the slot that stage kt+2 overwrites
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if constexpr (SCD_ABLATE == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else issue(nxt, slot == 0 ? 2 : slot - 1);
        const char* As = smem + slot * STAGE;
        const char* Bs = As + BM * 128;
        h16x8 af[2][4], bfr[2][4];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int co = ((s * 4 + lg) ^ l7) << 4;
#pragma unroll
            for (int a = 0; a < 4; ++a) af[s][a] = *(const h16x8*)(As + (wm * 64 + a * 16 + l16) * 128 + co);
#pragma unroll
            for (int b = 0; b < 4; ++b) bfr[s][b] = *(const h16x8*)(Bs + (wn * 64 + b * 16 + l16) * 128 + co);
        }
        if constexpr (SCD_ABLATE == 1) {
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int a = 0; a < 4; ++a) acc[a][0][0] += (float)af[s][a][0] + (float)bfr[s][a][0];
        } else {
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int a = 0; a < 4; ++a)
#pragma unroll
                    for (int b = 0; b < 4; ++b)
                        acc[a][b] = mfma_16x16x32_h16(bfr[s][b], af[s][a], acc[a][b]);
            __builtin_amdgcn_s_setprio(0);
        }
        slot = slot == 2 ? 0 : slot + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    gemm_epilogue<T, BM, BN, WN, HEADS, BNB>(p, acc, smem, tid, bid, mt, nt, M, QQ, ph);
}

// -------------------------------------------------------------------------------------
// Ping-pong bf16 gather-GEMM for the large shapes: 256 x BN tile (BN = 256 or 192), 8 waves in two
// groups of 4 (group g owns pixel rows 128g..128g+127, wave wc of a group owns BN/4 output channels),
// BK = 64, two LDS stage buffers.  Each K-stage runs as 4 phases (one 32-pixel quarter of the
// group's rows each); a phase is an L part (fragment reads + 2 LDS-DMA issues for the NEXT stage)
// and a C part (lgkmcnt(0), 4*NB MFMAs), each closed by an s_barrier.  Group 1 starts one barrier
// late, so on every SIMD one wave's MFMAs run while its partner reads LDS and issues DMA: the matrix
// pipe never waits for the fragment reads of the whole workgroup (the single-barrier ring kernel
// above spends ~40% of each K-step that way).
// DMA schedule per group and stage t (filling buffer (t+1)&1): P1 B rows part 1 (2 instr), P2 B part
// 2 (NB2), P3 own A rows 0..63 (2), P4 own A rows 64..127 (2); counted waits: end of L4 vmcnt(4)
// (both B parts of t+1 landed), end of C4 vmcnt(2) (A rows 0..63), end of C2 vmcnt(2+NB2) (A rows
// 64..127 of stage t).  Every region is rewritten >= 3 phases after its last fragment read.
template <int BN, bool HEADS, bool BNB = false>
__global__ __launch_bounds__(512, 1) void conv_gemm_pp_kernel(GemmParams p) {
    typedef h16 T;
    constexpr int BM = 256, BK = 64, EPC = 8;
    constexpr int NB = BN / 64;                 // 16-channel blocks per wave
    constexpr int WCOLS = BN / 4;               // channels per wave
    constexpr int NB2 = (BN / 2 - 64) / 32;     // B part-2 DMA instructions per thread (2 or 1)
    constexpr int STAGE = (BM + BN) * 128;
    constexpr int EROW = WCOLS * 2 + 16;        // epilogue staging row
    constexpr int EPI = 8 * 128 * EROW;
    constexpr int EPX = EPI + 4 * BN * 4 + (HEADS ? 256 * 8 * 4 : 0);    // + the heads' partial exchange
    constexpr int SMEM = (2 * STAGE > EPX) ? 2 * STAGE : EPX;
    static_assert(BN == 256 || BN == 192, "BN");
    __shared__ __attribute__((aligned(16))) char smem[SMEM];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2, wc = wave & 3;
    int bid;
    {
        const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7, xcd = blockIdx.x & 7;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (blockIdx.x >> 3);
    }
    int phase = 0;
#pragma unroll
    for (int i = 1; i < SCD_MAX_PHASES; ++i)
        if (i < p.nphase && bid >= p.tile_start[i]) phase = i;
    const scd_gemm_phase& ph = p.ph[phase];
    const int local = bid - p.tile_start[phase];
    const int mt = local / p.ntn;
    const int nt = local - mt * p.ntn;
    const int QQ = ph.Qh * ph.Qw;
    const int M = p.N * QQ;

    // DMA rows of this lane (the lane fetches chunk (lane&7)^(row&7) so that LDS slot lane&7 holds it)
    const int lrow = lane >> 3;
    const int cch = (lane & 7) ^ lrow;
    // A: rows 128*grp + 64*h + 16*wc + 8*j + lrow  (h, j in {0,1}); index i = 2h + j.  Per row the lane keeps
    // its byte offset at tap (0,0) of channel chunk 0 and a bit mask of the phase's taps that land inside
    // the image; a stage then costs one scalar delta ((dh*Wi + dw)*Ci + chunk*BK)*2, one add and one bit
    // test per DMA (no multiplies or bounds compares in the K loop)
    int a_base[4];
    unsigned a_mask[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = mt * BM + 128 * grp + 64 * (i >> 1) + 16 * wc + 8 * (i & 1) + lrow;
        const bool ok = m < M;
        const int mm = ok ? m : 0;
        const int n = mm / QQ;
        const int rem = mm - n * QQ;
        const int qh = rem / ph.Qw;
        const int qw = rem - qh * ph.Qw;
        const int ih0 = p.is * qh, iw0 = p.is * qw;
        a_base[i] = ((n * p.Hi + ih0) * p.Wi + iw0) * p.Ci * 2 + cch * EPC * 2;
        unsigned msk = 0;
        for (int t = 0; t < ph.ntaps; ++t) {
            const int ih = ih0 + ph.dh[t], iw = iw0 + ph.dw[t];
            if (ok && (unsigned)ih < (unsigned)p.Hi && (unsigned)iw < (unsigned)p.Wi) msk |= 1u << t;
        }
        a_mask[i] = msk;
    }
    // B: part 1 rows (BN/2)*grp + 16*wc + 8*j + lrow (j < 2); part 2 rows (BN/2)*grp + 64 + 8*NB2*wc + 8*(j-2) + lrow
    int b_base[2 + NB2];
    bool b_ok[2 + NB2];
#pragma unroll
    for (int j = 0; j < 2 + NB2; ++j) {
        const int r = (BN / 2) * grp + (j < 2 ? 16 * wc + 8 * j : 64 + 8 * NB2 * wc + 8 * (j - 2)) + lrow;
        const int nn = nt * BN + r;
        b_ok[j] = nn < p.Co;
        b_base[j] = ((b_ok[j] ? nn : 0) * p.wrow + cch * EPC) * 2;
    }
    const int cpt = p.Ci / BK;
    const int KT = ph.ntaps * cpt;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.xbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, p.wbytes, 0x00020000);

    struct StageArgs { int live, tap, adelta, bdelta; };
    auto stage_args = [&](int kt_req) {
        StageArgs a;
        a.live = kt_req < KT;
        const int kt = min(kt_req, KT - 1);
        const int chunk = kt / ph.ntaps, tap = kt - chunk * ph.ntaps;   // channel chunk outer, taps inner
        a.tap = tap;
        a.adelta = ((ph.dh[tap] * p.Wi + ph.dw[tap]) * p.Ci + chunk * BK) * 2;
        a.bdelta = (ph.wt[tap] * p.Ci + chunk * BK) * 2;
        return a;
    };
    auto issue_a = [&](const StageArgs& g, char* buf, int h) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int i = 2 * h + j;
            const bool ok = g.live && ((a_mask[i] >> g.tap) & 1u);
            dma16(xrs, buf + (128 * grp + 64 * h + 16 * wc + 8 * j) * 128, sel_off(ok, a_base[i] + g.adelta));
        }
    };
    auto issue_b = [&](const StageArgs& g, char* buf, int part) {
        char* Bs = buf + BM * 128;
#pragma unroll
        for (int j = (part ? 2 : 0); j < (part ? 2 + NB2 : 2); ++j) {
            const int r = (BN / 2) * grp + (j < 2 ? 16 * wc + 8 * j : 64 + 8 * NB2 * wc + 8 * (j - 2));
            dma16(wrs, Bs + r * 128, sel_off(g.live && b_ok[j], b_base[j] + g.bdelta));
        }
    };

    const int l16 = lane & 15, lg = lane >> 4;
    const int l7 = l16 & 7;
    const int co0 = ((0 * 4 + lg) ^ l7) << 4, co1 = ((1 * 4 + lg) ^ l7) << 4;
    f32x4 acc[8][NB];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < NB; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
    h16x8 bfr[NB][2], afx[2][2], afy[2][2];

    auto read_b = [&](const char* buf) {
        const char* Bs = buf + BM * 128;
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const char* row = Bs + (wc * WCOLS + b * 16 + l16) * 128;
            bfr[b][0] = *(const h16x8*)(row + co0);
            bfr[b][1] = *(const h16x8*)(row + co1);
        }
    };
    auto read_a = [&](const char* buf, int q, h16x8 (&af)[2][2]) {
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            const char* row = buf + (128 * grp + 32 * q + 16 * a + l16) * 128;
            af[a][0] = *(const h16x8*)(row + co0);
            af[a][1] = *(const h16x8*)(row + co1);
        }
    };
    auto mfma_q = [&](int q, const h16x8 (&af)[2][2]) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (SCD_ABLATE == 1) {       // ablation: fragments read, no MFMA
#pragma unroll
            for (int s = 0; s < 2; ++s) {
#pragma unroll
                for (int a = 0; a < 2; ++a) asm volatile("" ::"v"(af[a][s]));
#pragma unroll
                for (int b = 0; b < NB; ++b) asm volatile("" ::"v"(bfr[b][s]));
            }
            return;
        }
        if constexpr (PP_PRIO == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < NB; ++b)
                    acc[2 * q + a][b] = mfma_16x16x32_h16(bfr[b][s], af[a][s], acc[2 * q + a][b]);
        if constexpr (PP_PRIO == 1) __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
    };
    // ablations (SCD_GEMM_DEBUG): 3 = no DMA instructions in the loop, 4 = no fragment reads in the loop,
    // 5 = no barriers in the loop, 60 = no output stores, 61 = no epilogue (timing only; 3-5, 60, 61 give wrong
    // results; tools/pp_probe.py)
    constexpr int dbg = SCD_ABLATE;
    auto bar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (dbg != 5) __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };

    SCD_STAMP_BEGIN();
    if (KT > 0) {
        {
            const StageArgs g0 = stage_args(0);
            issue_b(g0, smem, 0);
            issue_b(g0, smem, 1);
            issue_a(g0, smem, 0);
            issue_a(g0, smem, 1);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bar();
        if constexpr (dbg == 4) { read_b(smem); read_a(smem, 0, afx); read_a(smem, 1, afy); }
        if (grp == 1) bar();                 // stagger: group 1 runs one barrier behind
        if constexpr (PP_PRIO == 2) { if (grp == 1) __builtin_amdgcn_s_setprio(1); }
        for (int t = 0; t < KT; ++t) {
            char* cur = smem + (t & 1) * STAGE;
            char* nxt = smem + ((t & 1) ^ 1) * STAGE;
            StageArgs g = stage_args(t + 1);
            if constexpr (dbg == 2) g.live = 0;      // ablation: loop DMAs read nothing
            // P1
            if constexpr (dbg != 4) read_b(cur);
            if constexpr (dbg != 4) read_a(cur, 0, afx);
            if constexpr (dbg != 3) issue_b(g, nxt, 0);
            bar();
            mfma_q(0, afx);
            bar();
            // P2
            if constexpr (dbg != 4) read_a(cur, 1, afy);
            if constexpr (dbg != 3) issue_b(g, nxt, 1);
            bar();
            mfma_q(1, afy);
            if constexpr (NB2 == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
            bar();
            // P3
            if constexpr (dbg != 4) read_a(cur, 2, afx);
            if constexpr (dbg != 3) issue_a(g, nxt, 0);
            bar();
            mfma_q(2, afx);
            bar();
            // P4
            if constexpr (dbg != 4) read_a(cur, 3, afy);
            if constexpr (dbg != 3) issue_a(g, nxt, 1);
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            bar();
            mfma_q(3, afy);
            asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
            bar();
        }
        if (grp == 0) bar();
        if constexpr (PP_PRIO == 2) __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    SCD_STAMP_END();
    if constexpr (dbg == 61) {                 // ablation 61: no epilogue (the accumulators kept live by a test)
        float s = 0.f;
#pragma unroll
        for (int a = 0; a < 8; ++a)
#pragma unroll
            for (int b = 0; b < NB; ++b) s += acc[a][b][0] + acc[a][b][1] + acc[a][b][2] + acc[a][b][3];
        if (s == 1234.5f) ((float*)p.y)[tid] = s;
        return;
    }

    // ---- epilogue: bias / relu in registers, BN partial sums, stage the wave's 128 x WCOLS tile, coalesced stores
    char* ep = smem + wave * 128 * EROW;
    float csum[NB][4], csq[NB][4];
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) { csum[b][r] = 0.f; csq[b][r] = 0.f; }
    constexpr int CPR = WCOLS * 2 / 16;                      // 16-B chunks per staged row (8 or 6)
    // output element offset of tile row `row` (< 128 of this group), channel `col` (M-range checked by the caller)
    // the store loops walk a lane's pixels m, m + RPI, m + 2 RPI, ... of the tile: (n, qh, qw) advanced by
    // additions instead of two integer divisions per 16-B store (~50 VALU each, 16 stores per lane and tile)
    struct PixPos { int n, qh, qw; };
    auto pix_of = [&](int m) -> PixPos {
        PixPos q;
        q.n = m / QQ;
        const int rem = m - q.n * QQ;
        q.qh = rem / ph.Qw;
        q.qw = rem - q.qh * ph.Qw;
        return q;
    };
    auto pix_advance = [&](PixPos& q, int step) {
        q.qw += step;
        while (q.qw >= ph.Qw) {
            q.qw -= ph.Qw;
            if (++q.qh == ph.Qh) { q.qh = 0; ++q.n; }
        }
    };
    auto out_off = [&](const PixPos& q, int col) -> long {
        const int oh = p.os * q.qh + ph.rho_h, ow = p.os * q.qw + ph.rho_w;
        if (p.shuf) {
            const int c4 = p.Co >> 2, sp = col / c4;
            return ((long)(q.n * 2 * p.Ho + 2 * oh + (sp >> 1)) * (2 * p.Wo) + 2 * ow + (sp & 1)) * c4 + (col - sp * c4);
        }
        return ((long)(q.n * p.Ho + oh) * p.Wo + ow) * p.Co + col;
    };
    // BN-backward mode (below): the lane's rows of the pre-BN activation are loaded now, in flight while the
    // accumulators are staged (the fragment registers are free after the main loop); PP_YPF=0 loads them in the
    // store loop
    float bias[NB][4];                                       // before the row loads (in-order returns)
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const int col0 = nt * BN + wc * WCOLS + b * 16 + lg * 4;
#pragma unroll
        for (int r = 0; r < 4; ++r) bias[b][r] = (p.bias && col0 + r < p.Co) ? p.bias[col0 + r] : 0.f;
    }
    constexpr int RPI = 64 / CPR;                            // rows per pass (8, or 10 with 4 lanes idle)
    constexpr int NIT = (128 + RPI - 1) / RPI;
    const int rsub = lane / CPR, chx = lane - (lane / CPR) * CPR;
    // Buffer loads with no branch around them (rows past M / columns past Co take an out-of-range offset and read
    // zeros), so the compiler's wait for the bias loads above them stays a counted one
    uint4 ypf[PP_YPF && BNB ? NIT : 1];
    if constexpr (PP_YPF && BNB) {
        const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.bny, (short)0, p.ybytes, 0x00020000);
        const int colb = nt * BN + wc * WCOLS + chx * EPC;
        const bool cok = rsub < RPI && colb < p.Co;
        const int cl = cok ? colb : 0;
        PixPos pq = pix_of(mt * BM + 128 * grp + rsub);
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int row = it * RPI + rsub;
            const bool ok = cok && row < 128 && mt * BM + 128 * grp + row < M;
            const int off = (int)out_off(pq, cl) * (int)sizeof(T);
            pix_advance(pq, RPI);
            ypf[it] = bload(yrs, sel_off(ok, off));
        }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
#pragma unroll
        for (int a = 0; a < 8; ++a) {
            const int m = mt * BM + 128 * grp + a * 16 + l16;
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                v[r] = acc[a][b][r] + bias[b][r];
                if (p.relu) v[r] = fmaxf(v[r], 0.f);
            }
            if constexpr (!BNB) {
                // a select per element, not a branch region per fragment (the sums never hold -0, so adding +0 for
                // rows past M leaves them unchanged)
                const bool mok = m < M;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float t = mok ? v[r] : 0.f;
                    csum[b][r] += t;
                    csq[b][r] += t * t;
                }
            }
            typedef __attribute__((ext_vector_type(4))) h16 bf16x4;
            bf16x4 o = {(h16)v[0], (h16)v[1], (h16)v[2], (h16)v[3]};
            *(bf16x4*)(ep + (a * 16 + l16) * EROW + (b * 16 + lg * 4) * 2) = o;
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     // the staged tile is wave-private
    // BN-backward mode (scd_conv_gemm_bnbwd: the output is the gradient of a following BN+ReLU layer): its backward
    // sums come from the stored gradient and the pre-BN activation, read in the store phase as whole 128-B row pieces
    // (lane: fixed 16-B channel chunk, RPI rows per pass) -- not as 8-B pieces per accumulator fragment
    float bs8[EPC], bq8[EPC];
    if constexpr (BNB) {
        const int colb = nt * BN + wc * WCOLS + chx * EPC;
        const bool cok = rsub < RPI && colb < p.Co;
        const int cl = cok ? colb : 0;
        float mu[EPC], is[EPC], sc[EPC], sh[EPC];
#pragma unroll
        for (int e = 0; e < EPC; e += 4) {
            const float4 f0 = *(const float4*)(p.bn_mean + cl + e), f1 = *(const float4*)(p.bn_invstd + cl + e);
            const float4 f2 = *(const float4*)(p.bn_rsc + cl + e), f3 = *(const float4*)(p.bn_rsh + cl + e);
            mu[e] = f0.x; mu[e + 1] = f0.y; mu[e + 2] = f0.z; mu[e + 3] = f0.w;
            is[e] = f1.x; is[e + 1] = f1.y; is[e + 2] = f1.z; is[e + 3] = f1.w;
            sc[e] = f2.x; sc[e + 1] = f2.y; sc[e + 2] = f2.z; sc[e + 3] = f2.w;
            sh[e] = f3.x; sh[e + 1] = f3.y; sh[e + 2] = f3.z; sh[e + 3] = f3.w;
        }
#pragma unroll
        for (int e = 0; e < EPC; ++e) { bs8[e] = 0.f; bq8[e] = 0.f; }
        // the accumulate branch outside the row loop: a load under a branch inside it makes the compiler's waitcnt
        // pass drain every outstanding access (the previous rows' stores included) at each row
        auto rows = [&](auto acc_c) {
            constexpr bool ACC = decltype(acc_c)::value;
            PixPos pq = pix_of(mt * BM + 128 * grp + rsub);
#pragma unroll
            for (int it = 0; it < NIT; ++it) {
                const int row = it * RPI + rsub;
                const int m = mt * BM + 128 * grp + row;
                const bool ok = cok && row < 128 && m < M;
                // every load from a valid address (row 0 / pixel 0 when masked off): no branch around the loads
                const long off = ok ? out_off(pq, cl) : 0;
                pix_advance(pq, RPI);
                uint4 v = *(const uint4*)(ep + (ok ? row : 0) * EROW + chx * 16);
                T* dst = (T*)(p.y) + off;
                if constexpr (ACC) {
                    float a8[EPC], o8[EPC];
                    Vec16<T>::load(&v, a8);
                    Vec16<T>::load(dst, o8);
#pragma unroll
                    for (int e = 0; e < EPC; ++e) a8[e] += o8[e];
                    Vec16<T>::store(&v, a8);
                }
                float d8[EPC], y8[EPC];
                Vec16<T>::load(&v, d8);
                if constexpr (PP_YPF && BNB) Vec16<T>::load(&ypf[it], y8);
                else Vec16<T>::load((const T*)p.bny + off, y8);
                // the sums on every row (+0 for rows masked off; they never hold -0) and only the store under the
                // branch: the BN parameters are then waited for once, not on every row behind the previous store
#pragma unroll
                for (int e = 0; e < EPC; ++e) {
                    const float dz = ok && y8[e] * sc[e] + sh[e] > 0.f ? d8[e] : 0.f;
                    bs8[e] += dz;
                    bq8[e] += dz * (y8[e] - mu[e]) * is[e];
                }
                if (ok) {
                    if constexpr (dbg == 60) asm volatile("" ::"v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));
                    else *(uint4*)dst = v;
                }
            }
        };
        if (p.accumulate) rows(std::true_type{});
        else rows(std::false_type{});
    } else {
        // lane: 16-B channel chunk chx of rows rsub, rsub + RPI, ... (RPI = 64 / CPR rows per pass; 4 lanes idle when
        // CPR = 6).  Rows past M / columns past Co compute on a valid address (pixel 0, channel 0) and skip only the
        // store: no branch around the accumulate load
        const int col = nt * BN + wc * WCOLS + chx * EPC;
        auto rows = [&](auto acc_c) {
            constexpr bool ACC = decltype(acc_c)::value;
            PixPos pq = pix_of(mt * BM + 128 * grp + rsub);
#pragma unroll 4
            for (int it = 0; it < NIT; ++it) {
                const int row = it * RPI + rsub;
                const int m = mt * BM + 128 * grp + row;
                const bool ok = rsub < RPI && row < 128 && m < M && col < p.Co;
                T* dst = (T*)(p.y) + (ok ? out_off(pq, col) : 0);
                pix_advance(pq, RPI);
                uint4 v = *(const uint4*)(ep + (ok ? row : 0) * EROW + chx * 16);
                if constexpr (ACC) {
                    float a[EPC], o[EPC];
                    Vec16<T>::load(&v, a);
                    Vec16<T>::load(dst, o);
#pragma unroll
                    for (int e = 0; e < EPC; ++e) a[e] += o[e];
                    Vec16<T>::store(&v, a);
                }
                if constexpr (dbg == 60) asm volatile("" ::"v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));   // ablation 60: no stores
                else if (ok) *(uint4*)dst = v;
            }
        };
        if (p.accumulate) rows(std::true_type{});
        else rows(std::false_type{});
    }
    if (p.stats) {
        float* red = (float*)(smem + EPI);    // [2 groups][BN][2]
        if constexpr (BNB) {
            // the lanes' partials into the wave's own staging rows (read above, wave-private), then channel c of the
            // wave summed over its RPI row lanes in a fixed order
            float* part = (float*)ep;                        // [64 lanes][2 * EPC]
#pragma unroll
            for (int e = 0; e < EPC; ++e) { part[lane * 2 * EPC + e] = bs8[e]; part[lane * 2 * EPC + EPC + e] = bq8[e]; }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane < WCOLS) {
                const int cx = lane / EPC, e = lane - (lane / EPC) * EPC;
                float s = 0.f, q = 0.f;
                for (int r = 0; r < RPI; ++r) {
                    s += part[(r * CPR + cx) * 2 * EPC + e];
                    q += part[(r * CPR + cx) * 2 * EPC + EPC + e];
                }
                red[(grp * BN + wc * WCOLS + lane) * 2 + 0] = s;
                red[(grp * BN + wc * WCOLS + lane) * 2 + 1] = q;
            }
        } else {
#pragma unroll
            for (int b = 0; b < NB; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float s = csum[b][r], q = csq[b][r];
                    if constexpr (PP_DPP) {
                        s = row16_sum(s);
                        q = row16_sum(q);
                    } else {
#pragma unroll
                        for (int o = 1; o < 16; o <<= 1) { s += __shfl_xor(s, o, 64); q += __shfl_xor(q, o, 64); }
                    }
                    if (l16 == 0) {
                        const int c = wc * WCOLS + b * 16 + lg * 4 + r;
                        red[(grp * BN + c) * 2 + 0] = s;
                        red[(grp * BN + c) * 2 + 1] = q;
                    }
                }
        }
        __syncthreads();
        if (tid < BN) {
            const int col = nt * BN + tid;
            if (col < p.Co) {
                const double s = (double)red[tid * 2] + (double)red[(BN + tid) * 2];
                const double q = (double)red[tid * 2 + 1] + (double)red[(BN + tid) * 2 + 1];
                const int rep = bid % SCD_STAT_REPLICAS;
                atomic_add_f64(p.stats + ((long)rep * 2 + 0) * p.Co + col, s);
                atomic_add_f64(p.stats + ((long)rep * 2 + 1) * p.Co + col, q);
            }
        }
    }
    if constexpr (HEADS) {
        // fused CenterNet tails (centerNetOffset.py:108-110): out_h[o] = b1_h[o] + sum_j w1_h[o][j] * hid[128h + j]
        // from the staged tile.  Waves 0-3 take the first BN/2 tile channels of pixels 64*wave + lane, waves 4-7
        // the second half of the same pixels: the half (hence every weight address) is wave-uniform, so the
        // 1x1 weights come in through the scalar cache, and the lanes' staged rows (EROW apart) are read without
        // bank conflicts.  The second-half partials meet the first half's through LDS; a head split between two
        // column tiles gets two partial sums, added onto its zeroed output (two commutative fp32 adds onto 0:
        // the same bits in either order).
        __syncthreads();
        const int half = wave >> 2;                            // wave-uniform
        const int r = (wave & 3) * 64 + lane;                  // tile pixel
        const int g = r >> 7, row = r & 127;
        const int hbase = (nt * BN) >> 7;
        const float* wA = p.head_w[hbase];
        const float* wB = hbase + 1 < 4 ? p.head_w[hbase + 1] : nullptr;
        float a0[4] = {0.f, 0.f, 0.f, 0.f}, a1[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int cc = 0; cc < BN / 2; cc += EPC) {
            const int c = half * (BN / 2) + cc;                // tile channel (wave-uniform)
            const int wv = c / WCOLS, cl = c - (c / WCOLS) * WCOLS;
            float v[EPC];
            Vec16<T>::load(smem + (4 * g + wv) * 128 * EROW + row * EROW + cl * 2, v);
            const int gc = nt * BN + c;
            const int hs = (gc >> 7) - hbase, j = gc & 127;
            const int od = p.head_od[hbase + hs];
            const float* w = hs ? wB : wA;
#pragma unroll
            for (int o = 0; o < 4; ++o) {
                if (o < od) {
                    float a = 0.f;
#pragma unroll
                    for (int e = 0; e < EPC; ++e) a += v[e] * w[o * 128 + j + e];
                    if (hs) a1[o] += a; else a0[o] += a;
                }
            }
        }
        float* xch = (float*)(smem + EPI + 4 * BN * 4);        // [256 px][8]: second-half partials
        if (half) {
#pragma unroll
            for (int o = 0; o < 4; ++o) { xch[r * 8 + o] = a0[o]; xch[r * 8 + 4 + o] = a1[o]; }
        }
        __syncthreads();
        const int m = mt * BM + r;
        if (half == 0 && m < M) {
#pragma unroll
            for (int o = 0; o < 4; ++o) { a0[o] += xch[r * 8 + o]; a1[o] += xch[r * 8 + 4 + o]; }
            const int n = m / QQ;
            const int rem = m - n * QQ;
            const int oh = rem / ph.Qw, ow = rem - (rem / ph.Qw) * ph.Qw;
            const long HWo = (long)p.Ho * p.Wo;
#pragma unroll
            for (int hs = 0; hs < 2; ++hs) {
                const int h = hbase + hs;
                if (h >= 4 || !p.head_out[h] || h * 128 >= nt * BN + BN) continue;
                const int od = p.head_od[h];
                const bool first = h * 128 >= nt * BN, full = first && h * 128 + 128 <= nt * BN + BN;
#pragma unroll
                for (int o = 0; o < 4; ++o) {
                    if (o >= od) continue;
                    const float val = (hs ? a1[o] : a0[o]) + (first ? p.head_b[h][o] : 0.f);
                    float* dst = p.head_out[h] + ((long)n * od + o) * HWo + (long)oh * p.Wo + ow;
                    if (full) *dst = val;
                    else atomic_add_f32(dst, val);
                }
            }
        }
    }
}

// -------------------------------------------------------------------------------------
// Two-workgroups-per-CU bf16 gather-GEMM ("duo", round 6).  The ping-pong kernel above holds a CU
// alone (two 64-KiB stages, 8 waves x ~206 VGPRs), so nothing runs while its tile epilogue stores 128 KiB and (BN
// backward) reads another 128 KiB: stamped in the step's shapes, the main loops take 53 % of the heatmap-head input
// gradient and 76 % of the deconv3 one (profiles/r6_clock.txt), the rest is per-tile epilogue and prologue with the
// matrix pipe idle.  Here a 256 x 128 tile belongs to a 4-wave workgroup (waves 2 x 2, 128 x 64 each: the
// ping-pong kernel's per-wave tile, fragment reads per MFMA and epilogue), its LDS is a 3-slot ring of BK = 32
// stages (rows of 64 B, 24 KiB per stage) that the epilogue reuses as its staging buffer, and its registers fit
// 2 waves per SIMD -- so TWO workgroups share each CU, and one's epilogue runs beside the other's MFMAs.  The
// workgroups of the first round's second slot (blockIdx in [CUs, 2 CUs)) start half a tile late (s_sleep), so the two
// slots of a CU stay half a tile apart for the whole launch.
// K order: (64-channel chunk, tap, 32-channel half), so both halves of a pixel's 128-B line are fetched in
// consecutive K-steps, and every output sees the same MFMA sequence as the ping-pong kernel's (chunk, tap, s = half):
// bit-identical results.
// LDS row r (64 B, 4 chunks of 16 B): chunk c in slot c ^ F[(r >> 2) & 3], F = {0, 2, 3, 1}: the 16 lanes of every
// ds_read_b128 lane group (rows l16, chunk lg) then hit 16 distinct 16-B units of the 256-B bank window; the DMA
// writes a wave-instruction's 1 KiB lane-linearly (16 rows), so the swizzle is applied to the source chunk.
// One barrier per K-step: wait for this wave's DMAs of stage k (vmcnt(6): stage k+1's 6 stay in flight), barrier,
// issue stage k+2 into the slot stage k-1 used, read the fragments of stage k, 32 MFMAs.
#ifndef DUO_PRIO
#define DUO_PRIO 1    // duo kernel: s_setprio 1 around a K-step's MFMAs (A/B build option)
#endif
#ifndef DUO_ILV
#define DUO_ILV 1     // duo kernel: DMA issues and fragment reads interleaved with the MFMAs (A/B build option)
#endif
__device__ __forceinline__ int duo_swz(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }

__global__ __launch_bounds__(256, 2) void conv_gemm_duo_kernel(GemmParams p) {
    typedef h16 T;
    constexpr int BM = 256, BN = 128, BK = 32, EPC = 8;
    constexpr int NB = 4, WCOLS = 64;            // per wave: 8 x 4 blocks of 16 x 16 (128 pixels x 64 channels)
    constexpr int ROWB = BK * 2;                 // 64-B LDS rows
    constexpr int STAGE = (BM + BN) * ROWB;      // 24 KiB
    constexpr int NSLOT = 3;
    constexpr int EROW = WCOLS * 2 + 16;         // epilogue staging row (144 B)
    constexpr int EPI = 4 * 128 * EROW;          // 72 KiB = the ring
    constexpr int RING = NSLOT * STAGE;
    constexpr int SMEM = (RING > EPI ? RING : EPI) + 2 * BN * 2 * 4;    // + the BN partial sums [2][BN][2]
    __shared__ __attribute__((aligned(16))) char smem[SMEM];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    int bid;
    {
        const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7, xcd = blockIdx.x & 7;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (blockIdx.x >> 3);
    }
    // the first round's second workgroup per CU starts about half a tile late (host-sized, p.duo_delay x 8K cycles)
    if ((int)blockIdx.x >= p.duo_ncu && (int)blockIdx.x < 2 * p.duo_ncu) {
        for (int i = 0; i < p.duo_delay; ++i) __builtin_amdgcn_s_sleep(127);
    }
    int phase = 0;
#pragma unroll
    for (int i = 1; i < SCD_MAX_PHASES; ++i)
        if (i < p.nphase && bid >= p.tile_start[i]) phase = i;
    const scd_gemm_phase& ph = p.ph[phase];
    const int local = bid - p.tile_start[phase];
    const int mt = local / p.ntn;
    const int nt = local - mt * p.ntn;
    const int QQ = ph.Qh * ph.Qw;
    const int M = p.N * QQ;

    // DMA: lane -> row lr = lane / 4 of a 16-row piece, LDS slot lane & 3, source chunk (lane & 3) ^ F[lane / 16]
    const int lr = lane >> 2;
    const int cch = (lane & 3) ^ duo_swz(lr);
    // A rows 64 * wave + 16 i + lr (i < 4): byte offset at tap (0, 0) of channel 0 + in-image tap mask
    int a_base[4];
    unsigned a_mask[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = mt * BM + 64 * wave + 16 * i + lr;
        const bool ok = m < M;
        const int mm = ok ? m : 0;
        const int n = mm / QQ;
        const int rem = mm - n * QQ;
        const int qh = rem / ph.Qw;
        const int qw = rem - qh * ph.Qw;
        const int ih0 = p.is * qh, iw0 = p.is * qw;
        a_base[i] = ((n * p.Hi + ih0) * p.Wi + iw0) * p.Ci * 2 + cch * 16;
        unsigned msk = 0;
        for (int t = 0; t < ph.ntaps; ++t) {
            const int ih = ih0 + ph.dh[t], iw = iw0 + ph.dw[t];
            if (ok && (unsigned)ih < (unsigned)p.Hi && (unsigned)iw < (unsigned)p.Wi) msk |= 1u << t;
        }
        a_mask[i] = msk;
    }
    // B rows 32 * wave + 16 j + lr (j < 2)
    int b_base[2];
    bool b_ok[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int nn = nt * BN + 32 * wave + 16 * j + lr;
        b_ok[j] = nn < p.Co;
        b_base[j] = (b_ok[j] ? nn : 0) * p.wrow * 2 + cch * 16;
    }
    const int KT = ph.ntaps * (p.Ci / 64) * 2;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.xbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, p.wbytes, 0x00020000);

    struct StageArgs { int live, tap, adelta, bdelta; };
    auto stage_args = [&](int kt_req) {
        StageArgs a;
        a.live = kt_req < KT;
        const int kt = min(kt_req, KT - 1);
        const int h = kt & 1, k2 = kt >> 1;
        const int chunk = k2 / ph.ntaps, tap = k2 - chunk * ph.ntaps;   // 64-channel chunk outer, tap, half inner
        a.tap = tap;
        a.adelta = ((ph.dh[tap] * p.Wi + ph.dw[tap]) * p.Ci + chunk * 64 + h * 32) * 2;
        a.bdelta = (ph.wt[tap] * p.Ci + chunk * 64 + h * 32) * 2;
        return a;
    };
    // the 6 DMA instructions of one K-step (always 6: the vmcnt counts are static)
    auto issue = [&](const StageArgs& g, char* buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const bool ok = g.live && ((a_mask[i] >> g.tap) & 1u);
            dma16(xrs, buf + (64 * wave + 16 * i) * ROWB, sel_off(ok, a_base[i] + g.adelta));
        }
        char* Bs = buf + BM * ROWB;
#pragma unroll
        for (int j = 0; j < 2; ++j)
            dma16(wrs, Bs + (32 * wave + 16 * j) * ROWB, sel_off(g.live && b_ok[j], b_base[j] + g.bdelta));
    };

    const int l16 = lane & 15, lg = lane >> 4;
    const int fo = (lg ^ duo_swz(l16)) << 4;     // this lane's chunk lg in any 16-row block
    f32x4 acc[8][NB];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < NB; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};

    SCD_STAMP_BEGIN();
    // fragments of stage k are read in iteration k and used by the MFMAs of iteration k + 1 (two register sets, X / Y):
    // the reads' latency hides behind the previous stage's MFMAs, and the next stage's DMA issues sit between them
    h16x8 bx[NB], ax[8], by[NB], ay[8];
    auto read_frags = [&](const char* As, h16x8 (&bf)[NB], h16x8 (&af)[8]) {
        const char* Bs = As + BM * ROWB;
#pragma unroll
        for (int b = 0; b < NB; ++b) bf[b] = *(const h16x8*)(Bs + (64 * wn + 16 * b + l16) * ROWB + fo);
#pragma unroll
        for (int a = 0; a < 8; ++a) af[a] = *(const h16x8*)(As + (128 * wm + 16 * a + l16) * ROWB + fo);
    };
    auto mfmas = [&](const h16x8 (&bf)[NB], const h16x8 (&af)[8]) {
        if constexpr (DUO_PRIO && !DUO_ILV) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int a = 0; a < 8; ++a)
#pragma unroll
            for (int b = 0; b < NB; ++b)
                acc[a][b] = mfma_16x16x32_h16(bf[b], af[a], acc[a][b]);
        if constexpr (DUO_PRIO && !DUO_ILV) __builtin_amdgcn_s_setprio(0);
    };
    // one K-step k >= 1: stage k landed everywhere (this wave: vmcnt(6) leaves stage k + 1's 6 in flight; its reads
    // of stage k - 1 drained: lgkmcnt(0), long done by now) -> barrier -> stage k + 2 into stage k - 1's slot ->
    // read stage k into (bn, an) -> MFMAs of stage k - 1 from (bo, ao)
    auto step = [&](int kt, int& cur, h16x8 (&bn)[NB], h16x8 (&an)[8], const h16x8 (&bo)[NB],
                    const h16x8 (&ao)[8]) {
        const StageArgs g = stage_args(kt + 2);
        asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const int nxs = cur == 0 ? 2 : cur - 1;
        if constexpr (!DUO_ILV) {
            issue(g, smem + nxs * STAGE);
            read_frags(smem + cur * STAGE, bn, an);
            mfmas(bo, ao);
        } else {
            // written in the interleaved order (the LDS-DMA builtin is a scheduling boundary, so the source order is
            // the issue order): per group one DMA issue, two fragment reads, four MFMAs of the previous stage
            if constexpr (DUO_PRIO) __builtin_amdgcn_s_setprio(1);
            char* nb = smem + nxs * STAGE;
            const char* As = smem + cur * STAGE;
            const char* Bs = As + BM * ROWB;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                if (q < 4) {
                    const bool ok = g.live && ((a_mask[q] >> g.tap) & 1u);
                    dma16(xrs, nb + (64 * wave + 16 * q) * ROWB, sel_off(ok, a_base[q] + g.adelta));
                } else if (q < 6) {
                    const int j = q - 4;
                    dma16(wrs, nb + BM * ROWB + (32 * wave + 16 * j) * ROWB,
                          sel_off(g.live && b_ok[j], b_base[j] + g.bdelta));
                }
                if (q < 2) {
                    bn[2 * q] = *(const h16x8*)(Bs + (64 * wn + 16 * (2 * q) + l16) * ROWB + fo);
                    bn[2 * q + 1] = *(const h16x8*)(Bs + (64 * wn + 16 * (2 * q + 1) + l16) * ROWB + fo);
                } else if (q < 6) {
                    const int a0 = 2 * (q - 2);
                    an[a0] = *(const h16x8*)(As + (128 * wm + 16 * a0 + l16) * ROWB + fo);
                    an[a0 + 1] = *(const h16x8*)(As + (128 * wm + 16 * (a0 + 1) + l16) * ROWB + fo);
                }
#pragma unroll
                for (int b = 0; b < NB; ++b)
                    acc[q][b] = mfma_16x16x32_h16(bo[b], ao[q], acc[q][b]);
            }
            if constexpr (DUO_PRIO) __builtin_amdgcn_s_setprio(0);
        }
        cur = cur == 2 ? 0 : cur + 1;
    };
    issue(stage_args(0), smem);
    issue(stage_args(1), smem + STAGE);
    {
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        issue(stage_args(2), smem + 2 * STAGE);
        read_frags(smem, by, ay);
    }
    int cur = 1;                                  // ring slot of stage kt
    int kt = 1;
    for (; kt + 1 < KT; kt += 2) {                // KT is even: pairs of steps 1..KT-2, then step KT-1
        step(kt, cur, bx, ax, by, ay);
        step(kt + 1, cur, by, ay, bx, ax);
    }
    step(kt, cur, bx, ax, by, ay);
    mfmas(bx, ax);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    SCD_STAMP_END();

    // ---- epilogue (the ping-pong kernel's, per wave 128 x 64): bias / relu, BN partial sums, the wave's tile staged in
    // the ring, coalesced 16-B NHWC stores (+= when accumulating; the BN-backward sums from the stored gradient)
    const int grp = wm, wc = wn;
    char* ep = smem + wave * 128 * EROW;
    float csum[NB][4], csq[NB][4];
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) { csum[b][r] = 0.f; csq[b][r] = 0.f; }
    constexpr int CPR = WCOLS * 2 / 16;                      // 8 chunks per staged row
    struct PixPos { int n, qh, qw; };
    auto pix_of = [&](int m) -> PixPos {
        PixPos q;
        q.n = m / QQ;
        const int rem = m - q.n * QQ;
        q.qh = rem / ph.Qw;
        q.qw = rem - q.qh * ph.Qw;
        return q;
    };
    auto pix_advance = [&](PixPos& q, int step) {
        q.qw += step;
        while (q.qw >= ph.Qw) {
            q.qw -= ph.Qw;
            if (++q.qh == ph.Qh) { q.qh = 0; ++q.n; }
        }
    };
    auto out_off = [&](const PixPos& q, int col) -> long {
        const int oh = p.os * q.qh + ph.rho_h, ow = p.os * q.qw + ph.rho_w;
        if (p.shuf) {
            const int c4 = p.Co >> 2, sp = col / c4;
            return ((long)(q.n * 2 * p.Ho + 2 * oh + (sp >> 1)) * (2 * p.Wo) + 2 * ow + (sp & 1)) * c4 + (col - sp * c4);
        }
        return ((long)(q.n * p.Ho + oh) * p.Wo + ow) * p.Co + col;
    };
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const int col0 = nt * BN + wc * WCOLS + b * 16 + lg * 4;
        float bias[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) bias[r] = (p.bias && col0 + r < p.Co) ? p.bias[col0 + r] : 0.f;
#pragma unroll
        for (int a = 0; a < 8; ++a) {
            const int m = mt * BM + 128 * grp + a * 16 + l16;
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                v[r] = acc[a][b][r] + bias[r];
                if (p.relu) v[r] = fmaxf(v[r], 0.f);
            }
            if (!p.bnbwd) {
                const bool mok = m < M;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float t = mok ? v[r] : 0.f;
                    csum[b][r] += t;
                    csq[b][r] += t * t;
                }
            }
            typedef __attribute__((ext_vector_type(4))) h16 bf16x4;
            bf16x4 o = {(h16)v[0], (h16)v[1], (h16)v[2], (h16)v[3]};
            *(bf16x4*)(ep + (a * 16 + l16) * EROW + (b * 16 + lg * 4) * 2) = o;
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     // the staged tile is wave-private
    constexpr int RPI = 64 / CPR;                            // 8 rows per pass
    constexpr int NIT = 128 / RPI;
    const int rsub = lane / CPR, chx = lane - (lane / CPR) * CPR;
    float bs8[EPC], bq8[EPC];
    if (p.bnbwd) {
        const int colb = nt * BN + wc * WCOLS + chx * EPC;
        const bool cok = colb < p.Co;
        const int cl = cok ? colb : 0;
        float mu[EPC], is[EPC], sc[EPC], sh[EPC];
#pragma unroll
        for (int e = 0; e < EPC; e += 4) {
            const float4 f0 = *(const float4*)(p.bn_mean + cl + e), f1 = *(const float4*)(p.bn_invstd + cl + e);
            const float4 f2 = *(const float4*)(p.bn_rsc + cl + e), f3 = *(const float4*)(p.bn_rsh + cl + e);
            mu[e] = f0.x; mu[e + 1] = f0.y; mu[e + 2] = f0.z; mu[e + 3] = f0.w;
            is[e] = f1.x; is[e + 1] = f1.y; is[e + 2] = f1.z; is[e + 3] = f1.w;
            sc[e] = f2.x; sc[e + 1] = f2.y; sc[e + 2] = f2.z; sc[e + 3] = f2.w;
            sh[e] = f3.x; sh[e + 1] = f3.y; sh[e + 2] = f3.z; sh[e + 3] = f3.w;
        }
#pragma unroll
        for (int e = 0; e < EPC; ++e) { bs8[e] = 0.f; bq8[e] = 0.f; }
        PixPos pq = pix_of(mt * BM + 128 * grp + rsub);
#pragma unroll 4
        for (int it = 0; it < NIT; ++it) {
            const int row = it * RPI + rsub;
            const int m = mt * BM + 128 * grp + row;
            const bool ok = cok && m < M;
            const long off = ok ? out_off(pq, cl) : 0;
            pix_advance(pq, RPI);
            uint4 v = *(const uint4*)(ep + row * EROW + chx * 16);
            T* dst = (T*)(p.y) + off;
            if (p.accumulate) {
                float a8[EPC], o8[EPC];
                Vec16<T>::load(&v, a8);
                Vec16<T>::load(dst, o8);
#pragma unroll
                for (int e = 0; e < EPC; ++e) a8[e] += o8[e];
                Vec16<T>::store(&v, a8);
            }
            float d8[EPC], y8[EPC];
            Vec16<T>::load(&v, d8);
            Vec16<T>::load((const T*)p.bny + off, y8);
            if (ok) {
#pragma unroll
                for (int e = 0; e < EPC; ++e) {
                    const float dz = y8[e] * sc[e] + sh[e] > 0.f ? d8[e] : 0.f;
                    bs8[e] += dz;
                    bq8[e] += dz * (y8[e] - mu[e]) * is[e];
                }
                *(uint4*)dst = v;
            }
        }
    } else {
        const int col = nt * BN + wc * WCOLS + chx * EPC;
        PixPos pq = pix_of(mt * BM + 128 * grp + rsub);
#pragma unroll 4
        for (int it = 0; it < NIT; ++it) {
            const int row = it * RPI + rsub;
            const int m = mt * BM + 128 * grp + row;
            const bool ok = m < M && col < p.Co;
            T* dst = (T*)(p.y) + (ok ? out_off(pq, col) : 0);
            pix_advance(pq, RPI);
            uint4 v = *(const uint4*)(ep + row * EROW + chx * 16);
            if (p.accumulate) {
                float a[EPC], o[EPC];
                Vec16<T>::load(&v, a);
                Vec16<T>::load(dst, o);
#pragma unroll
                for (int e = 0; e < EPC; ++e) a[e] += o[e];
                Vec16<T>::store(&v, a);
            }
            if (ok) *(uint4*)dst = v;
        }
    }
    if (p.stats) {
        float* red = (float*)(smem + (RING > EPI ? RING : EPI));    // [2 groups][BN][2]
        if (p.bnbwd) {
            float* part = (float*)ep;                        // [64 lanes][2 * EPC]
#pragma unroll
            for (int e = 0; e < EPC; ++e) { part[lane * 2 * EPC + e] = bs8[e]; part[lane * 2 * EPC + EPC + e] = bq8[e]; }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane < WCOLS) {
                const int cx = lane / EPC, e = lane - (lane / EPC) * EPC;
                float s = 0.f, q = 0.f;
                for (int r = 0; r < RPI; ++r) {
                    s += part[(r * CPR + cx) * 2 * EPC + e];
                    q += part[(r * CPR + cx) * 2 * EPC + EPC + e];
                }
                red[(grp * BN + wc * WCOLS + lane) * 2 + 0] = s;
                red[(grp * BN + wc * WCOLS + lane) * 2 + 1] = q;
            }
        } else {
#pragma unroll
            for (int b = 0; b < NB; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float s = row16_sum(csum[b][r]), q = row16_sum(csq[b][r]);
                    if (l16 == 0) {
                        const int c = wc * WCOLS + b * 16 + lg * 4 + r;
                        red[(grp * BN + c) * 2 + 0] = s;
                        red[(grp * BN + c) * 2 + 1] = q;
                    }
                }
        }
        __syncthreads();
        if (tid < BN) {
            const int col = nt * BN + tid;
            if (col < p.Co) {
                const double s = (double)red[tid * 2] + (double)red[(BN + tid) * 2];
                const double q = (double)red[tid * 2 + 1] + (double)red[(BN + tid) * 2 + 1];
                const int rep = bid % SCD_STAT_REPLICAS;
                atomic_add_f64(p.stats + ((long)rep * 2 + 0) * p.Co + col, s);
                atomic_add_f64(p.stats + ((long)rep * 2 + 1) * p.Co + col, q);
            }
        }
    }
}

// -------------------------------------------------------------------------------------
// CenterNet head convolution (centerNetOffset.py:106-110) for the three 128-wide heads: ONE 192 x 384 tile
// covers every hidden channel of 192 pixels, so the input (A) panel is read once (the 256 x 192 ping-pong
// tiles above read it twice, through L2) and each head's 1x1 tail sees its whole hidden vector in the same
// workgroup (no partial sums, no atomics, no memset).  8 waves in two staggered groups of 4 (ping-pong, as
// conv_gemm_pp_kernel): group g owns pixel rows 96g..96g+95, wave wc of a group owns channels 96wc..96wc+95
// (6 x 6 blocks of 16 x 16, 144 accumulator registers), BK = 64, two LDS stage buffers filled by LDS-DMA.
// A K-stage runs as 3 phases (one 32-pixel third of the group's rows each), each an L part (fragment reads
// + DMA issues for the next stage) and a C part (24 MFMAs: twice the MFMAs per DMA instruction and per
// barrier of the 256 x 192 tile).  DMA per wave and stage: P1 A third 0 + B rows 0..23 of the wave (4
// instructions), P2 B rows 24..47 (3), P3 A thirds 1, 2 (2).  Waits: end of L3 vmcnt(2) (A third 0 and all
// of B for the next stage: B is read by both groups, so every wave's B DMAs land before the barrier that
// opens the other group's next L1), end of C1 vmcnt(5) (A third 1 of this stage), end of C2 vmcnt(7)
// (A third 2).  Every region is rewritten >= 3 segments after its last fragment read.
// Epilogue: bias + ReLU, the 192 x 384 hidden tile staged in LDS (rows of 784 B), coalesced 16-B NHWC
// stores of the hidden activation, then the 1x1 tails: one thread per (pixel, head) with the head
// wave-uniform, so its 1x1 weights come through the scalar cache; outputs NCHW fp32.
__global__ __launch_bounds__(512, 1) void conv_gemm_heads384_kernel(GemmParams p) {
    typedef h16 T;
    constexpr int BM = 192, BN = 384, BK = 64, EPC = 8;
    constexpr int NA = 6, NB = 6;                     // 16-row / 16-column blocks per wave
    constexpr int STAGE = (BM + BN) * 128;
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2, wc = wave & 3;
    int bid;
    {
        const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7, xcd = blockIdx.x & 7;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (blockIdx.x >> 3);
    }
    const scd_gemm_phase& ph = p.ph[0];
    const int QQ = ph.Qh * ph.Qw;
    const int M = p.N * QQ;

    const int ntiles = (M + BM - 1) / BM;
    const int lrow = lane >> 3;
    const int cch = (lane & 7) ^ lrow;
    // A: this lane's DMA rows 96*grp + 32*j + 8*wc + lrow (j = third), byte offset at tap (0,0) + in-image tap mask
    int a_base[3];
    unsigned a_mask[3];
    auto tile_setup = [&](int mt) {
    #pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int m = mt * BM + 96 * grp + 32 * j + 8 * wc + lrow;
            const bool ok = m < M;
            const int mm = ok ? m : 0;
            const int n = mm / QQ;
            const int rem = mm - n * QQ;
            const int qh = rem / ph.Qw;
            const int qw = rem - qh * ph.Qw;
            a_base[j] = ((n * p.Hi + qh) * p.Wi + qw) * p.Ci * 2 + cch * EPC * 2;
            unsigned msk = 0;
            for (int t = 0; t < ph.ntaps; ++t) {
                const int ih = qh + ph.dh[t], iw = qw + ph.dw[t];
                if (ok && (unsigned)ih < (unsigned)p.Hi && (unsigned)iw < (unsigned)p.Wi) msk |= 1u << t;
            }
            a_mask[j] = msk;
        }
    };
    // B: rows 192*grp + 48*wc + 8*o + lrow, o = 0..5 (part 1: o < 3, part 2: o >= 3)
    int b_base[6];
    #pragma unroll
    for (int o = 0; o < 6; ++o) b_base[o] = ((192 * grp + 48 * wc + 8 * o + lrow) * p.wrow + cch * EPC) * 2;
    const int cpt = p.Ci / BK;
    const int KT = ph.ntaps * cpt;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.xbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, p.wbytes, 0x00020000);

    // Serpentine K order: every workgroup reads the whole 1.77-MB weight operand in K order, and by the time an XCD's
    // next round of tiles starts, its 4-MB L2 has streamed that round's input rows too, so the first K-stages'
    // weights are gone again (the ~150 MB of re-fetch in the PMC traffic).  Tiles of odd rounds (256 workgroups per
    // round, 32 per XCD) walk K backwards, starting on the stages the previous round used last.  The fp32 summation
    // order of those tiles changes; it is fixed per tile index, so every run gives the same bits.
    const bool krev = p.kserp && ((blockIdx.x >> 8) & 1);
    struct StageArgs { int live, tap, adelta, bdelta; };
    auto stage_args = [&](int kt_req) {
        StageArgs a;
        a.live = kt_req < KT;
        int kt = min(kt_req, KT - 1);
        kt = krev ? KT - 1 - kt : kt;
        const int chunk = kt / ph.ntaps, tap = kt - chunk * ph.ntaps;   // channel chunk outer, taps inner
        a.tap = tap;
        a.adelta = ((ph.dh[tap] * p.Wi + ph.dw[tap]) * p.Ci + chunk * BK) * 2;
        a.bdelta = (ph.wt[tap] * p.Ci + chunk * BK) * 2;
        return a;
    };
    auto issue_a = [&](const StageArgs& g, char* buf, int j) {
        const bool ok = g.live && ((a_mask[j] >> g.tap) & 1u);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(buf + (96 * grp + 32 * j + 8 * wc) * 128), 16,
                                                 sel_off(ok, a_base[j] + g.adelta), 0, 0, 0);
    };
    auto issue_b = [&](const StageArgs& g, char* buf, int part) {
        char* Bs = buf + BM * 128;
    #pragma unroll
        for (int o = 3 * part; o < 3 * part + 3; ++o)
            dma16(wrs, Bs + (192 * grp + 48 * wc + 8 * o) * 128, sel_off(g.live, b_base[o] + g.bdelta));
    };
    // the first K-stage of a tile into stage buffer 0
    auto issue_stage0 = [&]() {
        const StageArgs g0 = stage_args(0);
        issue_a(g0, smem, 0);
        issue_b(g0, smem, 0);
        issue_b(g0, smem, 1);
        issue_a(g0, smem, 1);
        issue_a(g0, smem, 2);
    };
    {
        const int mt = bid;
        (void)ntiles;
        tile_setup(mt);
        if (KT > 0) issue_stage0();
        const int l16 = lane & 15, lg = lane >> 4;
        const int l7 = l16 & 7;
        const int co0 = ((0 * 4 + lg) ^ l7) << 4, co1 = ((1 * 4 + lg) ^ l7) << 4;
        f32x4 acc[NA][NB];
    #pragma unroll
        for (int a = 0; a < NA; ++a)
    #pragma unroll
            for (int b = 0; b < NB; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
        h16x8 bfr[NB][2], af[2][2];

        auto read_b = [&](const char* buf) {
            const char* Bs = buf + BM * 128;
    #pragma unroll
            for (int b = 0; b < NB; ++b) {
                const char* row = Bs + (96 * wc + 16 * b + l16) * 128;
                bfr[b][0] = *(const h16x8*)(row + co0);
                bfr[b][1] = *(const h16x8*)(row + co1);
            }
        };
        auto read_a = [&](const char* buf, int q) {
    #pragma unroll
            for (int a = 0; a < 2; ++a) {
                const char* row = buf + (96 * grp + 32 * q + 16 * a + l16) * 128;
                af[a][0] = *(const h16x8*)(row + co0);
                af[a][1] = *(const h16x8*)(row + co1);
            }
        };
        auto mfma_q = [&](int q) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (PP_PRIO == 1) __builtin_amdgcn_s_setprio(1);
    #pragma unroll
            for (int s = 0; s < 2; ++s)
    #pragma unroll
                for (int a = 0; a < 2; ++a)
    #pragma unroll
                    for (int b = 0; b < NB; ++b)
                        acc[2 * q + a][b] = mfma_16x16x32_h16(bfr[b][s], af[a][s], acc[2 * q + a][b]);
            if constexpr (PP_PRIO == 1) __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_sched_barrier(0);
        };
        auto bar = [&]() {
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
        };

        SCD_STAMP_BEGIN();
        if (KT > 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            bar();
            if (grp == 1) bar();                 // stagger: group 1 runs one barrier behind
            if constexpr (PP_PRIO == 2) { if (grp == 1) __builtin_amdgcn_s_setprio(1); }
            for (int t = 0; t < KT; ++t) {
                char* cur = smem + (t & 1) * STAGE;
                char* nxt = smem + ((t & 1) ^ 1) * STAGE;
                const StageArgs g = stage_args(t + 1);
                // P1
                read_b(cur);
                read_a(cur, 0);
                issue_a(g, nxt, 0);
                issue_b(g, nxt, 0);
                bar();
                mfma_q(0);
                asm volatile("s_waitcnt vmcnt(5)" ::: "memory");     // A third 1 (P3 of t-1)
                bar();
                // P2
                read_a(cur, 1);
                issue_b(g, nxt, 1);
                bar();
                mfma_q(1);
                asm volatile("s_waitcnt vmcnt(7)" ::: "memory");     // A third 2 of this stage
                bar();
                // P3
                read_a(cur, 2);
                issue_a(g, nxt, 1);
                issue_a(g, nxt, 2);
                asm volatile("s_waitcnt vmcnt(2)" ::: "memory");     // next stage: A third 0 and every B row
                bar();
                mfma_q(2);
                bar();
            }
            if (grp == 0) bar();
            if constexpr (PP_PRIO == 2) __builtin_amdgcn_s_setprio(0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        SCD_STAMP_END();
        // ---- epilogue from the accumulators.  Lane (l16, lg) of block (a, b) holds hidden channels
        // 96wc + 16b + 4lg .. +3 of pixel 96grp + 16a + l16: after bias + ReLU those 4 bf16 are (1) an 8-B piece of
        // the pixel's NHWC row, stored at once, and (2) exactly the B operand of a 16x16x16 MFMA (B[k = 4lg + j][n =
        // l16]), so the 1x1 tails out[o][px] = sum_c W1[o][c] hid[c][px] run on the same registers: A = the
        // block-diagonal W1 slice of the wave's 16 channels (A[m = l16][k = 4lg + j], fp32 weights as bf16 hi + lo,
        // ~2^-17), 12 MFMAs per 16-pixel block.  The four channel waves of a group meet in LDS (48 KiB of fp32
        // partials), then one pass adds them, the bias, and writes the NCHW fp32 outputs.
        {
            typedef __attribute__((ext_vector_type(4))) h16 bf16x4;
            const int od0 = p.head_od[0], od1 = p.head_od[1], od2 = p.head_od[2];
            const int odsum = od0 + od1 + od2;
            const int o = l16;                                       // tail output row of this lane's W1 fragment
            const int hh = o < od0 ? 0 : o < od0 + od1 ? 1 : o < odsum ? 2 : -1;
            const int oo = hh == 0 ? o : hh == 1 ? o - od0 : o - od0 - od1;
            const float* wsel = hh == 0 ? p.head_w[0] : hh == 1 ? p.head_w[1] : p.head_w[2];
            f32x4 tl[NA];
    #pragma unroll
            for (int a = 0; a < NA; ++a) tl[a] = (f32x4){0.f, 0.f, 0.f, 0.f};
            // blocks in pairs (b, b+1): after the tails, v_permlane16_swap trades the odd rows' block-b halves for
            // the even rows' block-(b+1) halves, so every lane holds 8 consecutive channels (16-B stores: even rows
            // channels 16b + 4lg .., odd rows 16(b+1) + 4(lg-1) ..; 64 contiguous bytes per pixel and instruction)
            // hidden channels >= hid_cols are stored only at the pixels the keep map names (the size / offset heads'
            // sparse backward reads them there only; HeadsFn recomputes the whole tensor for any other backward)
            unsigned keep = (1u << NA) - 1;
            if (p.hid_keep) {                                        // the NA loads together, one wait
                unsigned char kv[NA];
    #pragma unroll
                for (int a = 0; a < NA; ++a) {
                    const int m = mt * BM + 96 * grp + 16 * a + l16;
                    kv[a] = p.hid_keep[m < M ? m : 0];
                }
                keep = 0;
    #pragma unroll
                for (int a = 0; a < NA; ++a)
                    if (mt * BM + 96 * grp + 16 * a + l16 < M && kv[a]) keep |= 1u << a;
            }
            // the bias and W1 slices of all NB blocks loaded up front, unconditionally (from a valid address, the
            // value selected after): a load inside the block loop, or under a branch, makes the compiler wait for
            // every access before it -- the previous blocks' hidden-row stores included
            hx4 whi[NB], wlo[NB];
            float bias[NB][4];
    #pragma unroll
            for (int b = 0; b < NB; ++b) {
                const int col0 = 96 * wc + 16 * b + 4 * lg;
                const float4 bb = *(const float4*)(p.bias + col0);
                bias[b][0] = bb.x; bias[b][1] = bb.y; bias[b][2] = bb.z; bias[b][3] = bb.w;
                // W1[o][col0 .. col0 + 3] when those channels belong to output o's head, else 0
                const bool wok = hh >= 0 && (col0 >> 7) == hh;
                const float4 wl = *(const float4*)((hh >= 0 ? wsel : p.head_w[0]) + (wok ? oo * 128 + (col0 & 127) : 0));
                const float4 wv = wok ? wl : make_float4(0.f, 0.f, 0.f, 0.f);
                const float w4[4] = {wv.x, wv.y, wv.z, wv.w};
    #pragma unroll
                for (int j = 0; j < 4; ++j) {
                    whi[b][j] = (h16)w4[j];
                    wlo[b][j] = (h16)(w4[j] - (float)whi[b][j]);
                }
            }
            // consumed here, before the first store (else the compiler's wait for the last ones lands after stores)
    #pragma unroll
            for (int b = 0; b < NB; ++b)
                asm volatile("" : "+v"(whi[b]), "+v"(wlo[b]), "+v"(bias[b][0]), "+v"(bias[b][1]), "+v"(bias[b][2]),
                             "+v"(bias[b][3]));
    #pragma unroll
            for (int b = 0; b < NB; b += 2) {
                const int colst = 96 * wc + 16 * b + ((lg & 1) ? 16 + 4 * (lg - 1) : 4 * lg);
    #pragma unroll
                for (int a = 0; a < NA; ++a) {
                    hx4 hv[2];
    #pragma unroll
                    for (int e = 0; e < 2; ++e)
    #pragma unroll
                        for (int r = 0; r < 4; ++r) hv[e][r] = (h16)fmaxf(acc[a][b + e][r] + bias[b + e][r], 0.f);
    #pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        tl[a] = mfma_16x16x16(whi[b + e], hv[e], tl[a]);
                        tl[a] = mfma_16x16x16(wlo[b + e], hv[e], tl[a]);
                    }
                    typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
                    const u32x2 x = __builtin_bit_cast(u32x2, hv[0]), y = __builtin_bit_cast(u32x2, hv[1]);
                    uint4 st;
                    {
                        const auto s0 = __builtin_amdgcn_permlane16_swap(x[0], y[0], false, false);
                        const auto s1 = __builtin_amdgcn_permlane16_swap(x[1], y[1], false, false);
                        st.x = s0[0]; st.y = s1[0]; st.z = s0[1]; st.w = s1[1];
                    }
                    const int m = mt * BM + 96 * grp + 16 * a + l16;
                    if (m < M && (colst < p.hid_cols || ((keep >> a) & 1u)))
                        *(uint4*)(p.y + ((long)m * BN + colst) * 2) = st;
                }
            }
            {
                // partials [wc][o][pixel of tile]: D[o = 4lg + r][px = l16] of block a
                float* part = (float*)smem;
    #pragma unroll
                for (int a = 0; a < NA; ++a)
    #pragma unroll
                    for (int r = 0; r < 4; ++r)
                        part[(wc * 16 + 4 * lg + r) * BM + 96 * grp + 16 * a + l16] = tl[a][r];
                __syncthreads();
                for (int idx = tid; idx < odsum * BM; idx += 512) {
                    const int oi = idx / BM, r = idx - oi * BM;
                    const int m = mt * BM + r;
                    if (m >= M) continue;
                    const float v = (part[(0 * 16 + oi) * BM + r] + part[(1 * 16 + oi) * BM + r]) +
                                    (part[(2 * 16 + oi) * BM + r] + part[(3 * 16 + oi) * BM + r]);
                    const int h = oi < od0 ? 0 : oi < od0 + od1 ? 1 : 2;
                    const int ob = oi - (h == 0 ? 0 : h == 1 ? od0 : od0 + od1);
                    const int odh = h == 0 ? od0 : h == 1 ? od1 : od2;
                    float* out = h == 0 ? p.head_out[0] : h == 1 ? p.head_out[1] : p.head_out[2];
                    const float bo = (h == 0 ? p.head_b[0] : h == 1 ? p.head_b[1] : p.head_b[2])[ob];
                    const int n = m / QQ, pix = m - (m / QQ) * QQ;
                    out[((long)n * odh + ob) * QQ + pix] = v + bo;
                }
            }
        }
        __syncthreads();                 // staging consumed before the next tile's prologue DMA
    }
}

// -------------------------------------------------------------------------------------
// weight gradient: ws[z][co][t*Ci+ci] = sum_pix g[pix][co] * x[gather(pix,t)][ci]
struct WgradParams {
    const char* g;
    const char* x;
    float* ws;
    int N, Ho, Wo, Cg, Hi, Wi, Ci, is, T, KK, chunk, ntm, ntn, nsplit;
    int cg0, cgn;       // output-gradient channel window of this launch: [cg0, cg0 + cgn) of Cg
    int gbytes, xbytes;
    int dh[SCD_MAX_TAPS], dw[SCD_MAX_TAPS];
};

// 1-D grid.  nsplit % 8 == 0: ntiles * nsplit blocks, block b -> XCD b % 8, split z = 8 * ((b / 8) / ntiles) + b % 8,
// tile (b / 8) % ntiles (every tile of split z on one XCD: the tiles re-reading the split's pixel rows share its L2).
// Otherwise (few splits of many tiles, whose operands sit in L2 / MALL anyway: layer4, deconv1): ntiles * nsplit
// blocks, tile b % ntiles, split b / ntiles, so one round of workgroups fills every XCD.  Returns false for padding.
__device__ __forceinline__ bool wgrad_block(const WgradParams& p, int& z, int& mt, int& nt) {
    const int T = p.ntm * p.ntn;
    int tile;
    if (p.nsplit & 7) {
        z = blockIdx.x / T;
        tile = blockIdx.x - z * T;
        mt = tile / p.ntn;
        nt = tile - mt * p.ntn;
        return z < p.nsplit;
    }
    const int j = blockIdx.x >> 3;
    z = 8 * (j / T) + (blockIdx.x & 7);
    tile = j - (j / T) * T;
    mt = tile / p.ntn;
    nt = tile - mt * p.ntn;
    return z < p.nsplit;
}

// LDS image of a [pixel][channel] stage for transposed (ds_read_b64_tr_b16) fragment reads: a row
// stride of 8 dwords mod 64 banks (288 B for <= 256-B rows, 544 B for 512-B rows) puts rows r..r+3 on
// disjoint 8-bank slots, and the column offset of rows with bit 3 set is XORed with 128 B, so rows
// {0-3, 8-11} read by one 32-lane half cover all 64 banks: the transposed reads are conflict free.
__host__ __device__ constexpr int wrow_stride(int rowbytes) { return rowbytes <= 256 ? 288 : rowbytes + 32; }
__device__ __forceinline__ int wswz(int row, int byte, int stride) {
    return row * stride + (byte ^ (((row >> 3) & 1) << 7));
}

// FASTX: a KP-pixel stage never straddles an image and covers either part of one output row (Wo % KP == 0)
// or whole rows (KP % Wo == 0).  The stage position (n, oh, ow) is then workgroup-uniform (scalar registers)
// and every X slot's gather offset is that stage base plus a per-lane constant: a few VALU per load instead
// of the per-row decomposition (the generic path is VALU-issue-bound: ~250 address instructions per stage
// against 32 MFMAs per wave).
template <typename T, int BM, int BN, int FASTX>
__global__ __launch_bounds__(256, WGRAD_OCC) void conv_wgrad_kernel(WgradParams p) {
    constexpr int ESZ = sizeof(T);
    constexpr int EPC = 16 / ESZ;
    constexpr int KP = ESZ == 2 ? 64 : 32;               // pixels per stage (2 bf16 MFMA k-steps)
    constexpr int GROWB = BM * ESZ;                      // bytes of one G row
    constexpr int XROWB = BN * ESZ;
    constexpr int GROW = ESZ == 2 ? wrow_stride(GROWB) : GROWB + 16;   // LDS row stride
    constexpr int XROW = ESZ == 2 ? wrow_stride(XROWB) : XROWB + 16;
    constexpr int GCPR = GROWB / 16;                     // chunks per G row
    constexpr int XCPR = XROWB / 16;
    constexpr int GCH = KP * GCPR / 256;                 // chunks per thread
    constexpr int XCH = KP * XCPR / 256;
    constexpr int GRS = 256 / GCPR;                      // rows per load pass
    constexpr int XRS = 256 / XCPR;
    constexpr int WN = BN / 64;
    constexpr int STAGE = KP * (GROW + XROW);
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

    const int tid = threadIdx.x;
    // XCD-aware split placement: every tile of split z runs on XCD z % 8 (blocks are dispatched to XCDs
    // round-robin on blockIdx), so the tiles re-reading the split's pixel rows share one L2
    int z, mt, nt;
    if (!wgrad_block(p, z, mt, nt)) return;
    const int M = p.N * p.Ho * p.Wo;
    const int pix0 = z * p.chunk;
    const int pix1 = min(M, pix0 + p.chunk);

    // G loads: fixed channel chunk per thread
    const int gc = tid % GCPR;
    const int gr0 = tid / GCPR;
    const int gcol = p.cg0 + mt * BM + gc * EPC;
    const bool gcol_ok = gcol < p.cg0 + p.cgn;
    // X loads: fixed (tap, ci) chunk per thread; pixel position advanced incrementally
    const int xc = tid % XCPR;
    const int xr0 = tid / XCPR;
    const int kk = nt * BN + xc * EPC;
    const bool kk_ok = kk < p.KK;
    const int tap = kk_ok ? kk / p.Ci : 0;
    const int ci = kk - tap * p.Ci;
    const int dh = p.dh[tap], dw = p.dw[tap];
    int xn[XCH], xoh[XCH], xow[XCH];
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
        xn[i] = xoh[i] = xow[i] = 0;
        if constexpr (FASTX != 0) continue;
        const int pix = pix0 + xr0 + i * XRS;
        const int HoWo = p.Ho * p.Wo;
        xn[i] = pix / HoWo;
        const int rem = pix - xn[i] * HoWo;
        xoh[i] = rem / p.Wo;
        xow[i] = rem - xoh[i] * p.Wo;
    }
    // FASTX: stage cursor (uniform) and per-slot constants
    int sn = 0, soh = 0, sow = 0;
    // FASTX 1 (Wo % KP == 0): a stage is part of one output row, slot i sits XRS*i pixels right of slot 0, so one
    // base value per quantity suffices (3 VGPRs); FASTX 2 (KP % Wo == 0): whole rows, per-slot constants
    constexpr int NXS = FASTX == 2 ? XCH : 1;
    int xA[NXS], xB[NXS], xL[NXS];
    if constexpr (FASTX != 0) {
        const int HoWo = p.Ho * p.Wo;
        sn = __builtin_amdgcn_readfirstlane(pix0 / HoWo);
        const int rem = pix0 - sn * HoWo;
        soh = __builtin_amdgcn_readfirstlane(rem / p.Wo);
        sow = __builtin_amdgcn_readfirstlane(rem - soh * p.Wo);
#pragma unroll
        for (int i = 0; i < NXS; ++i) {
            const int rr = xr0 + i * XRS;
            const int doh = FASTX == 1 ? 0 : rr / p.Wo, dow = FASTX == 1 ? rr : rr - (rr / p.Wo) * p.Wo;
            xA[i] = p.is * doh + dh;
            xB[i] = p.is * dow + dw;
            xL[i] = (xA[i] * p.Wi + xB[i]) * p.Ci + ci;
        }
    }
    auto advance = [&]() {     // every row advances by KP pixels
        if constexpr (FASTX != 0) {
            if (FASTX == 1) {
                sow += KP;
                const bool wrap = sow >= p.Wo;
                sow = wrap ? 0 : sow;
                soh += wrap ? 1 : 0;
            } else {
                soh += KP / p.Wo;
            }
            const bool wrap2 = soh >= p.Ho;
            soh = wrap2 ? 0 : soh;
            sn += wrap2 ? 1 : 0;
            // workgroup-uniform: keep the cursor in scalar registers
            sn = __builtin_amdgcn_readfirstlane(sn);
            soh = __builtin_amdgcn_readfirstlane(soh);
            sow = __builtin_amdgcn_readfirstlane(sow);
        } else {
#pragma unroll
            for (int i = 0; i < XCH; ++i) {
                xow[i] += KP;
                while (xow[i] >= p.Wo) {
                    xow[i] -= p.Wo;
                    if (++xoh[i] >= p.Ho) { xoh[i] = 0; ++xn[i]; }
                }
            }
        }
    };

    const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc((void*)p.g, (short)0, p.gbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.xbytes, 0x00020000);
    auto gload = [&](int k0, uint4 (&rg)[GCH], uint4 (&rx)[XCH]) {
        if constexpr (FASTX != 0) {
            const int S = __builtin_amdgcn_readfirstlane(((sn * p.Hi + p.is * soh) * p.Wi + p.is * sow) * p.Ci);
            const int ihs = __builtin_amdgcn_readfirstlane(p.is * soh), iws = __builtin_amdgcn_readfirstlane(p.is * sow);
            const int kr = pix1 - k0;        // rows of this stage inside the split
            const int gS = __builtin_amdgcn_readfirstlane(k0 * p.Cg);
#pragma unroll
            for (int i = 0; i < GCH; ++i) {
                const int r = gr0 + i * GRS;
                rg[i] = bload(grs, sel_off(gcol_ok & (r < kr), (gS + r * p.Cg + gcol) * ESZ));
            }
#pragma unroll
            for (int i = 0; i < XCH; ++i) {
                const int j = FASTX == 2 ? i : 0;
                const int xb = xB[j] + (FASTX == 1 ? p.is * XRS * i : 0);
                const int xl = xL[j] + (FASTX == 1 ? p.is * XRS * i * p.Ci : 0);
                // non-short-circuit &: straight-line selects, no exec-masked branches around the loads
                const bool ok = kk_ok & (xr0 + i * XRS < kr) & ((unsigned)(ihs + xA[j]) < (unsigned)p.Hi) &
                                ((unsigned)(iws + xb) < (unsigned)p.Wi);
                rx[i] = bload(xrs, sel_off(ok, (S + xl) * ESZ));
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < GCH; ++i) {
            const int pix = k0 + gr0 + i * GRS;
            rg[i] = bload(grs, sel_off(SCD_ABLATE != 22 && gcol_ok && pix < pix1, (pix * p.Cg + gcol) * ESZ));
        }
#pragma unroll
        for (int i = 0; i < XCH; ++i) {
            const int pix = k0 + xr0 + i * XRS;
            const int ih = p.is * xoh[i] + dh, iw = p.is * xow[i] + dw;
            const bool ok = SCD_ABLATE != 22 && kk_ok && pix < pix1 && (unsigned)ih < (unsigned)p.Hi && (unsigned)iw < (unsigned)p.Wi;
            rx[i] = bload(xrs, sel_off(ok, (((xn[i] * p.Hi + ih) * p.Wi + iw) * p.Ci + ci) * ESZ));
        }
    };
    auto lstore = [&](int buf, const uint4 (&rg)[GCH], const uint4 (&rx)[XCH]) {
        char* Gs = smem + buf * STAGE;
        char* Xs = Gs + KP * GROW;
#pragma unroll
        for (int i = 0; i < GCH; ++i) {
            const int row = gr0 + i * GRS;
            char* d = ESZ == 2 ? Gs + wswz(row, gc * 16, GROW) : Gs + row * GROW + gc * 16;
            *(uint4*)d = rg[i];
        }
#pragma unroll
        for (int i = 0; i < XCH; ++i) {
            const int row = xr0 + i * XRS;
            char* d = ESZ == 2 ? Xs + wswz(row, xc * 16, XROW) : Xs + row * XROW + xc * 16;
            *(uint4*)d = rx[i];
        }
    };

    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / WN, wn = wave - (wave / WN) * WN;
    const int l16 = lane & 15, lg = lane >> 4;

    f32x4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};

    auto compute = [&](int buf) {
        if constexpr (SCD_ABLATE == 23) return;      // ablation: no fragment reads, no MFMA
        const char* Gs = smem + buf * STAGE;
        const char* Xs = Gs + KP * GROW;
        if constexpr (ESZ == 2) {
            // ds_read_b64_tr_b16: lane 4q+p of 16-lane group lg supplies row (8lg+q[+4]) of the k-step,
            // columns c0+4p..4p+3; lane i of the group receives column c0+i of those 4 rows.
            const int q = l16 >> 2, pp = l16 & 3;
            typedef __attribute__((ext_vector_type(8))) short s16x8;
#pragma unroll
            for (int s = 0; s < KP / 32; ++s) {
                const int r0 = 32 * s + 8 * lg + q;
                h16x8 af[4], bfr[4];
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    const int cb = (wm * 64 + a * 16 + 4 * pp) * 2;
                    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Gs + wswz(r0, cb, GROW)));
                    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Gs + wswz(r0 + 4, cb, GROW)));
                    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                    af[a] = __builtin_bit_cast(h16x8, v);
                }
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const int cb = (wn * 64 + b * 16 + 4 * pp) * 2;
                    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Xs + wswz(r0, cb, XROW)));
                    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Xs + wswz(r0 + 4, cb, XROW)));
                    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                    bfr[b] = __builtin_bit_cast(h16x8, v);
                }
                if constexpr (SCD_ABLATE == 21) {
#pragma unroll
                    for (int a = 0; a < 4; ++a) { asm volatile("" ::"v"(af[a])); asm volatile("" ::"v"(bfr[a])); }
                } else {
#pragma unroll
                for (int a = 0; a < 4; ++a)
#pragma unroll
                    for (int b = 0; b < 4; ++b)
                        acc[a][b] = mfma_16x16x32_h16(af[a], bfr[b], acc[a][b]);
                }
                // FASTX frees the address registers the hoisted fragment reads of the next k-step would take:
                // keep one k-step of fragments live at a time (256-VGPR budget at two workgroups per CU)
                if constexpr (FASTX == 2) __builtin_amdgcn_sched_barrier(0);
            }
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int krow = 4 * j + lg;
                float av[4], bv[4];
#pragma unroll
                for (int a = 0; a < 4; ++a) av[a] = *(const float*)(Gs + krow * GROW + (wm * 64 + a * 16 + l16) * 4);
#pragma unroll
                for (int b = 0; b < 4; ++b) bv[b] = *(const float*)(Xs + krow * XROW + (wn * 64 + b * 16 + l16) * 4);
#pragma unroll
                for (int a = 0; a < 4; ++a)
#pragma unroll
                    for (int b = 0; b < 4; ++b)
                        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[a], bv[b], acc[a][b], 0, 0, 0);
            }
        }
    };

    const int nk = (pix1 > pix0) ? (pix1 - pix0 + KP - 1) / KP : 0;
    if (nk > 0) {
        // two stages of loads in flight (see conv_gemm_kernel); stages past the end read nothing
        uint4 rg0[GCH], rx0[XCH], rg1[GCH], rx1[XCH];
        gload(pix0, rg0, rx0);
        advance();
        gload(pix0 + KP, rg1, rx1);
        lstore(0, rg0, rx0);
        __syncthreads();
        for (int it = 0; it < nk; it += 2) {
            advance();
            gload(pix0 + (it + 2) * KP, rg0, rx0);
            compute(0);
            lstore(1, rg1, rx1);
            __syncthreads();
            if (it + 1 >= nk) break;
            advance();
            gload(pix0 + (it + 3) * KP, rg1, rx1);
            compute(1);
            lstore(0, rg0, rx0);
            __syncthreads();
        }
    }
    // ---- store fp32 partial tile: rows = Cg channel, cols = kk
    float* ws = p.ws + (long)z * p.Cg * p.KK;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = p.cg0 + mt * BM + wm * 64 + a * 16 + lg * 4 + r;
            if (row >= p.cg0 + p.cgn) continue;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int col = nt * BN + wn * 64 + b * 16 + l16;
                if (col < p.KK) ws[(long)row * p.KK + col] = acc[a][b][r];
            }
        }
}

// 32-B column-pair swizzle of the transposed-read stage images (conv_wgrad_pp2_kernel): f(r) over rows
// {r..r+3, r+8..r+11} takes 8 distinct values, so a 32-lane half's ds_read_b64_tr_b16 reads are conflict free
__device__ __forceinline__ int wr_f(int r) { return (r & 3) | ((r >> 1) & 4); }

// -------------------------------------------------------------------------------------
// Ping-pong bf16 weight gradient, 64-pixel stages (the conv_gemm_pp_kernel schedule applied to the
// weight gradient): tile 256 output-gradient channels (window cg0 + 256*mt) x 256 columns of taps x input
// channels, two LDS stage buffers of 64 KB, 8 waves in two staggered groups (group g: 128 channels = 8
// blocks, wave wc: 64 columns = 4 blocks), 4 phases per stage (phase q: channel blocks 2q, 2q+1 = 16
// MFMAs).  Each group's G operand is stored as four [64 px][64 B] quarter images (the 32 channels of
// one phase), so quarter q of stage t+1 is needed only at phase q of stage t+1 and is fetched at phase
// 3/4 of stage t, like the A rows of the forward kernel; X ([64 px][512 B], read whole in phase 1) is
// fetched in phases 1/2.  Counted waits as conv_gemm_pp_kernel (NB2 = 2).  Requires Wo % 64 == 0 and
// (Ho*Wo) % 64 == 0: a stage is part of one output row, addressed by a scalar cursor (see FASTX 1).
// NQ 2 (48-KB stages, half the MFMAs per stage of NQ 4): three stage buffers, two stages of DMA in flight -- a stage
// is ~1000 MFMA cycles, shorter than the operand fetch latency under load (SCD_PP2_NBUF=2: two buffers).
#ifndef SCD_PP2_NBUF
#define SCD_PP2_NBUF 3
#endif
template <int NQ>
__global__ __launch_bounds__(512, 1) void conv_wgrad_pp2_kernel(WgradParams p) {
    constexpr int KP = 64, EPC = 8;
    constexpr int QIMG = KP * 64;                     // one G quarter image: 64 px x 64 B
    constexpr int GBYTES = 2 * NQ * QIMG;             // 2 groups x NQ quarters
    constexpr int WIN = 64 * NQ;                      // channels per window (256, 192 or 128)
    static_assert(NQ >= 2 && NQ <= 4, "NQ");
    constexpr int STAGE = GBYTES + KP * 512;          // + X image
    constexpr int NBUF = NQ == 2 ? SCD_PP2_NBUF : 2;
    static_assert(NBUF == 2 || NBUF == 3, "NBUF");
    __shared__ __attribute__((aligned(16))) char smem[NBUF * STAGE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2, wc = wave & 3;
    int z, mt, nt;
    if (!wgrad_block(p, z, mt, nt)) return;
    const int M = p.N * p.Ho * p.Wo;
    const int pix0 = z * p.chunk;
    const int pix1 = min(M, pix0 + p.chunk);
    const int cbase = p.cg0 + mt * WIN + grp * 32 * NQ;   // this group's first channel

    // G DMA: quarter q, rows 16*wc + lane/4; the lane's 16-B slot (lane & 3) holds logical chunk c
    const int g_r = 16 * wc + (lane >> 2);
    int g_off;
    {
        const int slot = lane & 3;
        const int c = 2 * ((slot >> 1) ^ ((g_r >> 3) & 1)) + (slot & 1);
        g_off = cbase + c * EPC;
    }
    // X DMA: instruction k = 4*wave + j covers rows 2k, 2k+1; per slot constants.  A stage is 64 pixels of one
    // output row (Wo % 64 == 0) or 64 / Wo whole rows (64 % Wo == 0): pixel r of a stage sits at row r / Wo, column
    // r % Wo from the stage cursor either way (r < Wo in the first case)
    int x_r[4], xA[4], xB[4], xL[4];
    bool x_ok[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int r = 2 * (4 * wave + j) + (lane >> 5);
        const int slot = lane & 31;
        const int c = 2 * ((slot >> 1) ^ wr_f(r)) + (slot & 1);
        const int kk = nt * 256 + c * EPC;
        x_ok[j] = kk < p.KK;
        const int tap = x_ok[j] ? kk / p.Ci : 0;
        const int ci = kk - tap * p.Ci;
        const int doh = r / p.Wo, dow = r - doh * p.Wo;
        x_r[j] = r;
        xA[j] = p.is * doh + p.dh[tap];
        xB[j] = p.is * dow + p.dw[tap];
        xL[j] = (xA[j] * p.Wi + xB[j]) * p.Ci + ci;
    }
    const int rows_per_wrap = p.Wo >= KP ? 1 : KP / p.Wo;    // output rows a stage advances when it wraps
    int sn, soh, sow;
    {
        const int HoWo = p.Ho * p.Wo;
        sn = __builtin_amdgcn_readfirstlane(pix0 / HoWo);
        const int rem = pix0 - sn * HoWo;
        soh = __builtin_amdgcn_readfirstlane(rem / p.Wo);
        sow = __builtin_amdgcn_readfirstlane(rem - soh * p.Wo);
    }
    auto advance = [&]() {
        sow += KP;
        const bool wrap = sow >= p.Wo;
        sow = wrap ? 0 : sow;
        soh += wrap ? rows_per_wrap : 0;
        const bool wrap2 = soh >= p.Ho;
        soh = wrap2 ? 0 : soh;
        sn += wrap2 ? 1 : 0;
        sn = __builtin_amdgcn_readfirstlane(sn);
        soh = __builtin_amdgcn_readfirstlane(soh);
        sow = __builtin_amdgcn_readfirstlane(sow);
    };
    const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc((void*)p.g, (short)0, p.gbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.xbytes, 0x00020000);
    // stage whose first pixel is k0 (cursor = its position)
    auto issue_x = [&](int k0, char* stg, int half) {
        const int S = __builtin_amdgcn_readfirstlane(((sn * p.Hi + p.is * soh) * p.Wi + p.is * sow) * p.Ci);
        const int ihs = __builtin_amdgcn_readfirstlane(p.is * soh), iws = __builtin_amdgcn_readfirstlane(p.is * sow);
        const int kr = pix1 - k0;
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
            const int j = 2 * half + jj;
            const bool ok = x_ok[j] & (x_r[j] < kr) & ((unsigned)(ihs + xA[j]) < (unsigned)p.Hi) &
                            ((unsigned)(iws + xB[j]) < (unsigned)p.Wi);
            dma16_asm(xrs, stg + GBYTES + 2 * (4 * wave + j) * 512, sel_off(ok, (S + xL[j]) * 2));
        }
    };
    auto issue_g = [&](int k0, char* stg, int q) {
        const int kr = pix1 - k0;
        dma16_asm(grs, stg + (grp * NQ + q) * QIMG + 16 * wc * 64,
                  sel_off(g_r < kr, ((k0 + g_r) * p.Cg + g_off + q * 32) * 2));
    };

    const int l16 = lane & 15, lg = lane >> 4;
    const int q4 = l16 >> 2, pp = l16 & 3;
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    auto trf = [&](const char* lo_addr, const char* hi_addr) {
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)lo_addr);
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)hi_addr);
        s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(h16x8, v);
    };
    f32x4 acc[2 * NQ][4];
#pragma unroll
    for (int a = 0; a < 2 * NQ; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
    h16x8 xf[4][2], gfx[2][2], gfy[2][2];
    auto read_x = [&](const char* stg) {
        const char* X = stg + GBYTES;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int r0 = 32 * s + 8 * lg + q4;
            const int f0 = wr_f(r0), f1 = wr_f(r0 + 4);
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int cb = (wc * 64 + b * 16 + 4 * pp) * 2;
                const int pr = cb >> 5, lo8 = cb & 31;
                xf[b][s] = trf(X + r0 * 512 + ((pr ^ f0) << 5) + lo8, X + (r0 + 4) * 512 + ((pr ^ f1) << 5) + lo8);
            }
        }
    };
    auto read_g = [&](const char* stg, int q, h16x8 (&gf)[2][2]) {
        const char* G = stg + (grp * NQ + q) * QIMG;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int r0 = 32 * s + 8 * lg + q4;
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                const int plo = a ^ ((r0 >> 3) & 1), phi = a ^ (((r0 + 4) >> 3) & 1);
                gf[a][s] = trf(G + r0 * 64 + plo * 32 + 8 * pp, G + (r0 + 4) * 64 + phi * 32 + 8 * pp);
            }
        }
    };
    auto mfma_q = [&](int q, const h16x8 (&gf)[2][2]) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (PP_PRIO == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    acc[2 * q + a][b] = mfma_16x16x32_h16(xf[b][s], gf[a][s], acc[2 * q + a][b]);
        if constexpr (PP_PRIO == 1) __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto bar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };

    const int nk = (pix1 > pix0) ? (pix1 - pix0 + KP - 1) / KP : 0;
    if (nk > 0) {
        issue_x(pix0, smem, 0);
        issue_x(pix0, smem, 1);
#pragma unroll
        for (int q = 0; q < NQ; ++q) issue_g(pix0, smem, q);
        advance();
        if constexpr (NBUF == 3) {
            // stage 1 into the second buffer; wait for stage 0 only (6 DMAs a stage per wave)
            issue_x(pix0 + KP, smem + STAGE, 0);
            issue_x(pix0 + KP, smem + STAGE, 1);
            issue_g(pix0 + KP, smem + STAGE, 0);
            issue_g(pix0 + KP, smem + STAGE, 1);
            advance();
            asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        bar();
        if (grp == 1) bar();
        if constexpr (PP_PRIO == 2) { if (grp == 1) __builtin_amdgcn_s_setprio(1); }
        // schedule (stage t fetches stage t+1 into the other buffer): phase 1: X half 0, phase 2: X half 1,
        // phases 3(-4): the G quarters.  NQ 4: C2 vmcnt(4), L4 vmcnt(4), C4 vmcnt(2);
        // NQ 3: C1 vmcnt(3), C2 vmcnt(4), L3 vmcnt(3), C3 vmcnt(2);
        // NQ 2 (128-channel windows: the heatmap head, layer2): phase 1 issues all six DMAs of stage t+1 (X halves,
        // both G quarters), so they land across both phases; every wave's fragment reads are drained before the
        // phase-2 barrier (the partner group, one barrier ahead, then overwrites that buffer's G quarters).  Stage t+1
        // must be retired before the barrier after which group 0 reads it: group 0's post-MFMA barrier of phase 2,
        // which for group 1 (one barrier behind) is the barrier BEFORE its phase-2 MFMAs -- group 0 waits vmcnt(0)
        // after its MFMAs, group 1 before that barrier (waiting after it, as group 0 does, let group 0 read group 1's
        // half of the stage before it had landed: NaN weight gradients, layer2 downsample, cornerNetCPool B=32).
        // Three buffers: stage t issues stage t+2 into the buffer stage t-1 used (the same overwrite rule), and the
        // waits keep stage t+2's six DMAs in flight (vmcnt(6)) while retiring stage t+1's.
        int bcur = 0;
        for (int t = 0; t < nk; ++t) {
            char* cur = smem + bcur * STAGE;
            const int bnxt = NBUF == 3 ? (bcur == 0 ? 2 : bcur - 1) : (bcur ^ 1);
            char* nxt = smem + bnxt * STAGE;
            bcur = NBUF == 3 ? (bcur == 2 ? 0 : bcur + 1) : (bcur ^ 1);
            const int k1 = pix0 + (t + NBUF - 1) * KP;      // >= pix1 near the end: the DMAs read nothing
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                h16x8 (&gf)[2][2] = (q & 1) ? gfy : gfx;
                if (q == 0) read_x(cur);
                read_g(cur, q, gf);
                if constexpr (NQ == 2) {
                    if (q == 0) { issue_x(k1, nxt, 0); issue_x(k1, nxt, 1); issue_g(k1, nxt, 0); issue_g(k1, nxt, 1); }
                    if (q == 1) {
                        advance();
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        if (grp == 1) {
                            if constexpr (NBUF == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
                            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        }
                    }
                    bar();
                    mfma_q(q, gf);
                    if (q == 1 && grp == 0) {
                        if constexpr (NBUF == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
                        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    }
                    bar();
                    continue;
                }
                if (q < 2) issue_x(k1, nxt, q);
                if constexpr (NQ == 4) {
                    if (q == 2) { issue_g(k1, nxt, 0); issue_g(k1, nxt, 1); }
                    if (q == 3) { issue_g(k1, nxt, 2); issue_g(k1, nxt, 3); advance(); asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); }
                } else {
                    if (q == 2) { issue_g(k1, nxt, 0); issue_g(k1, nxt, 1); issue_g(k1, nxt, 2); advance(); asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); }
                }
                bar();
                mfma_q(q, gf);
                if constexpr (NQ == 4) {
                    if (q == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                    if (q == 3) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
                } else {
                    if (q == 0) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
                    if (q == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                    if (q == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
                }
                bar();
            }
        }
        if (grp == 0) bar();
        if constexpr (PP_PRIO == 2) __builtin_amdgcn_s_setprio(0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // fp32 slab: lane holds columns kk..kk+3 of channel row cg for every (m, b) block
    float* ws = p.ws + (long)z * p.Cg * p.KK;
#pragma unroll
    for (int m = 0; m < 2 * NQ; ++m) {
        const int row = cbase + m * 16 + l16;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int col = nt * 256 + wc * 64 + b * 16 + lg * 4;
            if (col < p.KK) *(f32x4*)(ws + (long)row * p.KK + col) = acc[m][b];
        }
    }
}

// -------------------------------------------------------------------------------------
// 64 -> 64 channel 3x3 stride-1 weight gradient (the layer1 convs of Res10/18/34, residuals.py:84-120; ws[z][co][kk],
// kk = tap * 64 + ci).  With 64 output-gradient channels every tile of the generic kernels is thin (64 x 256, and
// 576 = 2.25 tiles of 256 columns: a third of the last tile computes nothing) and each input pixel is fetched once
// per tap.  Here ONE workgroup computes all 64 x 576 outputs over its pixel range, and a stage of 64 output pixels
// (part of one output row) stages the input once as a halo of 3 rows x 66 columns (2.6x fewer bytes than the nine
// shifted copies) plus the 64 x 128 B output gradient, both by LDS-DMA.  The nine taps read the halo at shifted rows
// with ds_read_b64_tr_b16 (A operand = input columns, B = output-gradient channels, 16x16x32 bf16 MFMA).
// 8 waves: wave w owns the 16-channel input slice u = w & 3 of every tap (9 column blocks) and all four
// output-gradient channel blocks (36 accumulators), over k-step w >> 2 of each 64-pixel stage: 13 fragment pairs
// per 36 MFMAs (the earlier split -- two output-gradient blocks, both k-steps -- read 22 pairs per 36 MFMAs, and the
// fragment reads, not the MFMAs, bounded it: ablation build 42 ran 83.5 of its 99 us).  The two waves of an input
// slice sum their accumulators through LDS at the end.  Each halo row region is 80 rows apart (bits 0-3 of a row
// index do not change with the input row), so the fragment reads come from a few address registers plus immediate
// offsets (no per-read address VALU).  Stage t+1 is fetched into the other buffer while stage t is computed; one
// barrier per stage.
constexpr int L1W_KP = 64;                           // pixels per stage
constexpr int L1W_HC = L1W_KP + 2;                   // halo columns
constexpr int L1W_REG = 80;                          // LDS rows per halo row region (66 used)
constexpr int L1W_DMA_ROWS = 72;                     // rows of a region the DMA fills (whole 8-row instructions)
constexpr int L1W_HBYTES = 3 * L1W_REG * 128;
constexpr int L1W_STAGE = L1W_HBYTES + L1W_KP * 128;
constexpr int L1W_NHDMA = 3 * L1W_DMA_ROWS / 8;     // 27 halo DMA instructions per stage
// stage buffers: 2 (76 KiB of LDS, so the compute stream's kernels still fit beside it); 3 and 4 (ablation builds 45,
// 47) measured the same (56-57 us for the Res10 B=32 layer1 gradient: the fill is not what bounds it)
constexpr int L1W_NBUF = SCD_ABLATE == 45 ? 3 : SCD_ABLATE == 47 ? 4 : 2;

// 128-B rows, two per 256-B bank line: the 32-B unit u of row r is stored at u ^ f(r), so the transposed reads of
// rows {R..R+3, R+8..R+11} (any R: a tap shifts the base row) hit 8 distinct 32-B bank groups
__device__ __forceinline__ int l1w_f(int r) { return ((r >> 1) & 1) | (((r >> 3) & 1) << 1); }
__device__ __forceinline__ int l1w_addr(int r, int unit, int pp) { return r * 128 + ((unit ^ l1w_f(r)) << 5) + 8 * pp; }

__global__ __launch_bounds__(512, 1) void conv_wgrad_l1_kernel(WgradParams p) {
    __shared__ __attribute__((aligned(16))) char smem[L1W_NBUF * L1W_STAGE];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int u = wave & 3, ks = wave >> 2;         // input slice, k-step of each stage
    const int z = blockIdx.x;
    const int M = p.N * p.Ho * p.Wo;
    const int pix0 = min(M, z * p.chunk), pix1 = min(M, pix0 + p.chunk);
    const int H = p.Ho, W = p.Wo;

    // halo DMA: instruction i = wave + 8 j (i < 27) fills region i / 9, rows 8 (i % 9) .. +7; lane: row + lane / 8,
    // 16-B slot lane % 8 (source chunk swizzled)
    int h_dy[4], h_dx[4], h_c8[4];
    bool h_ok[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int i = wave + 8 * j;
        const int reg = i / 9, col = 8 * (i - reg * 9) + (lane >> 3);
        const int c = (lane & 7) ^ (l1w_f(col) << 1);
        h_ok[j] = col < L1W_HC;
        h_dy[j] = reg - 1;
        h_dx[j] = col - 1;
        h_c8[j] = c * 8;
    }
    const int g_R = 8 * wave + (lane >> 3);
    const int g_c8 = ((lane & 7) ^ (l1w_f(g_R) << 1)) * 8;

    int sn, soh, sow;
    {
        const int HW = H * W;
        sn = __builtin_amdgcn_readfirstlane(pix0 / HW);
        const int rem = pix0 - sn * HW;
        soh = __builtin_amdgcn_readfirstlane(rem / W);
        sow = __builtin_amdgcn_readfirstlane(rem - soh * W);
    }
    auto advance = [&]() {
        sow += L1W_KP;
        const bool wrap = sow >= W;
        sow = wrap ? 0 : sow;
        soh += wrap ? 1 : 0;
        const bool wrap2 = soh >= H;
        soh = wrap2 ? 0 : soh;
        sn += wrap2 ? 1 : 0;
        sn = __builtin_amdgcn_readfirstlane(sn);
        soh = __builtin_amdgcn_readfirstlane(soh);
        sow = __builtin_amdgcn_readfirstlane(sow);
    };
    const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc((void*)p.g, (short)0, p.gbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.xbytes, 0x00020000);
    auto issue = [&](int k0, char* buf) {
        const int S = __builtin_amdgcn_readfirstlane(((sn * H + soh) * W + sow) * 64);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = wave + 8 * j;
            if (i < L1W_NHDMA) {
                const int reg = i / 9;
                const bool ok = h_ok[j] & (k0 < pix1) & ((unsigned)(soh + h_dy[j]) < (unsigned)H) &
                                ((unsigned)(sow + h_dx[j]) < (unsigned)W);
                dma16_asm(xrs, buf + (reg * L1W_REG + 8 * (i - reg * 9)) * 128,
                          sel_off(ok, (S + (h_dy[j] * W + h_dx[j]) * 64 + h_c8[j]) * 2));
            }
        }
        dma16_asm(grs, buf + L1W_HBYTES + wave * 1024, sel_off(k0 + g_R < pix1, ((k0 + g_R) * 64 + g_c8) * 2));
    };

    const int l16 = lane & 15, lg = lane >> 4;
    const int q4 = l16 >> 2, pp = l16 & 3;
    const int r0 = 8 * lg + q4;                      // fragment row of k-step 0 (k-step 1: + 32 rows = + 4096 B)
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    auto trf = [&](const char* lo_addr, const char* hi_addr) {
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)lo_addr);
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)hi_addr);
        s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(h16x8, v);
    };
    // per-lane byte offsets: halo (tap column dw, lo/hi rows) and output gradient (block a; hi = lo + 4 rows)
    int xo[3][2], go[4];
#pragma unroll
    for (int dw = 0; dw < 3; ++dw)
#pragma unroll
        for (int h = 0; h < 2; ++h) xo[dw][h] = l1w_addr(r0 + dw + 4 * h, u, pp);
#pragma unroll
    for (int a = 0; a < 4; ++a) go[a] = L1W_HBYTES + l1w_addr(r0, a, pp);
    f32x4 acc[4][9];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[a][t] = (f32x4){0.f, 0.f, 0.f, 0.f};

    h16x8 gf[4], xf[9];
    auto reads = [&](const char* cur, int s2) {
#pragma unroll
        for (int a = 0; a < 4; ++a) gf[a] = trf(cur + go[a] + 4096 * s2, cur + go[a] + 4096 * s2 + 512);
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int off = (t / 3) * L1W_REG * 128 + 4096 * s2;
            xf[t] = trf(cur + xo[t % 3][0] + off, cur + xo[t % 3][1] + off);
        }
    };
    auto mfmas = [&]() {
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                if constexpr (SCD_ABLATE == 42) {          // ablation: fragment reads kept, no MFMA
                    asm volatile("" ::"v"(xf[t]), "v"(gf[a]));
                } else {
                    acc[a][t] = mfma_16x16x32_h16(xf[t], gf[a], acc[a][t]);
                }
            }
    };
    auto bar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();                 // raw: a __syncthreads() fence would drain the stages in flight
        __builtin_amdgcn_sched_barrier(0);
    };

    // L1W_NBUF stage buffers: stage t + NBUF - 1 is fetched while stage t is computed.  Every iteration issues a
    // whole stage -- past the end of the range with out-of-range offsets (zeros into a buffer nobody reads again, no
    // traffic) -- so the counts are uniform: this wave's DMAs per stage are n = its halo instructions (4 for waves
    // 0-2, 3 for the rest) + 1, and vmcnt((NBUF - 2) n) retires stage t+1 only.
    const int nk = (pix1 - pix0 + L1W_KP - 1) / L1W_KP;
    if (nk > 0) {
        const bool five = wave < L1W_NHDMA - 24;
        // retire stage t+1, leave stages t+2 .. t+NBUF-1 in flight
        auto wait_next = [&]() {
            if constexpr (SCD_ABLATE != 41) {
                if constexpr (L1W_NBUF == 4) {
                    if (five) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
                    else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                } else if constexpr (L1W_NBUF == 3) {
                    if (five) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
                    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
            }
        };
#pragma unroll
        for (int j = 0; j < L1W_NBUF - 1; ++j) {
            issue(pix0 + j * L1W_KP, smem + j * L1W_STAGE);
            advance();
        }
        if constexpr (L1W_NBUF == 4) {
            if (five) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else if constexpr (L1W_NBUF == 3) {
            if (five) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        bar();
        int b0 = 0;                                   // buffer of stage t
        for (int t = 0; t < nk; ++t) {
            const int b3 = b0 == 0 ? L1W_NBUF - 1 : b0 - 1;   // buffer of stage t+NBUF-1 (= that of stage t-1)
            const char* cur = smem + b0 * L1W_STAGE;
            if constexpr (SCD_ABLATE != 41) {         // ablation 41: no DMA after the prologue
                issue(pix0 + (t + L1W_NBUF - 1) * L1W_KP, smem + b3 * L1W_STAGE);
                advance();
            }
            reads(cur, ks);
            mfmas();
            wait_next();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            bar();
            b0 = b0 == L1W_NBUF - 1 ? 0 : b0 + 1;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // the k-step 1 waves hand their sums to the k-step 0 waves of the same input slice through LDS (the stage buffers,
    // two slices per round: 2 x 36 x 64 x 16 B = 72 KiB), which then write the fp32 slab: lane holds columns
    // kk .. kk+3 (kk = 64 t + 16 u + 4 lg) of channel 16 a + l16
    __syncthreads();
    static_assert(2 * 36 * 64 * 16 <= L1W_NBUF * L1W_STAGE, "reduction buffer");
    f32x4* xch = (f32x4*)smem;
#pragma unroll
    for (int round = 0; round < 2; ++round) {
        const bool mine = (u >> 1) == round;
        f32x4* slot = xch + (u & 1) * 36 * 64;
        if (mine && ks == 1) {
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int t = 0; t < 9; ++t) slot[(a * 9 + t) * 64 + lane] = acc[a][t];
        }
        __syncthreads();
        if (mine && ks == 0) {
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int t = 0; t < 9; ++t) acc[a][t] += slot[(a * 9 + t) * 64 + lane];
        }
        __syncthreads();
    }
    if (ks != 0) return;
    float* ws = p.ws + (long)z * 64 * 576;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        const int co = 16 * a + l16;
#pragma unroll
        for (int t = 0; t < 9; ++t)
            *(f32x4*)(ws + (long)co * 576 + 64 * t + 16 * u + 4 * lg) = acc[a][t];
    }
}

// row slices of one reduce launch (the three heads of a fused head weight gradient go to three parameters)
struct WredSlices {
    int n;
    int r0[4], r1[4];
    long ldn[4], ldc[4], ldt[4];
    float* dst[4];
};

// Split reduction: block (row, channel chunk) sums the nsplit slabs of its WRED_CB input channels x T taps of one
// slab row (coalesced 16-B reads, 8 slab loads in flight per thread, fixed summation order) into LDS, then writes the
// chunk in the destination's order (OIHW: taps fastest) so consecutive lanes store consecutive words.  The earlier
// form (one thread per 4 slab columns, stores 4 * ldc apart) read the slabs at ~2.2 TB/s behind its scattered
// stores (tools/wgrad_bench.py: 30 us for the layer4 conv2 gradient, 7 splits).
constexpr int WRED_CB = 128;                       // widest channel chunk (narrower when there are few rows)

// slab sum over splits g, g + S, g + 2S, ... of one 4-column unit (8 loads in flight), fixed order
__device__ __forceinline__ f32x4 wred_sum_strided(const float* src, int n, long zs, int g, int S) {
    f32x4 a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    int z = g;
    for (; z + 7 * S < n; z += 8 * S) {
        f32x4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = *(const f32x4*)(src + (long)(z + j * S) * zs);
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] += v[j];
    }
#pragma unroll
    for (int j = 0; j < 7; ++j)
        if (z + j * S < n) a[j] += *(const f32x4*)(src + (long)(z + j * S) * zs);
    return ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}

// block (row, channel chunk of cb): S thread groups per 4-column unit each sum every S-th split (S > 1 when the
// chunk has few units and there are many splits: the 64-row layer1 gradient over 256 splits), the S partials are
// added in LDS in a fixed order, and the chunk is written in the destination's order
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* ws, int nsplit, long zs, int T, int Ci,
                                                           int cvalid, WredSlices sl, int ncb, int cb, int S,
                                                           int accumulate, float alpha) {
    extern __shared__ float red[];                 // [T][cb + 1], then the S-way partials [S][units] (f32x4)
    const int tid = threadIdx.x;
    const int cbk = blockIdx.x % ncb;
    int rr = blockIdx.x / ncb;
    int s = 0;
    while (s < sl.n - 1 && rr >= sl.r1[s] - sl.r0[s]) { rr -= sl.r1[s] - sl.r0[s]; ++s; }
    const int row = sl.r0[s] + rr;
    const int c0 = cbk * cb, cn = min(cb, Ci - c0);
    const int upt = cn >> 2;                       // 4-column units per tap
    const int units = T * upt;
    const long KK = (long)T * Ci;
    const float* src = ws + (long)row * KK + c0;
    f32x4* part = (f32x4*)(red + ((T * (cb + 1) + 3) & ~3));
    if (S > 1) {
        for (int i = tid; i < units * S; i += blockDim.x) {
            const int u = i % units, g = i / units;
            const int t = u / upt, j = u - t * upt;
            part[g * units + u] = wred_sum_strided(src + (long)t * Ci + 4 * j, nsplit, zs, g, S);
        }
        __syncthreads();
    }
    for (int u = tid; u < units; u += blockDim.x) {
        const int t = u / upt, j = u - t * upt;
        f32x4 v;
        if (S > 1) {
            v = part[u];
            for (int g = 1; g < S; ++g) v += part[g * units + u];
        } else {
            v = wred_sum_strided(src + (long)t * Ci + 4 * j, nsplit, zs, 0, 1);
        }
        v *= alpha;
        float* d = red + t * (cb + 1) + 4 * j;
        d[0] = v[0]; d[1] = v[1]; d[2] = v[2]; d[3] = v[3];
    }
    __syncthreads();
    float* drow = sl.dst[s] + rr * sl.ldn[s];
    const long ldc = sl.ldc[s], ldt = sl.ldt[s];
    const bool taps_fast = ldt <= ldc;
    for (int i = tid; i < T * cn; i += blockDim.x) {
        int c, t;
        if (taps_fast) { c = i / T; t = i - c * T; }
        else { t = i / cn; c = i - t * cn; }
        if (c0 + c >= cvalid) continue;
        const float v = red[t * (cb + 1) + c];
        float* d = drow + (c0 + c) * ldc + t * ldt;
        *d = accumulate ? (*d + v) : v;
    }
}

template <typename T, int BM, int BN>
int launch_gemm(GemmParams& p, int Mtot_tiles, hipStream_t st, int ks = 1) {
    if constexpr (sizeof(T) == 2 && BM == 128 && BN == 128) {
        if (ks == 2 && !p.head_on) {
            if (p.bnbwd) hipLaunchKernelGGL((conv_gemm_kernel<T, BM, BN, false, true, 2>), dim3(Mtot_tiles), dim3(512), 0, st, p);
            else hipLaunchKernelGGL((conv_gemm_kernel<T, BM, BN, false, false, 2>), dim3(Mtot_tiles), dim3(512), 0, st, p);
            SCD_RETURN_LAUNCH();
        }
    }
    if (p.head_on) {
        if constexpr (BN == 128) hipLaunchKernelGGL((conv_gemm_kernel<T, BM, BN, true>), dim3(Mtot_tiles), dim3(256), 0, st, p);
        else return SCD_ERR_ARG;
    } else if (p.bnbwd) {
        if constexpr (sizeof(T) == 2) hipLaunchKernelGGL((conv_gemm_kernel<T, BM, BN, false, true>), dim3(Mtot_tiles), dim3(256), 0, st, p);
        else return SCD_ERR_ARG;
    } else {
        hipLaunchKernelGGL((conv_gemm_kernel<T, BM, BN, false>), dim3(Mtot_tiles), dim3(256), 0, st, p);
    }
    SCD_RETURN_LAUNCH();
}

// -------------------------------------------------------------------------------------
// Streaming 1x1 GEMM for the HBM-bound 1x1 convolutions: stride 1, K = Ci in {64, 128, 256} channels in, N = Co in
// {64, 128, 256} out, M pixels with M % 128 == 0 -- the Res50 Bottleneck layer1 convs and the conv3 / conv1 /
// downsample input gradients at 1024^2 (residuals.py:122-165).  y[m][n] = sum_k x[m][k] w[n][k] moves 2(K + N) bytes
// per pixel for 2KN flops (64 flops per byte at K = 256, N = 64), so HBM bounds it; the tiled GEMMs (one 256-pixel
// tile per workgroup, one workgroup per CU, load -> compute -> store in sequence) ran these shapes at 2-3 TB/s.
// Here the packed weights [N][K] stay in LDS for the workgroup's whole run (cpw chunks of 128 pixels, taken by the
// waves as units of 16 or 32 pixels in turn), the operand goes from HBM straight into the MFMA fragments (16-B loads, K/32
// per lane and unit) one unit ahead of its MFMAs, and 2-4 workgroups per CU keep 8-16 waves' loads outstanding.
// Operands of the epilogue (the old output when accumulating, the pre-BN activation for the BN-backward sums) are
// loaded before the next unit's operand, so no wait on them drains the prefetch.  SPL = 2: the waves work in pairs
// on the same pixels, each on half of the N channels (the pair's second operand read hits L2), SPL = 4 all four on a
// quarter each, so a wave's sums cover 64 channels at N = 128 / 256 as well.
// Per output the MFMA chain is that of the ping-pong / ring / register-staged kernels (k in steps of 32, ascending;
// weights as the A operand), so the outputs are the same bits.  Epilogue: channel blocks paired with
// v_permlane16_swap (a lane then holds 8 consecutive channels of one pixel: 16-B stores); MODE 0 stores (+ forward BN
// sums of the fp32 values when p.stats), 1 accumulates as the staged epilogues do (round(round(acc) + old)), 2 adds
// the following BN+ReLU layer's backward sums (scd_conv_gemm_bnbwd: dz = stored gradient where y*rsc + rsh > 0).
// The sums (64 channels per wave): per-lane partials over the run, 16-lane DPP sums, the waves' partials in a fixed
// order, one fp64 replica add per channel and workgroup.
// The LDS plan of an instance.  SPL > 1 (STG): the SPL waves on the same pixels would each load the unit's operand as
// fragment-shaped 16-B pieces (16 rows x 64 B per instruction, SPL times over); instead each loads 1 / SPL of it by
// LDS-DMA in whole 128-B lines into a double-buffered LDS unit (the weights' swizzle), and all read their fragments
// from there -- where the LDS holds it without cutting the workgroups per CU below two (or one where it held one).
template <int K, int N, int MODE, int SPL, int UA, int WV>
struct S1x1Plan {
    static constexpr int WBYTES = N * K * 2;
    static constexpr int PBYTES = MODE == 2 ? 4 * N * 4 : 0;       // BN parameters (mean, invstd, relu scale / shift)
    static constexpr int XU = 16 * UA * K * 2;                     // bytes of one pixel wave's unit
    static constexpr int XALL = 2 * (WV / SPL) * XU;               // two buffers per pixel wave
    static constexpr int OCC0 = 163840 / (WBYTES + PBYTES), OCC1 = 163840 / (WBYTES + PBYTES + XALL);
    static constexpr bool STG = S1X1_STG && SPL > 1 && OCC1 >= 1 && (OCC1 >= 2 || OCC0 < 2);
    static constexpr int XBYTES = STG ? XALL : 0;
};
template <int K, int N, int MODE, int SPL, int UA, int WV>
__global__ __launch_bounds__(64 * WV, 8 / WV) void conv1x1_stream_kernel(GemmParams p, int cpw) {
    typedef S1x1Plan<K, N, MODE, SPL, UA, WV> Plan;
    typedef h16 T;
    typedef __attribute__((ext_vector_type(4))) h16 hv4;
    typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
    constexpr int KS = K / 32;                              // MFMA k-steps
    constexpr int NH = N / SPL;                             // channels per wave
    constexpr int NB = NH / 16;                             // 16-channel blocks per wave
    constexpr int NT = 64 * WV;                             // threads (WV waves: 8 where the weights fill the LDS)
    constexpr int PXW = WV / SPL;                           // waves on different pixels
    constexpr int UP = 16 * UA;                             // pixels per unit (UA 16-pixel blocks)
    constexpr int XM = (K / 8 >= 16 ? 16 : K / 8) - 1;      // LDS swizzle: chunk c of row r at c ^ (r & XM)
    constexpr bool SUMS = NH == 64 && MODE != 1;
    constexpr int NS = SUMS ? 4 * NB : 1;                   // per-lane channel slots of the sums
    constexpr int WBYTES = Plan::WBYTES, PBYTES = Plan::PBYTES, XU = Plan::XU, XBYTES = Plan::XBYTES;
    constexpr bool STG = Plan::STG;
    static_assert(NB % 2 == 0 && K % 64 == 0 && WV % SPL == 0 && 128 % (16 * UA * PXW) == 0, "shape");
    static_assert(WBYTES >= PXW * N * 8, "sum exchange fits the weight buffer");
    static_assert(!STG || (UP * K / 8) % (64 * SPL) == 0, "whole LDS-DMA instructions per wave");
    __shared__ __attribute__((aligned(16))) char smem[WBYTES + PBYTES + XBYTES];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l16 = lane & 15, lg = lane >> 4;
    const int pw = wave / SPL;                              // pixel wave
    const int c0w = (wave % SPL) * NH;                      // the wave's first channel (of the workgroup's slice)
    const int cb = blockIdx.y * N;                          // the slice's first output channel (p.Co = N * gridDim.y)
    const int ldy = p.Co;                                   // output (and epilogue operand) row stride
    for (int i = tid; i < N * K / 8; i += NT) {
        const int r = i / (K / 8), c = i - r * (K / 8);
        const uint4 v = *(const uint4*)(p.w + ((long)(cb + r) * p.wrow + c * 8) * 2);
        *(uint4*)(smem + r * K * 2 + ((c ^ (r & XM)) << 4)) = v;
    }
    float* bnp = (float*)(smem + WBYTES);
    if constexpr (MODE == 2) {
        for (int i = tid; i < N; i += NT) {
            bnp[i] = p.bn_mean[cb + i];
            bnp[N + i] = p.bn_invstd[cb + i];
            bnp[2 * N + i] = p.bn_rsc[cb + i];
            bnp[3 * N + i] = p.bn_rsh[cb + i];
        }
    }
    __syncthreads();

    const long chunk0 = (long)blockIdx.x * cpw;
    const bool stats_on = SUMS && p.stats != nullptr;
    float ssum[NS], ssq[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) { ssum[j] = 0.f; ssq[j] = 0.f; }
    // lane's store column of channel-block pair (b, b + 1): even lg block b, odd lg block b + 1 (permlane16_swap)
    const int cst = c0w + 4 * lg + 12 * (lg & 1);
    // S1X1_FULLROW: a lane's place in the whole-128-B-row layout of a 64-channel piece (pixel l16 & 7 of the first or
    // second 8 of a 16-pixel block, channels fr_cw .. + 7 of the piece; see the stores in unit())
    const bool fr_hi = l16 >= 8;
    const int fr_cw = 32 * (l16 >> 3) + (cst & 31);
    // the epilogue operands in that layout too where a wave holds one 64-channel piece (wider waves: their conversion
    // temporaries spill)
    // (not for the BN-backward-sum instances at K = 256, which then spill)
    constexpr bool ST_FR = S1X1_FULLROW && !(MODE == 2 && K >= 256);
    constexpr bool EPI_FR = ST_FR && NB == 4;
    auto ror8 = [](const uint4& v) {
        uint4 r;
        r.x = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v.x, 0x128, 0xf, 0xf, false);   // row_ror:8
        r.y = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v.y, 0x128, 0xf, 0xf, false);
        r.z = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v.z, 0x128, 0xf, 0xf, false);
        r.w = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v.w, 0x128, 0xf, 0xf, false);
        return r;
    };
    auto sel4 = [](bool c, const uint4& a, const uint4& b) {
        uint4 r;
        r.x = c ? a.x : b.x; r.y = c ? a.y : b.y; r.z = c ? a.z : b.z; r.w = c ? a.w : b.w;
        return r;
    };

    auto pix0 = [&](int u) -> long { return chunk0 * 128 + (u * PXW + pw) * UP; };
    auto load_unit = [&](int u, h16x8 (&xf)[UA][KS]) {
#pragma unroll
        for (int a = 0; a < UA; ++a) {
            const char* row = p.x + ((pix0(u) + 16 * a + l16) * K + 8 * lg) * 2;
#pragma unroll
            for (int s = 0; s < KS; ++s) xf[a][s] = *(const h16x8*)(row + s * 64);
        }
    };
    auto load_epi = [&](int u, uint4 (&ev)[UA][NB / 2]) {
        if constexpr (MODE != 0) {
            const char* src = MODE == 1 ? (const char*)p.y : p.bny;
#pragma unroll
            for (int a = 0; a < UA; ++a) {
                if constexpr (EPI_FR) {
                    // whole 128-B row pieces, in the stores' layout (turned into the fragment layout where used)
                    const char* r0 = src + ((pix0(u) + 16 * a + (l16 & 7)) * ldy + cb + c0w + fr_cw) * 2;
#pragma unroll
                    for (int q = 0; q < NB / 4; ++q) {
                        ev[a][2 * q] = *(const uint4*)(r0 + 128 * q);
                        ev[a][2 * q + 1] = *(const uint4*)(r0 + 128 * q + 16 * ldy);
                    }
                } else {
#pragma unroll
                    for (int pb = 0; pb < NB / 2; ++pb)
                        ev[a][pb] = *(const uint4*)(src + ((pix0(u) + 16 * a + l16) * ldy + cb + 32 * pb + cst) * 2);
                }
            }
        }
    };
    auto unit = [&](int u, const h16x8 (&xf)[UA][KS], const uint4 (&ev)[UA][NB / 2]) {
        f32x4 acc[UA][NB];
#pragma unroll
        for (int a = 0; a < UA; ++a)
#pragma unroll
            for (int b = 0; b < NB; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
        // the weight fragments are re-read from LDS per unit (an opaque base keeps the compiler from hoisting all
        // KS x NB of them into registers for the whole run)
        int wo = (c0w + l16) * K * 2;
        asm volatile("" : "+v"(wo));
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                const int r = c0w + 16 * b + l16;
                const h16x8 wf = *(const h16x8*)(smem + wo + 16 * b * K * 2 + (((4 * s + lg) ^ (r & XM)) << 4));
#pragma unroll
                for (int a = 0; a < UA; ++a)
                    acc[a][b] = mfma_16x16x32_h16(wf, xf[a][s], acc[a][b]);
            }
        if constexpr (MODE == 0 && SUMS) {
            if (stats_on) {
#pragma unroll
                for (int a = 0; a < UA; ++a)
#pragma unroll
                    for (int b = 0; b < NB; ++b)
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const float v = acc[a][b][i];
                            ssum[4 * b + i] += v;
                            ssq[4 * b + i] += v * v;
                        }
            }
        }
#pragma unroll
        for (int a = 0; a < UA; ++a)
#pragma unroll
        for (int q = 0; q < NB / 4; ++q) {
        // one 64-channel piece (blocks 4q .. 4q + 3) at a time: the channel-block pairs 2q and 2q + 1
        uint4 stv[2], evv[2];
        if constexpr (MODE != 0 && EPI_FR) {                 // row-piece layout -> the fragment layout
            const uint4 w0 = ev[a][2 * q], w1 = ev[a][2 * q + 1];
            evv[0] = sel4(fr_hi, ror8(w1), w0);
            evv[1] = sel4(fr_hi, w1, ror8(w0));
        } else if constexpr (MODE != 0) {
            evv[0] = ev[a][2 * q];
            evv[1] = ev[a][2 * q + 1];
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int pb = 2 * q + j;
            const long m = pix0(u) + 16 * a + l16;
            hv4 h0, h1;
#pragma unroll
            for (int i = 0; i < 4; ++i) { h0[i] = (T)acc[a][2 * pb][i]; h1[i] = (T)acc[a][2 * pb + 1][i]; }
            const u32x2 x = __builtin_bit_cast(u32x2, h0), y = __builtin_bit_cast(u32x2, h1);
            const auto s0 = __builtin_amdgcn_permlane16_swap(x[0], y[0], false, false);
            const auto s1 = __builtin_amdgcn_permlane16_swap(x[1], y[1], false, false);
            uint4 st;
            st.x = s0[0]; st.y = s1[0]; st.z = s0[1]; st.w = s1[1];
            if constexpr (MODE == 1) {
                float a8[8], o8[8];
                Vec16<T>::load(&st, a8);
                Vec16<T>::load(&evv[j], o8);
#pragma unroll
                for (int e = 0; e < 8; ++e) a8[e] += o8[e];
                Vec16<T>::store(&st, a8);
            }
            if constexpr (MODE == 2) {
                float d8[8], y8[8], mu[8], is[8], sc[8], sh[8];
                Vec16<T>::load(&st, d8);
                Vec16<T>::load(&evv[j], y8);
                const int c0 = 32 * pb + cst;
#pragma unroll
                for (int e = 0; e < 8; e += 4) {
                    const float4 f0 = *(const float4*)(bnp + c0 + e), f1 = *(const float4*)(bnp + N + c0 + e);
                    const float4 f2 = *(const float4*)(bnp + 2 * N + c0 + e), f3 = *(const float4*)(bnp + 3 * N + c0 + e);
                    mu[e] = f0.x; mu[e + 1] = f0.y; mu[e + 2] = f0.z; mu[e + 3] = f0.w;
                    is[e] = f1.x; is[e + 1] = f1.y; is[e + 2] = f1.z; is[e + 3] = f1.w;
                    sc[e] = f2.x; sc[e + 1] = f2.y; sc[e + 2] = f2.z; sc[e + 3] = f2.w;
                    sh[e] = f3.x; sh[e + 1] = f3.y; sh[e + 2] = f3.z; sh[e + 3] = f3.w;
                }
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float dz = y8[e] * sc[e] + sh[e] > 0.f ? d8[e] : 0.f;
                    ssum[8 * pb + e] += dz;
                    ssq[8 * pb + e] += dz * (y8[e] - mu[e]) * is[e];
                }
            }
            if constexpr (ST_FR) stv[j] = st;
            else *(uint4*)((T*)p.y + m * ldy + cb + 32 * pb + cst) = st;
        }
        if constexpr (ST_FR) {
            // the piece as whole 128-B row pieces: the upper 8 lanes of each 16-lane row trade pair 2q + 1 of pixels
            // 0-7 for pair 2q of pixels 8-15 (DPP rotate by 8 within the row), so each store writes 8 whole row pieces
            // instead of 16 half ones
            T* dst = (T*)p.y + (pix0(u) + 16 * a + (l16 & 7)) * ldy + cb + c0w + 64 * q + fr_cw;
            *(uint4*)dst = sel4(fr_hi, ror8(stv[1]), stv[0]);
            *(uint4*)(dst + 8 * ldy) = sel4(fr_hi, stv[1], ror8(stv[0]));
        }
        }
    };

    h16x8 xa[UA][KS], xb[UA][KS];
    uint4 ea[UA][NB / 2], eb[UA][NB / 2];
    // an even number of units per wave; the prefetch past the run re-reads its last unit (clamped: every load from a
    // valid address)
    const int nu = cpw * (128 / (UP * PXW));
    if constexpr (STG) {
        char* xs = smem + WBYTES + PBYTES;                  // [2 buffers][PXW][UP rows][K] (chunk c of row r at c ^ (r & XM))
        constexpr int ND = UP * K / 8 / (64 * SPL);         // LDS-DMA instructions per wave and unit
        constexpr int EW = MODE != 0 ? UA * NB / 2 : 0;     // epilogue operand loads per wave and unit
        constexpr int SW = UA * NB / 2;                     // output stores per wave and unit
        const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.xbytes, 0x00020000);
        const int ws = wave % SPL;
        auto dma_unit = [&](int u, int b) {
            char* dst = xs + (b * PXW + pw) * XU;
            const int px = (int)pix0(u);
#pragma unroll
            for (int i = 0; i < ND; ++i) {
                const int q0 = (i * SPL + ws) * 64, q = q0 + lane;
                const int r = q / (K / 8), c = (q % (K / 8)) ^ (r & XM);
                dma16(xrs, dst + q0 * 16, ((px + r) * K + c * 8) * 2);
            }
        };
        auto read_unit = [&](int b, h16x8 (&xf)[UA][KS]) {
            const char* src = xs + (b * PXW + pw) * XU;
#pragma unroll
            for (int a = 0; a < UA; ++a) {
                const int r = 16 * a + l16;
#pragma unroll
                for (int s = 0; s < KS; ++s) xf[a][s] = *(const h16x8*)(src + r * K * 2 + (((4 * s + lg) ^ (r & XM)) << 4));
            }
        };
        // unit u sits in buffer u & 1; before a wave reads it, every wave's DMAs of it have landed (counted vmcnt: the
        // epilogue operand loads of the unit and the stores of the one before were issued after them) and every wave
        // is done with the unit before (the barrier), whose buffer the next DMA overwrites
        dma_unit(0, 0);
        load_epi(0, ea);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(EW) : "memory");
        __builtin_amdgcn_s_barrier();
        for (int u = 0; u < nu; u += 2) {
            if (u > 0) {
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(EW + SW) : "memory");
                __builtin_amdgcn_s_barrier();
            }
            read_unit(0, xa);
            asm volatile("" ::: "memory");
            dma_unit(u + 1, 1);
            load_epi(u + 1, eb);
            unit(u, xa, ea);
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(EW + SW) : "memory");
            __builtin_amdgcn_s_barrier();
            read_unit(1, xb);
            asm volatile("" ::: "memory");
            dma_unit(min(u + 2, nu - 1), 0);
            load_epi(min(u + 2, nu - 1), ea);
            unit(u + 1, xb, eb);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the clamped last DMA has landed before the LDS is reused
    } else {
        load_unit(0, xa);
        for (int u = 0; u < nu; u += 2) {
            load_epi(u, ea);
            load_unit(u + 1, xb);
            unit(u, xa, ea);
            load_epi(u + 1, eb);
            load_unit(min(u + 2, nu - 1), xa);
            unit(u + 1, xb, eb);
        }
    }
    if constexpr (SUMS) {
        if (MODE == 2 || stats_on) {
            __syncthreads();                                 // every wave is done with the weights: LDS reused
            float* red = (float*)smem;                       // [pixel wave][N][2]
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                const float s = row16_sum(ssum[j]), q = row16_sum(ssq[j]);
                if (l16 == 0) {
                    const int c = MODE == 2 ? 32 * (j >> 3) + cst + (j & 7) : c0w + 16 * (j >> 2) + 4 * lg + (j & 3);
                    red[(pw * N + c) * 2] = s;
                    red[(pw * N + c) * 2 + 1] = q;
                }
            }
            __syncthreads();
            for (int c = tid; c < N; c += NT) {
                double s = 0.0, q = 0.0;
#pragma unroll
                for (int w = 0; w < PXW; ++w) { s += red[(w * N + c) * 2]; q += red[(w * N + c) * 2 + 1]; }
                const int rep = (int)(blockIdx.x % SCD_STAT_REPLICAS);
                atomic_add_f64(p.stats + ((long)rep * 2 + 0) * p.Co + cb + c, s);
                atomic_add_f64(p.stats + ((long)rep * 2 + 1) * p.Co + cb + c, q);
            }
        }
    }
}

SCD_KERNEL_NS_END
}  // namespace

// conv1x1_stream_kernel: -1 when the shape is not one it takes, else the launch status.  SCD_GEMM_STREAM1X1 (read
// per call: tests compare the kernels bit for bit): 0 keeps these shapes on the tiled kernels, 2 (tests) makes every
// GEMM the stream kernel does not take fail with SCD_ERR_ARG
static int stream1x1_mode() {
    const char* e = getenv("SCD_GEMM_STREAM1X1");
    return e ? atoi(e) : 1;
}
// SCD_S1X1_OCC (read per call): at most this many stream workgroups per CU (0 / unset: as many as fit)
static int s1x1_occ_cap() {
    const char* e = getenv("SCD_S1X1_OCC");
    return e ? atoi(e) : 0;
}
static int num_cus();
static int launch_stream1x1(int dtype, GemmParams& p, int nphase, const scd_gemm_phase* phases, long Mtot,
                            hipStream_t st) {
    if (dtype != SCD_DT_BF16 || stream1x1_mode() == 0) return -1;
    if (nphase != 1 || p.is != 1 || p.os != 1 || p.head_on || p.bias || p.relu || p.shuf) return -1;
    const scd_gemm_phase& ph = phases[0];
    if (ph.ntaps != 1 || ph.dh[0] || ph.dw[0] || ph.wt[0] || ph.rho_h || ph.rho_w || ph.Qh != p.Ho || ph.Qw != p.Wo ||
        p.Hi != p.Ho || p.Wi != p.Wo || p.wrow != p.Ci)
        return -1;
    const int K = p.Ci, N = p.Co;
    if (Mtot % 128 || Mtot < 65536 || Mtot * (long)(K > N ? K : N) >= (1L << 30)) return -1;
    p.xbytes = (int)(Mtot * K * 2);                          // the operand's buffer range (LDS-DMA path)
    const bool sums = p.stats != nullptr;                    // forward statistics or BN-backward sums
    if (p.accumulate && sums) return -1;
    const long nchunks = Mtot / 128;
    const long cus = num_cus();
    const int mode = p.bnbwd ? 2 : (p.accumulate ? 1 : 0);
    // the whole N in one workgroup where an instance holds it, else slices of 256 output channels (grid.y; every
    // slice re-reads the operand, from L2 when the slices of a chunk run together)
    for (int attempt = 0; attempt < 2; ++attempt) {
    const int Nd = attempt == 0 ? N : 256;
    if (attempt == 1 && (N <= 256 || N % 256)) break;
    const int nsl = N / Nd;
    // about one round of resident workgroups: as many per CU as the instance's registers and LDS allow (capped by
    // SCD_S1X1_OCC when set), so every workgroup of the grid runs in the first round
    auto plan = [&](const void* kern, int threads, int& per_cache, long& cpw, int& grid) -> bool {
        if (per_cache < 0) {
            int per = 1;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, threads, 0) != hipSuccess || per < 1) per = 1;
            per_cache = per;
        }
        const int cap = s1x1_occ_cap();
        const long per = cap > 0 ? std::min(cap, per_cache) : per_cache;
        const long want = std::max(1L, per * cus / nsl);
        cpw = 2;                                             // (even: the waves take units in pairs)
        while (nchunks / cpw > want && nchunks % (2 * cpw) == 0) cpw *= 2;
        if (nchunks % cpw) return false;
        grid = (int)(nchunks / cpw);
        return true;
    };
    long cpw = 0;
    int grid = 0;
    // (two 16-pixel blocks per unit at K = 64 and <= 64 channels per wave: 4-KB operand loads per wave in flight; not
    // with the BN-backward sums, whose registers it would spill)
#define SCD_S1X1(KK, NN, MM, SS)                                                                                     \
    if (K == KK && Nd == NN && mode == MM) {                                                                         \
        constexpr int UA_ = (S1X1_UA2 && KK == 64 && NN / SS <= 64 && MM != 2) ? 2 : 1;                              \
        static int per_ = -1;                                                                                        \
        if (!plan((const void*)conv1x1_stream_kernel<KK, NN, MM, SS, UA_, 4>, 256, per_, cpw, grid)) return -1;      \
        hipLaunchKernelGGL((conv1x1_stream_kernel<KK, NN, MM, SS, UA_, 4>), dim3(grid, nsl), dim3(256), 0, st, p, (int)cpw); \
        SCD_RETURN_LAUNCH();                                                                                         \
    }
    // N = 64: one wave per pixel unit; N = 128 / 256: 2 / 4 waves split the channels when there are sums to take (the
    // per-lane partials of 64 channels), whole-width waves otherwise
    SCD_S1X1(64, 64, 0, 1) SCD_S1X1(64, 64, 1, 1) SCD_S1X1(64, 64, 2, 1)
    SCD_S1X1(128, 64, 0, 1) SCD_S1X1(128, 64, 1, 1) SCD_S1X1(128, 64, 2, 1)
    SCD_S1X1(256, 64, 0, 1) SCD_S1X1(256, 64, 1, 1) SCD_S1X1(256, 64, 2, 1)
    // K x N = 64 K elements (128-KB weight buffer): one workgroup of 8 waves per CU
#define SCD_S1X1W(KK, NN, MM, SS, UU)                                                                                \
    if (K == KK && Nd == NN && mode == MM) {                                                                         \
        static int per_ = -1;                                                                                        \
        if (!plan((const void*)conv1x1_stream_kernel<KK, NN, MM, SS, UU, 8>, 512, per_, cpw, grid)) return -1;       \
        hipLaunchKernelGGL((conv1x1_stream_kernel<KK, NN, MM, SS, UU, 8>), dim3(grid, nsl), dim3(512), 0, st, p, (int)cpw); \
        SCD_RETURN_LAUNCH();                                                                                         \
    }
    if (sums) {
        SCD_S1X1W(512, 128, 0, 2, 1) SCD_S1X1W(512, 128, 2, 2, 1) SCD_S1X1W(128, 512, 0, 8, 2)
        SCD_S1X1W(256, 256, 0, 4, 1) SCD_S1X1W(256, 256, 2, 4, 1)
    } else {
        SCD_S1X1W(512, 128, 0, 1, 1) SCD_S1X1W(512, 128, 1, 1, 1) SCD_S1X1W(128, 512, 0, 2, 1)
        SCD_S1X1W(128, 512, 1, 2, 1) SCD_S1X1W(256, 256, 0, 1, 1) SCD_S1X1W(256, 256, 1, 1, 1)
    }
#undef SCD_S1X1W
    if (sums) {
        SCD_S1X1(64, 128, 0, 2) SCD_S1X1(128, 128, 0, 2) SCD_S1X1(256, 128, 0, 2)
        SCD_S1X1(64, 128, 2, 2) SCD_S1X1(128, 128, 2, 2) SCD_S1X1(256, 128, 2, 2)
        SCD_S1X1(64, 256, 0, 4) SCD_S1X1(128, 256, 0, 4)
    } else {
        SCD_S1X1(64, 256, 0, 1) SCD_S1X1(64, 256, 1, 1) SCD_S1X1(128, 256, 0, 1)
        SCD_S1X1(64, 128, 0, 1) SCD_S1X1(64, 128, 1, 1) SCD_S1X1(128, 128, 0, 1) SCD_S1X1(128, 128, 1, 1)
        SCD_S1X1(256, 128, 0, 1) SCD_S1X1(256, 128, 1, 1)
    }
#undef SCD_S1X1
    }
    return -1;
}

// Kernel choice: the LDS-DMA ring kernel (256x128, bf16) for large outputs, the register-staged
// 128x128 kernel otherwise, 256x64 for narrow outputs (Co <= 64).  SCD_GEMM_RING=0/1 forces it off/on.
// Intra-workgroup split K of the register-staged 128x128 kernel (SCD_GEMM_KSPLIT: 0 off, 1 auto = grids of at
// most 1.5 tiles per CU with >= 16 K stages, 2 always where it applies)
static int ksplit_mode() {
    static int mode = -1;
    if (mode < 0) {
        const char* e = getenv("SCD_GEMM_KSPLIT");
        mode = e ? atoi(e) : 1;
    }
    return mode;
}

static int ring_mode() {
    static int mode = -2;
    if (mode == -2) {
        const char* e = getenv("SCD_GEMM_RING");
        mode = e ? atoi(e) : -1;
    }
    return mode;
}

static int narrow_ring_mode() {
    // SCD_GEMM_NARROW_RING=0: narrow 1x1 shapes on the register-staged 256 x 64 kernel (read per call: A/B).  On the
    // ring kernel: Res50 1024^2 fp16 +0.4 % (the 256 x 64 kernel's 88 launches of 268 us per 11 steps become ring
    // launches), Res10 neutral (profiles/r4_ab.txt)
    const char* e = getenv("SCD_GEMM_NARROW_RING");
    return e ? atoi(e) : 1;
}
static int pp_mode() {
    static int mode = -2;
    if (mode == -2) {
        const char* e = getenv("SCD_GEMM_PP");
        mode = e ? atoi(e) : 1;
    }
    return mode;
}

static int duo_mode() {
    // SCD_GEMM_DUO (read per call: tests compare the kernels): 0 = off, 1 = the ping-pong shapes (Co % 256 / 192 == 0)
    // on the two-workgroups-per-CU kernel, 2 = also the 256 x 128 ring shapes (Co % 128 == 0), 3 = only the ping-pong
    // shapes with the BN-backward-sum epilogue and >= 8 rounds of duo tiles (where the epilogue is what the two
    // workgroups per CU overlap: the heatmap-head input gradient; tools/duo_probe.py), 4 = only the ring shapes
    // (Co % 128 == 0, not a ping-pong width: the layer2 convs at 128 channels)
    const char* e = getenv("SCD_GEMM_DUO");
    return e ? atoi(e) : 0;
}

static int duo_delay_pct() {
    const char* e = getenv("SCD_DUO_DELAY");
    return e ? atoi(e) : 100;
}

static int heads384_mode() {
    static int mode = -2;
    if (mode == -2) {
        const char* e = getenv("SCD_GEMM_HEADS384");
        mode = e ? atoi(e) : 1;
    }
    return mode;
}

static int num_cus() {
    static int n = 0;
    if (n == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}

static int pp_bn(int dtype, int Co) {
    if (dtype != SCD_DT_BF16 || !pp_mode()) return 0;
    if (Co % 256 == 0) return 256;
    if (Co % 192 == 0) return 192;
    return 0;
}

static int halo64_mode() {
    // SCD_GEMM_HALO64=0: the register-staged kernel.  Read per launch (not cached): tests switch it to compare the
    // two bit for bit
    const char* e = getenv("SCD_GEMM_HALO64");
    return e ? atoi(e) : 1;
}

// conv_gemm_l1p_kernel's shapes: one phase of the 9 taps of a 3x3 / stride 1 / pad 1 convolution in the forward
// order (dh, dw, wt) = (r - 1, s - 1, 3r + s) -> 0, or the input-gradient order (1 - r, 1 - s, 3r + s) -> 1;
// 64 -> 64 channels, rows of 64 or 128 pixels, whole tiles of 256 pixels.  -1: not this kernel.
static int halo64_taps(const GemmParams& p, int nphase, const scd_gemm_phase* phases) {
    if (nphase != 1 || p.Ci != 64 || p.Co != 64 || p.is != 1 || p.os != 1 || p.head_on || p.wrow != 9 * 64) return -1;
    const scd_gemm_phase& ph = phases[0];
    if (ph.ntaps != 9 || ph.rho_h || ph.rho_w || ph.Qh != p.Ho || ph.Qw != p.Wo || p.Hi != p.Ho || p.Wi != p.Wo)
        return -1;
    if (p.Wo != 256 && p.Wo != 128 && p.Wo != 64) return -1;
    if (p.Wo < 256 && ph.Qh % (256 / p.Wo)) return -1;
    int fwd = 1, bwd = 1;
    for (int t = 0; t < 9; ++t) {
        const int r = t / 3, c = t % 3;
        if (ph.wt[t] != t) return -1;
        fwd &= ph.dh[t] == r - 1 && ph.dw[t] == c - 1;
        bwd &= ph.dh[t] == 1 - r && ph.dw[t] == 1 - c;
    }
    return fwd ? 0 : (bwd ? 1 : -1);
}

static int conv_gemm_launch(int dtype, GemmParams& p, int nphase, const scd_gemm_phase* phases, void* stream) {
    if (nphase < 1 || nphase > SCD_MAX_PHASES) return SCD_ERR_ARG;
    const int BK = dtype == SCD_DT_BF16 ? 64 : 32;
    const int EPC = dtype == SCD_DT_BF16 ? 8 : 4;
    if (p.Ci % BK != 0 || p.Co <= 0 || p.Co % EPC != 0 || p.N <= 0) return SCD_ERR_ARG;
    p.nphase = nphase;
    const int esz = dtype == SCD_DT_BF16 ? 2 : 4;
    const long xb = (long)p.N * p.Hi * p.Wi * p.Ci * esz;
    const bool narrow = p.Co <= 64;
    if (p.head_on && (narrow || p.Co != 128 * ((p.Co + 127) / 128))) return SCD_ERR_ARG;
    long Mtot = 0;
    for (int i = 0; i < nphase; ++i) {
        if (phases[i].ntaps < 0 || phases[i].ntaps > SCD_MAX_TAPS) return SCD_ERR_ARG;
        for (int t = 0; t < phases[i].ntaps; ++t)
            if (phases[i].wt[t] < 0 || (long)(phases[i].wt[t] + 1) * p.Ci > p.wrow) return SCD_ERR_ARG;
        Mtot += (long)p.N * phases[i].Qh * phases[i].Qw;
    }
    {
        const int rc = launch_stream1x1(dtype, p, nphase, phases, Mtot, (hipStream_t)stream);
        if (rc >= 0) return rc;
        if (stream1x1_mode() == 2) return SCD_ERR_ARG;
    }
    if (p.head_on && dtype == SCD_DT_BF16 && heads384_mode() && nphase == 1 && p.Co == 384 && p.head_out[0] &&
        p.head_out[1] && p.head_out[2] && !p.head_out[3] && p.is == 1 && p.os == 1 && p.Ho == phases[0].Qh &&
        p.Wo == phases[0].Qw && p.bias && p.relu && !p.accumulate && !p.stats) {
        // the three 128-wide CenterNet heads: one 192 x 384 tile per 192 pixels, tails fused
        const long wb = (long)p.Co * p.wrow * esz;
        if (xb >= (1L << 31) - 64 || wb >= (1L << 31) - 64) return SCD_ERR_ARG;
        p.xbytes = (int)xb;
        p.wbytes = (int)wb;
        p.ntn = 1;
        p.ph[0] = phases[0];
        for (int i = 0; i <= SCD_MAX_PHASES; ++i) p.tile_start[i] = 0;
        const int tiles = cdiv(Mtot, 192);
        hipLaunchKernelGGL(conv_gemm_heads384_kernel, dim3(tiles), dim3(512), 0, (hipStream_t)stream, p);
        SCD_RETURN_LAUNCH();
    }
    {
        // two 256 x 128 workgroups per CU (conv_gemm_duo_kernel) where the grid gives each CU >= 2 tiles
        const int dm = duo_mode();
        const bool shape = dtype == SCD_DT_BF16 && !p.head_on && p.Co % 128 == 0 &&
                           (dm == 4 ? !pp_bn(dtype, p.Co) : (pp_bn(dtype, p.Co) || dm >= 2));
        const long dtiles = (long)cdiv(Mtot, 256) * (p.Co / 128);
        const bool take = dm == 3 ? (p.bnbwd && dtiles >= 16L * num_cus()) : dtiles >= 2L * num_cus();
        if (dm && shape && take) {
            p.ntn = p.Co / 128;
            int tiles = 0;
            int ktmax = 0;
            for (int i = 0; i < SCD_MAX_PHASES; ++i) {
                p.tile_start[i] = tiles;
                if (i < nphase) {
                    p.ph[i] = phases[i];
                    tiles += cdiv((long)p.N * phases[i].Qh * phases[i].Qw, 256) * p.ntn;
                    ktmax = std::max(ktmax, phases[i].ntaps * (p.Ci / 64) * 2);
                }
            }
            p.tile_start[SCD_MAX_PHASES] = tiles;
            const long wb = (long)p.Co * p.wrow * esz;
            if (xb >= (1L << 31) - 64 || wb >= (1L << 31) - 64) return SCD_ERR_ARG;
            p.xbytes = (int)xb;
            p.wbytes = (int)wb;
            // half a tile: ~KT x 32 MFMAs x 16 cycles x 2 workgroups sharing the matrix pipe / 2, at ~75 % of it, in
            // s_sleep(127) quanta of 8,128 cycles
            p.duo_ncu = num_cus();
            p.duo_delay = (int)((long)ktmax * 680 * duo_delay_pct() / 100 / 8128);
            hipLaunchKernelGGL(conv_gemm_duo_kernel, dim3(tiles), dim3(256), 0, (hipStream_t)stream, p);
            SCD_RETURN_LAUNCH();
        }
    }
    {
        // ping-pong 256 x BN kernel when the grid fills the chip (fused head tails are run as a separate pass)
        const int bn = pp_bn(dtype, p.Co);
        if (bn && (long)cdiv(Mtot, 256) * (p.Co / bn) >= 256) {
            p.ntn = p.Co / bn;
            int tiles = 0;
            for (int i = 0; i < SCD_MAX_PHASES; ++i) {
                p.tile_start[i] = tiles;
                if (i < nphase) {
                    p.ph[i] = phases[i];
                    tiles += cdiv((long)p.N * phases[i].Qh * phases[i].Qw, 256) * p.ntn;
                }
            }
            p.tile_start[SCD_MAX_PHASES] = tiles;
            const long wb = (long)p.Co * p.wrow * esz;
            if (xb >= (1L << 31) - 64 || wb >= (1L << 31) - 64) return SCD_ERR_ARG;
            p.xbytes = (int)xb;
            p.wbytes = (int)wb;
            const long yb = p.bnbwd ? (long)p.N * p.Ho * p.Wo * p.Co * esz : 0;
            if (yb >= (1L << 31) - 64) return SCD_ERR_ARG;
            p.ybytes = (int)yb;
            hipStream_t st = (hipStream_t)stream;
            if (p.head_on) {
                // heads split between two column tiles accumulate two partial sums: zero them first
                for (int h = 0; h < 4 && p.head_out[h]; ++h)
                    if ((h * 128) / bn != (h * 128 + 127) / bn) {
                        hipError_t e = hipMemsetAsync(p.head_out[h], 0, sizeof(float) * p.head_od[h] * (size_t)p.N * p.Ho * p.Wo, st);
                        if (e != hipSuccess) return (int)e;
                    }
                if (bn == 256) hipLaunchKernelGGL((conv_gemm_pp_kernel<256, true>), dim3(tiles), dim3(512), 0, st, p);
                else hipLaunchKernelGGL((conv_gemm_pp_kernel<192, true>), dim3(tiles), dim3(512), 0, st, p);
            } else if (p.bnbwd) {
                if (bn == 256) hipLaunchKernelGGL((conv_gemm_pp_kernel<256, false, true>), dim3(tiles), dim3(512), 0, st, p);
                else hipLaunchKernelGGL((conv_gemm_pp_kernel<192, false, true>), dim3(tiles), dim3(512), 0, st, p);
            } else {
                if (bn == 256) hipLaunchKernelGGL((conv_gemm_pp_kernel<256, false>), dim3(tiles), dim3(512), 0, st, p);
                else hipLaunchKernelGGL((conv_gemm_pp_kernel<192, false>), dim3(tiles), dim3(512), 0, st, p);
            }
            SCD_RETURN_LAUNCH();
        }
    }
    if (p.bnbwd && dtype != SCD_DT_BF16) return SCD_ERR_ARG;   // BN-backward sums: 16-bit epilogues (caller falls back)
    {
        // 3x3 / s1 / p1, 64 -> 64 channels on whole rows of 64, 128 or 256 pixels: the persistent row-ring kernel
        const int flip = halo64_taps(p, nphase, phases);
        if (dtype == SCD_DT_BF16 && flip >= 0 && halo64_mode() && !p.bias && !p.relu) {
            if (p.Wo == 256 && p.bnbwd) return SCD_ERR_ARG;    // scd_conv_gemm_bnbwd: this kernel + separate reduce
            p.ntn = 1;
            p.ph[0] = phases[0];
            for (int i = 0; i <= SCD_MAX_PHASES; ++i) p.tile_start[i] = 0;
            const long wb = (long)p.Co * p.wrow * esz;
            if (xb >= (1L << 31) - 64 || wb >= (1L << 31) - 64) return SCD_ERR_ARG;
            p.xbytes = (int)xb;
            p.wbytes = (int)wb;
            const int tiles = (int)(Mtot / 256);
            hipStream_t st = (hipStream_t)stream;
            // `run` tiles per workgroup down one image (about one workgroup per CU)
            const int tpi = p.Wo >= 256 ? p.Ho : p.Ho / (256 / p.Wo);
            int run = 1;
            while (run < 16 && tpi % (2 * run) == 0 && tiles / (2 * run) >= num_cus()) run *= 2;
            const int grid = tiles / run;
#define SCD_L1P_LAUNCH(WO)                                                                                              \
    do {                                                                                                                 \
        if (WO != 256 && p.bnbwd) {                                                                                      \
            if (flip) hipLaunchKernelGGL((conv_gemm_l1p_kernel<WO, true, WO != 256>), dim3(grid), dim3(512), 0, st, p, run); \
            else hipLaunchKernelGGL((conv_gemm_l1p_kernel<WO, false, WO != 256>), dim3(grid), dim3(512), 0, st, p, run);    \
        } else {                                                                                                         \
            if (flip) hipLaunchKernelGGL((conv_gemm_l1p_kernel<WO, true, false>), dim3(grid), dim3(512), 0, st, p, run);  \
            else hipLaunchKernelGGL((conv_gemm_l1p_kernel<WO, false, false>), dim3(grid), dim3(512), 0, st, p, run);     \
        }                                                                                                                \
    } while (0)
            if (p.Wo == 256) SCD_L1P_LAUNCH(256);
            else if (p.Wo == 128) SCD_L1P_LAUNCH(128);
            else SCD_L1P_LAUNCH(64);
#undef SCD_L1P_LAUNCH
            SCD_RETURN_LAUNCH();
        }
    }
    bool ring = false;
    if (dtype == SCD_DT_BF16 && !narrow) {
        const int rm = ring_mode();
        ring = rm >= 0 ? rm != 0 : cdiv(Mtot, 256) * cdiv(p.Co, 128) >= 256;   // >= one tile per CU
    } else if (dtype == SCD_DT_BF16 && narrow_ring_mode() && nphase == 1 && phases[0].ntaps == 1 && p.Ci >= 128 &&
               cdiv(Mtot, 256) >= 256) {
        // 1x1 convs into <= 64 channels over many pixels (the Bottleneck conv1 forward and conv3 input gradient at
        // Res50 1024^2, residuals.py:122-165): HBM-bound skinny GEMMs on the LDS-DMA ring kernel, half its 128-column
        // tile empty, instead of the register-staged 256 x 64 kernel
        ring = true;
    }
    const int BM = ring ? 256 : (narrow ? 256 : 128), BN = (narrow && !ring) ? 64 : 128;
    p.ntn = cdiv(p.Co, BN);
    int tiles = 0;
    for (int i = 0; i < SCD_MAX_PHASES; ++i) {
        p.tile_start[i] = tiles;
        if (i < nphase) {
            p.ph[i] = phases[i];
            tiles += cdiv((long)p.N * phases[i].Qh * phases[i].Qw, BM) * p.ntn;
        }
    }
    p.tile_start[SCD_MAX_PHASES] = tiles;
    if (tiles == 0) return 0;
    const long wb = (long)p.Co * p.wrow * esz;
    if (xb >= (1L << 31) - 64 || wb >= (1L << 31) - 64) return SCD_ERR_ARG;   // 32-bit buffer offsets
    p.xbytes = (int)xb;
    p.wbytes = (int)wb;
    hipStream_t st = (hipStream_t)stream;
    if (ring) {
        if (p.head_on) hipLaunchKernelGGL((conv_gemm_ring_kernel<true>), dim3(tiles), dim3(512), 0, st, p);
        else if (p.bnbwd) hipLaunchKernelGGL((conv_gemm_ring_kernel<false, true>), dim3(tiles), dim3(512), 0, st, p);
        else hipLaunchKernelGGL((conv_gemm_ring_kernel<false>), dim3(tiles), dim3(512), 0, st, p);
        SCD_RETURN_LAUNCH();
    }
    if (dtype == SCD_DT_BF16) {
        if (narrow) return launch_gemm<h16, 256, 64>(p, tiles, st);
        int ks = 1;
        const int km = ksplit_mode();
        if (km && !p.head_on) {
            int kt = 0;
            for (int i = 0; i < nphase; ++i) kt = std::max(kt, phases[i].ntaps * (p.Ci / 64));
            if (km == 2 || (kt >= 16 && 2 * (long)tiles <= 3L * num_cus())) ks = 2;
        }
        return launch_gemm<h16, 128, 128>(p, tiles, st, ks);
    }
    if (dtype == SCD_DT_F32)
        return narrow ? launch_gemm<float, 256, 64>(p, tiles, st) : launch_gemm<float, 128, 128>(p, tiles, st);
    return SCD_ERR_ARG;
}

static void fill_params(GemmParams& p, const void* x, const void* w, void* y, const float* bias, double* stats, int N,
                        int Hi, int Wi, int Ci, int Ho, int Wo, int Co, int in_stride, int out_stride, int wrow,
                        int relu, int accumulate) {
    p.x = (const char*)x; p.w = (const char*)w; p.y = (char*)y; p.bias = bias; p.stats = stats;
    p.N = N; p.Hi = Hi; p.Wi = Wi; p.Ci = Ci; p.Ho = Ho; p.Wo = Wo; p.Co = Co;
    p.is = in_stride; p.os = out_stride; p.wrow = wrow; p.relu = relu; p.accumulate = accumulate;
    p.ybytes = 0;
    p.head_on = 0;
    p.bnbwd = 0; p.bny = nullptr; p.bn_mean = p.bn_invstd = p.bn_rsc = p.bn_rsh = nullptr;
    p.hid_keep = nullptr; p.hid_cols = 1 << 30;
    p.shuf = 0;
    p.stamps = scd_calib_stamp_buffer;
    p.duo_ncu = 0; p.duo_delay = 0;
    {
        // read per call (tests switch them to compare the variants)
        const char* e = getenv("SCD_HEADS_SERP");
        p.kserp = e ? atoi(e) : 1;
    }
    {
        static int dbg = -1;
        if (dbg < 0) { const char* e = getenv("SCD_GEMM_DEBUG"); dbg = e ? atoi(e) : 0; }
        p.debug = dbg;
    }
    for (int h = 0; h < 4; ++h) { p.head_od[h] = 0; p.head_w[h] = nullptr; p.head_b[h] = nullptr; p.head_out[h] = nullptr; }
}

extern "C" int scd_conv_gemm(int dtype, const void* x, const void* w, void* y, const float* bias, double* stats,
                             int N, int Hi, int Wi, int Ci, int Ho, int Wo, int Co, int in_stride, int out_stride,
                             int wrow, int relu, int accumulate, int nphase, const scd_gemm_phase* phases,
                             void* stream) {
    SCD_F16_FWD(scd_conv_gemm, x, w, y, bias, stats, N, Hi, Wi, Ci, Ho, Wo, Co, in_stride, out_stride, wrow, relu,
                accumulate, nphase, phases, stream);
    GemmParams p;
    fill_params(p, x, w, y, bias, stats, N, Hi, Wi, Ci, Ho, Wo, Co, in_stride, out_stride, wrow, relu, accumulate);
    return conv_gemm_launch(dtype, p, nphase, phases, stream);
}

extern "C" int scd_conv_gemm_bnbwd(int dtype, const void* x, const void* w, void* y, int N, int Hi, int Wi, int Ci,
                                   int Ho, int Wo, int Co, int in_stride, int out_stride, int wrow, int nphase,
                                   const scd_gemm_phase* phases, const void* bn_y, const float* mean,
                                   const float* invstd, const float* relu_scale, const float* relu_shift,
                                   double* bn_stats, void* stream) {
    SCD_F16_FWD(scd_conv_gemm_bnbwd, x, w, y, N, Hi, Wi, Ci, Ho, Wo, Co, in_stride, out_stride, wrow, nphase, phases,
                bn_y, mean, invstd, relu_scale, relu_shift, bn_stats, stream);
    if (!bn_y || !mean || !invstd || !relu_scale || !relu_shift || !bn_stats || Co % 4) return SCD_ERR_ARG;
    GemmParams p;
    fill_params(p, x, w, y, nullptr, bn_stats, N, Hi, Wi, Ci, Ho, Wo, Co, in_stride, out_stride, wrow, 0, 0);
    p.bnbwd = 1;
    p.bny = (const char*)bn_y; p.bn_mean = mean; p.bn_invstd = invstd; p.bn_rsc = relu_scale; p.bn_rsh = relu_shift;
    if (dtype == SCD_DT_BF16) {
        const int rc = conv_gemm_launch(dtype, p, nphase, phases, stream);
        if (rc != SCD_ERR_ARG) return rc;
    }
    // shapes the fused-sum kernels do not take: plain GEMM, then the separate BN-backward reduction
    fill_params(p, x, w, y, nullptr, nullptr, N, Hi, Wi, Ci, Ho, Wo, Co, in_stride, out_stride, wrow, 0, 0);
    const int rc = conv_gemm_launch(dtype, p, nphase, phases, stream);
    if (rc) return rc;
    return scd_bn_bwd_reduce(dtype, y, nullptr, bn_y, relu_scale, relu_shift, mean, invstd, Co, (long)N * Ho * Wo * Co,
                             bn_stats, stream);
}

extern "C" int scd_conv_dgrad_s2(int dtype, const void* dy, const void* w3, void* dx, int N, int Hq, int Wq, int Cg,
                                 int Cin, int accumulate, void* stream) {
    SCD_F16_FWD(scd_conv_dgrad_s2, dy, w3, dx, N, Hq, Wq, Cg, Cin, accumulate, stream);
    // the input gradient of a 3x3 / stride 2 / pad 1 conv (dy: N x Hq x Wq x Cg -> dx: N x 2Hq x 2Wq x Cin) as a
    // forward 2x2-tap GEMM over dy whose 4 Cin output columns are the four sub-pixel phases (operand: pack mode 3);
    // only where the ping-pong kernel takes it (its epilogue stores the phases as pixels)
    const int Co = 4 * Cin;
    const long Mtot = (long)N * Hq * Wq;
    const int bn = pp_bn(dtype, Co);
    if (!bn || Cin % 8 || (long)cdiv(Mtot, 256) * (Co / bn) < 256) return SCD_ERR_ARG;
    GemmParams p;
    fill_params(p, dy, w3, dx, nullptr, nullptr, N, Hq, Wq, Cg, Hq, Wq, Co, 1, 1, 4 * Cg, 0, accumulate);
    p.shuf = 1;
    scd_gemm_phase ph;
    ph.Qh = Hq; ph.Qw = Wq; ph.rho_h = 0; ph.rho_w = 0; ph.ntaps = 4;
    for (int t = 0; t < 4; ++t) { ph.dh[t] = t >> 1; ph.dw[t] = t & 1; ph.wt[t] = t; }
    return conv_gemm_launch(dtype, p, 1, &ph, stream);
}

extern "C" int scd_conv_gemm_heads(int dtype, const void* x, const void* w, void* hid, const float* bias, int N,
                                   int H, int W, int Ci, int nh, const int* od, const float* const* w1,
                                   const float* const* b1, float* const* outs, void* stream) {
    SCD_F16_FWD(scd_conv_gemm_heads, x, w, hid, bias, N, H, W, Ci, nh, od, w1, b1, outs, stream);
    return scd_conv_gemm_heads_keep(dtype, x, w, hid, bias, N, H, W, Ci, nh, od, w1, b1, outs, nullptr, 0, stream);
}

extern "C" int scd_conv_gemm_heads_keep(int dtype, const void* x, const void* w, void* hid, const float* bias, int N,
                                        int H, int W, int Ci, int nh, const int* od, const float* const* w1,
                                        const float* const* b1, float* const* outs, const unsigned char* keep,
                                        int keep_cols, void* stream) {
    SCD_F16_FWD(scd_conv_gemm_heads_keep, x, w, hid, bias, N, H, W, Ci, nh, od, w1, b1, outs, keep, keep_cols, stream);
    if (nh < 1 || nh > 4 || (keep && (keep_cols < 0 || keep_cols % 128))) return SCD_ERR_ARG;
    GemmParams p;
    fill_params(p, x, w, hid, bias, nullptr, N, H, W, Ci, H, W, nh * 128, 1, 1, 9 * Ci, 1, 0);
    if (keep) { p.hid_keep = keep; p.hid_cols = keep_cols; }
    p.head_on = 1;
    for (int h = 0; h < nh; ++h) {
        if (od[h] < 1 || od[h] > 4) return SCD_ERR_ARG;
        p.head_od[h] = od[h]; p.head_w[h] = w1[h]; p.head_b[h] = b1[h]; p.head_out[h] = outs[h];
    }
    scd_gemm_phase ph;
    ph.Qh = H; ph.Qw = W; ph.rho_h = 0; ph.rho_w = 0; ph.ntaps = 9;
    for (int t = 0; t < 9; ++t) { ph.dh[t] = t / 3 - 1; ph.dw[t] = t % 3 - 1; ph.wt[t] = t; }
    return conv_gemm_launch(dtype, p, 1, &ph, stream);
}

extern "C" size_t scd_conv_wgrad_workspace(int Cg, int T, int Ci, int nsplit) {
    return (size_t)nsplit * Cg * T * Ci * sizeof(float);
}

static bool wgrad_fastx() {
    static int mode = -2;
    if (mode == -2) { const char* e = getenv("SCD_WGRAD_FASTX"); mode = e ? atoi(e) : 1; }
    return mode != 0;
}

static void wgrad_tile(int dtype, long M, int Cg, int& tm, int& tn) {
    (void)dtype; (void)M;
    if (Cg <= 64) { tm = 64; tn = 256; }
    else { tm = 128; tn = 128; }
}

// the 64-pixel ping-pong weight gradient: bf16, a stage inside one output row, at least one 256-channel window
static bool wgrad_use_pp2(int dtype, long M, int Ho, int Wo, int Cg) {
    static int mode = -2;
    if (mode == -2) { const char* e = getenv("SCD_WGRAD_PP2"); mode = e ? atoi(e) : 1; }
    // a stage = 64 pixels of one output row, or 64 / Wo whole rows (Wo = 16, 32: layer3/4, deconv1/2)
    const bool stage_ok = Wo % 64 == 0 || (Wo >= 8 && 64 % Wo == 0);
    return mode && dtype == SCD_DT_BF16 && Cg >= 128 && stage_ok && ((long)Ho * Wo) % 64 == 0 && M >= 64 * 64;
}

// the layer1 weight gradient (conv_wgrad_l1_kernel): bf16, 64 -> 64 channels, 3x3 taps, stages inside one row
static bool wgrad_use_l1(int dtype, long M, int Ho, int Wo, int Cg, int T, int Ci) {
    static int mode = -2;
    if (mode == -2) { const char* e = getenv("SCD_WGRAD_L1"); mode = e ? atoi(e) : 1; }
    return mode && dtype == SCD_DT_BF16 && Cg == 64 && Ci == 64 && T == 9 && Wo % 64 == 0 && M % 64 == 0 &&
           (long)Ho * Wo * 64 <= (1L << 30) && M >= 64;
}

// >= 16 stages per workgroup, at most 192 workgroups (SCD_WGRAD_L1_NSPLIT): in the step this kernel shares the chip
// with the compute stream's last layer1 / stem kernels, and fewer splits shrink its 64 x 576 fp32 slab reduce
// (round 4: 128 measured +1% per step against 256; round 5: 192 +0.3% against 128 in 8 of 8 A/B pairs on two boxes,
// profiles/r5_ab.txt)
static int wgrad_l1_nsplit(long M) {
    static long cap = -2;
    if (cap == -2) { const char* e = getenv("SCD_WGRAD_L1_NSPLIT"); cap = e ? atol(e) : 192; }
    return (int)std::max(1L, std::min(cap, M / 64 / 16));
}

// channel window of the ping-pong weight gradient: 256 (NQ 4) or, for widths that are multiples of 192 only, 192
static int wgrad_pp2_win(int Cg) {
    if (Cg % 256 == 0) return 256;
    if (Cg % 192 == 0) return 192;
    return Cg < 256 ? 128 : 256;           // 128: NQ 2 (the heatmap head, layer2); else 256 windows + a remainder
}

// split count from a wave-quantisation cost model (SCD_WGRAD_NSMODEL=0: the fixed rules below it).  A launch of
// tiles x ns workgroups runs in ceil(tiles*ns / slots) rounds; a round costs its K stages (stage_us each) plus the
// workgroup's fp32 slab store (epi_us), and every split adds one slab to the reduce, priced at 0.8 TB/s
// (SCD_WGRAD_SLAB_TBPS): the reduce reads ~3.5 TB/s alone but a fraction of that inside the step, beside the compute
// stream's BN passes; pricing it at 3.5 measured 1% slower per step.  Candidates are whole XCD groups (multiples of
// 8) within the pixel and slab-memory caps.
static bool wgrad_nsmodel() {
    static int mode = -2;
    if (mode == -2) { const char* e = getenv("SCD_WGRAD_NSMODEL"); mode = e ? atoi(e) : 1; }
    return mode != 0;
}

static long wgrad_ns_model(long M, long tiles, int slots, int kp, double stage_us, double epi_us, double slab_bytes,
                           long ns_max, bool any_ns = false) {
    static double slab_rate = -1.0;          // bytes/us at which the reduce reads the slabs (SCD_WGRAD_SLAB_TBPS)
    if (slab_rate < 0) { const char* e = getenv("SCD_WGRAD_SLAB_TBPS"); slab_rate = (e ? atof(e) : 0.8) * 1e6; }
    long best = 8;
    double bt = 1e30;
    const long step = any_ns ? 1 : 8;
    for (long ns = step; ns <= std::max(8L, ns_max); ns += step) {
        const long stages = cdiv(cdiv(M, ns), (long)kp);
        const long rounds = cdiv(tiles * ns, (long)slots);
        const double t = rounds * (stages * stage_us + epi_us) + ns * slab_bytes / slab_rate;
        if (t < bt * 0.995) { bt = t; best = ns; }
    }
    return best;
}

static int wgrad_pp2_nsplit(long M, int Cg, int KK) {
    const int win = wgrad_pp2_win(Cg);
    const long tiles = (long)(Cg / win) * cdiv(KK, 256);
    // >= 8 stages per split (small layers need many splits to fill the chip: layer3 has 32 K pixels)
    const long cap_px = std::max(8L, M / 512 / 8 * 8);
    const long cap_mem = std::max(8L, (256L << 20) / std::max(1L, 4L * Cg * KK) / 8 * 8);
    if (wgrad_nsmodel()) {
        // one workgroup per CU; a 64-pixel stage ~ 2*win*256*64 flop at ~4.3 TF/s per CU; slab win x 256 fp32
        const double stage_us = 2.0 * win * 256 * 64 / 4.3e6;
        const double epi_us = 4.0 * win * 256 / (5.0e6 / 256);
        // many tiles: splits need not come in XCD groups of 8 (wgrad_block's linear map), so one round can be filled
        // slots: the CUs the model fills (SCD_WGRAD_SLOTS, read once; A/B of leaving CUs to the compute stream)
        static int slots = -1;
        if (slots < 0) { const char* e = getenv("SCD_WGRAD_SLOTS"); slots = e ? std::max(8, atoi(e)) : 256; }
        const long ns = wgrad_ns_model(M, tiles, slots, 64, stage_us, epi_us, 4.0 * Cg * KK, std::min(cap_px, cap_mem),
                                       tiles >= 24);
        return (int)ns;
    }
    // about two rounds of one-per-CU workgroups over the channel windows, whole XCD groups, >= 2048 pixels
    // per split, fp32 slabs capped at 256 MB
    long ns = std::max(8L, (512L / tiles + 4) / 8 * 8);
    ns = std::min(ns, cap_px);
    ns = std::min(ns, cap_mem);
    return (int)ns;
}

extern "C" int scd_conv_wgrad_nsplit2(int dtype, long M, int Ho, int Wo, int Cg, int T, int Ci) {
    SCD_F16_FWD(scd_conv_wgrad_nsplit2, M, Ho, Wo, Cg, T, Ci);
    if (wgrad_use_l1(dtype, M, Ho, Wo, Cg, T, Ci)) return wgrad_l1_nsplit(M);
    if (wgrad_use_pp2(dtype, M, Ho, Wo, Cg)) return wgrad_pp2_nsplit(M, Cg, T * Ci);
    return scd_conv_wgrad_nsplit(dtype, M, Cg, T, Ci);
}

extern "C" int scd_conv_wgrad_nsplit(int dtype, long M, int Cg, int T, int Ci) {
    SCD_F16_FWD(scd_conv_wgrad_nsplit, M, Cg, T, Ci);
    int tm, tn;
    wgrad_tile(dtype, M, Cg, tm, tn);
    const long tiles = (long)cdiv(Cg, tm) * cdiv((long)T * Ci, tn);
    // ~4 waves of two-per-CU workgroups over 256 CUs, >= 1024 pixels per split, fp32 slabs capped at 256 MB
    if (wgrad_nsmodel() && M >= 8 * 1024) {
        // 128x128: two workgroups per CU, 64x256: one (register-bound); a stage of KP pixels ~ 2*tm*tn*KP flop
        // at ~2.4 TF/s per CU; slab tm x tn fp32
        const int KP = dtype == SCD_DT_BF16 ? 64 : 32;
        const int slots = tm == 64 ? 256 : 512;
        const double stage_us = 2.0 * tm * tn * KP / (2.4e6 * 256 / slots);
        const double epi_us = 4.0 * tm * tn / (5.0e6 / slots);
        const long cap_px = std::max(8L, M / 1024 / 8 * 8);
        const long cap_mem = std::max(8L, (256L << 20) / std::max(1L, 4L * Cg * T * Ci) / 8 * 8);
        const long ns = wgrad_ns_model(M, tiles, slots, KP, stage_us, epi_us, 4.0 * Cg * T * Ci,
                                       std::min(cap_px, cap_mem));
        return (int)ns;
    }
    long ns = std::max(1L, std::min(1024L / std::max(1L, tiles), M / 1024));
    ns = std::max(1L, std::min(ns, (256L << 20) / std::max(1L, 4L * Cg * T * Ci)));
    if (ns >= 8) ns = ns / 8 * 8;          // whole XCD groups (see wgrad_block)
    return (int)ns;
}

extern "C" int scd_conv_wgrad(int dtype, const void* g, const void* x, float* ws, int nsplit, int N, int Ho, int Wo,
                              int Cg, int Hi, int Wi, int Ci, int in_stride, int T, const int* dh, const int* dw,
                              void* stream) {
    SCD_F16_FWD(scd_conv_wgrad, g, x, ws, nsplit, N, Ho, Wo, Cg, Hi, Wi, Ci, in_stride, T, dh, dw, stream);
    const int EPC = dtype == SCD_DT_BF16 ? 8 : 4;
    if (T < 1 || T > SCD_MAX_TAPS || Ci % EPC != 0 || Cg % EPC != 0 || nsplit < 1) return SCD_ERR_ARG;
    WgradParams p;
    p.g = (const char*)g; p.x = (const char*)x; p.ws = ws;
    p.N = N; p.Ho = Ho; p.Wo = Wo; p.Cg = Cg; p.Hi = Hi; p.Wi = Wi; p.Ci = Ci; p.is = in_stride; p.T = T;
    p.cg0 = 0; p.cgn = Cg;
    p.KK = T * Ci;
    {
        const int esz = dtype == SCD_DT_BF16 ? 2 : 4;
        const long gb = (long)N * Ho * Wo * Cg * esz, xb = (long)N * Hi * Wi * Ci * esz;
        if (gb >= (1L << 31) - 64 || xb >= (1L << 31) - 64) return SCD_ERR_ARG;
        p.gbytes = (int)gb;
        p.xbytes = (int)xb;
    }
    for (int t = 0; t < SCD_MAX_TAPS; ++t) { p.dh[t] = t < T ? dh[t] : 0; p.dw[t] = t < T ? dw[t] : 0; }
    const long M = (long)N * Ho * Wo;
    int chunk = cdiv(M, nsplit);
    chunk = (chunk + 63) / 64 * 64;
    p.chunk = chunk;
    if (wgrad_use_l1(dtype, M, Ho, Wo, Cg, T, Ci) && in_stride == 1 && Hi == Ho && Wi == Wo) {
        bool std_taps = true;        // taps (t / 3 - 1, t % 3 - 1): the halo row of tap t (conv_wgrad_l1_kernel)
        for (int t = 0; t < 9; ++t) std_taps &= dh[t] == t / 3 - 1 && dw[t] == t % 3 - 1;
        if (std_taps) {
            p.nsplit = nsplit;
            hipLaunchKernelGGL(conv_wgrad_l1_kernel, dim3(nsplit), dim3(512), 0, (hipStream_t)stream, p);
            SCD_RETURN_LAUNCH();
        }
    }
    if (wgrad_use_pp2(dtype, M, Ho, Wo, Cg) && chunk % 64 == 0) {
        // 256-channel windows on the ping-pong kernel, a remainder on the register-staged one
        hipStream_t st = (hipStream_t)stream;
        p.ntn = cdiv(p.KK, 256);
        p.nsplit = nsplit;
        const int n8 = nsplit;          // whole XCD groups of splits, or the linear map (wgrad_block)
        const int win = wgrad_pp2_win(Cg);
        p.cg0 = 0;
        p.cgn = Cg / win * win;
        p.ntm = Cg / win;
        if (win == 256) hipLaunchKernelGGL((conv_wgrad_pp2_kernel<4>), dim3(p.ntm * p.ntn * n8), dim3(512), 0, st, p);
        else if (win == 192) hipLaunchKernelGGL((conv_wgrad_pp2_kernel<3>), dim3(p.ntm * p.ntn * n8), dim3(512), 0, st, p);
        else hipLaunchKernelGGL((conv_wgrad_pp2_kernel<2>), dim3(p.ntm * p.ntn * n8), dim3(512), 0, st, p);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess || Cg % win == 0) return (int)e;
        p.cg0 = Cg / win * win;
        p.cgn = Cg % win;
        int BM, BN;
        wgrad_tile(dtype, M, p.cgn, BM, BN);
        p.ntm = cdiv(p.cgn, BM);
        p.ntn = cdiv(p.KK, BN);
        // stages of one row (FASTX 1, Wo % 64 == 0) or of whole rows (FASTX 2, 64 % Wo == 0; 64 x 256 tile only)
        const int fx = !(wgrad_fastx() && ((long)Ho * Wo) % 64 == 0) ? 0 : (Wo % 64 == 0 ? 1 : 2);
        dim3 grid(p.ntm * p.ntn * n8);
        if (BM == 64) {
            if (fx == 1) hipLaunchKernelGGL((conv_wgrad_kernel<h16, 64, 256, 1>), grid, dim3(256), 0, st, p);
            else if (fx == 2) hipLaunchKernelGGL((conv_wgrad_kernel<h16, 64, 256, 2>), grid, dim3(256), 0, st, p);
            else hipLaunchKernelGGL((conv_wgrad_kernel<h16, 64, 256, 0>), grid, dim3(256), 0, st, p);
        } else {
            if (fx == 1) hipLaunchKernelGGL((conv_wgrad_kernel<h16, 128, 128, 1>), grid, dim3(256), 0, st, p);
            else hipLaunchKernelGGL((conv_wgrad_kernel<h16, 128, 128, 0>), grid, dim3(256), 0, st, p);
        }
        SCD_RETURN_LAUNCH();
    }
    int BM, BN;
    wgrad_tile(dtype, M, Cg, BM, BN);
    p.ntm = cdiv(Cg, BM);
    p.ntn = cdiv(p.KK, BN);
    p.nsplit = nsplit;
    dim3 grid(p.ntm * p.ntn * nsplit);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == SCD_DT_BF16 || dtype == SCD_DT_F32) {
        // fast addressing when a stage of KP pixels stays inside one image and one row block
        const int KP = dtype == SCD_DT_BF16 ? 64 : 32;
        const bool fastok = wgrad_fastx() && ((long)Ho * Wo) % KP == 0 && chunk % KP == 0;
        const int fx = !fastok ? 0 : (Wo % KP == 0 ? 1 : (KP % Wo == 0 ? 2 : 0));
        // (the 128 x 128 tile has registers for FASTX 1 only)
        if (dtype == SCD_DT_BF16) {
            if (Cg <= 64) {
                if (fx == 1) hipLaunchKernelGGL((conv_wgrad_kernel<h16, 64, 256, 1>), grid, dim3(256), 0, st, p);
                else if (fx == 2) hipLaunchKernelGGL((conv_wgrad_kernel<h16, 64, 256, 2>), grid, dim3(256), 0, st, p);
                else hipLaunchKernelGGL((conv_wgrad_kernel<h16, 64, 256, 0>), grid, dim3(256), 0, st, p);
            } else {
                if (fx == 1) hipLaunchKernelGGL((conv_wgrad_kernel<h16, 128, 128, 1>), grid, dim3(256), 0, st, p);
                else hipLaunchKernelGGL((conv_wgrad_kernel<h16, 128, 128, 0>), grid, dim3(256), 0, st, p);
            }
        } else {
            if (Cg <= 64) {
                if (fx == 1) hipLaunchKernelGGL((conv_wgrad_kernel<float, 64, 256, 1>), grid, dim3(256), 0, st, p);
                else if (fx == 2) hipLaunchKernelGGL((conv_wgrad_kernel<float, 64, 256, 2>), grid, dim3(256), 0, st, p);
                else hipLaunchKernelGGL((conv_wgrad_kernel<float, 64, 256, 0>), grid, dim3(256), 0, st, p);
            } else {
                if (fx == 1) hipLaunchKernelGGL((conv_wgrad_kernel<float, 128, 128, 1>), grid, dim3(256), 0, st, p);
                else hipLaunchKernelGGL((conv_wgrad_kernel<float, 128, 128, 0>), grid, dim3(256), 0, st, p);
            }
        }
    } else {
        return SCD_ERR_ARG;
    }
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_wgrad_reduce_rows(const float* ws, int nsplit, int Cg, int T, int Ci, int nslices, const int* r0,
                                     const int* r1, const long* ld_n, const long* ld_c, const long* ld_t,
                                     float* const* dst, int cvalid, int accumulate, float alpha, void* stream) {
    if (nslices < 1 || nslices > 4 || nsplit < 1 || Ci % 4 != 0 || T < 1 || T > 64) return SCD_ERR_ARG;
    WredSlices sl;
    sl.n = nslices;
    long rows = 0;
    for (int s = 0; s < nslices; ++s) {
        if (r0[s] < 0 || r1[s] > Cg || r0[s] >= r1[s] || dst[s] == nullptr) return SCD_ERR_ARG;
        sl.r0[s] = r0[s]; sl.r1[s] = r1[s];
        sl.ldn[s] = ld_n[s]; sl.ldc[s] = ld_c[s]; sl.ldt[s] = ld_t[s];
        sl.dst[s] = dst[s];
        rows += r1[s] - r0[s];
    }
    const long zs = (long)Cg * T * Ci;
    // channel chunk: the widest (<= 128) that still gives >= 1024 workgroups (few rows x many splits, e.g. the
    // 64-row layer1 gradient over 256 splits, would otherwise leave the reduce latency-bound on 64 workgroups)
    int cb = WRED_CB;
    while (cb > 16 && rows * cdiv(Ci, cb) < 512) cb >>= 1;
    const int ncb = cdiv(Ci, cb);
    const int units = T * (std::min(cb, Ci) / 4);
    // split groups per unit: every thread keeps >= 8 slab loads to itself, up to 256 threads per block
    const int S = std::max(1, std::min(256 / std::max(1, units), nsplit / 8));
    const int threads = (int)std::min(256L, ((long)units * S + 63) / 64 * 64);
    const size_t lds = (size_t)((T * (cb + 1) + 3) & ~3) * sizeof(float) + (S > 1 ? (size_t)S * units * 16 : 0);
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)(rows * ncb)), dim3(threads), lds, (hipStream_t)stream, ws,
                       nsplit, zs, T, Ci, cvalid, sl, ncb, cb, S, accumulate, alpha);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_wgrad_reduce(const float* ws, int nsplit, int Cg, int T, int Ci, int r0, int r1, int cvalid,
                                long ld_n, long ld_c, long ld_t, float* dst, int accumulate, float alpha,
                                void* stream) {
    return scd_wgrad_reduce_rows(ws, nsplit, Cg, T, Ci, 1, &r0, &r1, &ld_n, &ld_c, &ld_t, &dst, cvalid, accumulate,
                                 alpha, stream);
}
