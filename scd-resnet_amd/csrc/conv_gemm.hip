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
#include "scd_common.h"

namespace {

constexpr int LDS_ROW = 144;   // 128 B of K + 16 B pad

struct GemmParams {
    const char* x;
    const char* w;
    char* y;
    const float* bias;
    double* stats;
    int N, Hi, Wi, Ci, Ho, Wo, Co;
    int is, os, wrow, relu, accumulate, nphase, ntn;
    int tile_start[SCD_MAX_PHASES + 1];
    scd_gemm_phase ph[SCD_MAX_PHASES];
};

template <typename T, int BM, int BN>
__global__ __launch_bounds__(256) void conv_gemm_kernel(GemmParams p) {
    constexpr int ESZ = sizeof(T);
    constexpr int EPC = 16 / ESZ;       // elements per 16-B chunk
    constexpr int BK = 128 / ESZ;       // K elements per stage
    constexpr int ACH = BM / 32;        // A chunks per thread
    constexpr int BCH = BN / 32;
    constexpr int WN = BN / 64;         // waves along N (each wave: 64x64)
    __shared__ __attribute__((aligned(16))) char smem[2 * (BM + BN) * LDS_ROW];

    const int tid = threadIdx.x;
    int bid = blockIdx.x;
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
    int a_pix[ACH], a_ih[ACH], a_iw[ACH];
    bool a_ok[ACH];
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
        int m = mt * BM + (tid >> 3) + 32 * i;
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
        int nn = nt * BN + (tid >> 3) + 32 * j;
        b_ok[j] = nn < p.Co;
        b_row[j] = b_ok[j] ? nn : 0;
    }
    const int cpt = p.Ci / BK;            // K stages per tap
    const int KT = ph.ntaps * cpt;

    uint4 ra[ACH], rb[BCH];
    auto gload = [&](int kt) {
        int tap = kt / cpt;
        int c0 = (kt - tap * cpt) * BK + cch * EPC;
        int dh = ph.dh[tap], dw = ph.dw[tap], wt = ph.wt[tap];
#pragma unroll
        for (int i = 0; i < ACH; ++i) {
            int ih = a_ih[i] + dh, iw = a_iw[i] + dw;
            bool ok = a_ok[i] && (unsigned)ih < (unsigned)p.Hi && (unsigned)iw < (unsigned)p.Wi;
            long off = ((long)(a_pix[i] + ih * p.Wi + iw) * p.Ci + c0) * ESZ;
            ra[i] = ok ? *(const uint4*)(p.x + off) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < BCH; ++j) {
            long off = ((long)b_row[j] * p.wrow + (long)wt * p.Ci + c0) * ESZ;
            rb[j] = b_ok[j] ? *(const uint4*)(p.w + off) : make_uint4(0, 0, 0, 0);
        }
    };
    auto lstore = [&](int buf) {
        char* As = smem + buf * (BM + BN) * LDS_ROW;
        char* Bs = As + BM * LDS_ROW;
#pragma unroll
        for (int i = 0; i < ACH; ++i) *(uint4*)(As + ((tid >> 3) + 32 * i) * LDS_ROW + cch * 16) = ra[i];
#pragma unroll
        for (int j = 0; j < BCH; ++j) *(uint4*)(Bs + ((tid >> 3) + 32 * j) * LDS_ROW + cch * 16) = rb[j];
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
        const char* As = smem + buf * (BM + BN) * LDS_ROW;
        const char* Bs = As + BM * LDS_ROW;
        if constexpr (ESZ == 2) {
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                bf16x8 af[4], bfr[4];
#pragma unroll
                for (int a = 0; a < 4; ++a)
                    af[a] = *(const bf16x8*)(As + (wm * 64 + a * 16 + l16) * LDS_ROW + s * 64 + lg * 16);
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    bfr[b] = *(const bf16x8*)(Bs + (wn * 64 + b * 16 + l16) * LDS_ROW + s * 64 + lg * 16);
#pragma unroll
                for (int a = 0; a < 4; ++a)
#pragma unroll
                    for (int b = 0; b < 4; ++b)
                        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
            }
        } else {
            // exact-f32 MFMA: lane group lg owns K elements [8lg, 8lg+8) of the 32-wide stage;
            // step j multiplies element 8lg+j of A and B (same permutation on both operands).
            float4 af[4][2], bfr[4][2];
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                const char* pa = As + (wm * 64 + a * 16 + l16) * LDS_ROW + lg * 32;
                af[a][0] = *(const float4*)pa;
                af[a][1] = *(const float4*)(pa + 16);
            }
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const char* pb = Bs + (wn * 64 + b * 16 + l16) * LDS_ROW + lg * 32;
                bfr[b][0] = *(const float4*)pb;
                bfr[b][1] = *(const float4*)(pb + 16);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    float av = (j < 4) ? af[a][0][j & 3] : af[a][1][j & 3];
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        float bv = (j < 4) ? bfr[b][0][j & 3] : bfr[b][1][j & 3];
                        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[a][b], 0, 0, 0);
                    }
                }
            }
        }
    };

    if (KT > 0) {
        gload(0);
        lstore(0);
        __syncthreads();
        for (int kt = 0; kt < KT; ++kt) {
            const int cur = kt & 1;
            if (kt + 1 < KT) gload(kt + 1);
            compute(cur);
            if (kt + 1 < KT) lstore(cur ^ 1);
            __syncthreads();
        }
    }

    // ---- epilogue: bias / relu / accumulate, NHWC store at the phase's output pixel
    float csum[4], csq[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) { csum[b] = 0.f; csq[b] = 0.f; }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = mt * BM + wm * 64 + a * 16 + lg * 4 + r;
            if (m >= M) continue;
            const int n = m / QQ;
            const int rem = m - n * QQ;
            const int qh = rem / ph.Qw;
            const int qw = rem - qh * ph.Qw;
            const int oh = p.os * qh + ph.rho_h, ow = p.os * qw + ph.rho_w;
            const long obase = ((long)(n * p.Ho + oh) * p.Wo + ow) * p.Co;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int col = nt * BN + wn * 64 + b * 16 + l16;
                if (col >= p.Co) continue;
                float v = acc[a][b][r];
                if (p.bias) v += p.bias[col];
                if (p.relu) v = fmaxf(v, 0.f);
                T* dst = (T*)(p.y) + obase + col;
                if (p.accumulate) v += to_f<T>(*dst);
                *dst = from_f<T>(v);
                csum[b] += v;
                csq[b] += v * v;
            }
        }
    }
    if (p.stats) {
        // reduce over the 4 lane groups sharing a column, then over the waves sharing it
        __syncthreads();
        float* red = (float*)smem;   // [BM/64][BN][2]
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            float s = csum[b], q = csq[b];
            s += __shfl_xor(s, 16, 64); s += __shfl_xor(s, 32, 64);
            q += __shfl_xor(q, 16, 64); q += __shfl_xor(q, 32, 64);
            if (lg == 0) {
                red[(wm * BN + wn * 64 + b * 16 + l16) * 2 + 0] = s;
                red[(wm * BN + wn * 64 + b * 16 + l16) * 2 + 1] = q;
            }
        }
        __syncthreads();
        if (tid < BN) {
            const int col = nt * BN + tid;
            if (col < p.Co) {
                double s = 0.0, q = 0.0;
#pragma unroll
                for (int w = 0; w < BM / 64; ++w) { s += red[(w * BN + tid) * 2]; q += red[(w * BN + tid) * 2 + 1]; }
                const int rep = (bid % SCD_STAT_REPLICAS);
                atomic_add_f64(p.stats + ((long)rep * 2 + 0) * p.Co + col, s);
                atomic_add_f64(p.stats + ((long)rep * 2 + 1) * p.Co + col, q);
            }
        }
    }
}

// -------------------------------------------------------------------------------------
// weight gradient: ws[z][co][t*Ci+ci] = sum_pix g[pix][co] * x[gather(pix,t)][ci]
struct WgradParams {
    const char* g;
    const char* x;
    float* ws;
    int N, Ho, Wo, Cg, Hi, Wi, Ci, is, T, KK, chunk, ntm, ntn;
    int dh[SCD_MAX_TAPS], dw[SCD_MAX_TAPS];
};

template <typename T, int BM, int BN>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgradParams p) {
    constexpr int ESZ = sizeof(T);
    constexpr int EPC = 16 / ESZ;
    constexpr int KP = 32;                               // pixels per stage
    constexpr int GROW = BM * ESZ + 16;                  // LDS row bytes (pixel rows)
    constexpr int XROW = BN * ESZ + 16;
    constexpr int GCPR = BM * ESZ / 16;                  // chunks per G row
    constexpr int XCPR = BN * ESZ / 16;
    constexpr int GCH = KP * GCPR / 256;                 // chunks per thread
    constexpr int XCH = KP * XCPR / 256;
    constexpr int WN = BN / 64;
    __shared__ __attribute__((aligned(16))) char smem[2 * KP * (GROW + XROW)];

    const int tid = threadIdx.x;
    const int z = blockIdx.z;
    const int mt = blockIdx.x / p.ntn;
    const int nt = blockIdx.x - mt * p.ntn;
    const int M = p.N * p.Ho * p.Wo;
    const int pix0 = z * p.chunk;
    const int pix1 = min(M, pix0 + p.chunk);
    const int HoWo = p.Ho * p.Wo;

    // G loads: fixed channel chunk per thread
    const int gc = tid % GCPR;
    const int gr0 = tid / GCPR;
    const int gcol = mt * BM + gc * EPC;
    const bool gcol_ok = gcol < p.Cg;
    // X loads: fixed (tap, ci) chunk per thread
    const int xc = tid % XCPR;
    const int xr0 = tid / XCPR;
    const int kk = nt * BN + xc * EPC;
    const bool kk_ok = kk < p.KK;
    const int tap = kk_ok ? kk / p.Ci : 0;
    const int ci = kk - tap * p.Ci;
    const int dh = p.dh[tap], dw = p.dw[tap];

    uint4 rg[GCH], rx[XCH];
    auto gload = [&](int k0) {
#pragma unroll
        for (int i = 0; i < GCH; ++i) {
            int pix = k0 + gr0 + i * (256 / GCPR);
            bool ok = gcol_ok && pix < pix1;
            rg[i] = ok ? *(const uint4*)(p.g + ((long)pix * p.Cg + gcol) * ESZ) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < XCH; ++i) {
            int pix = k0 + xr0 + i * (256 / XCPR);
            bool ok = kk_ok && pix < pix1;
            int n = pix / HoWo;
            int rem = pix - n * HoWo;
            int oh = rem / p.Wo;
            int ow = rem - oh * p.Wo;
            int ih = p.is * oh + dh, iw = p.is * ow + dw;
            ok = ok && (unsigned)ih < (unsigned)p.Hi && (unsigned)iw < (unsigned)p.Wi;
            long off = ((long)((n * p.Hi + ih) * p.Wi + iw) * p.Ci + ci) * ESZ;
            rx[i] = ok ? *(const uint4*)(p.x + off) : make_uint4(0, 0, 0, 0);
        }
    };
    auto lstore = [&](int buf) {
        char* Gs = smem + buf * KP * (GROW + XROW);
        char* Xs = Gs + KP * GROW;
#pragma unroll
        for (int i = 0; i < GCH; ++i) *(uint4*)(Gs + (gr0 + i * (256 / GCPR)) * GROW + gc * 16) = rg[i];
#pragma unroll
        for (int i = 0; i < XCH; ++i) *(uint4*)(Xs + (xr0 + i * (256 / XCPR)) * XROW + xc * 16) = rx[i];
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
        const char* Gs = smem + buf * KP * (GROW + XROW);
        const char* Xs = Gs + KP * GROW;
        if constexpr (ESZ == 2) {
            // ds_read_b64_tr_b16: lane 4q+p of 16-lane group lg supplies row (8lg+q[+4]),
            // columns c0+4p..4p+3; lane i of the group receives column c0+i, 4 rows.
            const int q = l16 >> 2, pp = l16 & 3;
            bf16x8 af[4], bfr[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                const char* base = Gs + (8 * lg + q) * GROW + (wm * 64 + a * 16 + 4 * pp) * 2;
                s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base));
                s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + 4 * GROW));
                typedef __attribute__((ext_vector_type(8))) short s16x8;
                s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                af[a] = __builtin_bit_cast(bf16x8, v);
            }
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const char* base = Xs + (8 * lg + q) * XROW + (wn * 64 + b * 16 + 4 * pp) * 2;
                s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base));
                s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + 4 * XROW));
                typedef __attribute__((ext_vector_type(8))) short s16x8;
                s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                bfr[b] = __builtin_bit_cast(bf16x8, v);
            }
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
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
        gload(pix0);
        lstore(0);
        __syncthreads();
        for (int it = 0; it < nk; ++it) {
            const int cur = it & 1;
            if (it + 1 < nk) gload(pix0 + (it + 1) * KP);
            compute(cur);
            if (it + 1 < nk) lstore(cur ^ 1);
            __syncthreads();
        }
    }
    // ---- store fp32 partial tile: rows = Cg channel, cols = kk
    float* ws = p.ws + (long)z * p.Cg * p.KK;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = mt * BM + wm * 64 + a * 16 + lg * 4 + r;
            if (row >= p.Cg) continue;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int col = nt * BN + wn * 64 + b * 16 + l16;
                if (col < p.KK) ws[(long)row * p.KK + col] = acc[a][b][r];
            }
        }
}

__global__ void wgrad_reduce_kernel(const float* ws, int nsplit, int Cg, int T, int Ci, int r0, int r1, int cvalid,
                                    long ld_n, long ld_c, long ld_t, float* dst, int accumulate) {
    const long KK = (long)T * Ci;
    const long total = (long)(r1 - r0) * KK;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int r = (int)(i / KK);
        const int k = (int)(i - r * KK);
        const int t = k / Ci;
        const int c = k - t * Ci;
        if (c >= cvalid) continue;
        float s = 0.f;
        const float* src = ws + (long)(r0 + r) * KK + k;
        for (int z = 0; z < nsplit; ++z) s += src[(long)z * Cg * KK];
        float* d = dst + r * ld_n + c * ld_c + t * ld_t;
        *d = accumulate ? (*d + s) : s;
    }
}

template <typename T, int BM, int BN>
int launch_gemm(GemmParams& p, int Mtot_tiles, hipStream_t st) {
    hipLaunchKernelGGL((conv_gemm_kernel<T, BM, BN>), dim3(Mtot_tiles), dim3(256), 0, st, p);
    SCD_RETURN_LAUNCH();
}

}  // namespace

extern "C" int scd_conv_gemm(int dtype, const void* x, const void* w, void* y, const float* bias, double* stats,
                             int N, int Hi, int Wi, int Ci, int Ho, int Wo, int Co, int in_stride, int out_stride,
                             int wrow, int relu, int accumulate, int nphase, const scd_gemm_phase* phases,
                             void* stream) {
    if (nphase < 1 || nphase > SCD_MAX_PHASES) return SCD_ERR_ARG;
    const int BK = dtype == SCD_DT_BF16 ? 64 : 32;
    if (Ci % BK != 0 || Co <= 0 || N <= 0) return SCD_ERR_ARG;
    GemmParams p;
    p.x = (const char*)x; p.w = (const char*)w; p.y = (char*)y; p.bias = bias; p.stats = stats;
    p.N = N; p.Hi = Hi; p.Wi = Wi; p.Ci = Ci; p.Ho = Ho; p.Wo = Wo; p.Co = Co;
    p.is = in_stride; p.os = out_stride; p.wrow = wrow; p.relu = relu; p.accumulate = accumulate;
    p.nphase = nphase;
    const bool narrow = Co <= 64;
    const int BM = narrow ? 256 : 128, BN = narrow ? 64 : 128;
    p.ntn = cdiv(Co, BN);
    int tiles = 0;
    for (int i = 0; i < SCD_MAX_PHASES; ++i) {
        if (i < nphase) {
            p.ph[i] = phases[i];
            if (phases[i].ntaps < 0 || phases[i].ntaps > SCD_MAX_TAPS) return SCD_ERR_ARG;
            for (int t = 0; t < phases[i].ntaps; ++t)
                if ((long)(phases[i].wt[t] + 1) * Ci > wrow) return SCD_ERR_ARG;
            p.tile_start[i] = tiles;
            tiles += cdiv((long)N * phases[i].Qh * phases[i].Qw, BM) * p.ntn;
        } else {
            p.tile_start[i] = tiles;
        }
    }
    p.tile_start[SCD_MAX_PHASES] = tiles;
    if (tiles == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == SCD_DT_BF16)
        return narrow ? launch_gemm<__bf16, 256, 64>(p, tiles, st) : launch_gemm<__bf16, 128, 128>(p, tiles, st);
    if (dtype == SCD_DT_F32)
        return narrow ? launch_gemm<float, 256, 64>(p, tiles, st) : launch_gemm<float, 128, 128>(p, tiles, st);
    return SCD_ERR_ARG;
}

extern "C" size_t scd_conv_wgrad_workspace(int Cg, int T, int Ci, int nsplit) {
    return (size_t)nsplit * Cg * T * Ci * sizeof(float);
}

extern "C" int scd_conv_wgrad(int dtype, const void* g, const void* x, float* ws, int nsplit, int N, int Ho, int Wo,
                              int Cg, int Hi, int Wi, int Ci, int in_stride, int T, const int* dh, const int* dw,
                              void* stream) {
    const int EPC = dtype == SCD_DT_BF16 ? 8 : 4;
    if (T < 1 || T > SCD_MAX_TAPS || Ci % EPC != 0 || Cg % EPC != 0 || nsplit < 1) return SCD_ERR_ARG;
    WgradParams p;
    p.g = (const char*)g; p.x = (const char*)x; p.ws = ws;
    p.N = N; p.Ho = Ho; p.Wo = Wo; p.Cg = Cg; p.Hi = Hi; p.Wi = Wi; p.Ci = Ci; p.is = in_stride; p.T = T;
    p.KK = T * Ci;
    for (int t = 0; t < SCD_MAX_TAPS; ++t) { p.dh[t] = t < T ? dh[t] : 0; p.dw[t] = t < T ? dw[t] : 0; }
    const long M = (long)N * Ho * Wo;
    int chunk = cdiv(M, nsplit);
    chunk = (chunk + 31) / 32 * 32;
    p.chunk = chunk;
    const bool narrow = Cg <= 64;
    const int BM = narrow ? 64 : 128, BN = narrow ? 256 : 128;
    p.ntm = cdiv(Cg, BM);
    p.ntn = cdiv(p.KK, BN);
    dim3 grid(p.ntm * p.ntn, 1, nsplit);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == SCD_DT_BF16) {
        if (narrow) hipLaunchKernelGGL((conv_wgrad_kernel<__bf16, 64, 256>), grid, dim3(256), 0, st, p);
        else hipLaunchKernelGGL((conv_wgrad_kernel<__bf16, 128, 128>), grid, dim3(256), 0, st, p);
    } else if (dtype == SCD_DT_F32) {
        if (narrow) hipLaunchKernelGGL((conv_wgrad_kernel<float, 64, 256>), grid, dim3(256), 0, st, p);
        else hipLaunchKernelGGL((conv_wgrad_kernel<float, 128, 128>), grid, dim3(256), 0, st, p);
    } else {
        return SCD_ERR_ARG;
    }
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_wgrad_reduce(const float* ws, int nsplit, int Cg, int T, int Ci, int r0, int r1, int cvalid,
                                long ld_n, long ld_c, long ld_t, float* dst, int accumulate, void* stream) {
    if (r0 < 0 || r1 > Cg || r0 >= r1) return SCD_ERR_ARG;
    const long total = (long)(r1 - r0) * T * Ci;
    const int blocks = (int)std::min<long>(4096, (total + 255) / 256);
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, ws, nsplit, Cg, T, Ci,
                       r0, r1, cvalid, ld_n, ld_c, ld_t, dst, accumulate);
    SCD_RETURN_LAUNCH();
}
