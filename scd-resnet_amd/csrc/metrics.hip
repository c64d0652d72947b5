// CenterNet validation metrics on the GPU.
//
// Reference: models/centerNetOffset.py:253-354 (centerNetEvaluation: predicted / ground-truth boxes in three
// flavours, validMask = score >= 0.3) and evaluations/detection.py:11-180 (IoU, Orthogonity, MAE,
// IoUConfidence: every (detection k, ground truth l) pair of an image tested for overlap and the surviving
// values masked_select-ed in (n, k, l) row-major order), :183-230 (averagePrecisionPlots /
// averagePrecisionAll), trainer/model/centerOffsetRes10.py:18-106 (expression: means and AP30/50/70/90).
//
// Layout: one workgroup per image.  The per-detection and per-object boxes are built once into LDS
// (fp32, each torch op rounded separately: no contraction), then the K x L pairs are walked in row-major
// order in chunks of 256; five masks (box, box with a non-degenerate gt major axis, centre/centre,
// centre/offset, offset/offset) are compacted with wave ballots so that the output order is exactly
// masked_select's.  Pass 1 counts per image; pass 2 recomputes and writes at the image's offset (the
// exclusive sum of the earlier images' counts), so the host allocates exact-size outputs after one
// small counts read -- the reference's .item() calls are gone.
//
// The summary kernel is one 1024-thread workgroup: fp64 means of the nine streams and the reference's
// interpolated AP at four IoU thresholds.  Detections are ordered by descending score with ties by
// DESCENDING pair index (= the reference's torch.sort ascending + flip when that sort is stable; torch's
// CPU sort is unstable above 16 elements, so the reference's own tie order is unspecified).
#include "scd_common.h"

#pragma clang fp contract(off)

namespace {

constexpr int CE_MAXK = 256;
constexpr int CE_MAXL = 64;
constexpr int CE_THREADS = 256;
constexpr int CE_NMASK = 5;
constexpr int CE_NSTREAM = 9;

struct DetBox {
    float b[4], c[4], o[4];       // bounds, boundsCenter, boundsOffset (tlx, tly, brx, bry)
    float mx, my, ml, r2, r3, score;
    int valid;
};
struct GtBox {
    float b[4], c[4], o[4];       // groundTruthLocs, ...Center, ...Offset
    float mx, my, ml, g4, g5;
};

struct CEvalIn {
    const float* scores;          // (N,K)
    const int64_t* cty;           // (N,K)
    const int64_t* ctx;           // (N,K)
    const float* offset;          // (N,K,2)
    const float* regr;            // (N,K,4) = [majx, majy, minl, halo]
    const float* gt_regr;         // (N,L,6) = [offx, offy, majx, majy, minl, halo]
    const void* gt_loc;           // (N,L) int64 heat indices (loc_mode 0) or (N,L,loc_w) f32 [x, y, ...] (mode 1)
    int N, K, L, H, loc_mode, loc_w;
    float thr;
};

__device__ __forceinline__ float q4(float v) { return __fdiv_rn(v, 4.f); }
__device__ __forceinline__ float hyp(float a, float b) { return __fsqrt_rn(__fadd_rn(__fmul_rn(a, a), __fmul_rn(b, b))); }

// centerNetOffset.py:264-281 (predicted boxes, 128x heatmap units)
__device__ void build_det(const CEvalIn& p, int n, int k, DetBox& d) {
    long i = (long)n * p.K + k;
    const float* r = p.regr + i * 4;
    float o0 = q4(p.offset[i * 2]), o1 = q4(p.offset[i * 2 + 1]);
    long x = p.ctx[i], y = p.cty[i];
    float fx = (float)x, fy = (float)y;
    d.ml = hyp(r[0], r[1]);
    d.b[0] = __fadd_rn(__fsub_rn(fx, d.ml), o0);
    d.b[1] = __fadd_rn(__fsub_rn(fy, r[2]), o1);
    d.b[2] = __fadd_rn(__fadd_rn(fx, d.ml), o0);
    d.b[3] = __fadd_rn(__fadd_rn(fy, r[2]), o1);
    d.c[0] = (float)(x - 2); d.c[1] = (float)(y - 2); d.c[2] = (float)(x + 2); d.c[3] = (float)(y + 2);
    d.o[0] = __fadd_rn(d.c[0], o0); d.o[1] = __fadd_rn(d.c[1], o1);
    d.o[2] = __fadd_rn(d.c[2], o0); d.o[3] = __fadd_rn(d.c[3], o1);
    d.mx = r[0]; d.my = r[1]; d.r2 = r[2]; d.r3 = r[3];
    d.score = p.scores[i];
    d.valid = d.score >= p.thr;   // centerNetOffset.py:345
}

// centerNetOffset.py:283-306 (ground truth; ys[3] is either heat indices (dim 2) or locs rows (dim 3))
__device__ void build_gt(const CEvalIn& p, int n, int l, GtBox& g) {
    long i = (long)n * p.L + l;
    const float* t = p.gt_regr + i * 6;
    float cx, cy, c0, c1, c2, c3;
    if (p.loc_mode == 0) {
        long idx = ((const int64_t*)p.gt_loc)[i];
        long yy = idx >= 0 ? idx / p.H : -((-idx + p.H - 1) / p.H);   // torch floor division
        long xx = idx - yy * p.H;
        cx = (float)xx; cy = (float)yy;
        c0 = (float)(xx - 2); c1 = (float)(yy - 2); c2 = (float)(xx + 2); c3 = (float)(yy + 2);
    } else {
        const float* lr = (const float*)p.gt_loc + i * p.loc_w;
        cx = lr[0]; cy = lr[1];
        c0 = __fsub_rn(cx, 2.f); c1 = __fsub_rn(cy, 2.f); c2 = __fadd_rn(cx, 2.f); c3 = __fadd_rn(cy, 2.f);
    }
    float o0 = q4(t[0]), o1 = q4(t[1]);
    g.ml = hyp(t[2], t[3]);
    g.b[0] = __fadd_rn(__fsub_rn(cx, g.ml), o0);
    g.b[1] = __fadd_rn(__fsub_rn(cy, t[4]), o1);
    g.b[2] = __fadd_rn(__fadd_rn(cx, g.ml), o0);
    g.b[3] = __fadd_rn(__fadd_rn(cy, t[4]), o1);
    g.c[0] = c0; g.c[1] = c1; g.c[2] = c2; g.c[3] = c3;
    g.o[0] = __fadd_rn(c0, o0); g.o[1] = __fadd_rn(c1, o1); g.o[2] = __fadd_rn(c2, o0); g.o[3] = __fadd_rn(c3, o1);
    g.mx = t[2]; g.my = t[3]; g.g4 = t[4]; g.g5 = t[5];
}

// detection.py:27-46: overlap test and IoU of one pair (the test's thresholds are float32 1e-5)
__device__ __forceinline__ bool overlap(const float* d, const float* g, bool valid, float& iou) {
    float darea = __fmul_rn(__fsub_rn(d[2], d[0]), __fsub_rn(d[3], d[1]));
    float garea = __fmul_rn(__fsub_rn(g[2], g[0]), __fsub_rn(g[3], g[1]));
    float dx = __fsub_rn(fminf(d[2], g[2]), fmaxf(d[0], g[0]));
    float dy = __fsub_rn(fminf(d[3], g[3]), fmaxf(d[1], g[1]));
    const float eps = 1e-5f;
    bool m = (dx > eps) && (dy > eps) && (garea > eps) && valid;
    float inter = __fmul_rn(dx, dy);
    iou = __fdiv_rn(inter, __fsub_rn(__fadd_rn(darea, garea), inter));
    return m;
}

struct PairOut {
    unsigned mask;                // bit m: pair survives mask m
    float v[CE_NSTREAM];
};

__device__ void eval_pair(const DetBox& d, const GtBox& g, PairOut& r) {
    float iou_b, iou_cc, iou_co, iou_oo;
    bool mb = overlap(d.b, g.b, d.valid, iou_b);
    bool mb2 = mb && (g.ml > 1e-5f);
    bool mcc = overlap(d.c, g.c, d.valid, iou_cc);
    bool mco = overlap(d.c, g.o, d.valid, iou_co);
    bool moo = overlap(d.o, g.o, d.valid, iou_oo);
    r.mask = (unsigned)mb | ((unsigned)mb2 << 1) | ((unsigned)mcc << 2) | ((unsigned)mco << 3) | ((unsigned)moo << 4);
    // detection.py:80-81 (Orthogonity)
    float cs = __fdiv_rn(__fadd_rn(__fmul_rn(d.mx, g.mx), __fmul_rn(d.my, g.my)), __fmul_rn(d.ml, g.ml));
    float sn = __fsqrt_rn(__fsub_rn(1.f, __fmul_rn(cs, cs)));
    r.v[0] = iou_b; r.v[1] = d.score; r.v[2] = sn; r.v[3] = iou_cc; r.v[4] = iou_co; r.v[5] = iou_oo;
    // detection.py:132-134 (MAE with regr = [majL, minL, halo])
    r.v[6] = fabsf(__fsub_rn(d.ml, g.ml));
    r.v[7] = fabsf(__fsub_rn(d.r2, g.g4));
    r.v[8] = fabsf(__fsub_rn(d.r3, g.g5));
}

__constant__ int c_stream_mask[CE_NSTREAM] = {0, 0, 1, 2, 3, 4, 1, 1, 1};

struct CEvalOut {
    float* s[CE_NSTREAM];
};

// EMIT = false: counts[n][m] only.  EMIT = true: values written at (earlier images' counts) + in-image rank.
template <bool EMIT>
__global__ __launch_bounds__(CE_THREADS) void ceval_pairs_kernel(CEvalIn p, int* counts, CEvalOut out) {
    __shared__ DetBox sd[CE_MAXK];
    __shared__ GtBox sg[CE_MAXL];
    __shared__ int wtot[CE_THREADS / 64][CE_NMASK];
    __shared__ int base[CE_NMASK];
    const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (int k = tid; k < p.K; k += CE_THREADS) build_det(p, n, k, sd[k]);
    for (int l = tid; l < p.L; l += CE_THREADS) build_gt(p, n, l, sg[l]);
    if (EMIT) {
        // this image's output offsets: the earlier images' counts, summed by the whole workgroup
        int part[CE_NMASK] = {0, 0, 0, 0, 0};
        for (int j = tid; j < n; j += CE_THREADS)
#pragma unroll
            for (int m = 0; m < CE_NMASK; ++m) part[m] += counts[j * CE_NMASK + m];
#pragma unroll
        for (int m = 0; m < CE_NMASK; ++m) {
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) part[m] += __shfl_xor(part[m], o, 64);
            if (lane == 0) wtot[wv][m] = part[m];
        }
        __syncthreads();
        if (tid < CE_NMASK) {
            int b = 0;
            for (int w = 0; w < CE_THREADS / 64; ++w) b += wtot[w][tid];
            base[tid] = b;
        }
    } else if (tid < CE_NMASK) {
        base[tid] = 0;
    }
    __syncthreads();
    const int npairs = p.K * p.L;
    for (int c0 = 0; c0 < npairs; c0 += CE_THREADS) {
        int q = c0 + tid;
        PairOut r;
        r.mask = 0;
        if (q < npairs) eval_pair(sd[q / p.L], sg[q % p.L], r);
        unsigned long long lt = (1ull << lane) - 1ull;
        int rank[CE_NMASK];
#pragma unroll
        for (int m = 0; m < CE_NMASK; ++m) {
            unsigned long long bal = __ballot((r.mask >> m) & 1u);
            rank[m] = __popcll(bal & lt);
            if (lane == 0) wtot[wv][m] = __popcll(bal);
        }
        __syncthreads();
        if (EMIT) {
#pragma unroll
            for (int s = 0; s < CE_NSTREAM; ++s) {
                int m = c_stream_mask[s];
                if ((r.mask >> m) & 1u) {
                    int off = base[m] + rank[m];
                    for (int w = 0; w < wv; ++w) off += wtot[w][m];
                    out.s[s][off] = r.v[s];
                }
            }
        }
        __syncthreads();
        if (tid < CE_NMASK) {
            int t = 0;
            for (int w = 0; w < CE_THREADS / 64; ++w) t += wtot[w][tid];
            base[tid] += t;
        }
        __syncthreads();
    }
    if (!EMIT && tid < CE_NMASK) counts[n * CE_NMASK + tid] = base[tid];
}

// ---------------------------------------------------------------- summary (means + interpolated AP)
constexpr int SM_T = 1024;

struct SummaryIn {
    const float* s[CE_NSTREAM];
    long len[CE_NSTREAM];
};

__device__ double block_sum_d(double v, double* red) {
    v = wave_sum_d(v);
    int tid = threadIdx.x;
    __syncthreads();
    if ((tid & 63) == 0) red[tid >> 6] = v;
    __syncthreads();
    double t = 0.0;
    for (int w = 0; w < SM_T / 64; ++w) t += red[w];
    __syncthreads();
    return t;
}

// inclusive Hillis-Steele scan in LDS (op: 0 sum of int, 1 max of int)
__device__ int block_scan_i(int v, int* a, int op) {
    int tid = threadIdx.x;
    a[tid] = v;
    __syncthreads();
    for (int o = 1; o < SM_T; o <<= 1) {
        int u = tid >= o ? a[tid - o] : (op == 0 ? 0 : -1);
        __syncthreads();
        a[tid] = op == 0 ? a[tid] + u : max(a[tid], u);
        __syncthreads();
    }
    int r = a[tid];
    __syncthreads();
    return r;
}
__device__ double block_scan_max_d(double v, double* a) {
    int tid = threadIdx.x;
    a[tid] = v;
    __syncthreads();
    for (int o = 1; o < SM_T; o <<= 1) {
        double u = tid >= o ? a[tid - o] : 0.0;
        __syncthreads();
        a[tid] = fmax(a[tid], u);
        __syncthreads();
    }
    double r = a[tid];
    __syncthreads();
    return r;
}

__device__ __forceinline__ unsigned long long sort_key(float s, unsigned idx) {
    unsigned u = __float_as_uint(s);
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);   // order-preserving
    return ((unsigned long long)u << 32) | idx;
}

// out[0..8] = means of the nine streams (stream 2, orthogonity, over its non-NaN values only),
// out[9..9+nthr) = AP at thr[] (trainer/model/centerOffsetRes10.py:81-88).
// ws: keys u64[P] + cum int[P] + prev-record int[P], P = next pow2 >= len[0].
__global__ __launch_bounds__(SM_T) void ceval_summary_kernel(SummaryIn in, long objnum, const float* thr, int nthr,
                                                             double* out, unsigned long long* keys, int* cum,
                                                             int P) {
    __shared__ double red[SM_T / 64];
    __shared__ double dsc[SM_T];
    __shared__ int isc[SM_T];
    const int tid = threadIdx.x;
    for (int s = 0; s < CE_NSTREAM; ++s) {
        double acc = 0.0, cnt = 0.0;
        for (long i = tid; i < in.len[s]; i += SM_T) {
            float v = in.s[s][i];
            if (s == 2 && v != v) continue;
            acc += (double)v;
            cnt += 1.0;
        }
        acc = block_sum_d(acc, red);
        cnt = block_sum_d(cnt, red);
        if (tid == 0) out[s] = cnt > 0.0 ? acc / cnt : 0.0;
    }
    // sort (score desc, pair index desc) -- bitonic over P keys in global memory, one workgroup
    const long n = in.len[0];
    for (long i = tid; i < P; i += SM_T) keys[i] = i < n ? sort_key(in.s[1][i], (unsigned)i) : 0ull;
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < P; i += SM_T) {
                int ixj = i ^ j;
                if (ixj > i) {
                    unsigned long long a = keys[i], b = keys[ixj];
                    bool desc = (i & k) == 0;
                    if (desc ? (a < b) : (a > b)) { keys[i] = b; keys[ixj] = a; }
                }
            }
            __syncthreads();
        }
    }
    const double total = (double)(objnum > n ? objnum : n);
    for (int t = 0; t < nthr; ++t) {
        const float th = thr[t];
        // cumulative true positives in sorted order (detection.py:199-206: iou < threshold is a false one)
        int carry = 0;
        for (long c0 = 0; c0 < n; c0 += SM_T) {
            long i = c0 + tid;
            int tp = 0;
            if (i < n) tp = !(in.s[0][(unsigned)(keys[i] & 0xffffffffu)] < th);
            int incl = block_scan_i(tp, isc, 0) + carry;
            if (i < n) cum[i] = incl;
            if (tid == SM_T - 1) isc[0] = incl;
            __syncthreads();
            carry = isc[0];
            __syncthreads();
        }
        // records: precision strictly above every later one (detection.py:219-226); scanned from the end
        double sufmax = 0.0;
        for (long c1 = n; c1 > 0; c1 -= SM_T) {
            long i = c1 - 1 - tid;
            double pr = i >= 0 ? (double)cum[i] / (double)(i + 1) : 0.0;
            double incl = fmax(block_scan_max_d(pr, dsc), sufmax);   // max over [i, end)
            // exclusive (max over (i, end)): the previous thread's inclusive value
            dsc[tid] = incl;
            __syncthreads();
            double excl = tid > 0 ? dsc[tid - 1] : sufmax;
            bool rec = i >= 0 && pr > excl;
            if (i >= 0) cum[i] = rec ? -cum[i] - 1 : cum[i];   // tag records in place (cum >= 0)
            double last = dsc[SM_T - 1];
            __syncthreads();
            sufmax = last;
        }
        // each record j_a adds (r[j_a] - r[j_b + 1]) * p[j_a], j_b the nearest record before it; the first
        // record adds r * p (averagePrecisionAll's x1/x2 walk, detection.py:214-230)
        double ap = 0.0;
        int carry_rec = -1;
        for (long c0 = 0; c0 < n; c0 += SM_T) {
            long i = c0 + tid;
            int cv = i < n ? cum[i] : 0;
            bool rec = cv < 0;
            int c = rec ? -cv - 1 : cv;
            int last_rec = max(block_scan_i(rec ? (int)i : -1, isc, 1), carry_rec);   // last record <= i
            isc[tid] = last_rec;
            __syncthreads();
            int prev = tid > 0 ? isc[tid - 1] : carry_rec;                        // last record < i
            int nxt_carry = isc[SM_T - 1];
            __syncthreads();
            if (i < n && rec) {
                double pr = (double)c / (double)(i + 1), rc = (double)c / total;
                if (prev >= 0) {
                    int cb = cum[prev + 1];
                    cb = cb < 0 ? -cb - 1 : cb;
                    ap += (rc - (double)cb / total) * pr;
                } else {
                    ap += rc * pr;
                }
            }
            carry_rec = nxt_carry;
        }
        ap = block_sum_d(ap, red);
        if (tid == 0) out[CE_NSTREAM + t] = ap;
        __syncthreads();
    }
}

bool ceval_args_ok(int N, int K, int L, int H, int loc_mode, int loc_w) {
    return N >= 1 && K >= 1 && K <= CE_MAXK && L >= 1 && L <= CE_MAXL && H >= 1 && (loc_mode == 0 || loc_mode == 1) &&
           (loc_mode == 0 || loc_w >= 2);
}

}  // namespace

extern "C" int scd_ceval_count(const float* scores, const int64_t* cty, const int64_t* ctx, const float* offset,
                               const float* regr, const float* gt_regr, const void* gt_loc, int loc_mode, int loc_w,
                               int N, int K, int L, int H, float thr, int* counts, void* stream) {
    if (!ceval_args_ok(N, K, L, H, loc_mode, loc_w)) return SCD_ERR_ARG;
    CEvalIn p{scores, cty, ctx, offset, regr, gt_regr, gt_loc, N, K, L, H, loc_mode, loc_w, thr};
    CEvalOut o{};
    hipLaunchKernelGGL(ceval_pairs_kernel<false>, dim3(N), dim3(CE_THREADS), 0, (hipStream_t)stream, p, counts, o);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_ceval_emit(const float* scores, const int64_t* cty, const int64_t* ctx, const float* offset,
                              const float* regr, const float* gt_regr, const void* gt_loc, int loc_mode, int loc_w,
                              int N, int K, int L, int H, float thr, const int* counts, float* const* streams,
                              void* stream) {
    if (!ceval_args_ok(N, K, L, H, loc_mode, loc_w)) return SCD_ERR_ARG;
    CEvalIn p{scores, cty, ctx, offset, regr, gt_regr, gt_loc, N, K, L, H, loc_mode, loc_w, thr};
    CEvalOut o;
    for (int s = 0; s < CE_NSTREAM; ++s) o.s[s] = streams[s];
    hipLaunchKernelGGL(ceval_pairs_kernel<true>, dim3(N), dim3(CE_THREADS), 0, (hipStream_t)stream, p,
                       (int*)counts, o);
    SCD_RETURN_LAUNCH();
}

static int pow2_at_least(long n) {
    int P = 1;
    while (P < n) P <<= 1;
    return P;
}

extern "C" size_t scd_ceval_summary_workspace(long n) {
    if (n < 0 || n >= (1L << 30)) return 0;
    return (size_t)pow2_at_least(n) * (sizeof(unsigned long long) + sizeof(int));
}

extern "C" int scd_ceval_summary(const float* const* streams, const long* lens, long objnum, const float* thr,
                                 int nthr, double* out, void* workspace, void* stream) {
    SummaryIn in;
    for (int s = 0; s < CE_NSTREAM; ++s) {
        in.s[s] = streams[s];
        in.len[s] = lens[s];
        if (lens[s] < 0 || lens[s] >= (1L << 30)) return SCD_ERR_ARG;
    }
    if (lens[1] != lens[0] || nthr < 0 || nthr > 16) return SCD_ERR_ARG;
    int P = pow2_at_least(lens[0] > 0 ? lens[0] : 1);
    unsigned long long* keys = (unsigned long long*)workspace;
    int* cum = (int*)(keys + P);
    hipLaunchKernelGGL(ceval_summary_kernel, dim3(1), dim3(SM_T), 0, (hipStream_t)stream, in, objnum, thr, nthr, out,
                       keys, cum, P);
    SCD_RETURN_LAUNCH();
}
