// CenterNet loss (focal.py:25-53, regression.py:37-44, centerNetOffset.py:182-217) and
// decode (centerNetOffset.py:219-251, utility.py:87-118) on device, with no host syncs:
// normalisers (#pos, #mask) stay in device memory and are consumed by the backward scale.
#include <algorithm>

#include "scd_common.h"

namespace {

constexpr int FOCAL_ACC = 4;     // posL, negL, npos, pad

__global__ void focal_fwd_kernel(const float* x, const float* gt, long n, float* g, double* acc) {
    float posl = 0.f, negl = 0.f, npos = 0.f;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const float xi = x[i], t = gt[i];
        const float p = 1.f / (1.f + expf(-xi));
        const bool pass = (p >= 1e-4f) && (p <= 1.f - 1e-4f);
        const float pc = fminf(fmaxf(p, 1e-4f), 1.f - 1e-4f);
        float dterm = 0.f;
        if (t == 1.f) {
            const float om = 1.f - pc;
            const float lg = logf(pc);
            posl += lg * (om * om);
            npos += 1.f;
            dterm = om * om / pc - 2.f * om * lg;
        } else if (t < 1.f) {
            const float om = 1.f - t;
            const float w = (om * om) * (om * om);
            const float l1m = logf(1.f - pc);
            negl += l1m * (pc * pc) * w;
            dterm = w * (-(pc * pc) / (1.f - pc) + 2.f * pc * l1m);
        }
        g[i] = pass ? dterm * p * (1.f - p) : 0.f;
    }
    __shared__ double red[3][4];
    double a = wave_sum_d((double)posl), b = wave_sum_d((double)negl), c = wave_sum_d((double)npos);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) { red[0][w] = a; red[1][w] = b; red[2][w] = c; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double* dst = acc + (long)(blockIdx.x % SCD_STAT_REPLICAS) * FOCAL_ACC;
        const int nw = blockDim.x / 64;
        double s0 = 0, s1 = 0, s2 = 0;
        for (int k = 0; k < nw; ++k) { s0 += red[0][k]; s1 += red[1][k]; s2 += red[2][k]; }
        atomic_add_f64(dst + 0, s0);
        atomic_add_f64(dst + 1, s1);
        atomic_add_f64(dst + 2, s2);
    }
}

// masked L1 on features gathered at inds (NCHW fp32).  g must be zero on entry.
__global__ void l1_gather_kernel(const float* feat, int N, int C, int HW, const int64_t* inds, const uint8_t* mask,
                                 const float* target, int K, int tstride, int toff, float* g, double* acc) {
    float s = 0.f, cnt = 0.f;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < N * K; i += gridDim.x * blockDim.x) {
        const int n = i / K;
        if (!mask[i]) continue;
        cnt += 1.f;
        const long ind = inds[i];
        for (int c = 0; c < C; ++c) {
            const long fi = ((long)n * C + c) * HW + ind;
            const float d = feat[fi] - target[(long)i * tstride + toff + c];
            s += fabsf(d);
            const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
            if (sg != 0.f) atomic_add_f32(g + fi, sg);
        }
    }
    __shared__ double red[2][4];
    double a = wave_sum_d((double)s), b = wave_sum_d((double)cnt);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) { red[0][w] = a; red[1][w] = b; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double s0 = 0, s1 = 0;
        for (int k = 0; k < (int)(blockDim.x / 64); ++k) { s0 += red[0][k]; s1 += red[1][k]; }
        atomic_add_f64(acc + 0, s0);
        atomic_add_f64(acc + 1, s1);
    }
}

struct LossFin {
    float l1w[8];
};

// one block of 64 threads: thread 0 forms the loss terms, then the block re-zeroes both accumulators
// (persistent, consumer-cleared buffers: no memset launch before the next step's loss)
__global__ void loss_finalize_kernel(double* facc, int nfocal, double* lacc, int nl1, LossFin w, float* out,
                                     float* factors) {
    if (blockIdx.x != 0) return;
    if (threadIdx.x == 0) {
        double total = 0.0;
        for (int f = 0; f < nfocal; ++f) {
            double pl = 0, nl = 0, np = 0;
            for (int r = 0; r < SCD_STAT_REPLICAS; ++r) {
                const double* a = facc + ((long)f * SCD_STAT_REPLICAS + r) * FOCAL_ACC;
                pl += a[0]; nl += a[1]; np += a[2];
            }
            // focal.py:47-51: no positives -> -negL ; else -(posL+negL)/#pos
            const float posl = (float)pl, negl = (float)nl, npos = (float)np;
            const float v = np == 0.0 ? -negl : -(posl + negl) / npos;
            out[1 + f] = v;
            factors[f] = np == 0.0 ? -1.f : -1.f / npos;
            total += v;
        }
        for (int l = 0; l < nl1; ++l) {
            const double s = lacc[2 * l], cnt = lacc[2 * l + 1];
            const float v = w.l1w[l] * ((float)s / ((float)cnt + 1e-4f));
            out[1 + nfocal + l] = v;
            factors[nfocal + l] = w.l1w[l] / ((float)cnt + 1e-4f);
            total += v;
        }
        out[0] = (float)total;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nfocal * SCD_STAT_REPLICAS * FOCAL_ACC; i += blockDim.x) facc[i] = 0.0;
    if (lacc)
        for (int i = threadIdx.x; i < 2 * nl1; i += blockDim.x) lacc[i] = 0.0;
}

__global__ void scale_by_device_kernel(float* g, long n, const float* factors, int idx, const float* go) {
    const float f = factors[idx] * (go ? go[0] : 1.f);
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) g[i] *= f;
}

// ---------------------------------------------------------------- CenterNetLoss in two launches
// (centerNetOffset.py:182-217): (A) focal loss + gradient on the heatmap and the zero fill of the size / offset
// gradient buffer (both element-wise over the batch); (B) one workgroup: the two masked L1 terms on the gathered
// size / offset values (gradient +-1 added at the gathered pixels: integer-valued, so exact in any order), then the
// finalize of loss_finalize_kernel (focal replicas + L1 sums -> loss, stats, backward factors).
__global__ void centernet_loss_a_kernel(const float* x, const float* gt, long n, float* g, double* acc, float* gz,
                                        long nz) {
    float posl = 0.f, negl = 0.f, npos = 0.f;
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
        const float xi = x[i], t = gt[i];
        const float p = 1.f / (1.f + expf(-xi));
        const bool pass = (p >= 1e-4f) && (p <= 1.f - 1e-4f);
        const float pc = fminf(fmaxf(p, 1e-4f), 1.f - 1e-4f);
        float dterm = 0.f;
        if (t == 1.f) {
            const float om = 1.f - pc;
            const float lg = logf(pc);
            posl += lg * (om * om);
            npos += 1.f;
            dterm = om * om / pc - 2.f * om * lg;
        } else if (t < 1.f) {
            const float om = 1.f - t;
            const float w = (om * om) * (om * om);
            const float l1m = logf(1.f - pc);
            negl += l1m * (pc * pc) * w;
            dterm = w * (-(pc * pc) / (1.f - pc) + 2.f * pc * l1m);
        }
        g[i] = pass ? dterm * p * (1.f - p) : 0.f;
    }
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < nz; i += stride) gz[i] = 0.f;
    __shared__ double red[3][4];
    double a = wave_sum_d((double)posl), b = wave_sum_d((double)negl), c = wave_sum_d((double)npos);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) { red[0][w] = a; red[1][w] = b; red[2][w] = c; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double* dst = acc + (long)(blockIdx.x % SCD_STAT_REPLICAS) * FOCAL_ACC;
        const int nw = blockDim.x / 64;
        double s0 = 0, s1 = 0, s2 = 0;
        for (int k = 0; k < nw; ++k) { s0 += red[0][k]; s1 += red[1][k]; s2 += red[2][k]; }
        atomic_add_f64(dst + 0, s0);
        atomic_add_f64(dst + 1, s1);
        atomic_add_f64(dst + 2, s2);
    }
}

static_assert(SCD_STAT_REPLICAS == 64, "centernet_loss_b_kernel sums the focal replicas with one wave");

struct L1Term {
    const float* feat;
    float* g;
    int C, toff;
};

__global__ __launch_bounds__(1024) void centernet_loss_b_kernel(int N, int HW, const int64_t* inds, const uint8_t* mask,
                                                               const float* target, int K, int tstride, L1Term t0,
                                                               L1Term t1, double* facc, LossFin w, float* out,
                                                               float* factors) {
    float s[2] = {0.f, 0.f}, cnt = 0.f;
    for (int i = threadIdx.x; i < N * K; i += blockDim.x) {
        if (!mask[i]) continue;
        cnt += 1.f;
        const int n = i / K;
        const long ind = inds[i];
#pragma unroll
        for (int l = 0; l < 2; ++l) {
            const L1Term& t = l ? t1 : t0;
            for (int c = 0; c < t.C; ++c) {
                const long fi = ((long)n * t.C + c) * HW + ind;
                const float d = t.feat[fi] - target[(long)i * tstride + t.toff + c];
                s[l] += fabsf(d);
                const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
                if (sg != 0.f) atomic_add_f32(t.g + fi, sg);
            }
        }
    }
    __shared__ double red[3][16], frd[3];
    const double a = wave_sum_d((double)s[0]), b = wave_sum_d((double)s[1]), c = wave_sum_d((double)cnt);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 0) { red[0][wv] = a; red[1][wv] = b; red[2][wv] = c; }
    if (wv == 0) {
        // the focal replicas: one lane each (SCD_STAT_REPLICAS == 64), summed across the wave
        const double* q = facc + (long)lane * FOCAL_ACC;
        const double pl = wave_sum_d(q[0]), nl = wave_sum_d(q[1]), np = wave_sum_d(q[2]);
        if (lane == 0) { frd[0] = pl; frd[1] = nl; frd[2] = np; }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double ls[2] = {0.0, 0.0}, lc = 0.0;
        for (int k = 0; k < (int)(blockDim.x / 64); ++k) { ls[0] += red[0][k]; ls[1] += red[1][k]; lc += red[2][k]; }
        const double pl = frd[0], nl = frd[1], np = frd[2];
        // focal.py:47-51: no positives -> -negL ; else -(posL+negL)/#pos; regression.py:37-44: sum|d| / (#mask + 1e-4)
        const float posl = (float)pl, negl = (float)nl, npos = (float)np;
        const float v = np == 0.0 ? -negl : -(posl + negl) / npos;
        out[1] = v;
        factors[0] = np == 0.0 ? -1.f : -1.f / npos;
        double total = v;
        for (int l = 0; l < 2; ++l) {
            const float vl = w.l1w[l] * ((float)ls[l] / ((float)lc + 1e-4f));
            out[2 + l] = vl;
            factors[1 + l] = w.l1w[l] / ((float)lc + 1e-4f);
            total += vl;
        }
        out[0] = (float)total;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < SCD_STAT_REPLICAS * FOCAL_ACC; i += blockDim.x) facc[i] = 0.0;
}

// backward: g_heat *= factors[0] * go (dense); the size / offset gradients are zero except at the gathered pixels,
// so only those are scaled (factors[1], factors[2]), each pixel once (its first slot in the image)
__global__ void centernet_loss_scale_kernel(float* gh, long nh, int N, int HW, const int64_t* inds, int K, float* g0,
                                            int C0, float* g1, int C1, const float* factors, const float* go) {
    const float gs = go ? go[0] : 1.f;
    const float f0 = factors[0] * gs;
    const long stride = (long)gridDim.x * blockDim.x;
    const long t0 = blockIdx.x * (long)blockDim.x + threadIdx.x;
    for (long i = t0; i < nh; i += stride) gh[i] *= f0;
    const float f1 = factors[1] * gs, f2 = factors[2] * gs;
    for (long s = t0; s < (long)N * K; s += stride) {
        const int n = (int)(s / K), k = (int)(s - (long)n * K);
        const int64_t ind = inds[s];
        if (ind < 0 || ind >= HW) continue;
        bool first = true;
        for (int k2 = 0; k2 < k; ++k2) first &= inds[(long)n * K + k2] != ind;
        if (!first) continue;
        for (int c = 0; c < C0; ++c) g0[((long)n * C0 + c) * HW + ind] *= f1;
        for (int c = 0; c < C1; ++c) g1[((long)n * C1 + c) * HW + ind] *= f2;
    }
}

// ---------------------------------------------------------------- decode
// t[n][i] = sigmoid(x) kept where it equals its 3x3 (k x k) max (pad -inf), else 0
__global__ void decode_nms_kernel(const float* heat, int N, int H, int W, int k, float* t) {
    const long total = (long)N * H * W;
    const int r = (k - 1) / 2;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int n = (int)(i / ((long)H * W));
        const int rem = (int)(i - (long)n * H * W);
        const int y = rem / W, x = rem - (rem / W) * W;
        const float* hp = heat + (long)n * H * W;
        const float v = 1.f / (1.f + expf(-hp[rem]));
        float m = -INFINITY;
        for (int dy = -r; dy <= r; ++dy) {
            const int yy = y + dy;
            if ((unsigned)yy >= (unsigned)H) continue;
            for (int dx = -r; dx <= r; ++dx) {
                const int xx = x + dx;
                if ((unsigned)xx >= (unsigned)W) continue;
                m = fmaxf(m, 1.f / (1.f + expf(-hp[yy * W + xx])));
            }
        }
        t[i] = (m == v) ? v : 0.f;
    }
}

// one 1024-thread block per image: radix-select the K-th largest (non-negative floats
// order like their bit patterns), collect, then bitonic sort by (score desc, index asc).
__global__ __launch_bounds__(1024) void decode_select_kernel(const float* t, int HW, int W, int K,
                                                             const float* offset, int od_off, const float* regr,
                                                             int od_regr, float* scores, int64_t* inds, int64_t* ys,
                                                             int64_t* xs, float* off_out, float* regr_out) {
    __shared__ unsigned hist[256];
    __shared__ unsigned s_prefix, s_krem, s_count, s_eqtaken;
    __shared__ unsigned long long keys[1024];
    const int n = blockIdx.x;
    const unsigned* bits = (const unsigned*)(t + (long)n * HW);
    const int tid = threadIdx.x;
    unsigned prefix = 0, pmask = 0, krem = (unsigned)K;
    for (int pass = 0; pass < 4; ++pass) {
        const int shift = 24 - 8 * pass;
        for (int i = tid; i < 256; i += blockDim.x) hist[i] = 0;
        __syncthreads();
        for (int i = tid; i < HW; i += blockDim.x) {
            const unsigned b = bits[i];
            if ((b & pmask) == prefix) atomicAdd(&hist[(b >> shift) & 255], 1u);
        }
        __syncthreads();
        if (tid == 0) {
            unsigned cum = 0, d = 0;
            for (int b = 255; b >= 0; --b) {
                if (cum + hist[b] >= krem) { d = (unsigned)b; break; }
                cum += hist[b];
            }
            s_prefix = prefix | (d << shift);
            s_krem = krem - cum;
        }
        __syncthreads();
        prefix = s_prefix;
        krem = s_krem;
        pmask |= 255u << shift;
        __syncthreads();
    }
    // prefix = bits of the K-th largest value; krem = how many elements equal to it are needed
    if (tid == 0) { s_count = 0; s_eqtaken = 0; }
    for (int i = tid; i < 1024; i += blockDim.x) keys[i] = 0ull;
    __syncthreads();
    const unsigned thr = prefix;
    for (int i = tid; i < HW; i += blockDim.x) {
        const unsigned b = bits[i];
        if (b > thr) {
            const unsigned slot = atomicAdd(&s_count, 1u);
            keys[slot] = ((unsigned long long)b << 32) | (unsigned)(0xFFFFFFFFu - (unsigned)i);
        }
    }
    __syncthreads();
    // ties at the threshold: take the lowest indices, in index order (chunks of blockDim)
    for (int base = 0; base < HW; base += blockDim.x) {
        __syncthreads();
        const unsigned taken = s_eqtaken;
        if (taken >= krem) break;
        const int i = base + tid;
        const bool eq = i < HW && bits[i] == thr;
        // block-wide exclusive prefix count of eq flags
        const unsigned long long bal = __ballot(eq);
        const int lane = tid & 63, wv = tid >> 6;
        __shared__ unsigned wcount[16];
        if (lane == 0) wcount[wv] = __popcll(bal);
        __syncthreads();
        unsigned before = 0;
        for (int k = 0; k < wv; ++k) before += wcount[k];
        before += __popcll(bal & ((1ull << lane) - 1ull));
        if (eq && taken + before < krem) {
            const unsigned slot = (unsigned)K - krem + taken + before;
            keys[slot] = ((unsigned long long)thr << 32) | (unsigned)(0xFFFFFFFFu - (unsigned)i);
        }
        __syncthreads();
        if (tid == 0) {
            unsigned tot = 0;
            for (int k = 0; k < (int)(blockDim.x / 64); ++k) tot += wcount[k];
            s_eqtaken = taken + tot;
        }
    }
    __syncthreads();
    // bitonic sort keys[0..P) descending (P = next pow2 >= K, zero keys sort last)
    int P = 1;
    while (P < K) P <<= 1;
    for (int size = 2; size <= P; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = tid; i < P; i += blockDim.x) {
                const int j = i ^ stride;
                if (j > i) {
                    const bool desc = (i & size) == 0;
                    const unsigned long long a = keys[i], b = keys[j];
                    if (desc ? (a < b) : (a > b)) { keys[i] = b; keys[j] = a; }
                }
            }
            __syncthreads();
        }
    }
    for (int k = tid; k < K; k += blockDim.x) {
        const unsigned long long key = keys[k];
        const unsigned b = (unsigned)(key >> 32);
        const int idx = (int)(0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFu));
        const long o = (long)n * K + k;
        scores[o] = __uint_as_float(b);
        inds[o] = idx;
        ys[o] = idx / W;
        xs[o] = idx % W;
        for (int c = 0; c < od_off; ++c) off_out[o * od_off + c] = offset[((long)n * od_off + c) * HW + idx];
        if (regr)
            for (int c = 0; c < od_regr; ++c) regr_out[o * od_regr + c] = regr[((long)n * od_regr + c) * HW + idx];
    }
}

inline int ew_blocks(long n) { return (int)std::min<long>(4096, std::max<long>(1, (n + 255) / 256)); }

}  // namespace

extern "C" int scd_focal_fwd(const float* logits, const float* gt, long n, float* g, double* acc, void* stream) {
    hipLaunchKernelGGL(focal_fwd_kernel, dim3(ew_blocks(n)), dim3(256), 0, (hipStream_t)stream, logits, gt, n, g, acc);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_l1_gather_fwd(const float* feat, int N, int C, int HW, const int64_t* inds, const uint8_t* mask,
                                 const float* target, int K, int tstride, int toff, float* g, double* acc, void* stream) {
    const int blocks = std::max(1, std::min(64, cdiv((long)N * K, 256)));
    hipLaunchKernelGGL(l1_gather_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, feat, N, C, HW, inds, mask,
                       target, K, tstride, toff, g, acc);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_centernet_loss_finalize(double* focal_acc, int nfocal, double* l1_acc, int nl1,
                                           const float* l1_weights, float* out, float* factors, void* stream) {
    if (nl1 > 8) return SCD_ERR_ARG;
    LossFin w;
    for (int i = 0; i < 8; ++i) w.l1w[i] = i < nl1 ? l1_weights[i] : 0.f;
    hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, focal_acc, nfocal, l1_acc, nl1, w,
                       out, factors);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_centernet_loss_fwd(const float* heat, const float* gt, long n_heat, const float* regr, int Cr,
                                      const float* off, int Co, int N, int HW, const int64_t* inds, const uint8_t* mask,
                                      const float* target, int K, int tstride, int toff_r, int toff_o,
                                      const float* l1_weights, float* g_heat, float* g_regr, float* g_off,
                                      double* focal_acc, float* out, float* factors, void* stream) {
    if (n_heat < 1 || K < 1 || N < 1 || g_off != g_regr + (long)N * Cr * HW) return SCD_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    const long nz = (long)N * (Cr + Co) * HW;
    hipLaunchKernelGGL(centernet_loss_a_kernel, dim3(ew_blocks(std::max(n_heat, nz))), dim3(256), 0, st, heat, gt, n_heat,
                       g_heat, focal_acc, g_regr, nz);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    LossFin w;
    for (int i = 0; i < 8; ++i) w.l1w[i] = i < 2 ? l1_weights[i] : 0.f;
    L1Term t0{regr, g_regr, Cr, toff_r}, t1{off, g_off, Co, toff_o};
    hipLaunchKernelGGL(centernet_loss_b_kernel, dim3(1), dim3(1024), 0, st, N, HW, inds, mask, target, K, tstride, t0, t1,
                       focal_acc, w, out, factors);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_centernet_loss_bwd_scale(float* g_heat, long n_heat, int N, int HW, const int64_t* inds, int K,
                                            float* g_regr, int Cr, float* g_off, int Co, const float* factors,
                                            const float* go, void* stream) {
    hipLaunchKernelGGL(centernet_loss_scale_kernel, dim3(ew_blocks(n_heat)), dim3(256), 0, (hipStream_t)stream, g_heat,
                       n_heat, N, HW, inds, K, g_regr, Cr, g_off, Co, factors, go);
    SCD_RETURN_LAUNCH();
}

// Keep map of the pixels a CenterNet loss gathers (inds[n][k], all K slots): one workgroup, the previous call's
// pixels (prev, flattened n*HW + p; -1 = none) cleared first, then the new ones set and remembered, so the persistent
// map needs no full-size memset per step.
__global__ __launch_bounds__(1024) void heads_keep_map_kernel(const int64_t* inds, int N, int K, int HW, int64_t* prev,
                                                              int nprev, uint8_t* keep) {
    for (int i = threadIdx.x; i < nprev; i += blockDim.x) {
        const int64_t q = prev[i];
        if (q >= 0) keep[q] = 0;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < N * K; i += blockDim.x) {
        const int n = i / K;
        const int64_t v = inds[i];
        const int64_t q = (v >= 0 && v < HW) ? (int64_t)n * HW + v : -1;
        if (q >= 0) keep[q] = 1;
        prev[i] = q;
    }
    for (int i = N * K + threadIdx.x; i < nprev; i += blockDim.x) prev[i] = -1;
}

extern "C" int scd_heads_keep_map(const int64_t* inds, int N, int K, int HW, int64_t* prev, int nprev, uint8_t* keep,
                                  void* stream) {
    if (N < 1 || K < 1 || HW < 1 || nprev < N * K) return SCD_ERR_ARG;
    hipLaunchKernelGGL(heads_keep_map_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, inds, N, K, HW, prev, nprev,
                       keep);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_scale_by_device(float* g, long n, const float* factors, int idx, const float* go, void* stream) {
    hipLaunchKernelGGL(scale_by_device_kernel, dim3(ew_blocks(n)), dim3(256), 0, (hipStream_t)stream, g, n, factors, idx,
                       go);
    SCD_RETURN_LAUNCH();
}

extern "C" size_t scd_decode_workspace(int N, int HW) { return (size_t)N * HW * sizeof(float); }

extern "C" int scd_decode_topk(const float* heat, int N, int H, int W, int K, const float* offset, int od_off,
                               const float* regr, int od_regr, float* scores, int64_t* inds, int64_t* ys, int64_t* xs,
                               float* off_out, float* regr_out, void* workspace, void* stream) {
    if (K < 1 || K > 1024 || K > H * W) return SCD_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    float* t = (float*)workspace;
    hipLaunchKernelGGL(decode_nms_kernel, dim3(ew_blocks((long)N * H * W)), dim3(256), 0, st, heat, N, H, W, 3, t);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(decode_select_kernel, dim3(N), dim3(1024), 0, st, t, H * W, W, K, offset, od_off, regr, od_regr,
                       scores, inds, ys, xs, off_out, regr_out);
    SCD_RETURN_LAUNCH();
}
