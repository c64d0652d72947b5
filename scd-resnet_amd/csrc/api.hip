// The reference's functional helpers as HIP kernels, for user code that calls them directly
// (the training / decode path uses the fused kernels of loss_decode.hip instead):
//   nonMaximumSuppression   models/backbones/utility.py:87-92   scd_nms
//   extractTopK             models/backbones/utility.py:106-118 scd_topk
//   focalLoss               models/losses/focal.py:25-53        scd_focal_prob_fwd (+ scd_centernet_loss_finalize)
//   L1LossMask / smoothL1LossMask  models/losses/regression.py:28-44  scd_masked_l1_fwd (+ finalize)
// Forward passes also write the per-element gradient; the normalisers stay on the device (finalize factors), so
// no entry point synchronises with the host.
#include <algorithm>

#include "scd_common.h"

namespace {

inline int ew_blocks(long n) { return (int)std::min<long>(4096, std::max<long>(1, (n + 255) / 256)); }

// out = x where x equals its k x k neighbourhood max (padding -inf), else 0 -- heat * (maxpool(heat) == heat)
__global__ void nms_kernel(const float* x, long planes, int H, int W, int k, float* out) {
    const long total = planes * H * W;
    const int r = (k - 1) / 2;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const long pl = i / ((long)H * W);
        const int rem = (int)(i - pl * H * W);
        const int y = rem / W, xx = rem - (rem / W) * W;
        const float* hp = x + pl * H * W;
        const float v = hp[rem];
        float m = -INFINITY;
        for (int dy = -r; dy <= k - 1 - r; ++dy) {
            const int yy = y + dy;
            if ((unsigned)yy >= (unsigned)H) continue;
            for (int dx = -r; dx <= k - 1 - r; ++dx) {
                const int xc = xx + dx;
                if ((unsigned)xc >= (unsigned)W) continue;
                m = fmaxf(m, hp[yy * W + xc]);
            }
        }
        out[i] = v * (m == v ? 1.f : 0.f);
    }
}

// order-preserving key of a float (larger float -> larger unsigned)
__device__ __forceinline__ unsigned fkey(float f) {
    const unsigned b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float fkey_inv(unsigned k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// one 1024-thread block per row: radix-select the K-th largest key, collect the larger ones and the lowest-index
// ties, bitonic sort by (value desc, index asc); then the reference's category / index / y / x split
__global__ __launch_bounds__(1024) void topk_kernel(const float* s, long n, int K, int HW, int W, float* scores,
                                                    int64_t* inds, int* cats, float* ys, float* xs) {
    __shared__ unsigned hist[256];
    __shared__ unsigned s_prefix, s_krem, s_count, s_eqtaken;
    __shared__ unsigned long long keys[1024];
    __shared__ unsigned wcount[16];
    const long row = blockIdx.x;
    const float* v = s + row * n;
    const int tid = threadIdx.x;
    unsigned prefix = 0, pmask = 0, krem = (unsigned)K;
    for (int pass = 0; pass < 4; ++pass) {
        const int shift = 24 - 8 * pass;
        for (int i = tid; i < 256; i += blockDim.x) hist[i] = 0;
        __syncthreads();
        for (long i = tid; i < n; i += blockDim.x) {
            const unsigned b = fkey(v[i]);
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
    if (tid == 0) { s_count = 0; s_eqtaken = 0; }
    for (int i = tid; i < 1024; i += blockDim.x) keys[i] = 0ull;
    __syncthreads();
    const unsigned thr = prefix;
    for (long i = tid; i < n; i += blockDim.x) {
        const unsigned b = fkey(v[i]);
        if (b > thr) {
            const unsigned slot = atomicAdd(&s_count, 1u);
            keys[slot] = ((unsigned long long)b << 32) | (unsigned)(0xFFFFFFFFu - (unsigned)i);
        }
    }
    __syncthreads();
    for (long base = 0; base < n; base += blockDim.x) {
        __syncthreads();
        const unsigned taken = s_eqtaken;
        if (taken >= krem) break;
        const long i = base + tid;
        const bool eq = i < n && fkey(v[i]) == thr;
        const unsigned long long bal = __ballot(eq);
        const int lane = tid & 63, wv = tid >> 6;
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
        const long idx = (long)(0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFu));
        const long o = row * K + k;
        scores[o] = fkey_inv((unsigned)(key >> 32));
        const long sp = idx % HW;
        inds[o] = sp;
        cats[o] = (int)(idx / HW);
        ys[o] = (float)(sp / W);
        xs[o] = (float)(sp % W);
    }
}

constexpr int FOCAL_ACC = 4;     // posL, negL, npos, pad (the layout scd_centernet_loss_finalize reads)

// focal.py:25-53 on probabilities p (no sigmoid / clamp here: the caller's clampSigmoid did that): per element
// dL/dp up to the normaliser, and the posL / negL / #pos sums into fp64 replica slots
__global__ void focal_prob_kernel(const float* p, const float* gt, long n, float* g, double* acc) {
    float posl = 0.f, negl = 0.f, npos = 0.f;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const float pc = p[i], t = gt[i];
        float d = 0.f;
        if (t == 1.f) {
            const float om = 1.f - pc;
            const float lg = logf(pc);
            posl += lg * (om * om);
            npos += 1.f;
            d = om * om / pc - 2.f * om * lg;
        } else if (t < 1.f) {
            const float om = 1.f - t;
            const float w = (om * om) * (om * om);
            const float l1m = logf(1.f - pc);
            negl += l1m * (pc * pc) * w;
            d = w * (-(pc * pc) / (1.f - pc) + 2.f * pc * l1m);
        }
        g[i] = d;
    }
    __shared__ double red[3][4];
    double a = wave_sum_d((double)posl), b = wave_sum_d((double)negl), c = wave_sum_d((double)npos);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) { red[0][w] = a; red[1][w] = b; red[2][w] = c; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double* dst = acc + (long)(blockIdx.x % SCD_STAT_REPLICAS) * FOCAL_ACC;
        double s0 = 0, s1 = 0, s2 = 0;
        for (int k = 0; k < (int)(blockDim.x / 64); ++k) { s0 += red[0][k]; s1 += red[1][k]; s2 += red[2][k]; }
        atomic_add_f64(dst + 0, s0);
        atomic_add_f64(dst + 1, s1);
        atomic_add_f64(dst + 2, s2);
    }
}

// regression.py:28-44 on gathered (rows, C) tensors: masked |d| (or smooth-L1, beta 1) summed, the mask count, and
// the per-element gradient (sign(d), or d clipped to [-1, 1]) -- 0 on masked-out rows
__global__ void masked_l1_kernel(const float* r, const float* t, const uint8_t* mask, long rows, int C, int smooth,
                                 float* g, double* acc) {
    float s = 0.f, cnt = 0.f;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < rows; i += (long)gridDim.x * blockDim.x) {
        const bool on = mask[i] != 0;
        cnt += on ? 1.f : 0.f;
        for (int c = 0; c < C; ++c) {
            const long e = i * C + c;
            float gv = 0.f;
            if (on) {
                const float d = r[e] - t[e];
                const float ad = fabsf(d);
                if (smooth && ad < 1.f) {
                    s += 0.5f * d * d;
                    gv = d;
                } else {
                    s += smooth ? ad - 0.5f : ad;
                    gv = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
                }
            }
            g[e] = gv;
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

}  // namespace

extern "C" int scd_nms(const float* x, long planes, int H, int W, int k, float* out, void* stream) {
    if (planes < 0 || H < 1 || W < 1 || k < 1 || k % 2 == 0) return SCD_ERR_ARG;
    hipLaunchKernelGGL(nms_kernel, dim3(ew_blocks(planes * H * W)), dim3(256), 0, (hipStream_t)stream, x, planes, H, W,
                       k, out);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_topk(const float* scores, int B, long n, int K, int HW, int W, float* out_scores, int64_t* inds,
                        int* cats, float* ys, float* xs, void* stream) {
    if (B < 1 || K < 1 || K > 1024 || K > n || n >= (1L << 32) - 1 || HW < 1 || W < 1) return SCD_ERR_ARG;
    hipLaunchKernelGGL(topk_kernel, dim3(B), dim3(1024), 0, (hipStream_t)stream, scores, n, K, HW, W, out_scores, inds,
                       cats, ys, xs);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_focal_prob_fwd(const float* p, const float* gt, long n, float* g, double* acc, void* stream) {
    hipLaunchKernelGGL(focal_prob_kernel, dim3(ew_blocks(n)), dim3(256), 0, (hipStream_t)stream, p, gt, n, g, acc);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_masked_l1_fwd(const float* r, const float* t, const uint8_t* mask, long rows, int C, int smooth,
                                 float* g, double* acc, void* stream) {
    if (C < 1) return SCD_ERR_ARG;
    const int blocks = std::max(1, std::min(256, cdiv(rows, 256)));
    hipLaunchKernelGGL(masked_l1_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, r, t, mask, rows, C, smooth, g,
                       acc);
    SCD_RETURN_LAUNCH();
}
