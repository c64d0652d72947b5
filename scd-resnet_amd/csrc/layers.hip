// Layer glue kernels: weight packing, stem im2col, stem BN+ReLU+MaxPool (fwd/bwd),
// fused CenterNet head tails (1x1 convs), Adam.  All HBM-bound; 16-B vectorised where the
// layout allows.
#include <algorithm>

#include "scd_common.h"

namespace {

// ---------------------------------------------------------------- weight packing
template <typename T>
__global__ void pack_weight_kernel(const float* w, T* out, int A, int B, int Tt, int mode, int ldp, int row_off) {
    const int rows = mode == 0 ? A : B;
    const long total = (long)rows * ldp;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int r = (int)(i / ldp);
        const int k = (int)(i - (long)r * ldp);
        float v = 0.f;
        if (mode == 0) {        // out[a][t*B+b] = w[a][b][t]
            const int t = k / B, b = k - (k / B) * B;
            if (t < Tt) v = w[((long)r * B + b) * Tt + t];
        } else {                // out[b][t*A+a] = w[a][b][t]
            const int t = k / A, a = k - (k / A) * A;
            if (t < Tt) v = w[((long)a * B + r) * Tt + t];
        }
        out[(long)(row_off + r) * ldp + k] = from_f<T>(v);
    }
}

// ---------------------------------------------------------------- stem im2col
template <typename T>
__global__ void im2col_stem_kernel(const float* x, T* cols, int N, int H, int W, int Ho, int Wo, int kh, int kw,
                                   int stride, int pad, int Kpad) {
    constexpr int E = Vec16<T>::N;
    const int cpp = Kpad / E;
    const long total = (long)N * Ho * Wo * cpp;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const long pix = i / cpp;
        const int ch = (int)(i - pix * cpp);
        const int n = (int)(pix / ((long)Ho * Wo));
        const int rem = (int)(pix - (long)n * Ho * Wo);
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
        Vec16<T>::store(cols + pix * Kpad + ch * E, v);
    }
}

// ---------------------------------------------------------------- stem BN+ReLU+MaxPool(3,2,1)
template <typename T>
__global__ void stem_pool_fwd_kernel(const T* y, const float* scale, const float* shift, T* out, uint8_t* argmax,
                                     int N, int H, int W, int C, int Ho, int Wo) {
    constexpr int E = Vec16<T>::N;
    const int cpp = C / E;
    const long total = (long)N * Ho * Wo * cpp;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const long pix = i / cpp;
        const int ch = (int)(i - pix * cpp);
        const int n = (int)(pix / ((long)Ho * Wo));
        const int rem = (int)(pix - (long)n * Ho * Wo);
        const int oh = rem / Wo, ow = rem - (rem / Wo) * Wo;
        float best[E], sc[E], sh[E];
        int arg[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            best[e] = -INFINITY; arg[e] = 0;
            sc[e] = scale[ch * E + e]; sh[e] = shift[ch * E + e];
        }
        for (int di = 0; di < 3; ++di) {
            const int h = 2 * oh - 1 + di;
            if ((unsigned)h >= (unsigned)H) continue;
            for (int dj = 0; dj < 3; ++dj) {
                const int w = 2 * ow - 1 + dj;
                if ((unsigned)w >= (unsigned)W) continue;
                float v[E];
                Vec16<T>::load(y + (((long)n * H + h) * W + w) * C + ch * E, v);
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const float z = fmaxf(v[e] * sc[e] + sh[e], 0.f);
                    if (z > best[e]) { best[e] = z; arg[e] = di * 3 + dj; }
                }
            }
        }
        Vec16<T>::store(out + pix * C + ch * E, best);
#pragma unroll
        for (int e = 0; e < E; ++e) argmax[pix * C + ch * E + e] = (uint8_t)arg[e];
    }
}

template <typename T>
__global__ void stem_pool_bwd_kernel(const T* dout, const uint8_t* argmax, const T* y, const float* scale,
                                     const float* shift, T* dz, int N, int H, int W, int C, int Ho, int Wo) {
    constexpr int E = Vec16<T>::N;
    const int cpp = C / E;
    const long total = (long)N * H * W * cpp;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const long pix = i / cpp;
        const int ch = (int)(i - pix * cpp);
        const int n = (int)(pix / ((long)H * W));
        const int rem = (int)(pix - (long)n * H * W);
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

// ---------------------------------------------------------------- CenterNet head tails
struct HeadsDesc {
    int nh, Hd, od[4], orow[4], nout;
    const float* w1[4];
    const float* b1[4];
    const float* dout[4];
    float* out[4];
};

template <typename T>
__global__ void heads_fwd_kernel(const T* hid, int N, int HW, HeadsDesc d) {
    constexpr int E = Vec16<T>::N;
    __shared__ float w1s[8 * 512];
    const int Ctot = d.nh * d.Hd;
    for (int i = threadIdx.x; i < d.nout * d.Hd; i += blockDim.x) {
        int row = i / d.Hd, c = i - (i / d.Hd) * d.Hd;
        int h = 0;
        while (h + 1 < d.nh && row >= d.orow[h + 1]) ++h;
        w1s[i] = d.w1[h][(row - d.orow[h]) * d.Hd + c];
    }
    __syncthreads();
    const long total = (long)N * HW;
    for (long px = blockIdx.x * (long)blockDim.x + threadIdx.x; px < total; px += (long)gridDim.x * blockDim.x) {
        const int n = (int)(px / HW);
        const int q = (int)(px - (long)n * HW);
        const T* hp = hid + px * Ctot;
        for (int h = 0; h < d.nh; ++h) {
            float acc[4] = {0.f, 0.f, 0.f, 0.f};
            for (int c = 0; c < d.Hd; c += E) {
                float v[E];
                Vec16<T>::load(hp + h * d.Hd + c, v);
#pragma unroll
                for (int o = 0; o < 4; ++o) {
                    if (o < d.od[h]) {
                        const float* wr = w1s + (d.orow[h] + o) * d.Hd + c;
#pragma unroll
                        for (int e = 0; e < E; ++e) acc[o] += v[e] * wr[e];
                    }
                }
            }
            for (int o = 0; o < d.od[h]; ++o)
                d.out[h][((long)n * d.od[h] + o) * HW + q] = acc[o] + d.b1[h][o];
        }
    }
}

template <typename T>
__global__ void heads_bwd_data_kernel(const T* hid, int N, int HW, HeadsDesc d, T* dhid) {
    constexpr int E = Vec16<T>::N;
    __shared__ float w1s[8 * 512];
    const int Ctot = d.nh * d.Hd;
    for (int i = threadIdx.x; i < d.nout * d.Hd; i += blockDim.x) {
        int row = i / d.Hd, c = i - (i / d.Hd) * d.Hd;
        int h = 0;
        while (h + 1 < d.nh && row >= d.orow[h + 1]) ++h;
        w1s[i] = d.w1[h][(row - d.orow[h]) * d.Hd + c];
    }
    __syncthreads();
    const long total = (long)N * HW;
    for (long px = blockIdx.x * (long)blockDim.x + threadIdx.x; px < total; px += (long)gridDim.x * blockDim.x) {
        const int n = (int)(px / HW);
        const int q = (int)(px - (long)n * HW);
        for (int h = 0; h < d.nh; ++h) {
            float g[4] = {0.f, 0.f, 0.f, 0.f};
            for (int o = 0; o < d.od[h]; ++o) g[o] = d.dout[h][((long)n * d.od[h] + o) * HW + q];
            for (int c = 0; c < d.Hd; c += E) {
                float v[E], r[E];
                Vec16<T>::load(hid + px * Ctot + h * d.Hd + c, v);
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    float s = 0.f;
#pragma unroll
                    for (int o = 0; o < 4; ++o)
                        if (o < d.od[h]) s += g[o] * w1s[(d.orow[h] + o) * d.Hd + c + e];
                    r[e] = v[e] > 0.f ? s : 0.f;
                }
                Vec16<T>::store(dhid + px * Ctot + h * d.Hd + c, r);
            }
        }
    }
}

// acc layout per replica: [nout*Hd dW1][nout db1][nh*Hd db0]
template <typename T>
__global__ void heads_bwd_weight_kernel(const T* hid, const T* dhid, int N, int HW, HeadsDesc d, int ppb,
                                        double* acc, int accsz) {
    const int Ctot = d.nh * d.Hd;
    const int c = threadIdx.x;                 // one thread per hidden channel (blockDim == Ctot)
    const int h = c / d.Hd;
    const int cl = c - h * d.Hd;
    const long total = (long)N * HW;
    const long p0 = (long)blockIdx.x * ppb;
    const long p1 = min(total, p0 + ppb);
    float aw[4] = {0.f, 0.f, 0.f, 0.f};
    float ab[4] = {0.f, 0.f, 0.f, 0.f};
    float a0 = 0.f;
    for (long px = p0; px < p1; ++px) {
        const int n = (int)(px / HW);
        const int q = (int)(px - (long)n * HW);
        const float hv = to_f<T>(hid[px * Ctot + c]);
        a0 += to_f<T>(dhid[px * Ctot + c]);
#pragma unroll
        for (int o = 0; o < 4; ++o) {
            if (o < d.od[h]) {
                const float g = d.dout[h][((long)n * d.od[h] + o) * HW + q];
                aw[o] += g * hv;
                ab[o] += g;
            }
        }
    }
    double* a = acc + (long)(blockIdx.x % SCD_STAT_REPLICAS) * accsz;
    for (int o = 0; o < d.od[h]; ++o) atomic_add_f64(a + (d.orow[h] + o) * d.Hd + cl, (double)aw[o]);
    if (cl == 0)
        for (int o = 0; o < d.od[h]; ++o) atomic_add_f64(a + d.nout * d.Hd + d.orow[h] + o, (double)ab[o]);
    atomic_add_f64(a + d.nout * d.Hd + d.nout + c, (double)a0);
}

struct HeadsGrad {
    float* dw1[4];
    float* db1[4];
    float* db0[4];
};

__global__ void heads_bwd_weight_finalize_kernel(const double* acc, int accsz, HeadsDesc d, HeadsGrad g, int accumulate) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < accsz; i += gridDim.x * blockDim.x) {
        double s = 0.0;
        for (int r = 0; r < SCD_STAT_REPLICAS; ++r) s += acc[(long)r * accsz + i];
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
        *dst = accumulate ? (*dst + (float)s) : (float)s;
    }
}

bool make_desc(HeadsDesc& d, int nh, int Hd, const int* od) {
    if (nh < 1 || nh > 4 || Hd % 8 != 0) return false;
    d.nh = nh; d.Hd = Hd; d.nout = 0;
    for (int h = 0; h < 4; ++h) {
        d.od[h] = h < nh ? od[h] : 0;
        if (d.od[h] > 4) return false;
        d.orow[h] = d.nout;
        d.nout += d.od[h];
        d.w1[h] = nullptr; d.b1[h] = nullptr; d.dout[h] = nullptr; d.out[h] = nullptr;
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

inline int ew_blocks(long n) { return (int)std::min<long>(8192, std::max<long>(1, (n + 255) / 256)); }

}  // namespace

extern "C" int scd_pack_weight(int dtype, const float* w, void* out, int A, int B, int T, int mode, int ldp, int row_off,
                               void* stream) {
    const long total = (long)(mode == 0 ? A : B) * ldp;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == SCD_DT_BF16)
        hipLaunchKernelGGL((pack_weight_kernel<__bf16>), dim3(ew_blocks(total)), dim3(256), 0, st, w, (__bf16*)out, A, B,
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
    hipStream_t st = (hipStream_t)stream;
    if (Kpad % 8 || Kpad < kh * kw) return SCD_ERR_ARG;
    const long total = (long)N * Ho * Wo * (Kpad / (dtype == SCD_DT_BF16 ? 8 : 4));
    if (dtype == SCD_DT_BF16)
        hipLaunchKernelGGL((im2col_stem_kernel<__bf16>), dim3(ew_blocks(total)), dim3(256), 0, st, x, (__bf16*)cols, N, H,
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
    hipStream_t st = (hipStream_t)stream;
    const int E = dtype == SCD_DT_BF16 ? 8 : 4;
    if (C % E) return SCD_ERR_ARG;
    const long total = (long)N * Ho * Wo * (C / E);
    if (dtype == SCD_DT_BF16)
        hipLaunchKernelGGL((stem_pool_fwd_kernel<__bf16>), dim3(ew_blocks(total)), dim3(256), 0, st, (const __bf16*)y,
                           scale, shift, (__bf16*)out, argmax, N, H, W, C, Ho, Wo);
    else if (dtype == SCD_DT_F32)
        hipLaunchKernelGGL((stem_pool_fwd_kernel<float>), dim3(ew_blocks(total)), dim3(256), 0, st, (const float*)y,
                           scale, shift, (float*)out, argmax, N, H, W, C, Ho, Wo);
    else
        return SCD_ERR_ARG;
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_stem_pool_bwd(int dtype, const void* dout, const uint8_t* argmax, const void* y, const float* scale,
                                 const float* shift, void* dz, int N, int H, int W, int C, int Ho, int Wo, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    const int E = dtype == SCD_DT_BF16 ? 8 : 4;
    if (C % E) return SCD_ERR_ARG;
    const long total = (long)N * H * W * (C / E);
    if (dtype == SCD_DT_BF16)
        hipLaunchKernelGGL((stem_pool_bwd_kernel<__bf16>), dim3(ew_blocks(total)), dim3(256), 0, st,
                           (const __bf16*)dout, argmax, (const __bf16*)y, scale, shift, (__bf16*)dz, N, H, W, C, Ho, Wo);
    else if (dtype == SCD_DT_F32)
        hipLaunchKernelGGL((stem_pool_bwd_kernel<float>), dim3(ew_blocks(total)), dim3(256), 0, st, (const float*)dout,
                           argmax, (const float*)y, scale, shift, (float*)dz, N, H, W, C, Ho, Wo);
    else
        return SCD_ERR_ARG;
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_heads_fwd(int dtype, const void* hid, int N, int HW, int nh, int Hd, const int* od,
                             const float* const* w1, const float* const* b1, float* const* outs, void* stream) {
    HeadsDesc d;
    if (!make_desc(d, nh, Hd, od)) return SCD_ERR_ARG;
    for (int h = 0; h < nh; ++h) { d.w1[h] = w1[h]; d.b1[h] = b1[h]; d.out[h] = outs[h]; }
    hipStream_t st = (hipStream_t)stream;
    const long total = (long)N * HW;
    const int blocks = (int)std::min<long>(4096, (total + 255) / 256);
    if (dtype == SCD_DT_BF16)
        hipLaunchKernelGGL((heads_fwd_kernel<__bf16>), dim3(blocks), dim3(256), 0, st, (const __bf16*)hid, N, HW, d);
    else if (dtype == SCD_DT_F32)
        hipLaunchKernelGGL((heads_fwd_kernel<float>), dim3(blocks), dim3(256), 0, st, (const float*)hid, N, HW, d);
    else
        return SCD_ERR_ARG;
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_heads_bwd_data(int dtype, const void* hid, int N, int HW, int nh, int Hd, const int* od,
                                  const float* const* w1, const float* const* douts, void* dhid, void* stream) {
    HeadsDesc d;
    if (!make_desc(d, nh, Hd, od)) return SCD_ERR_ARG;
    for (int h = 0; h < nh; ++h) { d.w1[h] = w1[h]; d.dout[h] = douts[h]; }
    hipStream_t st = (hipStream_t)stream;
    const long total = (long)N * HW;
    const int blocks = (int)std::min<long>(4096, (total + 255) / 256);
    if (dtype == SCD_DT_BF16)
        hipLaunchKernelGGL((heads_bwd_data_kernel<__bf16>), dim3(blocks), dim3(256), 0, st, (const __bf16*)hid, N, HW, d,
                           (__bf16*)dhid);
    else if (dtype == SCD_DT_F32)
        hipLaunchKernelGGL((heads_bwd_data_kernel<float>), dim3(blocks), dim3(256), 0, st, (const float*)hid, N, HW, d,
                           (float*)dhid);
    else
        return SCD_ERR_ARG;
    SCD_RETURN_LAUNCH();
}

extern "C" size_t scd_heads_bwd_weight_accsize(int nh, int Hd, const int* od) {
    int nout = 0;
    for (int h = 0; h < nh; ++h) nout += od[h];
    return (size_t)SCD_STAT_REPLICAS * (nout * Hd + nout + nh * Hd) * sizeof(double);
}

extern "C" int scd_heads_bwd_weight(int dtype, const void* hid, const void* dhid, int N, int HW, int nh, int Hd,
                                    const int* od, const float* const* douts, double* acc, void* stream) {
    HeadsDesc d;
    if (!make_desc(d, nh, Hd, od)) return SCD_ERR_ARG;
    for (int h = 0; h < nh; ++h) d.dout[h] = douts[h];
    const int Ctot = nh * Hd;
    if (Ctot > 1024) return SCD_ERR_ARG;
    const int accsz = d.nout * Hd + d.nout + Ctot;
    const long total = (long)N * HW;
    const int ppb = 256;
    const int blocks = cdiv(total, ppb);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == SCD_DT_BF16)
        hipLaunchKernelGGL((heads_bwd_weight_kernel<__bf16>), dim3(blocks), dim3(Ctot), 0, st, (const __bf16*)hid,
                           (const __bf16*)dhid, N, HW, d, ppb, acc, accsz);
    else if (dtype == SCD_DT_F32)
        hipLaunchKernelGGL((heads_bwd_weight_kernel<float>), dim3(blocks), dim3(Ctot), 0, st, (const float*)hid,
                           (const float*)dhid, N, HW, d, ppb, acc, accsz);
    else
        return SCD_ERR_ARG;
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_heads_bwd_weight_finalize(const double* acc, int nh, int Hd, const int* od, float* const* dw1,
                                             float* const* db1, float* const* db0, int accumulate, void* stream) {
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
                       accsz, d, g, accumulate);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_adam_step(float* p, const float* g, float* m, float* v, long n, float lr, float beta1, float beta2,
                             float eps, float bc1, float bc2, float gscale, void* stream) {
    hipLaunchKernelGGL(adam_kernel, dim3(ew_blocks(n)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, lr, beta1,
                       beta2, eps, bc1, sqrtf(bc2), gscale);
    SCD_RETURN_LAUNCH();
}
