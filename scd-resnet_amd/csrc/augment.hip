// SCD tile augmentation on the GPU (the sample half; the target half is targets.hip).
//
// Reference: datasets/scds/scdx16p100.py:416-441 (SCD.argumentation: random x / y flips, then normalize,
// varianceJitter, gaussianNoise) and datasets/argumentations.py:38-64:
//   normalize:      mean = mean(t); var = mean((t - mean)^2); t = (t - mean) / sqrt(var)
//   varianceJitter: t * (1 + 0.05 * g),  g ~ N(0,1) one draw per tile
//   gaussianNoise:  t + n * 0.05,        n ~ N(0,1) per pixel
// The validation set uses normalize alone (scdx16p100.py:216).
//
// Two launches per batch: (1) per-(tile, slice) fp64 partial sums of x and x^2 into the caller's workspace
// (deterministic: no atomics); (2) every block re-reduces its tile's partials (64 values), derives mean and
// variance in fp64, and writes the flipped, normalised, jittered, noised tile with float4 loads / stores.
// Per-pixel noise comes from the caller (a device tensor: parity tests replay the reference's draws) or from
// a counter-based generator (splitmix64 of (seed, tile, pixel) -> Box-Muller), so the batch path needs no
// host random numbers.
#include "scd_common.h"

#pragma clang fp contract(off)

namespace {

constexpr int AUG_SLICES = 64;
constexpr int AUG_THREADS = 256;

__global__ __launch_bounds__(AUG_THREADS) void aug_stats_kernel(const float* __restrict__ in, long hw,
                                                                double* __restrict__ part) {
    const int b = blockIdx.y, s = blockIdx.x, tid = threadIdx.x;
    const long n4 = hw >> 2;
    const long per = (n4 + AUG_SLICES - 1) / AUG_SLICES;
    const long beg = s * per, end = min(n4, beg + per);
    const float4* p = (const float4*)(in + (long)b * hw);
    double s1 = 0.0, s2 = 0.0;
    for (long i = beg + tid; i < end; i += AUG_THREADS) {
        float4 v = p[i];
        s1 += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
        s2 += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
    }
    __shared__ double red[2][AUG_THREADS / 64];
    s1 = wave_sum_d(s1);
    s2 = wave_sum_d(s2);
    if ((tid & 63) == 0) { red[0][tid >> 6] = s1; red[1][tid >> 6] = s2; }
    __syncthreads();
    if (tid == 0) {
        double a = 0.0, c = 0.0;
        for (int w = 0; w < AUG_THREADS / 64; ++w) { a += red[0][w]; c += red[1][w]; }
        part[((long)b * AUG_SLICES + s) * 2] = a;
        part[((long)b * AUG_SLICES + s) * 2 + 1] = c;
    }
}

__device__ __forceinline__ unsigned long long splitmix64(unsigned long long z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// two N(0,1) values per 64-bit draw (Box-Muller on two 24-bit uniforms in (0,1])
__device__ __forceinline__ float2 gauss2(unsigned long long seed, unsigned long long ctr) {
    unsigned long long r = splitmix64(seed ^ splitmix64(ctr));
    float u1 = ((float)(r & 0xffffffu) + 1.f) * (1.f / 16777216.f);
    float u2 = (float)((r >> 24) & 0xffffffu) * (1.f / 16777216.f);
    float rad = sqrtf(-2.f * logf(u1));
    float sn, cs;
    sincosf(6.283185307179586f * u2, &sn, &cs);
    return make_float2(rad * cs, rad * sn);
}

struct AugArgs {
    const float* in;
    float* out;
    const double* part;
    const uint8_t* flips;    // (B,2): [flip x (dim 2), flip y (dim 1)]
    const float* jitter;     // (B): the factor (1 + 0.05 g), nullable = 1
    const float* noise;      // (B,H,W) N(0,1) draws, nullable -> counter-based generator
    float noise_sv;          // 0 disables the noise term
    unsigned long long seed;
    int H, W;
};

__global__ __launch_bounds__(AUG_THREADS) void aug_apply_kernel(AugArgs a) {
    const int b = blockIdx.y, tid = threadIdx.x;
    const long hw = (long)a.H * a.W;
    __shared__ float coef[2];
    if (tid < 64) {
        double s1 = a.part[((long)b * AUG_SLICES + tid) * 2], s2 = a.part[((long)b * AUG_SLICES + tid) * 2 + 1];
        s1 = wave_sum_d(s1);
        s2 = wave_sum_d(s2);
        if (tid == 0) {
            double mean = s1 / (double)hw;
            double var = s2 / (double)hw - mean * mean;
            coef[0] = (float)mean;
            coef[1] = __fsqrt_rn((float)(var > 0.0 ? var : 0.0));
        }
    }
    __syncthreads();
    const float mean = coef[0], sd = coef[1];
    const float jit = a.jitter ? a.jitter[b] : 1.f;
    const bool fx = a.flips && a.flips[b * 2], fy = a.flips && a.flips[b * 2 + 1];
    const int w4 = a.W >> 2;
    const long n4 = hw >> 2;
    const float* src = a.in + (long)b * hw;
    float* dst = a.out + (long)b * hw;
    for (long i = (long)blockIdx.x * AUG_THREADS + tid; i < n4; i += (long)gridDim.x * AUG_THREADS) {
        int y = (int)(i / w4), x4 = (int)(i - (long)y * w4);
        int sy = fy ? a.H - 1 - y : y;
        int sx4 = fx ? w4 - 1 - x4 : x4;
        float4 v = *(const float4*)(src + (long)sy * a.W + sx4 * 4);
        if (fx) v = make_float4(v.w, v.z, v.y, v.x);
        float r[4] = {v.x, v.y, v.z, v.w};
        float nz[4] = {0.f, 0.f, 0.f, 0.f};
        if (a.noise_sv != 0.f) {
            if (a.noise) {
                float4 q = *(const float4*)(a.noise + (long)b * hw + i * 4);
                nz[0] = q.x; nz[1] = q.y; nz[2] = q.z; nz[3] = q.w;
            } else {
                unsigned long long ctr = ((unsigned long long)b << 40) + (unsigned long long)i * 2;
                float2 g0 = gauss2(a.seed, ctr), g1 = gauss2(a.seed, ctr + 1);
                nz[0] = g0.x; nz[1] = g0.y; nz[2] = g1.x; nz[3] = g1.y;
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float t = __fdiv_rn(__fsub_rn(r[j], mean), sd);
            t = __fmul_rn(t, jit);
            r[j] = __fadd_rn(t, __fmul_rn(nz[j], a.noise_sv));
        }
        *(float4*)(dst + i * 4) = make_float4(r[0], r[1], r[2], r[3]);
    }
}

}  // namespace

extern "C" size_t scd_augment_workspace(int B) { return (size_t)B * AUG_SLICES * 2 * sizeof(double); }

extern "C" int scd_augment_tiles(const float* in, float* out, int B, int H, int W, const uint8_t* flips,
                                 const float* jitter, const float* noise, float noise_sv, unsigned long long seed,
                                 void* workspace, void* stream) {
    if (B < 1 || H < 1 || W < 4 || (W & 3) || (long)H * W >= (1L << 31) || in == out) return SCD_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    const long hw = (long)H * W;
    double* part = (double*)workspace;
    hipLaunchKernelGGL(aug_stats_kernel, dim3(AUG_SLICES, B), dim3(AUG_THREADS), 0, st, in, hw, part);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    AugArgs a{in, out, part, flips, jitter, noise, noise_sv, seed, H, W};
    int bx = (int)min(64L, (hw / 4 + AUG_THREADS - 1) / AUG_THREADS);
    hipLaunchKernelGGL(aug_apply_kernel, dim3(bx, B), dim3(AUG_THREADS), 0, st, a);
    SCD_RETURN_LAUNCH();
}
