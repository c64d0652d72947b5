// Whole-slide tiled inference on the GPU.
//
// Reference: test.py:19-32 (grayscale: round(0.1140 c0 + 0.5870 c1 + 0.2989 c2) in float64), :38-87 (resize to
// whole 384-px strides + 2 x 64 margin, torch 'reflect' padding, then the opencv-style column fix-up:
// col[x] = col[127 - x] for x < 64 and col[x] = col[6271 - x] for 3136 <= x < 3200, clips of 512 x 512 taken
// x-major, each normalised in float64 and cast to float32), :90-135 (score > 0.3, detections projected back:
// (int(x * 384 - padLR + cx * 4 + offx), int(y * 384 - padTB + cy * 4 + offy), ratio = (4 halo - 4 minl) /
// (2 * 4 minl))).
//
// scd_slide_tiles: two launches.  (1) per (tile, slice) exact fp64 sums of the grey values (integers
// 0..255, so every sum is exact) read straight from the RGB slide through the padding / fix-up index map;
// (2) normalise: (g - mean) / sqrt(var) in float64, stored as float32 (B,1,512,512).  No padded slide is
// materialised.  scd_slide_detections: one workgroup walks the decoded (10, T, K) stack tile by tile,
// compacting the kept detections in the reference's order with wave ballots.
#include "scd_common.h"

#pragma clang fp contract(off)

namespace {

constexpr int SL_SLICES = 32;
constexpr int SL_THREADS = 256;

struct SlideGeom {
    const uint8_t* rgb;     // (H, W, C) interleaved, C >= 3
    int H, W, C;
    int tile, stride;       // 512, 384
    int clipH, clipV;       // tiles along x, along y
    int padLR, padTB;
    int resizeW;
    int fix;                // apply the opencv column fix-up (test.py:79-82)
};

__device__ __forceinline__ int reflect101(int i, int n) {
    if (i < 0) i = -i;
    if (i >= n) i = 2 * (n - 1) - i;
    return i;
}

// grey value of padded pixel (py, px)
__device__ __forceinline__ double grey_at(const SlideGeom& g, int py, int px) {
    if (g.fix) {
        if (px < 64) px = 127 - px;
        else if (px >= 3136 && px < 3200) px = 6271 - px;
    }
    int sy = reflect101(py - g.padTB, g.H), sx = reflect101(px - g.padLR, g.W);
    const uint8_t* p = g.rgb + ((long)sy * g.W + sx) * g.C;
    double v = 0.1140 * (double)p[0] + 0.5870 * (double)p[1];
    v = v + 0.2989 * (double)p[2];
    return rint(v);
}

__device__ __forceinline__ void tile_origin(const SlideGeom& g, int t, int& oy, int& ox) {
    int i = t / g.clipV, j = t - (t / g.clipV) * g.clipV;   // x-major (test.py:84-87)
    ox = i * g.stride;
    oy = j * g.stride;
}

__global__ __launch_bounds__(SL_THREADS) void slide_stats_kernel(SlideGeom g, double* part) {
    const int t = blockIdx.y, s = blockIdx.x, tid = threadIdx.x;
    int oy, ox;
    tile_origin(g, t, oy, ox);
    const int rows = (g.tile + SL_SLICES - 1) / SL_SLICES;
    double s1 = 0.0, s2 = 0.0;
    for (int r = s * rows; r < min(g.tile, (s + 1) * rows); ++r)
        for (int c = tid; c < g.tile; c += SL_THREADS) {
            double v = grey_at(g, oy + r, ox + c);
            s1 += v;
            s2 += v * v;
        }
    __shared__ double red[2][SL_THREADS / 64];
    s1 = wave_sum_d(s1);
    s2 = wave_sum_d(s2);
    if ((tid & 63) == 0) { red[0][tid >> 6] = s1; red[1][tid >> 6] = s2; }
    __syncthreads();
    if (tid == 0) {
        double a = 0.0, b = 0.0;
        for (int w = 0; w < SL_THREADS / 64; ++w) { a += red[0][w]; b += red[1][w]; }
        part[((long)t * SL_SLICES + s) * 2] = a;
        part[((long)t * SL_SLICES + s) * 2 + 1] = b;
    }
}

__global__ __launch_bounds__(SL_THREADS) void slide_apply_kernel(SlideGeom g, const double* part, float* out) {
    const int t = blockIdx.y, tid = threadIdx.x;
    __shared__ double coef[2];
    if (tid < 64) {
        double a = tid < SL_SLICES ? part[((long)t * SL_SLICES + tid) * 2] : 0.0;
        double b = tid < SL_SLICES ? part[((long)t * SL_SLICES + tid) * 2 + 1] : 0.0;
        a = wave_sum_d(a);
        b = wave_sum_d(b);
        if (tid == 0) {
            double n = (double)g.tile * g.tile;
            double mean = a / n;
            coef[0] = mean;
            coef[1] = sqrt(b / n - mean * mean);
        }
    }
    __syncthreads();
    const double mean = coef[0], sd = coef[1];
    int oy, ox;
    tile_origin(g, t, oy, ox);
    const long n = (long)g.tile * g.tile;
    float* dst = out + (long)t * n;
    for (long i = (long)blockIdx.x * SL_THREADS + tid; i < n; i += (long)gridDim.x * SL_THREADS) {
        int r = (int)(i / g.tile), c = (int)(i - (long)r * g.tile);
        dst[i] = (float)((grey_at(g, oy + r, ox + c) - mean) / sd);
    }
}

// decoded stack rows (Wrapper order, trainer/wrappers/centerOffsetResidual.py:10-23):
// 0 scores, 1 inds, 2 ys, 3 xs, 4 majx, 5 majy, 6 minl, 7 halo, 8 offx, 9 offy
__global__ __launch_bounds__(1024) void slide_detect_kernel(const float* dec, int T, int K, int stride, int padLR,
                                                            int padTB, int clipV, float thr, int* xy, double* ratio,
                                                            int* count) {
    __shared__ int wtot[16];
    __shared__ int base_s;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const long plane = (long)T * K;
    if (tid == 0) base_s = 0;
    __syncthreads();
    for (long c0 = 0; c0 < plane; c0 += 1024) {
        long q = c0 + tid;
        bool keep = false;
        int px = 0, py = 0;
        double rt = 0.0;
        if (q < plane) {
            keep = dec[q] > thr;
            int t = (int)(q / K);
            int i = t / clipV, j = t - (t / clipV) * clipV;
            double cx = dec[3 * plane + q], cy = dec[2 * plane + q];
            double ofx = dec[8 * plane + q], ofy = dec[9 * plane + q];
            px = (int)((double)(i * stride - padLR) + cx * 4.0 + ofx);
            py = (int)((double)(j * stride - padTB) + cy * 4.0 + ofy);
            double minl = (double)dec[6 * plane + q] * 4.0, halo = (double)dec[7 * plane + q] * 4.0;
            rt = (halo - minl) / (2.0 * minl);
        }
        unsigned long long bal = __ballot(keep);
        int rank = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wtot[wv] = __popcll(bal);
        __syncthreads();
        if (keep) {
            int off = base_s + rank;
            for (int w = 0; w < wv; ++w) off += wtot[w];
            xy[2 * off] = px;
            xy[2 * off + 1] = py;
            ratio[off] = rt;
        }
        __syncthreads();
        if (tid == 0) {
            int s = 0;
            for (int w = 0; w < 16; ++w) s += wtot[w];
            base_s += s;
        }
        __syncthreads();
    }
    if (tid == 0) *count = base_s;
}

}  // namespace

extern "C" size_t scd_slide_workspace(int ntiles) { return (size_t)ntiles * SL_SLICES * 2 * sizeof(double); }

extern "C" int scd_slide_tiles(const uint8_t* rgb, int H, int W, int C, int tile, int stride, int clipH, int clipV,
                               int padLR, int padTB, int fix, float* out, void* workspace, void* stream) {
    if (H < 2 || W < 2 || C < 3 || tile < 1 || stride < 1 || clipH < 1 || clipV < 1 || padLR < 0 || padTB < 0 ||
        padLR >= W || padTB >= H || (long)tile * tile >= (1L << 31))
        return SCD_ERR_ARG;
    const int resizeW = (clipH - 1) * stride + tile, resizeH = (clipV - 1) * stride + tile;
    if (resizeW > W + 2 * padLR || resizeH > H + 2 * padTB) return SCD_ERR_ARG;
    if (fix && resizeW < 3200) return SCD_ERR_ARG;   // the reference's fix-up indexes columns up to 3199
    SlideGeom g{rgb, H, W, C, tile, stride, clipH, clipV, padLR, padTB, resizeW, fix};
    hipStream_t st = (hipStream_t)stream;
    double* part = (double*)workspace;
    const int T = clipH * clipV;
    hipLaunchKernelGGL(slide_stats_kernel, dim3(SL_SLICES, T), dim3(SL_THREADS), 0, st, g, part);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(slide_apply_kernel, dim3(64, T), dim3(SL_THREADS), 0, st, g, (const double*)part, out);
    SCD_RETURN_LAUNCH();
}

extern "C" int scd_slide_detections(const float* decoded, int T, int K, int stride, int padLR, int padTB, int clipV,
                                    float thr, int* xy, double* ratio, int* count, void* stream) {
    if (T < 1 || K < 1 || clipV < 1 || (long)T * K >= (1L << 31)) return SCD_ERR_ARG;
    hipLaunchKernelGGL(slide_detect_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, decoded, T, K, stride, padLR,
                       padTB, clipV, thr, xy, ratio, count);
    SCD_RETURN_LAUNCH();
}
