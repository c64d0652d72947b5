// CenterNet training targets rendered on the GPU: the reference renders them per sample in
// Python (datasets/scds/scdx16p100.py:514-531 object loop, :575-591 drawGaussian, datasets/utility.py:11-16
// gaussianMargin2D, evaluations/intersection.py:46-63 centerThresholdRadius).  One workgroup per tile:
// phase 1 decodes the tile's objects (radius, clipped window, sigma, mask, flat index, regression row) into
// LDS (every workgroup of the tile repeats it; workgroup y == 0 also writes mask / index / regression rows),
// phase 2 walks the workgroup's share of the heatmap pixels and applies the objects IN ORDER per pixel, h = min(f32(g + h), 1)
// with g = exp(-(dx^2 + dy^2) / (2 sigma sigma)) in double -- the reference's float64 Gaussian added to the
// float32 map, rounded back, clipped after every splat -- so overlapping objects clip exactly as there.
// Grid: B tiles x gridDim.y pixel slices (enough workgroups to fill the chip at B = 32).
#include <math.h>

#include <algorithm>

#include "scd_common.h"

// numpy evaluates every product and sum separately: no fused multiply-adds in this file
#pragma clang fp contract(off)

namespace {

constexpr int MAXOBJ = 64;

struct ObjBox {
    int x, y, l, t, r, b, inside;
    double den;       // 2 * sigma * sigma
};

// centerThresholdRadius (intersection.py:46-63) in the reference's operation order, float64
__device__ double center_radius(double width, double height, double thr) {
    const double a1 = 1, b1 = height + width, c1 = width * height * (1 - thr) / (1 + thr);
    const double r1 = (b1 + sqrt(b1 * b1 - 4 * a1 * c1)) / 2;
    const double a2 = 4, b2 = 2 * (height + width), c2 = (1 - thr) * width * height;
    const double r2 = (b2 + sqrt(b2 * b2 - 4 * a2 * c2)) / 2;
    const double a3 = 4 * thr, b3 = -2 * thr * (height + width), c3 = (thr - 1) * width * height;
    const double r3 = (b3 + sqrt(b3 * b3 - 4 * a3 * c3)) / 2;
    return fmin(fmin(r1, r2), r3);
}

__global__ __launch_bounds__(256) void render_center_kernel(const float* __restrict__ locs, const int* __restrict__ counts,
                                                            int K, int H, float thr, float* __restrict__ heat,
                                                            uint8_t* __restrict__ mask, float* __restrict__ regr,
                                                            int64_t* __restrict__ inds) {
    __shared__ ObjBox box[MAXOBJ];
    const int n = blockIdx.x;
    const int cnt = min(counts[n], K);
    const float* L = locs + (size_t)n * K * 8;
    for (int k = threadIdx.x; k < K; k += blockDim.x) {
        const float* o = L + k * 8;
        ObjBox bx;
        bx.inside = 0;
        if (k < cnt) {
            const int x = (int)o[0], y = (int)o[1];               // int(loc[0]), int(loc[1]): truncation
            bx.x = x; bx.y = y;
            bx.inside = (x >= 0 && x < H && y >= 0 && y < H) ? 1 : 0;
            if (bx.inside) {
                const float major2 = o[4] * o[4] + o[5] * o[5];    // float32, as the dataset computes it
                const double radius = center_radius(2.0 * sqrt((double)major2), 2.0 * (double)o[6], (double)thr);
                const int roi = (int)ceil(radius * 2);
                bx.l = min(roi, x); bx.r = min(roi, H - x - 1);
                bx.t = min(roi, y); bx.b = min(roi, H - y - 1);
                const double sigma = radius / 3;
                bx.den = 2 * sigma * sigma;
            }
        }
        if (k < MAXOBJ) box[k] = bx;
        if (blockIdx.y != 0) continue;
        // mask / index / regression rows of every slot (slots past the count stay zero)
        mask[(size_t)n * K + k] = (uint8_t)bx.inside;
        inds[(size_t)n * K + k] = bx.inside ? (int64_t)floorf(o[1]) * H + (int64_t)floorf(o[0]) : 0;
#pragma unroll
        for (int j = 0; j < 6; ++j) regr[((size_t)n * K + k) * 6 + j] = k < cnt ? o[2 + j] : 0.f;
    }
    __syncthreads();
    float* hm = heat + (size_t)n * H * H;
    for (int p = blockIdx.y * blockDim.x + threadIdx.x; p < H * H; p += gridDim.y * blockDim.x) {
        const int py = p / H, px = p - (p / H) * H;
        float h = 0.f;
        for (int k = 0; k < cnt; ++k) {
            const ObjBox& bx = box[k];
            if (!bx.inside) continue;
            const int dx = px - bx.x, dy = py - bx.y;
            if (dx < -bx.l || dx > bx.r || dy < -bx.t || dy > bx.b) continue;
            const double g = exp(-(double)(dx * dx + dy * dy) / bx.den);
            const float s = (float)(g + (double)h);
            h = s > 1.f ? 1.f : s;                                // heatmap[heatmap > 1] = 1 (NaN stays NaN)
        }
        hm[p] = h;
    }
}

}  // namespace

extern "C" int scd_render_center_targets(const float* locs, const int* counts, int B, int K, int H, float threshold,
                                         float* heat, uint8_t* mask, float* regr, int64_t* inds, void* stream) {
    if (B < 1 || K < 1 || K > MAXOBJ || H < 1 || (long)H * H >= (1L << 31)) return SCD_ERR_ARG;
    const int slices = std::max(1, std::min(64, cdiv((long)H * H, 256)));
    hipLaunchKernelGGL(render_center_kernel, dim3(B, slices), dim3(256), 0, (hipStream_t)stream, locs, counts, K, H, threshold,
                       heat, mask, regr, inds);
    SCD_RETURN_LAUNCH();
}
