// Directional corner pooling (models/backbones/cornerPooling/source/{top,bottom,left,right}Pool.cpp)
// on NHWC activations.  The reference issues ~H sequential ATen launches forward and ~5H
// backward per pool; here one launch per direction: each thread owns a (n, line, channel-chunk)
// and scans the line in registers (coalesced across channels, 8 positions of loads in flight).
// Backward routes each dy to the running argmax of the same scan; ties keep the first-scanned
// position (strict '>' update, topPool.cpp:61-65); runs are summed in the reference's scan order
// (no memset, deterministic, fp32 bit-identical to the reference).  HBM-bound: fwd reads x (+ the
// addend) and writes y, bwd reads x and dy and writes dx.
#include "scd_common.h"

namespace {

// One thread owns a (n, line, 16-B channel chunk) and scans the line in registers.  Loads of the next
// U positions are issued before the current U are used (software pipeline; clamped indices, so no
// branch surrounds a load and the waitcnt pass keeps them in flight).  dir: 0 top (scan h descending),
// 1 bottom (h ascending), 2 left (w descending), 3 right (w ascending).
// VB-byte vector of T <-> floats (VB = 16: one dwordx4 per lane; 8: dwordx2, twice the lines in flight)
template <typename T, int VB> struct Vec;
template <typename T> struct Vec<T, 16> {
    typedef uint4 raw;
    static constexpr int N = Vec16<T>::N;
    __device__ static void load(const raw* p, float* f) { Vec16<T>::load(p, f); }
    __device__ static void store(void* p, const float* f) { Vec16<T>::store(p, f); }
};
template <> struct Vec<__bf16, 8> {
    typedef uint2 raw;
    static constexpr int N = 4;
    __device__ static void load(const raw* p, float* f) {
        const uint2 v = *p;
        f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
        f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
    }
    __device__ static void store(void* p, const float* f) {
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        *(bf16x4*)p = (bf16x4){(__bf16)f[0], (__bf16)f[1], (__bf16)f[2], (__bf16)f[3]};
    }
};
template <> struct Vec<float, 8> {
    typedef uint2 raw;
    static constexpr int N = 2;
    __device__ static void load(const raw* p, float* f) { f[0] = __uint_as_float(p->x); f[1] = __uint_as_float(p->y); }
    __device__ static void store(void* p, const float* f) { *(float2*)p = make_float2(f[0], f[1]); }
};

struct Line {
    long start;     // element offset of the first scanned position
    long sstep;     // signed element step between scanned positions
    int L;          // scan length
};
__device__ __forceinline__ Line line_of(int dir, long i, int N, int H, int W, int C, int E) {
    const int cpp = C / E;
    const bool vert = dir < 2;
    const int L = vert ? H : W;
    const int O = vert ? W : H;
    const int ch = (int)(i % cpp);
    const long r = i / cpp;
    const int o = (int)(r % O);
    const int n = (int)(r / O);
    const long base = vert ? (((long)n * H) * W + o) * C + ch * E : (((long)n * H + o) * W) * C + ch * E;
    const long step = vert ? (long)W * C : (long)C;
    const bool desc = (dir == 0 || dir == 2);
    Line ln;
    ln.L = L;
    ln.start = desc ? base + (long)(L - 1) * step : base;
    ln.sstep = desc ? -step : step;
    return ln;
}

template <typename T, int U, bool ADD, int VB>
__global__ __launch_bounds__(256) void cpool_fwd_kernel(int dir, const T* __restrict__ x, const T* __restrict__ addend,
                                                        T* __restrict__ y, int N, int H, int W, int C, long lines) {
    typedef Vec<T, VB> V;
    typedef typename V::raw R;
    constexpr int E = V::N;
    const long i = blockIdx.x * 256L + threadIdx.x;
    if (i >= lines) return;
    const Line ln = line_of(dir, i, N, H, W, C, E);
    const int L = ln.L;
    R cx[U], ca[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const long off = ln.start + (long)min(u, L - 1) * ln.sstep;
        cx[u] = *(const R*)(x + off);
        if constexpr (ADD) ca[u] = *(const R*)(addend + off);
    }
    float m[E];
    for (int k0 = 0; k0 < L; k0 += U) {
        R nx[U], na[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {          // prefetch the next U positions (clamped: always a valid address)
            const long off = ln.start + (long)min(k0 + U + u, L - 1) * ln.sstep;
            nx[u] = *(const R*)(x + off);
            if constexpr (ADD) na[u] = *(const R*)(addend + off);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = k0 + u;
            if (k >= L) break;
            float v[E];
            V::load(&cx[u], v);
#pragma unroll
            for (int e = 0; e < E; ++e) m[e] = (k == 0) ? v[e] : fmaxf(m[e], v[e]);
            T* dst = y + ln.start + (long)k * ln.sstep;
            if constexpr (ADD) {
                float a[E], o[E];
                V::load(&ca[u], a);
#pragma unroll
                for (int e = 0; e < E; ++e) o[e] = m[e] + a[e];
                V::store(dst, o);
            } else {
                V::store(dst, m);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) { cx[u] = nx[u]; if constexpr (ADD) ca[u] = na[u]; }
    }
}

// Backward in ONE forward register scan per line (x and dy read once, dx written once): position k is a record of
// element e iff k == 0 or x[k][e] > the running max (strict: ties keep the first-scanned position,
// topPool.cpp:61-65), and dy[k] joins the run of element e's current record.  The run is summed in scan order,
// acc = dy[r], then acc += dy[r+1], ... -- the order of the reference's scatter_add loop (topPool.cpp:56-70:
// output[argmax] += grad[k] for k along the scan), so dx is bit-identical to the reference's in fp32.  Every position
// is written once as a 16-B vector of zeros when it is scanned; a closed run's sum goes to its record position as one
// element store when the element's next record is reached (and for every element at the end of the line): records
// are few (~ln L per element on random data), and the element store follows the zero vector at that position in
// this thread's program order.
template <typename T, int U, int VB>
__global__ __launch_bounds__(256) void cpool_bwd_kernel(int dir, const T* __restrict__ x, const T* __restrict__ dy,
                                                        T* __restrict__ dx, int N, int H, int W, int C, long lines) {
    typedef Vec<T, VB> V;
    typedef typename V::raw R;
    constexpr int E = V::N;
    const long i = blockIdx.x * 256L + threadIdx.x;
    if (i >= lines) return;
    const Line ln = line_of(dir, i, N, H, W, C, E);
    const int L = ln.L;
    R cx[U], cg[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const long off = ln.start + (long)min(u, L - 1) * ln.sstep;
        cx[u] = *(const R*)(x + off);
        cg[u] = *(const R*)(dy + off);
    }
    float mv[E], acc[E], zero[E];
    int rk[E];
#pragma unroll
    for (int e = 0; e < E; ++e) { mv[e] = 0.f; acc[e] = 0.f; rk[e] = 0; zero[e] = 0.f; }
    for (int k0 = 0; k0 < L; k0 += U) {
        R nx[U], ng[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {          // prefetch the next U positions (clamped: always a valid address)
            const long off = ln.start + (long)min(k0 + U + u, L - 1) * ln.sstep;
            nx[u] = *(const R*)(x + off);
            ng[u] = *(const R*)(dy + off);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = k0 + u;
            if (k >= L) break;
            float v[E], g[E];
            V::load(&cx[u], v);
            V::load(&cg[u], g);
            V::store(dx + ln.start + (long)k * ln.sstep, zero);
            // the record test and the run state as selects; the closed runs' element stores in ONE branch region
            // per position, entered only when some element has a record here (rare after the first positions)
            bool rec[E];
            bool any = false;
#pragma unroll
            for (int e = 0; e < E; ++e) {
                rec[e] = (k == 0) || (v[e] > mv[e]);
                any |= rec[e] && k > 0;
            }
            if (any) {
#pragma unroll
                for (int e = 0; e < E; ++e)
                    if (rec[e]) dx[ln.start + (long)rk[e] * ln.sstep + e] = from_f<T>(acc[e]);
            }
#pragma unroll
            for (int e = 0; e < E; ++e) {
                mv[e] = rec[e] ? v[e] : mv[e];
                acc[e] = rec[e] ? g[e] : acc[e] + g[e];
                rk[e] = rec[e] ? k : rk[e];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) { cx[u] = nx[u]; cg[u] = ng[u]; }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) dx[ln.start + (long)rk[e] * ln.sstep + e] = from_f<T>(acc[e]);
}

#ifndef CPOOL_FWD_VB
#define CPOOL_FWD_VB 16
#endif

template <typename T>
int launch_fwd(int dir, const void* x, const void* addend, void* y, int N, int H, int W, int C, hipStream_t st) {
    constexpr int VB = CPOOL_FWD_VB;
    const long lines = (long)N * (dir < 2 ? W : H) * (C / Vec<T, VB>::N);
    if (lines == 0) return 0;
    const int grid = (int)((lines + 255) / 256);
    if (addend)
        hipLaunchKernelGGL((cpool_fwd_kernel<T, 8, true, VB>), dim3(grid), dim3(256), 0, st, dir, (const T*)x,
                           (const T*)addend, (T*)y, N, H, W, C, lines);
    else
        hipLaunchKernelGGL((cpool_fwd_kernel<T, 8, false, VB>), dim3(grid), dim3(256), 0, st, dir, (const T*)x,
                           (const T*)nullptr, (T*)y, N, H, W, C, lines);
    SCD_RETURN_LAUNCH();
}

template <typename T, int U, int VB>
int launch_bwd_v(int dir, const void* x, const void* dy, void* dx, int N, int H, int W, int C, hipStream_t st) {
    const long lines = (long)N * (dir < 2 ? W : H) * (C / Vec<T, VB>::N);
    if (lines == 0) return 0;
    const int grid = (int)((lines + 255) / 256);
    hipLaunchKernelGGL((cpool_bwd_kernel<T, U, VB>), dim3(grid), dim3(256), 0, st, dir, (const T*)x, (const T*)dy,
                       (T*)dx, N, H, W, C, lines);
    SCD_RETURN_LAUNCH();
}

// 8-B vectors (4 bf16 / 2 fp32 elements per thread: twice the lines of 16-B vectors, 94 VGPRs) with 8 positions in
// flight: 96-110 us for the (32, 128, 128, 128) bf16 pool against 127-139 us with 16-B vectors (tools/hbm_bench.py,
// round 5); the two-pass reverse-order kernel it replaces took 84 us but summed each run in reverse, not bit-identical
// to the reference
template <typename T>
int launch_bwd(int dir, const void* x, const void* dy, void* dx, int N, int H, int W, int C, hipStream_t st) {
    return launch_bwd_v<T, 8, 8>(dir, x, dy, dx, N, H, W, C, st);
}

}  // namespace

extern "C" int scd_cpool_fwd(int dtype, int dir, const void* x, const void* addend, void* y, int N, int H, int W, int C,
                             void* stream) {
    if (dir < 0 || dir > 3 || N < 0 || H < 1 || W < 1) return SCD_ERR_ARG;
    const int E = dtype == SCD_DT_BF16 ? 8 : 4;
    if (C % E) return SCD_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == SCD_DT_BF16) return launch_fwd<__bf16>(dir, x, addend, y, N, H, W, C, st);
    if (dtype == SCD_DT_F32) return launch_fwd<float>(dir, x, addend, y, N, H, W, C, st);
    return SCD_ERR_ARG;
}

extern "C" int scd_cpool_bwd(int dtype, int dir, const void* x, const void* dy, void* dx, int N, int H, int W, int C,
                             void* stream) {
    if (dir < 0 || dir > 3 || N < 0 || H < 1 || W < 1) return SCD_ERR_ARG;
    const int E = dtype == SCD_DT_BF16 ? 8 : 4;
    if (C % E) return SCD_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == SCD_DT_BF16) return launch_bwd<__bf16>(dir, x, dy, dx, N, H, W, C, st);
    if (dtype == SCD_DT_F32) return launch_bwd<float>(dir, x, dy, dx, N, H, W, C, st);
    return SCD_ERR_ARG;
}

