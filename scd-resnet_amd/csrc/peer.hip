// One-shot all-reduce of small fp64 vectors over peer memory (SyncBN statistics; networkFactory.py:128-133 turns
// SyncBatchNorm on for multi-GPU runs).  Each BN layer reduces 2C doubles (<= 4096) twice per step; through RCCL
// that is a library call per layer on the critical path.  Here every rank owns a fine-grained "mailbox" that the
// others map through hipIpc handles (xGMI on MI355X): one kernel writes the rank's vector into its slot of every
// mailbox, raises its flag (the call's epoch) in each, waits for all flags in its own mailbox and sums the slots in
// rank order -- the same bits on every rank.  Slots alternate by epoch parity, so a fast rank's next call never
// overwrites a slot a slow rank is still summing (a rank can only be one call ahead: it waits for everyone's flag).
// A slow rank is not an error: the wait is bounded only by `timeout_ms` (the host's SCD_PEER_TIMEOUT_S, 120 s by
// default -- longer than a checkpoint write or a validation pass on one rank), sleeping between polls so it holds one
// wave.  A peer that never comes (a dead process) ends the wait: the kernel records the failing epoch in *err, fills
// `data` with NaN (the step's results are visibly wrong rather than silently reduced over this rank only) and writes
// the POISON flag into its slot of every peer's mailbox, so a peer that is waiting -- or arrives later -- fails at once
// instead of after a timeout of its own, and poisons its peers in turn.  The error is sticky: every later call sees
// *err != 0, re-posts the poison, fills its data with NaN and returns without waiting, so the ranks cannot drift into
// reading slots of different epochs, and the host raises on its next poll.
// Mailbox layout: [2 parities][R slots][cap doubles] then [R] 64-bit flags.
#include <string.h>

#include "scd_common.h"

namespace {

constexpr int PEER_MAX = 8;
constexpr unsigned long long POISON = ~0ull;        // a flag no epoch reaches: "this rank has failed"

struct Boxes {
    double* box[PEER_MAX];
};

__device__ __forceinline__ unsigned long long* flags_of(double* box, int R, int cap) {
    return (unsigned long long*)(box + (size_t)2 * R * cap);
}

__global__ __launch_bounds__(256) void peer_allreduce_kernel(double* data, int n, int rank, int R, Boxes b, int cap,
                                                             unsigned long long epoch, unsigned long long* err,
                                                             unsigned long long timeout_ticks) {
    const int tid = threadIdx.x;
    const int par = (int)(epoch & 1ull);
    // failure path: NaN into the data, the poison flag into every peer's mailbox (remote stores over xGMI)
    auto fail = [&]() {
        const double qnan = __builtin_nan("");
        for (int i = tid; i < n; i += blockDim.x) data[i] = qnan;
        __threadfence_system();
        if (tid < R && tid != rank)
            __hip_atomic_store(flags_of(b.box[tid], R, cap) + rank, POISON, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    };
    // sticky failure: an earlier call failed, every later call fails at once
    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0ull) {
        fail();
        return;
    }
    // 1. this rank's vector into slot `rank` of every mailbox (remote stores over xGMI for the peers)
    for (int p = 0; p < R; ++p) {
        double* dst = b.box[p] + ((size_t)par * R + rank) * cap;
        for (int i = tid; i < n; i += blockDim.x) dst[i] = data[i];
    }
    __threadfence_system();
    __syncthreads();
    if (tid < R)
        __hip_atomic_store(flags_of(b.box[tid], R, cap) + rank, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    // 2. every rank's flag for this epoch in our own mailbox (or a peer's poison)
    __shared__ int failed;
    if (tid == 0) failed = 0;
    __syncthreads();
    if (tid < R) {
        unsigned long long* f = flags_of(b.box[rank], R, cap) + tid;
        const unsigned long long t0 = wall_clock64();
        unsigned polls = 0;
        for (;;) {
            const unsigned long long v = __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
            if (v == POISON) {                                   // the peer failed: fail now, do not wait it out
                failed = 1;
                break;
            }
            if (v >= epoch) break;
            if (wall_clock64() - t0 > timeout_ticks) {           // wall_clock64: 100 MHz constant clock
                failed = 1;
                break;
            }
            // tight polling for the common microsecond-scale skew, then back off (a rank seconds late)
            if (++polls < 4096) __builtin_amdgcn_s_sleep(2);
            else __builtin_amdgcn_s_sleep(127);
        }
    }
    __syncthreads();
    if (failed) {
        if (tid == 0) atomicCAS(err, 0ull, epoch);             // the first failing epoch
        fail();
        return;
    }
    __threadfence_system();
    // 3. the sum in rank order (identical on every rank)
    const double* mine = b.box[rank] + (size_t)par * R * cap;
    for (int i = tid; i < n; i += blockDim.x) {
        double s = 0.0;
        for (int r = 0; r < R; ++r) s += mine[(size_t)r * cap + i];
        data[i] = s;
    }
}

}  // namespace

extern "C" size_t scd_peer_mailbox_bytes(int R, int cap) {
    return (size_t)2 * R * cap * sizeof(double) + (size_t)R * sizeof(unsigned long long);
}

extern "C" int scd_peer_alloc(size_t bytes, void** ptr) {
    if (!ptr || bytes == 0) return SCD_ERR_ARG;
    hipError_t e = hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached);
    if (e != hipSuccess) return (int)e;
    return (int)hipMemset(*ptr, 0, bytes);
}

extern "C" int scd_peer_free(void* ptr) { return ptr ? (int)hipFree(ptr) : 0; }

extern "C" int scd_peer_ipc_handle(void* ptr, void* handle64) {
    if (!ptr || !handle64) return SCD_ERR_ARG;
    return (int)hipIpcGetMemHandle((hipIpcMemHandle_t*)handle64, ptr);
}

extern "C" int scd_peer_ipc_open(const void* handle64, void** ptr) {
    if (!ptr || !handle64) return SCD_ERR_ARG;
    hipIpcMemHandle_t h;
    memcpy(&h, handle64, sizeof(h));
    return (int)hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

extern "C" int scd_peer_ipc_close(void* ptr) { return ptr ? (int)hipIpcCloseMemHandle(ptr) : 0; }

extern "C" int scd_peer_allreduce_f64(double* data, int n, int rank, int R, void* const* boxes, int cap,
                                      unsigned long long epoch, unsigned long long* err, unsigned timeout_ms,
                                      void* stream) {
    if (!data || !boxes || !err || R < 1 || R > PEER_MAX || rank < 0 || rank >= R || n < 0 || n > cap || epoch == 0)
        return SCD_ERR_ARG;
    Boxes b;
    for (int i = 0; i < PEER_MAX; ++i) b.box[i] = i < R ? (double*)boxes[i] : nullptr;
    hipLaunchKernelGGL(peer_allreduce_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, data, n, rank, R, b, cap,
                       epoch, err, (unsigned long long)timeout_ms * 100000ull);
    SCD_RETURN_LAUNCH();
}
