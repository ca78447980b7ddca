// launch.h -- kernel launch with optional live timing.
//
// When the engine's profiler enables a kernel id, the launch goes through
// hipExtLaunchKernelGGL with a start/stop event pair: the events are stamped by the
// dispatch packet itself, so the measured time is the kernel's execution time (what
// rocprofv3 --kernel-trace reports), not the gap between two queued event markers.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <stdexcept>
#include <string>

#include "kernels.h"

extern thread_local KernelProfiler* g_prof;
#include <atomic>
// every kernel launch of the process (aesfhe_launch_count): launch census per API call / step
extern std::atomic<unsigned long long> g_launches;
// algorithmic bytes (rounded to whole bytes) and launches of EVERY launch per kernel id, timed or
// not (aesfhe_alg_bytes): the numerator of bench.py's whole-step roofline
extern std::atomic<unsigned long long> g_alg_bytes[KID_N];
extern std::atomic<unsigned long long> g_alg_launches[KID_N];
// launch census by (C-ABI entry point, kernel) (AESFHE_CENSUS=1, aesfhe_launch_census): which API
// call issues which kernels how often -- tools/op_kernel_census.py; off: one predicted branch
extern const bool g_census_on;
extern thread_local const char* g_census_op;
void census_add(const void* fn);
size_t census_dump(char* buf, size_t cap, bool reset);
inline void alg_account(int kid, double bytes) {
    if (kid < 0 || kid >= KID_N) return;
    g_alg_bytes[kid].fetch_add((unsigned long long)(bytes + 0.5), std::memory_order_relaxed);
    g_alg_launches[kid].fetch_add(1, std::memory_order_relaxed);
}

// every launch is checked: a bad configuration fails the API call that issued it (the C-ABI
// turns the exception into an error status) instead of surfacing later as wrong data
inline void launch_check() {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw std::runtime_error(std::string("kernel launch failed: ") + hipGetErrorString(e));
}

// Host-side validation of every launch configuration BEFORE it is queued:
// a malformed dispatch must fail the API call that issued it, never reach the queue.
//  - grid: every dimension >= 1 (an empty launch is a caller bug: the wrappers return before
//    launching nothing) and within the hardware limits (x < 2^31, y / z <= 65535);
//  - block: 1 .. the kernel's __launch_bounds__ (hipFuncGetAttributes maxThreadsPerBlock);
//  - LDS: static + dynamic <= 160 KiB (gfx950 per-CU LDS);
//  - kernarg: the by-value argument block (NttAux, LinMacArgs, ConvBatch, LimbConsts ...) laid
//    out with the C alignment rules, <= kMaxKernarg.
constexpr size_t kMaxKernarg = 4096;
constexpr size_t kMaxLds = 160 * 1024;
template <typename... Args>
constexpr size_t kernarg_bytes() {
    size_t off = 0;
    ((off = (off + alignof(Args) - 1) / alignof(Args) * alignof(Args) + sizeof(Args)), ...);
    return off;
}
struct LaunchLimits {
    int max_threads;
    size_t static_lds;
};
const LaunchLimits& launch_limits(const void* fn);  // cached hipFuncGetAttributes (kernels.hip)
[[noreturn]] void launch_reject(const void* fn, const char* what, dim3 grid, dim3 block, size_t lds, size_t kernarg);
template <typename F, typename... Args>
inline void launch_validate(F kernel, dim3 grid, dim3 block, size_t lds) {
    static_assert(kernarg_bytes<Args...>() <= kMaxKernarg, "kernel argument block exceeds the kernarg limit");
    const void* fn = reinterpret_cast<const void*>(kernel);
    constexpr size_t ka = kernarg_bytes<Args...>();
    g_launches.fetch_add(1, std::memory_order_relaxed);
    if (g_census_on) census_add(fn);
    if (grid.x < 1 || grid.y < 1 || grid.z < 1 || grid.x > 0x7fffffffu || grid.y > 65535u || grid.z > 65535u)
        launch_reject(fn, "grid dimension out of range", grid, block, lds, ka);
    const LaunchLimits& lim = launch_limits(fn);
    const unsigned threads = block.x * block.y * block.z;
    if (threads < 1 || (int)threads > lim.max_threads) launch_reject(fn, "block larger than the kernel's launch bounds", grid, block, lds, ka);
    if (lds + lim.static_lds > kMaxLds) launch_reject(fn, "LDS above 160 KiB", grid, block, lds, ka);
}

template <typename F, typename... Args>
inline void prof_launch(int kid, double bytes, F kernel, dim3 grid, dim3 block, size_t lds, hipStream_t st, Args... args) {
    launch_validate<F, Args...>(kernel, grid, block, lds);
    alg_account(kid, bytes);
    KernelProfiler* p = g_prof;
    if (p && (p->mask >> kid & 1u) && (p->seen[kid]++ % p->every) == 0) {
        hipEvent_t a = p->get(), b = p->get();
        hipExtLaunchKernelGGL(kernel, grid, block, (std::uint32_t)lds, st, a, b, 0u, args...);
        p->recs.push_back({a, b, kid, bytes, 0.0});
    } else {
        hipLaunchKernelGGL(kernel, grid, block, lds, st, args...);
    }
    launch_check();
}

// launch of a kernel whose last parameter is an in-kernel clock slot (nullptr = untimed);
// `work` (NTT: butterflies) is accumulated beside the bytes for a VALU roofline
template <typename F, typename... Args>
inline void prof_launch_tsw(int kid, double bytes, double work, F kernel, dim3 grid, dim3 block, size_t lds, hipStream_t st,
                            Args... args) {
    launch_validate<F, Args..., unsigned long long*>(kernel, grid, block, lds);
    alg_account(kid, bytes);
    KernelProfiler* p = g_prof;
    unsigned long long* ts = nullptr;
    static const bool events = std::getenv("AESFHE_PROF_EVENTS") && std::getenv("AESFHE_PROF_EVENTS")[0] == '1';
    if (p && p->mask && !events) {
        // this launch's index in the process's launch order (launch_validate counted it)
        const unsigned long long idx = g_launches.load(std::memory_order_relaxed);
        const bool own = (p->mask >> kid & 1u) && (p->seen[kid]++ % p->every) == 0;
        // the successor of a sampled launch: next in the process's launch order AND on the same stream
        // (with branch threads or several contexts the next launch may be another stream's, whose
        // start says nothing about this stream's boundary)
        const bool succ = p->pend_slot >= 0 && idx == p->pend_idx + 1 && st == p->pend_stream;
        if (own || succ) ts = p->ts_slot(kid, bytes, work, own, succ ? p->pend_slot : -1);
        p->pend_slot = (own && ts) ? (int)((ts - p->d_ts) / KernelProfiler::kTsRec) : -1;
        p->pend_idx = idx;
        p->pend_stream = st;
    } else if (p && (p->mask >> kid & 1u) && (p->seen[kid]++ % p->every) == 0) {
        // AESFHE_PROF_EVENTS=1: dispatch-stamped events (~3 us longer per timed launch)
        hipEvent_t a = p->get(), b = p->get();
        hipExtLaunchKernelGGL(kernel, grid, block, (std::uint32_t)lds, st, a, b, 0u, args..., ts);
        p->recs.push_back({a, b, kid, bytes, work});
        launch_check();
        return;
    }
    hipLaunchKernelGGL(kernel, grid, block, lds, st, args..., ts);
    launch_check();
}
template <typename F, typename... Args>
inline void prof_launch_ts(int kid, double bytes, F kernel, dim3 grid, dim3 block, size_t lds, hipStream_t st, Args... args) {
    prof_launch_tsw(kid, bytes, 0.0, kernel, grid, block, lds, st, args...);
}

// device side.  Start: the first 8 blocks in dispatch order and <= ~256 evenly spaced ones
// (a skipped block -- a ModUp NTT's own-digit rows -- stamps nothing, so the first blocks alone
// can be absent).  End: <= ~2048 evenly spaced blocks plus the last 256 in dispatch order, where
// the last-finishing block almost always is (<= 256 evenly spaced ones missed it on the
// 256-thread NTT row passes' larger grids: 13.6 us live against rocprofv3's 15.4 us).  Each
// stamp is an atomicMax into one of kTsSub 128-byte lines (block id mod kTsSub), so the atomics
// of a launch's first and last waves do not queue on one address (a single line for 1,024
// sampled blocks read 36 us for a 20 us key_inner).
__device__ __forceinline__ unsigned ts_lin() { return blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z); }
__device__ __forceinline__ void ts_begin(unsigned long long* ts) {
    if (!ts || threadIdx.x != 0) return;
    const unsigned nb = gridDim.x * gridDim.y * gridDim.z, lin = ts_lin();
    const unsigned stride = nb > 256 ? nb / 256 : 1;
    if (lin < 8 || lin % stride == 0)
        atomicMax(ts + KernelProfiler::kTsLine * (lin & (KernelProfiler::kTsSub - 1)), ~(unsigned long long)__builtin_amdgcn_s_memrealtime());
}
__device__ __forceinline__ void ts_end(unsigned long long* ts) {
    if (ts) {  // uniform: every thread of the block reaches the barrier
        __syncthreads();
        const unsigned nb = gridDim.x * gridDim.y * gridDim.z, lin = ts_lin();
        const unsigned stride = nb > 2048 ? nb / 2048 : 1;
        if (threadIdx.x == 0 && (lin % stride == 0 || lin + 256 >= nb))
            atomicMax(ts + KernelProfiler::kTsLine * (KernelProfiler::kTsSub + (lin & (KernelProfiler::kTsSub - 1))),
                      (unsigned long long)__builtin_amdgcn_s_memrealtime());
    }
}
