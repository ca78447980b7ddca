// launch.h -- kernel launch with optional live timing.
//
// When the engine's profiler enables a kernel id, the launch goes through
// hipExtLaunchKernelGGL with a start/stop event pair: the events are stamped by the
// dispatch packet itself, so the measured time is the kernel's execution time (what
// rocprofv3 --kernel-trace reports), not the gap between two queued event markers.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "kernels.h"

extern thread_local KernelProfiler* g_prof;

template <typename F, typename... Args>
inline void prof_launch(int kid, double bytes, F kernel, dim3 grid, dim3 block, size_t lds, hipStream_t st, Args... args) {
    KernelProfiler* p = g_prof;
    if (p && (p->mask >> kid & 1u)) {
        hipEvent_t a = p->get(), b = p->get();
        hipExtLaunchKernelGGL(kernel, grid, block, (std::uint32_t)lds, st, a, b, 0u, args...);
        p->recs.push_back({a, b, kid, bytes});
    } else {
        hipLaunchKernelGGL(kernel, grid, block, lds, st, args...);
    }
}
