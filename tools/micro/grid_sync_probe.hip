// How long does a grid-wide barrier take on this GPU, against a kernel boundary?  A grid of B
// blocks x 512 threads (all co-resident, cooperative launch) runs S barriers; the same grid as
// S + 1 back-to-back launches of an empty kernel is the boundary's cost.  Prints JSON.
#include <hip/hip_runtime.h>
#include <hip/hip_cooperative_groups.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

namespace cg = cooperative_groups;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("{\"error\": \"%s line %d\"}\n", hipGetErrorString(e), __LINE__); std::exit(1); } } while (0)

__global__ void __launch_bounds__(512) k_sync(unsigned* buf, int steps) {
    cg::grid_group g = cg::this_grid();
    unsigned v = 0;
    for (int s = 0; s < steps; ++s) {
        buf[(size_t)blockIdx.x * 512 + threadIdx.x] = v + s;  // a vector store per thread per step
        g.sync();
        v += buf[(size_t)((blockIdx.x + 1) % gridDim.x) * 512 + threadIdx.x];  // read a neighbour's
    }
    buf[(size_t)blockIdx.x * 512 + threadIdx.x] = v;
}
// the same with a hand-written barrier: one monotonic counter, a vector atomic add per block and an
// acquire spin on a vector atomic load (no cooperative-groups machinery)
__device__ __forceinline__ void bar_sync(unsigned* bar, unsigned& gen) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned target = (gen + 1) * gridDim.x;
        __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        while (__hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) __builtin_amdgcn_s_sleep(1);
    }
    ++gen;
    __syncthreads();
}
__global__ void __launch_bounds__(512) k_sync2(unsigned* buf, unsigned* bar, int steps) {
    unsigned v = 0, gen = 0;
    for (int s = 0; s < steps; ++s) {
        buf[(size_t)blockIdx.x * 512 + threadIdx.x] = v + s;
        bar_sync(bar, gen);
        v += buf[(size_t)((blockIdx.x + 1) % gridDim.x) * 512 + threadIdx.x];
    }
    buf[(size_t)blockIdx.x * 512 + threadIdx.x] = v;
}
__global__ void __launch_bounds__(512) k_step(unsigned* buf, int s) {
    const unsigned v = buf[(size_t)((blockIdx.x + 1) % gridDim.x) * 512 + threadIdx.x];
    buf[(size_t)blockIdx.x * 512 + threadIdx.x] = v + s;
}

int main() {
    int dev = 0, coop = 0;
    CK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev));
    int per_cu = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_sync, 512, 0));
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, dev));
    std::printf("{\"cooperative\": %d, \"cus\": %d, \"blocks_per_cu\": %d, \"runs\": [", coop, p.multiProcessorCount, per_cu);
    unsigned* buf = nullptr;
    CK(hipMalloc(&buf, (size_t)4096 * 512 * sizeof(unsigned)));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    const int steps = 200;
    bool first = true;
    for (int blocks : {64, 256, 512}) {
        if (blocks > per_cu * p.multiProcessorCount) continue;
        int s_arg = steps;
        void* args[] = {&buf, &s_arg};
        for (int rep = 0; rep < 2; ++rep)
            CK(hipLaunchCooperativeKernel((const void*)k_sync, dim3(blocks), dim3(512), args, 0, st));
        CK(hipStreamSynchronize(st));
        auto t0 = std::chrono::steady_clock::now();
        CK(hipLaunchCooperativeKernel((const void*)k_sync, dim3(blocks), dim3(512), args, 0, st));
        CK(hipStreamSynchronize(st));
        auto t1 = std::chrono::steady_clock::now();
        for (int s = 0; s <= steps; ++s) k_step<<<blocks, 512, 0, st>>>(buf, s);
        CK(hipStreamSynchronize(st));
        auto t2 = std::chrono::steady_clock::now();
        for (int s = 0; s <= steps; ++s) k_step<<<blocks, 512, 0, st>>>(buf, s);
        CK(hipStreamSynchronize(st));
        auto t3 = std::chrono::steady_clock::now();
        unsigned* bar = nullptr;
        CK(hipMalloc(&bar, 64));
        CK(hipMemset(bar, 0, 64));
        void* args2[] = {&buf, &bar, &s_arg};
        CK(hipLaunchCooperativeKernel((const void*)k_sync2, dim3(blocks), dim3(512), args2, 0, st));
        CK(hipStreamSynchronize(st));
        CK(hipMemset(bar, 0, 64));
        auto t4 = std::chrono::steady_clock::now();
        CK(hipLaunchCooperativeKernel((const void*)k_sync2, dim3(blocks), dim3(512), args2, 0, st));
        CK(hipStreamSynchronize(st));
        auto t5 = std::chrono::steady_clock::now();
        CK(hipFree(bar));
        const double us_bar = std::chrono::duration<double, std::micro>(t5 - t4).count() / steps;
        const double us_sync = std::chrono::duration<double, std::micro>(t1 - t0).count() / steps;
        const double us_launch = std::chrono::duration<double, std::micro>(t3 - t2).count() / (steps + 1);
        std::printf("%s{\"blocks\": %d, \"us_per_grid_sync\": %.3f, \"us_per_atomic_barrier\": %.3f, \"us_per_kernel_boundary\": %.3f}", first ? "" : ", ", blocks, us_sync, us_bar, us_launch);
        first = false;
    }
    std::printf("]}\n");
    CK(hipFree(buf));
    return 0;
}
