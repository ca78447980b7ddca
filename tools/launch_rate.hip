// launch_rate.hip -- host cost of one hipLaunchKernelGGL on this box (the engine's C2 step is
// ~33k launches): 20000 launches of a small element-wise kernel (grid 64 x 20,
// 256 threads, eight arguments), host time per launch with the queue kept non-empty, and the
// same launches replayed from a hipGraph.
// Build: hipcc --offload-arch=gfx950 -O3 -o launch_rate launch_rate.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void k_small(unsigned* out, const unsigned* a, const unsigned* b, int n, int m, unsigned c, unsigned long long g, int logn) {
    const size_t i = ((size_t)blockIdx.y << logn) + (size_t)blockIdx.x * 256 + threadIdx.x;
    out[i] = a[i] + b[i] * c + (unsigned)g + n + m;
}

struct Big {
    unsigned v[256];  // 1 KiB kernel argument, as ConvBatch / LinMacArgs / LimbConsts
};
__global__ void k_big(unsigned* out, Big b, int logn) {
    const size_t i = ((size_t)blockIdx.y << logn) + (size_t)blockIdx.x * 256 + threadIdx.x;
    out[i] = b.v[threadIdx.x];
}

int main() {
    const int logn = 14, rows = 20, iters = 20000;
    unsigned *o, *a, *b;
    (void)hipMalloc(&o, sizeof(unsigned) * rows << logn);
    (void)hipMalloc(&a, sizeof(unsigned) * rows << logn);
    (void)hipMalloc(&b, sizeof(unsigned) * rows << logn);
    hipStream_t st;
    (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    const dim3 grid((1u << logn) / 256, rows);
    for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k_small, grid, dim3(256), 0, st, o, a, b, 1, 2, 3u, 4ull, logn);
    (void)hipStreamSynchronize(st);
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(k_small, grid, dim3(256), 0, st, o, a, b, i, 2, 3u, 4ull, logn);
    auto t1 = std::chrono::steady_clock::now();
    (void)hipStreamSynchronize(st);
    auto t2 = std::chrono::steady_clock::now();
    const double host_us = std::chrono::duration<double, std::micro>(t1 - t0).count() / iters;
    const double total_us = std::chrono::duration<double, std::micro>(t2 - t0).count() / iters;

    Big bg{};
    auto t6 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; ++i) {
        bg.v[i & 255] = i;
        hipLaunchKernelGGL(k_big, grid, dim3(256), 0, st, o, bg, logn);
    }
    auto t7 = std::chrono::steady_clock::now();
    (void)hipStreamSynchronize(st);
    std::printf("{\"big_kernarg_launch_host_us\": %.3f}\n", std::chrono::duration<double, std::micro>(t7 - t6).count() / iters);
    hipGraph_t graph;
    hipGraphExec_t exec;
    (void)hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed);
    for (int i = 0; i < 2000; ++i) hipLaunchKernelGGL(k_small, grid, dim3(256), 0, st, o, a, b, i, 2, 3u, 4ull, logn);
    (void)hipStreamEndCapture(st, &graph);
    (void)hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    (void)hipGraphLaunch(exec, st);
    (void)hipStreamSynchronize(st);
    auto t3 = std::chrono::steady_clock::now();
    for (int r = 0; r < 10; ++r) (void)hipGraphLaunch(exec, st);
    auto t4 = std::chrono::steady_clock::now();
    (void)hipStreamSynchronize(st);
    auto t5 = std::chrono::steady_clock::now();
    std::printf("{\"launch_host_us\": %.3f, \"launch_total_us\": %.3f, \"graph_host_us_per_node\": %.3f, \"graph_total_us_per_node\": %.3f}\n",
                host_us, total_us, std::chrono::duration<double, std::micro>(t4 - t3).count() / 20000,
                std::chrono::duration<double, std::micro>(t5 - t3).count() / 20000);
    return 0;
}
