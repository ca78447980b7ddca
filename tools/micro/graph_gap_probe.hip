// Per-kernel GPU cost of a chain of small dependent kernels: stream launches (host kept ahead)
// against the same chain replayed from a hipGraph, for several grid sizes.  Prints JSON.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("{\"error\": \"%s line %d\"}\n", hipGetErrorString(e), __LINE__); std::exit(1); } } while (0)

__global__ void __launch_bounds__(512) k_step(unsigned* buf, int s) {
    const unsigned v = buf[(size_t)((blockIdx.x + 1) % gridDim.x) * 512 + threadIdx.x];
    buf[(size_t)blockIdx.x * 512 + threadIdx.x] = v + s;
}

int main() {
    unsigned* buf = nullptr;
    CK(hipMalloc(&buf, (size_t)4096 * 512 * sizeof(unsigned)));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const int chain = 400;
    std::printf("{\"runs\": [");
    bool first = true;
    for (int blocks : {64, 256, 1024, 4096}) {
        for (int s = 0; s < chain; ++s) k_step<<<blocks, 512, 0, st>>>(buf, s);
        CK(hipStreamSynchronize(st));
        // stream: enqueue the whole chain behind a long first kernel so the host stays ahead
        auto t0 = std::chrono::steady_clock::now();
        for (int s = 0; s < chain; ++s) k_step<<<blocks, 512, 0, st>>>(buf, s);
        auto th = std::chrono::steady_clock::now();
        CK(hipStreamSynchronize(st));
        auto t1 = std::chrono::steady_clock::now();
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
        for (int s = 0; s < chain; ++s) k_step<<<blocks, 512, 0, st>>>(buf, s);
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        auto t2 = std::chrono::steady_clock::now();
        CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        auto t3 = std::chrono::steady_clock::now();
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
        std::printf("%s{\"blocks\": %d, \"stream_us_per_kernel\": %.3f, \"stream_host_us_per_launch\": %.3f, \"graph_us_per_kernel\": %.3f}",
                    first ? "" : ", ", blocks, std::chrono::duration<double, std::micro>(t1 - t0).count() / chain,
                    std::chrono::duration<double, std::micro>(th - t0).count() / chain,
                    std::chrono::duration<double, std::micro>(t3 - t2).count() / chain);
        first = false;
    }
    std::printf("]}\n");
    return 0;
}
