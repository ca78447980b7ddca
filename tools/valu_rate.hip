// valu_rate.hip -- measured issue rate of the u32 VALU operations the NTT butterfly is made of
// (v_add_u32, v_min_u32, v_mul_lo_u32, v_mul_hi_u32) on the whole chip, for the VALU roofline
// of the NTT kernels.  8 independent chains per thread, 1024 blocks x 256
// threads, timed with hipEvents.  Build: hipcc --offload-arch=gfx950 -O3 -o valu_rate valu_rate.hip
#include <hip/hip_runtime.h>

#include <cstdio>

template <int OP>
__global__ void __launch_bounds__(256) k_rate(unsigned* out, unsigned seed, int iters) {
    unsigned x[8];
    unsigned long long acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = seed * (threadIdx.x + 1) + i * 0x9E3779B9u, acc[i] = x[i];
    const unsigned c = seed | 1u;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                // inline asm: exactly one instruction of the kind measured, no algebraic folding
                if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[i]) : "v"(c));
                if (OP == 1) asm volatile("v_min_u32 %0, %0, %1" : "+v"(x[i]) : "v"(c));
                if (OP == 2) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[i]) : "v"(c));
                if (OP == 3) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[i]) : "v"(c));
                if (OP == 4) {  // the 32x32 -> 64-bit multiply-add of the base conversion / key inner product
                    unsigned long long cc;
                    asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[i]), "=s"(cc) : "v"(x[i]), "v"(c));
                }
            }
    }
    unsigned s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s ^= x[i] ^ (unsigned)acc[i];
    if (s == 0x12345678u) out[0] = s;  // keeps the chains alive
}

template <int OP>
double rate(const char* name, int ops_per_step) {
    unsigned* out;
    (void)hipMalloc(&out, 4);
    const int blocks = 1024 * 8, iters = 2000;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(k_rate<OP>, dim3(blocks), dim3(256), 0, 0, out, 7u, 10);
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL(k_rate<OP>, dim3(blocks), dim3(256), 0, 0, out, 7u, iters);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double lane_ops = (double)blocks * 256 * iters * 16 * 8 * ops_per_step;
    const double r = lane_ops / (ms * 1e-3);
    std::printf("{\"op\": \"%s\", \"lane_ops_per_s\": %.4e, \"ms\": %.3f}\n", name, r, ms);
    (void)hipFree(out);
    return r;
}

int main() {
    rate<0>("v_add_u32", 1);
    rate<1>("v_min_u32", 1);
    rate<2>("v_mul_lo_u32", 1);
    rate<3>("v_mul_hi_u32", 1);
    rate<4>("v_mad_u64_u32", 1);
    return 0;
}
