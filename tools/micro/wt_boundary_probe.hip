// Does a kernel's dirty L2 cost its successor?  MI355X_MICROARCH.md gives a dependent kernel
// boundary as ~1.7-1.9 us + B / 6 TB/s for B bytes the predecessor leaves dirty in its XCD L2s.
// A writer kernel stores B bytes (16 B per lane) either plainly (lines stay dirty in L2 until the
// boundary's write-back) or write-through (`global_store_dwordx4 ... sc1`: each line leaves L2 with
// its store); a tiny reader kernel follows.  Per (writer, reader) pair: us, chained 200 times on one
// stream, timed with events.  Prints JSON.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("{\"error\": \"%s line %d\"}\n", hipGetErrorString(e), __LINE__); std::exit(1); } } while (0)

typedef __attribute__((ext_vector_type(4))) unsigned v4u;

template <bool WT>
__global__ void __launch_bounds__(256) k_write(uint4* out, size_t n16, unsigned s) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const uint4 v = make_uint4((unsigned)i + s, s, (unsigned)(i >> 32), 7u);
        if (WT) {
            v4u d = {v.x, v.y, v.z, v.w};
            uint4* p = out + i;
            asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" :: "v"(p), "v"(d) : "memory");
        } else {
            out[i] = v;
        }
    }
}
__global__ void __launch_bounds__(256) k_read(const uint4* in, unsigned* sink, size_t n16) {
    const size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 97 % n16;
    const uint4 v = in[i];
    if (v.w == 12345u) sink[0] = v.x;  // never true: keeps the load
}

int main() {
    const int reps = 200;
    uint4* buf = nullptr;
    unsigned* sink = nullptr;
    const size_t max_bytes = (size_t)64 << 20;
    CK(hipMalloc(&buf, max_bytes));
    CK(hipMalloc(&sink, 64));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::printf("{\"what\": \"(writer + tiny reader) per pair, us\", \"runs\": [");
    bool first = true;
    for (size_t mb : {1, 4, 16, 64}) {
        const size_t n16 = (mb << 20) / 16;
        const int blocks = (int)std::min<size_t>(2048, (n16 + 255) / 256);
        float t[3] = {0, 0, 0};
        for (int mode = 0; mode < 3; ++mode) {  // 0 plain writer + reader, 1 write-through + reader, 2 plain writer alone
            for (int warm = 0; warm < 2; ++warm) {
                CK(hipEventRecord(a, st));
                for (int r = 0; r < reps; ++r) {
                    if (mode == 1) k_write<true><<<blocks, 256, 0, st>>>(buf, n16, r);
                    else k_write<false><<<blocks, 256, 0, st>>>(buf, n16, r);
                    if (mode != 2) k_read<<<256, 256, 0, st>>>(buf, sink, n16);
                }
                CK(hipEventRecord(b, st));
                CK(hipEventSynchronize(b));
                CK(hipEventElapsedTime(&t[mode], a, b));
            }
        }
        std::printf("%s{\"MB\": %zu, \"plain_pair_us\": %.3f, \"wt_pair_us\": %.3f, \"plain_writer_alone_us\": %.3f}", first ? "" : ", ", mb,
                    1000.0 * t[0] / reps, 1000.0 * t[1] / reps, 1000.0 * t[2] / reps);
        first = false;
    }
    std::printf("]}\n");
    return 0;
}
