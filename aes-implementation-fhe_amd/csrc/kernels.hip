// kernels.hip -- CDNA4 (gfx950) kernels of the RNS-CKKS engine.
//
// Data layout in HBM: an RNS tensor is [rows][N] uint32 with rows = npoly * nl, limb
// l = row % nl living modulo prime map.prime(l).  Wave64 / 256-thread blocks; every
// global access below is unit-stride across consecutive lanes.
#include "kernels.h"

#define CHECK_LAUNCH() (void)hipGetLastError()

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ u64 mix64(u64 z) {
    z ^= z >> 30; z *= 0xbf58476d1ce4e5b9ULL;
    z ^= z >> 27; z *= 0x94d049bb133111ebULL;
    z ^= z >> 31; return z;
}
__device__ __forceinline__ u64 prng_key(u64 seed, u64 stream) { return mix64(seed ^ mix64(stream + 0x9E3779B97F4A7C15ULL)); }
__device__ __forceinline__ u64 prng_at(u64 key, u64 ctr) { return mix64(key + (ctr + 1) * 0x9E3779B97F4A7C15ULL); }

// ------------------------------------------------------------------------------------
// NTT.  N = R * ROWS with R = 256 contiguous elements per row.  Pass "cols" runs the
// log2(ROWS) stages whose butterfly span is >= R (each column of the R x ROWS view is an
// independent ROWS-point transform); pass "rows" runs the last 8 stages inside each
// contiguous 256-element row.  Both stage the tile through LDS.
// ------------------------------------------------------------------------------------
constexpr int kR = 256;
constexpr int kColTile = 16;
constexpr int kRowsPerBlock = 4;

__global__ void __launch_bounds__(kBlock) k_ntt_cols_fwd(u32* data, int nl, LimbMap map, const PrimeConst* pc, const u32* psi,
                                                         const u32* psip, int logn) {
    extern __shared__ u32 sm[];
    const int S1 = logn - 8, ROWS = 1 << S1, LD = kColTile + 1;
    const int row = blockIdx.y;
    const int prime = map.prime(row % nl);
    const u32 q = pc[prime].q;
    const u32* w = psi + ((size_t)prime << logn);
    const u32* wp = psip + ((size_t)prime << logn);
    u32* base = data + ((size_t)row << logn) + blockIdx.x * kColTile;
    for (int e = threadIdx.x; e < ROWS * kColTile; e += kBlock) {
        int r = e / kColTile, c = e % kColTile;
        sm[r * LD + c] = base[(size_t)r * kR + c];
    }
    __syncthreads();
    for (int s = 0; s < S1; ++s) {
        const int m = 1 << s, t = ROWS >> (s + 1);
        for (int b = threadIdx.x; b < (ROWS / 2) * kColTile; b += kBlock) {
            int c = b % kColTile, p = b / kColTile;
            int i = p / t, j = p % t, r0 = 2 * i * t + j;
            u32 W = w[m + i], Wp = wp[m + i];
            u32 u = sm[r0 * LD + c];
            u32 v = shoup_mul(sm[(r0 + t) * LD + c], W, Wp, q);
            sm[r0 * LD + c] = add_mod(u, v, q);
            sm[(r0 + t) * LD + c] = sub_mod(u, v, q);
        }
        __syncthreads();
    }
    for (int e = threadIdx.x; e < ROWS * kColTile; e += kBlock) {
        int r = e / kColTile, c = e % kColTile;
        base[(size_t)r * kR + c] = sm[r * LD + c];
    }
}

__global__ void __launch_bounds__(kBlock) k_ntt_rows_fwd(u32* data, int nl, LimbMap map, const PrimeConst* pc, const u32* psi,
                                                         const u32* psip, int logn) {
    __shared__ u32 sm[kRowsPerBlock * kR];
    const int S1 = logn - 8;
    const int row = blockIdx.y;
    const int prime = map.prime(row % nl);
    const u32 q = pc[prime].q;
    const u32* w = psi + ((size_t)prime << logn);
    const u32* wp = psip + ((size_t)prime << logn);
    const int r_first = blockIdx.x * kRowsPerBlock;
    u32* base = data + ((size_t)row << logn) + (size_t)r_first * kR;
    for (int e = threadIdx.x; e < kRowsPerBlock * kR; e += kBlock) sm[e] = base[e];
    __syncthreads();
    for (int s = S1; s < logn; ++s) {
        const int m = 1 << s, t = kR >> (s - S1 + 1);
        for (int b = threadIdx.x; b < kRowsPerBlock * kR / 2; b += kBlock) {
            int rr = b / (kR / 2), p = b % (kR / 2);
            int il = p / t, j = p % t, j0 = 2 * il * t + j;
            int ig = (r_first + rr) * (kR / (2 * t)) + il;
            u32 W = w[m + ig], Wp = wp[m + ig];
            u32* x = sm + rr * kR;
            u32 u = x[j0];
            u32 v = shoup_mul(x[j0 + t], W, Wp, q);
            x[j0] = add_mod(u, v, q);
            x[j0 + t] = sub_mod(u, v, q);
        }
        __syncthreads();
    }
    for (int e = threadIdx.x; e < kRowsPerBlock * kR; e += kBlock) base[e] = sm[e];
}

__global__ void __launch_bounds__(kBlock) k_ntt_rows_inv(u32* data, int nl, LimbMap map, const PrimeConst* pc, const u32* ipsi,
                                                         const u32* ipsip, int logn) {
    __shared__ u32 sm[kRowsPerBlock * kR];
    const int S1 = logn - 8;
    const int row = blockIdx.y;
    const int prime = map.prime(row % nl);
    const u32 q = pc[prime].q;
    const u32* w = ipsi + ((size_t)prime << logn);
    const u32* wp = ipsip + ((size_t)prime << logn);
    const int r_first = blockIdx.x * kRowsPerBlock;
    u32* base = data + ((size_t)row << logn) + (size_t)r_first * kR;
    for (int e = threadIdx.x; e < kRowsPerBlock * kR; e += kBlock) sm[e] = base[e];
    __syncthreads();
    for (int s = logn - 1; s >= S1; --s) {
        const int m = 1 << s, t = kR >> (s - S1 + 1);
        for (int b = threadIdx.x; b < kRowsPerBlock * kR / 2; b += kBlock) {
            int rr = b / (kR / 2), p = b % (kR / 2);
            int il = p / t, j = p % t, j0 = 2 * il * t + j;
            int ig = (r_first + rr) * (kR / (2 * t)) + il;
            u32 W = w[m + ig], Wp = wp[m + ig];
            u32* x = sm + rr * kR;
            u32 u = x[j0], v = x[j0 + t];
            x[j0] = add_mod(u, v, q);
            x[j0 + t] = shoup_mul(u + q - v, W, Wp, q);
        }
        __syncthreads();
    }
    for (int e = threadIdx.x; e < kRowsPerBlock * kR; e += kBlock) base[e] = sm[e];
}

__global__ void __launch_bounds__(kBlock) k_ntt_cols_inv(u32* data, int nl, LimbMap map, const PrimeConst* pc, const u32* ipsi,
                                                         const u32* ipsip, int logn) {
    extern __shared__ u32 sm[];
    const int S1 = logn - 8, ROWS = 1 << S1, LD = kColTile + 1;
    const int row = blockIdx.y;
    const int prime = map.prime(row % nl);
    const PrimeConst P = pc[prime];
    const u32 q = P.q;
    const u32* w = ipsi + ((size_t)prime << logn);
    const u32* wp = ipsip + ((size_t)prime << logn);
    u32* base = data + ((size_t)row << logn) + blockIdx.x * kColTile;
    for (int e = threadIdx.x; e < ROWS * kColTile; e += kBlock) {
        int r = e / kColTile, c = e % kColTile;
        sm[r * LD + c] = base[(size_t)r * kR + c];
    }
    __syncthreads();
    for (int s = S1 - 1; s >= 0; --s) {
        const int m = 1 << s, t = ROWS >> (s + 1);
        for (int b = threadIdx.x; b < (ROWS / 2) * kColTile; b += kBlock) {
            int c = b % kColTile, p = b / kColTile;
            int i = p / t, j = p % t, r0 = 2 * i * t + j;
            u32 W = w[m + i], Wp = wp[m + i];
            u32 u = sm[r0 * LD + c], v = sm[(r0 + t) * LD + c];
            sm[r0 * LD + c] = add_mod(u, v, q);
            sm[(r0 + t) * LD + c] = shoup_mul(u + q - v, W, Wp, q);
        }
        __syncthreads();
    }
    for (int e = threadIdx.x; e < ROWS * kColTile; e += kBlock) {
        int r = e / kColTile, c = e % kColTile;
        base[(size_t)r * kR + c] = shoup_mul(sm[r * LD + c], P.ninv, P.ninv_p, q);
    }
}

// ------------------------------------------------------------------------------------
// element-wise kernels: one thread per coefficient, rows on blockIdx.y
// ------------------------------------------------------------------------------------
#define EW_PROLOGUE                                                  \
    const int row = blockIdx.y;                                      \
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;      \
    const int limb = row % nl;                                       \
    const PrimeConst P = pc[map.prime(limb)];                        \
    const size_t idx = ((size_t)row << logn) + k;                    \
    (void)limb; (void)P;

__global__ void k_add(u32* out, const u32* a, const u32* b, int nl, LimbMap map, const PrimeConst* pc, int logn) {
    EW_PROLOGUE
    out[idx] = add_mod(a[idx], b[idx], P.q);
}
__global__ void k_sub(u32* out, const u32* a, const u32* b, int nl, LimbMap map, const PrimeConst* pc, int logn) {
    EW_PROLOGUE
    out[idx] = sub_mod(a[idx], b[idx], P.q);
}
__global__ void k_neg(u32* out, const u32* a, int nl, LimbMap map, const PrimeConst* pc, int logn) {
    EW_PROLOGUE
    u32 v = a[idx];
    out[idx] = v ? P.q - v : 0;
}
__global__ void k_square(u32* out, const u32* a, int nl, LimbMap map, const PrimeConst* pc, int logn) {
    EW_PROLOGUE
    u32 v = a[idx];
    out[idx] = barrett_mul(v, v, P.q, P.mu);
}
__global__ void k_fma_poly(u32* out, const u32* a, const u32* b, const u32* c, int nl, LimbMap map, const PrimeConst* pc, int logn) {
    EW_PROLOGUE
    const size_t cidx = ((size_t)limb << logn) + k;
    out[idx] = add_mod(a[idx], barrett_mul(b[idx], c[cidx], P.q, P.mu), P.q);
}
__global__ void k_mul_poly(u32* out, const u32* in, const u32* pt, int nl, LimbMap map, const PrimeConst* pc, int logn) {
    EW_PROLOGUE
    const size_t pidx = ((size_t)limb << logn) + k;
    out[idx] = barrett_mul(in[idx], pt[pidx], P.q, P.mu);
}
__global__ void k_tensor(u32* out, const u32* a, const u32* b, int nl, LimbMap map, const PrimeConst* pc, int logn) {
    EW_PROLOGUE  // row < nl here
    const size_t off = (size_t)nl << logn;
    const u32 q = P.q, mu = P.mu;
    u32 a0 = a[idx], a1 = a[idx + off], b0 = b[idx], b1 = b[idx + off];
    out[idx] = barrett_mul(a0, b0, q, mu);
    out[idx + off] = add_mod(barrett_mul(a0, b1, q, mu), barrett_mul(a1, b0, q, mu), q);
    out[idx + 2 * off] = barrett_mul(a1, b1, q, mu);
}
__global__ void k_mul_const_half(u32* out, const u32* in, const u32* cst, int nl, LimbMap map, const PrimeConst* pc, int logn) {
    EW_PROLOGUE
    const int hi = (int)(k >> (logn - 1));
    const u32* c = cst + 4 * limb + 2 * hi;
    out[idx] = shoup_mul(in[idx], c[0], c[1], P.q);
}
__global__ void k_add_const_half(u32* out, const u32* in, const u32* cst, int nl, LimbMap map, const PrimeConst* pc, int logn) {
    EW_PROLOGUE
    const int hi = (int)(k >> (logn - 1));
    out[idx] = add_mod(in[idx], cst[2 * limb + hi], P.q);
}

// X -> X^g: NTT slot i holds a(psi^{2 brv(i) + 1}); the image at i is slot j with
// 2 brv(j) + 1 = (2 brv(i) + 1) g mod 2N
__global__ void k_automorph(u32* out, const u32* in, u64 g, int logn) {
    const int row = blockIdx.y;
    const u32 i = blockIdx.x * kBlock + threadIdx.x;
    const u32 mask2n = (2u << logn) - 1;
    const u32 e = 2u * (__brev(i) >> (32 - logn)) + 1u;
    const u32 eg = (u32)(((u64)e * (g & mask2n)) & mask2n);
    const u32 j = __brev((eg - 1u) >> 1) >> (32 - logn);
    out[((size_t)row << logn) + i] = in[((size_t)row << logn) + j];
}

// ------------------------------------------------------------------------------------
// rescale
// ------------------------------------------------------------------------------------
__global__ void k_rescale_spread(u32* v, const u32* last, int nt, u32 q_last, const PrimeConst* pc, int logn) {
    const int p = blockIdx.z, t = blockIdx.y;
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const u32 x = last[((size_t)p << logn) + k];
    const u32 q = pc[t].q;
    u32 r;
    if (x > (q_last >> 1)) {       // centred representative x - q_last < 0
        u32 neg = q_last - x;      // in (0, q_last/2]
        neg = neg % q;
        r = neg ? q - neg : 0;
    } else {
        r = x % q;
    }
    v[(((size_t)p * nt + t) << logn) + k] = r;
}
__global__ void k_rescale_finish(u32* out, const u32* x, const u32* v, const u32* qinv, int nt, int nl_in, const PrimeConst* pc,
                                 int logn) {
    const int p = blockIdx.z, t = blockIdx.y;
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const u32 q = pc[t].q;
    const u32 a = x[(((size_t)p * nl_in + t) << logn) + k];
    const u32 b = v[(((size_t)p * nt + t) << logn) + k];
    out[(((size_t)p * nt + t) << logn) + k] = shoup_mul(a + q - b, qinv[2 * t], qinv[2 * t + 1], q);
}

// ------------------------------------------------------------------------------------
// key switching
// ------------------------------------------------------------------------------------
constexpr int kMaxDigit = 32;

// one thread per coefficient; loops over the nt target rows.  Centred conversion
// (DESIGN.md §3.6): u = round(sum_i y_i / q_i) from a 32-bit fixed-point estimate
// (mu_i = floor(2^62/q_i)), ext_t = sum_i y_i qhat_i - u Q  (mod t).
__global__ void __launch_bounds__(kBlock) k_base_convert(u32* ext, const u32* x, int h, int d0, int nt, LimbMap map, int skip0,
                                                         const u32* tab, const u32* qhinv, const u32* negq, const PrimeConst* pc,
                                                         int logn) {
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;
    u32 y[kMaxDigit];
    u64 f = 0;
#pragma unroll 4
    for (int i = 0; i < h; ++i) {
        const PrimeConst Pi = pc[d0 + i];
        y[i] = shoup_mul(x[((size_t)i << logn) + k], qhinv[2 * i], qhinv[2 * i + 1], Pi.q);
        f += ((u64)y[i] * Pi.mu) >> 30;
    }
    const u32 u = (u32)((f + (1ull << 31)) >> 32);
    for (int t = 0; t < nt; ++t) {
        if (t >= skip0 && t < skip0 + h) continue;
        const PrimeConst P = pc[map.prime(t)];
        u64 acc = (u64)u * negq[t];
        const u32* tt = tab + 2 * (size_t)t;
        for (int i = 0; i < h; ++i) acc += shoup_mul(y[i], tt[2 * (size_t)i * nt], tt[2 * (size_t)i * nt + 1], P.q);
        ext[((size_t)t << logn) + k] = barrett_reduce64(acc, P.q, P.mu);
    }
}

__global__ void k_key_inner(u32* acc, const u32* ext, const u32* key, int nd, int ne, int nl, int nkey, int nks, LimbMap map,
                            const PrimeConst* pc, int logn) {
    const int x = blockIdx.y;
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const PrimeConst P = pc[map.prime(x)];
    const int krow = x < nl ? x : nks + (x - nl);
    u32 s0 = 0, s1 = 0;
    for (int j = 0; j < nd; ++j) {
        const u32 e = ext[(((size_t)j * ne + x) << logn) + k];
        const u32* kb = key + (((size_t)j * 2 * nkey + krow) << logn) + k;
        const u32* ka = kb + ((size_t)nkey << logn);
        s0 = add_mod(s0, barrett_mul(e, *kb, P.q, P.mu), P.q);
        s1 = add_mod(s1, barrett_mul(e, *ka, P.q, P.mu), P.q);
    }
    acc[((size_t)x << logn) + k] = s0;
    acc[(((size_t)ne + x) << logn) + k] = s1;
}

__global__ void k_moddown_finish(u32* out, const u32* acc, const u32* conv, const u32* pinv, const u32* add0, const u32* add1,
                                 int nl, int ne, const PrimeConst* pc, int logn) {
    const int p = blockIdx.z, t = blockIdx.y;
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const u32 q = pc[t].q;
    const u32 a = acc[(((size_t)p * ne + t) << logn) + k];
    const u32 c = conv[(((size_t)p * nl + t) << logn) + k];
    u32 r = shoup_mul(a + q - c, pinv[2 * t], pinv[2 * t + 1], q);
    const u32* add = p == 0 ? add0 : add1;
    if (add) r = add_mod(r, add[((size_t)t << logn) + k], q);
    out[(((size_t)p * nl + t) << logn) + k] = r;
}

// ------------------------------------------------------------------------------------
// sampling and key generation
// ------------------------------------------------------------------------------------
__global__ void k_sample_small(u32* out, int nl, LimbMap map, u64 seed, u64 stream, int kind, const PrimeConst* pc, int logn) {
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const u64 r = prng_at(prng_key(seed, stream), k);
    int v;
    if (kind == 0) v = (int)(r % 3) - 1;
    else v = __popcll(r & 0x1FFFFFull) - __popcll((r >> 21) & 0x1FFFFFull);
    for (int l = 0; l < nl; ++l) {
        const u32 q = pc[map.prime(l)].q;
        out[((size_t)l << logn) + k] = v >= 0 ? (u32)v : q - (u32)(-v);
    }
}
__global__ void k_sample_uniform(u32* out, int nl, LimbMap map, u64 seed, u64 stream, const PrimeConst* pc, int logn) {
    const int l = blockIdx.y;
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const int prime = map.prime(l);
    const u64 key = prng_key(seed, stream);
    const u32 q = pc[prime].q;
    out[((size_t)l << logn) + k] = (u32)(prng_at(key, ((u64)prime << logn) + k) % q);
}
__global__ void k_keygen_combine(u32* b, const u32* a, const u32* s, const u32* e, const u32* sp, const u32* gadget, int nl,
                                 LimbMap map, int glo, int ghi, const PrimeConst* pc, int logn) {
    const int l = blockIdx.y;
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const int prime = map.prime(l);
    const PrimeConst P = pc[prime];
    const size_t idx = ((size_t)l << logn) + k;
    u32 v = sub_mod(e[idx], barrett_mul(a[idx], s[((size_t)prime << logn) + k], P.q, P.mu), P.q);
    if (l >= glo && l < ghi) v = add_mod(v, shoup_mul(sp[idx], gadget[2 * l], gadget[2 * l + 1], P.q), P.q);
    b[idx] = v;
}

inline dim3 ew_grid(int logn, int rows) { return dim3((1u << logn) / kBlock, rows); }

}  // namespace

// ======================================================================================
// live timing
// ======================================================================================
static thread_local KernelProfiler* g_prof = nullptr;
void prof_set(KernelProfiler* p) { g_prof = p; }

hipEvent_t KernelProfiler::get() {
    if (!pool.empty()) {
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
    hipEvent_t e;
    (void)hipEventCreate(&e);
    return e;
}
void KernelProfiler::flush() {
    for (auto& r : recs) {
        float t = 0.f;
        (void)hipEventSynchronize(r.b);
        (void)hipEventElapsedTime(&t, r.a, r.b);
        ms[r.kid] += t;
        bytes[r.kid] += r.bytes;
        launches[r.kid] += 1;
        pool.push_back(r.a);
        pool.push_back(r.b);
    }
    recs.clear();
}
void KernelProfiler::reset() {
    flush();
    for (int k = 0; k < KID_N; ++k) ms[k] = bytes[k] = 0, launches[k] = 0;
}

namespace {
// records a start/stop event pair around one launch when its kernel id is enabled
struct ProfScope {
    KernelProfiler* p;
    hipStream_t st;
    int kid;
    double bytes;
    hipEvent_t a = nullptr;
    ProfScope(hipStream_t s, int k, double b) : p(g_prof), st(s), kid(k), bytes(b) {
        if (p && (p->mask >> kid & 1u)) {
            a = p->get();
            (void)hipEventRecord(a, st);
        } else {
            p = nullptr;
        }
    }
    ~ProfScope() {
        if (!p) return;
        hipEvent_t b = p->get();
        (void)hipEventRecord(b, st);
        p->recs.push_back({a, b, kid, bytes});
    }
};
inline double words(double w) { return 4.0 * w; }
}  // namespace

// ======================================================================================
// launch wrappers
// ======================================================================================
void launch_ntt_fwd(hipStream_t st, const DevTables& T, u32* data, int rows, int nl, LimbMap map) {
    const int S1 = T.logn - 8, ROWS = 1 << S1;
    const size_t lds = sizeof(u32) * ROWS * (kColTile + 1);
    const double io = words(2.0 * rows * (1u << T.logn));
    {
        ProfScope ps(st, KID_NTT_COLS_FWD, io);
        hipLaunchKernelGGL(k_ntt_cols_fwd, dim3(kR / kColTile, rows), dim3(kBlock), lds, st, data, nl, map, T.pc, T.psi, T.psip, T.logn);
    }
    {
        ProfScope ps(st, KID_NTT_ROWS_FWD, io);
        hipLaunchKernelGGL(k_ntt_rows_fwd, dim3(ROWS / kRowsPerBlock, rows), dim3(kBlock), 0, st, data, nl, map, T.pc, T.psi, T.psip,
                           T.logn);
    }
    CHECK_LAUNCH();
}
void launch_ntt_inv(hipStream_t st, const DevTables& T, u32* data, int rows, int nl, LimbMap map) {
    const int S1 = T.logn - 8, ROWS = 1 << S1;
    const size_t lds = sizeof(u32) * ROWS * (kColTile + 1);
    const double io = words(2.0 * rows * (1u << T.logn));
    {
        ProfScope ps(st, KID_NTT_ROWS_INV, io);
        hipLaunchKernelGGL(k_ntt_rows_inv, dim3(ROWS / kRowsPerBlock, rows), dim3(kBlock), 0, st, data, nl, map, T.pc, T.ipsi, T.ipsip,
                           T.logn);
    }
    {
        ProfScope ps(st, KID_NTT_COLS_INV, io);
        hipLaunchKernelGGL(k_ntt_cols_inv, dim3(kR / kColTile, rows), dim3(kBlock), lds, st, data, nl, map, T.pc, T.ipsi, T.ipsip, T.logn);
    }
    CHECK_LAUNCH();
}
#define EW_WRAP(bytes_words) ProfScope ps_(st, KID_ELEMENTWISE, words((double)(bytes_words) * (1u << T.logn)))
void launch_add(hipStream_t st, const DevTables& T, u32* out, const u32* a, const u32* b, int rows, int nl, LimbMap map) {
    EW_WRAP(3.0 * rows);
    hipLaunchKernelGGL(k_add, ew_grid(T.logn, rows), dim3(kBlock), 0, st, out, a, b, nl, map, T.pc, T.logn);
}
void launch_sub(hipStream_t st, const DevTables& T, u32* out, const u32* a, const u32* b, int rows, int nl, LimbMap map) {
    EW_WRAP(3.0 * rows);
    hipLaunchKernelGGL(k_sub, ew_grid(T.logn, rows), dim3(kBlock), 0, st, out, a, b, nl, map, T.pc, T.logn);
}
void launch_neg(hipStream_t st, const DevTables& T, u32* out, const u32* a, int rows, int nl, LimbMap map) {
    EW_WRAP(2.0 * rows);
    hipLaunchKernelGGL(k_neg, ew_grid(T.logn, rows), dim3(kBlock), 0, st, out, a, nl, map, T.pc, T.logn);
}
void launch_square(hipStream_t st, const DevTables& T, u32* out, const u32* a, int rows, int nl, LimbMap map) {
    EW_WRAP(2.0 * rows);
    hipLaunchKernelGGL(k_square, ew_grid(T.logn, rows), dim3(kBlock), 0, st, out, a, nl, map, T.pc, T.logn);
}
void launch_tensor(hipStream_t st, const DevTables& T, u32* out, const u32* a, const u32* b, int nl, LimbMap map) {
    ProfScope ps(st, KID_TENSOR, words(7.0 * nl * (1u << T.logn)));
    hipLaunchKernelGGL(k_tensor, ew_grid(T.logn, nl), dim3(kBlock), 0, st, out, a, b, nl, map, T.pc, T.logn);
}
void launch_mul_poly(hipStream_t st, const DevTables& T, u32* out, const u32* in, const u32* pt, int npoly, int nl, LimbMap map) {
    EW_WRAP((2.0 * npoly + 1.0) * nl);
    hipLaunchKernelGGL(k_mul_poly, ew_grid(T.logn, npoly * nl), dim3(kBlock), 0, st, out, in, pt, nl, map, T.pc, T.logn);
}
void launch_fma_poly(hipStream_t st, const DevTables& T, u32* out, const u32* a, const u32* b, const u32* c, int rows, int nl,
                     LimbMap map) {
    EW_WRAP(3.0 * rows + nl);
    hipLaunchKernelGGL(k_fma_poly, ew_grid(T.logn, rows), dim3(kBlock), 0, st, out, a, b, c, nl, map, T.pc, T.logn);
}
void launch_mul_const_half(hipStream_t st, const DevTables& T, u32* out, const u32* in, const u32* cst, int rows, int nl, LimbMap map) {
    EW_WRAP(2.0 * rows);
    hipLaunchKernelGGL(k_mul_const_half, ew_grid(T.logn, rows), dim3(kBlock), 0, st, out, in, cst, nl, map, T.pc, T.logn);
}
void launch_add_const_half(hipStream_t st, const DevTables& T, u32* out, const u32* in, const u32* cst, int rows, int nl, LimbMap map) {
    EW_WRAP(2.0 * rows);
    hipLaunchKernelGGL(k_add_const_half, ew_grid(T.logn, rows), dim3(kBlock), 0, st, out, in, cst, nl, map, T.pc, T.logn);
}
void launch_automorph(hipStream_t st, const DevTables& T, u32* out, const u32* in, u64 g, int rows) {
    ProfScope ps(st, KID_AUTOMORPH, words(2.0 * rows * (1u << T.logn)));
    hipLaunchKernelGGL(k_automorph, ew_grid(T.logn, rows), dim3(kBlock), 0, st, out, in, g, T.logn);
}
void launch_rescale_spread(hipStream_t st, const DevTables& T, u32* v, const u32* last, int npoly, int nt, u32 q_last) {
    ProfScope ps(st, KID_RESCALE, words((double)npoly * (1 + nt) * (1u << T.logn)));
    hipLaunchKernelGGL(k_rescale_spread, dim3((1u << T.logn) / kBlock, nt, npoly), dim3(kBlock), 0, st, v, last, nt, q_last, T.pc,
                       T.logn);
}
void launch_rescale_finish(hipStream_t st, const DevTables& T, u32* out, const u32* x, const u32* v, const u32* qinv, int npoly, int nt,
                           int nl_in) {
    ProfScope ps(st, KID_RESCALE, words(3.0 * npoly * nt * (1u << T.logn)));
    hipLaunchKernelGGL(k_rescale_finish, dim3((1u << T.logn) / kBlock, nt, npoly), dim3(kBlock), 0, st, out, x, v, qinv, nt, nl_in,
                       T.pc, T.logn);
}
void launch_base_convert(hipStream_t st, const DevTables& T, u32* ext, const u32* x, int h, int d0, int nt, LimbMap map, int skip0,
                         const u32* tab, const u32* qhinv, const u32* negq) {
    const int skipped = (skip0 >= 0 && skip0 < nt) ? h : 0;
    ProfScope ps(st, KID_BASE_CONVERT, words((double)(h + nt - skipped) * (1u << T.logn)));
    hipLaunchKernelGGL(k_base_convert, dim3((1u << T.logn) / kBlock), dim3(kBlock), 0, st, ext, x, h, d0, nt, map, skip0, tab, qhinv,
                       negq, T.pc, T.logn);
}
void launch_key_inner(hipStream_t st, const DevTables& T, u32* acc, const u32* ext, const u32* key, int nd, int ne, int nl, int nkey,
                      int nks, LimbMap map) {
    // ext (nd x ne) + key (nd x 2 x ne) read, acc (2 x ne) written
    ProfScope ps(st, KID_KEY_INNER, words((3.0 * nd + 2.0) * ne * (1u << T.logn)));
    hipLaunchKernelGGL(k_key_inner, ew_grid(T.logn, ne), dim3(kBlock), 0, st, acc, ext, key, nd, ne, nl, nkey, nks, map, T.pc, T.logn);
}
void launch_moddown_finish(hipStream_t st, const DevTables& T, u32* out, const u32* acc, const u32* conv, const u32* pinv,
                           const u32* add0, const u32* add1, int nl, int ne) {
    ProfScope ps(st, KID_MODDOWN, words((6.0 + (add0 ? 1 : 0) + (add1 ? 1 : 0)) * nl * (1u << T.logn)));
    hipLaunchKernelGGL(k_moddown_finish, dim3((1u << T.logn) / kBlock, nl, 2), dim3(kBlock), 0, st, out, acc, conv, pinv, add0, add1,
                       nl, ne, T.pc, T.logn);
}
void launch_sample_small(hipStream_t st, const DevTables& T, u32* out, int nl, LimbMap map, u64 seed, u64 stream, int kind) {
    ProfScope ps(st, KID_SAMPLE, words((double)nl * (1u << T.logn)));
    hipLaunchKernelGGL(k_sample_small, dim3((1u << T.logn) / kBlock), dim3(kBlock), 0, st, out, nl, map, seed, stream, kind, T.pc,
                       T.logn);
}
void launch_sample_uniform(hipStream_t st, const DevTables& T, u32* out, int nl, LimbMap map, u64 seed, u64 stream) {
    ProfScope ps(st, KID_SAMPLE, words((double)nl * (1u << T.logn)));
    hipLaunchKernelGGL(k_sample_uniform, ew_grid(T.logn, nl), dim3(kBlock), 0, st, out, nl, map, seed, stream, T.pc, T.logn);
}
void launch_keygen_combine(hipStream_t st, const DevTables& T, u32* b, const u32* a, const u32* s, const u32* e, const u32* sp,
                           const u32* gadget, int nl, LimbMap map, int glo, int ghi) {
    EW_WRAP(4.0 * nl);
    hipLaunchKernelGGL(k_keygen_combine, ew_grid(T.logn, nl), dim3(kBlock), 0, st, b, a, s, e, sp, gadget, nl, map, glo, ghi, T.pc,
                       T.logn);
}
