// kernels.hip -- CDNA4 (gfx950) kernels of the RNS-CKKS engine.
//
// Data layout in HBM: an RNS tensor is [rows][N] uint32 with rows = npoly * nl, limb
// l = row % nl living modulo prime map.prime(l).  Wave64 / 256-thread blocks; every
// global access below is unit-stride across consecutive lanes.
#include <cstring>
#include <map>
#include <mutex>
#include <string>

#include "kernels.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <stdexcept>
#include <unordered_map>

#include "launch.h"


namespace {

constexpr int kBlock = 256;


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
// a +- b on rows < common; rows in [common, rows): the longer operand alone (a, or +-b)
__global__ void k_addsub_tail(u32* out, const u32* a, const u32* b, int common, int a_longer, int sub, int nl, LimbMap map,
                              const PrimeConst* pc, int logn) {
    EW_PROLOGUE
    if (row < common) {
        out[idx] = sub ? sub_mod(a[idx], b[idx], P.q) : add_mod(a[idx], b[idx], P.q);
    } else if (a_longer) {
        out[idx] = a[idx];
    } else {
        const u32 v = b[idx];
        out[idx] = sub ? (v ? P.q - v : 0u) : v;
    }
}
// plain device copy of whole rows (16 B per lane): cheaper to issue than a runtime D2D blit
__global__ void k_copy_rows(uint4* out, const uint4* in, int logn) {
    const size_t i = ((size_t)blockIdx.y << (logn - 2)) + (size_t)blockIdx.x * kBlock + threadIdx.x;
    out[i] = in[i];
}
__global__ void k_copy_members(MemberPtrs mp, int logn) {
    const size_t i = ((size_t)blockIdx.y << (logn - 2)) + (size_t)blockIdx.x * kBlock + threadIdx.x;
    reinterpret_cast<uint4*>(mp.dst[blockIdx.z])[i] = reinterpret_cast<const uint4*>(mp.src[blockIdx.z])[i];
}
__global__ void k_add_members(u32* out, MemberPtrs mp, int n, LimbMap map, const PrimeConst* pc, int logn, int accumulate) {
    const int row = blockIdx.y;
    const size_t at = ((size_t)row << logn) + (size_t)blockIdx.x * kBlock + threadIdx.x;
    const u32 q = pc[map.prime(row)].q;
    u32 v = accumulate ? out[at] : 0u;
    for (int s = 0; s < n; ++s) v = add_mod(v, mp.src[s][at], q);
    out[at] = v;
}
__global__ void k_tensor_ptrs(u32* out, TensorPtrs tp, int nl, LimbMap map, const PrimeConst* pc, int logn) {
    const int row = blockIdx.y;
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const int m = row / nl, limb = row - m * nl;
    const PrimeConst P = pc[map.prime(limb)];
    const size_t off = (size_t)nl << logn, idx = ((size_t)limb << logn) + k;
    const u32* a = tp.a[m];
    const u32* b = tp.b[m];
    out += (size_t)m * 3 * off;
    const u32 q = P.q, mu = P.mu;
    const u32 a0 = a[idx], a1 = a[idx + off], b0 = b[idx], b1 = b[idx + off];
    out[idx] = barrett_mul(a0, b0, q, mu);
    out[idx + off] = add_mod(barrett_mul(a0, b1, q, mu), barrett_mul(a1, b0, q, mu), q);
    out[idx + 2 * off] = barrett_mul(a1, b1, q, mu);
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
// out row (poly, limb) = sum_{i < n} in_i (.) pt_i over n <= kMaxMembers ciphertext x plaintext products
// (the masked sums of MixColumns' entry, MixColFinal.sr_entry): 64-bit sums of the 60-bit products, one
// reduction -- one launch for what n lazy plaintext products and n - 1 additions did
__global__ void k_mul_poly_sum(u32* out, PtSumArgs a, int n, int nl, LimbMap map, const PrimeConst* pc, int logn) {
    EW_PROLOGUE
    const size_t pidx = ((size_t)limb << logn) + k;
    u64 acc = 0;
    for (int i = 0; i < n; ++i) acc += (u64)a.in[i][idx] * a.pt[i][pidx];
    out[idx] = reduce64(acc, P.q, P.mu, P.r32);
}
__global__ void k_tensor(u32* out, const u32* a, const u32* b, int nl, LimbMap map, const PrimeConst* pc, int logn) {
    // row = m * nl + limb: ciphertext m of a stacked batch ([m][2][nl] in, [m][3][nl] out)
    const int row = blockIdx.y;
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const int m = row / nl, limb = row - m * nl;
    const PrimeConst P = pc[map.prime(limb)];
    const size_t off = (size_t)nl << logn, idx = ((size_t)limb << logn) + k;
    a += (size_t)m * 2 * off, b += (size_t)m * 2 * off, out += (size_t)m * 3 * off;
    const u32 q = P.q, mu = P.mu;
    u32 a0 = a[idx], a1 = a[idx + off], b0 = b[idx], b1 = b[idx + off];
    out[idx] = barrett_mul(a0, b0, q, mu);
    out[idx + off] = add_mod(barrett_mul(a0, b1, q, mu), barrett_mul(a1, b0, q, mu), q);
    out[idx + 2 * off] = barrett_mul(a1, b1, q, mu);
}
// in: polys of src_nl limbs (>= nl; the first nl of each are read), out: polys of nl limbs
__global__ void k_mul_const_half(u32* out, const u32* in, LimbConsts cst, int nl, int src_nl, LimbMap map, const PrimeConst* pc,
                                 int logn) {
    EW_PROLOGUE
    const int hi = (int)(k >> (logn - 1));
    const u32* c = cst.v + 4 * limb + 2 * hi;
    const size_t sidx = ((size_t)((row / nl) * src_nl + limb) << logn) + k;
    out[idx] = shoup_mul(in[sidx], c[0], c[1], P.q);
}
__global__ void k_mul_const_half_members(u32* out, MemberPtrs mp, LimbConsts cst, int rows, int nl, int src_nl, LimbMap map,
                                         const PrimeConst* pc, int logn) {
    const int m = blockIdx.z;
    const u32* in = mp.src[m];
    out += ((size_t)m * rows) << logn;
    EW_PROLOGUE
    const int hi = (int)(k >> (logn - 1));
    const u32* c = cst.v + 4 * limb + 2 * hi;
    const size_t sidx = ((size_t)((row / nl) * src_nl + limb) << logn) + k;
    out[idx] = shoup_mul(in[sidx], c[0], c[1], P.q);
}
__global__ void k_add_const_half(u32* out, const u32* in, LimbConsts cst, int nl, LimbMap map, const PrimeConst* pc, int logn) {
    EW_PROLOGUE
    const int hi = (int)(k >> (logn - 1));
    out[idx] = add_mod(in[idx], cst.v[2 * limb + hi], P.q);
}

// out = ka a + s b + c: ka a Gaussian-integer constant (Shoup pairs per limb and slot half), b
// optional with sign s = +-1, c an additive constant on the first polynomial of every member
// (per polys per member) -- EvalMod's 2 T_a T_b - T_(a-b) / 2 T^2 - 1 and add_scalar in one launch
__global__ void k_lincomb(u32* out, const u32* a, LimbConsts ka, const u32* b, int bsign, LimbConsts cadd, int has_c, int per, int nl,
                          LimbMap map, const PrimeConst* pc, int logn) {
    EW_PROLOGUE
    const int hi = (int)(k >> (logn - 1));
    const u32* c = ka.v + 4 * limb + 2 * hi;
    u32 v = shoup_mul(a[idx], c[0], c[1], P.q);
    if (b) v = bsign > 0 ? add_mod(v, b[idx], P.q) : sub_mod(v, b[idx], P.q);
    if (has_c && (row / nl) % per == 0) v = add_mod(v, cadd.v[2 * limb + hi], P.q);
    out[idx] = v;
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
// ModRaise from the two base limbs (q0, q1): x = x0 + q0 ((x1 - x0) q0^{-1} mod q1) in
// [0, q0 q1), centred (x - q0 q1 when x > q0 q1 / 2), reduced mod every target prime
__global__ void k_crt2_spread(u32* v, const u32* src, int nt, u32 q0, u32 q1, u32 q0inv, u32 q0inv_p, const PrimeConst* pc,
                              int logn) {
    const int p = blockIdx.z, t = blockIdx.y;
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const u32 x0 = src[((size_t)(2 * p) << logn) + k], x1 = src[((size_t)(2 * p + 1) << logn) + k];
    const u32 d = x1 >= x0 % q1 ? x1 - x0 % q1 : x1 + q1 - x0 % q1;
    const u32 y = shoup_mul(d, q0inv, q0inv_p, q1);
    const u64 Q = (u64)q0 * q1, x = (u64)x0 + (u64)q0 * y;
    const PrimeConst P = pc[t];
    u32 r;
    if (x > (Q >> 1)) {  // negative representative x - Q
        const u32 m = reduce64(Q - x, P.q, P.mu, P.r32);
        r = m ? P.q - m : 0;
    } else {
        r = reduce64(x, P.q, P.mu, P.r32);
    }
    v[(((size_t)p * nt + t) << logn) + k] = r;
}
// ------------------------------------------------------------------------------------
// key switching
// ------------------------------------------------------------------------------------
// One launch converts every group (ModUp: each digit; ModDown: each polynomial).  Grid
// (N / 256, target chunks of kConvTargets, groups).  Each thread recomputes the h values
// y_i = x_i qhat_i^{-1} (kept in VGPRs: fixed-size guarded unroll, no scratch) and the
// centred overflow estimate u = round(sum y_i / q_i), then emits its chunk of targets:
// ext_t = sum_i y_i [qhat_i]_t + u [-Q]_t  (mod t).
// The block's constants (source primes, qhat^{-1}, the h x kConvTargets table slice, -Q,
// target primes) are staged in LDS (behind the residue loads): read from global memory next to the stores to
// ext they would be re-fetched, one dependent load per multiply-add.
#ifndef AESFHE_CONV_TARGETS
#define AESFHE_CONV_TARGETS 16
#endif
constexpr int kConvTargets = AESFHE_CONV_TARGETS;
// H sources, compile-time.  The block's source residues are loaded FIRST, then the weight
// tables staged in LDS behind the barrier: the two memory latencies overlap instead of the
// residue loads waiting for the table loads and the barrier.  Targets outside [t0, t1) or
// inside the own range compute on zero weights and are not stored
__device__ __forceinline__ void conv_stage(const ConvBatch& cb, int gi, int h, int d0, int t0, int t1, int nt, LimbMap map,
                                           const PrimeConst* pc, u32 (*s_w)[kMaxConvH], u32 (*s_tq)[4], u32 (*s_src)[4]) {
    const int tid = threadIdx.x;
    for (int x = tid; x < kConvTargets * kMaxConvH; x += kBlock) {
        const int tl = x / kMaxConvH, i = x % kMaxConvH, t = t0 + tl;
        s_w[tl][i] = (i < h && t < t1) ? cb.tab[gi][2 * ((size_t)i * nt + t)] : 0u;
    }
    for (int tl = tid; tl < kConvTargets; tl += kBlock) {
        const int t = t0 + tl;
        if (t < t1) {
            const PrimeConst P = pc[map.prime(t)];
            s_tq[tl][0] = P.q, s_tq[tl][1] = P.mu, s_tq[tl][2] = P.r32, s_tq[tl][3] = cb.negq[gi][t];
        }
    }
    for (int i = tid; i < h; i += kBlock) {
        const int sp = cb.split[gi];
        const PrimeConst P = pc[(sp > 0 && i >= sp) ? cb.d1[gi] + (i - sp) : d0 + i];
        s_src[i][0] = P.q, s_src[i][1] = P.mu, s_src[i][2] = cb.qhinv[gi][2 * i], s_src[i][3] = cb.qhinv[gi][2 * i + 1];
    }
}
// V consecutive coefficients per thread (1 or 2: one 4- / 8-byte access per source and target
// row; 4 needs 260 VGPRs at H = 16 and spills): each LDS-staged weight then feeds V multiply-adds, and a launch issues V times
// fewer load / store instructions; the arithmetic per coefficient is unchanged (bit-exact)
template <int V>
struct ConvVec;
template <>
struct ConvVec<1> {
    using T = u32;
    static __device__ __forceinline__ void get(const T& t, u32* o) { o[0] = t; }
    static __device__ __forceinline__ T make(const u32* o) { return o[0]; }
};
template <>
struct ConvVec<2> {
    using T = uint2;
    static __device__ __forceinline__ void get(const T& t, u32* o) { o[0] = t.x, o[1] = t.y; }
    static __device__ __forceinline__ T make(const u32* o) { return make_uint2(o[0], o[1]); }
};
template <int H, int V>
__device__ __forceinline__ void conv_body(const ConvBatch& cb, int gi, int t0, int t1, int nt, LimbMap map, const PrimeConst* pc, int logn,
                                          u32 (*s_w)[kMaxConvH], u32 (*s_tq)[4], u32 (*s_src)[4]) {
    using CV = ConvVec<V>;
    const u32* __restrict__ x = cb.src[gi];
    u32* __restrict__ ext = cb.dst[gi];
    const int skip0 = cb.skip0[gi];
    const size_t k = ((size_t)blockIdx.x * kBlock + threadIdx.x) * V;
    u32 y[H][V];
#pragma unroll
    for (int i = 0; i < H; ++i) CV::get(*reinterpret_cast<const typename CV::T*>(x + ((size_t)i << logn) + k), y[i]);
    conv_stage(cb, gi, H, cb.d0[gi], t0, t1, nt, map, pc, s_w, s_tq, s_src);
    __syncthreads();
    u32 u[V];
    {
        u64 f[V] = {};
        const bool pre = cb.pre != 0;  // block-uniform
#pragma unroll
        for (int i = 0; i < H; ++i) {
            const u32 q = s_src[i][0], mu = s_src[i][1], w = s_src[i][2], wp = s_src[i][3];
#pragma unroll
            for (int v = 0; v < V; ++v) {
                if (!pre) y[i][v] = shoup_mul(y[i][v], w, wp, q);
                f[v] += ((u64)y[i][v] * mu) >> 29;  // y_i / q_i in 32.32 fixed point (mu = 2^61 / q)
            }
        }
#pragma unroll
        for (int v = 0; v < V; ++v) u[v] = (u32)((f[v] + (1ull << 31)) >> 32);
    }
#pragma unroll
    for (int tl = 0; tl < kConvTargets; ++tl) {
        const int t = t0 + tl;
        if (t >= t1) break;
        const u32 q = s_tq[tl][0], r32 = s_tq[tl][2];
        // plain 32x32 -> 64-bit multiply-adds (v_mad_u64_u32); y_i < q_i < 2^30 (fully reduced)
        // and w < q_t < 2^30, so each product is below 2^60 and the u * (-Q) start below 2^35:
        // up to 15 sources sum below 2^64 with no fold (the conversion's kernel is VALU-bound,
        // the fold was ~1/5 of its per-target work); only H = 16 folds once, after eight
        u64 acc[V];
#pragma unroll
        for (int v = 0; v < V; ++v) acc[v] = (u64)u[v] * s_tq[tl][3];
#pragma unroll
        for (int i = 0; i < H; ++i) {
            const u32 w = s_w[tl][i];
#pragma unroll
            for (int v = 0; v < V; ++v) {
                if (H > 15 && i == 8) acc[v] = fold64(acc[v], q, r32);
                acc[v] += (u64)y[i][v] * w;
            }
        }
        if (t < skip0 || t >= skip0 + H) {
            u32 o[V];
#pragma unroll
            for (int v = 0; v < V; ++v) o[v] = reduce64(acc[v], q, s_tq[tl][1], r32);
            *reinterpret_cast<typename CV::T*>(ext + ((size_t)t << logn) + k) = CV::make(o);
        }
    }
}
template <int V>
__global__ void __launch_bounds__(kBlock) k_base_convert(ConvBatch cb, int nt, LimbMap map, const PrimeConst* pc, int logn,
                                                         unsigned long long* ts) {
    const int gi = blockIdx.z;
    const int h = cb.h[gi], skip0 = cb.skip0[gi];
    const int t0 = blockIdx.y * kConvTargets, t1 = min(t0 + kConvTargets, nt);
    if (t0 >= skip0 && t1 <= skip0 + h) return;  // chunk entirely inside the own range
    ts_begin(ts);
    __shared__ u32 s_w[kConvTargets][kMaxConvH];
    __shared__ u32 s_tq[kConvTargets][4];  // q, mu, r32, -Q mod q
    __shared__ u32 s_src[kMaxConvH][4];    // q, mu, qhat^-1, Shoup companion
    switch (h) {
#define CONV_CASE(H) \
    case H: conv_body<H, V>(cb, gi, t0, t1, nt, map, pc, logn, s_w, s_tq, s_src); break;
        CONV_CASE(1) CONV_CASE(2) CONV_CASE(3) CONV_CASE(4) CONV_CASE(5) CONV_CASE(6) CONV_CASE(7) CONV_CASE(8)
        CONV_CASE(9) CONV_CASE(10) CONV_CASE(11) CONV_CASE(12) CONV_CASE(13) CONV_CASE(14) CONV_CASE(15) CONV_CASE(16)
#undef CONV_CASE
        default: break;
    }
    ts_end(ts);
}

// digit j's own limbs (x < nl, x / alpha == j) come straight from the NTT-form input d
// NTT-domain index read by the automorphism X -> X^g at output index i (bit-reversed order)
__device__ __forceinline__ u32 galois_src(u32 i, u64 g, int logn) {
    const u32 mask2n = (2u << logn) - 1;
    const u32 e = 2u * (__brev(i) >> (32 - logn)) + 1u;
    const u32 eg = (u32)(((u64)e * (g & mask2n)) & mask2n);
    return __brev((eg - 1u) >> 1) >> (32 - logn);
}

// g != 0: the inputs (ext and d) are read through the automorphism X -> X^g -- a hoisted
// rotation: one ModUp of c1 serves every rotation of the same ciphertext
// four consecutive coefficients per thread: 16-byte key / ext / acc accesses (the kernel is
// HBM-bound on the key and ext reads); g != 0 gathers ext and d through X -> X^g.
// ND > 0: the digit count is a compile-time constant, so the digit loop unrolls and every digit's
// key and ext loads are in flight together (with the run-time bound each iteration waited for
// its own loads: one memory round trip per digit); ND = 0 keeps the run-time loop
template <int NBM, int ND = 0>
__global__ void __launch_bounds__(kBlock) k_key_inner(u32* acc, const u32* ext, const u32* d, const u32* key, int nd, int ne, int nl,
                                                      int alpha, int nkey, int nks, u64 g, LimbMap map, const PrimeConst* pc, int logn,
                                                      int nb, size_t ext_ms, size_t d_ms, size_t acc_ms, KsFold fold, int accum,
                                                      unsigned long long* ts) {
    ts_begin(ts);
    const int x = blockIdx.y;
    const size_t k = ((size_t)blockIdx.x * kBlock + threadIdx.x) * 4;
    u32 ks[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) ks[v] = g ? galois_src((u32)(k + v), g, logn) : (u32)(k + v);
    const PrimeConst P = pc[map.prime(x)];
    const int krow = x < nl ? x : nks + (x - nl);
    const int own = x < nl ? x / alpha : -1;
    // 64-bit multiply-adds (operands < q < 2^30: eight products fit beside a folded sum), folded every 8 digits;
    // the key residues are loaded once for every batched ciphertext
    u64 s0[NBM][4] = {}, s1[NBM][4] = {};
    const int ndd = ND > 0 ? ND : nd;
#pragma unroll
    for (int j = 0; j < ndd; ++j) {
        if (j && (j & 7) == 0) {
#pragma unroll
            for (int m = 0; m < NBM; ++m)
#pragma unroll
                for (int v = 0; v < 4; ++v) s0[m][v] = fold64(s0[m][v], P.q, P.r32), s1[m][v] = fold64(s1[m][v], P.q, P.r32);
        }
        const size_t kr = (((size_t)j * 2 * nkey + krow) << logn) + k;
        const uint4 vb = *reinterpret_cast<const uint4*>(key + kr);
        const uint4 va = *reinterpret_cast<const uint4*>(key + kr + ((size_t)nkey << logn));
        const u32 kb4[4] = {vb.x, vb.y, vb.z, vb.w}, ka4[4] = {va.x, va.y, va.z, va.w};
#pragma unroll
        for (int m = 0; m < NBM; ++m) {
            if (m >= nb) break;
            u32 e[4];
            if (fold.ta[0] && j == own) {  // tensor mode (g == 0): the own digit's c2 = a1 (.) b1, formed here
                const size_t at = ((size_t)(fold.tnl + x) << logn) + k;
                const uint4 a = *reinterpret_cast<const uint4*>(fold.ta[m] + at), b = *reinterpret_cast<const uint4*>(fold.tb[m] + at);
                e[0] = barrett_mul(a.x, b.x, P.q, P.mu), e[1] = barrett_mul(a.y, b.y, P.q, P.mu);
                e[2] = barrett_mul(a.z, b.z, P.q, P.mu), e[3] = barrett_mul(a.w, b.w, P.q, P.mu);
            } else if (fold.rev_d && j == own) {  // (g == 0) the own digit's d read reversed: element v <- word N - 1 - (k + v)
                const uint4 t = *reinterpret_cast<const uint4*>(d + m * d_ms + ((size_t)x << logn) + ((size_t)1 << logn) - 4 - k);
                e[0] = t.w, e[1] = t.z, e[2] = t.y, e[3] = t.x;
            } else {
                const u32* src = j == own ? d + m * d_ms + ((size_t)x << logn) : ext + m * ext_ms + (((size_t)j * ne + x) << logn);
                if (g) {
#pragma unroll
                    for (int v = 0; v < 4; ++v) e[v] = src[ks[v]];
                } else {
                    const uint4 t = *reinterpret_cast<const uint4*>(src + k);
                    e[0] = t.x, e[1] = t.y, e[2] = t.z, e[3] = t.w;
                }
            }
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                s0[m][v] += (u64)e[v] * kb4[v];
                s1[m][v] += (u64)e[v] * ka4[v];
            }
        }
    }
#pragma unroll
    for (int m = 0; m < NBM; ++m) {
        if (m >= nb) break;
        u32 r0[4], r1[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) r0[v] = reduce64(s0[m][v], P.q, P.mu, P.r32), r1[v] = reduce64(s1[m][v], P.q, P.mu, P.r32);
        if (fold.gad && x < nl) {
            const u32 gv = fold.gad[2 * x], gp = fold.gad[2 * x + 1];
            u32 a0v[4], a1v[4];
            if (fold.ta[0]) {  // tensor mode: c0 = a0 b0, c1 = a0 b1 + a1 b0 (k_tensor_ptrs' arithmetic)
                const size_t at = ((size_t)x << logn) + k, o1 = (size_t)fold.tnl << logn;
                const uint4 A0 = *reinterpret_cast<const uint4*>(fold.ta[m] + at), A1 = *reinterpret_cast<const uint4*>(fold.ta[m] + at + o1);
                const uint4 B0 = *reinterpret_cast<const uint4*>(fold.tb[m] + at), B1 = *reinterpret_cast<const uint4*>(fold.tb[m] + at + o1);
                const u32 a0[4] = {A0.x, A0.y, A0.z, A0.w}, a1[4] = {A1.x, A1.y, A1.z, A1.w};
                const u32 b0[4] = {B0.x, B0.y, B0.z, B0.w}, b1[4] = {B1.x, B1.y, B1.z, B1.w};
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    a0v[v] = barrett_mul(a0[v], b0[v], P.q, P.mu);
                    a1v[v] = add_mod(barrett_mul(a0[v], b1[v], P.q, P.mu), barrett_mul(a1[v], b0[v], P.q, P.mu), P.q);
                }
            } else {
                const size_t at = m * fold.ms + ((size_t)x << logn) + k;
                const uint4 f0 = *reinterpret_cast<const uint4*>(fold.add0 + at), f1 = *reinterpret_cast<const uint4*>(fold.add1 + at);
                a0v[0] = f0.x, a0v[1] = f0.y, a0v[2] = f0.z, a0v[3] = f0.w;
                a1v[0] = f1.x, a1v[1] = f1.y, a1v[2] = f1.z, a1v[3] = f1.w;
            }
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                r0[v] = add_mod(r0[v], shoup_mul(a0v[v], gv, gp, P.q), P.q);
                r1[v] = add_mod(r1[v], shoup_mul(a1v[v], gv, gp, P.q), P.q);
            }
        }
        uint4* a0 = reinterpret_cast<uint4*>(acc + m * acc_ms + ((size_t)x << logn) + k);
        uint4* a1 = reinterpret_cast<uint4*>(acc + m * acc_ms + (((size_t)ne + x) << logn) + k);
        if (accum) {
            const uint4 p0 = *a0, p1 = *a1;
            r0[0] = add_mod(r0[0], p0.x, P.q), r0[1] = add_mod(r0[1], p0.y, P.q), r0[2] = add_mod(r0[2], p0.z, P.q), r0[3] = add_mod(r0[3], p0.w, P.q);
            r1[0] = add_mod(r1[0], p1.x, P.q), r1[1] = add_mod(r1[1], p1.y, P.q), r1[2] = add_mod(r1[2], p1.z, P.q), r1[3] = add_mod(r1[3], p1.w, P.q);
        }
        st_out16(a0, make_uint4(r0[0], r0[1], r0[2], r0[3]));
        st_out16(a1, make_uint4(r1[0], r1[1], r1[2], r1[3]));
    }
    ts_end(ts);
}

// XCD-aware block -> (column block, row) map of a (nbx x rows) grid: workgroups are dealt
// round-robin over the 8 XCDs (linear id b and b + 8 share one, MI355X_MICROARCH.md "Workgroup
// dispatch"), so with the plain map the nbx blocks of one row land on all 8 XCDs and EVERY XCD
// fetches the whole gathered source row into its own L2.  Here the blocks of one row sit on one
// XCD: rows are taken in bands of 8, row 8 band + (b mod 8) <- blocks b with b / 8 in the band's
// range.  A last partial band of r < 8 rows: each XCD's r nbx / 8 tail blocks in turn, XCD by
// XCD, fill the rows one after the other -- a row spans at most ceil(8 / r) + 1 XCDs instead of 8.
// A bijection either way (speed only; needs 8 | nbx).
__device__ __forceinline__ void xcd_rows(int lognbx, int rows, int& bx, int& row) {
    const int nbx = 1 << lognbx;
    const int id = blockIdx.x + (blockIdx.y << lognbx);
    const int full = rows & ~7;
    if (id < (full << lognbx)) {
        const int m = id >> 3;
        bx = m & (nbx - 1);
        row = ((m >> lognbx) << 3) + (id & 7);
    } else {
        const int t = id - (full << lognbx), per = ((rows - full) << lognbx) >> 3;  // tail blocks per XCD
        const int pos = (t & 7) * per + (t >> 3);
        bx = pos & (nbx - 1);
        row = full + (pos >> lognbx);
    }
}

// J hoisted rotations summed in one pass (KsSumArgs): the trace step's three key inner products,
// grid z = stacked member; 64-bit multiply-adds folded every 8 products
// ND > 0: compile-time digit count (k_key_inner's ND: each rotation's digit loads in flight together)
template <int ND = 0>
__global__ void __launch_bounds__(kBlock) k_key_inner_sum(u32* acc, const u32* ext, const u32* d, KsSumArgs ka, int nd, int ne, int nl,
                                                          int alpha, int nkey, int nks, LimbMap map, const PrimeConst* pc, int logn,
                                                          size_t ext_ms, size_t d_ms, size_t acc_ms, unsigned long long* ts) {
    ts_begin(ts);
    // the J gathers of a row's ext through different automorphisms: all blocks of one row on one
    // XCD (xcd_rows), so each XCD fetches a gathered row into its L2 once
    int x = blockIdx.y, bx = blockIdx.x;
    xcd_rows(logn - 10, ne, bx, x);
    const int m = blockIdx.z;
    const size_t k = ((size_t)bx * kBlock + threadIdx.x) * 4;
    const PrimeConst P = pc[map.prime(x)];
    const int krow = x < nl ? x : nks + (x - nl);
    const int own = x < nl ? x / alpha : -1;
    u64 s0[4] = {}, s1[4] = {};
    int cnt = 0;
    for (int i = 0; i < ka.J; ++i) {
        u32 ks[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) ks[v] = galois_src((u32)(k + v), ka.g[i], logn);
        const u32* key = ka.key[i];
        const int ndd = ND > 0 ? ND : nd;
#pragma unroll
        for (int j = 0; j < ndd; ++j, ++cnt) {
            if (cnt && (cnt & 7) == 0) {
#pragma unroll
                for (int v = 0; v < 4; ++v) s0[v] = fold64(s0[v], P.q, P.r32), s1[v] = fold64(s1[v], P.q, P.r32);
            }
            const size_t kr = (((size_t)j * 2 * nkey + krow) << logn) + k;
            const uint4 vb = *reinterpret_cast<const uint4*>(key + kr);
            const uint4 va = *reinterpret_cast<const uint4*>(key + kr + ((size_t)nkey << logn));
            const u32 kb4[4] = {vb.x, vb.y, vb.z, vb.w}, ka4[4] = {va.x, va.y, va.z, va.w};
            const u32* src = j == own ? d + m * d_ms + ((size_t)x << logn) : ext + m * ext_ms + (((size_t)j * ne + x) << logn);
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const u32 e = src[ks[v]];
                s0[v] += (u64)e * kb4[v];
                s1[v] += (u64)e * ka4[v];
            }
        }
    }
    uint4* a0 = reinterpret_cast<uint4*>(acc + m * acc_ms + ((size_t)x << logn) + k);
    uint4* a1 = reinterpret_cast<uint4*>(acc + m * acc_ms + (((size_t)ne + x) << logn) + k);
    st_out16(a0, make_uint4(reduce64(s0[0], P.q, P.mu, P.r32), reduce64(s0[1], P.q, P.mu, P.r32), reduce64(s0[2], P.q, P.mu, P.r32),
                            reduce64(s0[3], P.q, P.mu, P.r32)));
    st_out16(a1, make_uint4(reduce64(s1[0], P.q, P.mu, P.r32), reduce64(s1[1], P.q, P.mu, P.r32), reduce64(s1[2], P.q, P.mu, P.r32),
                            reduce64(s1[3], P.q, P.mu, P.r32)));
    ts_end(ts);
}
// c0 + its J automorphisms (the trace step's ModDown addend), one launch for nb members
__global__ void k_automorph_sum(u32* out, const u32* in, KsSumArgs ka, int nl, size_t ms, LimbMap map, const PrimeConst* pc, int logn) {
    const int row = blockIdx.y, m = blockIdx.z;
    const u32 i = blockIdx.x * kBlock + threadIdx.x;
    const PrimeConst P = pc[map.prime(row % nl)];
    const u32* src = in + m * ms + ((size_t)row << logn);
    u32 v = src[i];
    for (int j = 0; j < ka.J; ++j) v = add_mod(v, src[galois_src(i, ka.g[j], logn)], P.q);
    out[m * ms + ((size_t)row << logn) + i] = v;
}

// heterogeneous members (KsMultiArgs): grid z = member, each member its own key, Galois element
// and ModUp source; otherwise the arithmetic of k_key_inner<1> (four coefficients per thread,
// 64-bit multiply-adds folded every 8 digits)
// ND > 0: compile-time digit count (k_key_inner's ND)
template <int ND = 0>
__global__ void __launch_bounds__(kBlock) k_key_inner_multi(u32* acc, const u32* ext, const u32* d, KsMultiArgs ka, int nd, int ne,
                                                            int nl, int alpha, int nkey, int nks, LimbMap map, const PrimeConst* pc,
                                                            int logn, size_t ext_ms, size_t d_ms, size_t acc_ms, unsigned long long* ts) {
    ts_begin(ts);
    const int x = blockIdx.y, m = blockIdx.z;
    const u64 g = ka.g[m];
    const u32* key = ka.key[m];
    const int sm = ka.src[m];
    const size_t k = ((size_t)blockIdx.x * kBlock + threadIdx.x) * 4;
    u32 ks[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) ks[v] = g ? galois_src((u32)(k + v), g, logn) : (u32)(k + v);
    const PrimeConst P = pc[map.prime(x)];
    const int krow = x < nl ? x : nks + (x - nl);
    const int own = x < nl ? x / alpha : -1;
    u64 s0[4] = {}, s1[4] = {};
    const int ndd = ND > 0 ? ND : nd;
#pragma unroll
    for (int j = 0; j < ndd; ++j) {
        if (j && (j & 7) == 0) {
#pragma unroll
            for (int v = 0; v < 4; ++v) s0[v] = fold64(s0[v], P.q, P.r32), s1[v] = fold64(s1[v], P.q, P.r32);
        }
        const size_t kr = (((size_t)j * 2 * nkey + krow) << logn) + k;
        const uint4 vb = *reinterpret_cast<const uint4*>(key + kr);
        const uint4 va = *reinterpret_cast<const uint4*>(key + kr + ((size_t)nkey << logn));
        const u32 kb4[4] = {vb.x, vb.y, vb.z, vb.w}, ka4[4] = {va.x, va.y, va.z, va.w};
        const u32* src = j == own ? d + sm * d_ms + ((size_t)x << logn) : ext + sm * ext_ms + (((size_t)j * ne + x) << logn);
        u32 e[4];
        if (g) {
#pragma unroll
            for (int v = 0; v < 4; ++v) e[v] = src[ks[v]];
        } else {
            const uint4 t = *reinterpret_cast<const uint4*>(src + k);
            e[0] = t.x, e[1] = t.y, e[2] = t.z, e[3] = t.w;
        }
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            s0[v] += (u64)e[v] * kb4[v];
            s1[v] += (u64)e[v] * ka4[v];
        }
    }
    u32 r0[4], r1[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) r0[v] = reduce64(s0[v], P.q, P.mu, P.r32), r1[v] = reduce64(s1[v], P.q, P.mu, P.r32);
    uint4* a0 = reinterpret_cast<uint4*>(acc + m * acc_ms + ((size_t)x << logn) + k);
    uint4* a1 = reinterpret_cast<uint4*>(acc + m * acc_ms + (((size_t)ne + x) << logn) + k);
    st_out16(a0, make_uint4(r0[0], r0[1], r0[2], r0[3]));
    st_out16(a1, make_uint4(r1[0], r1[1], r1[2], r1[3]));
    ts_end(ts);
}
__global__ void k_automorph_multi(u32* out, size_t out_ms, AutoMulti am, int logn) {
    const int row = blockIdx.y, m = blockIdx.z;
    const u32 i = blockIdx.x * kBlock + threadIdx.x;
    const u64 g = am.g[m];
    const u32 mask2n = (2u << logn) - 1;
    const u32 e = 2u * (__brev(i) >> (32 - logn)) + 1u;
    const u32 eg = (u32)(((u64)e * (g & mask2n)) & mask2n);
    const u32 j = __brev((eg - 1u) >> 1) >> (32 - logn);
    out[m * out_ms + ((size_t)row << logn) + i] = am.src[m][((size_t)row << logn) + j];
}

// ------------------------------------------------------------------------------------
// sampling and key generation
// ------------------------------------------------------------------------------------
__global__ void k_sample_small(u32* out, int nl, LimbMap map, PrngKey key, u64 stream, int kind, const PrimeConst* pc, int logn) {
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const u64 r = chacha_u64(key, stream, k);
    int v;
    if (kind == 0) v = (int)(r % 3) - 1;
    else v = __popcll(r & 0x1FFFFFull) - __popcll((r >> 21) & 0x1FFFFFull);
    for (int l = 0; l < nl; ++l) {
        const u32 q = pc[map.prime(l)].q;
        out[((size_t)l << logn) + k] = v >= 0 ? (u32)v : q - (u32)(-v);
    }
}
// v (ternary), e0, e1 (binomial) of nm encryptions: grid (N / kBlock, 3 nm), row block y = 3 m + w
__global__ void k_sample_enc(u32* out, int nl, PrngKey key, EncCtrs ctr, const u32* msg, size_t msg_ms, const PrimeConst* pc, int logn) {
    const int y = blockIdx.y, m = y / 3, w = y - 3 * m;
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const u64 stream = ((u64)(6 + w) << 56) | (ctr.base + (u64)m);  // stream_id(6 + w, 0, ctr)
    const u64 r = chacha_u64(key, stream, k);
    const int v = w == 0 ? (int)(r % 3) - 1 : __popcll(r & 0x1FFFFFull) - __popcll((r >> 21) & 0x1FFFFFull);
    u32* o = out + ((size_t)y * nl << logn);
    const u32* mm = (msg && w == 1) ? msg + m * msg_ms : nullptr;  // e0 + message (launch_sample_enc)
    for (int l = 0; l < nl; ++l) {
        const u32 q = pc[l].q;
        u32 x = v >= 0 ? (u32)v : q - (u32)(-v);
        if (mm) x = add_mod(x, mm[((size_t)l << logn) + k], q);
        o[((size_t)l << logn) + k] = x;
    }
}
// c0 = (e0 + msg) + pk0 v, c1 = e1 + pk1 v (the add / fma sequence of Engine::encrypt_ntt, bit for bit)
__global__ void k_enc_combine(u32* top, const u32* vee, const u32* msg, size_t msg_ms, const u32* pk, int pk_rows, int nl,
                              const PrimeConst* pc, int logn) {
    const int y = blockIdx.y, m = y / nl, l = y - m * nl;
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const PrimeConst P = pc[l];
    const size_t row = (size_t)l << logn, pl = (size_t)nl << logn;
    const u32* V = vee + (size_t)m * 3 * pl;
    const u32 v = V[row + k], e0 = V[pl + row + k], e1 = V[2 * pl + row + k];
    const u32 mv = msg ? msg[m * msg_ms + row + k] : 0u;  // null: the message rode in e0 (launch_sample_enc)
    u32* o = top + (size_t)m * 2 * pl;
    o[row + k] = add_mod(add_mod(e0, mv, P.q), barrett_mul(pk[row + k], v, P.q, P.mu), P.q);
    o[pl + row + k] = add_mod(e1, barrett_mul(pk[((size_t)pk_rows << logn) + row + k], v, P.q, P.mu), P.q);
}
// raw decryption rows of up to two channels (renorm): x[c][t] = c0 + c1 s + c2 s^2 on t < kd[c]
__global__ void k_dec_raw(u32* x, DecRaw dr, const u32* s, const u32* s2, const PrimeConst* pc, int logn) {
    const int ch = blockIdx.y >> 2, t = blockIdx.y & 3;
    const int c = ch / dr.members, mb = ch - c * dr.members;
    if (t >= dr.kd[c]) return;
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const PrimeConst P = pc[t];
    const size_t row = ((size_t)t << logn) + k, pl = (size_t)dr.nlc[c] << logn;
    const u32* ct = dr.ct[c] + mb * dr.ms[c];
    u32 v = ct[row];
    v = add_mod(v, barrett_mul(ct[pl + row], s[row], P.q, P.mu), P.q);
    if (dr.npoly[c] == 3) v = add_mod(v, barrett_mul(ct[2 * pl + row], s2[row], P.q, P.mu), P.q);
    x[((size_t)(ch * 4 + t) << logn) + k] = v;
}
__global__ void k_sample_uniform(u32* out, int nl, LimbMap map, PrngKey key, u64 stream, const PrimeConst* pc, int logn) {
    const int l = blockIdx.y;
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const int prime = map.prime(l);
    const u32 q = pc[prime].q;
    out[((size_t)l << logn) + k] = (u32)(chacha_u64(key, stream, ((u64)prime << logn) + k) % q);
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
thread_local KernelProfiler* g_prof = nullptr;
void prof_set(KernelProfiler* p) { g_prof = p; }
std::atomic<unsigned long long> g_launches{0};
std::atomic<unsigned long long> g_alg_bytes[KID_N] = {};
std::atomic<unsigned long long> g_alg_launches[KID_N] = {};
const bool g_census_on = std::getenv("AESFHE_CENSUS") && std::atoi(std::getenv("AESFHE_CENSUS")) != 0;
thread_local const char* g_census_op = nullptr;
static std::mutex g_census_mu;
static std::map<std::pair<std::string, const void*>, unsigned long long> g_census;
void census_add(const void* fn) {
    std::lock_guard<std::mutex> lk(g_census_mu);
    ++g_census[{g_census_op ? g_census_op : "(internal)", fn}];
}
// "op\tkernel\tlaunches\n" lines into buf (NUL-terminated); returns the bytes needed
size_t census_dump(char* buf, size_t cap, bool reset) {
    std::lock_guard<std::mutex> lk(g_census_mu);
    std::string out;
    for (const auto& kv : g_census) {
        const char* nm = hipKernelNameRefByPtr(kv.first.second, nullptr);
        out += kv.first.first + "\t" + (nm ? nm : "?") + "\t" + std::to_string(kv.second) + "\n";
    }
    if (buf && cap) {
        const size_t n = std::min(cap - 1, out.size());
        std::memcpy(buf, out.data(), n);
        buf[n] = 0;
    }
    if (reset) g_census.clear();
    return out.size() + 1;
}

// ======================================================================================
// launch validation (launch.h launch_validate): per-kernel limits, queried once
// ======================================================================================
const LaunchLimits& launch_limits(const void* fn) {
    static std::mutex mu;
    static std::unordered_map<const void*, LaunchLimits> cache;
    std::lock_guard<std::mutex> lock(mu);
    auto it = cache.find(fn);
    if (it != cache.end()) return it->second;
    hipFuncAttributes a{};
    if (hipFuncGetAttributes(&a, fn) != hipSuccess) throw std::runtime_error("launch validation: hipFuncGetAttributes failed");
    return cache.emplace(fn, LaunchLimits{a.maxThreadsPerBlock, a.sharedSizeBytes}).first->second;
}
void launch_reject(const void* fn, const char* what, dim3 grid, dim3 block, size_t lds, size_t kernarg) {
    char buf[256];
    std::snprintf(buf, sizeof buf, "launch rejected (%s): kernel %p grid (%u, %u, %u) block (%u, %u, %u) lds %zu kernarg %zu", what, fn,
                  grid.x, grid.y, grid.z, block.x, block.y, block.z, lds, kernarg);
    throw std::runtime_error(buf);
}

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
    ts_flush();
    for (auto& r : recs) {
        float t = 0.f;
        (void)hipEventSynchronize(r.b);
        (void)hipEventElapsedTime(&t, r.a, r.b);
        ms[r.kid] += t;
        bytes[r.kid] += r.bytes;
        work[r.kid] += r.work;
        launches[r.kid] += 1;
        pool.push_back(r.a);
        pool.push_back(r.b);
    }
    recs.clear();
}
unsigned long long* KernelProfiler::ts_slot(int kid, double b, double w, bool count, int prev) {
    const size_t words = (size_t)kTsSlots * kTsRec;
    if (!d_ts) {
        void* p = nullptr;
        if (hipMalloc(&p, sizeof(unsigned long long) * words) != hipSuccess) return nullptr;
        d_ts = (unsigned long long*)p;
        (void)hipMemset(d_ts, 0, sizeof(unsigned long long) * words);
    }
    if (ts_next == kTsSlots) {
        ts_flush();
        prev = -1;  // the predecessor's slot was just recycled
    }
    ts_recs.push_back({ts_next, kid, b, w, count, prev});
    return d_ts + (size_t)kTsRec * ts_next++;
}
void KernelProfiler::ts_flush() {
    pend_slot = -1;
    if (!d_ts || ts_recs.empty()) return;
    (void)hipDeviceSynchronize();
    const size_t words = (size_t)kTsRec * ts_next;
    std::vector<unsigned long long> h(words);
    (void)hipMemcpy(h.data(), d_ts, sizeof(unsigned long long) * words, hipMemcpyDeviceToHost);
    // {earliest start, latest end} of a slot (0 / 0 when no block stamped)
    auto span = [&](int slot, unsigned long long& a, unsigned long long& e) {
        const unsigned long long* rec = h.data() + (size_t)kTsRec * slot;
        a = ~0ull, e = 0;
        for (int j = 0; j < kTsSub; ++j) {
            if (rec[kTsLine * j]) a = std::min(a, ~rec[kTsLine * j]);
            e = std::max(e, rec[kTsLine * (kTsSub + j)]);
        }
        return a != ~0ull && e >= a;
    };
    for (const auto& r : ts_recs) {
        unsigned long long a, e;
        if (!span(r.slot, a, e)) continue;
        if (r.count) {
            ms[r.kid] += (double)(e - a) * 1e-5;  // 100 MHz ticks -> ms
            bytes[r.kid] += r.bytes;
            work[r.kid] += r.work;
            launches[r.kid] += 1;
        }
        unsigned long long pa, pe;
        // the boundary gap: this launch's first stamped start after its predecessor's last end, on
        // one stream (a launch of another stream in between would start before that end: dropped)
        if (r.prev >= 0 && span(r.prev, pa, pe) && a >= pe && a - pe < 100000) {
            gap_ms[r.kid] += (double)(a - pe) * 1e-5;
            gap_n[r.kid] += 1;
        }
    }
    ts_recs.clear();
    (void)hipMemset(d_ts, 0, sizeof(unsigned long long) * words);
    ts_next = 0;
}
void KernelProfiler::reset() {
    flush();
    for (int k = 0; k < KID_N; ++k) ms[k] = bytes[k] = work[k] = gap_ms[k] = 0, launches[k] = gap_n[k] = 0;
}

namespace {
// ------------------------------------------------------------------------------------
// device Zeta16 renorm codec
// ------------------------------------------------------------------------------------
__device__ __forceinline__ double crt_centered(const u32* r, int kd, const CrtConsts& cc) {
    u32 a[4];
    a[0] = r[0];
    for (int i = 1; i < kd; ++i) {
        const u32 qi = cc.q[i];
        u64 v = 0;
        for (int j = 0; j < i; ++j) v += (u64)a[j] * cc.p_mod[i][j];  // < 3 * 2^62
        const u32 vm = (u32)(v % qi);
        const u32 d = r[i] >= vm ? r[i] - vm : r[i] + qi - vm;
        a[i] = (u32)((u64)d * cc.minv[i] % qi);
    }
    // negative iff the top digit is in the upper half (|m| << Q, so never near Q/2)
    if (a[kd - 1] >= (cc.q[kd - 1] >> 1)) {
        double s = 1.0;  // Q - v = sum (q_i - 1 - a_i) P_i + 1
        for (int i = 0; i < kd; ++i) s += (double)(cc.q[i] - 1 - a[i]) * cc.pd[i];
        return -s;
    }
    double s = 0.0;
    for (int i = 0; i < kd; ++i) s += (double)a[i] * cc.pd[i];
    return s;
}

__global__ void __launch_bounds__(kBlock) k_decode16(const u32* x, int kd0, int kd1, CrtConsts cc0, CrtConsts cc1, Slot16 sl,
                                                     double is0, double is1, double* acc, int logn) {
    const int c = blockIdx.y;
    const int n = 1 << logn;
    const int k = blockIdx.x * kBlock + threadIdx.x;
    const int kd = c ? kd1 : kd0;
    u32 r[4];
    for (int i = 0; i < kd; ++i) r[i] = x[((size_t)(c * 4 + i) << logn) + k];
    const double m = crt_centered(r, kd, c ? cc1 : cc0) * (c ? is1 : is0);
    __shared__ double red[kBlock / 64][32];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const u32 mask = 2u * n - 1;
    const double inv_n = 1.0 / n;
    for (int i = 0; i < 16; ++i) {
        double sn, cs;
        sincospi((double)((sl.e[i] * (u32)k) & mask) * inv_n, &sn, &cs);
        double vr = m * cs, vi = m * sn;
        for (int o = 32; o > 0; o >>= 1) vr += __shfl_down(vr, o, 64), vi += __shfl_down(vi, o, 64);
        if (lane == 0) red[wv][2 * i] = vr, red[wv][2 * i + 1] = vi;
    }
    __syncthreads();
    if (threadIdx.x < 32) {
        double t = 0.0;
        for (int w = 0; w < kBlock / 64; ++w) t += red[w][threadIdx.x];
        atomicAdd(acc + c * 32 + threadIdx.x, t);
    }
}

// 32 slot values of one decryption (the packed period-32 state): partial sums per block, atomically added
__global__ void __launch_bounds__(kBlock) k_decode32(const u32* x, int kd, CrtConsts cc, Slot32 sl, double is, double* acc, int logn) {
    const int n = 1 << logn;
    const int k = blockIdx.x * kBlock + threadIdx.x;
    u32 r[4];
    for (int i = 0; i < kd; ++i) r[i] = x[((size_t)i << logn) + k];
    const double m = crt_centered(r, kd, cc) * is;
    __shared__ double red[kBlock / 64][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const u32 mask = 2u * n - 1;
    const double inv_n = 1.0 / n;
    for (int i = 0; i < 32; ++i) {
        double sn, cs;
        sincospi((double)((sl.e[i] * (u32)k) & mask) * inv_n, &sn, &cs);
        double vr = m * cs, vi = m * sn;
        for (int o = 32; o > 0; o >>= 1) vr += __shfl_down(vr, o, 64), vi += __shfl_down(vi, o, 64);
        if (lane == 0) red[wv][2 * i] = vr, red[wv][2 * i + 1] = vi;
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        double t = 0.0;
        for (int w = 0; w < kBlock / 64; ++w) t += red[w][threadIdx.x];
        atomicAdd(acc + threadIdx.x, t);
    }
}
// slot t's snap: nibble = round(-angle 16 / 2 pi) mod 16, w = zeta16^nibble - 1
__device__ __forceinline__ int snap_slot(const double* acc, int t, double& wr, double& wi) {
    const double ang = atan2(acc[2 * t + 1], acc[2 * t]);
    const double kf = rint(-ang * 16.0 / (2.0 * M_PI));
    const int v = (int)((((long)kf) % 16 + 16) % 16);
    double sn, cs;
    sincospi(-2.0 * v / 16.0, &sn, &cs);
    wr = cs - 1.0;
    wi = sn;
    return v;
}
// SNAP: the encode derives the 32 snapped values itself from the decode's accumulator acc (each
// block, into LDS: no k_snap16 launch), and block 0 zeroes zacc -- the accumulator the PREVIOUS
// renorm on this stream used, free since that renorm's encode finished -- for the next decode
__device__ __forceinline__ const double* snap_block(const double* acc, double* zacc, double* sw) {
    if (threadIdx.x < 32) snap_slot(acc, threadIdx.x, sw[2 * threadIdx.x], sw[2 * threadIdx.x + 1]);
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 64) zacc[threadIdx.x] = 0.0;
    __syncthreads();
    return sw;
}
// ONE 32-periodic message from its 32 snapped slot deviations w (w_j = zeta^nib - 1): only the
// coefficients k == 0 mod N/64 are nonzero, m_k = (1/32) sum_j Re(w_j zeta^(-e_j k)) (+1 at k = 0)
template <bool SNAP>
__global__ void __launch_bounds__(kBlock) k_encode32(u32* out, const double* w, double* zacc, Slot32 sl, double scale, int nq,
                                                     const PrimeConst* pc, int logn) {
    __shared__ double sw[SNAP ? 64 : 1];
    if (SNAP) w = snap_block(w, zacc, sw);
    const int n = 1 << logn;
    const int k = blockIdx.x * kBlock + threadIdx.x;
    const u32 mask = 2u * n - 1, kmask = (u32)(n / 64) - 1;
    const double inv_n = 1.0 / n;
    double v = 0.0;
    if (((u32)k & kmask) == 0)
        for (int i = 0; i < 32; ++i) {
            double sn, cs;
            sincospi((double)((sl.e[i] * (u32)k) & mask) * inv_n, &sn, &cs);
            v += w[2 * i] * cs + w[2 * i + 1] * sn;
        }
    v = v / 32.0 + (k == 0 ? 1.0 : 0.0);
    const double x = rint(v * scale);
    for (int t = 0; t < nq; ++t) {
        const double q = (double)pc[t].q;
        double r = fma(-q, floor(x / q), x);
        if (r < 0) r += q;
        if (r >= q) r -= q;
        out[((size_t)t << logn) + k] = (u32)r;
    }
}

// ---- the renorm's re-encryption from a pool of zero encryptions (Engine::zero_enc)
// The snapped message of a channel of NS slots (period NS per channel: k_encode32 with NS = 32, the
// periodic k_encode16 with NS = 16) has D = 2 NS nonzero coefficients, k = j N / D, formed here exactly
// as those kernels form them: x_j = rint((fac sum_i Re(w_i zeta^(-e_i k)) + [k = 0]) scale).  Its
// negacyclic NTT (Cooley-Tukey, bit-reversed out: value i at psi^(2 brv(i) + 1)) takes D distinct values:
// NTT(m)[i] = W[i >> (logn - log2 D)], W[d] = sum_j x_j g^((2 brv_D(d) + 1) j), g = psi^(N / D) a
// primitive 2D-th root (gtab[t][e] = g_t^e, e < 2D).  One block per channel: x into LDS, the residues,
// the D x D sums (one reduced product per term).
template <int NS, bool SNAP>
__global__ void __launch_bounds__(256) k_renorm_wtab(u32* W, const double* w, double* zacc, SlotTab<NS> sl, double scale, int nl,
                                                     const u32* gtab, const PrimeConst* pc, int logn) {
    constexpr int D = 2 * NS, LD = (NS == 32) ? 6 : 5;
    static_assert((1 << LD) == D, "D = 2 NS, a power of two");
    __shared__ double sw[SNAP ? 64 : 1];
    __shared__ double xs[D];
    __shared__ u32 res[kRenormMaxLimbs * D];
    if (SNAP) w = snap_block(w, zacc, sw);
    const int c = blockIdx.x, n = 1 << logn;
    const u32 mask = 2u * n - 1;
    const double inv_n = 1.0 / n;
    if (threadIdx.x < D) {
        const int j = threadIdx.x;
        const u32 k = (u32)j * (u32)(n / D);
        double v = 0.0;
        for (int i = 0; i < NS; ++i) {
            double sn, cs;
            sincospi((double)((sl.e[i] * k) & mask) * inv_n, &sn, &cs);
            v += w[c * 2 * NS + 2 * i] * cs + w[c * 2 * NS + 2 * i + 1] * sn;
        }
        v = v / (double)NS + (j == 0 ? 1.0 : 0.0);
        xs[j] = rint(v * scale);
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < nl * D; idx += blockDim.x) {
        const int t = idx / D, j = idx - t * D;
        const double q = (double)pc[t].q, x = xs[j];
        double r = fma(-q, floor(x / q), x);
        if (r < 0) r += q;
        if (r >= q) r -= q;
        res[idx] = (u32)r;
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < nl * D; idx += blockDim.x) {
        const int t = idx / D, d = idx - t * D;
        const u32 q = pc[t].q, mu = pc[t].mu;
        const u32 rv = (u32)(__brev((unsigned)d) >> (32 - LD));
        const u32 e1 = 2u * rv + 1u;
        const u32* g = gtab + (size_t)t * 2 * D;
        u32 acc = 0;
        for (int j = 0; j < D; ++j) acc = add_mod(acc, barrett_mul(res[t * D + j], g[(e1 * (u32)j) & (2u * D - 1)], q, mu), q);
        W[((size_t)c * nl + t) * D + d] = acc;
    }
}
// ---- the renorm's sparse decryption (round 6): the snap reads only the D subring coefficients k = j N / D of
// m = c0 + c1 s (+ c2 s^2) -- the coefficients a message of D / 2 slots per channel can have; the others
// carry noise only, which the decode drops (the trace projection of the decrypted polynomial).  From the
// NTT form, coefficient j N / D = N^{-1} sum_i a_i psi^{-(2 brv(i) + 1) j N / D}, and the power depends on
// i only through its top log2 D bits b: with B_b = the sum of the N / D consecutive a_i of block b, it is
// the D-point inverse transform N^{-1} sum_b B_b g^{-(2 brv_D(b) + 1) j} (g = psi^(N / D)).
// k_dec_blocksum: one block per (block b, limb t, channel c) -> B[c][t][b]
template <int D>
__global__ void __launch_bounds__(256) k_dec_blocksum(u32* B, DecRaw dr, const u32* s, const u32* s2, const PrimeConst* pc, int logn) {
    const int b = blockIdx.x, t = blockIdx.y, c = blockIdx.z;
    if (t >= dr.kd[c]) return;
    const PrimeConst P = pc[t];
    const int len = (1 << logn) / D;
    const size_t base = ((size_t)t << logn) + (size_t)b * len, pl = (size_t)dr.nlc[c] << logn;
    const u32* ct = dr.ct[c];
    const bool three = dr.npoly[c] == 3;
    unsigned long long acc = 0;
    for (int k = threadIdx.x; k < len; k += 256) {
        const size_t row = base + k;
        u32 v = add_mod(ct[row], barrett_mul(ct[pl + row], s[row], P.q, P.mu), P.q);
        if (three) v = add_mod(v, barrett_mul(ct[2 * pl + row], s2[row], P.q, P.mu), P.q);
        acc += v;
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    __shared__ unsigned long long red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) B[((size_t)c * 4 + t) * D + b] = (u32)((red[0] + red[1] + red[2] + red[3]) % P.q);
}
// one block per channel: the D coefficients' residues (the inverse D-point transform of B), their centred
// CRT value, the NS slots (m evaluated at zeta^(e_i), as k_decode32 / k_decode16 but over the subring
// coefficients), the snap (k_snap16's rule), and the snapped message's NTT table W (k_renorm_wtab's)
template <int NS>
__global__ void __launch_bounds__(256) k_renorm_sparse(u32* W, const u32* B, SparseDec sd, SlotTab<NS> sl, double scale, int nl,
                                                       const u32* gtab, const PrimeConst* pc, int logn) {
    // every table the phases read is staged in LDS first: the serial D-term sums then wait on LDS, not on
    // L2 (a first form read B and gtab from global memory in its inner loops: 31 us per launch)
    constexpr int D = 2 * NS, LD = (NS == 32) ? 6 : 5;
    __shared__ u32 cr[4 * D];
    __shared__ u32 bs[4 * D];
    __shared__ u32 gs[kRenormMaxLimbs * 2 * D];
    __shared__ double mv[D];
    __shared__ double ws[2 * NS];
    __shared__ double xs[D];
    __shared__ double cs_[NS * D], sn_[NS * D];  // the angles pi (e_i j N / D mod 2N) / N of slot i, coefficient j
    __shared__ u32 res[kRenormMaxLimbs * D];
    const int c = blockIdx.x, kd = sd.kd[c], n = 1 << logn;
    const int nt = nl > kd ? nl : kd;
    const u32 mask = 2u * n - 1;
    const double inv_n = 1.0 / n;
    for (int idx = threadIdx.x; idx < nt * 2 * D; idx += blockDim.x) gs[idx] = gtab[idx];
    for (int idx = threadIdx.x; idx < kd * D; idx += blockDim.x) bs[idx] = B[((size_t)c * 4) * D + idx];
    for (int idx = threadIdx.x; idx < NS * D; idx += blockDim.x) {
        const int i = idx / D, j = idx - i * D;
        double sn, cs;
        sincospi((double)((sl.e[i] * (u32)(j * (n / D))) & mask) * inv_n, &sn, &cs);
        cs_[idx] = cs, sn_[idx] = sn;
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < kd * D; idx += blockDim.x) {
        const int t = idx / D, j = idx - t * D;
        const PrimeConst P = pc[t];
        const u32* g = gs + t * 2 * D;
        const u32* Bc = bs + t * D;
        unsigned long long acc = 0;  // D reduced products < 2^36: one reduction, no dependent add_mod chain
#pragma unroll 8
        for (int b = 0; b < D; ++b) {
            const u32 rv = (u32)(__brev((unsigned)b) >> (32 - LD));
            const u32 e = (2u * D - (((2u * rv + 1u) * (u32)j) & (2u * D - 1))) & (2u * D - 1);
            acc += barrett_mul(Bc[b], g[e], P.q, P.mu);
        }
        cr[idx] = shoup_mul((u32)(acc % P.q), P.ninv, P.ninv_p, P.q);
    }
    __syncthreads();
    if (threadIdx.x < D) {
        u32 r[4];
        for (int t = 0; t < kd; ++t) r[t] = cr[t * D + threadIdx.x];
        mv[threadIdx.x] = crt_centered(r, kd, sd.cc[c]);
    }
    __syncthreads();
    if (threadIdx.x < NS) {  // slot i: sum_j m_j zeta^(e_i j N / D), snapped (k_snap16 / snap_slot's rule)
        const int i = threadIdx.x;
        double vr = 0.0, vi = 0.0;
        for (int j = 0; j < D; ++j) vr += mv[j] * cs_[i * D + j], vi += mv[j] * sn_[i * D + j];
        const double ang = atan2(vi, vr);
        const double kf = rint(-ang * 16.0 / (2.0 * M_PI));
        const int v = (int)((((long)kf) % 16 + 16) % 16);
        double sn, cs;
        sincospi(-2.0 * v / 16.0, &sn, &cs);
        ws[2 * i] = cs - 1.0, ws[2 * i + 1] = sn;
    }
    __syncthreads();
    if (threadIdx.x < D) {  // k_renorm_wtab's coefficients from the snapped deviations
        const int j = threadIdx.x;
        double v = 0.0;
        for (int i = 0; i < NS; ++i) v += ws[2 * i] * cs_[i * D + j] + ws[2 * i + 1] * sn_[i * D + j];
        v = v / (double)NS + (j == 0 ? 1.0 : 0.0);
        xs[j] = rint(v * scale);
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < nl * D; idx += blockDim.x) {
        const int t = idx / D, j = idx - t * D;
        const double q = (double)pc[t].q, x = xs[j];
        double r = fma(-q, floor(x / q), x);
        if (r < 0) r += q;
        if (r >= q) r -= q;
        res[idx] = (u32)r;
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < nl * D; idx += blockDim.x) {
        const int t = idx / D, d = idx - t * D;
        const u32 q = pc[t].q, mu = pc[t].mu;
        const u32 rv = (u32)(__brev((unsigned)d) >> (32 - LD));
        const u32 e1 = 2u * rv + 1u;
        const u32* g = gs + t * 2 * D;
        unsigned long long acc = 0;
#pragma unroll 8
        for (int j = 0; j < D; ++j) acc += barrett_mul(res[t * D + j], g[(e1 * (u32)j) & (2u * D - 1)], q, mu);
        W[((size_t)c * nl + t) * D + d] = (u32)(acc % q);
    }
}
// out_c (2 polys x nl limbs) = the zero encryption pool_c + (W_c broadcast over runs of N / D on c0)
__global__ void k_renorm_combine(RenormOut ro, const u32* W, int nl, int ld, const PrimeConst* pc, int logn) {
    const int c = blockIdx.z, row = blockIdx.y, t = row % nl, p = row / nl;
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t idx = ((size_t)row << logn) + k;
    u32 v = ro.pool[c][idx];
    if (p == 0) v = add_mod(v, W[((size_t)c * nl + t) * (1u << ld) + (k >> (logn - ld))], pc[t].q);
    ro.out[c][idx] = v;
}

// acc is zeroed behind its read: the next renorm's decode accumulates into a clean buffer
// without a fill launch of its own (the buffer is zeroed once when allocated)
__global__ void k_snap16(double* acc, double* w, int* nib) {
    const int t = threadIdx.x;  // 32 = 2 ciphertexts x 16 slots
    if (t >= 32) return;
    nib[t] = snap_slot(acc, t, w[2 * t], w[2 * t + 1]);
    acc[2 * t] = 0.0, acc[2 * t + 1] = 0.0;
}

// kmask = 0: the reference layout (16 slots deviate from 1; every coefficient, factor 2/N);
// kmask = N/32 - 1: the 16-periodic layout (slot j == slot j mod 16, sl.e = 5^i): only the
// coefficients k == 0 mod N/32 are nonzero, m_k = (1/16) sum_i Re(w_i zeta^(-e_i k)) (+1 at k = 0)
template <bool SNAP>
__global__ void __launch_bounds__(kBlock) k_encode16(u32* out, const double* w, double* zacc, Slot16 sl, double scale, int nq,
                                                     const PrimeConst* pc, int logn, u32 kmask, double fac) {
    __shared__ double sw[SNAP ? 64 : 1];
    if (SNAP) w = snap_block(w, zacc, sw);
    const int c = blockIdx.y;
    const int n = 1 << logn;
    const int k = blockIdx.x * kBlock + threadIdx.x;
    const u32 mask = 2u * n - 1;
    const double inv_n = 1.0 / n;
    double v = 0.0;
    if (((u32)k & kmask) == 0)
        for (int i = 0; i < 16; ++i) {
            double sn, cs;
            sincospi((double)((sl.e[i] * (u32)k) & mask) * inv_n, &sn, &cs);
            v += w[c * 32 + 2 * i] * cs + w[c * 32 + 2 * i + 1] * sn;
        }
    v = v * fac + (k == 0 ? 1.0 : 0.0);
    const double x = rint(v * scale);
    for (int t = 0; t < nq; ++t) {
        const double q = (double)pc[t].q;
        double r = fma(-q, floor(x / q), x);
        if (r < 0) r += q;
        if (r >= q) r -= q;
        out[((size_t)(c * nq + t) << logn) + k] = (u32)r;
    }
}

// ------------------------------------------------------------------------------------
// slot-packed renorm: fp64 canonical embedding on the device (four-step FFT)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ int fft_log1(int logn) { return logn - logn / 2; }  // log N1 (N1 >= N2)

__global__ void __launch_bounds__(kBlock) k_decode_twist(const u32* x, int kd0, int kd1, CrtConsts cc0, CrtConsts cc1, double is0,
                                                         double is1, double2* z, int logn, int members) {
    const int c = blockIdx.y, w = c / members;
    const int k = blockIdx.x * kBlock + threadIdx.x;
    const int kd = w ? kd1 : kd0;
    u32 r[4];
    for (int i = 0; i < kd; ++i) r[i] = x[((size_t)(c * 4 + i) << logn) + k];
    const double m = crt_centered(r, kd, w ? cc1 : cc0) * (w ? is1 : is0);
    double sn, cs;
    sincospi((double)k / (double)(1 << logn), &sn, &cs);
    z[((size_t)c << logn) + k] = make_double2(m * cs, m * sn);
}

// kFftTpb transforms of length L = 2^logl per block, one LDS row each, radix-2 DIT after a
// bit-reversed load.  pass 0: the columns of the N1 x N2 matrix (element stride N2), then the
// four-step twiddle e^{sign 2 pi i n2 k1 / N}; pass 1: its rows (contiguous)
constexpr int kFftTpb = 16;
__global__ void __launch_bounds__(kBlock) k_fft_pass(double2* data, int logn, int pass, int sign) {
    __shared__ double2 buf[kFftTpb][257];
    const int l1 = fft_log1(logn), l2 = logn - l1;
    const int logl = pass ? l2 : l1;
    const int L = 1 << logl, n2 = 1 << l2;
    double2* d = data + ((size_t)blockIdx.y << logn);
    const int t0 = blockIdx.x * kFftTpb;  // first column (pass 0) / row (pass 1)
    for (int idx = threadIdx.x; idx < kFftTpb * L; idx += kBlock) {
        int e, i;
        size_t a;
        if (pass == 0) e = idx / kFftTpb, i = idx % kFftTpb, a = (size_t)e * n2 + t0 + i;
        else i = idx >> logl, e = idx & (L - 1), a = (size_t)(t0 + i) * n2 + e;
        buf[i][__brev((unsigned)e) >> (32 - logl)] = d[a];
    }
    __syncthreads();
    for (int h = 1; h < L; h <<= 1) {
        for (int b = threadIdx.x; b < kFftTpb * L / 2; b += kBlock) {
            const int i = b >> (logl - 1), j = b & (L / 2 - 1);
            const int pos = j & (h - 1);
            const int i0 = ((j - pos) << 1) + pos, i1 = i0 + h;
            double sn, cs;
            sincospi((double)(sign * pos) / (double)h, &sn, &cs);
            const double2 u = buf[i][i0], v = buf[i][i1];
            const double2 vw = make_double2(v.x * cs - v.y * sn, v.x * sn + v.y * cs);
            buf[i][i0] = make_double2(u.x + vw.x, u.y + vw.y);
            buf[i][i1] = make_double2(u.x - vw.x, u.y - vw.y);
        }
        __syncthreads();
    }
    const double inv_half_n = 2.0 / (double)(1 << logn);
    for (int idx = threadIdx.x; idx < kFftTpb * L; idx += kBlock) {
        if (pass == 0) {
            const int e = idx / kFftTpb, i = idx % kFftTpb;
            const long tw = (long)(t0 + i) * e;  // n2 k1 < N
            double sn, cs;
            sincospi((double)(sign * tw) * inv_half_n, &sn, &cs);
            const double2 v = buf[i][e];
            d[(size_t)e * n2 + t0 + i] = make_double2(v.x * cs - v.y * sn, v.x * sn + v.y * cs);
        } else {
            const int i = idx >> logl, e = idx & (L - 1);
            d[(size_t)(t0 + i) * n2 + e] = buf[i][e];
        }
    }
}

__device__ __forceinline__ size_t fft_loc(u32 t, int logn) {
    const int l1 = fft_log1(logn);
    return ((size_t)(t & ((1u << l1) - 1)) << (logn - l1)) + (t >> l1);
}

// unpack > 0: output c (0 = hi, 1 = lo) takes slot (j mod unpack) + c unpack of the FIRST input
// -- the hi | lo halves of a 2 unpack-periodic packed state (pipeline's packed XOR stage)
__global__ void __launch_bounds__(kBlock) k_snap_slots(const double2* zin, double2* w, const u32* slot_pos, int states, int unpack,
                                                       int logn, int members) {
    const int oc = blockIdx.y, c = oc / members, mb = oc - c * members;
    const int j = blockIdx.x * kBlock + threadIdx.x;  // slot < N/2
    const int n = 1 << logn;
    const u32 t = slot_pos[j];
    const int stride = (n / 2) / 16;
    double2 v = make_double2(1.0, 0.0);
    if (j % stride < states) {
        const int src_c = unpack ? mb : oc;
        const u32 ts = unpack ? slot_pos[(j & (unpack - 1)) + c * unpack] : t;
        const double2 z = zin[((size_t)src_c << logn) + fft_loc(ts, logn)];
        const double kf = rint(-atan2(z.y, z.x) * 16.0 / (2.0 * M_PI));
        const int nib = (int)((((long)kf) % 16 + 16) % 16);
        double sn, cs;
        sincospi(-2.0 * nib / 16.0, &sn, &cs);
        v = make_double2(cs, sn);
    }
    double2* wc = w + ((size_t)oc << logn);
    wc[t] = v;
    wc[n - 1 - t] = make_double2(v.x, -v.y);
}

__global__ void __launch_bounds__(kBlock) k_encode_untwist(u32* out, const double2* v, double scale, int nq, const PrimeConst* pc,
                                                           int logn) {
    const int c = blockIdx.y;
    const int k = blockIdx.x * kBlock + threadIdx.x;
    const double2 z = v[((size_t)c << logn) + fft_loc((u32)k, logn)];
    double sn, cs;
    sincospi((double)k / (double)(1 << logn), &sn, &cs);
    const double m = (z.x * cs + z.y * sn) / (double)(1 << logn);
    const double x = rint(m * scale);
    for (int t = 0; t < nq; ++t) {
        const double q = (double)pc[t].q;
        double r = fma(-q, floor(x / q), x);
        if (r < 0) r += q;
        if (r >= q) r -= q;
        out[((size_t)(c * nq + t) << logn) + k] = (u32)r;
    }
}

// ------------------------------------------------------------------------------------
// fused LUT evaluation: one launch per LUT instead of a tensor + constant + add per term
// ------------------------------------------------------------------------------------
// grid z = member of stacked elements: element p of member m at a[p] + m 2 na[p] N (b likewise),
// the output at out + m 3 nl N
// the coefficient half (conjugate split) is block-uniform (kBlock divides N / 2), so the
// coefficient loads are uniform; the term loops are unrolled by 4 so that four terms' operand
// loads are in flight together
__global__ void __launch_bounds__(kBlock) k_lut_bivariate(u32* out, LutOperands op, int n_a, const u32* __restrict__ cst, int nl,
                                                          const PrimeConst* pc, int logn) {
    const int t = blockIdx.y, mb = blockIdx.z;
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const int half = (int)(((size_t)blockIdx.x * kBlock) >> (logn - 1));
    const PrimeConst P = pc[t];
    const u32 q = P.q;
    const size_t off = ((size_t)t << logn) + k;
    out += (size_t)mb * 3 * ((size_t)nl << logn);
    // 64-bit multiply-adds (operands < q < 2^30: 8 products fit beside a folded sum), one
    // reduction per inner sum and per output -- the same residues as a reduction per term
    u64 acc0 = 0, acc1 = 0, acc2 = 0;
    int pc_ = 0;
    for (int p = 0; p < n_a; ++p) {
        const int t0 = op.p_start[p], t1 = op.p_start[p + 1];
        if (t0 == t1) continue;
        u64 s0 = 0, s1 = 0;
#pragma unroll 4
        for (int j = t0; j < t1; ++j) {
            if (j > t0 && ((j - t0) & 7) == 0) s0 = fold64(s0, q, P.r32), s1 = fold64(s1, q, P.r32);
            const int qq = op.q_of[j];
            const u32* bq = op.b[qq] + (size_t)mb * 2 * ((size_t)op.nb[qq] << logn);
            const u32 c = cst[((size_t)j * nl + t) * 4 + 2 * half];
            s0 += (u64)bq[off] * c;
            s1 += (u64)bq[((size_t)op.nb[qq] << logn) + off] * c;
        }
        const u32 u0 = reduce64(s0, q, P.mu, P.r32), u1 = reduce64(s1, q, P.mu, P.r32);
        const u32* ap = op.a[p] + (size_t)mb * 2 * ((size_t)op.na[p] << logn);
        const u32 a0 = ap[off], a1 = ap[((size_t)op.na[p] << logn) + off];
        if (pc_ == 4) acc0 = fold64(acc0, q, P.r32), acc1 = fold64(acc1, q, P.r32), acc2 = fold64(acc2, q, P.r32), pc_ = 0;
        acc0 += (u64)a0 * u0;
        acc1 += (u64)a0 * u1 + (u64)a1 * u0;  // two products per step: fold every 4 steps
        acc2 += (u64)a1 * u1;
        ++pc_;
    }
    out[off] = reduce64(acc0, q, P.mu, P.r32);
    out[((size_t)nl << logn) + off] = reduce64(acc1, q, P.mu, P.r32);
    out[((size_t)(2 * nl) << logn) + off] = reduce64(acc2, q, P.mu, P.r32);
}

// k_lut_bivariate with the B elements staged once per thread: each thread reads B_q at its own offset once
// (into LDS used as per-thread indexable storage: a thread reads back only what it wrote, no barrier) instead
// of once per A_p term group -- the same terms, folds and reductions in the same order, so the same residues.
// Dynamic LDS: 2 n_b kBlock words
// (used: the B indices some term reads -- the others may be unset)
__global__ void __launch_bounds__(kBlock) k_lut_bivariate_lds(u32* out, LutOperands op, int n_a, int n_b, unsigned used, const u32* __restrict__ cst,
                                                              int nl, const PrimeConst* pc, int logn) {
    extern __shared__ u32 sbv[];
    const int t = blockIdx.y, mb = blockIdx.z;
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const int half = (int)(((size_t)blockIdx.x * kBlock) >> (logn - 1));
    const PrimeConst P = pc[t];
    const u32 q = P.q;
    const size_t off = ((size_t)t << logn) + k;
    out += (size_t)mb * 3 * ((size_t)nl << logn);
    for (int qq = 0; qq < n_b; ++qq) {
        if (!((used >> qq) & 1u)) continue;
        const u32* bq = op.b[qq] + (size_t)mb * 2 * ((size_t)op.nb[qq] << logn);
        sbv[(2 * qq) * kBlock + threadIdx.x] = bq[off];
        sbv[(2 * qq + 1) * kBlock + threadIdx.x] = bq[((size_t)op.nb[qq] << logn) + off];
    }
    u64 acc0 = 0, acc1 = 0, acc2 = 0;
    int pc_ = 0;
    for (int p = 0; p < n_a; ++p) {
        const int t0 = op.p_start[p], t1 = op.p_start[p + 1];
        if (t0 == t1) continue;
        u64 s0 = 0, s1 = 0;
#pragma unroll 4
        for (int j = t0; j < t1; ++j) {
            if (j > t0 && ((j - t0) & 7) == 0) s0 = fold64(s0, q, P.r32), s1 = fold64(s1, q, P.r32);
            const int qq = op.q_of[j];
            const u32 c = cst[((size_t)j * nl + t) * 4 + 2 * half];
            s0 += (u64)sbv[(2 * qq) * kBlock + threadIdx.x] * c;
            s1 += (u64)sbv[(2 * qq + 1) * kBlock + threadIdx.x] * c;
        }
        const u32 u0 = reduce64(s0, q, P.mu, P.r32), u1 = reduce64(s1, q, P.mu, P.r32);
        const u32* ap = op.a[p] + (size_t)mb * 2 * ((size_t)op.na[p] << logn);
        const u32 a0 = ap[off], a1 = ap[((size_t)op.na[p] << logn) + off];
        if (pc_ == 4) acc0 = fold64(acc0, q, P.r32), acc1 = fold64(acc1, q, P.r32), acc2 = fold64(acc2, q, P.r32), pc_ = 0;
        acc0 += (u64)a0 * u0;
        acc1 += (u64)a0 * u1 + (u64)a1 * u0;
        acc2 += (u64)a1 * u1;
        ++pc_;
    }
    out[off] = reduce64(acc0, q, P.mu, P.r32);
    out[((size_t)nl << logn) + off] = reduce64(acc1, q, P.mu, P.r32);
    out[((size_t)(2 * nl) << logn) + off] = reduce64(acc2, q, P.mu, P.r32);
}

// grid z = member of stacked elements (element j of member m at x[j] + m npoly nx[j] N, out / acc
// at + m npoly nl N)
// (k_lut_bivariate's uniform coefficient half and unrolled term loop)
// has_c: cadd's constant added to every member's first polynomial after the reduction (as k_lincomb's
// add_scalar launch would: the EvalMod Chebyshev leaves' c_0)
__global__ void __launch_bounds__(kBlock) k_lut_univariate(u32* out, const u32* acc, LutChunk ch, int n, const u32* __restrict__ cst,
                                                           int npoly, int nl, const PrimeConst* pc, int logn, LimbConsts cadd, int has_c) {
    const int t = blockIdx.y, mb = blockIdx.z;
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const int half = (int)(((size_t)blockIdx.x * kBlock) >> (logn - 1));
    const PrimeConst P = pc[t];
    const u32 q = P.q;
    const size_t off = ((size_t)t << logn) + k;
    const size_t mo = (size_t)mb * npoly * ((size_t)nl << logn);
    for (int p = 0; p < npoly; ++p) {
        const size_t o = mo + ((size_t)(p * nl) << logn) + off;
        u64 v = acc ? acc[o] : 0;  // 64-bit multiply-adds, folded every 8 terms, one reduction
#pragma unroll 4
        for (int j = 0; j < n; ++j) {
            if (j && (j & 7) == 0) v = fold64(v, q, P.r32);
            const u32 c = cst[((size_t)j * nl + t) * 4 + 2 * half];
            const u32* xj = ch.x[j] + (size_t)mb * npoly * ((size_t)ch.nx[j] << logn);
            v += (u64)xj[((size_t)(p * ch.nx[j]) << logn) + off] * c;
        }
        u32 r = reduce64(v, q, P.mu, P.r32);
        if (has_c && p == 0) r = add_mod(r, cadd.v[2 * t + half], q);
        out[o] = r;
    }
}

inline double words(double w) { return 4.0 * w; }
}  // namespace

// ======================================================================================
// launch wrappers
// ======================================================================================
#define EW_BYTES(bytes_words) words((double)(bytes_words) * (1u << T.logn))
void launch_add(hipStream_t st, const DevTables& T, u32* out, const u32* a, const u32* b, int rows, int nl, LimbMap map) {
    prof_launch(KID_ELEMENTWISE, EW_BYTES(3.0 * rows), k_add, ew_grid(T.logn, rows), dim3(kBlock), 0, st, out, a, b, nl, map, T.pc, T.logn);
}
void launch_sub(hipStream_t st, const DevTables& T, u32* out, const u32* a, const u32* b, int rows, int nl, LimbMap map) {
    prof_launch(KID_ELEMENTWISE, EW_BYTES(3.0 * rows), k_sub, ew_grid(T.logn, rows), dim3(kBlock), 0, st, out, a, b, nl, map, T.pc, T.logn);
}
void launch_copy_rows(hipStream_t st, const DevTables& T, u32* out, const u32* in, size_t rows) {
    if (rows == 0 || out == in) return;
    if (rows > 65535) throw std::runtime_error("launch_copy_rows: too many rows");
    prof_launch(KID_ELEMENTWISE, EW_BYTES(2.0 * rows), k_copy_rows, dim3((1u << T.logn) / (4 * kBlock), (unsigned)rows), dim3(kBlock), 0, st,
                reinterpret_cast<uint4*>(out), reinterpret_cast<const uint4*>(in), T.logn);
}
void launch_copy_members(hipStream_t st, const DevTables& T, const MemberPtrs& mp, int n, int rows) {
    if (n <= 0 || rows <= 0) return;
    if (n > kMaxMembers) throw std::runtime_error("launch_copy_members: too many members");
    prof_launch(KID_ELEMENTWISE, EW_BYTES(2.0 * n * rows), k_copy_members, dim3((1u << T.logn) / (4 * kBlock), rows, n), dim3(kBlock), 0,
                st, mp, T.logn);
}
void launch_add_members(hipStream_t st, const DevTables& T, u32* out, const MemberPtrs& mp, int n, int rows, LimbMap map, bool accumulate) {
    if (n <= 0 || n > kMaxMembers) throw std::runtime_error("launch_add_members: 1..8 sources");
    prof_launch(KID_ELEMENTWISE, EW_BYTES((n + 1.0 + (accumulate ? 1.0 : 0.0)) * rows), k_add_members, ew_grid(T.logn, rows), dim3(kBlock), 0,
                st, out, mp, n, map, T.pc, T.logn, (int)accumulate);
}
void launch_tensor_ptrs(hipStream_t st, const DevTables& T, u32* out, const TensorPtrs& tp, int n, int nl, LimbMap map) {
    if (n <= 0 || n > kMaxMembers) throw std::runtime_error("launch_tensor_ptrs: 1..8 products");
    prof_launch(KID_TENSOR, words(7.0 * n * nl * (1u << T.logn)), k_tensor_ptrs, ew_grid(T.logn, n * nl), dim3(kBlock), 0, st, out, tp, nl,
                map, T.pc, T.logn);
}
void launch_neg(hipStream_t st, const DevTables& T, u32* out, const u32* a, int rows, int nl, LimbMap map) {
    prof_launch(KID_ELEMENTWISE, EW_BYTES(2.0 * rows), k_neg, ew_grid(T.logn, rows), dim3(kBlock), 0, st, out, a, nl, map, T.pc, T.logn);
}
void launch_square(hipStream_t st, const DevTables& T, u32* out, const u32* a, int rows, int nl, LimbMap map) {
    prof_launch(KID_ELEMENTWISE, EW_BYTES(2.0 * rows), k_square, ew_grid(T.logn, rows), dim3(kBlock), 0, st, out, a, nl, map, T.pc, T.logn);
}
void launch_tensor(hipStream_t st, const DevTables& T, u32* out, const u32* a, const u32* b, int nl, LimbMap map, int nb) {
    prof_launch(KID_TENSOR, words(7.0 * nb * nl * (1u << T.logn)), k_tensor, ew_grid(T.logn, nb * nl), dim3(kBlock), 0, st, out, a, b, nl,
                map, T.pc, T.logn);
}
void launch_mul_poly(hipStream_t st, const DevTables& T, u32* out, const u32* in, const u32* pt, int npoly, int nl, LimbMap map) {
    prof_launch(KID_ELEMENTWISE, EW_BYTES((2.0 * npoly + 1.0) * nl), k_mul_poly, ew_grid(T.logn, npoly * nl), dim3(kBlock), 0, st, out, in, pt, nl, map, T.pc, T.logn);
}
void launch_mul_poly_sum(hipStream_t st, const DevTables& T, u32* out, const PtSumArgs& a, int n, int npoly, int nl, LimbMap map) {
    if (n < 1 || n > kMaxMembers) throw std::runtime_error("launch_mul_poly_sum: 1..8 products");
    prof_launch(KID_ELEMENTWISE, EW_BYTES((double)npoly * nl * (n + 1) + (double)n * nl), k_mul_poly_sum, ew_grid(T.logn, npoly * nl), dim3(kBlock), 0,
                st, out, a, n, nl, map, T.pc, T.logn);
}
void launch_fma_poly(hipStream_t st, const DevTables& T, u32* out, const u32* a, const u32* b, const u32* c, int rows, int nl,
                     LimbMap map) {
    prof_launch(KID_ELEMENTWISE, EW_BYTES(3.0 * rows + nl), k_fma_poly, ew_grid(T.logn, rows), dim3(kBlock), 0, st, out, a, b, c, nl, map, T.pc, T.logn);
}
void launch_mul_const_half(hipStream_t st, const DevTables& T, u32* out, const u32* in, const LimbConsts& cst, int rows, int nl, LimbMap map,
                           int src_nl) {
    prof_launch(KID_ELEMENTWISE, EW_BYTES(2.0 * rows), k_mul_const_half, ew_grid(T.logn, rows), dim3(kBlock), 0, st, out, in, cst, nl,
                src_nl > 0 ? src_nl : nl, map, T.pc, T.logn);
}
void launch_mul_const_half_members(hipStream_t st, const DevTables& T, u32* out, const MemberPtrs& mp, int n, const LimbConsts& cst,
                                   int rows, int nl, LimbMap map, int src_nl) {
    if (n < 1 || n > kMaxMembers) throw std::runtime_error("launch_mul_const_half_members: 1..8 members");
    prof_launch(KID_ELEMENTWISE, EW_BYTES(2.0 * rows * n), k_mul_const_half_members, dim3((1u << T.logn) / kBlock, rows, n), dim3(kBlock), 0,
                st, out, mp, cst, rows, nl, src_nl, map, T.pc, T.logn);
}
void launch_addsub_tail(hipStream_t st, const DevTables& T, u32* out, const u32* a, const u32* b, int common, int rows, bool a_longer,
                        bool sub, int nl, LimbMap map) {
    prof_launch(KID_ELEMENTWISE, EW_BYTES(3.0 * common + 2.0 * (rows - common)), k_addsub_tail, ew_grid(T.logn, rows), dim3(kBlock), 0,
                st, out, a, b, common, (int)a_longer, (int)sub, nl, map, T.pc, T.logn);
}
void launch_add_const_half(hipStream_t st, const DevTables& T, u32* out, const u32* in, const LimbConsts& cst, int rows, int nl, LimbMap map) {
    prof_launch(KID_ELEMENTWISE, EW_BYTES(2.0 * rows), k_add_const_half, ew_grid(T.logn, rows), dim3(kBlock), 0, st, out, in, cst, nl, map, T.pc, T.logn);
}
void launch_lincomb(hipStream_t st, const DevTables& T, u32* out, const u32* a, const LimbConsts& ka, const u32* b, int bsign,
                    const LimbConsts* cadd, int per, int rows, int nl, LimbMap map) {
    static const LimbConsts kNone{};
    prof_launch(KID_ELEMENTWISE, EW_BYTES((b ? 3.0 : 2.0) * rows), k_lincomb, ew_grid(T.logn, rows), dim3(kBlock), 0, st, out, a, ka, b, bsign,
                cadd ? *cadd : kNone, cadd ? 1 : 0, per, nl, map, T.pc, T.logn);
}
void launch_automorph(hipStream_t st, const DevTables& T, u32* out, const u32* in, u64 g, int rows) {
    prof_launch(KID_AUTOMORPH, words(2.0 * rows * (1u << T.logn)), k_automorph, ew_grid(T.logn, rows), dim3(kBlock), 0, st, out, in, g, T.logn);
}
void launch_rescale_spread(hipStream_t st, const DevTables& T, u32* v, const u32* last, int npoly, int nt, u32 q_last) {
    prof_launch(KID_RESCALE, words((double)npoly * (1 + nt) * (1u << T.logn)), k_rescale_spread, dim3((1u << T.logn) / kBlock, nt, npoly), dim3(kBlock), 0, st, v, last, nt, q_last, T.pc,
                       T.logn);
}
void launch_crt2_spread(hipStream_t st, const DevTables& T, u32* v, const u32* src, int npoly, int nt, u32 q0, u32 q1) {
    if (q0 >= q1 && q0 % q1 == 0) throw std::runtime_error("launch_crt2_spread: bad primes");
    u64 inv = 1, b = q0 % q1, e = q1 - 2;  // q0^{-1} mod q1 (Fermat)
    while (e) {
        if (e & 1) inv = inv * b % q1;
        b = b * b % q1;
        e >>= 1;
    }
    prof_launch(KID_RESCALE, words((double)npoly * (2 + nt) * (1u << T.logn)), k_crt2_spread, dim3((1u << T.logn) / kBlock, nt, npoly),
                dim3(kBlock), 0, st, v, src, nt, q0, q1, (u32)inv, shoup_pre((u32)inv, q1), T.pc, T.logn);
}
// coefficients per thread of k_base_convert (AESFHE_CONV_VEC = 1 or 2)
inline int conv_vec() {
    static const int v = [] {
        const char* e = std::getenv("AESFHE_CONV_VEC");
        const int x = e ? std::atoi(e) : 1;
        return x == 2 ? 2 : 1;
    }();
    return v;
}
void launch_base_convert(hipStream_t st, const DevTables& T, const ConvBatch& cb, int nt, LimbMap map) {
    double w = 0;
    for (int g = 0; g < cb.n; ++g) {
        const bool own = cb.skip0[g] >= 0 && cb.skip0[g] < nt;
        w += cb.h[g] + nt - (own ? std::min(cb.h[g], nt - cb.skip0[g]) : 0);
    }
    const dim3 grid_y((nt + kConvTargets - 1) / kConvTargets, cb.n);
    switch (conv_vec()) {
        case 2:
            prof_launch_ts(KID_BASE_CONVERT, words(w * (1u << T.logn)), k_base_convert<2>, dim3((1u << T.logn) / (2 * kBlock), grid_y.x, grid_y.y),
                           dim3(kBlock), 0, st, cb, nt, map, T.pc, T.logn);
            break;
        default:
            prof_launch_ts(KID_BASE_CONVERT, words(w * (1u << T.logn)), k_base_convert<1>, dim3((1u << T.logn) / kBlock, grid_y.x, grid_y.y),
                           dim3(kBlock), 0, st, cb, nt, map, T.pc, T.logn);
    }
}

namespace {
// out[p][t] = sum_j x_j[p][t] * pt_j[t]  (mod the limb's prime): the diagonal products of
// a linear transform, all terms of one giant step in one pass (64-bit multiply-adds)
__global__ void k_mac(u32* out, MacTerms m, size_t xs, size_t os, LimbMap map, const PrimeConst* pc, int logn) {
    const int t = blockIdx.y, p = blockIdx.z;
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t at = ((size_t)t << logn) + k;
    const PrimeConst P = pc[map.prime(t)];
    u64 acc = 0;
    for (int j = 0; j < m.n; ++j) {
        if (j && (j & 7) == 0) acc = fold64(acc, P.q, P.r32);
        acc += (u64)m.x[j][p * xs + at] * m.pt[j][at];
    }
    out[p * os + at] = reduce64(acc, P.q, P.mu, P.r32);
}
// see launch_lin_mac (kernels.h); grid (N / 256, ne rows, nb batched ciphertexts).  The
// diagonals are read once per residue and applied to every batched ciphertext (member loop
// inside the thread); kLinG x 3 accumulators per member.
// ND > 0: the digit count is a compile-time constant, so the digit loop of a baby step's key
// inner product unrolls and its 2 * ND key loads and NB * ND ext gathers are all in flight
// together (the loop with a run-time bound waited for each digit's loads in turn: the
// kernel was load-latency-bound at ~1.3 TB/s); ND = 0 keeps the run-time loop (nd > 8)
template <int NB, int ND>
__device__ __forceinline__ void lin_mac_body(const LinMacArgs& m, int nl, int ne, const PrimeConst& P, int t, size_t k, int logn) {
    const bool qrow = t < nl;
    const size_t at = ((size_t)t << logn) + k;
    const size_t po = (size_t)ne << logn;  // poly stride of u / outp
    u64 acc0[NB][kLinG], ap0[NB][kLinG], ap1[NB][kLinG];
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int g = 0; g < kLinG; ++g) acc0[b][g] = ap0[b][g] = ap1[b][g] = 0;
    for (int j = 0; j < m.B; ++j) {
        if (j && (j & 7) == 0) {
#pragma unroll
            for (int b = 0; b < NB; ++b)
#pragma unroll
                for (int g = 0; g < kLinG; ++g) {
                    acc0[b][g] = fold64(acc0[b][g], P.q, P.r32);
                    ap0[b][g] = fold64(ap0[b][g], P.q, P.r32);
                    ap1[b][g] = fold64(ap1[b][g], P.q, P.r32);
                }
        }
        u32 av[NB], u0[NB], u1[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            av[b] = 0u;
            if (qrow && m.a[j])
                av[b] = m.a[j][b * m.q_ms + ((size_t)t << logn) + (m.gal[j] ? galois_src((u32)k, m.gal[j], logn) : k)];
            u0[b] = u1[b] = 0;
            if (m.u[j]) u0[b] = m.u[j][b * m.p_ms + at], u1[b] = m.u[j][b * m.p_ms + po + at];
        }
        if (m.key[j]) {  // the baby step's key inner product, in place (k_key_inner's sum)
            const size_t ks = galois_src((u32)k, m.gal[j], logn);
            const int krow = qrow ? t : m.nks + (t - nl);
            const int own = qrow ? t / m.alpha : -1;
            u64 s0[NB] = {}, s1[NB] = {};
            const int nd = ND > 0 ? ND : m.nd;
#pragma unroll
            for (int dj = 0; dj < nd; ++dj) {
                if (dj && (dj & 7) == 0) {
#pragma unroll
                    for (int b = 0; b < NB; ++b) s0[b] = fold64(s0[b], P.q, P.r32), s1[b] = fold64(s1[b], P.q, P.r32);
                }
                const u32* kb = m.key[j] + (((size_t)dj * 2 * m.nkey + krow) << logn) + k;
                const u64 vb = kb[0], va = kb[(size_t)m.nkey << logn];
#pragma unroll
                for (int b = 0; b < NB; ++b) {
                    const u32 e = dj == own ? m.ks_d[b * m.d_ms + ((size_t)t << logn) + ks]
                                            : m.ks_ext[b * m.ext_ms + (((size_t)dj * ne + t) << logn) + ks];
                    s0[b] += e * vb;
                    s1[b] += e * va;
                }
            }
#pragma unroll
            for (int b = 0; b < NB; ++b) u0[b] = reduce64(s0[b], P.q, P.mu, P.r32), u1[b] = reduce64(s1[b], P.q, P.mu, P.r32);
        }
#pragma unroll
        for (int g = 0; g < kLinG; ++g) {
            if (g >= m.G || !m.pt[g][j]) continue;
            const u32 pv = m.pt_shift ? m.pt[g][j][((size_t)t << m.pt_logc) + (k >> m.pt_shift)] : m.pt[g][j][at];
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                acc0[b][g] += (u64)av[b] * pv;  // q < 2^30: 8 products fit beside a folded accumulator
                ap0[b][g] += (u64)u0[b] * pv;
                ap1[b][g] += (u64)u1[b] * pv;
            }
        }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const u32 c1v = qrow ? m.c1[b * m.q_ms + at] : 0u;
#pragma unroll
        for (int g = 0; g < kLinG; ++g) {
            if (g >= m.G) continue;
            u32 o0 = 0, o1 = 0;
            if (qrow) {
                o0 = reduce64(acc0[b][g], P.q, P.mu, P.r32);
                if (m.pt[g][0]) {
                    const u32 p0 = m.pt_shift ? m.pt[g][0][((size_t)t << m.pt_logc) + (k >> m.pt_shift)] : m.pt[g][0][at];
                    o1 = reduce64((u64)c1v * p0, P.q, P.mu, P.r32);
                }
            }
            const bool fold = m.gad && m.outp[g];
            if (qrow && !fold) {
                m.out0[g][b * m.q_ms + at] = o0;
                if (m.out1[g]) m.out1[g][b * m.q_ms + at] = o1;
            }
            if (m.outp[g]) {
                u32 p0 = reduce64(ap0[b][g], P.q, P.mu, P.r32), p1 = reduce64(ap1[b][g], P.q, P.mu, P.r32);
                if (fold && qrow) {
                    const u32 gv = m.gad[2 * t], gp = m.gad[2 * t + 1];
                    p0 = add_mod(p0, shoup_mul(o0, gv, gp, P.q), P.q);
                    p1 = add_mod(p1, shoup_mul(o1, gv, gp, P.q), P.q);
                }
                m.outp[g][b * m.p_ms + at] = p0;
                m.outp[g][b * m.p_ms + po + at] = p1;
            }
        }
    }
}
template <int NB, int ND>
__global__ void __launch_bounds__(kBlock) k_lin_mac(LinMacArgs m, int nl, int ne, LimbMap map, const PrimeConst* pc, int logn, int xcd) {
    int t = blockIdx.y, bx = blockIdx.x;
    // the baby steps gather c0 and ext of row t through B different automorphisms: one XCD per row
    if (xcd) xcd_rows(logn - 8, ne, bx, t);
    const size_t k = (size_t)bx * kBlock + threadIdx.x;
    const PrimeConst P = pc[map.prime(t)];
    lin_mac_body<NB, ND>(m, nl, ne, P, t, k, logn);
}
// AESFHE_XCD_ROWS=0: the plain block map (A/B runs)
inline int xcd_rows_on() {
    static const int v = [] {
        const char* e = std::getenv("AESFHE_XCD_ROWS");
        return e ? std::atoi(e) : 1;
    }();
    return v;
}
// AESFHE_LIN_MAC_NB1=1: stacked members one per launch instead of pairs (A/B of the stacked
// bootstrap's L2 working set: a pair's gathered c0 / ext row bands are twice a single member's)
inline bool lin_mac_nb1() {
    static const bool v = std::getenv("AESFHE_LIN_MAC_NB1") && std::atoi(std::getenv("AESFHE_LIN_MAC_NB1")) != 0;
    return v;
}
// AESFHE_LIN_MAC_NB4=1: a four-member chunk in one launch (A/B; off: see launch_lin_mac)
inline bool lin_mac_nb4() {
    static const bool v = std::getenv("AESFHE_LIN_MAC_NB4") && std::atoi(std::getenv("AESFHE_LIN_MAC_NB4")) != 0;
    return v;
}
template <int NB>
void launch_lin_mac_nb(hipStream_t st, const DevTables& T, const LinMacArgs& m, int nl, int ne, LimbMap map, double bytes) {
    static_assert(kBlock == 256, "xcd_rows assumes N / 256 column blocks");
    const dim3 g = ew_grid(T.logn, ne), b(kBlock);
    const int xcd = xcd_rows_on();
    switch (m.nd) {  // the digit counts of the bootstrap plans (dnum <= 8); others take the run-time loop
#define LIN_MAC_ND(D) \
    case D: prof_launch(KID_LIN_MAC, bytes, k_lin_mac<NB, D>, g, b, 0, st, m, nl, ne, map, T.pc, T.logn, xcd); break;
        LIN_MAC_ND(1) LIN_MAC_ND(2) LIN_MAC_ND(3) LIN_MAC_ND(4) LIN_MAC_ND(5) LIN_MAC_ND(6) LIN_MAC_ND(7) LIN_MAC_ND(8)
#undef LIN_MAC_ND
        default: prof_launch(KID_LIN_MAC, bytes, k_lin_mac<NB, 0>, g, b, 0, st, m, nl, ne, map, T.pc, T.logn, xcd);
    }
}
}  // namespace

void launch_lin_mac(hipStream_t st, const DevTables& T, const LinMacArgs& m, int nl, int ne, LimbMap map) {
    if (m.B < 1 || m.B > kLinB || m.G < 1 || m.G > kLinG) throw std::runtime_error("launch_lin_mac: 1..16 baby, 1..5 giant steps");
    // algorithmic bytes: every distinct input row read once (the baby steps re-read c0 and the
    // hoisted ext through their automorphisms -- from L2 / MALL), every output written once
    double member = 0, writes = 0, shared = 0;  // rows of N words; member: per batched ciphertext
    bool any_a = false, any_key = false;
    for (int b = 0; b < m.B; ++b) {
        any_a = any_a || m.a[b];
        any_key = any_key || m.key[b];
        if (m.u[b]) member += 2.0 * ne;
        if (m.key[b]) shared += 2.0 * m.nd * ne;  // the key, read once for every batched ciphertext
        for (int g = 0; g < m.G; ++g)
            if (m.pt[g][b]) shared += m.pt_shift ? ne * (double)(1 << m.pt_logc) / (1u << T.logn) : ne;  // the diagonals likewise
    }
    if (any_a) member += nl;                      // c0
    if (any_key) member += (double)m.nd * ne;     // the hoisted ModUp of c1 (ext)
    member += nl;                                 // c1
    for (int g = 0; g < m.G; ++g)
        writes += (m.gad && m.outp[g]) ? 2.0 * ne : nl + (m.out1[g] ? nl : 0) + (m.outp[g] ? 2.0 * ne : 0);
    const double bytes = words((m.nb * (member + writes) + shared) * (1u << T.logn));
    static const bool trace = std::getenv("AESFHE_LINMAC_TRACE") != nullptr;
    if (trace) {
        int nkeys = 0, npt = 0, na = 0, nu = 0;
        for (int b = 0; b < m.B; ++b) {
            nkeys += m.key[b] != nullptr, na += m.a[b] != nullptr, nu += m.u[b] != nullptr;
            for (int g = 0; g < m.G; ++g) npt += m.pt[g][b] != nullptr;
        }
        std::fprintf(stderr, "lin_mac B=%d G=%d nb=%d nd=%d nl=%d ne=%d keys=%d pts=%d a=%d u=%d rows_member=%.0f rows_write=%.0f rows_shared=%.0f MB=%.1f\n",
                     m.B, m.G, m.nb, m.nd, nl, ne, nkeys, npt, na, nu, member, writes, shared, bytes / 1e6);
    }
    if (m.nb == 1) {
        launch_lin_mac_nb<1>(st, T, m, nl, ne, map, bytes);
    } else if (m.nb == 2 && !lin_mac_nb1()) {
        launch_lin_mac_nb<2>(st, T, m, nl, ne, map, bytes);
    } else if (m.nb == 4 && lin_mac_nb4()) {
        // a stacked bootstrap chunk of four members in ONE launch (AESFHE_LIN_MAC_NB4=1, off): each
        // key and diagonal residue read once for all four -- but the baby steps' gathers of c0 and
        // the hoisted ext rows of four members (~6 MB per row band) no longer fit one XCD's 4 MB L2:
        // 2,846 us per launch against 2 x 435 us as two pair launches (64-pair stack,
        // profiles/r5_linmac_nb4_ab.txt)
        launch_lin_mac_nb<4>(st, T, m, nl, ne, map, bytes);
    } else if (m.nb >= 2) {
        // wider batches (a stacked bootstrap chunk of more than two members): pairs of members, one
        // launch each, every member-strided operand offset to the pair's first member
        const int step = lin_mac_nb1() ? 1 : 2;
        for (int m0 = 0; m0 < m.nb; m0 += step) {
            LinMacArgs s = m;
            s.nb = std::min(step, m.nb - m0);
            const size_t qo = (size_t)m0 * m.q_ms, po = (size_t)m0 * m.p_ms;
            for (int b = 0; b < m.B; ++b) {
                if (s.a[b]) s.a[b] += qo;
                if (s.u[b]) s.u[b] += po;
            }
            if (s.c1) s.c1 += qo;
            for (int g = 0; g < m.G; ++g) {
                if (s.out0[g]) s.out0[g] += qo;
                if (s.out1[g]) s.out1[g] += qo;
                if (s.outp[g]) s.outp[g] += po;
            }
            if (s.ks_ext) s.ks_ext += (size_t)m0 * m.ext_ms;
            if (s.ks_d) s.ks_d += (size_t)m0 * m.d_ms;
            const double b2 = bytes * s.nb / m.nb;
            if (s.nb == 1) launch_lin_mac_nb<1>(st, T, s, nl, ne, map, b2);
            else launch_lin_mac_nb<2>(st, T, s, nl, ne, map, b2);
        }
    } else {
        throw std::runtime_error("launch_lin_mac: at least one ciphertext");
    }
}

void launch_mac(hipStream_t st, const DevTables& T, u32* out, const MacTerms& m, size_t xs, size_t os, int rows, int npoly, LimbMap map) {
    if (m.n < 1 || m.n > kMacMax) throw std::runtime_error("launch_mac: 1..16 terms");
    prof_launch(KID_ELEMENTWISE, words((2.0 * m.n + 1.0) * npoly * rows * (1u << T.logn)), k_mac,
                dim3((1u << T.logn) / kBlock, rows, npoly), dim3(kBlock), 0, st, out, m, xs, os, map, T.pc, T.logn);
}

// AESFHE_KI_UNROLL=0: k_key_inner with the run-time digit loop for every launch (A/B runs)
inline bool ki_unroll() {
    static const bool v = [] {
        const char* e = std::getenv("AESFHE_KI_UNROLL");
        return !(e && std::atoi(e) == 0);
    }();
    return v;
}
template <int NBM>
void key_inner_nd(int ndc, double bytes, dim3 grid, hipStream_t st, u32* acc, const u32* ext, const u32* d, const u32* key, int nd, int ne,
                  int nl, int alpha, int nkey, int nks, u64 g, LimbMap map, const DevTables& T, int nb, size_t ext_ms, size_t d_ms,
                  size_t acc_ms, KsFold fold, bool accum) {
    switch (ndc) {
#define KI_ND(D) \
    case D: \
        prof_launch_ts(KID_KEY_INNER, bytes, k_key_inner<NBM, D>, grid, dim3(kBlock), 0, st, acc, ext, d, key, nd, ne, nl, alpha, nkey, nks, g, \
                       map, T.pc, T.logn, nb, ext_ms, d_ms, acc_ms, fold, (int)accum); \
        break;
        KI_ND(1) KI_ND(2) KI_ND(3) KI_ND(4) KI_ND(5) KI_ND(6) KI_ND(7) KI_ND(8)
#undef KI_ND
        default:
            prof_launch_ts(KID_KEY_INNER, bytes, k_key_inner<NBM>, grid, dim3(kBlock), 0, st, acc, ext, d, key, nd, ne, nl, alpha, nkey, nks,
                           g, map, T.pc, T.logn, nb, ext_ms, d_ms, acc_ms, fold, (int)accum);
    }
}
void launch_key_inner(hipStream_t st, const DevTables& T, u32* acc, const u32* ext, const u32* d, const u32* key, int nd, int ne, int nl,
                      int alpha, int nkey, int nks, LimbMap map, u64 g, int nb, size_t ext_ms, size_t d_ms, size_t acc_ms, KsFold fold,
                      bool accum) {
    if (nb < 1 || nb > kMaxKsBatch) throw std::runtime_error("launch_key_inner: 1..8 batched ciphertexts");
    if (fold.gad && g) throw std::runtime_error("launch_key_inner: fold with an automorphism");
    // the reversed own-digit read is the conjugation's (identity Galois element, no tensor fold): with
    // g != 0 the kernel would ignore g on the own digit, in tensor mode it never reaches the branch
    if (fold.rev_d && (g || fold.ta[0])) throw std::runtime_error("launch_key_inner: reversed d needs g == 0 and no tensor fold");
    // per ciphertext ext/d (nd x ne) read and acc (2 x ne) written; the key (nd x 2 x ne) once;
    // the fold reads 2 x nl more rows per ciphertext
    // tensor mode (fold.ta): the fold reads a0, a1, b0, b1 and the own digit a1, b1 (one row more
    // per q limb than the materialised c2) instead of c0, c1
    const double fw = (fold.gad ? (fold.ta[0] ? 5.0 : 2.0) * nb * nl : 0.0) + (accum ? 2.0 * nb * ne : 0.0);
    const double bytes = words(((nb * (nd + 2.0) + 2.0 * nd) * ne + fw) * (1u << T.logn));
    const dim3 grid((1u << T.logn) / (4 * kBlock), ne);
    // register footprint follows the batch: 1, 2, 4 or 8 ciphertexts; up to 4, the digit count
    // as a template constant (ki_unroll(), k_key_inner's ND)
    const int ndc = (ki_unroll() && nd >= 1 && nd <= 8 && nb <= 4) ? nd : 0;
    if (nb == 1)
        key_inner_nd<1>(ndc, bytes, grid, st, acc, ext, d, key, nd, ne, nl, alpha, nkey, nks, g, map, T, nb, ext_ms, d_ms, acc_ms, fold, accum);
    else if (nb == 2)
        key_inner_nd<2>(ndc, bytes, grid, st, acc, ext, d, key, nd, ne, nl, alpha, nkey, nks, g, map, T, nb, ext_ms, d_ms, acc_ms, fold, accum);
    else if (nb <= 4)
        key_inner_nd<4>(ndc, bytes, grid, st, acc, ext, d, key, nd, ne, nl, alpha, nkey, nks, g, map, T, nb, ext_ms, d_ms, acc_ms, fold, accum);
    else
        prof_launch_ts(KID_KEY_INNER, bytes, k_key_inner<8>, grid, dim3(kBlock), 0, st, acc, ext, d, key, nd, ne, nl, alpha, nkey, nks, g,
                       map, T.pc, T.logn, nb, ext_ms, d_ms, acc_ms, fold, (int)accum);
}
void launch_key_inner_sum(hipStream_t st, const DevTables& T, u32* acc, const u32* ext, const u32* d, const KsSumArgs& ka, int nb, int nd,
                          int ne, int nl, int alpha, int nkey, int nks, LimbMap map, size_t ext_ms, size_t d_ms, size_t acc_ms) {
    if (ka.J < 1 || ka.J > 4 || nb < 1) throw std::runtime_error("launch_key_inner_sum: 1..4 rotations");
    for (int i = 0; i < ka.J; ++i)
        if (!ka.key[i] || !ka.g[i]) throw std::runtime_error("launch_key_inner_sum: missing key or Galois element");
    // ext / d read once per member (the J gathers of a row hit L2), the J keys once, acc written
    const double bytes = words(((nb * (nd + 2.0) + 2.0 * nd * ka.J) * ne) * (1u << T.logn));
    switch ((ki_unroll() && nd >= 1 && nd <= 8) ? nd : 0) {
#define KIS_ND(D) \
    case D: \
        prof_launch_ts(KID_KEY_INNER, bytes, k_key_inner_sum<D>, dim3((1u << T.logn) / (4 * kBlock), ne, nb), dim3(kBlock), 0, st, acc, ext, d, ka, nd, \
                       ne, nl, alpha, nkey, nks, map, T.pc, T.logn, ext_ms, d_ms, acc_ms); \
        break;
        KIS_ND(1) KIS_ND(2) KIS_ND(3) KIS_ND(4) KIS_ND(5) KIS_ND(6) KIS_ND(7) KIS_ND(8)
#undef KIS_ND
        default:
            prof_launch_ts(KID_KEY_INNER, bytes, k_key_inner_sum<>, dim3((1u << T.logn) / (4 * kBlock), ne, nb), dim3(kBlock), 0, st, acc, ext,
                           d, ka, nd, ne, nl, alpha, nkey, nks, map, T.pc, T.logn, ext_ms, d_ms, acc_ms);
    }
}
void launch_automorph_sum(hipStream_t st, const DevTables& T, u32* out, const u32* in, const KsSumArgs& ka, int nb, int rows, size_t ms,
                          LimbMap map) {
    prof_launch(KID_AUTOMORPH, words(2.0 * rows * nb * (1u << T.logn)), k_automorph_sum, dim3((1u << T.logn) / kBlock, rows, nb), dim3(kBlock),
                0, st, out, in, ka, rows, ms, map, T.pc, T.logn);
}
void launch_key_inner_multi(hipStream_t st, const DevTables& T, u32* acc, const u32* ext, const u32* d, const KsMultiArgs& ka, int nm,
                            int nsrc, int nd, int ne, int nl, int alpha, int nkey, int nks, LimbMap map, size_t ext_ms, size_t d_ms,
                            size_t acc_ms) {
    if (nm < 1 || nm > kKsMulti) throw std::runtime_error("launch_key_inner_multi: 1..16 members");
    for (int m = 0; m < nm; ++m)
        if (!ka.key[m] || ka.src[m] < 0 || ka.src[m] >= nsrc) throw std::runtime_error("launch_key_inner_multi: bad member");
    // each member reads its source's ext / d and its key, writes acc; distinct sources' ext once
    const double bytes = words(((nsrc * (double)nd + nm * (2.0 * nd + 2.0)) * ne) * (1u << T.logn));
    switch ((ki_unroll() && nd >= 1 && nd <= 8) ? nd : 0) {
#define KIM_ND(D) \
    case D: \
        prof_launch_ts(KID_KEY_INNER, bytes, k_key_inner_multi<D>, dim3((1u << T.logn) / (4 * kBlock), ne, nm), dim3(kBlock), 0, st, acc, ext, d, \
                       ka, nd, ne, nl, alpha, nkey, nks, map, T.pc, T.logn, ext_ms, d_ms, acc_ms); \
        break;
        KIM_ND(1) KIM_ND(2) KIM_ND(3) KIM_ND(4) KIM_ND(5) KIM_ND(6) KIM_ND(7) KIM_ND(8)
#undef KIM_ND
        default:
        prof_launch_ts(KID_KEY_INNER, bytes, k_key_inner_multi<>, dim3((1u << T.logn) / (4 * kBlock), ne, nm), dim3(kBlock), 0, st, acc, ext, d,
                       ka, nd, ne, nl, alpha, nkey, nks, map, T.pc, T.logn, ext_ms, d_ms, acc_ms);
    }
}
void launch_automorph_multi(hipStream_t st, const DevTables& T, u32* out, size_t out_ms, const AutoMulti& am, int n, int rows) {
    if (n < 1 || n > kKsMulti) throw std::runtime_error("launch_automorph_multi: 1..16 members");
    prof_launch(KID_AUTOMORPH, words(2.0 * n * rows * (1u << T.logn)), k_automorph_multi, dim3((1u << T.logn) / kBlock, rows, n),
                dim3(kBlock), 0, st, out, out_ms, am, T.logn);
}
void launch_sample_small(hipStream_t st, const DevTables& T, u32* out, int nl, LimbMap map, const PrngKey& key, u64 stream, int kind) {
    prof_launch(KID_SAMPLE, words((double)nl * (1u << T.logn)), k_sample_small, dim3((1u << T.logn) / kBlock), dim3(kBlock), 0, st, out, nl, map, key, stream, kind, T.pc,
                       T.logn);
}
void launch_sample_enc(hipStream_t st, const DevTables& T, u32* out, int nl, int nm, const PrngKey& key, const EncCtrs& ctr, const u32* msg,
                       size_t msg_ms) {
    if (nm < 1 || nm > kEncMax) throw std::runtime_error("launch_sample_enc: too many encryptions");
    prof_launch(KID_SAMPLE, words((3.0 + (msg ? 1.0 : 0.0)) * nm * nl * (1u << T.logn)), k_sample_enc, dim3((1u << T.logn) / kBlock, 3 * nm),
                dim3(kBlock), 0, st, out, nl, key, ctr, msg, msg_ms, T.pc, T.logn);
}
void launch_enc_combine(hipStream_t st, const DevTables& T, u32* top, const u32* vee, const u32* msg, size_t msg_ms, const u32* pk,
                        int pk_rows, int nl, int nm) {
    prof_launch(KID_ELEMENTWISE, words((3.0 + (msg ? 1.0 : 0.0) + 2.0 + 2.0) * nm * nl * (1u << T.logn)), k_enc_combine, ew_grid(T.logn, nm * nl),
                dim3(kBlock), 0, st, top, vee, msg, msg_ms, pk, pk_rows, nl, T.pc, T.logn);
}
void launch_dec_raw(hipStream_t st, const DevTables& T, u32* x, const DecRaw& dr, int nch, const u32* s, const u32* s2) {
    if (nch < 1 || nch > 2) throw std::runtime_error("launch_dec_raw: 1 or 2 channels");
    double w = 0;
    for (int c = 0; c < nch; ++c) {
        if (dr.kd[c] < 1 || dr.kd[c] > 4 || dr.kd[c] > dr.nlc[c]) throw std::runtime_error("launch_dec_raw: bad limb count");
        w += (2.0 * dr.npoly[c] + 1.0) * dr.kd[c];
    }
    if (dr.members < 1 || 4 * nch * dr.members > 65535) throw std::runtime_error("launch_dec_raw: bad member count");
    prof_launch(KID_ELEMENTWISE, words(w * dr.members * (1u << T.logn)), k_dec_raw, dim3((1u << T.logn) / kBlock, 4 * nch * dr.members),
                dim3(kBlock), 0, st, x, dr, s, s2, T.pc, T.logn);
}
void launch_sample_uniform(hipStream_t st, const DevTables& T, u32* out, int nl, LimbMap map, const PrngKey& key, u64 stream) {
    prof_launch(KID_SAMPLE, words((double)nl * (1u << T.logn)), k_sample_uniform, ew_grid(T.logn, nl), dim3(kBlock), 0, st, out, nl, map, key, stream, T.pc, T.logn);
}
void launch_keygen_combine(hipStream_t st, const DevTables& T, u32* b, const u32* a, const u32* s, const u32* e, const u32* sp,
                           const u32* gadget, int nl, LimbMap map, int glo, int ghi) {
    prof_launch(KID_ELEMENTWISE, EW_BYTES(4.0 * nl), k_keygen_combine, ew_grid(T.logn, nl), dim3(kBlock), 0, st, b, a, s, e, sp, gadget, nl, map, glo, ghi, T.pc,
                       T.logn);
}

void launch_decode16(hipStream_t st, const DevTables& T, const u32* x, const int kd[2], const CrtConsts cc[2], const Slot16& sl,
                     const double inv_scale[2], double* acc) {
    prof_launch(KID_ELEMENTWISE, words((double)(kd[0] + kd[1]) * (1u << T.logn)), k_decode16, dim3((1u << T.logn) / kBlock, 2),
                dim3(kBlock), 0, st, x, kd[0], kd[1], cc[0], cc[1], sl, inv_scale[0], inv_scale[1], acc, T.logn);
}
void launch_decode32(hipStream_t st, const DevTables& T, const u32* x, int kd, const CrtConsts& cc, const Slot32& sl, double inv_scale, double* acc) {
    prof_launch(KID_ELEMENTWISE, words((double)kd * (1u << T.logn)), k_decode32, dim3((1u << T.logn) / kBlock), dim3(kBlock), 0, st, x, kd, cc, sl,
                inv_scale, acc, T.logn);
}
void launch_encode32(hipStream_t st, const DevTables& T, u32* out, const double* w, const Slot32& sl, double scale, int nq, double* zacc) {
    if (zacc)
        prof_launch(KID_ELEMENTWISE, words((double)nq * (1u << T.logn)), k_encode32<true>, dim3((1u << T.logn) / kBlock), dim3(kBlock), 0, st, out,
                    w, zacc, sl, scale, nq, T.pc, T.logn);
    else
        prof_launch(KID_ELEMENTWISE, words((double)nq * (1u << T.logn)), k_encode32<false>, dim3((1u << T.logn) / kBlock), dim3(kBlock), 0, st, out,
                    w, zacc, sl, scale, nq, T.pc, T.logn);
}
void launch_snap16(hipStream_t st, double* acc, double* w, int* nib) {
    prof_launch(KID_ELEMENTWISE, 0.0, k_snap16, dim3(1), dim3(64), 0, st, acc, w, nib);
}
void launch_encode16(hipStream_t st, const DevTables& T, u32* out, const double* w, const Slot16& sl, double scale, int nq, bool periodic,
                     double* zacc) {
    const u32 n = 1u << T.logn;
    const u32 kmask = periodic ? n / 32 - 1 : 0u;
    const double fac = periodic ? 1.0 / 16.0 : 2.0 / n;
    if (zacc)
        prof_launch(KID_ELEMENTWISE, words(2.0 * nq * (1u << T.logn)), k_encode16<true>, dim3((1u << T.logn) / kBlock, 2), dim3(kBlock), 0, st,
                    out, w, zacc, sl, scale, nq, T.pc, T.logn, kmask, fac);
    else
        prof_launch(KID_ELEMENTWISE, words(2.0 * nq * (1u << T.logn)), k_encode16<false>, dim3((1u << T.logn) / kBlock, 2), dim3(kBlock), 0, st,
                    out, w, zacc, sl, scale, nq, T.pc, T.logn, kmask, fac);
}

void launch_renorm_wtab32(hipStream_t st, const DevTables& T, u32* W, const double* w, double* zacc, const Slot32& sl, double scale, int nl,
                          const u32* gtab) {
    if (nl < 1 || nl > kRenormMaxLimbs) throw std::runtime_error("launch_renorm_wtab: limb count out of range");
    SlotTab<32> tab;
    for (int i = 0; i < 32; ++i) tab.e[i] = sl.e[i];
    if (zacc)
        prof_launch(KID_ELEMENTWISE, 4.0 * 64 * nl, k_renorm_wtab<32, true>, dim3(1), dim3(256), 0, st, W, w, zacc, tab, scale, nl, gtab, T.pc, T.logn);
    else
        prof_launch(KID_ELEMENTWISE, 4.0 * 64 * nl, k_renorm_wtab<32, false>, dim3(1), dim3(256), 0, st, W, w, zacc, tab, scale, nl, gtab, T.pc, T.logn);
}
void launch_renorm_wtab16(hipStream_t st, const DevTables& T, u32* W, const double* w, double* zacc, const Slot16& sl, double scale, int nl,
                          const u32* gtab) {
    if (nl < 1 || nl > kRenormMaxLimbs) throw std::runtime_error("launch_renorm_wtab: limb count out of range");
    SlotTab<16> tab;
    for (int i = 0; i < 16; ++i) tab.e[i] = sl.e[i];
    if (zacc)
        prof_launch(KID_ELEMENTWISE, 4.0 * 2 * 32 * nl, k_renorm_wtab<16, true>, dim3(2), dim3(256), 0, st, W, w, zacc, tab, scale, nl, gtab, T.pc, T.logn);
    else
        prof_launch(KID_ELEMENTWISE, 4.0 * 2 * 32 * nl, k_renorm_wtab<16, false>, dim3(2), dim3(256), 0, st, W, w, zacc, tab, scale, nl, gtab, T.pc, T.logn);
}
void launch_renorm_sparse(hipStream_t st, const DevTables& T, u32* W, u32* B, const DecRaw& dr, int nch, const SparseDec& sd, const Slot32& sl32,
                          const Slot16& sl16, double scale, int nl, const u32* gtab, const u32* s, const u32* s2) {
    if (nl < 1 || nl > kRenormMaxLimbs) throw std::runtime_error("launch_renorm_sparse: limb count out of range");
    const double n = (double)(1u << T.logn);
    double w = 0.0;
    for (int c = 0; c < nch; ++c) w += (double)dr.kd[c] * (dr.npoly[c] + 1);
    if (nch == 1) {  // one 32-slot channel (the packed period-32 renorm)
        SlotTab<32> tab;
        for (int i = 0; i < 32; ++i) tab.e[i] = sl32.e[i];
        prof_launch(KID_ELEMENTWISE, words(w * n), k_dec_blocksum<64>, dim3(64, 4, 1), dim3(256), 0, st, B, dr, s, s2, T.pc, T.logn);
        prof_launch(KID_ELEMENTWISE, 4.0 * 64 * (4 + nl), k_renorm_sparse<32>, dim3(1), dim3(256), 0, st, W, (const u32*)B, sd, tab, scale, nl, gtab,
                    T.pc, T.logn);
    } else {  // two 16-slot channels (the periodic pair renorm)
        SlotTab<16> tab;
        for (int i = 0; i < 16; ++i) tab.e[i] = sl16.e[i];
        prof_launch(KID_ELEMENTWISE, words(w * n), k_dec_blocksum<32>, dim3(32, 4, 2), dim3(256), 0, st, B, dr, s, s2, T.pc, T.logn);
        prof_launch(KID_ELEMENTWISE, 4.0 * 2 * 32 * (4 + nl), k_renorm_sparse<16>, dim3(2), dim3(256), 0, st, W, (const u32*)B, sd, tab, scale, nl,
                    gtab, T.pc, T.logn);
    }
}
void launch_renorm_combine(hipStream_t st, const DevTables& T, const RenormOut& ro, int nch, const u32* W, int nl, int ld) {
    if (nch < 1 || nch > 2) throw std::runtime_error("launch_renorm_combine: 1 or 2 channels");
    prof_launch(KID_ELEMENTWISE, words(4.0 * nch * nl * (1u << T.logn)), k_renorm_combine, dim3((1u << T.logn) / kBlock, 2 * nl, nch), dim3(kBlock), 0,
                st, ro, W, nl, ld, T.pc, T.logn);
}

void launch_decode_twist(hipStream_t st, const DevTables& T, const u32* x, const int kd[2], const CrtConsts cc[2],
                         const double inv_scale[2], double* z, int nch, int members) {
    const double n = (double)(1u << T.logn);
    prof_launch(KID_ELEMENTWISE, words((double)kd[0] * n * (nch > members ? 2 : 1) * members) + 16.0 * nch * n, k_decode_twist,
                dim3((1u << T.logn) / kBlock, nch), dim3(kBlock), 0, st, x, kd[0], kd[1], cc[0], cc[1], inv_scale[0], inv_scale[1], (double2*)z,
                T.logn, members);
}
void launch_fft2(hipStream_t st, const DevTables& T, double* z, int sign, int nch) {
    const int l1 = T.logn - T.logn / 2, l2 = T.logn - l1;
    for (int pass = 0; pass < 2; ++pass)
        prof_launch(KID_ELEMENTWISE, 32.0 * nch * (1u << T.logn), k_fft_pass, dim3((1u << (pass ? l1 : l2)) / kFftTpb, nch), dim3(kBlock), 0, st,
                    (double2*)z, T.logn, pass, sign);
}
void launch_snap_slots(hipStream_t st, const DevTables& T, const double* zin, double* w, const u32* slot_pos, int states, int unpack,
                       int nch, int members) {
    const double s = (double)(1u << (T.logn - 1));
    prof_launch(KID_ELEMENTWISE, nch * (16.0 * s + 4.0 * s + 32.0 * s), k_snap_slots, dim3((1u << (T.logn - 1)) / kBlock, nch),
                dim3(kBlock), 0, st, (const double2*)zin, (double2*)w, slot_pos, states, unpack, T.logn, members);
}
void launch_encode_untwist(hipStream_t st, const DevTables& T, u32* out, const double* v, double scale, int nq, int nch) {
    const double n = (double)(1u << T.logn);
    prof_launch(KID_ELEMENTWISE, 16.0 * nch * n + words((double)nch * nq * n), k_encode_untwist, dim3((1u << T.logn) / kBlock, nch), dim3(kBlock), 0,
                st, out, (const double2*)v, scale, nq, T.pc, T.logn);
}

void launch_lut_bivariate(hipStream_t st, const DevTables& T, u32* out, const LutOperands& op, int n_a, const u32* cst, int nl, int members) {
    double reads = 0;
    for (int p = 0; p < n_a; ++p)
        if (op.p_start[p + 1] > op.p_start[p]) reads += 2;
    // AESFHE_LUT_LDS=0: every term reads its B element from memory (k_lut_bivariate, A/B runs)
    static const bool lds = !(std::getenv("AESFHE_LUT_LDS") && std::atoi(std::getenv("AESFHE_LUT_LDS")) == 0);
    int n_b = 0;
    unsigned used = 0;
    for (int j = 0; j < op.p_start[n_a]; ++j) {
        if (op.q_of[j] < 0 || op.q_of[j] >= kLutMax || !op.b[op.q_of[j]]) throw std::runtime_error("launch_lut_bivariate: bad B operand");
        n_b = std::max(n_b, op.q_of[j] + 1);
        used |= 1u << op.q_of[j];
    }
    if (lds && n_b > 0) {
        reads += 2.0 * n_b;
        prof_launch(KID_ELEMENTWISE, words((reads + 3.0) * nl * members * (1u << T.logn)), k_lut_bivariate_lds,
                    dim3((1u << T.logn) / kBlock, nl, members), dim3(kBlock), (unsigned)(2 * n_b * kBlock * sizeof(u32)), st, out, op, n_a, n_b,
                    used, cst, nl, T.pc, T.logn);
        return;
    }
    reads += 2.0 * kLutMax;  // upper bound on the B elements read
    prof_launch(KID_ELEMENTWISE, words((reads + 3.0) * nl * members * (1u << T.logn)), k_lut_bivariate,
                dim3((1u << T.logn) / kBlock, nl, members), dim3(kBlock), 0, st, out, op, n_a, cst, nl, T.pc, T.logn);
}
void launch_lut_univariate(hipStream_t st, const DevTables& T, u32* out, const u32* acc, const LutChunk& ch, int n, const u32* cst,
                           int npoly, int nl, int members, const LimbConsts* cadd) {
    static const LimbConsts kNoC{};
    prof_launch(KID_ELEMENTWISE, words((double)(n + (acc ? 2 : 1)) * npoly * nl * members * (1u << T.logn)), k_lut_univariate,
                dim3((1u << T.logn) / kBlock, nl, members), dim3(kBlock), 0, st, out, acc, ch, n, cst, npoly, nl, T.pc, T.logn,
                cadd ? *cadd : kNoC, cadd ? 1 : 0);
}

