// ntt.hip -- negacyclic NTT / inverse NTT for CDNA4.
//
// N = R1 x 256 (R1 = 2^(logn-8), 32..256).  View a limb as R1 rows of 256 contiguous
// words.  Forward (Cooley-Tukey, natural -> bit-reversed, psi^{bitrev} twiddles):
//   pass 1 ("cols"): stages 0..log2(R1)-1, butterflies between rows; a 512-thread block
//                    owns CB = 512 * 16 / R1 columns of all R1 rows,
//   pass 2 ("rows"): stages log2(R1)..logn-1 inside each 256-word row; a block of NT
//                    threads owns NT / 16 rows (256 threads by default, p2_nt()).
// Each thread keeps 16 elements in VGPRs.  Phase A holds elements 16 apart (rows
// g + T k in pass 1, words j + 16 k in pass 2) and runs the first 4 stages in registers;
// one LDS exchange regroups them into 16 consecutive elements (rows 16 g + k, words
// 16 j + k) for the remaining stages.  So a pass is: one global read, 4 register stages,
// one LDS round trip, up to 4 register stages, one global write -- instead of one LDS
// round trip and barrier per stage.  The inverse (Gentleman-Sande) runs the same passes
// backwards (rows first, then cols with the N^{-1} scaling fused into the store).
//
// Global access: pass 1 reads/writes 32..256 consecutive columns per row (>= 128 B
// segments); pass 2's phase-B side moves 16 contiguous words per thread (4 x b128).
// LDS: pass 1 tile [R1][CB] -- every 32-lane half touches 32 consecutive columns, no
// conflicts; pass 2 tile [NT / 16][272] with the 16-word-group XOR swizzle swz(), conflict-free
// for both the (j + 16 k) and the (16 j + k) pattern (rows r, r+1 share a half-wave and
// sit 272 = 16 mod 32 banks apart).
//
// Rows of one launch are addressed through a RowMap (out-of-place, strided groups), so
// callers never copy limbs around just to transform them.
#include <algorithm>
#include <cstdlib>
#include <stdexcept>

#include "kernels.h"
#include "launch.h"

namespace {

constexpr int kThreads = 512;
constexpr int kPitchP2 = 272;

// Harvey's lazy butterflies (every prime < 2^30, so 4q < 2^32): the forward transform keeps
// residues in [0, 4q) and the inverse in [0, 2q) between stages; only the last stage of a
// transform reduces to [0, q).  Shoup's product without its correction, one min-based
// reduction of the sum operand, and the product's last two steps as ONE 32x32+64 multiply-add
// (v_mad_u64_u32, full rate on gfx950): the forward table holds -w mod 2^32, so
//   tn = mulhi(b, w') q - b w = -t (mod 2^32),  a' = x - tn,  b' = x + 2q + tn  (v_add3_u32)
// -- 7 VALU operations per forward butterfly (9 before), 8 per inverse one; the values are
// the same as the plain lazy butterfly's, bit for bit.
__device__ __forceinline__ u32 red2(u32 x, u32 q2) { return min(x, x - q2); }  // [0, 2 q2) -> [0, q2)
__device__ __forceinline__ u32 canon4(u32 x, u32 q) { return red2(red2(x, 2 * q), q); }  // [0, 4q) -> [0, q)
__device__ __forceinline__ void ct_bfly(u32& a, u32& b, u32 nw, u32 wp, u32 q2, u32 q) {
    const u32 tn = (u32)((u64)mulhi32(b, wp) * q + (u32)(b * nw));  // -(b w - floor(b w'/2^32) q), t in [0, 2q)
    const u32 x = red2(a, q2);                                        // [0, 2q)
    a = x - tn;                                                       // x + t in [0, 4q)
    b = x + q2 + tn;                                                  // x - t + 2q in (0, 4q)
}
__device__ __forceinline__ void gs_bfly(u32& a, u32& b, u32 w, u32 wp, u32 q2, u32 nq) {
    const u32 u = a, v = b;                                           // [0, 2q)
    a = red2(u + v, q2);                                              // [0, 2q)
    const u32 d = u - v + q2;                                         // (0, 4q)
    b = (u32)((u64)mulhi32(d, wp) * nq + (u32)(d * w));              // d w - floor(d w'/2^32) q in [0, 2q)
}
// the inverse butterfly with its twiddle as a product g r (two lazy Shoup products, each in
// [0, 2q) for any 32-bit input): k_ntt2_inv's factored stages
__device__ __forceinline__ void gs_bfly2(u32& a, u32& b, uint2 g, uint2 r, u32 q2, u32 nq) {
    const u32 u = a, v = b;
    a = red2(u + v, q2);
    const u32 d = u - v + q2;
    const u32 e = (u32)((u64)mulhi32(d, g.y) * nq + (u32)(d * g.x));
    b = (u32)((u64)mulhi32(e, r.y) * nq + (u32)(e * r.x));
}
__device__ __forceinline__ int swz(int w) { return w ^ ((w >> 4) & 15); }

// ---- the fused core at 8 residues per thread (k_ntt2_ki8, AESFHE_KI8; VERDICT r4 "do this" 3)
// k_ntt2_ki holds 16 residues per thread: 64 VGPRs of 64-bit accumulators, 242 in all, 2 waves /
// SIMD.  Here a 256-thread block owns 8 rows (32 threads per 256-word row, 8 residues each), so
// the accumulators take 32 VGPRs and the grid has twice the blocks.  The row pass runs its 8
// stages in three register phases joined by two LDS exchanges:
//   A  words t + 32 k      stages 0-2 (partners 4, 2, 1 apart in k)
//   B  words 32 a + 4 m + b (a = t >> 2, b = t & 3)   stages 3-5 (partners 4, 2, 1 apart in m)
//   C  words 8 t + m       stages 6-7 (partners 2, 1 apart in m)
// every stage's butterflies and twiddles (index 2^(LOGR1 + s) + R 2^s + (word >> (8 - s))) are
// k_ntt2_fwd's / k_ntt2_inv's, so every stored residue is the one the 16-residue kernel stores
// (the inverse's lazy residues may differ in representative, its column pass ends canonical: the
// ModDown's output is the same bit for bit; tests/test_gpu_fused_ki.py).
// LDS swizzles (ds_read_b32 / ds_write_b32 bank = dword mod 32, one 32-lane half = one row):
//   A <-> B: w ^ (((w >> 5) & 7) << 2)     B <-> C: w ^ ((((w >> 5) & 3) << 3) | ((w >> 5) & 7))
// both conflict-free for both access patterns of their exchange.
constexpr int kPitch8 = 256;
__device__ __forceinline__ int swzAB(int w) { return w ^ (((w >> 5) & 7) << 2); }
__device__ __forceinline__ int swzBC(int w) { return w ^ ((((w >> 5) & 3) << 3) | ((w >> 5) & 7)); }
__device__ __forceinline__ int ki8_wordB(int t, int m) { return ((t >> 2) << 5) | (m << 2) | (t & 3); }
template <int LOGR1>
__device__ __forceinline__ int ki8_tw(int s, int R, int w) { return (1 << (LOGR1 + s)) + (R << s) + (w >> (8 - s)); }
// forward: x[k] = word t + 32 k of row R (pass-1 output, [0, 4q)) -> x[m] = word 8 t + m, canonical
template <int LOGR1>
__device__ __forceinline__ void ki8_fwd_rows(u32 (&x)[8], u32* row, const uint2* w, int R, int t, u32 q, u32 q2) {
#pragma unroll
    for (int s = 0; s < 3; ++s) {
        const int h = 4 >> s;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (!(k & h)) {
                const uint2 tw = w[ki8_tw<LOGR1>(s, R, t + 32 * k)];
                ct_bfly(x[k], x[k + h], tw.x, tw.y, q2, q);
            }
    }
    __syncthreads();  // the previous user of the LDS row is done reading it
#pragma unroll
    for (int k = 0; k < 8; ++k) row[swzAB(t + 32 * k)] = x[k];
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 8; ++m) x[m] = row[swzAB(ki8_wordB(t, m))];
#pragma unroll
    for (int s = 3; s < 6; ++s) {
        const int h = 1 << (5 - s);
#pragma unroll
        for (int m = 0; m < 8; ++m)
            if (!(m & h)) {
                const uint2 tw = w[ki8_tw<LOGR1>(s, R, ki8_wordB(t, m))];
                ct_bfly(x[m], x[m + h], tw.x, tw.y, q2, q);
            }
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 8; ++m) row[swzBC(ki8_wordB(t, m))] = x[m];
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 8; ++m) x[m] = row[swzBC(8 * t + m)];
#pragma unroll
    for (int s = 6; s < 8; ++s) {
        const int h = 1 << (7 - s);
#pragma unroll
        for (int m = 0; m < 8; ++m)
            if (!(m & h)) {
                const uint2 tw = w[ki8_tw<LOGR1>(s, R, 8 * t + m)];
                ct_bfly(x[m], x[m + h], tw.x, tw.y, q2, q);
            }
    }
#pragma unroll
    for (int m = 0; m < 8; ++m) x[m] = canon4(x[m], q);
}
// inverse: x[m] = word 8 t + m of row R ([0, 2q)) -> x[k] = word t + 32 k, [0, 2q) (Gentleman-Sande,
// stages 7 .. 0).  FACT: stages 7-5 take their twiddle as (row factor rowf[s - 5]) x (shared factor
// gam[2^s + (word >> (8 - s))]), k_ntt2_inv's factored form
template <int LOGR1, bool FACT>
__device__ __forceinline__ void ki8_inv_rows(u32 (&x)[8], u32* row, const uint2* w, const uint2* rowf, const uint2* gam, int R, int t,
                                             u32 q, u32 q2) {
    const u32 nq = 0u - q;
#pragma unroll
    for (int s = 7; s >= 6; --s) {
        const int h = 1 << (7 - s);
        const uint2 rf = FACT ? rowf[s - 5] : make_uint2(0, 0);
#pragma unroll
        for (int m = 0; m < 8; ++m)
            if (!(m & h)) {
                const int wd = 8 * t + m;
                if (FACT) {
                    gs_bfly2(x[m], x[m + h], gam[(1 << s) + (wd >> (8 - s))], rf, q2, nq);
                } else {
                    const uint2 tw = w[ki8_tw<LOGR1>(s, R, wd)];
                    gs_bfly(x[m], x[m + h], tw.x, tw.y, q2, nq);
                }
            }
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 8; ++m) row[swzBC(8 * t + m)] = x[m];
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 8; ++m) x[m] = row[swzBC(ki8_wordB(t, m))];
#pragma unroll
    for (int s = 5; s >= 3; --s) {
        const int h = 1 << (5 - s);
#pragma unroll
        for (int m = 0; m < 8; ++m)
            if (!(m & h)) {
                const int wd = ki8_wordB(t, m);
                if (FACT && s == 5) {
                    gs_bfly2(x[m], x[m + h], gam[(1 << s) + (wd >> (8 - s))], rowf[0], q2, nq);
                } else {
                    const uint2 tw = w[ki8_tw<LOGR1>(s, R, wd)];
                    gs_bfly(x[m], x[m + h], tw.x, tw.y, q2, nq);
                }
            }
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 8; ++m) row[swzAB(ki8_wordB(t, m))] = x[m];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = row[swzAB(t + 32 * k)];
#pragma unroll
    for (int s = 2; s >= 0; --s) {
        const int h = 4 >> s;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (!(k & h)) {
                const uint2 tw = w[ki8_tw<LOGR1>(s, R, t + 32 * k)];
                gs_bfly(x[k], x[k + h], tw.x, tw.y, q2, nq);
            }
    }
}
__device__ __forceinline__ void ld8(u32 (&e)[8], const u32* p) {
    const uint4* v = reinterpret_cast<const uint4*>(p);
    const uint4 a = v[0], b = v[1];
    e[0] = a.x, e[1] = a.y, e[2] = a.z, e[3] = a.w, e[4] = b.x, e[5] = b.y, e[6] = b.z, e[7] = b.w;
}
__device__ __forceinline__ void st8(u32* p, const u32 (&e)[8]) {
    uint4* v = reinterpret_cast<uint4*>(p);
    st_out16(v, make_uint4(e[0], e[1], e[2], e[3]));
    st_out16(v + 1, make_uint4(e[4], e[5], e[6], e[7]));
}

enum { kPlain = 0, kSpread = 1, kFinish = 1, kSpread2 = 2 };

// rows below which a launch of 512-thread blocks (8 per row) leaves CUs idle: half-size
// blocks instead (AESFHE_NTT_SMALL_ROWS overrides, 0 = never)
inline int small_rows_limit() {
    static const int v = [] {
        const char* e = std::getenv("AESFHE_NTT_SMALL_ROWS");
        return e ? std::atoi(e) : 16;
    }();
    return v;
}
inline bool small_launch(int rows) { return rows < small_rows_limit(); }
// threads per block of the column pass (pass 1) at >= small_rows_limit() rows: AESFHE_NTT_P1_NT=256
// forces the half-size blocks (16-column tiles) at every size (A/B sweeps, tools/ntt_grid_sweep.py)
inline int p1_nt() {
    static const int v = [] {
        const char* e = std::getenv("AESFHE_NTT_P1_NT");
        return e ? std::atoi(e) : 512;
    }();
    return v;
}
// threads per block of the row pass (pass 2) for launches of >= small_rows_limit() rows, forward
// (AESFHE_NTT_P2_NT) and inverse (AESFHE_NTT_P2I_NT): 512, 256 or 128 (NT / 16 rows per block).
// Smaller blocks spread a launch of a few hundred blocks more evenly over the 256 CUs (a block is
// ~2.3 us of VALU work; at 512 threads a 40-row launch leaves 64 CUs with two blocks and 192
// with one), while pass 1 keeps its 512-thread blocks' 128-byte column segments
// AESFHE_NTT_AUTO=1: block sizes by launch size from the row sweep (profiles/r4_ntt_grid_sweep.json):
// 128-thread row-pass blocks below 41 rows, 256-thread inverse column-pass blocks at 50..80 rows
inline bool ntt_auto() {
    static const bool v = std::getenv("AESFHE_NTT_AUTO") && std::atoi(std::getenv("AESFHE_NTT_AUTO")) != 0;
    return v;
}
inline int p2_nt_rows(bool inverse, int rows);
inline int p1_nt_rows(bool inverse, int rows);
inline int p2_nt(bool inverse) {
    static const int f = [] {
        const char* e = std::getenv("AESFHE_NTT_P2_NT");
        return e ? std::atoi(e) : 256;
    }();
    static const int i = [] {
        const char* e = std::getenv("AESFHE_NTT_P2I_NT");
        return e ? std::atoi(e) : 256;
    }();
    return inverse ? i : f;
}
inline int p2_nt_rows(bool inverse, int rows) {
    if (ntt_auto() && rows >= 12 && rows < 41) return 128;
    return p2_nt(inverse);
}
inline int p1_nt_rows(bool inverse, int rows) {
    if (ntt_auto() && inverse && rows >= 50 && rows <= 80) return 256;
    return p1_nt();
}
// AESFHE_NTT_FIN_OCC=1: the finish mode capped at 128 VGPRs (A/B runs; off: with 256-thread row
// blocks the cap's spills cost more than the extra wave per SIMD gains, profiles/r3_ntt_p2_ab.json)
inline bool fin_occ_on() {
    static const bool v = [] {
        const char* e = std::getenv("AESFHE_NTT_FIN_OCC");
        return e && std::atoi(e) != 0;
    }();
    return v;
}
template <int LOGR1>
constexpr int R1_of() { return 1 << LOGR1; }

// key-switching ModUp: digit g's own limbs [g alpha, min(nl, (g + 1) alpha)) are not
// transformed (they are already in NTT form in the input); block-uniform early exit
__device__ __forceinline__ bool skipped(const RowMap& rm) {
    const int g0 = blockIdx.z, i = blockIdx.y;
    if (g0 * rm.cnt + i >= rm.nrows) return true;  // past the last row of a partial group
    if (rm.skip_alpha <= 0) return false;
    const int g = rm.skip_groups > 0 ? g0 % rm.skip_groups : g0;
    return i < rm.skip_nl && i / rm.skip_alpha == g;
}

struct RowAddr {
    const u32* src;
    u32* dst;
    int prime;
};
template <int LOGN>
__device__ __forceinline__ RowAddr row_addr(u32* dst, const u32* src, const RowMap& rm, const LimbMap& map) {
    const int g = blockIdx.z, i = blockIdx.y;
    RowAddr a;
    a.src = src + ((size_t)(rm.src_off + g * rm.src_stride + i) << LOGN);
    a.dst = dst + ((size_t)(rm.dst_off + g * rm.dst_stride + i) << LOGN);
    a.prime = map.prime(i);
    return a;
}

// pass 1's butterflies on the 16 elements a thread loaded (rows g + T k of its column), the LDS
// regroup and the store of rows 16 g + k (dst = the limb's first word of the column)
template <int LOGR1, int NT>
__device__ __forceinline__ void ntt1_fwd_stages(u32 (&x)[16], u32* sm, const uint2* w, u32 q, u32 q2, int g, int col, u32* dst) {
    constexpr int R1 = 1 << LOGR1, T = R1 / 16, CB = NT / T;
    // stages 0..3: row distance R1 / 2^(s+1) = T * (8 >> s); block index k >> (4 - s)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int h = 8 >> s;
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (!(k & h)) {
                const int ti = (1 << s) + (k >> (4 - s));
                ct_bfly(x[k], x[k + h], w[ti].x, w[ti].y, q2, q);
            }
    }
    // the twiddles of stages 4..LOGR1-1 (2^(s+4-LOGR1) per stage and thread) loaded BEFORE the
    // barrier: their latency overlaps the exchange instead of following it
    constexpr int C4 = 1 << (8 - LOGR1), NB = 16 - C4;
    uint2 tb[NB > 0 ? NB : 1];
#pragma unroll
    for (int s = 4; s < LOGR1; ++s) {
        const int c = 1 << (s + 4 - LOGR1), base = (1 << s) + (g << (s + 4 - LOGR1));
#pragma unroll
        for (int u = 0; u < c; ++u) tb[c - C4 + u] = w[base + u];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) sm[(g + T * k) * CB + col] = x[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = sm[(16 * g + k) * CB + col];
    // stages 4..LOGR1-1 on rows 16 g + k: twiddle (1 << s) + ((16 g + k) >> (LOGR1 - s))
#pragma unroll
    for (int s = 4; s < LOGR1; ++s) {
        const int h = 1 << (LOGR1 - 1 - s), c = 1 << (s + 4 - LOGR1);
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (!(k & h)) {
                const uint2 t = tb[c - C4 + (k >> (LOGR1 - s))];
                ct_bfly(x[k], x[k + h], t.x, t.y, q2, q);
            }
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) dst[(size_t)(16 * g + k) * 256] = x[k];
}

// ---------------------------------------------------------------- forward, pass 1
// MODE kPlain: x = src row.  MODE kSpread (rescale): the source is one coefficient-form
// row per group modulo aux.q_last (src row = src_off + g * src_stride, independent of the
// limb) and x = its centred representative reduced mod the target prime.
template <int LOGR1, int MODE, int NT>
__global__ void __launch_bounds__(NT) k_ntt1_fwd(u32* dst, const u32* src, RowMap rm, LimbMap map, const PrimeConst* pc,
                                                       const uint2* tw, NttAux aux, unsigned long long* ts) {
    constexpr int LOGN = LOGR1 + 8, R1 = 1 << LOGR1, T = R1 / 16, CB = NT / T;
    __shared__ u32 sm[R1 * CB];
    if (skipped(rm)) return;
    ts_begin(ts);
    RowAddr ra = row_addr<LOGN>(dst, src, rm, map);
    const u32 q = pc[ra.prime].q, q2 = 2 * q;
    const uint2* w = tw + ((size_t)ra.prime << LOGN);  // {psi^brv, Shoup companion} pairs
    const int col = threadIdx.x % CB, g = threadIdx.x / CB;
    const int c = blockIdx.x * CB + col;
    u32 x[16];
    if (MODE == kSpread) {
        const int grp = blockIdx.z;
        ra.src = src + ((size_t)(rm.src_off + grp * rm.src_stride) << LOGN);
        const u32 ql = aux.q_last, half = ql >> 1;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const u32 v = ra.src[(size_t)(g + T * k) * 256 + c];
            // every prime lies in (2^29, 2^30), so q_last < 2q: the reductions are single conditional subtracts
            x[k] = v > half ? q - (ql - v) : csub(v, q);
        }
    } else if (MODE == kSpread2) {
        // two dropped limbs a, b (rows src_off + grp * src_stride + {0, 1}): mixed-radix CRT
        // v = x_a + qa ((x_b - x_a) qa^{-1} mod qb) in [0, qa qb), centred, reduced mod q
        const int grp = blockIdx.z;
        const u32* sa = src + ((size_t)(rm.src_off + grp * rm.src_stride) << LOGN);
        const u32* sb = sa + ((size_t)1 << LOGN);
        const u32 qa = aux.q_last, qb = aux.q_last2;
        const u64 Q2 = (u64)qa * qb, half = Q2 >> 1;
        const u32 mu = pc[ra.prime].mu;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const size_t at = (size_t)(g + T * k) * 256 + c;
            const u32 xa = sa[at], xb = sb[at];
            const u32 d = shoup_mul(xb + qb - csub(xa, qb), aux.qa_inv, aux.qa_inv_p, qb);
            const u64 v = (u64)xa + (u64)qa * d;
            if (v > half) {
                const u32 r = barrett_reduce64(Q2 - v, q, mu);
                x[k] = r ? q - r : 0u;
            } else {
                x[k] = barrett_reduce64(v, q, mu);
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) x[k] = ra.src[(size_t)(g + T * k) * 256 + c];
    }
    ntt1_fwd_stages<LOGR1, NT>(x, sm, w, q, q2, g, col, ra.dst + c);
    ts_end(ts);
}

// ---------------------------------------------------------------- forward, pass 1 fused with the base conversion
// The ModUp / ModDown conversion (kernels.hip k_base_convert, same arithmetic in the same order,
// so bit for bit its values) computed in pass 1's load instead of a separate launch: row t of
// group z (blockIdx.y / .z, the RowMap's) is target t of ConvBatch group z; every element reads
// the group's H source residues at its position (y_i, the INTT having already multiplied by
// qhat_i^{-1}: launch_ntt_inv's `post`), u = round(sum y_i / q_i), and
// x = (u (-Q mod q_t) + sum y_i (Q / q_i mod q_t)) mod q_t.  Saves the converted rows' write
// and re-read and one launch per ModUp / ModDown.
template <int LOGR1, int NT, int H>
__global__ void __launch_bounds__(NT) k_ntt1_fwd_conv(u32* dst, RowMap rm, LimbMap map, const PrimeConst* pc, const uint2* tw, ConvBatch cb,
                                                            unsigned long long* ts) {
    constexpr int LOGN = LOGR1 + 8, R1 = 1 << LOGR1, T = R1 / 16, CB = NT / T;
    __shared__ u32 sm[R1 * CB];
    if (skipped(rm)) return;
    ts_begin(ts);
    const int z = blockIdx.z, t = blockIdx.y, nt = rm.cnt;
    const RowAddr ra = row_addr<LOGN>(dst, dst, rm, map);
    const PrimeConst P = pc[ra.prime];
    const u32 q = P.q, q2 = 2 * q;
    const uint2* w = tw + ((size_t)ra.prime << LOGN);
    const int col = threadIdx.x % CB, g = threadIdx.x / CB;
    const int c = blockIdx.x * CB + col;
    const u32* tab = cb.tab[z];
    const int sp = cb.split[z], hz = cb.h[z];
    // H = the launch's largest source count; a group with fewer sources (ModUp's last digit)
    // runs with zero weights on the missing ones (and re-reads its last row: no branch)
    u32 wt[H], ms[H];
#pragma unroll
    for (int i = 0; i < H; ++i) {
        wt[i] = i < hz ? tab[2 * ((size_t)i * nt + t)] : 0u;
        ms[i] = i < hz ? pc[(sp > 0 && i >= sp) ? cb.d1[z] + (i - sp) : cb.d0[z] + i].mu : 0u;
    }
    const u32 negq = cb.negq[z][t];
    const u32* src = cb.src[z];
    u32 x[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const size_t at = (size_t)(g + T * k) * 256 + c;
        u32 y[H];
#pragma unroll
        for (int i = 0; i < H; ++i) y[i] = src[((size_t)min(i, hz - 1) << LOGN) + at];
        u64 f = 0;
#pragma unroll
        for (int i = 0; i < H; ++i) f += ((u64)y[i] * ms[i]) >> 29;  // y_i / q_i in 32.32 fixed point
        const u32 u = (u32)((f + (1ull << 31)) >> 32);
        u64 acc = (u64)u * negq;
#pragma unroll
        for (int i = 0; i < H; ++i) {
            if (i == 8) acc = fold64(acc, q, P.r32);
            acc += (u64)y[i] * wt[i];
        }
        x[k] = reduce64(acc, q, P.mu, P.r32);
    }
    ntt1_fwd_stages<LOGR1, NT>(x, sm, w, q, q2, g, col, ra.dst + c);
    ts_end(ts);
}

// ---------------------------------------------------------------- forward, pass 2 (in place on dst rows)
// MODE kPlain: result stored in place.  MODE kFinish (rescale / ModDown): with
// g = group, i = limb, out[g][i] = (cur[g][i] - x) * qinv_i (+ add_g[i]), rows addressed
// through aux (cur row g * cur_stride + i, out row g * out_stride + i).
// OCC: minimum waves per SIMD the register allocation must allow.  The finish mode's prefetched
// cur / add operands take it to 130 VGPRs unconstrained (3 waves per SIMD); OCC = 4 caps it at
// 128 with 6 dwords spilled (AESFHE_NTT_FIN_OCC, off by default)
template <int LOGR1, int MODE, int NT, int OCC = 1>
__global__ void __launch_bounds__(NT, OCC) k_ntt2_fwd(u32* data, RowMap rm, LimbMap map, const PrimeConst* pc, const uint2* tw,
                                                       NttAux aux, unsigned long long* ts) {
    constexpr int LOGN = LOGR1 + 8;
    __shared__ u32 sm[(NT / 16) * kPitchP2];
    if (skipped(rm)) return;
    ts_begin(ts);
    const RowAddr ra = row_addr<LOGN>(data, data, rm, map);
    const u32 q = pc[ra.prime].q, q2 = 2 * q;
    const uint2* w = tw + ((size_t)ra.prime << LOGN);  // {psi^brv, Shoup companion} pairs
    const int r = threadIdx.x >> 4, j = threadIdx.x & 15;
    const int R = blockIdx.x * (NT / 16) + r;
    u32* p = ra.dst + (size_t)R * 256;
    u32 x[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = p[j + 16 * k];
    // stage LOGR1 + s: twiddle index 2^(LOGR1+s) + R 2^s + (word >> (8 - s))
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int h = 8 >> s;
        const int base = (1 << (LOGR1 + s)) + (R << s);
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (!(k & h)) {
                const int ti = base + (k >> (4 - s));
                ct_bfly(x[k], x[k + h], w[ti].x, w[ti].y, q2, q);
            }
    }
    // phase B's twiddles (stage s: 2^(s-4) per thread, word 16 j + k -> offset k >> (8 - s)) and,
    // in the finish mode, the cur / add rows loaded BEFORE the barrier (latency overlapped)
    uint2 tb[15];
#pragma unroll
    for (int s = 4; s < 8; ++s) {
        const int c = 1 << (s - 4), base = (1 << (LOGR1 + s)) + (R << s) + (j << (s - 4));
#pragma unroll
        for (int u = 0; u < c; ++u) tb[c - 1 + u] = w[base + u];
    }
    uint4 cvp[MODE == kFinish ? 4 : 1], avp[MODE == kFinish ? 4 : 1];
    bool has_add = false;
    if (MODE == kFinish) {
        const int grp = blockIdx.z, li = blockIdx.y;
        const size_t woff = (size_t)R * 256 + 16 * j;
        const uint4* cu = reinterpret_cast<const uint4*>(aux.cur + ((size_t)(grp * aux.cur_stride + li) << LOGN) + woff);
        const u32* addp = (grp & 1) ? aux.add1 : aux.add0;
        if (grp > 1) addp = (addp && aux.add_mstride) ? addp + (grp >> 1) * aux.add_mstride : nullptr;
        has_add = addp != nullptr;
#pragma unroll
        for (int v = 0; v < 4; ++v) cvp[v] = cu[v];
        if (has_add && aux.add_rev && !(grp & 1)) {  // element e <- word N - 1 - (woff + e)
            const uint4* ad = reinterpret_cast<const uint4*>(addp + ((size_t)li << LOGN) + ((size_t)1 << LOGN) - 16 - woff);
            uint4 t[4];
#pragma unroll
            for (int v = 0; v < 4; ++v) t[v] = ad[v];
#pragma unroll
            for (int v = 0; v < 4; ++v) avp[v] = make_uint4(t[3 - v].w, t[3 - v].z, t[3 - v].y, t[3 - v].x);
        } else if (has_add) {
            const uint4* ad = reinterpret_cast<const uint4*>(addp + ((size_t)li << LOGN) + woff);
#pragma unroll
            for (int v = 0; v < 4; ++v) avp[v] = ad[v];
        }
    }
    u32* row = sm + r * kPitchP2;
#pragma unroll
    for (int k = 0; k < 16; ++k) row[swz(j + 16 * k)] = x[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = row[swz(16 * j + k)];
#pragma unroll
    for (int s = 4; s < 8; ++s) {
        const int h = 1 << (7 - s), c = 1 << (s - 4);
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (!(k & h)) {
                const uint2 t = tb[c - 1 + (k >> (8 - s))];  // twiddle base + ((16 j + k) >> (8 - s))
                ct_bfly(x[k], x[k + h], t.x, t.y, q2, q);
            }
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = canon4(x[k], q);  // last stage: [0, 4q) -> [0, q)
    if (MODE == kFinish) {
        const int grp = blockIdx.z, li = blockIdx.y;
        const size_t woff = (size_t)R * 256 + 16 * j;
        u32* const om = aux.outm[(grp >> 1) & 7];
        uint4* o = reinterpret_cast<uint4*>((om ? om + ((size_t)((grp & 1) * aux.out_stride + li) << LOGN)
                                               : aux.out + ((size_t)(grp * aux.out_stride + li) << LOGN)) + woff);
        const u32 qi = aux.qinv[2 * li], qip = aux.qinv[2 * li + 1];
        if (aux.cmul) {  // block-uniform: a level conversion's constant on cur (canonical in, canonical out)
            const u32 cm = aux.cmul[2 * li], cmp = aux.cmul[2 * li + 1];
#pragma unroll
            for (int v = 0; v < 4; ++v)
                cvp[v] = make_uint4(shoup_mul(cvp[v].x, cm, cmp, q), shoup_mul(cvp[v].y, cm, cmp, q), shoup_mul(cvp[v].z, cm, cmp, q),
                                    shoup_mul(cvp[v].w, cm, cmp, q));
        }
        // the epilogue 2 r + c (aux.dbl / aux.cst, block-uniform): c on polynomial 0 only, its
        // half (lo / hi slots) by the row -- words R 256 .. of the limb lie in half R >= R1 / 2
        const int mem = (grp >> 1) & 7;
        const bool dbl = (aux.dbl >> mem) & 1u;
        const u32* cs = (grp & 1) ? nullptr : aux.cst[mem];
        const u32 cadd = cs ? cs[2 * li + (R >= (1 << LOGR1) / 2 ? 1 : 0)] : 0u;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const uint4 cv = cvp[v];
            uint4 r;
            r.x = shoup_mul(cv.x + q - x[4 * v], qi, qip, q);
            r.y = shoup_mul(cv.y + q - x[4 * v + 1], qi, qip, q);
            r.z = shoup_mul(cv.z + q - x[4 * v + 2], qi, qip, q);
            r.w = shoup_mul(cv.w + q - x[4 * v + 3], qi, qip, q);
            if (has_add) {
                const uint4 a = avp[v];
                r.x = add_mod(r.x, a.x, q), r.y = add_mod(r.y, a.y, q), r.z = add_mod(r.z, a.z, q), r.w = add_mod(r.w, a.w, q);
            }
            if (dbl) r.x = add_mod(r.x, r.x, q), r.y = add_mod(r.y, r.y, q), r.z = add_mod(r.z, r.z, q), r.w = add_mod(r.w, r.w, q);
            if (cs) r.x = add_mod(r.x, cadd, q), r.y = add_mod(r.y, cadd, q), r.z = add_mod(r.z, cadd, q), r.w = add_mod(r.w, cadd, q);
            st_out16(o + v, r);
        }
    } else {
        uint4* o = reinterpret_cast<uint4*>(p + 16 * j);
#pragma unroll
        for (int v = 0; v < 4; ++v) st_out16(o + v, make_uint4(x[4 * v], x[4 * v + 1], x[4 * v + 2], x[4 * v + 3]));
    }
    ts_end(ts);
}

// the forward row pass at 8 residues per thread (AESFHE_NTT_FWD8, default on): k_ntt2_fwd's modes (plain, and
// the finish with its cur / add / cmul / 2 r + c epilogue) on 256-thread blocks of 8 rows through
// ki8_fwd_rows -- the same butterflies, twiddles and canonical outputs, so the same residues
template <int LOGR1, int MODE>
__global__ void __launch_bounds__(256) k_ntt2_fwd8(u32* data, RowMap rm, LimbMap map, const PrimeConst* pc, const uint2* tw, NttAux aux,
                                                   unsigned long long* ts) {
    constexpr int LOGN = LOGR1 + 8;
    __shared__ u32 sm[8 * kPitch8];
    if (skipped(rm)) return;
    ts_begin(ts);
    const RowAddr ra = row_addr<LOGN>(data, data, rm, map);
    const u32 q = pc[ra.prime].q, q2 = 2 * q;
    const int r = threadIdx.x >> 5, t = threadIdx.x & 31;
    const int R = blockIdx.x * 8 + r;
    u32* p = ra.dst + (size_t)R * 256;
    u32 x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = p[t + 32 * k];
    ki8_fwd_rows<LOGR1>(x, sm + r * kPitch8, tw + ((size_t)ra.prime << LOGN), R, t, q, q2);
    if (MODE == kFinish) {
        const int grp = blockIdx.z, li = blockIdx.y;
        const size_t woff = (size_t)R * 256 + 8 * t;
        u32 cv[8], av[8];
        ld8(cv, aux.cur + ((size_t)(grp * aux.cur_stride + li) << LOGN) + woff);
        const u32* addp = (grp & 1) ? aux.add1 : aux.add0;
        if (grp > 1) addp = (addp && aux.add_mstride) ? addp + (grp >> 1) * aux.add_mstride : nullptr;
        const bool has_add = addp != nullptr;
        if (has_add && aux.add_rev && !(grp & 1)) {  // element e <- word N - 1 - (woff + e)
            u32 tmp[8];
            ld8(tmp, addp + ((size_t)li << LOGN) + ((size_t)1 << LOGN) - 8 - woff);
#pragma unroll
            for (int e = 0; e < 8; ++e) av[e] = tmp[7 - e];
        } else if (has_add) {
            ld8(av, addp + ((size_t)li << LOGN) + woff);
        }
        u32* const om = aux.outm[(grp >> 1) & 7];
        u32* o = (om ? om + ((size_t)((grp & 1) * aux.out_stride + li) << LOGN) : aux.out + ((size_t)(grp * aux.out_stride + li) << LOGN)) + woff;
        const u32 qi = aux.qinv[2 * li], qip = aux.qinv[2 * li + 1];
        if (aux.cmul) {
            const u32 cm = aux.cmul[2 * li], cmp = aux.cmul[2 * li + 1];
#pragma unroll
            for (int e = 0; e < 8; ++e) cv[e] = shoup_mul(cv[e], cm, cmp, q);
        }
        const int mem = (grp >> 1) & 7;
        const bool dbl = (aux.dbl >> mem) & 1u;
        const u32* cs = (grp & 1) ? nullptr : aux.cst[mem];
        const u32 cadd = cs ? cs[2 * li + (R >= (1 << LOGR1) / 2 ? 1 : 0)] : 0u;
        u32 res[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            u32 v = shoup_mul(cv[e] + q - x[e], qi, qip, q);
            if (has_add) v = add_mod(v, av[e], q);
            if (dbl) v = add_mod(v, v, q);
            if (cs) v = add_mod(v, cadd, q);
            res[e] = v;
        }
        st8(o, res);
    } else {
        st8(p + 8 * t, x);
    }
    ts_end(ts);
}
// default on since round 6 (strict C2 +0.6 %, three passes each, profiles/r6_fwd8_ab.txt); AESFHE_NTT_FWD8=0: k_ntt2_fwd
inline bool fwd8_on() {
    static const bool v = !(std::getenv("AESFHE_NTT_FWD8") && std::atoi(std::getenv("AESFHE_NTT_FWD8")) == 0);
    return v;
}

// ---------------------------------------------------------------- inverse, pass 2 (src -> dst)
// FACT: stages 7, 6, 5 (255 - 31 of a row's 255 twiddles, each thread its own) read their
// twiddle as (row factor) x (shared factor): psi^-(2^(7-s) (2 brv(R) + 1)) -- three per row --
// times psi^-((N / 2^s) brv_s(t)) -- 224 per prime, shared by every row, L1 / L2 resident --
// one more lazy Shoup product per butterfly of those stages instead of 8 twiddle bytes, so the
// launch reads ~280 twiddle bytes per 1 KB row instead of 2 KB
// IN = 1: the input row is the product a (.) b of group g's rows (launch_ntt_inv_prod), src unused;
// IN = 2: the source row read in reversed coefficient order (launch_ntt_inv_rev)
template <int LOGR1, int NT, bool FACT, int IN>
__global__ void __launch_bounds__(NT) k_ntt2_inv(u32* dst, const u32* src, RowMap rm, LimbMap map, const PrimeConst* pc,
                                                       const uint2* tw, const uint2* irow, const uint2* igam, TensorPtrs tp,
                                                       unsigned long long* ts) {
    constexpr int LOGN = LOGR1 + 8;
    __shared__ u32 sm[(NT / 16) * kPitchP2];
    if (skipped(rm)) return;
    ts_begin(ts);
    const RowAddr ra = row_addr<LOGN>(dst, src, rm, map);
    const u32 q = pc[ra.prime].q, q2 = 2 * q;
    const uint2* w = tw + ((size_t)ra.prime << LOGN);  // {psi^-brv, Shoup companion} pairs
    const int r = threadIdx.x >> 4, j = threadIdx.x & 15;
    const int R = blockIdx.x * (NT / 16) + r;
    u32 x[16];
    if (IN == 2) {  // element e of row R <- word N - 1 - (256 R + 16 j + e) = row R1 - 1 - R, word 255 - 16 j - e
        const uint4* in = reinterpret_cast<const uint4*>(ra.src + (size_t)((1 << LOGR1) - 1 - R) * 256 + 240 - 16 * j);
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const uint4 t = in[v];
            x[15 - 4 * v] = t.x, x[14 - 4 * v] = t.y, x[13 - 4 * v] = t.z, x[12 - 4 * v] = t.w;
        }
    } else if (IN == 1) {
        const u32 mu = pc[ra.prime].mu;
        const size_t off = ((size_t)blockIdx.y << LOGN) + (size_t)R * 256 + 16 * j;
        const uint4* pa = reinterpret_cast<const uint4*>(tp.a[blockIdx.z] + off);
        const uint4* pb = reinterpret_cast<const uint4*>(tp.b[blockIdx.z] + off);
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const uint4 a = pa[v], b = pb[v];
            x[4 * v] = barrett_mul(a.x, b.x, q, mu), x[4 * v + 1] = barrett_mul(a.y, b.y, q, mu);
            x[4 * v + 2] = barrett_mul(a.z, b.z, q, mu), x[4 * v + 3] = barrett_mul(a.w, b.w, q, mu);
        }
    } else {
        const uint4* in = reinterpret_cast<const uint4*>(ra.src + (size_t)R * 256 + 16 * j);
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const uint4 t = in[v];
            x[4 * v] = t.x, x[4 * v + 1] = t.y, x[4 * v + 2] = t.z, x[4 * v + 3] = t.w;
        }
    }
    const uint2* rowf = irow + ((size_t)ra.prime << LOGR1) * 4 + (size_t)R * 4;
    const uint2* gam = igam + ((size_t)ra.prime << 8);
#pragma unroll
    for (int s = 7; s >= 4; --s) {
        const int h = 1 << (7 - s);
        const int base = (1 << (LOGR1 + s)) + (R << s);
        if (FACT && s >= 5) {
            const uint2 rf = rowf[s - 5];
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (!(k & h)) gs_bfly2(x[k], x[k + h], gam[(1 << s) + ((16 * j + k) >> (8 - s))], rf, q2, 0u - q);
            continue;
        }
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (!(k & h)) {
                const int ti = base + ((16 * j + k) >> (8 - s));
                gs_bfly(x[k], x[k + h], w[ti].x, w[ti].y, q2, 0u - q);
            }
    }
    // stages 3..0's twiddles (2^s per thread) loaded before the barrier
    uint2 tb[15];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int base = (1 << (LOGR1 + s)) + (R << s);
#pragma unroll
        for (int u = 0; u < (1 << s); ++u) tb[(1 << s) - 1 + u] = w[base + u];
    }
    u32* row = sm + r * kPitchP2;
#pragma unroll
    for (int k = 0; k < 16; ++k) row[swz(16 * j + k)] = x[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = row[swz(j + 16 * k)];
#pragma unroll
    for (int s = 3; s >= 0; --s) {
        const int h = 8 >> s;
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (!(k & h)) {
                const uint2 t = tb[(1 << s) - 1 + (k >> (4 - s))];  // twiddle base + (k >> (4 - s))
                gs_bfly(x[k], x[k + h], t.x, t.y, q2, 0u - q);
            }
    }
    u32* p = ra.dst + (size_t)R * 256;
#pragma unroll
    for (int k = 0; k < 16; ++k) p[j + 16 * k] = x[k];
    ts_end(ts);
}

// the inverse row pass at 8 residues per thread (AESFHE_NTT_INV8, default on): 256-thread blocks of
// 8 rows (twice k_ntt2_inv's blocks per launch, ~half the serial work per thread) through
// ki8_inv_rows -- the same butterflies and twiddles, so the column pass that follows ends on the
// same canonical residues (bit-identical transforms); IN as k_ntt2_inv (0 plain, 1 product on load,
// 2 reversed read)
template <int LOGR1, bool FACT, int IN>
__global__ void __launch_bounds__(256) k_ntt2_inv8(u32* dst, const u32* src, RowMap rm, LimbMap map, const PrimeConst* pc,
                                                   const uint2* tw, const uint2* irow, const uint2* igam, TensorPtrs tp,
                                                   unsigned long long* ts) {
    constexpr int LOGN = LOGR1 + 8;
    __shared__ u32 sm[8 * kPitch8];
    if (skipped(rm)) return;
    ts_begin(ts);
    const RowAddr ra = row_addr<LOGN>(dst, src, rm, map);
    const u32 q = pc[ra.prime].q, q2 = 2 * q;
    const int r = threadIdx.x >> 5, t = threadIdx.x & 31;
    const int R = blockIdx.x * 8 + r;
    u32 x[8];
    if (IN == 2) {  // element e of row R <- word N - 1 - (256 R + 8 t + e) = row R1 - 1 - R, word 255 - 8 t - e
        const uint4* in = reinterpret_cast<const uint4*>(ra.src + (size_t)((1 << LOGR1) - 1 - R) * 256 + 248 - 8 * t);
#pragma unroll
        for (int v = 0; v < 2; ++v) {
            const uint4 a = in[v];
            x[7 - 4 * v] = a.x, x[6 - 4 * v] = a.y, x[5 - 4 * v] = a.z, x[4 - 4 * v] = a.w;
        }
    } else if (IN == 1) {
        const u32 mu = pc[ra.prime].mu;
        const size_t off = ((size_t)blockIdx.y << LOGN) + (size_t)R * 256 + 8 * t;
        const uint4* pa = reinterpret_cast<const uint4*>(tp.a[blockIdx.z] + off);
        const uint4* pb = reinterpret_cast<const uint4*>(tp.b[blockIdx.z] + off);
#pragma unroll
        for (int v = 0; v < 2; ++v) {
            const uint4 a = pa[v], b = pb[v];
            x[4 * v] = barrett_mul(a.x, b.x, q, mu), x[4 * v + 1] = barrett_mul(a.y, b.y, q, mu);
            x[4 * v + 2] = barrett_mul(a.z, b.z, q, mu), x[4 * v + 3] = barrett_mul(a.w, b.w, q, mu);
        }
    } else {
        ld8(x, ra.src + (size_t)R * 256 + 8 * t);
    }
    const uint2* w = tw + ((size_t)ra.prime << LOGN);
    const uint2* rowf = irow + ((size_t)ra.prime << LOGR1) * 4 + (size_t)R * 4;
    const uint2* gam = igam + ((size_t)ra.prime << 8);
    ki8_inv_rows<LOGR1, FACT>(x, sm + r * kPitch8, w, rowf, gam, R, t, q, q2);
    u32* p = ra.dst + (size_t)R * 256;
#pragma unroll
    for (int k = 0; k < 8; ++k) p[t + 32 * k] = x[k];
    ts_end(ts);
}
inline bool inv8_on() {
    static const bool v = !(std::getenv("AESFHE_NTT_INV8") && std::atoi(std::getenv("AESFHE_NTT_INV8")) == 0);
    return v;
}

// ---------------------------------------------------------------- inverse, pass 1 (in place on dst rows)
template <int LOGR1, int NT>
__global__ void __launch_bounds__(NT) k_ntt1_inv(u32* data, RowMap rm, LimbMap map, const PrimeConst* pc, const uint2* tw,
                                                       const u32* post, unsigned long long* ts) {
    constexpr int LOGN = LOGR1 + 8, R1 = 1 << LOGR1, T = R1 / 16, CB = NT / T;
    __shared__ u32 sm[R1 * CB];
    if (skipped(rm)) return;
    ts_begin(ts);
    const RowAddr ra = row_addr<LOGN>(data, data, rm, map);
    const PrimeConst P = pc[ra.prime];
    const u32 q = P.q, q2 = 2 * q;
    const uint2* w = tw + ((size_t)ra.prime << LOGN);  // {psi^-brv, Shoup companion} pairs
    const int col = threadIdx.x % CB, g = threadIdx.x / CB;
    const int c = blockIdx.x * CB + col;
    u32 x[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = ra.dst[(size_t)(16 * g + k) * 256 + c];
#pragma unroll
    for (int s = LOGR1 - 1; s >= 4; --s) {
        const int h = 1 << (LOGR1 - 1 - s);
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (!(k & h)) {
                const int ti = (1 << s) + ((16 * g + k) >> (LOGR1 - s));
                gs_bfly(x[k], x[k + h], w[ti].x, w[ti].y, q2, 0u - q);
            }
    }
    uint2 tb[15];  // stages 3..0's twiddles (block-uniform), loaded before the barrier
#pragma unroll
    for (int i = 0; i < 15; ++i) tb[i] = w[1 + i];
#pragma unroll
    for (int k = 0; k < 16; ++k) sm[(16 * g + k) * CB + col] = x[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = sm[(g + T * k) * CB + col];
#pragma unroll
    for (int s = 3; s >= 0; --s) {
        const int h = 8 >> s;
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (!(k & h)) {
                const uint2 t = tb[(1 << s) - 1 + (k >> (4 - s))];  // twiddle (1 << s) + (k >> (4 - s))
                gs_bfly(x[k], x[k + h], t.x, t.y, q2, 0u - q);
            }
    }
    if (post) {  // times post[row] too (a base conversion's qhat^{-1}): ONE multiply by N^{-1} post, formed per thread
        const u32 pw = shoup_mul(post[2 * blockIdx.y], P.ninv, P.ninv_p, q), pwp = shoup_pre_mu(pw, q, P.mu);
#pragma unroll
        for (int k = 0; k < 16; ++k) ra.dst[(size_t)(g + T * k) * 256 + c] = shoup_mul(x[k], pw, pwp, q);
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) ra.dst[(size_t)(g + T * k) * 256 + c] = shoup_mul(x[k], P.ninv, P.ninv_p, q);
    }
    ts_end(ts);
}

// pass 2 (rows) with NT threads per block; AESFHE_NTT_FIN_OCC=1 caps the finish mode at 128 VGPRs
// (4 waves per SIMD; unconstrained it takes 130)
template <int LOGR1, int M2, int NT>
void ntt2_fwd_launch(hipStream_t st, const DevTables& Tb, u32* dst, RowMap rm, LimbMap map, int groups, double io, double work,
                     const NttAux& aux) {
    if (fwd8_on()) {
        prof_launch_tsw(KID_NTT_ROWS_FWD, io, work, k_ntt2_fwd8<LOGR1, M2>, dim3((1 << LOGR1) / 8, rm.cnt, groups), dim3(256), 0, st, dst, rm, map,
                        Tb.pc, Tb.tw, aux);
        return;
    }
    const dim3 grid((1 << LOGR1) / (NT / 16), rm.cnt, groups);
    if (M2 == kFinish && fin_occ_on())
        prof_launch_tsw(KID_NTT_ROWS_FWD, io, work, k_ntt2_fwd<LOGR1, M2, NT, 4>, grid, dim3(NT), 0, st, dst, rm, map, Tb.pc, Tb.tw, aux);
    else
        prof_launch_tsw(KID_NTT_ROWS_FWD, io, work, k_ntt2_fwd<LOGR1, M2, NT>, grid, dim3(NT), 0, st, dst, rm, map, Tb.pc, Tb.tw, aux);
}
template <int LOGR1, int M2>
void ntt2_fwd_select(hipStream_t st, const DevTables& Tb, u32* dst, RowMap rm, LimbMap map, int groups, double io, double work,
                     const NttAux& aux) {
    switch (p2_nt_rows(false, rm.nrows)) {
        case 128: ntt2_fwd_launch<LOGR1, M2, 128>(st, Tb, dst, rm, map, groups, io, work, aux); break;
        case 512: ntt2_fwd_launch<LOGR1, M2, 512>(st, Tb, dst, rm, map, groups, io, work, aux); break;
        default: ntt2_fwd_launch<LOGR1, M2, 256>(st, Tb, dst, rm, map, groups, io, work, aux); break;
    }
}

// io_rows: rows actually transformed (launch rows minus skipped ones), for the byte count
template <int LOGR1, int M1, int M2>
void ntt_fwd_t(hipStream_t st, const DevTables& Tb, u32* dst, const u32* src, int rows, int io_rows, RowMap rm, LimbMap map,
               const NttAux& aux) {
    constexpr int R1 = 1 << LOGR1;
    rm.nrows = rows;
    const int groups = (rows + rm.cnt - 1) / rm.cnt;
    const double row_bytes = 4.0 * 256.0 * R1;
    const double io1 = 2.0 * io_rows * row_bytes;
    const double io2 = (M2 == kFinish ? (3.0 + (aux.add0 ? 0.5 : 0.0) + (aux.add1 ? 0.5 : 0.0)) : 2.0) * io_rows * row_bytes;
    const double bfly = (double)io_rows * 128.0 * R1;  // N / 2 butterflies per stage and row
    // launches of few rows: half-size blocks, so that the grid still spreads over every CU
    if (small_launch(rows)) {
        constexpr int NT = kThreads / 2, CB = NT / (R1 / 16);
        prof_launch_tsw(KID_NTT_COLS_FWD, io1, bfly * LOGR1, k_ntt1_fwd<LOGR1, M1, NT>, dim3(256 / CB, rm.cnt, groups), dim3(NT), 0, st, dst, src,
                        rm, map, Tb.pc, Tb.tw, aux);
        ntt2_fwd_launch<LOGR1, M2, NT>(st, Tb, dst, rm, map, groups, io2, bfly * 8.0, aux);
        return;
    }
    if (p1_nt_rows(false, rows) == 256) {
        constexpr int NT = kThreads / 2, CB = NT / (R1 / 16);
        prof_launch_tsw(KID_NTT_COLS_FWD, io1, bfly * LOGR1, k_ntt1_fwd<LOGR1, M1, NT>, dim3(256 / CB, rm.cnt, groups), dim3(NT), 0, st, dst, src,
                        rm, map, Tb.pc, Tb.tw, aux);
    } else {
        constexpr int CB = kThreads / (R1 / 16);
        prof_launch_tsw(KID_NTT_COLS_FWD, io1, bfly * LOGR1, k_ntt1_fwd<LOGR1, M1, kThreads>, dim3(256 / CB, rm.cnt, groups), dim3(kThreads), 0, st,
                        dst, src, rm, map, Tb.pc, Tb.tw, aux);
    }
    ntt2_fwd_select<LOGR1, M2>(st, Tb, dst, rm, map, groups, io2, bfly * 8.0, aux);
}
// AESFHE_NTT_INV_FACT=0: the inverse pass 2 reads every twiddle from the table (A/B runs)
inline bool inv_fact_on() {
    static const bool v = [] {
        const char* e = std::getenv("AESFHE_NTT_INV_FACT");
        return !(e && std::atoi(e) == 0);
    }();
    return v;
}
template <int LOGR1, int NT>
void ntt2_inv_launch(hipStream_t st, const DevTables& Tb, u32* dst, const u32* src, RowMap rm, LimbMap map, int groups, double io,
                     double work, const TensorPtrs* tp, bool rev) {
    if (inv8_on()) {
        static const TensorPtrs kNone8{};
        const dim3 g8(R1_of<LOGR1>() / 8, rm.cnt, groups);
#define INV8(F, IN, TP) prof_launch_tsw(KID_NTT_ROWS_INV, io, work, k_ntt2_inv8<LOGR1, F, IN>, g8, dim3(256), 0, st, dst, src, rm, map, Tb.pc, \
                                        Tb.itw, Tb.irow, Tb.igam, TP)
        if (tp) INV8(true, 1, *tp);
        else if (rev && inv_fact_on()) INV8(true, 2, kNone8);
        else if (rev) INV8(false, 2, kNone8);
        else if (inv_fact_on()) INV8(true, 0, kNone8);
        else INV8(false, 0, kNone8);
#undef INV8
        return;
    }
    const dim3 grid(R1_of<LOGR1>() / (NT / 16), rm.cnt, groups);
    if (tp) {
        prof_launch_tsw(KID_NTT_ROWS_INV, io, work, k_ntt2_inv<LOGR1, NT, true, 1>, grid, dim3(NT), 0, st, dst, src, rm, map, Tb.pc, Tb.itw,
                        Tb.irow, Tb.igam, *tp);
        return;
    }
    static const TensorPtrs kNone{};
    if (rev && inv_fact_on())
        prof_launch_tsw(KID_NTT_ROWS_INV, io, work, k_ntt2_inv<LOGR1, NT, true, 2>, grid, dim3(NT), 0, st, dst, src, rm, map, Tb.pc, Tb.itw,
                        Tb.irow, Tb.igam, kNone);
    else if (rev)  // AESFHE_NTT_INV_FACT=0 covers the conjugations' reversed ModUp too
        prof_launch_tsw(KID_NTT_ROWS_INV, io, work, k_ntt2_inv<LOGR1, NT, false, 2>, grid, dim3(NT), 0, st, dst, src, rm, map, Tb.pc, Tb.itw,
                        Tb.irow, Tb.igam, kNone);
    else if (inv_fact_on())
        prof_launch_tsw(KID_NTT_ROWS_INV, io, work, k_ntt2_inv<LOGR1, NT, true, 0>, grid, dim3(NT), 0, st, dst, src, rm, map, Tb.pc, Tb.itw,
                        Tb.irow, Tb.igam, kNone);
    else
        prof_launch_tsw(KID_NTT_ROWS_INV, io, work, k_ntt2_inv<LOGR1, NT, false, 0>, grid, dim3(NT), 0, st, dst, src, rm, map, Tb.pc, Tb.itw,
                        Tb.irow, Tb.igam, kNone);
}
template <int LOGR1>
void ntt_inv_t(hipStream_t st, const DevTables& Tb, u32* dst, const u32* src, int rows, RowMap rm, LimbMap map, const u32* post,
               const TensorPtrs* tp = nullptr, bool rev = false) {
    constexpr int R1 = 1 << LOGR1;
    rm.nrows = rows;
    const int groups = (rows + rm.cnt - 1) / rm.cnt;
    const double io = 4.0 * 2.0 * rows * (256.0 * R1);  // the inverse is never launched with skips
    const double io2 = tp ? 4.0 * 3.0 * rows * (256.0 * R1) : io;  // the product form reads two rows
    const double bfly = (double)rows * 128.0 * R1;
    if (small_launch(rows)) {
        constexpr int NT = kThreads / 2, CB = NT / (R1 / 16);
        ntt2_inv_launch<LOGR1, NT>(st, Tb, dst, src, rm, map, groups, io2, bfly * 8.0, tp, rev);
        prof_launch_tsw(KID_NTT_COLS_INV, io, bfly * LOGR1, k_ntt1_inv<LOGR1, NT>, dim3(256 / CB, rm.cnt, groups), dim3(NT), 0, st, dst, rm, map,
                        Tb.pc, Tb.itw, post);
        return;
    }
    switch (p2_nt_rows(true, rows)) {
        case 128: ntt2_inv_launch<LOGR1, 128>(st, Tb, dst, src, rm, map, groups, io2, bfly * 8.0, tp, rev); break;
        case 256: ntt2_inv_launch<LOGR1, 256>(st, Tb, dst, src, rm, map, groups, io2, bfly * 8.0, tp, rev); break;
        default: ntt2_inv_launch<LOGR1, kThreads>(st, Tb, dst, src, rm, map, groups, io2, bfly * 8.0, tp, rev); break;
    }
    if (p1_nt_rows(true, rows) == 256) {
        constexpr int NT = kThreads / 2, CB = NT / (R1 / 16);
        prof_launch_tsw(KID_NTT_COLS_INV, io, bfly * LOGR1, k_ntt1_inv<LOGR1, NT>, dim3(256 / CB, rm.cnt, groups), dim3(NT), 0, st, dst, rm, map,
                        Tb.pc, Tb.itw, post);
        return;
    }
    constexpr int CB = kThreads / (R1 / 16);
    prof_launch_tsw(KID_NTT_COLS_INV, io, bfly * LOGR1, k_ntt1_inv<LOGR1, kThreads>, dim3(256 / CB, rm.cnt, groups), dim3(kThreads), 0, st, dst, rm,
                    map, Tb.pc, Tb.itw, post);
}

// the column pass alone (the ModUp whose row pass runs inside k_ntt2_ki; the ModDown INTT whose row
// pass did): the same launches ntt_fwd_t / ntt_inv_t issue for that pass
template <int LOGR1>
void ntt_fwd_cols_t(hipStream_t st, const DevTables& Tb, u32* dst, const u32* src, int rows, int io_rows, RowMap rm, LimbMap map) {
    constexpr int R1 = 1 << LOGR1;
    rm.nrows = rows;
    const int groups = (rows + rm.cnt - 1) / rm.cnt;
    const double io1 = 2.0 * io_rows * 4.0 * 256.0 * R1, bfly = (double)io_rows * 128.0 * R1;
    if (small_launch(rows) || p1_nt_rows(false, rows) == 256) {
        constexpr int NT = kThreads / 2, CB = NT / (R1 / 16);
        prof_launch_tsw(KID_NTT_COLS_FWD, io1, bfly * LOGR1, k_ntt1_fwd<LOGR1, kPlain, NT>, dim3(256 / CB, rm.cnt, groups), dim3(NT), 0, st, dst,
                        src, rm, map, Tb.pc, Tb.tw, NttAux{});
        return;
    }
    constexpr int CB = kThreads / (R1 / 16);
    prof_launch_tsw(KID_NTT_COLS_FWD, io1, bfly * LOGR1, k_ntt1_fwd<LOGR1, kPlain, kThreads>, dim3(256 / CB, rm.cnt, groups), dim3(kThreads), 0, st,
                    dst, src, rm, map, Tb.pc, Tb.tw, NttAux{});
}
template <int LOGR1>
void ntt_inv_cols_t(hipStream_t st, const DevTables& Tb, u32* data, int rows, RowMap rm, LimbMap map, const u32* post) {
    constexpr int R1 = 1 << LOGR1;
    rm.nrows = rows;
    const int groups = (rows + rm.cnt - 1) / rm.cnt;
    const double io = 4.0 * 2.0 * rows * (256.0 * R1), bfly = (double)rows * 128.0 * R1;
    if (small_launch(rows) || p1_nt_rows(true, rows) == 256) {
        constexpr int NT = kThreads / 2, CB = NT / (R1 / 16);
        prof_launch_tsw(KID_NTT_COLS_INV, io, bfly * LOGR1, k_ntt1_inv<LOGR1, NT>, dim3(256 / CB, rm.cnt, groups), dim3(NT), 0, st, data, rm, map,
                        Tb.pc, Tb.itw, post);
        return;
    }
    constexpr int CB = kThreads / (R1 / 16);
    prof_launch_tsw(KID_NTT_COLS_INV, io, bfly * LOGR1, k_ntt1_inv<LOGR1, kThreads>, dim3(256 / CB, rm.cnt, groups), dim3(kThreads), 0, st, data,
                    rm, map, Tb.pc, Tb.itw, post);
}

// pass 1 fused with the base conversion (k_ntt1_fwd_conv), then pass 2 in mode M2
template <int LOGR1, int NT, int H>
void ntt1_conv_launch(hipStream_t st, const DevTables& Tb, u32* dst, const ConvBatch& cb, RowMap rm, LimbMap map, int groups, double io,
                      double work) {
    constexpr int CB = NT / ((1 << LOGR1) / 16);
    prof_launch_tsw(KID_NTT_COLS_FWD, io, work, k_ntt1_fwd_conv<LOGR1, NT, H>, dim3(256 / CB, rm.cnt, groups), dim3(NT), 0, st, dst, rm, map,
                    Tb.pc, Tb.tw, cb);
}
template <int LOGR1, int NT>
void ntt1_conv_dispatch(hipStream_t st, const DevTables& Tb, u32* dst, const ConvBatch& cb, int h, RowMap rm, LimbMap map, int groups,
                        double io, double work) {
    switch (h) {
#define CONV_H(H) \
    case H: ntt1_conv_launch<LOGR1, NT, H>(st, Tb, dst, cb, rm, map, groups, io, work); break;
        CONV_H(1) CONV_H(2) CONV_H(3) CONV_H(4) CONV_H(5) CONV_H(6) CONV_H(7) CONV_H(8)
        CONV_H(9) CONV_H(10) CONV_H(11) CONV_H(12) CONV_H(13) CONV_H(14) CONV_H(15) CONV_H(16)
#undef CONV_H
        default: throw std::runtime_error("ntt_fwd_conv: unsupported source count");
    }
}
template <int M2>
void ntt_fwd_conv_t(hipStream_t st, const DevTables& Tb, u32* dst, const ConvBatch& cb, int rows, int io_rows, RowMap rm, LimbMap map,
                    const NttAux& aux) {
    constexpr int LOGR1 = 8, R1 = 1 << LOGR1;
    rm.nrows = rows;
    const int groups = (rows + rm.cnt - 1) / rm.cnt;
    if (groups != cb.n) throw std::runtime_error("ntt_fwd_conv: one conversion group per row group expected");
    int h = 0, src_rows = 0;
    for (int z = 0; z < cb.n; ++z) {
        if (cb.h[z] < 1) throw std::runtime_error("ntt_fwd_conv: a conversion group without sources");
        h = std::max(h, cb.h[z]);
        src_rows += cb.h[z];
    }
    const double row_bytes = 4.0 * 256.0 * R1;
    const double io1 = (double)(io_rows + src_rows) * row_bytes;  // sources read once, converted rows written
    const double io2 = (M2 == kFinish ? (3.0 + (aux.add0 ? 0.5 : 0.0) + (aux.add1 ? 0.5 : 0.0)) : 2.0) * io_rows * row_bytes;
    const double bfly = (double)io_rows * 128.0 * R1;
    if (small_launch(rows)) {
        constexpr int NT = kThreads / 2;
        ntt1_conv_dispatch<LOGR1, NT>(st, Tb, dst, cb, h, rm, map, groups, io1, bfly * LOGR1);
        ntt2_fwd_launch<LOGR1, M2, NT>(st, Tb, dst, rm, map, groups, io2, bfly * 8.0, aux);
        return;
    }
    ntt1_conv_dispatch<LOGR1, kThreads>(st, Tb, dst, cb, h, rm, map, groups, io1, bfly * LOGR1);
    ntt2_fwd_select<LOGR1, M2>(st, Tb, dst, rm, map, groups, io2, bfly * 8.0, aux);
}

// ---------------------------------------------------------------- fused key-switch core
// ONE launch for what was three: the ModUp's forward row pass (pass 2) of every digit's extended
// rows, the key inner product acc = sum_j ext_j (.) key_j (k_key_inner, incl. its fold / tensor /
// reversed-own-digit forms and a second summed source), and the row pass of the ModDown's inverse
// NTT on the acc rows the ModDown converts.  A block owns one 4,096-coefficient chunk (16 rows of
// 256 words) of one target limb x of one member: the NTT-domain ext values never leave registers
// (no ext write + re-read), and the rows >= kept go to the ModDown as its inverse pass-1 input (no
// acc write + re-read of those rows).  Every stored value is the one the separate kernels store
// (canonical acc; the inverse row pass's lazy residues by the same butterfly sequence), so the
// ciphertexts are bit-identical (tests/test_gpu_fused_ki.py).
// forward pass-2 stages on x[k] = word jt + 16 k of row R ([0, 4q) from pass 1) -> x[k] = word
// 16 jt + k, canonical (k_ntt2_fwd's arithmetic)
template <int LOGR1>
__device__ __forceinline__ void ki_fwd_rows(u32 (&x)[16], u32* row, const uint2* w, int R, int j, u32 q, u32 q2) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int h = 8 >> s;
        const int base = (1 << (LOGR1 + s)) + (R << s);
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (!(k & h)) {
                const int ti = base + (k >> (4 - s));
                ct_bfly(x[k], x[k + h], w[ti].x, w[ti].y, q2, q);
            }
    }
    uint2 tb[15];
#pragma unroll
    for (int s = 4; s < 8; ++s) {
        const int c = 1 << (s - 4), base = (1 << (LOGR1 + s)) + (R << s) + (j << (s - 4));
#pragma unroll
        for (int u = 0; u < c; ++u) tb[c - 1 + u] = w[base + u];
    }
    __syncthreads();  // the previous user of the LDS row is done reading it
#pragma unroll
    for (int k = 0; k < 16; ++k) row[swz(j + 16 * k)] = x[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = row[swz(16 * j + k)];
#pragma unroll
    for (int s = 4; s < 8; ++s) {
        const int h = 1 << (7 - s), c = 1 << (s - 4);
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (!(k & h)) {
                const uint2 t = tb[c - 1 + (k >> (8 - s))];
                ct_bfly(x[k], x[k + h], t.x, t.y, q2, q);
            }
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = canon4(x[k], q);
}
// inverse pass-2 stages on x[k] = word 16 jt + k of row R (canonical) -> x[k] = word jt + 16 k, the
// residues k_ntt2_inv<LOGR1, NT, FACT, 0> stores (same butterflies, same twiddles, same order)
template <int LOGR1, bool FACT>
__device__ __forceinline__ void ki_inv_rows(u32 (&x)[16], u32* row, const uint2* w, const uint2* rowf, const uint2* gam, int R, int j,
                                            u32 q, u32 q2) {
#pragma unroll
    for (int s = 7; s >= 4; --s) {
        const int h = 1 << (7 - s);
        const int base = (1 << (LOGR1 + s)) + (R << s);
        if (FACT && s >= 5) {
            const uint2 rf = rowf[s - 5];
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (!(k & h)) gs_bfly2(x[k], x[k + h], gam[(1 << s) + ((16 * j + k) >> (8 - s))], rf, q2, 0u - q);
            continue;
        }
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (!(k & h)) {
                const int ti = base + ((16 * j + k) >> (8 - s));
                gs_bfly(x[k], x[k + h], w[ti].x, w[ti].y, q2, 0u - q);
            }
    }
    uint2 tb[15];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int base = (1 << (LOGR1 + s)) + (R << s);
#pragma unroll
        for (int u = 0; u < (1 << s); ++u) tb[(1 << s) - 1 + u] = w[base + u];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) row[swz(16 * j + k)] = x[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = row[swz(j + 16 * k)];
#pragma unroll
    for (int s = 3; s >= 0; --s) {
        const int h = 8 >> s;
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (!(k & h)) {
                const uint2 t = tb[(1 << s) - 1 + (k >> (4 - s))];
                gs_bfly(x[k], x[k + h], t.x, t.y, q2, 0u - q);
            }
    }
}
__device__ __forceinline__ void ld16(u32 (&e)[16], const u32* p) {
    const uint4* v = reinterpret_cast<const uint4*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint4 t = v[i];
        e[4 * i] = t.x, e[4 * i + 1] = t.y, e[4 * i + 2] = t.z, e[4 * i + 3] = t.w;
    }
}
__device__ __forceinline__ void st16(u32* p, const u32 (&e)[16]) {
    uint4* v = reinterpret_cast<uint4*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) st_out16(v + i, make_uint4(e[4 * i], e[4 * i + 1], e[4 * i + 2], e[4 * i + 3]));
}
// PF: the digit's key rows are loaded right after its ext rows and before the forward row pass, so
// their latency overlaps the butterflies instead of following them (AESFHE_KI_PF, default on: 44.6
// -> 43.8 us per launch, C2 +0.3 %, profiles/r4_ab_ki_pf.txt; the loads are issued ext first:
// vmcnt retires in order, the pass waits only for the ext values; 242 VGPRs, still 2 waves / SIMD)
template <int LOGR1, bool FACT, bool PF>
__global__ void __launch_bounds__(256) k_ntt2_ki(KiArgs a, LimbMap map, const PrimeConst* pc, const uint2* tw, const uint2* itw,
                                                 const uint2* irow, const uint2* igam, unsigned long long* ts) {
    constexpr int LOGN = LOGR1 + 8, CH = (1 << LOGR1) / 16;  // 16-row chunks per limb
    __shared__ u32 sm[16 * kPitchP2];
    // block -> (member, limb, chunk): the members of one (limb, chunk) -- which read the same key
    // chunk -- consecutive on ONE XCD (blocks are dealt round-robin over the 8 XCDs), so the key
    // chunk is fetched into that XCD's L2 once for all members
    const int b = blockIdx.x, nb = a.nb;
    int m, u;
    if (((CH * a.ne) & 7) == 0) {
        const int w = b >> 3;
        m = w % nb;
        u = (w / nb) * 8 + (b & 7);
    } else {
        m = b % nb;
        u = b / nb;
    }
    const int chunk = u % CH, x = u / CH;
    ts_begin(ts);
    const int prime = map.prime(x);
    const PrimeConst P = pc[prime];
    const u32 q = P.q, q2 = 2 * q;
    const int r = threadIdx.x >> 4, jt = threadIdx.x & 15, R = chunk * 16 + r;
    const size_t c0 = (size_t)R * 256 + 16 * jt;  // this thread's 16 consecutive coefficients
    u32* row = sm + r * kPitchP2;
    const int krow = x < a.nl ? x : a.nks + (x - a.nl);
    const int own = x < a.nl ? x / a.alpha : -1;
    u64 s0[16], s1[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) s0[k] = s1[k] = 0;
    int cnt = 0;
    for (int src = 0; src < a.nsrc; ++src) {
        for (int jd = 0; jd < a.nd; ++jd, ++cnt) {
            if (cnt && (cnt & 7) == 0) {
#pragma unroll
                for (int k = 0; k < 16; ++k) s0[k] = fold64(s0[k], q, P.r32), s1[k] = fold64(s1[k], q, P.r32);
            }
            u32 e[16];
            const u32* kb = a.key[src] + (((size_t)jd * 2 * a.nkey + krow) << LOGN) + c0;
            const u32* ka = kb + ((size_t)a.nkey << LOGN);
            uint4 vk0[4], vk1[4];
            bool kld = false;
            if (jd == own) {  // block-uniform: the digit's own limb comes from the NTT-form input
                if (a.fold.ta[0]) {  // tensor mode: c2 = a1 (.) b1 of the product, formed here
                    const size_t at = ((size_t)(a.fold.tnl + x) << LOGN) + c0;
                    const uint4* pa = reinterpret_cast<const uint4*>(a.fold.ta[m] + at);
                    const uint4* pb = reinterpret_cast<const uint4*>(a.fold.tb[m] + at);
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const uint4 va = pa[i], vb = pb[i];
                        e[4 * i] = barrett_mul(va.x, vb.x, q, P.mu), e[4 * i + 1] = barrett_mul(va.y, vb.y, q, P.mu);
                        e[4 * i + 2] = barrett_mul(va.z, vb.z, q, P.mu), e[4 * i + 3] = barrett_mul(va.w, vb.w, q, P.mu);
                    }
                } else if (a.fold.rev_d) {  // the conjugation: element v <- word N - 1 - (c0 + v)
                    const uint4* v = reinterpret_cast<const uint4*>(a.d[src] + m * a.d_ms + ((size_t)x << LOGN) + ((size_t)1 << LOGN) - 16 - c0);
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const uint4 t = v[i];
                        e[15 - 4 * i] = t.x, e[14 - 4 * i] = t.y, e[13 - 4 * i] = t.z, e[12 - 4 * i] = t.w;
                    }
                } else {
                    ld16(e, a.d[src] + m * a.d_ms + ((size_t)x << LOGN) + c0);
                }
            } else {
                const u32* p = a.ext[src] + m * a.ext_ms + (((size_t)jd * a.ne + x) << LOGN) + (size_t)R * 256;
#pragma unroll
                for (int k = 0; k < 16; ++k) e[k] = p[jt + 16 * k];
                if (PF) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) vk0[i] = reinterpret_cast<const uint4*>(kb)[i], vk1[i] = reinterpret_cast<const uint4*>(ka)[i];
                    kld = true;
                }
                ki_fwd_rows<LOGR1>(e, row, tw + ((size_t)prime << LOGN), R, jt, q, q2);
            }
            if (!kld)
#pragma unroll
                for (int i = 0; i < 4; ++i) vk0[i] = reinterpret_cast<const uint4*>(kb)[i], vk1[i] = reinterpret_cast<const uint4*>(ka)[i];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint4 vb = vk0[i], va = vk1[i];
                s0[4 * i] += (u64)e[4 * i] * vb.x, s1[4 * i] += (u64)e[4 * i] * va.x;
                s0[4 * i + 1] += (u64)e[4 * i + 1] * vb.y, s1[4 * i + 1] += (u64)e[4 * i + 1] * va.y;
                s0[4 * i + 2] += (u64)e[4 * i + 2] * vb.z, s1[4 * i + 2] += (u64)e[4 * i + 2] * va.z;
                s0[4 * i + 3] += (u64)e[4 * i + 3] * vb.w, s1[4 * i + 3] += (u64)e[4 * i + 3] * va.w;
            }
        }
    }
    u32 r0[16], r1[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) r0[k] = reduce64(s0[k], q, P.mu, P.r32), r1[k] = reduce64(s1[k], q, P.mu, P.r32);
    if (a.fold.gad && x < a.nl) {  // + P (c0, c1) on the Q rows (k_key_inner's fold), four words at a time
        const u32 gv = a.fold.gad[2 * x], gp = a.fold.gad[2 * x + 1];
        const bool tens = a.fold.ta[0] != nullptr;
        const size_t at = tens ? ((size_t)x << LOGN) + c0 : m * a.fold.ms + ((size_t)x << LOGN) + c0;
        const size_t o1 = (size_t)a.fold.tnl << LOGN;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            u32 f0[4], f1[4];
            if (tens) {  // tensor mode: c0 = a0 b0, c1 = a0 b1 + a1 b0
                const uint4 A0 = reinterpret_cast<const uint4*>(a.fold.ta[m] + at)[i], A1 = reinterpret_cast<const uint4*>(a.fold.ta[m] + at + o1)[i];
                const uint4 B0 = reinterpret_cast<const uint4*>(a.fold.tb[m] + at)[i], B1 = reinterpret_cast<const uint4*>(a.fold.tb[m] + at + o1)[i];
                const u32 a0[4] = {A0.x, A0.y, A0.z, A0.w}, a1[4] = {A1.x, A1.y, A1.z, A1.w};
                const u32 b0[4] = {B0.x, B0.y, B0.z, B0.w}, b1[4] = {B1.x, B1.y, B1.z, B1.w};
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    f0[v] = barrett_mul(a0[v], b0[v], q, P.mu);
                    f1[v] = add_mod(barrett_mul(a0[v], b1[v], q, P.mu), barrett_mul(a1[v], b0[v], q, P.mu), q);
                }
            } else {
                const uint4 F0 = reinterpret_cast<const uint4*>(a.fold.add0 + at)[i], F1 = reinterpret_cast<const uint4*>(a.fold.add1 + at)[i];
                f0[0] = F0.x, f0[1] = F0.y, f0[2] = F0.z, f0[3] = F0.w;
                f1[0] = F1.x, f1[1] = F1.y, f1[2] = F1.z, f1[3] = F1.w;
            }
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                r0[4 * i + v] = add_mod(r0[4 * i + v], shoup_mul(f0[v], gv, gp, q), q);
                r1[4 * i + v] = add_mod(r1[4 * i + v], shoup_mul(f1[v], gv, gp, q), q);
            }
        }
    }
    if (x < a.kept) {  // kept rows: the ModDown finish's cur operand, acc layout [m][2][ne]
        st16(a.acc + m * a.acc_ms + ((size_t)x << LOGN) + c0, r0);
        st16(a.acc + m * a.acc_ms + ((size_t)(a.ne + x) << LOGN) + c0, r1);
    } else {  // converted rows: the ModDown's inverse row pass, into its pass-1 input ys [m][2][ys_rows]
        const uint2* iw = itw + ((size_t)prime << LOGN);
        const uint2* rowf = irow + ((size_t)prime << LOGR1) * 4 + (size_t)R * 4;
        const uint2* gam = igam + ((size_t)prime << 8);
        ki_inv_rows<LOGR1, FACT>(r0, row, iw, rowf, gam, R, jt, q, q2);
        u32* y0 = a.ys + m * a.ys_ms + ((size_t)(x - a.kept) << LOGN) + (size_t)R * 256;
#pragma unroll
        for (int k = 0; k < 16; ++k) y0[jt + 16 * k] = r0[k];
        ki_inv_rows<LOGR1, FACT>(r1, row, iw, rowf, gam, R, jt, q, q2);
        u32* y1 = a.ys + m * a.ys_ms + ((size_t)(a.ys_rows + x - a.kept) << LOGN) + (size_t)R * 256;
#pragma unroll
        for (int k = 0; k < 16; ++k) y1[jt + 16 * k] = r1[k];
    }
    ts_end(ts);
}
// k_ntt2_ki's work with 8 residues per thread (the row-pass helpers ki8_*: top of this file); the same arguments, block -> (member,
// limb, 8-row chunk) with the same XCD grouping of a chunk's members
template <int LOGR1>
__global__ void __launch_bounds__(256) k_ntt2_ki8(KiArgs a, LimbMap map, const PrimeConst* pc, const uint2* tw, const uint2* itw,
                                                  const uint2* irow, const uint2* igam, unsigned long long* ts) {
    constexpr int LOGN = LOGR1 + 8, CH = (1 << LOGR1) / 8;  // 8-row chunks per limb
    __shared__ u32 sm[8 * kPitch8];
    const int b = blockIdx.x, nb = a.nb;
    int m, u;
    if (((CH * a.ne) & 7) == 0) {
        const int wv = b >> 3;
        m = wv % nb;
        u = (wv / nb) * 8 + (b & 7);
    } else {
        m = b % nb;
        u = b / nb;
    }
    const int chunk = u % CH, x = u / CH;
    ts_begin(ts);
    const int prime = map.prime(x);
    const PrimeConst P = pc[prime];
    const u32 q = P.q, q2 = 2 * q;
    const int r = threadIdx.x >> 5, t = threadIdx.x & 31, R = chunk * 8 + r;
    const size_t c0 = (size_t)R * 256 + 8 * t;  // this thread's 8 consecutive coefficients (phase C)
    u32* row = sm + r * kPitch8;
    const int krow = x < a.nl ? x : a.nks + (x - a.nl);
    const int own = x < a.nl ? x / a.alpha : -1;
    u64 s0[8], s1[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) s0[k] = s1[k] = 0;
    int cnt = 0;
    for (int src = 0; src < a.nsrc; ++src) {
        for (int jd = 0; jd < a.nd; ++jd, ++cnt) {
            if (cnt && (cnt & 7) == 0) {
#pragma unroll
                for (int k = 0; k < 8; ++k) s0[k] = fold64(s0[k], q, P.r32), s1[k] = fold64(s1[k], q, P.r32);
            }
            u32 e[8];
            const u32* kb = a.key[src] + (((size_t)jd * 2 * a.nkey + krow) << LOGN) + c0;
            const u32* ka = kb + ((size_t)a.nkey << LOGN);
            if (jd == own) {  // block-uniform: the digit's own limb comes from the NTT-form input
                if (a.fold.ta[0]) {  // tensor mode: c2 = a1 (.) b1 of the product, formed here
                    const size_t at = ((size_t)(a.fold.tnl + x) << LOGN) + c0;
                    const uint4* pa = reinterpret_cast<const uint4*>(a.fold.ta[m] + at);
                    const uint4* pb = reinterpret_cast<const uint4*>(a.fold.tb[m] + at);
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        const uint4 va = pa[i], vb = pb[i];
                        e[4 * i] = barrett_mul(va.x, vb.x, q, P.mu), e[4 * i + 1] = barrett_mul(va.y, vb.y, q, P.mu);
                        e[4 * i + 2] = barrett_mul(va.z, vb.z, q, P.mu), e[4 * i + 3] = barrett_mul(va.w, vb.w, q, P.mu);
                    }
                } else if (a.fold.rev_d) {  // the conjugation: element v <- word N - 1 - (c0 + v)
                    const uint4* v = reinterpret_cast<const uint4*>(a.d[src] + m * a.d_ms + ((size_t)x << LOGN) + ((size_t)1 << LOGN) - 8 - c0);
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        const uint4 tt = v[i];
                        e[7 - 4 * i] = tt.x, e[6 - 4 * i] = tt.y, e[5 - 4 * i] = tt.z, e[4 - 4 * i] = tt.w;
                    }
                } else {
                    ld8(e, a.d[src] + m * a.d_ms + ((size_t)x << LOGN) + c0);
                }
            } else {
                const u32* p = a.ext[src] + m * a.ext_ms + (((size_t)jd * a.ne + x) << LOGN) + (size_t)R * 256;
#pragma unroll
                for (int k = 0; k < 8; ++k) e[k] = p[t + 32 * k];
                ki8_fwd_rows<LOGR1>(e, row, tw + ((size_t)prime << LOGN), R, t, q, q2);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const uint4 vb = reinterpret_cast<const uint4*>(kb)[i], va = reinterpret_cast<const uint4*>(ka)[i];
                s0[4 * i] += (u64)e[4 * i] * vb.x, s1[4 * i] += (u64)e[4 * i] * va.x;
                s0[4 * i + 1] += (u64)e[4 * i + 1] * vb.y, s1[4 * i + 1] += (u64)e[4 * i + 1] * va.y;
                s0[4 * i + 2] += (u64)e[4 * i + 2] * vb.z, s1[4 * i + 2] += (u64)e[4 * i + 2] * va.z;
                s0[4 * i + 3] += (u64)e[4 * i + 3] * vb.w, s1[4 * i + 3] += (u64)e[4 * i + 3] * va.w;
            }
        }
    }
    u32 r0[8], r1[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) r0[k] = reduce64(s0[k], q, P.mu, P.r32), r1[k] = reduce64(s1[k], q, P.mu, P.r32);
    if (a.fold.gad && x < a.nl) {  // + P (c0, c1) on the Q rows (k_key_inner's fold), four words at a time
        const u32 gv = a.fold.gad[2 * x], gp = a.fold.gad[2 * x + 1];
        const bool tens = a.fold.ta[0] != nullptr;
        const size_t at = tens ? ((size_t)x << LOGN) + c0 : m * a.fold.ms + ((size_t)x << LOGN) + c0;
        const size_t o1 = (size_t)a.fold.tnl << LOGN;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            u32 f0[4], f1[4];
            if (tens) {  // tensor mode: c0 = a0 b0, c1 = a0 b1 + a1 b0
                const uint4 A0 = reinterpret_cast<const uint4*>(a.fold.ta[m] + at)[i], A1 = reinterpret_cast<const uint4*>(a.fold.ta[m] + at + o1)[i];
                const uint4 B0 = reinterpret_cast<const uint4*>(a.fold.tb[m] + at)[i], B1 = reinterpret_cast<const uint4*>(a.fold.tb[m] + at + o1)[i];
                const u32 a0[4] = {A0.x, A0.y, A0.z, A0.w}, a1[4] = {A1.x, A1.y, A1.z, A1.w};
                const u32 b0[4] = {B0.x, B0.y, B0.z, B0.w}, b1[4] = {B1.x, B1.y, B1.z, B1.w};
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    f0[v] = barrett_mul(a0[v], b0[v], q, P.mu);
                    f1[v] = add_mod(barrett_mul(a0[v], b1[v], q, P.mu), barrett_mul(a1[v], b0[v], q, P.mu), q);
                }
            } else {
                const uint4 F0 = reinterpret_cast<const uint4*>(a.fold.add0 + at)[i], F1 = reinterpret_cast<const uint4*>(a.fold.add1 + at)[i];
                f0[0] = F0.x, f0[1] = F0.y, f0[2] = F0.z, f0[3] = F0.w;
                f1[0] = F1.x, f1[1] = F1.y, f1[2] = F1.z, f1[3] = F1.w;
            }
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                r0[4 * i + v] = add_mod(r0[4 * i + v], shoup_mul(f0[v], gv, gp, q), q);
                r1[4 * i + v] = add_mod(r1[4 * i + v], shoup_mul(f1[v], gv, gp, q), q);
            }
        }
    }
    if (x < a.kept) {  // kept rows: the ModDown finish's cur operand, acc layout [m][2][ne]
        st8(a.acc + m * a.acc_ms + ((size_t)x << LOGN) + c0, r0);
        st8(a.acc + m * a.acc_ms + ((size_t)(a.ne + x) << LOGN) + c0, r1);
    } else {  // converted rows: the ModDown's inverse row pass, into its pass-1 input ys [m][2][ys_rows]
        const uint2* iw = itw + ((size_t)prime << LOGN);
        const uint2* rowf = irow + ((size_t)prime << LOGR1) * 4 + (size_t)R * 4;
        const uint2* gam = igam + ((size_t)prime << 8);
        ki8_inv_rows<LOGR1, true>(r0, row, iw, rowf, gam, R, t, q, q2);
        u32* y0 = a.ys + m * a.ys_ms + ((size_t)(x - a.kept) << LOGN) + (size_t)R * 256;
#pragma unroll
        for (int k = 0; k < 8; ++k) y0[t + 32 * k] = r0[k];
        ki8_inv_rows<LOGR1, true>(r1, row, iw, rowf, gam, R, t, q, q2);
        u32* y1 = a.ys + m * a.ys_ms + ((size_t)(a.ys_rows + x - a.kept) << LOGN) + (size_t)R * 256;
#pragma unroll
        for (int k = 0; k < 8; ++k) y1[t + 32 * k] = r1[k];
    }
    ts_end(ts);
}
inline bool ki8_on() {
    static const bool v = [] {
        const char* e = std::getenv("AESFHE_KI8");
        return e ? std::atoi(e) != 0 : true;
    }();
    return v;
}
inline bool ki_pf() {
    static const bool v = [] {
        const char* e = std::getenv("AESFHE_KI_PF");
        return e ? std::atoi(e) != 0 : true;
    }();
    return v;
}
template <int LOGR1>
void ki_launch(hipStream_t st, const DevTables& Tb, const KiArgs& a, LimbMap map) {
    constexpr int CH = (1 << LOGR1) / 16;
    const double row = 4.0 * (256.0 * (1 << LOGR1));
    // per member: the digits' extended rows read once (own-digit rows from d), the key once per
    // launch (members share it), acc / ys rows written; fold rows read
    int ext_rows = 0;
    for (int x = 0; x < a.ne; ++x)
        for (int j = 0; j < a.nd; ++j) ext_rows += !(x < a.nl && x / a.alpha == j);
    const double per_m = a.nsrc * (double)(ext_rows + std::min(a.nl, a.nd * a.alpha)) + 2.0 * a.ne +
                         (a.fold.gad ? (a.fold.ta[0] ? 4.0 : 2.0) * a.nl : 0.0);
    const double bytes = row * (a.nb * per_m + a.nsrc * 2.0 * a.nd * a.ne);
    const double bfly = 128.0 * (1 << LOGR1) * 8.0 * (a.nb * (a.nsrc * (double)ext_rows + 2.0 * (a.ne - a.kept)));
    if (ki8_on()) {
        // (capped at 128 VGPRs -- 4 waves per SIMD, 36 VGPRs spilled -- it ran slower: C2 80.7 -> 72.8
        // rounds/s, a 64-pair stack 96.2 -> 106.0 ms per pair, profiles/r6_ki8_occ_ab.txt)
        prof_launch_tsw(KID_KEY_INNER, bytes, bfly, k_ntt2_ki8<LOGR1>, dim3(2 * CH * a.ne * a.nb), dim3(256), 0, st, a, map, Tb.pc, Tb.tw,
                        Tb.itw, Tb.irow, Tb.igam);
        return;
    }
    const dim3 grid(CH * a.ne * a.nb);
#define KI_GO(F, PF) prof_launch_tsw(KID_KEY_INNER, bytes, bfly, k_ntt2_ki<LOGR1, F, PF>, grid, dim3(256), 0, st, a, map, Tb.pc, Tb.tw, Tb.itw, Tb.irow, Tb.igam)
    if (inv_fact_on()) {
        if (ki_pf()) KI_GO(true, true);
        else KI_GO(true, false);
    } else {
        if (ki_pf()) KI_GO(false, true);
        else KI_GO(false, false);
    }
#undef KI_GO
}


// ---------------------------------------------------------------- column-domain basis extension
// ONE launch for the middle of a ModUp / ModDown: the inverse NTT's column pass of a group's H
// source limbs (their row pass already done: k_ntt2_inv, or k_ntt2_ki for the ModDown's P rows),
// the base conversion to the group's target limbs (k_base_convert's arithmetic, in its order) and
// the forward NTT's column pass of every target limb (k_ntt1_fwd's) -- before, three launches with
// the coefficient-form sources and the converted rows each written and re-read in between.
// A block owns an 8-column tile of all 256 rows (N = 2^16: 256 x 256) of one group, for a range of
// its targets: it runs the H inverse column transforms itself (every target range of the group
// repeats them -- the price of needing no other block's data), keeps the H x 8 converted-source
// residues per thread in VGPRs, and transforms each target in three register passes of 3 / 3 / 2
// butterfly stages with two LDS exchanges (alternating buffers: one barrier each).  The values
// stored are congruent to the separate kernels' at every hand-off and canonical where those are
// (the INTT output, the conversion output), so the ciphertexts are bit-identical
// (tests/test_gpu_bx_cols.py).
// Thread (p = tid / 8, c = tid % 8) holds column 8 tile + c, rows by layout:
//   A  p + 32 e                (stages 0-2 forward / 1-0 inverse)
//   Bf (p&3) + 32 (p>>2) + 4 e (forward stages 3-5)   Bi (p&7) + 64 (p>>3) + 8 e (inverse 4-2)
//   C  8 p + e                 (forward 6-7 / inverse 7-5)
// LDS word of (row, c): a 32-word block per 4 rows, rotated by 8 ((row >> 3) & 3): every layout's
// half-wave touches 32 distinct banks (checked exhaustively, tools/bx_layout_check.py).
enum { kBxA = 0, kBxBf = 1, kBxBi = 2, kBxC = 3 };
template <int L>
__device__ __forceinline__ int bx_row(int p, int e) {
    return L == kBxA ? p + 32 * e : L == kBxBf ? (p & 3) + 32 * (p >> 2) + 4 * e : L == kBxBi ? (p & 7) + 64 * (p >> 3) + 8 * e : 8 * p + e;
}
__device__ __forceinline__ int bx_lds(int row, int c) { return (row >> 2) * 32 + (((row & 3) * 8 + c + 8 * ((row >> 3) & 3)) & 31); }
// stage S (row distance 128 >> S) on the elements of layout L that differ in bit H of e
template <int L, int S, int H>
__device__ __forceinline__ void bx_fwd(u32 (&x)[8], const uint2* w, int p, u32 q2, u32 q) {
#pragma unroll
    for (int e = 0; e < 8; ++e)
        if (!(e & H)) {
            const uint2 t = w[(1 << S) + (bx_row<L>(p, e) >> (8 - S))];
            ct_bfly(x[e], x[e + H], t.x, t.y, q2, q);
        }
}
template <int L, int S, int H>
__device__ __forceinline__ void bx_inv(u32 (&x)[8], const uint2* w, int p, u32 q2, u32 nq) {
#pragma unroll
    for (int e = 0; e < 8; ++e)
        if (!(e & H)) {
            const uint2 t = w[(1 << S) + (bx_row<L>(p, e) >> (8 - S))];
            gs_bfly(x[e], x[e + H], t.x, t.y, q2, nq);
        }
}
template <int LA, int LB>
__device__ __forceinline__ void bx_xchg(u32 (&x)[8], u32* sm, int p, int c) {
#pragma unroll
    for (int e = 0; e < 8; ++e) sm[bx_lds(bx_row<LA>(p, e), c)] = x[e];
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = sm[bx_lds(bx_row<LB>(p, e), c)];
}
// source I of the group (template recursion: every y[I] index is a compile-time constant, so the
// residues stay in VGPRs at any HM -- a run-time loop this large is not unrolled and goes to scratch)
// nx: source I's residues, loaded by the previous step; source I + 1's are issued here before
// source I's transform, so their latency overlaps it
__device__ __forceinline__ void bx_load(u32 (&x)[8], const u32* s, int p, int col) {
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = s[(size_t)bx_row<kBxC>(p, e) * 256 + col];
}
template <int I, int HM>
__device__ __forceinline__ void bx_sources(u32 (&y)[HM][8], u32 (&nx)[8], const ConvBatch& cb, int z, int hz, int sp, const PrimeConst* pc,
                                           const uint2* itw, u32 (*sm)[2048], int& buf, int p, int c, int col) {
    if constexpr (I < HM) {
        constexpr int LOGN = 16;
        if (I < hz) {  // block-uniform
            const int prime = (sp > 0 && I >= sp) ? cb.d1[z] + (I - sp) : cb.d0[z] + I;
            const PrimeConst P = pc[prime];
            const u32 q = P.q, q2 = 2 * q, nq = 0u - q;
            const uint2* w = itw + ((size_t)prime << LOGN);
            u32 x[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) x[e] = nx[e];
            if (I + 1 < hz) bx_load(nx, cb.src[z] + ((size_t)(I + 1) << LOGN), p, col);
            bx_inv<kBxC, 7, 1>(x, w, p, q2, nq);
            bx_inv<kBxC, 6, 2>(x, w, p, q2, nq);
            bx_inv<kBxC, 5, 4>(x, w, p, q2, nq);
            bx_xchg<kBxC, kBxBi>(x, sm[buf], p, c);
            buf ^= 1;
            bx_inv<kBxBi, 4, 1>(x, w, p, q2, nq);
            bx_inv<kBxBi, 3, 2>(x, w, p, q2, nq);
            bx_inv<kBxBi, 2, 4>(x, w, p, q2, nq);
            bx_xchg<kBxBi, kBxA>(x, sm[buf], p, c);
            buf ^= 1;
            bx_inv<kBxA, 1, 2>(x, w, p, q2, nq);
            bx_inv<kBxA, 0, 4>(x, w, p, q2, nq);
            // k_ntt1_inv's N^-1 (canonical), then k_base_convert's qhat^-1 and its y / q fixed point
            const u32 qw = cb.qhinv[z][2 * I], qwp = cb.qhinv[z][2 * I + 1];
#pragma unroll
            for (int e = 0; e < 8; ++e) y[I][e] = shoup_mul(shoup_mul(x[e], P.ninv, P.ninv_p, q), qw, qwp, q);
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) y[I][e] = 0u;
        }
        bx_sources<I + 1, HM>(y, nx, cb, z, hz, sp, pc, itw, sm, buf, p, c, col);
    }
}
template <int HM>
__global__ void __launch_bounds__(256) k_bx_cols(ConvBatch cb, int nt, int ntg, LimbMap map, const PrimeConst* pc, const uint2* tw,
                                                 const uint2* itw, unsigned long long* ts) {
    constexpr int LOGN = 16;
    __shared__ u32 sm[2][2048];
    // block -> (tile, target range, group): the four tiles of one 128-byte column segment on one
    // XCD (blocks are dealt round-robin over the 8 XCDs), so a source line is fetched into that
    // XCD's L2 once for its four tiles and every target range of the group
    const int b = blockIdx.x;
    const int tile = 4 * (b & 7) + ((b >> 3) & 3), rest = b >> 5, tg = rest % ntg, z = rest / ntg;
    const int hz = cb.h[z], sp = cb.split[z], skip0 = cb.skip0[z];
    const int tper = (nt + ntg - 1) / ntg, t0 = tg * tper, t1 = min(nt, t0 + tper);
    if (t0 >= t1 || (t0 >= skip0 && t1 <= skip0 + hz)) return;  // nothing to convert (block-uniform)
    ts_begin(ts);
    const int c = threadIdx.x & 7, p = threadIdx.x >> 3, col = tile * 8 + c;
    int buf = 0;
    u32 y[HM][8];
    u32 nx[8];
    bx_load(nx, cb.src[z], p, col);
    bx_sources<0, HM>(y, nx, cb, z, hz, sp, pc, itw, sm, buf, p, c, col);
    // u = round(sum y_i / q_i), k_base_convert's 32.32 fixed point in its source order (summed
    // here, after the transforms, so the sums are not live through them)
    u32 mu[HM];
#pragma unroll
    for (int i = 0; i < HM; ++i) mu[i] = i < hz ? pc[(sp > 0 && i >= sp) ? cb.d1[z] + (i - sp) : cb.d0[z] + i].mu : 0u;
    u32 u[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        u64 f = 0;
#pragma unroll
        for (int i = 0; i < HM; ++i) f += ((u64)y[i][e] * mu[i]) >> 29;
        u[e] = (u32)((f + (1ull << 31)) >> 32);
    }
    u32* dst = cb.dst[z];
    for (int t = t0; t < t1; ++t) {
        if (t >= skip0 && t < skip0 + hz) continue;  // the ModUp digit's own limbs (block-uniform)
        const int prime = map.prime(t);
        const PrimeConst P = pc[prime];
        const u32 q = P.q, q2 = 2 * q, negq = cb.negq[z][t];
        u32 wt[HM];
#pragma unroll
        for (int i = 0; i < HM; ++i) wt[i] = i < hz ? cb.tab[z][2 * ((size_t)i * nt + t)] : 0u;
        u32 x[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            u64 acc = (u64)u[e] * negq;
#pragma unroll
            for (int i = 0; i < HM; ++i) {
                if (i == 8) acc = fold64(acc, q, P.r32);  // (a zero-weight tail may add this fold: same residue)
                acc += (u64)y[i][e] * wt[i];
            }
            x[e] = reduce64(acc, q, P.mu, P.r32);
        }
        const uint2* w = tw + ((size_t)prime << LOGN);
        bx_fwd<kBxA, 0, 4>(x, w, p, q2, q);
        bx_fwd<kBxA, 1, 2>(x, w, p, q2, q);
        bx_fwd<kBxA, 2, 1>(x, w, p, q2, q);
        bx_xchg<kBxA, kBxBf>(x, sm[buf], p, c);
        buf ^= 1;
        bx_fwd<kBxBf, 3, 4>(x, w, p, q2, q);
        bx_fwd<kBxBf, 4, 2>(x, w, p, q2, q);
        bx_fwd<kBxBf, 5, 1>(x, w, p, q2, q);
        bx_xchg<kBxBf, kBxC>(x, sm[buf], p, c);
        buf ^= 1;
        bx_fwd<kBxC, 6, 2>(x, w, p, q2, q);
        bx_fwd<kBxC, 7, 1>(x, w, p, q2, q);
        u32* d = dst + ((size_t)t << LOGN);
#pragma unroll
        for (int e = 0; e < 8; ++e) d[(size_t)bx_row<kBxC>(p, e) * 256 + col] = x[e];
    }
    ts_end(ts);
}
template <int HM>
void bx_go(hipStream_t st, const DevTables& Tb, const ConvBatch& cb, int nt, int ntg, LimbMap map, double bytes) {
    prof_launch_tsw(KID_BASE_CONVERT, bytes, 0.0, k_bx_cols<HM>, dim3(32 * ntg * cb.n), dim3(256), 0, st, cb, nt, ntg, map, Tb.pc, Tb.tw, Tb.itw);
}

}  // namespace

int ntt_conv_fused_mask(const DevTables& T) {
    static const int m = [] {
        const char* e = std::getenv("AESFHE_FUSED_CONV");
        return e ? std::atoi(e) : 0;
    }();
    return T.logn == 16 ? m : 0;
}
void launch_ntt_fwd_conv(hipStream_t st, const DevTables& T, u32* dst, const ConvBatch& cb, int rows, RowMap rm, LimbMap map) {
    if (rows <= 0) return;
    int io_rows = rows;
    if (rm.skip_alpha > 0)
        for (int y = 0; y < rows; ++y) {
            const int g = y / rm.cnt, i = y - g * rm.cnt;
            if (i < rm.skip_nl && i / rm.skip_alpha == (rm.skip_groups > 0 ? g % rm.skip_groups : g)) --io_rows;
        }
    ntt_fwd_conv_t<kPlain>(st, T, dst, cb, rows, io_rows, rm, map, NttAux{});
}
void launch_ntt_finish_conv(hipStream_t st, const DevTables& T, u32* out, u32* conv, const ConvBatch& cb, const u32* cur, int cur_stride,
                            const u32* qinv, const u32* add0, const u32* add1, int npoly, int nt, size_t add_mstride, u32* const* outm) {
    NttAux aux{};
    aux.cur = cur, aux.out = out, aux.qinv = qinv, aux.cur_stride = cur_stride, aux.out_stride = nt, aux.add0 = add0, aux.add1 = add1;
    aux.add_mstride = add_mstride;
    if (outm) {
        if (npoly > 16 || npoly % 2) throw std::runtime_error("launch_ntt_finish: per-member outputs for at most 8 two-polynomial members");
        for (int m = 0; m < npoly / 2; ++m) aux.outm[m] = outm[m];
    }
    ntt_fwd_conv_t<kFinish>(st, T, conv, cb, npoly * nt, npoly * nt, rows_dense(nt), LimbMap{1 << 30, 0, 0}, aux);
}

template <int M1, int M2>
void ntt_fwd_dispatch(hipStream_t st, const DevTables& T, u32* dst, const u32* src, int rows, int io_rows, RowMap rm, LimbMap map,
                      const NttAux& aux) {
    if (rows <= 0) return;
    switch (T.logn) {
        case 13: ntt_fwd_t<5, M1, M2>(st, T, dst, src, rows, io_rows, rm, map, aux); break;
        case 14: ntt_fwd_t<6, M1, M2>(st, T, dst, src, rows, io_rows, rm, map, aux); break;
        case 15: ntt_fwd_t<7, M1, M2>(st, T, dst, src, rows, io_rows, rm, map, aux); break;
        case 16: ntt_fwd_t<8, M1, M2>(st, T, dst, src, rows, io_rows, rm, map, aux); break;
        default: break;  // HostParams::build rejects other ring sizes
    }
}

void launch_ntt_fwd(hipStream_t st, const DevTables& T, u32* dst, const u32* src, int rows, RowMap rm, LimbMap map) {
    int io_rows = rows;
    if (rm.skip_alpha > 0)
        for (int y = 0; y < rows; ++y) {
            const int g = y / rm.cnt, i = y - g * rm.cnt;
            if (i < rm.skip_nl && i / rm.skip_alpha == (rm.skip_groups > 0 ? g % rm.skip_groups : g)) --io_rows;
        }
    ntt_fwd_dispatch<kPlain, kPlain>(st, T, dst, src, rows, io_rows, rm, map, NttAux{});
}
void launch_rescale_ntt(hipStream_t st, const DevTables& T, u32* out, const u32* cur, const u32* last, u32* v, const u32* qinv,
                        int npoly, int nt, int nl_in, u32 q_last, const u32* cmul) {
    NttAux aux{};
    aux.cur = cur, aux.out = out, aux.qinv = qinv, aux.cur_stride = nl_in, aux.out_stride = nt, aux.q_last = q_last;
    aux.cmul = cmul;
    const RowMap rm{nt, 1, nt, 0, 0};
    ntt_fwd_dispatch<kSpread, kFinish>(st, T, v, last, npoly * nt, npoly * nt, rm, LimbMap{1 << 30, 0, 0}, aux);
}
void launch_rescale2_ntt(hipStream_t st, const DevTables& T, u32* out, const u32* cur, const u32* last, u32* v, const u32* qinv,
                         int npoly, int nt, int nl_in, u32 qa, u32 qb, u32 qa_inv, u32 qa_inv_p, const u32* cmul) {
    NttAux aux{};
    aux.cur = cur, aux.out = out, aux.qinv = qinv, aux.cur_stride = nl_in, aux.out_stride = nt;
    aux.cmul = cmul;
    aux.q_last = qa, aux.q_last2 = qb, aux.qa_inv = qa_inv, aux.qa_inv_p = qa_inv_p;
    const RowMap rm{nt, 2, nt, 0, 0};
    ntt_fwd_dispatch<kSpread2, kFinish>(st, T, v, last, npoly * nt, npoly * nt, rm, LimbMap{1 << 30, 0, 0}, aux);
}
void launch_ntt_finish(hipStream_t st, const DevTables& T, u32* out, u32* conv, const u32* cur, int cur_stride, const u32* qinv,
                       const u32* add0, const u32* add1, int npoly, int nt, size_t add_mstride, u32* const* outm, unsigned dbl,
                       const u32* const* cst, bool add_rev) {
    NttAux aux{};
    aux.cur = cur, aux.out = out, aux.qinv = qinv, aux.cur_stride = cur_stride, aux.out_stride = nt, aux.add0 = add0, aux.add1 = add1;
    aux.add_mstride = add_mstride;
    if (outm) {
        if (npoly > 16 || npoly % 2) throw std::runtime_error("launch_ntt_finish: per-member outputs for at most 8 two-polynomial members");
        for (int m = 0; m < npoly / 2; ++m) aux.outm[m] = outm[m];
    }
    if (dbl || cst) {
        if (npoly > 16 || npoly % 2) throw std::runtime_error("launch_ntt_finish: the 2 r + c epilogue for at most 8 two-polynomial members");
        aux.dbl = dbl;
        if (cst)
            for (int m = 0; m < npoly / 2; ++m) aux.cst[m] = cst[m];
    }
    aux.add_rev = add_rev ? 1 : 0;
    ntt_fwd_dispatch<kPlain, kFinish>(st, T, conv, conv, npoly * nt, npoly * nt, rows_dense(nt), LimbMap{1 << 30, 0, 0}, aux);
}
void launch_ntt_inv(hipStream_t st, const DevTables& T, u32* dst, const u32* src, int rows, RowMap rm, LimbMap map, const u32* post) {
    if (rows <= 0) return;
    switch (T.logn) {
        case 13: ntt_inv_t<5>(st, T, dst, src, rows, rm, map, post); break;
        case 14: ntt_inv_t<6>(st, T, dst, src, rows, rm, map, post); break;
        case 15: ntt_inv_t<7>(st, T, dst, src, rows, rm, map, post); break;
        case 16: ntt_inv_t<8>(st, T, dst, src, rows, rm, map, post); break;
        default: break;
    }
}
void launch_ntt_inv_prod(hipStream_t st, const DevTables& T, u32* dst, const TensorPtrs& tp, int rows, RowMap rm, LimbMap map, const u32* post) {
    if (rows <= 0) return;
    switch (T.logn) {
        case 13: ntt_inv_t<5>(st, T, dst, nullptr, rows, rm, map, post, &tp); break;
        case 14: ntt_inv_t<6>(st, T, dst, nullptr, rows, rm, map, post, &tp); break;
        case 15: ntt_inv_t<7>(st, T, dst, nullptr, rows, rm, map, post, &tp); break;
        case 16: ntt_inv_t<8>(st, T, dst, nullptr, rows, rm, map, post, &tp); break;
        default: break;
    }
}
void launch_ntt_inv_rev(hipStream_t st, const DevTables& T, u32* dst, const u32* src, int rows, RowMap rm, LimbMap map, const u32* post) {
    if (rows <= 0) return;
    switch (T.logn) {
        case 13: ntt_inv_t<5>(st, T, dst, src, rows, rm, map, post, nullptr, true); break;
        case 14: ntt_inv_t<6>(st, T, dst, src, rows, rm, map, post, nullptr, true); break;
        case 15: ntt_inv_t<7>(st, T, dst, src, rows, rm, map, post, nullptr, true); break;
        case 16: ntt_inv_t<8>(st, T, dst, src, rows, rm, map, post, nullptr, true); break;
        default: break;
    }
}
void launch_ntt_ki(hipStream_t st, const DevTables& T, const KiArgs& a, LimbMap map) {
    if (a.nb < 1 || a.nb > kMaxKsBatch || a.nsrc < 1 || a.nsrc > kMaxKiSrc || a.kept < 0 || a.kept > a.ne)
        throw std::runtime_error("launch_ntt_ki: bad member / source / row counts");
    if (a.fold.rev_d && a.fold.ta[0]) throw std::runtime_error("launch_ntt_ki: reversed d needs no tensor fold");
    if (a.kept < a.ne && !a.ys) throw std::runtime_error("launch_ntt_ki: converted rows need a ys buffer");
    switch (T.logn) {
        case 13: ki_launch<5>(st, T, a, map); break;
        case 14: ki_launch<6>(st, T, a, map); break;
        case 15: ki_launch<7>(st, T, a, map); break;
        case 16: ki_launch<8>(st, T, a, map); break;
        default: break;
    }
}
void launch_ntt_fwd_cols(hipStream_t st, const DevTables& T, u32* dst, const u32* src, int rows, RowMap rm, LimbMap map) {
    if (rows <= 0) return;
    int io_rows = rows;
    if (rm.skip_alpha > 0)
        for (int y = 0; y < rows; ++y) {
            const int g = y / rm.cnt, i = y - g * rm.cnt;
            if (i < rm.skip_nl && i / rm.skip_alpha == (rm.skip_groups > 0 ? g % rm.skip_groups : g)) --io_rows;
        }
    switch (T.logn) {
        case 13: ntt_fwd_cols_t<5>(st, T, dst, src, rows, io_rows, rm, map); break;
        case 14: ntt_fwd_cols_t<6>(st, T, dst, src, rows, io_rows, rm, map); break;
        case 15: ntt_fwd_cols_t<7>(st, T, dst, src, rows, io_rows, rm, map); break;
        case 16: ntt_fwd_cols_t<8>(st, T, dst, src, rows, io_rows, rm, map); break;
        default: break;
    }
}
void launch_ntt_inv_cols(hipStream_t st, const DevTables& T, u32* data, int rows, RowMap rm, LimbMap map, const u32* post) {
    if (rows <= 0) return;
    switch (T.logn) {
        case 13: ntt_inv_cols_t<5>(st, T, data, rows, rm, map, post); break;
        case 14: ntt_inv_cols_t<6>(st, T, data, rows, rm, map, post); break;
        case 15: ntt_inv_cols_t<7>(st, T, data, rows, rm, map, post); break;
        case 16: ntt_inv_cols_t<8>(st, T, data, rows, rm, map, post); break;
        default: break;
    }
}

// k_bx_cols exists for N = 2^16 (the engine's AESFHE_BX_COLS switch decides where it runs)
int bx_cols_on(const DevTables& T) { return T.logn == 16 ? 1 : 0; }
void launch_bx_cols(hipStream_t st, const DevTables& T, const ConvBatch& cb, int nt, LimbMap map) {
    if (T.logn != 16) throw std::runtime_error("launch_bx_cols: N = 2^16 only");
    if (cb.n < 1 || cb.n > kMaxConvGroups) throw std::runtime_error("launch_bx_cols: bad group count");
    int hmax = 0, eff = 0;
    double rows = 0.0;
    for (int z = 0; z < cb.n; ++z) {
        if (cb.h[z] < 1 || cb.h[z] > kMaxConvH) throw std::runtime_error("launch_bx_cols: source count out of range");
        if (!cb.src[z] || !cb.dst[z] || !cb.tab[z] || !cb.qhinv[z] || !cb.negq[z]) throw std::runtime_error("launch_bx_cols: missing operand");
        hmax = std::max(hmax, cb.h[z]);
        int own = 0;
        for (int t = 0; t < nt; ++t) own += t >= cb.skip0[z] && t < cb.skip0[z] + cb.h[z];
        eff = std::max(eff, nt - own);
        rows += cb.h[z] + (nt - own);
    }
    // target ranges per group: enough blocks to cover the chip (AESFHE_BX_BLOCKS, default 256), at
    // least 3 targets per block to amortise its H inverse transforms
    static const int want = [] {
        const char* e = std::getenv("AESFHE_BX_BLOCKS");
        return e ? std::max(32, std::atoi(e)) : 256;
    }();
    int ntg = (want + 32 * cb.n - 1) / (32 * cb.n);
    ntg = std::max(1, std::min(ntg, std::max(1, eff / 3)));
    const double bytes = rows * 4.0 * 65536.0;
    if (hmax <= 4) bx_go<4>(st, T, cb, nt, ntg, map, bytes);
    else if (hmax <= 8) bx_go<8>(st, T, cb, nt, ntg, map, bytes);
    else if (hmax <= 10) bx_go<10>(st, T, cb, nt, ntg, map, bytes);
    else if (hmax <= 11) bx_go<11>(st, T, cb, nt, ntg, map, bytes);
    else if (hmax <= 12) bx_go<12>(st, T, cb, nt, ntg, map, bytes);
    else throw std::runtime_error("launch_bx_cols: more than 12 sources per group (the residues would not fit in VGPRs)");
}
// the inverse NTT's row pass alone (k_bx_cols then runs the column pass): plain, product (tp) or
// reversed (rev) input, the launches ntt_inv_t issues for that pass (N = 2^16)
void launch_ntt_inv_rows(hipStream_t st, const DevTables& T, u32* dst, const u32* src, int rows, RowMap rm, LimbMap map,
                         const TensorPtrs* tp, bool rev) {
    if (rows <= 0) return;
    if (T.logn != 16) throw std::runtime_error("launch_ntt_inv_rows: N = 2^16 only");
    constexpr int LOGR1 = 8, R1 = 1 << LOGR1;
    rm.nrows = rows;
    const int groups = (rows + rm.cnt - 1) / rm.cnt;
    const double io = (tp ? 3.0 : 2.0) * 4.0 * rows * (256.0 * R1), bfly = (double)rows * 128.0 * R1 * 8.0;
    if (small_launch(rows)) {
        ntt2_inv_launch<LOGR1, kThreads / 2>(st, T, dst, src, rm, map, groups, io, bfly, tp, rev);
        return;
    }
    switch (p2_nt_rows(true, rows)) {
        case 128: ntt2_inv_launch<LOGR1, 128>(st, T, dst, src, rm, map, groups, io, bfly, tp, rev); break;
        case 256: ntt2_inv_launch<LOGR1, 256>(st, T, dst, src, rm, map, groups, io, bfly, tp, rev); break;
        default: ntt2_inv_launch<LOGR1, kThreads>(st, T, dst, src, rm, map, groups, io, bfly, tp, rev); break;
    }
}
// the forward NTT's row pass alone, in place (after k_bx_cols), with the RowMap's skips
void launch_ntt_fwd_rows(hipStream_t st, const DevTables& T, u32* data, int rows, RowMap rm, LimbMap map) {
    if (rows <= 0) return;
    if (T.logn != 16) throw std::runtime_error("launch_ntt_fwd_rows: N = 2^16 only");
    int io_rows = rows;
    if (rm.skip_alpha > 0)
        for (int y = 0; y < rows; ++y) {
            const int g = y / rm.cnt, i = y - g * rm.cnt;
            if (i < rm.skip_nl && i / rm.skip_alpha == (rm.skip_groups > 0 ? g % rm.skip_groups : g)) --io_rows;
        }
    constexpr int LOGR1 = 8, R1 = 1 << LOGR1;
    rm.nrows = rows;
    const int groups = (rows + rm.cnt - 1) / rm.cnt;
    ntt2_fwd_select<LOGR1, kPlain>(st, T, data, rm, map, groups, 2.0 * io_rows * 4.0 * 256.0 * R1, (double)io_rows * 128.0 * R1 * 8.0, NttAux{});
}
// launch_ntt_finish's row pass alone (its column pass ran inside k_bx_cols)
void launch_ntt_finish_rows(hipStream_t st, const DevTables& T, u32* out, u32* conv, const u32* cur, int cur_stride, const u32* qinv,
                            const u32* add0, const u32* add1, int npoly, int nt, size_t add_mstride, u32* const* outm, bool add_rev,
                            unsigned dbl, const u32* const* cst) {
    if (T.logn != 16) throw std::runtime_error("launch_ntt_finish_rows: N = 2^16 only");
    NttAux aux{};
    aux.cur = cur, aux.out = out, aux.qinv = qinv, aux.cur_stride = cur_stride, aux.out_stride = nt, aux.add0 = add0, aux.add1 = add1;
    aux.add_mstride = add_mstride;
    if (outm) {
        if (npoly > 16 || npoly % 2) throw std::runtime_error("launch_ntt_finish: per-member outputs for at most 8 two-polynomial members");
        for (int m = 0; m < npoly / 2; ++m) aux.outm[m] = outm[m];
    }
    if (dbl || cst) {
        if (npoly > 16 || npoly % 2) throw std::runtime_error("launch_ntt_finish: the 2 r + c epilogue for at most 8 two-polynomial members");
        aux.dbl = dbl;
        if (cst)
            for (int m = 0; m < npoly / 2; ++m) aux.cst[m] = cst[m];
    }
    aux.add_rev = add_rev ? 1 : 0;
    constexpr int LOGR1 = 8, R1 = 1 << LOGR1;
    RowMap rm = rows_dense(nt);
    const int rows = npoly * nt;
    rm.nrows = rows;
    const double io2 = (3.0 + (add0 ? 0.5 : 0.0) + (add1 ? 0.5 : 0.0)) * rows * 4.0 * 256.0 * R1;
    ntt2_fwd_select<LOGR1, kFinish>(st, T, conv, rm, LimbMap{1 << 30, 0, 0}, npoly, io2, (double)rows * 128.0 * R1 * 8.0, aux);
}
void launch_ntt_fwd(hipStream_t st, const DevTables& T, u32* data, int rows, int nl, LimbMap map) {
    launch_ntt_fwd(st, T, data, data, rows, rows_dense(nl), map);
}
void launch_ntt_inv(hipStream_t st, const DevTables& T, u32* data, int rows, int nl, LimbMap map) {
    launch_ntt_inv(st, T, data, data, rows, rows_dense(nl), map);
}
