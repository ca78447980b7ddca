// kernels.h -- launch wrappers for the CDNA4 kernels (kernels.hip).
//
// RNS tensors are row-major [rows][N] u32 with rows = npoly * nl; row r lives modulo
// prime map.prime(r % nl).  All wrappers are asynchronous on `st`.
#pragma once
#include <vector>

#include "common.h"

// --- live kernel timing (HIP events on the launch stream) ----------------------------
// Kernel ids for per-kernel accounting; bytes are ALGORITHMIC bytes of one launch
// (every input word read once, every output word written once).
enum KernelId {
    KID_NTT_COLS_FWD, KID_NTT_ROWS_FWD, KID_NTT_ROWS_INV, KID_NTT_COLS_INV, KID_BASE_CONVERT, KID_KEY_INNER,
    KID_MODDOWN, KID_TENSOR, KID_RESCALE, KID_AUTOMORPH, KID_ELEMENTWISE, KID_SAMPLE, KID_N
};
struct KernelProfiler {
    unsigned mask = 0;  // bit k enables event timing of KernelId k
    struct Rec {
        hipEvent_t a, b;
        int kid;
        double bytes;
    };
    std::vector<Rec> recs;
    std::vector<hipEvent_t> pool;
    double ms[KID_N] = {}, bytes[KID_N] = {};
    unsigned long long launches[KID_N] = {};
    hipEvent_t get();
    void flush();   // waits for recorded events and folds them into the totals
    void reset();
};
// the profiler of the engine currently issuing launches (set per API call)
void prof_set(KernelProfiler* p);

struct DevTables {
    const PrimeConst* pc = nullptr;  // [n_tot]
    const u32* psi = nullptr;        // [n_tot][N]  psi^{bitrev(k)}
    const u32* psip = nullptr;       //             Shoup companions
    const u32* ipsi = nullptr;       // [n_tot][N]  psi^{-bitrev(k)}
    const u32* ipsip = nullptr;
    int logn = 16;
};

// --- number-theoretic transforms -------------------------------------------------
void launch_ntt_fwd(hipStream_t st, const DevTables& T, u32* data, int rows, int nl, LimbMap map);
void launch_ntt_inv(hipStream_t st, const DevTables& T, u32* data, int rows, int nl, LimbMap map);

// --- element-wise ------------------------------------------------------------------
void launch_add(hipStream_t st, const DevTables& T, u32* out, const u32* a, const u32* b, int rows, int nl, LimbMap map);
void launch_sub(hipStream_t st, const DevTables& T, u32* out, const u32* a, const u32* b, int rows, int nl, LimbMap map);
void launch_neg(hipStream_t st, const DevTables& T, u32* out, const u32* a, int rows, int nl, LimbMap map);
// out = (a0 b0, a0 b1 + a1 b0, a1 b1); a, b: 2 x nl rows; out: 3 x nl rows
void launch_tensor(hipStream_t st, const DevTables& T, u32* out, const u32* a, const u32* b, int nl, LimbMap map);
// out = in * pt (pt: nl rows), npoly polys
void launch_mul_poly(hipStream_t st, const DevTables& T, u32* out, const u32* in, const u32* pt, int npoly, int nl, LimbMap map);
// out = a + b*c  (b, c: rows; used for decryption and encryption)
void launch_fma_poly(hipStream_t st, const DevTables& T, u32* out, const u32* a, const u32* b, const u32* c, int rows, int nl, LimbMap map);
// out[row][k] = in[row][k] * (k < N/2 ? clo[l] : chi[l]) with l = row % nl (Shoup pairs in cst)
// cst layout: [nl][4] = {clo, clo', chi, chi'}
void launch_mul_const_half(hipStream_t st, const DevTables& T, u32* out, const u32* in, const u32* cst, int rows, int nl, LimbMap map);
// out[row][k] = in[row][k] + (k < N/2 ? alo[l] : ahi[l]); cst layout [nl][2]
void launch_add_const_half(hipStream_t st, const DevTables& T, u32* out, const u32* in, const u32* cst, int rows, int nl, LimbMap map);
// X -> X^g in the NTT domain (bit-reversed evaluation order)
void launch_automorph(hipStream_t st, const DevTables& T, u32* out, const u32* in, u64 g, int rows);

// --- rescale -------------------------------------------------------------------------
// last: npoly rows (coefficient form, prime q_last); writes v[p][t] = centred(last) mod q_t
void launch_rescale_spread(hipStream_t st, const DevTables& T, u32* v, const u32* last, int npoly, int nt, u32 q_last);
// out[p][t] = (x[p][t] - v[p][t]) * qinv_t ; x has nl_in rows per poly, out/v have nt rows per poly
void launch_rescale_finish(hipStream_t st, const DevTables& T, u32* out, const u32* x, const u32* v, const u32* qinv, int npoly, int nt, int nl_in);

// --- key switching -----------------------------------------------------------------
// digit coefficient rows x[i] (i < h, primes d0 + i) -> ext rows for all targets of
// map (nt rows), skipping rows [skip0, skip0 + h) which are copied from src_ntt.
// tab: [h][nt] Shoup pairs of (qhat_i mod t); qhinv: [h] Shoup pairs of qhat_i^{-1} mod q_i;
// negq: [nt] values of (-Q mod t), Q = prod of the h source primes (centred conversion)
void launch_base_convert(hipStream_t st, const DevTables& T, u32* ext, const u32* x, int h, int d0, int nt, LimbMap map,
                         int skip0, const u32* tab, const u32* qhinv, const u32* negq);
// acc[0|1][x] = sum_j ext[j][x] * key[j][b|a][krow(x)]; ext: [nd][ne][N]; key: [dnum][2][nkey][N]
void launch_key_inner(hipStream_t st, const DevTables& T, u32* acc, const u32* ext, const u32* key, int nd, int ne, int nl,
                      int nkey, int nks, LimbMap map);
// out[p][t] = (acc[p][t] - conv[p][t]) * Pinv_t (+ add0[t] for p = 0, + add1[t] for p = 1; nullable)
void launch_moddown_finish(hipStream_t st, const DevTables& T, u32* out, const u32* acc, const u32* conv, const u32* pinv,
                           const u32* add0, const u32* add1, int nl, int ne);

// --- sampling --------------------------------------------------------
// kind: 0 ternary, 1 centred binomial (eta = 21); writes value mod prime into nl rows
void launch_sample_small(hipStream_t st, const DevTables& T, u32* out, int nl, LimbMap map, u64 seed, u64 stream, int kind);
// uniform residues: row l gets prng(seed, stream, prime(l) * N + k) mod q
void launch_sample_uniform(hipStream_t st, const DevTables& T, u32* out, int nl, LimbMap map, u64 seed, u64 stream);
// b = -a*s + e (+ gadget*s' on rows with flag) : used by key generation
void launch_keygen_combine(hipStream_t st, const DevTables& T, u32* b, const u32* a, const u32* s, const u32* e, const u32* sp,
                           const u32* gadget, int nl, LimbMap map, int gadget_lo, int gadget_hi);
// out = a*a (dyadic square)
void launch_square(hipStream_t st, const DevTables& T, u32* out, const u32* a, int rows, int nl, LimbMap map);
