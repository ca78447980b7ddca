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
    KID_MODDOWN, KID_TENSOR, KID_RESCALE, KID_AUTOMORPH, KID_ELEMENTWISE, KID_SAMPLE, KID_LIN_MAC, KID_N
};
struct KernelProfiler {
    unsigned mask = 0;  // bit k enables event timing of KernelId k
    unsigned every = 1; // time one launch in `every` of an enabled kernel (live sample)
    unsigned long long seen[KID_N] = {};
    struct Rec {
        hipEvent_t a, b;
        int kid;
        double bytes, work;
    };
    std::vector<Rec> recs;
    std::vector<hipEvent_t> pool;
    double ms[KID_N] = {}, bytes[KID_N] = {};
    double work[KID_N] = {};  // NTT kernels: radix-2 butterflies of the timed launches (VALU roofline)
    unsigned long long launches[KID_N] = {};
    hipEvent_t get();
    void flush();   // waits for recorded events and clock slots and folds them into the totals
    void reset();
    // In-kernel clock (s_memrealtime, 100 MHz) for the NTT, base-conversion and key-switch
    // kernels: a timed launch gets a slot {earliest start, latest end} over a sample of its
    // blocks (launch.h ts_begin / ts_end); it agrees with rocprofv3 --kernel-trace averages of
    // the same launches.  Dispatch-stamped event pairs (hipExtLaunchKernelGGL; the element-wise
    // kernels, or every kernel with AESFHE_PROF_EVENTS=1) read ~3 us longer per launch than
    // rocprofv3 does: the event's completion signal adds its own end-of-kernel release.
    // A slot is one record of kTsRec words: kTsSub start lines holding ~(earliest start)
    // (atomicMax of ~t, so a zeroed line is "unset"), then kTsSub end lines, each word on its own
    // 128-byte line (a block stamps line (block id mod kTsSub): the atomics of a launch's first
    // and last waves spread over 8 lines instead of queueing on one address).
    static constexpr int kTsSlots = 1 << 14, kTsSub = 8, kTsLine = 16, kTsRec = kTsLine * 2 * kTsSub;
    unsigned long long* d_ts = nullptr;  // [kTsSlots][kTsRec]
    int ts_next = 0;
    struct TsRec {
        int slot, kid;
        double bytes, work;
        bool count;  // a sampled launch of its own kid (span accounted); false: stamped only as a successor
        int prev;    // slot of the sampled launch issued right before it (-1: none): the boundary gap
    };
    std::vector<TsRec> ts_recs;
    unsigned long long* ts_slot(int kid, double bytes, double work = 0.0, bool count = true, int prev = -1);
    void ts_flush();
    // Dispatch-inclusive timing: the launch issued right after a sampled one
    // (next in the process's launch order, a clock-slot kernel) is stamped too, and the gap
    // start(next) - end(sampled) -- the sampled kernel's drain plus the next one's dispatch ramp,
    // the time rocprofv3's durations add to the in-kernel span -- is accounted to the NEXT
    // launch's kid: a kid's dispatch-inclusive average = its span average + its gap average.
    int pend_slot = -1;
    unsigned long long pend_idx = 0;
    hipStream_t pend_stream = nullptr;  // a gap pairs two launches of ONE stream only
    double gap_ms[KID_N] = {};
    unsigned long long gap_n[KID_N] = {};
};
// the profiler of the engine currently issuing launches (set per API call)
void prof_set(KernelProfiler* p);

struct DevTables {
    const PrimeConst* pc = nullptr;  // [n_tot]
    const uint2* tw = nullptr;       // [n_tot][N]  {-psi^{bitrev(k)} mod 2^32, Shoup companion of psi^{bitrev(k)}}: one 8-byte load per twiddle
    const uint2* itw = nullptr;      // [n_tot][N]  {psi^{-bitrev(k)}, Shoup companion}
    // inverse pass 2, stages 5..7 as twiddle = row factor x shared factor (ntt.hip k_ntt2_inv):
    const uint2* irow = nullptr;     // [n_tot][R1][4]  {psi^{-2^(7-s) (2 bitrev(R) + 1)}, companion} at [s - 5]
    const uint2* igam = nullptr;     // [n_tot][256]    {psi^{-(N / 2^s) bitrev_s(t)}, companion} at [2^s + t]
    int logn = 16;
};

// --- number-theoretic transforms (ntt.hip) ----------------------------------------------
// launch row y -> group g = y / cnt, index i = y % cnt (the limb index fed to LimbMap);
// source row = src_off + g * src_stride + i, destination row = dst_off + g * dst_stride + i
// skip_alpha > 0 (forward only): rows with i < skip_nl and i / skip_alpha == g are left
// untouched (ModUp: a digit's own limbs); skip_groups > 0: g taken mod skip_groups (the
// digits of several batched ciphertexts in one launch)
// launch row y = g * cnt + i: group g (grid z), row i of the group (grid y) -- a 3-D grid, so
// kernels read g and i from blockIdx without a (VALU-emulated) integer division
struct RowMap {
    int cnt, src_stride, dst_stride, src_off, dst_off;
    int skip_alpha = 0, skip_nl = 0, skip_groups = 0;
    int nrows = 0;  // launch rows (set by the launcher; the last group may be partial)
};
inline RowMap rows_dense(int nl) { return RowMap{nl, nl, nl, 0, 0}; }
// fused prologue / epilogue operands of the forward NTT (ntt.hip)
struct NttAux {
    const u32* cur = nullptr;  // finish: rows g * cur_stride + i
    u32* out = nullptr;        // finish: rows g * out_stride + i
    const u32* qinv = nullptr; // finish: [i] Shoup pairs
    const u32* add0 = nullptr; // finish: optional addend rows for group 0 / 1 (even / odd groups
    const u32* add1 = nullptr; //   when batched: group 2 m + p adds add_p + m * add_mstride words)
    size_t add_mstride = 0;
    int cur_stride = 0, out_stride = 0;
    u32 q_last = 0;            // spread: modulus of the source row
    u32 q_last2 = 0;           // spread2: second dropped prime (source rows a, b per group)
    u32 qa_inv = 0, qa_inv_p = 0;  // spread2: q_last^{-1} mod q_last2 (Shoup pair)
    // finish: member m's result (groups 2m, 2m + 1) written to outm[m] (2 polys x out_stride rows)
    // when set -- the members of a batched key switch straight into their own buffers, no unstack copy
    u32* outm[8] = {};
    // finish epilogue per member m (groups 2m, 2m + 1): (dbl >> m & 1) doubles the result, then
    // cst[m] (nullable, [limb][lo, hi] residues) is added to its polynomial 0 -- an EvalMod
    // 2 x^2 - c in the relinearisation's own launch, the residues of k_lincomb's (Engine::Affine)
    unsigned dbl = 0;
    const u32* cst[8] = {};
    // finish: add0 read in reversed coefficient order (word N - 1 - i for word i): the conjugation
    // X -> X^(2N-1) in this NTT order, its c0 addend permuted on load (Engine::galois_lazy)
    int add_rev = 0;
    // finish: cur read times cmul[i] (Shoup pairs per limb, nullable) -- a level conversion's
    // exact-scale constant folded into the limb drop that follows it (Engine::convert)
    const u32* cmul = nullptr;
};
// out-of-place (src may equal dst); supported ring sizes 2^13 .. 2^16
void launch_ntt_fwd(hipStream_t st, const DevTables& T, u32* dst, const u32* src, int rows, RowMap rm, LimbMap map);
// post (nullable): [rows per group] Shoup pairs, row i of every group also multiplied by post[i]
// (a base conversion's qhat^{-1}, folded into the inverse's N^{-1} scaling for k_ntt1_fwd_conv)
void launch_ntt_inv(hipStream_t st, const DevTables& T, u32* dst, const u32* src, int rows, RowMap rm, LimbMap map, const u32* post = nullptr);
// rescale by the prime q_last, fused: v[p][t] = centred(last[p]) mod q_t -> NTT ->
// out[p][t] = (cur[p][t] - v) * qinv_t;  cur has nl_in rows per poly, out/v have nt
// cmul (nullable): cur's limb t times cmul[t] (Shoup pairs) first
void launch_rescale_ntt(hipStream_t st, const DevTables& T, u32* out, const u32* cur, const u32* last, u32* v, const u32* qinv,
                        int npoly, int nt, int nl_in, u32 q_last, const u32* cmul = nullptr);
// rescale by the two primes qa = q_last, qb = q_last2 at once (double-prime levels):
// v = centred CRT of last[p][0..1] (mod qa qb) reduced mod q_t -> NTT ->
// out[p][t] = (cur[p][t] - v) * (qa qb)^{-1}_t;  last has 2 rows per poly
void launch_rescale2_ntt(hipStream_t st, const DevTables& T, u32* out, const u32* cur, const u32* last, u32* v, const u32* qinv,
                         int npoly, int nt, int nl_in, u32 qa, u32 qb, u32 qa_inv, u32 qa_inv_p, const u32* cmul = nullptr);
// NTT of conv (npoly x nt dense rows, destroyed) fused with
// out[p][t] = (cur[p * cur_stride + t] - NTT(conv)[p][t]) * qinv_t (+ add_p[t])   (ModDown)
// npoly = 2 nb for nb batched ciphertexts: group 2 m + p adds add_p + m add_mstride (words)
// dbl / cst: NttAux's per-member epilogue 2 r + c (cst: nb entries, nullable)
void launch_ntt_finish(hipStream_t st, const DevTables& T, u32* out, u32* conv, const u32* cur, int cur_stride, const u32* qinv,
                       const u32* add0, const u32* add1, int npoly, int nt, size_t add_mstride = 0, u32* const* outm = nullptr,
                       unsigned dbl = 0, const u32* const* cst = nullptr, bool add_rev = false);
// inverse NTT reading each source row in reversed coefficient order (the conjugation's permutation
// of the source fused into the load; otherwise launch_ntt_inv)
void launch_ntt_inv_rev(hipStream_t st, const DevTables& T, u32* dst, const u32* src, int rows, RowMap rm, LimbMap map, const u32* post = nullptr);
// in place on rows = npoly * nl dense rows
void launch_ntt_fwd(hipStream_t st, const DevTables& T, u32* data, int rows, int nl, LimbMap map);
void launch_ntt_inv(hipStream_t st, const DevTables& T, u32* data, int rows, int nl, LimbMap map);

// --- element-wise ------------------------------------------------------------------
void launch_add(hipStream_t st, const DevTables& T, u32* out, const u32* a, const u32* b, int rows, int nl, LimbMap map);
void launch_sub(hipStream_t st, const DevTables& T, u32* out, const u32* a, const u32* b, int rows, int nl, LimbMap map);
void launch_neg(hipStream_t st, const DevTables& T, u32* out, const u32* a, int rows, int nl, LimbMap map);
// out = in over `rows` rows of N words (device to device)
void launch_copy_rows(hipStream_t st, const DevTables& T, u32* out, const u32* in, size_t rows);
// n (<= kMaxMembers) independent copies of `rows` rows each: dst[m] = src[m] (one launch;
// stacking / unstacking batched ciphertexts)
constexpr int kMaxMembers = 8;
struct MemberPtrs {
    const u32* src[kMaxMembers] = {};
    u32* dst[kMaxMembers] = {};
};
void launch_copy_members(hipStream_t st, const DevTables& T, const MemberPtrs& mp, int n, int rows);
// out = (accumulate ? out : 0) + sum_{s < n} mp.src[s] over `rows` rows (limb = row, map)
void launch_add_members(hipStream_t st, const DevTables& T, u32* out, const MemberPtrs& mp, int n, int rows, LimbMap map, bool accumulate);
// tensor products of n independent pairs (a[m], b[m]: 2 x nl rows each) into one stacked
// [m][3][nl] output (mul_many)
struct TensorPtrs {
    const u32* a[kMaxMembers] = {};
    const u32* b[kMaxMembers] = {};
};
void launch_tensor_ptrs(hipStream_t st, const DevTables& T, u32* out, const TensorPtrs& tp, int n, int nl, LimbMap map);
// inverse NTT of the products a[g] (.) b[g] formed on load (limb i of group g at tp.a[g] + i N and
// tp.b[g] + i N, Barrett products as k_tensor_ptrs'): a relinearisation's third tensor polynomial
// transformed without being written (Engine::relin_rescale_tensor)
void launch_ntt_inv_prod(hipStream_t st, const DevTables& T, u32* dst, const TensorPtrs& tp, int rows, RowMap rm, LimbMap map,
                         const u32* post = nullptr);
// out = (a0 b0, a0 b1 + a1 b0, a1 b1); a, b: 2 x nl rows; out: 3 x nl rows
// nb > 1: nb ciphertexts stacked ([m][2][nl] in, [m][3][nl] out), one launch
void launch_tensor(hipStream_t st, const DevTables& T, u32* out, const u32* a, const u32* b, int nl, LimbMap map, int nb = 1);
// out = in * pt (pt: nl rows), npoly polys
void launch_mul_poly(hipStream_t st, const DevTables& T, u32* out, const u32* in, const u32* pt, int npoly, int nl, LimbMap map);
// out = sum_{i < n} in[i] (.) pt[i] (npoly polys of nl limbs each; pt[i]: nl limbs), n <= kMaxMembers
struct PtSumArgs {
    const u32* in[kMaxMembers] = {};
    const u32* pt[kMaxMembers] = {};
};
void launch_mul_poly_sum(hipStream_t st, const DevTables& T, u32* out, const PtSumArgs& a, int n, int npoly, int nl, LimbMap map);
// out = a + b*c  (b, c: rows; used for decryption and encryption)
void launch_fma_poly(hipStream_t st, const DevTables& T, u32* out, const u32* a, const u32* b, const u32* c, int rows, int nl, LimbMap map);
// per-limb constants passed BY VALUE as a kernel argument (1 KiB kernarg, read with scalar
// loads): no host->device copy per scalar operation
constexpr int kMaxConstLimbs = 64;
struct LimbConsts {
    u32 v[4 * kMaxConstLimbs];
};
// out[row][k] = in[row][k] * (k < N/2 ? clo[l] : chi[l]) with l = row % nl (Shoup pairs)
// layout: v[4 l .. 4 l + 3] = {clo, clo', chi, chi'}
// src_nl > 0: `in` holds polys of src_nl >= nl limbs (first nl read), e.g. a level drop
void launch_mul_const_half(hipStream_t st, const DevTables& T, u32* out, const u32* in, const LimbConsts& cst, int rows, int nl, LimbMap map,
                           int src_nl = 0);
// the same for n members read from separate ciphertexts (mp.src[m], polys of src_nl limbs) into one
// stacked output [m][rows] (mp.dst unused): the copy-and-scale step of n exact-scale level drops
void launch_mul_const_half_members(hipStream_t st, const DevTables& T, u32* out, const MemberPtrs& mp, int n, const LimbConsts& cst,
                                   int rows, int nl, LimbMap map, int src_nl);
// out = a +- b on the first `common` rows, then the longer operand alone (+-b when b is longer)
void launch_addsub_tail(hipStream_t st, const DevTables& T, u32* out, const u32* a, const u32* b, int common, int rows, bool a_longer,
                        bool sub, int nl, LimbMap map);
// out[row][k] = in[row][k] + (k < N/2 ? alo[l] : ahi[l]); layout v[2 l .. 2 l + 1]
void launch_add_const_half(hipStream_t st, const DevTables& T, u32* out, const u32* in, const LimbConsts& cst, int rows, int nl, LimbMap map);
// out = ka a + bsign b (b optional) + cadd on the rows of the first polynomial of every member
// (per polys per member); ka: Shoup pairs {lo, lo', hi, hi'} per limb, cadd: {lo, hi} per limb
void launch_lincomb(hipStream_t st, const DevTables& T, u32* out, const u32* a, const LimbConsts& ka, const u32* b, int bsign,
                    const LimbConsts* cadd, int per, int rows, int nl, LimbMap map);
// X -> X^g in the NTT domain (bit-reversed evaluation order)
void launch_automorph(hipStream_t st, const DevTables& T, u32* out, const u32* in, u64 g, int rows);

// --- rescale -------------------------------------------------------------------------
// last: npoly rows (coefficient form, prime q_last); writes v[p][t] = centred(last) mod q_t
void launch_rescale_spread(hipStream_t st, const DevTables& T, u32* v, const u32* last, int npoly, int nt, u32 q_last);
// ModRaise of coefficient-form polynomials over the two base limbs (q0, q1): src [npoly][2][N]
// -> v [npoly][nt][N], the centred CRT value mod primes 0 .. nt - 1
void launch_crt2_spread(hipStream_t st, const DevTables& T, u32* v, const u32* src, int npoly, int nt, u32 q0, u32 q1);

// --- key switching -----------------------------------------------------------------
// fast base conversion of several groups in one launch (ModUp: one group per digit,
// ModDown: one per polynomial).  Group g: h source coefficient rows (primes d0 ..
// d0 + h - 1) -> nt target rows of dst (primes map.prime(t)); targets
// [skip0, skip0 + h) are skipped (the digit's own limbs; 1 << 30 = none).
// tab: [h][nt] Shoup pairs of (qhat_i mod t); qhinv: [h] Shoup pairs of qhat_i^{-1} mod q_i;
// negq: [nt] values of (-Q mod t), Q = prod of the h source primes (centred conversion)
constexpr int kMaxConvGroups = 24;  // ModUp digits (or ModDown polys) x batched ciphertexts
constexpr int kMaxConvH = 16;
struct ConvBatch {
    int n = 0;
    int h[kMaxConvGroups] = {}, d0[kMaxConvGroups] = {}, skip0[kMaxConvGroups] = {};
    // split > 0: sources i >= split are primes d1 + (i - split) (ModDown fused with rescale:
    // the dropped Q limbs, then P)
    int split[kMaxConvGroups] = {}, d1[kMaxConvGroups] = {};
    const u32* src[kMaxConvGroups] = {};
    u32* dst[kMaxConvGroups] = {};
    const u32* tab[kMaxConvGroups] = {};
    const u32* qhinv[kMaxConvGroups] = {};
    const u32* negq[kMaxConvGroups] = {};
    // pre != 0: every group's sources are already times qhat_i^{-1} (folded into the N^{-1} scaling of
    // the INTT that made them: launch_ntt_inv's `post`), so k_base_convert does not multiply again
    int pre = 0;
};
void launch_base_convert(hipStream_t st, const DevTables& T, const ConvBatch& cb, int nt, LimbMap map);
// the base conversion fused into the forward NTT's first pass (ntt.hip k_ntt1_fwd_conv): the
// conversion of cb (sources already times qhat^{-1}: launch_ntt_inv's post) written as its NTT.
// Row group z of the RowMap is conversion group z (cb.dst unused).  ntt_conv_fused_mask: where it
// is used (N = 2^16 only): bit 0 the ModUps, bit 1 the ModDowns (AESFHE_FUSED_CONV, default 0: slower on this GPU)
int ntt_conv_fused_mask(const DevTables& T);
void launch_ntt_fwd_conv(hipStream_t st, const DevTables& T, u32* dst, const ConvBatch& cb, int rows, RowMap rm, LimbMap map);
// launch_ntt_finish with conv computed in the NTT's load from cb (the ModDown conversion)
void launch_ntt_finish_conv(hipStream_t st, const DevTables& T, u32* out, u32* conv, const ConvBatch& cb, const u32* cur, int cur_stride,
                            const u32* qinv, const u32* add0, const u32* add1, int npoly, int nt, size_t add_mstride = 0,
                            u32* const* outm = nullptr);
// acc[0|1][x] = sum_j e_j[x] * key[j][b|a][krow(x)] with e_j = ext[j] except on digit j's
// own limbs (x < nl, x / alpha == j) where e_j = d (the NTT-form input);
// ext: [nd][ne][N]; key: [dnum][2][nkey][N]
// g != 0: ext and d are read through the automorphism X -> X^g (hoisted rotation)
// nb > 1: nb ciphertexts' key switches with the SAME key in one launch (the key is read once
// per residue for all of them); member m uses ext + m ext_ms, d + m d_ms, acc + m acc_ms (words)
constexpr int kMaxKsBatch = 8;
// accum: acc += the inner product (giant steps summed in Q*P, one ModDown for all of them)
// fold (g == 0 only): acc[p][x] += gad_x add_p[x] on the Q rows x < nl (member m: add_p + m ms),
// gad = P mod q_x Shoup pairs -- the relinearised P (c0, c1) + acc before a ModDown that also
// divides by the dropped limbs
struct KsFold {
    const u32* add0 = nullptr;
    const u32* add1 = nullptr;
    size_t ms = 0;
    const u32* gad = nullptr;
    // tensor mode (ta[0] set): member m is the product of the 2-polynomial ciphertexts ta[m], tb[m]
    // (tnl limbs per polynomial), never materialised -- the fold's (c0, c1) and the own digit's
    // c2 rows are formed on load as k_tensor_ptrs forms them (add0 / add1 / d unused)
    const u32* ta[kMaxKsBatch] = {};
    const u32* tb[kMaxKsBatch] = {};
    int tnl = 0;
    // rev_d (g == 0): the own digit's rows of d read in reversed coefficient order (the conjugation)
    int rev_d = 0;
};
void launch_key_inner(hipStream_t st, const DevTables& T, u32* acc, const u32* ext, const u32* d, const u32* key, int nd, int ne, int nl,
                      int alpha, int nkey, int nks, LimbMap map, u64 g = 0, int nb = 1, size_t ext_ms = 0, size_t d_ms = 0,
                      size_t acc_ms = 0, KsFold fold = {}, bool accum = false);
// Fused key-switch core (ntt.hip k_ntt2_ki): the ModUp's forward row pass of every
// digit's extended rows (ext: the column pass's output, [member][nd][ne] rows), the key inner
// product (k_key_inner's arithmetic: fold / tensor / reversed own digit; up to 2 sources summed,
// each with its own key, ext and d) and, for the acc rows x >= kept, the row pass of the ModDown's
// inverse NTT into ys ([member][2][ys_rows], row x - kept); rows x < kept go to acc [member][2][ne].
// Identity Galois element only (a rotation's automorphism permutes across chunks).
// summed key-switch sources of one fused launch: the lazy conjugation's two (sigma(s), sigma(s)^2),
// or the rotated giant steps of a double-hoisted linear-transform group (each its own ModUp'd
// input and key), all accumulated in the same 64-bit sums before the one ModDown
constexpr int kMaxKiSrc = 8;
struct KiArgs {
    const u32* ext[kMaxKiSrc] = {};
    const u32* d[kMaxKiSrc] = {};
    const u32* key[kMaxKiSrc] = {};
    int nsrc = 1;
    int nd = 0, ne = 0, nl = 0, alpha = 1, nkey = 0, nks = 0;
    int kept = 0, ys_rows = 0, nb = 1;
    size_t ext_ms = 0, d_ms = 0, acc_ms = 0, ys_ms = 0;
    u32* acc = nullptr;
    u32* ys = nullptr;
    KsFold fold;
};
void launch_ntt_ki(hipStream_t st, const DevTables& T, const KiArgs& a, LimbMap map);
// the forward NTT's column pass alone (pass 1; the row pass then runs inside launch_ntt_ki)
void launch_ntt_fwd_cols(hipStream_t st, const DevTables& T, u32* dst, const u32* src, int rows, RowMap rm, LimbMap map);
// the inverse NTT's column pass alone, in place (its row pass ran inside launch_ntt_ki)
void launch_ntt_inv_cols(hipStream_t st, const DevTables& T, u32* data, int rows, RowMap rm, LimbMap map, const u32* post = nullptr);
// column-domain basis extension (ntt.hip k_bx_cols, N = 2^16): for every group z of cb, the inverse
// NTT's column pass of its h[z] source rows src[z] (row pass done), their conversion to the nt
// targets (k_base_convert's tables and arithmetic; targets in [skip0, skip0 + h) skipped) and the
// forward NTT's column pass of each target, written to dst[z] + t N.  bx_cols_on: the ring has it
int bx_cols_on(const DevTables& T);
void launch_bx_cols(hipStream_t st, const DevTables& T, const ConvBatch& cb, int nt, LimbMap map);
// single passes around it (N = 2^16): the inverse row pass (plain / product / reversed input), the
// forward row pass in place (RowMap skips honoured), launch_ntt_finish's row pass
void launch_ntt_inv_rows(hipStream_t st, const DevTables& T, u32* dst, const u32* src, int rows, RowMap rm, LimbMap map,
                         const TensorPtrs* tp = nullptr, bool rev = false);
void launch_ntt_fwd_rows(hipStream_t st, const DevTables& T, u32* data, int rows, RowMap rm, LimbMap map);
void launch_ntt_finish_rows(hipStream_t st, const DevTables& T, u32* out, u32* conv, const u32* cur, int cur_stride, const u32* qinv,
                            const u32* add0, const u32* add1, int npoly, int nt, size_t add_mstride = 0, u32* const* outm = nullptr,
                            bool add_rev = false, unsigned dbl = 0u, const u32* const* cst = nullptr);
// Heterogeneous batched key switch (Engine::ks_multi): member m of one launch
// reads its own key and Galois element.  acc_m [2][ne] (acc + m acc_ms) = sum_j e_j ⊙ key_m[j]
// with e_j = ext_{src_m}[j] (ext + src_m ext_ms), d_{src_m} (d + src_m d_ms) on digit j's own
// limbs, both read through X -> X^g_m (g_m = 0: identity).  Several members may share a source:
// the hoisted rotations of one ciphertext (one ModUp for all of them).
constexpr int kKsMulti = 16;
struct KsMultiArgs {
    const u32* key[kKsMulti] = {};
    u64 g[kKsMulti] = {};
    int src[kKsMulti] = {};
};
void launch_key_inner_multi(hipStream_t st, const DevTables& T, u32* acc, const u32* ext, const u32* d, const KsMultiArgs& ka, int nm,
                            int nsrc, int nd, int ne, int nl, int alpha, int nkey, int nks, LimbMap map, size_t ext_ms, size_t d_ms,
                            size_t acc_ms);
// acc_m [2][ne] (acc + m acc_ms) = sum_{i < J} sum_j e_j(g_i) ⊙ key_i[j]: J hoisted rotations of the
// same ModUp'ed ciphertext summed in Q*P in ONE launch (the bootstrap's radix-4 trace step, J = 3),
// e_j(g) = ext_m[j] / d_m on digit j's own limbs, read through X -> X^g; nb stacked members (grid z)
struct KsSumArgs {
    const u32* key[4] = {};
    u64 g[4] = {};
    int J = 0;
};
void launch_key_inner_sum(hipStream_t st, const DevTables& T, u32* acc, const u32* ext, const u32* d, const KsSumArgs& ka, int nb, int nd,
                          int ne, int nl, int alpha, int nkey, int nks, LimbMap map, size_t ext_ms, size_t d_ms, size_t acc_ms);
// out_m (rows rows, out + m ms) = in_m + sum_{i < J} in_m through X -> X^g_i (in + m ms), nb members
void launch_automorph_sum(hipStream_t st, const DevTables& T, u32* out, const u32* in, const KsSumArgs& ka, int nb, int rows, size_t ms,
                          LimbMap map);
// out + m out_ms (rows rows) = in_m through X -> X^g_m, m < n (one launch; g_m = 1: a copy)
struct AutoMulti {
    const u32* src[kKsMulti] = {};
    u64 g[kKsMulti] = {};
};
void launch_automorph_multi(hipStream_t st, const DevTables& T, u32* out, size_t out_ms, const AutoMulti& am, int n, int rows);
// out[p][t] = sum_j x_j[p][t] pt_j[t] over rows t < rows, polys p < npoly (x poly stride xs,
// out poly stride os, in words)
constexpr int kMacMax = 16;
struct MacTerms {
    const u32* x[kMacMax];
    const u32* pt[kMacMax];
    int n;
};
void launch_mac(hipStream_t st, const DevTables& T, u32* out, const MacTerms& m, size_t xs, size_t os, int rows, int npoly, LimbMap map);
// every giant step of one hoisted BSGS linear-transform group in ONE pass:
// row t < ne of the extended basis (Q limbs t < nl, then the P block), for each giant gg < G:
//   out0[gg] = sum_b a_b P[gg][b]        (t < nl; a_0 = c0, a_b = automorphed c0)
//   out1[gg] = c1 P[gg][0]               (t < nl, when out1[gg])
//   outp[gg] = sum_{b>=1} u_b P[gg][b]   (2 polys of ne rows; u_b = hoisted key inner products)
// Each input residue is read once for all giant steps (the per-giant k_mac re-read every
// rotated baby step and every diagonal twice).  Null pointers mark absent terms.
constexpr int kLinB = 16, kLinG = 5;
// nb > 1 batched ciphertexts share the diagonals: member m's a / c1 / out0 / out1 are at
// + m * q_ms words, its u / outp at + m * p_ms words
struct LinMacArgs {
    const u32* a[kLinB];
    const u32* u[kLinB];
    const u32* c1;
    const u32* pt[kLinG][kLinB];
    u32* out0[kLinG];
    u32* out1[kLinG];
    u32* outp[kLinG];
    int B, G;
    int nb = 1;
    size_t q_ms = 0, p_ms = 0;
    // gad (P mod q_t Shoup pairs): giant steps with outp fold P * (out0, out1) into outp's Q
    // rows instead of storing out0 / out1 (ModDown fused with the rescale)
    const u32* gad = nullptr;
    // gal[b] != 0: a[b] is read through X -> X^gal[b] (the baby step's automorphism of c0,
    // fused: no rotated copy of c0 is written)
    u64 gal[kLinB] = {};
    // key[b] set: baby step b's key inner product is computed in the kernel from the hoisted
    // ModUp (ks_ext: [member][nd][ne], ks_d: the input's c1 on the own-digit limbs), both read
    // through X -> X^gal[b], instead of being read from u[b]
    const u32* key[kLinB] = {};
    const u32* ks_ext = nullptr;
    const u32* ks_d = nullptr;
    int nd = 0, alpha = 1, nkey = 0, nks = 0;
    size_t ext_ms = 0, d_ms = 0;
    // pt_shift > 0: compact diagonals (a sparse plan's, engine group_pts): limb t's residue at
    // coefficient k is pt[(t << pt_logc) + (k >> pt_shift)] -- runs of 2^pt_shift equal values
    int pt_shift = 0, pt_logc = 0;
};
void launch_lin_mac(hipStream_t st, const DevTables& T, const LinMacArgs& m, int nl, int ne, LimbMap map);

// --- fused public-key encryption of a batch of messages (renorm re-encryption) -----------
// one launch samples v, e0, e1 of every member (member m: streams stream_id(6|7|8, 0, base + m),
// the same samples as launch_sample_small), one combines c0 = (e0 + msg) + pk0 v, c1 = e1 + pk1 v
constexpr int kEncMax = 16384;  // grid y = 3 members
struct EncCtrs {
    u64 base = 0;  // member m uses encryption counter base + m
};
// out: [m][3][nl] (v, e0, e1 residues, coefficient form)
// msg (nullable): coefficient-form messages (member m at msg + m msg_ms) added to e0 before the
// NTT -- NTT(e0 + m) = NTT(e0) + NTT(m) residue for residue, so the combine then adds none and
// the message needs no NTT launch of its own (the renorms' re-encryption)
void launch_sample_enc(hipStream_t st, const DevTables& T, u32* out, int nl, int nm, const PrngKey& key, const EncCtrs& ctr,
                       const u32* msg = nullptr, size_t msg_ms = 0);
// top: [m][2][nl]; vee: [m][3][nl] NTT form; msg: member m at msg + m msg_ms words; pk: [2][pk_rows][N]
void launch_enc_combine(hipStream_t st, const DevTables& T, u32* top, const u32* vee, const u32* msg, size_t msg_ms, const u32* pk,
                        int pk_rows, int nl, int nm);
// raw decryption of up to 2 channels on their first kd[c] limbs: x[c][t] = c0 + c1 s (+ c2 s^2),
// x: [2][4][N]; channel c reads ct[c] (npoly[c] polys of nlc[c] limbs); s, s2: NTT rows of s, s^2
struct DecRaw {
    const u32* ct[2] = {};
    int npoly[2] = {}, nlc[2] = {}, kd[2] = {};
    int members = 1;         // stacked inputs: channel c = w members + m reads input w's member m
    size_t ms[2] = {0, 0};   // member stride (words) of each input
};
// x: [channel][4][N] with nch x members channels
void launch_dec_raw(hipStream_t st, const DevTables& T, u32* x, const DecRaw& dr, int nch, const u32* s, const u32* s2);

// --- sampling --------------------------------------------------------
// kind: 0 ternary, 1 centred binomial (eta = 21); writes value mod prime into nl rows
void launch_sample_small(hipStream_t st, const DevTables& T, u32* out, int nl, LimbMap map, const PrngKey& key, u64 stream, int kind);
// uniform residues: row l gets prng(seed, stream, prime(l) * N + k) mod q
void launch_sample_uniform(hipStream_t st, const DevTables& T, u32* out, int nl, LimbMap map, const PrngKey& key, u64 stream);
// b = -a*s + e (+ gadget*s' on rows with flag) : used by key generation
void launch_keygen_combine(hipStream_t st, const DevTables& T, u32* b, const u32* a, const u32* s, const u32* e, const u32* sp,
                           const u32* gadget, int nl, LimbMap map, int gadget_lo, int gadget_hi);
// out = a*a (dyadic square)
void launch_square(hipStream_t st, const DevTables& T, u32* out, const u32* a, int rows, int nl, LimbMap map);

// --- device Zeta16 renorm codec (REF/pipeline.py:65-69, REF/state_encoder.py:17-38) ----
// mixed-radix CRT constants for up to 4 limbs: p_mod[i][j] = (q_0 ... q_{j-1}) mod q_i,
// minv[i] = (q_0 ... q_{i-1})^{-1} mod q_i, pd[i] = q_0 ... q_{i-1} as a double
struct CrtConsts {
    u32 q[4], minv[4], p_mod[4][4];
    double pd[4];
};
// the 16 state slots i * stride: evaluation exponents e_i = 5^(i stride) mod 2N
struct Slot16 {
    u32 e[16];
};
// x: [2][4][N] coefficient residues of the two decryptions (kd[c] limbs used);
// acc[c][i][re|im] += sum_k (m_k / scale_c) e^{i pi e_i k / N}   (acc zeroed by the caller)
// CONTRACT: acc must be zero on entry, and every decode must be followed on the same stream by a
// launch_snap16 on the same accumulator (it reads acc and re-zeroes it for the next decode) or by a
// snapping encode whose zacc is the OTHER buffer of a double-buffered pair (the next decode then uses
// that one) -- a decode without either leaves stale sums that the next renorm would add onto
void launch_decode16(hipStream_t st, const DevTables& T, const u32* x, const int kd[2], const CrtConsts cc[2], const Slot16& sl,
                     const double inv_scale[2], double* acc);
// per slot: nibble = round(-angle 16 / 2 pi) mod 16, w = zeta16^nibble - 1 (acc -> w, nib)
void launch_snap16(hipStream_t st, double* acc, double* w, int* nib);
// out[c][t][k] = round(scale (delta_{k0} + (2/N) Re sum_i w_ci e^{-i pi e_i k / N})) mod q_t, t < nq
// periodic: the 16-periodic layout (positions sl.e = 5^i, only k == 0 mod N/32 nonzero)
// zacc (nullable): w is the decode's ACCUMULATOR instead -- the encode snaps it itself (no
// launch_snap16) and zeroes zacc, the other accumulator of a double-buffered pair (Engine::renorm)
void launch_encode16(hipStream_t st, const DevTables& T, u32* out, const double* w, const Slot16& sl, double scale, int nq, bool periodic = false,
                     double* zacc = nullptr);
// direct codec of a small-period packed renorm (period 32: the hi | lo halves of the packed XOR
// stage): acc[i] = the 32 slot values (slot j at 5^j) of ONE decryption (acc zeroed by the
// caller); launch_snap16 snaps them as 2 x 16; encode32 re-encodes w as ONE 32-periodic message
// (unpack instead: launch_encode16(periodic) of the two 16-value halves)
struct Slot32 {
    u32 e[32];
};
// the renorm's pooled re-encryption (k_renorm_wtab / k_renorm_combine, Engine::zero_enc)
constexpr int kRenormMaxLimbs = 24;  // the fresh level has 19 limbs
template <int NS>
struct SlotTab {
    u32 e[NS];
};
struct RenormOut {
    const u32* pool[2] = {};
    u32* out[2] = {};
};
// W[c][t][d] (nl limbs, D = 64 = 2 x 32 slots, one channel): the NTT of the snapped 32-periodic message
void launch_renorm_wtab32(hipStream_t st, const DevTables& T, u32* W, const double* w, double* zacc, const Slot32& sl, double scale, int nl,
                          const u32* gtab);
// the same for two 16-periodic channels (D = 32 each)
void launch_renorm_wtab16(hipStream_t st, const DevTables& T, u32* W, const double* w, double* zacc, const Slot16& sl, double scale, int nl,
                          const u32* gtab);
// the sparse decryption (k_dec_blocksum + k_renorm_sparse): per channel the CRT limbs and constants
struct SparseDec {
    int kd[2] = {};
    CrtConsts cc[2];
};
// nch = 1: one 32-slot channel (D = 64, sl32); nch = 2: two 16-slot channels (D = 32 each, sl16).  B: a
// [2][4][64] scratch; W as launch_renorm_wtab32 / 16; s, s2: the secret (and its square) in NTT form
void launch_renorm_sparse(hipStream_t st, const DevTables& T, u32* W, u32* B, const DecRaw& dr, int nch, const SparseDec& sd, const Slot32& sl32,
                          const Slot16& sl16, double scale, int nl, const u32* gtab, const u32* s, const u32* s2);
// out_c = pool_c + W_c on c0 (runs of N / 2^ld equal values), nch <= 2 channels of 2 x nl rows
void launch_renorm_combine(hipStream_t st, const DevTables& T, const RenormOut& ro, int nch, const u32* W, int nl, int ld);
// CONTRACT (as launch_decode16): acc zero on entry; the snap follows on the same stream, either inside the
// snapping encode (the default, AESFHE_SNAP_ENCODE: it reads acc and zeroes the other buffer of its
// double-buffered pair for the next decode) or as launch_snap16 on acc (AESFHE_SNAP_ENCODE=0)
void launch_decode32(hipStream_t st, const DevTables& T, const u32* x, int kd, const CrtConsts& cc, const Slot32& sl, double inv_scale, double* acc);
void launch_encode32(hipStream_t st, const DevTables& T, u32* out, const double* w, const Slot32& sl, double scale, int nq, double* zacc = nullptr);

// --- slot-packed Zeta16 renorm ----------------------
// Full canonical-embedding decode / encode on the device in fp64: the slots of a real
// polynomial m are a length-N DFT of the twisted coefficients m_k zeta^k (encoder.cpp),
// computed as a four-step FFT over an N1 x N2 row-major matrix (N1 = 2^ceil(logn/2)).
// Element t of a transform's output is stored at fft_loc(t) = (t mod N1) N2 + t / N1.
// x: [2][4][N] coefficient residues (kd[c] limbs) -> z[c][k] = m_k / scale_c * zeta^k
// members > 1: channel c belongs to input c / members (stacked renorm)
void launch_decode_twist(hipStream_t st, const DevTables& T, const u32* x, const int kd[2], const CrtConsts cc[2],
                         const double inv_scale[2], double* z, int nch = 2, int members = 1);
// in-place X_k = sum_n x_n e^{sign 2 pi i n k / N} on 2 vectors (complex double, [2][N]);
// input in natural order, output at fft_loc
void launch_fft2(hipStream_t st, const DevTables& T, double* z, int sign, int nch = 2);
// snap: slot j (value at fft_loc(slot_pos[j]) of zin) -> zeta16 power if (j mod stride) < states,
// else 1; writes w[slot_pos[j]] = v and w[N - 1 - slot_pos[j]] = conj(v) (natural order)
// unpack = n > 0: both outputs read the first input's 2n-periodic packed state, output 0 its
// slots (j mod n), output 1 its slots (j mod n) + n
// members > 1 with unpack: output channel c = half (c / members) of input channel c % members
void launch_snap_slots(hipStream_t st, const DevTables& T, const double* zin, double* w, const u32* slot_pos, int states, int unpack = 0,
                       int nch = 2, int members = 1);
// out[c][t][k] = round(scale Re(v[fft_loc(k)] zeta^{-k}) / N) mod q_t, t < nq
void launch_encode_untwist(hipStream_t st, const DevTables& T, u32* out, const double* v, double scale, int nq, int nch = 2);
// nch (all four): channels processed (grid y); 1 = channel 0 only (one input decrypted, or one output)

// --- fused LUT evaluation ---------------------------
// Elements are canonical ciphertexts at data levels >= the output level l; only their first
// nl(l) limbs are read (exact modulo Q_l) and each element's own scale is folded into the
// integer constants.  Constants: cst[term][limb][half][Shoup pair] (half = slot half of
// the constant a + b X^{N/2}).
constexpr int kLutMax = 16;
struct LutOperands {
    const u32* a[kLutMax];  // A_p, 2 polys of na[p] limbs each
    const u32* b[kLutMax];
    int na[kLutMax], nb[kLutMax];
    int p_start[kLutMax + 1];  // terms of A_p: [p_start[p], p_start[p + 1]) in q_of
    int q_of[kLutMax * kLutMax];  // int, not byte: a uniform dword read by the scalar unit (a byte load is a vector load + wait)
};
// out (3 polys, nl rows each) = sum_p A_p (x) (sum_q C_pq B_q)
// members > 1: every element a stack of `members` ciphertexts (member stride 2 x its limbs x N),
// the output a stack of 3-polynomial tensors
void launch_lut_bivariate(hipStream_t st, const DevTables& T, u32* out, const LutOperands& op, int n_a, const u32* cst, int nl,
                          int members = 1);
// chunk of a univariate sum: out (npoly x nl) = (acc ? acc : 0) + sum_{k < n} C_k X_k
constexpr int kLutChunk = 32;
struct LutChunk {
    const u32* x[kLutChunk];
    int nx[kLutChunk];
};
void launch_lut_univariate(hipStream_t st, const DevTables& T, u32* out, const u32* acc, const LutChunk& ch, int n, const u32* cst,
                           int npoly, int nl, int members = 1, const LimbConsts* cadd = nullptr);

