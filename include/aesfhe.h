/*
 * aesfhe.h -- C ABI of the MI355X-native CKKS engine (libaesfhe.so).
 *
 * This is the drop-in boundary for the reference's hot path: every CKKS primitive the
 * reference reaches through EngineContext (REF/engine_context.py:56-204), i.e. through
 * the closed-source `desilofhe.Engine` (REF/engine_context.py:1,17-50), is one entry
 * point here.  Signatures use plain pointers, sizes and opaque 64-bit handles; the
 * Python shim (aes-implementation-fhe_amd/mi355x_ckks.py) binds them with ctypes.
 *
 * Conventions
 *   - Every function returns 0 on success or a negative status; the message is then
 *     available from aesfhe_last_error(ctx).  Level exhaustion messages contain the
 *     word "level" and relinearising a 2-polynomial ciphertext reports
 *     "should have 3 polynomials" (the strings REF/engine_context.py:139-145,186-195
 *     and REF/xor4_lut.py:33-51 branch on).
 *   - Results are always new handles; inputs are never modified.  Free every handle
 *     with aesfhe_free.
 *   - Slots are passed as separate real/imaginary double arrays of slot_count entries.
 *   - rotate(ct, steps) == np.roll(slots, steps)  (SURVEY.md quirk 4e).
 *   - A context is bound to one HIP device and one stream; it is not thread safe, but
 *     independent contexts (one per GPU) are.
 */
#ifndef AESFHE_H
#define AESFHE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct aesfhe_ctx aesfhe_ctx;
typedef uint64_t aesfhe_handle;

/* --- context / keys -------------------------------------------------------------- */
/* replaces desilofhe.Engine(...) construction, REF/engine_context.py:17-39 */
int aesfhe_create(aesfhe_ctx** out, int log_n, int max_level, int dnum, int device_id, uint64_t seed);
/* bootstrappable parameter set: fresh ciphertexts at fresh_level, the chain extended by
 * aesfhe_bootstrap_depth() levels (CoeffToSlot/EvalMod on double-prime levels) */
int aesfhe_create_boot(aesfhe_ctx** out, int log_n, int fresh_level, int dnum, int device_id, uint64_t seed);
/* Randomness: every key and encryption sample is a ChaCha20 block under a 256-bit context key
 * (DESIGN.md §3.4).  aesfhe_create / aesfhe_create_boot take a 64-bit seed as key words 0-1
 * (reproducible test and parity contexts); aesfhe_create_keyed takes the full 32-byte key
 * (little-endian words; the Python Engine draws it from os.urandom unless a seed is given).
 * bootstrappable != 0: max_level is the fresh level of a bootstrappable set (aesfhe_create_boot). */
int aesfhe_create_keyed(aesfhe_ctx** out, int log_n, int max_level, int dnum, int device_id, const uint8_t* key,
                        int bootstrappable);
/* Encryption randomness (v, e0, e1 of every encryption, the renorms' re-encryptions included)
 * is drawn under the context key with `nonce` folded into key words 6-7; key material is not
 * affected.  Processes sharing one context key (the ranks of a multi-GPU job) must
 * set different nonces, otherwise their i-th encryptions reuse (v, e) and the difference of two
 * ranks' ciphertexts is a noiseless encoding of the plaintext difference.  Default 0; the Python
 * Engine draws a random one per process (os.urandom) unless pinned.  No reference counterpart:
 * desilofhe.Engine.encrypt (REF/engine_context.py:56-57) samples internally. */
int aesfhe_set_enc_nonce(aesfhe_ctx* ctx, uint64_t nonce);
/* limbs per level 0..max_level (a ciphertext at level l has npoly x limbs[l] x N words) */
int aesfhe_level_limbs(aesfhe_ctx* ctx, int32_t* out);
int aesfhe_destroy(aesfhe_ctx* ctx);
const char* aesfhe_last_error(aesfhe_ctx* ctx);

/* Concurrency (MI355X-side; the reference engine is single-stream).  A context owns
 * aesfhe_streams() HIP streams.  Stream 0 serves every host thread by default; a host
 * thread that calls aesfhe_bind_stream(ctx, k) queues its work on stream k.
 * aesfhe_fork() makes streams 1.. start after all work queued so far on stream 0;
 * aesfhe_join() makes stream 0 continue only after them.  Between fork and join the
 * branches must be independent (they may read handles created before the fork); handles
 * freed by branch threads are recycled at the join.  Calls are serialised by a context
 * mutex and errors are per thread. */
int aesfhe_streams(aesfhe_ctx* ctx);
int aesfhe_bind_stream(aesfhe_ctx* ctx, int index);
int aesfhe_fork(aesfhe_ctx* ctx);
/* applies a handle's deferred work now, so branches that share it read one
 * canonical copy instead of each normalising its own */
int aesfhe_settle(aesfhe_ctx* ctx, aesfhe_handle c);
int aesfhe_join(aesfhe_ctx* ctx);
/* replaces create_secret_key / create_public_key / create_relinearization_key /
 * create_conjugation_key, REF/engine_context.py:44-48 (rotation keys are made on first use) */
int aesfhe_keygen(aesfhe_ctx* ctx);
/* engine.slot_count, read by every module (e.g. REF/state_encoder.py:14) */
int aesfhe_slot_count(aesfhe_ctx* ctx);
int aesfhe_max_level(aesfhe_ctx* ctx);
/* level of fresh encryptions (default max_level; lower when the chain is extended for bootstrapping) */
int aesfhe_set_fresh_level(aesfhe_ctx* ctx, int level);
/* info: [n, L, n_q, n_ks, n_p, alpha, dnum, log_n] */
int aesfhe_info(aesfhe_ctx* ctx, int32_t* info8);
int aesfhe_moduli(aesfhe_ctx* ctx, uint32_t* out);   /* n_q + n_p primes */
int aesfhe_scales(aesfhe_ctx* ctx, double* out);     /* delta_0 .. delta_L */
int aesfhe_sync(aesfhe_ctx* ctx);
int aesfhe_free(aesfhe_ctx* ctx, aesfhe_handle h);
int aesfhe_level(aesfhe_ctx* ctx, aesfhe_handle ct, int32_t* level, int32_t* npoly);

/* --- plaintexts / codec ------------------------------------------------------------ */
/* engine.encode(vec), REF/engine_context.py:62-63 (level-agnostic; encoded on use) */
int aesfhe_plaintext(aesfhe_ctx* ctx, const double* re, const double* im, int n, aesfhe_handle* out);
/* engine.encrypt(data, public_key), REF/engine_context.py:56-57 */
int aesfhe_encrypt(aesfhe_ctx* ctx, const double* re, const double* im, int n, aesfhe_handle* out);
/* engine.decrypt(ct, secret_key), REF/engine_context.py:59-60 */
int aesfhe_decrypt(aesfhe_ctx* ctx, aesfhe_handle ct, double* re, double* im, int n);

/* --- arithmetic ---------------------------------------------------------------------- */
/* engine.add / engine.subtract, REF/engine_context.py:70-74 (levels auto-aligned) */
int aesfhe_add(aesfhe_ctx* ctx, aesfhe_handle a, aesfhe_handle b, aesfhe_handle* out);
int aesfhe_sub(aesfhe_ctx* ctx, aesfhe_handle a, aesfhe_handle b, aesfhe_handle* out);
/* engine.add(ct, pt) / engine.add_plain(ct, scalar), REF/engine_context.py:76-98 */
int aesfhe_add_pt(aesfhe_ctx* ctx, aesfhe_handle ct, aesfhe_handle pt, aesfhe_handle* out);
int aesfhe_add_scalar(aesfhe_ctx* ctx, aesfhe_handle ct, double re, double im, aesfhe_handle* out);
/* engine.multiply(ct, scalar|pt), REF/engine_context.py:65-68,106-125 */
int aesfhe_mul_scalar(aesfhe_ctx* ctx, aesfhe_handle ct, double re, double im, aesfhe_handle* out);
int aesfhe_mul_pt(aesfhe_ctx* ctx, aesfhe_handle ct, aesfhe_handle pt, aesfhe_handle* out);
/* engine.multiply(a, b, relinearization_key), REF/engine_context.py:65-67:
 * tensor + relinearise + rescale; relin = 0 returns the 3-polynomial tensor (rescaled) */
int aesfhe_mul(aesfhe_ctx* ctx, aesfhe_handle a, aesfhe_handle b, int relin, aesfhe_handle* out);
/* Fused LUT evaluation.  One kernel replaces the per-term product loops of
 *   REF/xor4_lut.py:63-74           XOR4LUT.apply:        sum_{p,q} C[p,q] A^p B^q
 *   REF/mixcol_final.py:80-91       _gf_poly_eval_2var    (same form, GF LUT coefficients)
 *   REF/invmixcolumns_fhe.py:76-87  _poly2_eval           (same form)
 *   REF/sub_bytes_lut.py:46-74      lift / hi / lo sums:  c0 + sum_k C[k] X^k
 *   REF/lut.py:71-94                LUTEvaluator.apply    (same univariate form)
 * lut_create stores the n_a x n_b coefficient matrix (row-major re / im; n_b = 1 makes a
 * univariate LUT with constant term c0; bivariate LUTs are at most 16 x 16).  lut_eval takes
 * the element handles a[0..n_a) (and b[0..n_b) for bivariate LUTs; entries whose coefficients
 * are all zero may be 0) and returns the sum at the logical level of the per-term products
 * (lowest element level - 2, resp. - 1); it fails with a message containing "level" when the
 * elements are too low for the fused form, and the caller falls back to the product loop. */
int aesfhe_lut_create(aesfhe_ctx* ctx, int n_a, int n_b, const double* re, const double* im, double c0_re, double c0_im,
                      aesfhe_handle* out);
int aesfhe_lut_eval(aesfhe_ctx* ctx, aesfhe_handle lut, const aesfhe_handle* a, const aesfhe_handle* b, aesfhe_handle* out);
/* Releases a LUT's coefficient set and every per-level device constant cached for it (the
 * evaluator's plaintext caches, REF/lut.py:71-94 keeps them per object); fails if `lut` is not
 * a LUT handle.  aesfhe_free also accepts LUT handles; this entry states the intent. */
int aesfhe_lut_free(aesfhe_ctx* ctx, aesfhe_handle lut);
/* Deferred evaluation switch, default on: API-level ct x ct products
 * leave relinearisation and their rescale to the first consumer that needs a
 * 2-polynomial canonical ciphertext (rotate, conjugate, ct x ct, power basis, bootstrap,
 * export), and non-integer scalar / plaintext products defer their rescale.  Sums of such
 * terms are combined before any key switch.  Results decrypt identically up to CKKS
 * rounding; 0 restores eager relinearise-and-rescale after every product. */
int aesfhe_set_lazy(aesfhe_ctx* ctx, int on);
/* engine.relinearize, REF/engine_context.py:134-145 */
int aesfhe_relinearize(aesfhe_ctx* ctx, aesfhe_handle ct, aesfhe_handle* out);
int aesfhe_rescale(aesfhe_ctx* ctx, aesfhe_handle ct, aesfhe_handle* out);
/* drop to a lower level with exact scale */
int aesfhe_level_down(aesfhe_ctx* ctx, aesfhe_handle ct, int level, aesfhe_handle* out);
/* engine.rotate(ct, rotation_key, steps), REF/engine_context.py:127-132 */
int aesfhe_rotate(aesfhe_ctx* ctx, aesfhe_handle ct, int steps, aesfhe_handle* out);
/* engine.conjugate(ct, conjugation_key), REF/engine_context.py:103-104 */
int aesfhe_conjugate(aesfhe_ctx* ctx, aesfhe_handle ct, aesfhe_handle* out);
/* Batched variants (SURVEY.md §8(b) "optional batched variants taking h[] arrays"; DESIGN.md
 * §3.12): n independent engine.multiply(a[i], b[i], relinearization_key) products
 * (REF/engine_context.py:65-67, always relinearised and rescaled) resp. n
 * engine.conjugate(in[i], conjugation_key) calls (REF/engine_context.py:103-104).  Operands
 * at one level are stacked and share one tensor launch and one key switch per chunk of four;
 * the results equal the separate calls bit for bit.  out[i] receives a new handle. */
int aesfhe_mul_many(aesfhe_ctx* ctx, int n, const aesfhe_handle* a, const aesfhe_handle* b, aesfhe_handle* out);
/* sum_{i<n} cts[i] * pts[i] (1 <= n <= 8 single ciphertexts times non-constant plaintexts), at the
 * operands' common lowest level, as ONE kernel; the same value as n engine.multiply(ct, pt) calls summed
 * with engine.add (REF/engine_context.py:65-68, :77-80) -- the masked rotations of REF/shift_rows.py:39-56
 * feeding MixColumns (REF/mixcol_final.py:124-154) summed in one launch (MixColFinal.sr_entry). */
int aesfhe_mul_pt_sum(aesfhe_ctx* ctx, int n, const aesfhe_handle* cts, const aesfhe_handle* pts, aesfhe_handle* out);
/* the secret-key renorm's pool of zero encryptions: size = encryptions made per
 * refill (0: every renorm encrypts its own message; < 0: keep the size), every pool emptied -- the
 * re-encryption of REF/pipeline.py:65-69 (decrypt -> snap -> encrypt) drawn as Enc(0) + message */
int aesfhe_renorm_pool(aesfhe_ctx* ctx, int size);
/* members per packed bootstrap of a stacked periodic ciphertext (aesfhe_bootstrap_sparse on a stack):
 * up to `members` (a power of two dividing the stack size) monomial-packed into one message of
 * `members` times the period, one bootstrap each.  1: every member its own
 * bootstrap (bit-exact with single bootstraps); default 16 (AESFHE_STACK_PACK). */
int aesfhe_set_stack_pack(aesfhe_ctx* ctx, int members);
int aesfhe_conjugate_many(aesfhe_ctx* ctx, int n, const aesfhe_handle* in, aesfhe_handle* out);
/* n automorphisms of possibly DIFFERENT ciphertexts, each with its own Galois element galois[i]
 * (odd, < 2N): engine.rotate(ct, rotation_key, steps) (REF/engine_context.py:127-132; Galois
 * element 5^(-steps) mod 2N) and engine.conjugate(ct, conjugation_key) (:103-104; 2N - 1) calls
 * of one AES step -- the masked row rotations of ShiftRows (REF/shift_rows.py:39-56) and the
 * column shifts of MixColumns (REF/mixcol_final.py:124-154) for both nibble halves -- as ONE
 * heterogeneous batched key switch per level: one ModUp per distinct input,
 * one key-inner-product launch with a key per member, one stacked ModDown.  Same results as the
 * separate calls; galois[i] = 1 returns a copy. */
int aesfhe_galois_multi(aesfhe_ctx* ctx, int n, const aesfhe_handle* in, const uint64_t* galois, aesfhe_handle* out);

/* Stacked ciphertexts (multi-pair batches, BASELINE configs 3-5 with one state per pair; DESIGN.md
 * §3.16).  aesfhe_stack: n single ciphertexts -> ONE handle holding n members (canonical form,
 * dropped to the lowest member level).  Every operation then takes the stack as one operand and
 * returns a stack: element-wise work in one launch over all members, key switches in chunks of
 * members that read each key once, LUT sums with a member grid dimension, renorms decrypting /
 * re-encrypting every member in one set of launches, bootstraps in chunks of two members.
 * Operands of one operation must be stacks of the same size (no broadcasting); decrypt needs a
 * single ciphertext.  aesfhe_unstack: the n members as single handles (n = member count);
 * aesfhe_members: the member count (1 for a single ciphertext).  Replaces the reference's loop
 * over independent ciphertext pairs (REF/main.py:121-140 runs one pair per state). */
int aesfhe_stack(aesfhe_ctx* ctx, int n, const aesfhe_handle* in, aesfhe_handle* out);
int aesfhe_unstack(aesfhe_ctx* ctx, aesfhe_handle in, int n, aesfhe_handle* out);
int aesfhe_members(aesfhe_ctx* ctx, aesfhe_handle h, int* members);
/* n rotations of ONE ciphertext, engine.rotate(ct, rotation_key, steps[i])
 * (REF/engine_context.py:127-132; the column shifts of REF/mixcol_final.py:124-154 and the
 * row rotations of REF/shift_rows.py:39-56), hoisted: one ModUp for all of them.  Same
 * results as n aesfhe_rotate calls. */
int aesfhe_rotate_hoisted(aesfhe_ctx* ctx, aesfhe_handle ct, int n, const int* steps, aesfhe_handle* out);
/* engine.make_power_basis(ct, degree, relinearization_key), REF/engine_context.py:100-101;
 * out[k-1] = ct^k, k = 1..degree */
int aesfhe_power_basis(aesfhe_ctx* ctx, aesfhe_handle ct, int degree, aesfhe_handle* out);
/* engine.ntt / engine.intt, REF/engine_context.py:173-177 */
int aesfhe_to_ntt(aesfhe_ctx* ctx, aesfhe_handle ct, aesfhe_handle* out);
int aesfhe_to_intt(aesfhe_ctx* ctx, aesfhe_handle ct, aesfhe_handle* out);
/* engine.bootstrap(ct, relin, conj, bootstrap_key), REF/engine_context.py:147-162.
 * Full-slot complex bootstrapping: sparse-secret encapsulation, ModRaise,
 * CoeffToSlot, EvalMod, SlotToCoeff.  Input slots must satisfy |z| <= 1; the output is at
 * level max_level - aesfhe_bootstrap_depth() of the bootstrappable parameter set. */
int aesfhe_bootstrap(aesfhe_ctx* ctx, aesfhe_handle ct, aesfhe_handle* out);
/* the two bootstraps of a hi / lo pair (REF/mixcol_final.py:158-162, REF/invmixcolumns_fhe.py:166-168)
 * as one batched bootstrap: same results as two aesfhe_bootstrap calls, each key switch reads
 * its key and each linear transform its diagonals once for both */
int aesfhe_bootstrap_pair(aesfhe_ctx* ctx, aesfhe_handle a, aesfhe_handle b, aesfhe_handle* out_a, aesfhe_handle* out_b);
/* bootstrap(ct) * gain and its pair form, gain in (0, 1] folded into the level-0 scaling (no
 * extra level): the true-FHE renorm's bootstrap hands the snap u = kappa x (REF
 * zeta16_noise_reducter.py:6-57 bootstrap_before=True) */
int aesfhe_bootstrap_scaled(aesfhe_ctx* ctx, aesfhe_handle ct, double gain, aesfhe_handle* out);
/* Sparse-slot bootstrap: for a message whose slots repeat with period `period`
 * (slot j == slot j mod period; a power of two in [16, slot_count)), i.e. a polynomial in the
 * subring Z[X^(N / 2 period)].  Same result as aesfhe_bootstrap on such a message (within the
 * bootstrap's error) at a fraction of the cost: a trace to the subring after ModRaise, then the
 * period-sized CoeffToSlot / SlotToCoeff; it starts from a lower level.  A message that is not
 * periodic is NOT refreshed correctly.  gain as for aesfhe_bootstrap_scaled (1.0 = none).
 * Replaces the same engine.bootstrap calls (REF/engine_context.py:147-162) when the caller
 * knows its layout is periodic (StateEncoder(periodic=True)). */
int aesfhe_bootstrap_sparse(aesfhe_ctx* ctx, aesfhe_handle ct, int period, double gain, aesfhe_handle* out);
/* Secret-key renorm of a (hi, lo) pair in the periodic layout (slot j == slot j mod period,
 * a power of two >= 16): period 16 decodes / re-encodes its 16 slots directly, other periods
 * snap every slot; level < 0 = the fresh level (as aesfhe_renorm_at otherwise). */
int aesfhe_renorm_periodic(aesfhe_ctx* ctx, aesfhe_handle hi, aesfhe_handle lo, int period, int level, aesfhe_handle* out_hi,
                           aesfhe_handle* out_lo);
/* Secret-key renorm of ONE ciphertext whose every slot holds a Zeta16 nibble (a packed state
 * of the pipeline's packed XOR stage): every slot snapped and re-encrypted at
 * `level` (< 0 = fresh).  Replaces the renorm of REF/pipeline.py:65-69 for that form. */
int aesfhe_renorm_single(aesfhe_ctx* ctx, aesfhe_handle ct, int level, aesfhe_handle* out);
/* aesfhe_renorm_single of a ciphertext known to be `period`-periodic (the packed form: period =
 * 2 x the state period): period 32 decodes / re-encodes its 32 slots directly (no FFT); other
 * periods as aesfhe_renorm_single. */
int aesfhe_renorm_packed(aesfhe_ctx* ctx, aesfhe_handle ct, int period, int level, aesfhe_handle* out);
/* Secret-key renorm that unpacks: `packed` holds the hi nibbles of an n-periodic state pair in
 * slots (j mod 2n) < n and the lo nibbles in the others (period = n, a power of two, 2n <=
 * slots); out_hi / out_lo are the snapped n-periodic hi / lo states at `level` -- the
 * (hi, lo) pair REF/pipeline.py:65-69's renorm returns. */
int aesfhe_renorm_unpack(aesfhe_ctx* ctx, aesfhe_handle packed, int period, int level, aesfhe_handle* out_hi,
                         aesfhe_handle* out_lo);
/* aesfhe_renorm_periodic / _packed / _unpack of ct + conj(ct_conj) (per channel for the pair): a conjugate-split LUT's S1 + conj(S2)
 * renormalised without its conjugation key switch (both decrypted, conj(m2) = m2(X^-1) added before
 * the codec); inputs of different level / scale are summed homomorphically first.  Engine-side
 * fusion of REF's `ctx.add(s1, ctx.conjugate(s2))` followed by the renorm (REF/pipeline.py:65-69). */
/* the periodic pair renorm (period 16, one state pair) whose output is ONE ciphertext in the packed
 * period-32 form (hi on slots j mod 32 < 16, lo on the others: StateEncoder.pack's layout) -- the
 * renorm of pack(hi, lo) without the pack's mask products and level; hi_conj / lo_conj (both or
 * neither, 0 = none): the pair's conjugate partners as aesfhe_renorm_periodic_conj. */
/* the periodic pair renorm (period 16, one state pair) with a byte permutation folded in: output slot
 * i (byte i) takes input byte perm16[i] (ShiftRows: REF/shift_rows.py's slot rotations after the renorm
 * of REF/pipeline.py:65-69, at no level); optional conjugate partners as aesfhe_renorm_periodic_conj;
 * pack_out != 0: one packed output as aesfhe_renorm_pack (out_lo unused). */
int aesfhe_renorm_periodic_perm(aesfhe_ctx* ctx, aesfhe_handle hi, aesfhe_handle lo, aesfhe_handle hi_conj, aesfhe_handle lo_conj,
                                const int32_t* perm16, int pack_out, int period, int level, aesfhe_handle* out_hi, aesfhe_handle* out_lo);
/* aesfhe_renorm_unpack (period 16) with a byte permutation folded in, applied to both unpacked
 * halves (InvShiftRows after the renorm that follows InvMixColumns); packed_conj: 0 or a conjugate partner */
int aesfhe_renorm_unpack_perm(aesfhe_ctx* ctx, aesfhe_handle packed, aesfhe_handle packed_conj, const int32_t* perm16, int period, int level,
                              aesfhe_handle* out_hi, aesfhe_handle* out_lo);
int aesfhe_renorm_pack(aesfhe_ctx* ctx, aesfhe_handle hi, aesfhe_handle lo, aesfhe_handle hi_conj, aesfhe_handle lo_conj, int period, int level,
                       aesfhe_handle* out);
int aesfhe_renorm_periodic_conj(aesfhe_ctx* ctx, aesfhe_handle hi, aesfhe_handle lo, aesfhe_handle hi_conj, aesfhe_handle lo_conj,
                                int period, int level, aesfhe_handle* out_hi, aesfhe_handle* out_lo);
int aesfhe_renorm_packed_conj(aesfhe_ctx* ctx, aesfhe_handle ct, aesfhe_handle ct_conj, int period, int level, aesfhe_handle* out);
int aesfhe_renorm_unpack_conj(aesfhe_ctx* ctx, aesfhe_handle packed, aesfhe_handle packed_conj, int period, int level,
                              aesfhe_handle* out_hi, aesfhe_handle* out_lo);
int aesfhe_bootstrap_pair_sparse(aesfhe_ctx* ctx, aesfhe_handle a, aesfhe_handle b, int period, double gain, aesfhe_handle* out_a,
                                 aesfhe_handle* out_b);
int aesfhe_bootstrap_pair_scaled(aesfhe_ctx* ctx, aesfhe_handle a, aesfhe_handle b, double gain, aesfhe_handle* out_a,
                                 aesfhe_handle* out_b);
/* four n-periodic ciphertexts (4 period <= slots) refreshed by ONE bootstrap at period 4n: the pairs
 * (in[0], in[1]) and (in[2], in[3]) monomial-packed as in aesfhe_bootstrap_pair_sparse, the two packs
 * packed once more (X^(N/8n)), split back by rotations by 2n then n slots.  out[m] = gain * in[m]
 * refreshed (the true-FHE MixColumns renorms of two ciphertext pairs at one point of a round;
 * replaces two aesfhe_bootstrap_pair_sparse calls, REF/zeta16_noise_reducter.py:108-169 /
 * REF/mixcol_final.py:104-106's renorm points). */
int aesfhe_bootstrap_quad_sparse(aesfhe_ctx* ctx, const aesfhe_handle* in, int period, double gain, aesfhe_handle* out);
int aesfhe_bootstrap_depth(void);
/* host self-check of the bootstrap plan: err[0] SlotToCoeff, err[1] CoeffToSlot vs the
 * canonical embedding, err[2] EvalMod Chebyshev error (no GPU needed) */
int aesfhe_debug_bootplan(int log_n, double* err3);
/* the same self-check for a sparse (period-n) plan, packed real form or not: err2 = [StC, CtS] */
int aesfhe_debug_sparseplan(int n, int pack, double* err2);
/* debug: run bootstrap up to a stage (1..11, see engine.hip) and return that ciphertext */
int aesfhe_debug_boot_stage(aesfhe_ctx* ctx, aesfhe_handle ct, int stage, aesfhe_handle* out);
/* Sparse-slot bootstrap stages and groups (tests only, no reference counterpart:
 * the pieces of the bootstrap that replaces engine.bootstrap at REF/mixcol_final.py:158-162).
 * debug_boot_stage_sparse: the period-`period` bootstrap stopped after a stage (as
 * aesfhe_debug_boot_stage; 12 = back on the dense secret BEFORE the trace to the subring, 4 =
 * after it, 9 = the packed real form w' + conj(w'), 10 = after EvalMod).  debug_sparse_group:
 * one CoeffToSlot (which < #CtS) / SlotToCoeff group of that plan (pair != 0: the pair-packed
 * plan; its last index is the lo form of SlotToCoeff's first group); debug_sparse_group_plain:
 * the same group on the host on the first info3[0] slots (one period of its diagonals), tiled
 * over all slot_count outputs; info3[1] = CoeffToSlot groups, info3[2] = all groups.  debug_mono_pack: a + X^(N / 4 period) b at level 0;
 * debug_mono_split: (m + rot_period(m), X^-k (m - rot_period(m))) -- the monomial pair packing
 * and its split around ONE bootstrap of both messages. */
int aesfhe_debug_boot_stage_sparse(aesfhe_ctx* ctx, aesfhe_handle ct, int stage, int period, aesfhe_handle* out);
int aesfhe_debug_sparse_group(aesfhe_ctx* ctx, aesfhe_handle ct, int period, int which, int pair, aesfhe_handle* out);
int aesfhe_debug_sparse_group_plain(aesfhe_ctx* ctx, int period, int which, int pair, const double* re, const double* im,
                                    double* out_re, double* out_im, int* info3);
int aesfhe_debug_mono_pack(aesfhe_ctx* ctx, aesfhe_handle a, aesfhe_handle b, int period, aesfhe_handle* out);
int aesfhe_debug_mono_split(aesfhe_ctx* ctx, aesfhe_handle m, int period, aesfhe_handle* out_hi, aesfhe_handle* out_lo);
/* ephemeral sparse secret (NTT form, all limbs) */
int aesfhe_export_sparse(aesfhe_ctx* ctx, uint32_t* out);
int aesfhe_debug_lin_group(aesfhe_ctx* ctx, aesfhe_handle ct, int which, aesfhe_handle* out);
/* The same group applied on the host to slot_count complex slots (re, im) -> (out_re, out_im):
 * the plan model a decryption of aesfhe_debug_lin_group is checked against (test only). */
int aesfhe_debug_lin_group_plain(aesfhe_ctx* ctx, int which, const double* re, const double* im, double* out_re,
                                 double* out_im);
/* [s_bt, k1, top, K, r, deg, log2 modulus of the dense->sparse key (Q0 P', Q0 = q0 q1), sparse
 * secret weight h, special primes in P', base limbs in Q0, message bits b (s_bt = Q0 / 2^b)]
 *  */
int aesfhe_boot_info(aesfhe_ctx* ctx, double* out11);
/* Zeta16 secret-key renorm of a (hi, lo) state pair (REF/pipeline.py:65-69): decrypt,
 * snap the 16 strided slots to the nearest codeword, refill others with 1, re-encrypt */
int aesfhe_renorm_pair(aesfhe_ctx* ctx, aesfhe_handle hi, aesfhe_handle lo, aesfhe_handle* out_hi, aesfhe_handle* out_lo);
/* the same renorm for the slot-packed layout: `states` AES states per
 * ciphertext pair, byte i of state b in slot i*stride + b (1 <= states <= slot_count/16);
 * every slot with (j mod stride) < states is snapped, the others refilled with 1.
 * Replaces the per-state loop over REF/pipeline.py:65-69 for a batch of states. */
int aesfhe_renorm_states(aesfhe_ctx* ctx, aesfhe_handle hi, aesfhe_handle lo, int states, aesfhe_handle* out_hi,
                         aesfhe_handle* out_lo);
/* renorm_states re-encrypting at min(level, fresh) (< 0 = the fresh level) instead of the
 * fresh level: a caller that knows the depth of its next step saves limbs */
int aesfhe_renorm_at(aesfhe_ctx* ctx, aesfhe_handle hi, aesfhe_handle lo, int states, int level, aesfhe_handle* out_hi,
                     aesfhe_handle* out_lo);

/* --- raw access (tests, parity against the oracle) ------------------------------------ */
/* limbs of a ciphertext: npoly x (level+2) x N uint32, NTT form */
int aesfhe_export(aesfhe_ctx* ctx, aesfhe_handle ct, uint32_t* out, uint64_t words);
int aesfhe_import(aesfhe_ctx* ctx, int level, int npoly, const uint32_t* data, aesfhe_handle* out);
/* secret key (NTT form, all n_q + n_p limbs) / public key / key-switching key of galois g (0 = relin) */
int aesfhe_export_secret(aesfhe_ctx* ctx, uint32_t* out);
int aesfhe_export_pk(aesfhe_ctx* ctx, uint32_t* out);
int aesfhe_export_ksk(aesfhe_ctx* ctx, uint64_t galois, uint32_t* out);
/* forward / inverse NTT of host rows whose limb l is prime first_prime + l */
int aesfhe_debug_ntt(aesfhe_ctx* ctx, uint32_t* data, int rows, int first_prime, int inverse);
/* key switch of a raw polynomial d (level+2 limbs, NTT) with the key of galois g */
int aesfhe_debug_keyswitch(aesfhe_ctx* ctx, int level, uint64_t galois, const uint32_t* d, uint32_t* out);
/* per-kernel timing of the last N ops (HIP events); op counters */
/* Micro-benchmark of one primitive, iters back-to-back launches on the engine stream;
 * *us = microseconds per iteration (device time incl. launch gaps).  op 0: NTT of arg
 * rows, 1: inverse NTT of arg rows, 2: key switch at level arg, 3: rescale at level arg,
 * 4: ct x ct + relinearise + rescale at level arg.  MI355X-side tooling. */
int aesfhe_bench_op(aesfhe_ctx* ctx, int op, int arg, int iters, double* us);
int aesfhe_counters(aesfhe_ctx* ctx, uint64_t* out, int n);
/* time only one launch in `every` of each enabled kernel (default 1): an unbiased live sample
 * with less event overhead in the measured run */
int aesfhe_profile_every(aesfhe_ctx* ctx, int every);
/* live kernel timing with HIP events on the engine stream: bit k of mask enables kernel id k
 * (order: ntt_cols_fwd, ntt_rows_fwd, ntt_rows_inv, ntt_cols_inv, base_convert, key_inner,
 * moddown, tensor, rescale, automorph, elementwise, sample); stats: per id
 * [launches, total ms, algorithmic bytes] */
int aesfhe_profile(aesfhe_ctx* ctx, uint32_t mask);
int aesfhe_kernel_stats(aesfhe_ctx* ctx, double* out, int n, int reset);
/* radix-2 butterflies of the timed NTT launches per kernel id (out[n]; call before a resetting
 * aesfhe_kernel_stats): the numerator of the NTT's VALU roofline */
int aesfhe_kernel_work(aesfhe_ctx* ctx, double* out, int n);
/* dispatch-inclusive timing: per kernel id k, out[2k] = boundary gaps measured, out[2k + 1] = their
 * total ms -- the gap between the last block end of a sampled launch and the first block start of
 * the launch issued right after it, accounted to the latter's id (its drain + dispatch ramp, what
 * rocprofv3 durations add to the in-kernel span); call before a resetting aesfhe_kernel_stats */
int aesfhe_kernel_gaps(aesfhe_ctx* ctx, double* out, int n);
/* per-level work tallies since the last aesfhe_reset_counters: out[l] (l < n) = kind 0 key switches
 * of one polynomial (hoisted rotations counted one each), 1 ct x ct products (tensor + relinearise +
 * rescale; their key switch counted in kind 0), 2 plaintext-diagonal products of the linear transforms,
 * at level l.  The CPU baseline replays a bootstrap's work from them on the C oracle (bench.py). */
int aesfhe_level_counters(aesfhe_ctx* ctx, int kind, uint64_t* out, int n);
int aesfhe_reset_counters(aesfhe_ctx* ctx);
/* device memory pool: out[0] = bytes the context's buffer pools hold (in use + cached), out[1] =
 * allocations that failed, released the cached free lists and were retried (a second failure is
 * an error status).  AESFHE_POOL_LIMIT_MB caps the pool bytes (test switch) */
int aesfhe_pool_stats(aesfhe_ctx* ctx, uint64_t* out);
/* kernel launches issued by this process so far (all contexts): the launch census of
 * tools/launch_census.py and bench.py's launches-per-encrypt (MI355X-side tooling) */
uint64_t aesfhe_launch_count(void);
/* launch census by (C-ABI entry point, kernel name), collected when the process starts with
 * AESFHE_CENSUS=1: "entry\tkernel\tlaunches\n" lines into buf (NUL-terminated, truncated to cap);
 * returns the bytes the whole census needs; reset != 0 clears it (tools/op_kernel_census.py) */
uint64_t aesfhe_launch_census(char* buf, uint64_t cap, int reset);
/* per kernel id (the aesfhe_profile order): algorithmic bytes and launches of
 * every launch this process issued so far, timed or not -- bench.py's whole-step roofline
 * (sum of algorithmic bytes of the timed steps / wall / 8 TB/s) */
int aesfhe_alg_bytes(double* bytes, uint64_t* launches, int n);

#ifdef __cplusplus
}
#endif
#endif
