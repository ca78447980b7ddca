/*
 * oracle/ckks_oracle.c -- TEST INFRASTRUCTURE, NOT PRODUCT CODE.
 *
 * Plain-C CPU restatement of the RNS-CKKS primitives that the reference reaches
 * through its EngineContext adapter (REF/engine_context.py:56-204).  The
 * reference's arithmetic lives in the third-party `desilofhe` package
 * (REF/engine_context.py:1), which is closed source, unpinned (no requirements /
 * lockfile in REF) and absent from this image.  This file
 * therefore restates the published RNS-CKKS algorithms (Cheon-Kim-Kim-Song
 * 2017; full-RNS variant Cheon-Han-Kim-Kim-Song 2018; hybrid key switching
 * Han-Ki 2020) under the conventions fixed in DESIGN.md §3, so that the HIP
 * engine can be checked bit-exactly limb by limb.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library.  It is deliberately written in the simplest loop form (one
 * butterfly at a time, one coefficient at a time) and shares no code with
 * aes-implementation-fhe_amd/csrc.
 *
 * Memory conventions (all caller-allocated, numpy friendly):
 *   polynomial  = [limb][N] uint32, limbs 0..l+1 for level l (2 base limbs)
 *   ciphertext  = [poly][limb][N]
 *   key-switch key = [digit][b|a][ext limb][N], ext limbs = Q limbs 0..n_ks-1
 *                    followed by the alpha special limbs.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef uint32_t u32;
typedef uint64_t u64;
typedef int64_t i64;
typedef __int128 i128;
typedef unsigned __int128 u128;

typedef struct {
    int logn, n, L, dnum, alpha;
    int n_q;  /* 2 base + L chain + 1 encryption limb */
    int n_ks; /* limbs reachable by key switching: L + 2 */
    int n_p;  /* special limbs */
    u32 *mod; /* n_q + n_p */
    u32 **psi_rev, **ipsi_rev;
    u32 *ninv;
    double *delta; /* delta[l], l = 0..L */
    u32 key[8];    /* ChaCha20 key of all sampling */
    int L1;        /* top of the single-prime region (== L without the bootstrapping region) */
} orc_t;

/* limbs of a level: l + 2 up to L1, two more per level above */
static int NL(const orc_t *o, int l) {
    if (l > o->L) return NL(o, o->L) + 1;  /* transient level L + 1 of a top-level encryption */
    return l <= o->L1 ? l + 2 : o->L1 + 2 + 2 * (l - o->L1);
}

/* ------------------------------------------------------------------ */
/* scalar modular arithmetic                                           */
/* ------------------------------------------------------------------ */
static u32 mulm(u32 a, u32 b, u32 q) { return (u32)(((u64)a * b) % q); }
static u32 addm(u32 a, u32 b, u32 q) { u64 s = (u64)a + b; return (u32)(s >= q ? s - q : s); }
/* Exact Barrett reduction for the hot loops (round 3: the oracle is also the CPU baseline, and a
 * hardware 64-bit division per product made it a strawman).  bq.mu = floor(2^64 / q); for any
 * 64-bit x, x - floor(x mu / 2^64) q lies in [0, 3q): at most two corrections.  Same residues as
 * the % forms, bit for bit. */
typedef struct { u32 q; u64 mu; u64 r64; } barrett_t;  /* r64 = 2^64 mod q */
static barrett_t bq_make(u32 q) {
    barrett_t b;
    b.q = q;
    b.mu = (u64)(((u128)1 << 64) / q);
    b.r64 = (u64)((((u128)1 << 64)) % q);
    return b;
}
static inline u32 bred64(u64 x, const barrett_t *b) {
    u64 est = (u64)(((u128)x * b->mu) >> 64);
    u64 r = x - est * b->q;
    if (r >= b->q) r -= b->q;
    if (r >= b->q) r -= b->q;
    return (u32)r;
}
static inline u32 bred128(u128 x, const barrett_t *b) {  /* x < 2^64 * 2^32 */
    u64 hi = (u64)(x >> 64), lo = (u64)x;
    return addm(bred64(lo, b), bred64(hi * b->r64, b), b->q);  /* hi < 2^32, r64 < 2^30: no overflow */
}
static inline u32 bmul(u32 a, u32 c, const barrett_t *b) { return bred64((u64)a * c, b); }
/* Shoup product by a fixed operand w (wp = floor(w 2^32 / q)): the NTT twiddles */
static inline u32 shoup_pre32(u32 w, u32 q) { return (u32)(((u64)w << 32) / q); }
static inline u32 smul(u32 a, u32 w, u32 wp, u32 q) {
    u32 t = (u32)(((u64)a * wp) >> 32);
    u32 r = a * w - t * q;
    return r >= q ? r - q : r;
}
static u32 subm(u32 a, u32 b, u32 q) { return a >= b ? a - b : a + q - b; }
static u32 powm(u32 a, u64 e, u32 q) {
    u64 r = 1, b = a % q;
    while (e) { if (e & 1) r = r * b % q; b = b * b % q; e >>= 1; }
    return (u32)r;
}
static u32 invm(u32 a, u32 q) { return powm(a, q - 2, q); }

static int is_prime32(u32 n) {
    if (n < 2) return 0;
    static const u32 small[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
    for (int i = 0; i < 12; i++) { if (n == small[i]) return 1; if (n % small[i] == 0) return 0; }
    u32 d = n - 1; int r = 0;
    while (!(d & 1)) { d >>= 1; r++; }
    static const u32 bases[] = {2, 7, 61};
    for (int i = 0; i < 3; i++) {
        u64 x = powm(bases[i], d, n);
        if (x == 1 || x == n - 1) continue;
        int comp = 1;
        for (int k = 1; k < r; k++) { x = x * x % n; if (x == n - 1) { comp = 0; break; } }
        if (comp) return 0;
    }
    return 1;
}

static u32 bitrev(u32 x, int bits) {
    u32 r = 0;
    for (int i = 0; i < bits; i++) { r = (r << 1) | (x & 1); x >>= 1; }
    return r;
}

/* psi = first x^((q-1)/2N), x = 2,3,..., whose N-th power is -1 */
static u32 find_psi(u32 q, int logn) {
    u64 twon = 2ull << logn;
    for (u32 x = 2;; x++) {
        u32 c = powm(x, (q - 1) / twon, q);
        if (powm(c, twon >> 1, q) == q - 1) return c;
    }
}

/* ------------------------------------------------------------------ */
/* PRNG: ChaCha20 block function (Bernstein 2008: 20   */
/* rounds, words 12-13 a 64-bit block counter, 14-15 a 64-bit nonce) as */
/* a PRF; a sample = the first 64 bits of block(key, ctr, stream)       */
/* ------------------------------------------------------------------ */
#define ROTL32(x, r) (((x) << (r)) | ((x) >> (32 - (r))))
#define QR(a, b, c, d)                          \
    a += b; d ^= a; d = ROTL32(d, 16);          \
    c += d; b ^= c; b = ROTL32(b, 12);          \
    a += b; d ^= a; d = ROTL32(d, 8);           \
    c += d; b ^= c; b = ROTL32(b, 7);
void orc_chacha_block(const u32 *key, u64 ctr, u64 nonce, u32 *out) {
    static const u32 sigma[4] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
    u32 in[16], x[16];
    for (int i = 0; i < 4; i++) in[i] = sigma[i];
    for (int i = 0; i < 8; i++) in[4 + i] = key[i];
    in[12] = (u32)ctr; in[13] = (u32)(ctr >> 32); in[14] = (u32)nonce; in[15] = (u32)(nonce >> 32);
    memcpy(x, in, sizeof(x));
    for (int r = 0; r < 10; r++) {
        QR(x[0], x[4], x[8], x[12]) QR(x[1], x[5], x[9], x[13]) QR(x[2], x[6], x[10], x[14]) QR(x[3], x[7], x[11], x[15])
        QR(x[0], x[5], x[10], x[15]) QR(x[1], x[6], x[11], x[12]) QR(x[2], x[7], x[8], x[13]) QR(x[3], x[4], x[9], x[14])
    }
    for (int i = 0; i < 16; i++) out[i] = x[i] + in[i];
}
static u64 prng(const u32 *key, u64 stream, u64 ctr) {
    u32 b[16];
    orc_chacha_block(key, ctr, stream, b);
    return (u64)b[0] | ((u64)b[1] << 32);
}
static void seed_key(orc_t *o, u64 seed) {
    memset(o->key, 0, sizeof(o->key));
    o->key[0] = (u32)seed; o->key[1] = (u32)(seed >> 32);
}
/* the full 256-bit key (32 bytes, little-endian words; aesfhe_create_keyed) */
void orc_set_key(void *h, const unsigned char *k) {
    orc_t *o = (orc_t *)h;
    for (int i = 0; i < 8; i++)
        o->key[i] = (u32)k[4 * i] | ((u32)k[4 * i + 1] << 8) | ((u32)k[4 * i + 2] << 16) | ((u32)k[4 * i + 3] << 24);
}
#define STREAM(kind, a, b) (((u64)(kind) << 56) | ((u64)(a) << 16) | (u64)(b))
static int ternary(u64 r) { return (int)(r % 3) - 1; }
static int cbd21(u64 r) {
    return __builtin_popcountll(r & 0x1FFFFFull) - __builtin_popcountll((r >> 21) & 0x1FFFFFull);
}
static u32 signed_to_mod(i64 v, u32 q) { i64 m = v % (i64)q; if (m < 0) m += q; return (u32)m; }

/* ------------------------------------------------------------------ */
/* parameter set                                      */
/* ------------------------------------------------------------------ */
static int prime_used(const u32 *list, int cnt, u32 p) {
    for (int i = 0; i < cnt; i++) if (list[i] == p) return 1;
    return 0;
}

void *orc_create(int logn, int L, int dnum, u64 seed) {
    orc_t *o = (orc_t *)calloc(1, sizeof(orc_t));
    o->logn = logn; o->n = 1 << logn; o->L = L; o->dnum = dnum; seed_key(o, seed); o->L1 = L;
    o->n_q = L + 3; o->n_ks = L + 2;
    o->alpha = (o->n_ks + dnum - 1) / dnum;
    o->n_p = o->alpha + 1; /* P exceeds every digit modulus by one prime */
    int tot = o->n_q + o->n_p;
    o->mod = (u32 *)calloc(tot, sizeof(u32));
    u32 *used = (u32 *)calloc(tot, sizeof(u32));
    int nused = 0;
    u64 twon = 2ull << logn;
    /* every prime lies in (2^29, 2^30) so that 4q < 2^32.
     * Largest such NTT-friendly primes: base(2), special(alpha), encryption(1). */
    const u64 PMAX = 1ull << 30, PMIN = 1ull << 29;
    u64 cand = (PMAX - 1) / twon * twon + 1;
    int want = 2 + o->n_p + 1, got = 0;
    u32 big[64];
    while (got < want) { if (cand < PMAX && is_prime32((u32)cand)) big[got++] = (u32)cand; cand -= twon; }
    o->mod[0] = big[0]; o->mod[1] = big[1];
    for (int k = 0; k < o->n_p; k++) o->mod[o->n_q + k] = big[2 + k];
    o->mod[o->n_q - 1] = big[2 + o->n_p];
    for (int i = 0; i < want; i++) used[nused++] = big[i];
    /* rescaling chain: level l drops limb l+1; delta_L = 0.9 * 2^30 and each
     * chain prime is the unused one closest to delta_l^2 / (0.9 * 2^30) */
    const double TARGET = 966367641.6;
    o->delta = (double *)calloc(L + 1, sizeof(double));
    o->delta[L] = TARGET;
    for (int l = L; l >= 1; l--) {
        double target = o->delta[l] * o->delta[l] / TARGET;
        u64 center = (u64)((target - 1.0) / (double)twon + 0.5) * twon + 1;
        u32 best = 0; double bestd = 1e300;
        for (i64 s = 0; s < 100000; s++) {
            for (int sgn = -1; sgn <= 1; sgn += 2) {
                i64 c = (i64)center + sgn * s * (i64)twon;
                if (c <= (i64)PMIN || c >= (i64)PMAX) continue;
                if (!is_prime32((u32)c) || prime_used(used, nused, (u32)c)) continue;
                double d = fabs((double)c - target);
                if (d < bestd || (d == bestd && (u32)c < best)) { bestd = d; best = (u32)c; }
            }
            if (best && (double)s * twon > bestd + twon) break;
        }
        o->mod[l + 1] = best;
        used[nused++] = best;
        o->delta[l - 1] = o->delta[l] * o->delta[l] / (double)best;
    }
    free(used);
    o->psi_rev = (u32 **)calloc(tot, sizeof(u32 *));
    o->ipsi_rev = (u32 **)calloc(tot, sizeof(u32 *));
    o->ninv = (u32 *)calloc(tot, sizeof(u32));
    for (int i = 0; i < tot; i++) {
        u32 q = o->mod[i];
        u32 psi = find_psi(q, logn), ipsi = invm(psi, q);
        o->psi_rev[i] = (u32 *)malloc(sizeof(u32) * o->n);
        o->ipsi_rev[i] = (u32 *)malloc(sizeof(u32) * o->n);
        u32 p = 1, ip = 1;
        for (int k = 0; k < o->n; k++) {
            u32 r = bitrev((u32)k, logn);
            o->psi_rev[i][r] = p; o->ipsi_rev[i][r] = ip;
            p = mulm(p, psi, q); ip = mulm(ip, ipsi, q);
        }
        o->ninv[i] = invm((u32)o->n, q);
    }
    return o;
}

/* the bootstrappable chain (params.cpp HostParams::build): single-prime levels 0..L1 as
 * above, then n_double levels each dropping a prime pair (qa closest to sqrt(want), qb
 * closest to want / qa, want = delta_l^2 / T^2), delta_L = T^2, and the transition pair at
 * level L1 + 1 (two primes closest to T).  The same "unused prime closest to" rule and the
 * same selection order, so both builders pick the same primes. */
static u32 closest_prime(u32 *used, int *nused, u64 twon, double want) {
    const u64 PMAX = 1ull << 30, PMIN = 1ull << 29;
    u64 center = (u64)((want - 1.0) / (double)twon + 0.5) * twon + 1;
    u32 best = 0; double bestd = 1e300;
    for (i64 s = 0; s < 100000; s++) {
        for (int sgn = -1; sgn <= 1; sgn += 2) {
            i64 c = (i64)center + sgn * s * (i64)twon;
            if (c <= (i64)PMIN || c >= (i64)PMAX) continue;
            if (!is_prime32((u32)c) || prime_used(used, *nused, (u32)c)) continue;
            double d = fabs((double)c - want);
            if (d < bestd || (d == bestd && (u32)c < best)) { bestd = d; best = (u32)c; }
        }
        if (best && (double)s * twon > bestd + twon) break;
    }
    if (best) used[(*nused)++] = best;
    return best;
}

void *orc_create_boot(int logn, int L1, int n_double, int dnum, u64 seed) {
    orc_t *o = (orc_t *)calloc(1, sizeof(orc_t));
    int L = L1 + n_double;
    o->logn = logn; o->n = 1 << logn; o->L = L; o->L1 = L1; o->dnum = dnum; seed_key(o, seed);
    o->n_ks = NL(o, L); o->n_q = o->n_ks + 1;
    o->alpha = (o->n_ks + dnum - 1) / dnum;
    o->n_p = o->alpha + 1;
    int tot = o->n_q + o->n_p;
    o->mod = (u32 *)calloc(tot, sizeof(u32));
    u32 *used = (u32 *)calloc(tot + 8, sizeof(u32));
    int nused = 0;
    u64 twon = 2ull << logn;
    const u64 PMAX = 1ull << 30;
    u64 cand = (PMAX - 1) / twon * twon + 1;
    int want = 2 + o->n_p + 1, got = 0;
    u32 big[96];
    while (got < want) { if (cand < PMAX && is_prime32((u32)cand)) big[got++] = (u32)cand; cand -= twon; }
    o->mod[0] = big[0]; o->mod[1] = big[1];
    for (int k = 0; k < o->n_p; k++) o->mod[o->n_q + k] = big[2 + k];
    o->mod[o->n_q - 1] = big[2 + o->n_p];
    for (int i = 0; i < want; i++) used[nused++] = big[i];
    const double T = 966367641.6;
    o->delta = (double *)calloc(L + 1, sizeof(double));
    o->delta[L1] = T;
    for (int l = L1; l >= 1; l--) {
        u32 q = closest_prime(used, &nused, twon, o->delta[l] * o->delta[l] / T);
        o->mod[l + 1] = q;
        o->delta[l - 1] = o->delta[l] * o->delta[l] / (double)q;
    }
    if (L > L1) {
        o->delta[L] = T * T;
        for (int l = L; l >= L1 + 2; l--) {
            double w = o->delta[l] * o->delta[l] / (T * T);
            u32 qa = closest_prime(used, &nused, twon, sqrt(w));
            u32 qb = closest_prime(used, &nused, twon, w / (double)qa);
            o->mod[NL(o, l) - 1] = qa;
            o->mod[NL(o, l) - 2] = qb;
            o->delta[l - 1] = o->delta[l] * o->delta[l] / ((double)qa * (double)qb);
        }
        u32 qa = closest_prime(used, &nused, twon, T), qb = closest_prime(used, &nused, twon, T);
        o->mod[NL(o, L1 + 1) - 1] = qa;
        o->mod[NL(o, L1 + 1) - 2] = qb;
    }
    free(used);
    o->psi_rev = (u32 **)calloc(tot, sizeof(u32 *));
    o->ipsi_rev = (u32 **)calloc(tot, sizeof(u32 *));
    o->ninv = (u32 *)calloc(tot, sizeof(u32));
    for (int i = 0; i < tot; i++) {
        u32 q = o->mod[i];
        u32 psi = find_psi(q, logn), ipsi = invm(psi, q);
        o->psi_rev[i] = (u32 *)malloc(sizeof(u32) * o->n);
        o->ipsi_rev[i] = (u32 *)malloc(sizeof(u32) * o->n);
        u32 p = 1, ip = 1;
        for (int k = 0; k < o->n; k++) {
            u32 r = bitrev((u32)k, logn);
            o->psi_rev[i][r] = p; o->ipsi_rev[i][r] = ip;
            p = mulm(p, psi, q); ip = mulm(ip, ipsi, q);
        }
        o->ninv[i] = invm((u32)o->n, q);
    }
    return o;
}

void orc_destroy(void *h) {
    orc_t *o = (orc_t *)h;
    if (!o) return;
    for (int i = 0; i < o->n_q + o->n_p; i++) { free(o->psi_rev[i]); free(o->ipsi_rev[i]); }
    free(o->psi_rev); free(o->ipsi_rev); free(o->ninv); free(o->mod); free(o->delta); free(o);
}

void orc_info(void *h, int *out) {
    orc_t *o = (orc_t *)h;
    out[0] = o->n; out[1] = o->L; out[2] = o->n_q; out[3] = o->n_ks;
    out[4] = o->n_p; out[5] = o->alpha; out[6] = o->dnum; out[7] = o->logn;
}
void orc_moduli(void *h, u32 *out) { orc_t *o = (orc_t *)h; memcpy(out, o->mod, sizeof(u32) * (o->n_q + o->n_p)); }
void orc_deltas(void *h, double *out) { orc_t *o = (orc_t *)h; memcpy(out, o->delta, sizeof(double) * (o->L + 1)); }

/* ------------------------------------------------------------------ */
/* negacyclic NTT: Cooley-Tukey, natural in -> bit-reversed out;       */
/* inverse: Gentleman-Sande, bit-reversed in -> natural out            */
/* ------------------------------------------------------------------ */
static void ntt_limb(const orc_t *o, int li, u32 *a) {
    u32 q = o->mod[li]; const u32 *w = o->psi_rev[li];
    int n = o->n;
    for (int m = 1, t = n >> 1; m < n; m <<= 1, t >>= 1)
        for (int i = 0; i < m; i++) {
            u32 wi = w[m + i], wp = shoup_pre32(wi, q);
            for (int j = 2 * i * t; j < 2 * i * t + t; j++) {
                u32 u = a[j], v = smul(a[j + t], wi, wp, q);
                a[j] = addm(u, v, q); a[j + t] = subm(u, v, q);
            }
        }
}
static void intt_limb(const orc_t *o, int li, u32 *a) {
    u32 q = o->mod[li]; const u32 *w = o->ipsi_rev[li];
    int n = o->n;
    for (int m = n >> 1, t = 1; m >= 1; m >>= 1, t <<= 1)
        for (int i = 0; i < m; i++) {
            u32 wi = w[m + i], wp = shoup_pre32(wi, q);
            for (int j = 2 * i * t; j < 2 * i * t + t; j++) {
                u32 u = a[j], v = a[j + t];
                a[j] = addm(u, v, q); a[j + t] = smul(subm(u, v, q), wi, wp, q);
            }
        }
    u32 ni = o->ninv[li], nip = shoup_pre32(ni, q);
    for (int j = 0; j < n; j++) a[j] = smul(a[j], ni, nip, q);
}

void orc_ntt(void *h, const int *limbs, int nl, u32 *data) {
    orc_t *o = (orc_t *)h;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < nl; i++) ntt_limb(o, limbs[i], data + (size_t)i * o->n);
}
void orc_intt(void *h, const int *limbs, int nl, u32 *data) {
    orc_t *o = (orc_t *)h;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < nl; i++) intt_limb(o, limbs[i], data + (size_t)i * o->n);
}

/* ------------------------------------------------------------------ */
/* canonical embedding                                */
/* ------------------------------------------------------------------ */
static void fft_inplace(double *re, double *im, int n, int sign) {
    for (int i = 1, j = 0; i < n; i++) {
        int bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) { double t = re[i]; re[i] = re[j]; re[j] = t; t = im[i]; im[i] = im[j]; im[j] = t; }
    }
    for (int len = 2; len <= n; len <<= 1) {
        double ang = sign * 2.0 * M_PI / len;
        for (int i = 0; i < n; i += len)
            for (int k = 0; k < len / 2; k++) {
                double wr = cos(ang * k), wi = sin(ang * k);
                double ur = re[i + k], ui = im[i + k];
                double vr = re[i + k + len / 2] * wr - im[i + k + len / 2] * wi;
                double vi = re[i + k + len / 2] * wi + im[i + k + len / 2] * wr;
                re[i + k] = ur + vr; im[i + k] = ui + vi;
                re[i + k + len / 2] = ur - vr; im[i + k + len / 2] = ui - vi;
            }
    }
}

/* real coefficients m_k (before scaling) of the polynomial whose slots are z */
void orc_embed_inverse(void *h, const double *zre, const double *zim, double *m_out) {
    orc_t *o = (orc_t *)h;
    int n = o->n, s = n / 2;
    u64 twon = 2ull * n;
    double *re = (double *)calloc(n, sizeof(double)), *im = (double *)calloc(n, sizeof(double));
    u64 e = 1;
    for (int j = 0; j < s; j++) {
        u64 t = (e - 1) / 2, tc = (twon - e - 1) / 2;
        re[t] = zre[j]; im[t] = zim[j];
        re[tc] = zre[j]; im[tc] = -zim[j];
        e = e * 5 % twon;
    }
    fft_inplace(re, im, n, -1); /* y_k = (1/N) sum_t vals[t] e^{-2 pi i t k / N} */
    for (int k = 0; k < n; k++) {
        double a = M_PI * k / n; /* y_k * zeta^{-k} */
        double yr = re[k] / n, yi = im[k] / n;
        m_out[k] = yr * cos(a) + yi * sin(a);
    }
    free(re); free(im);
}

void orc_embed(void *h, const double *m, double *zre, double *zim) {
    orc_t *o = (orc_t *)h;
    int n = o->n, s = n / 2;
    u64 twon = 2ull * n;
    double *re = (double *)malloc(sizeof(double) * n), *im = (double *)malloc(sizeof(double) * n);
    for (int k = 0; k < n; k++) { double a = M_PI * k / n; re[k] = m[k] * cos(a); im[k] = m[k] * sin(a); }
    fft_inplace(re, im, n, +1);
    u64 e = 1;
    for (int j = 0; j < s; j++) { u64 t = (e - 1) / 2; zre[j] = re[t]; zim[j] = im[t]; e = e * 5 % twon; }
    free(re); free(im);
}

static i128 round_i128(double x) {
    if (fabs(x) < 4503599627370496.0) return (i128)llround(x);
    return (i128)x;
}

/* encode z at `scale` onto limbs 0..nl-1 (NTT form) */
void orc_encode(void *h, const double *zre, const double *zim, double scale, int nl, u32 *out) {
    orc_t *o = (orc_t *)h;
    int n = o->n;
    double *m = (double *)malloc(sizeof(double) * n);
    orc_embed_inverse(h, zre, zim, m);
    for (int k = 0; k < n; k++) {
        i128 v = round_i128(m[k] * scale);
        for (int i = 0; i < nl; i++) {
            i128 r = v % (i128)o->mod[i];
            if (r < 0) r += o->mod[i];
            out[(size_t)i * n + k] = (u32)r;
        }
    }
    free(m);
    for (int i = 0; i < nl; i++) ntt_limb(o, i, out + (size_t)i * n);
}

/* ------------------------------------------------------------------ */
/* keys                                               */
/* ------------------------------------------------------------------ */
void orc_secret(void *h, int *s_out) {
    orc_t *o = (orc_t *)h;
    for (int k = 0; k < o->n; k++) s_out[k] = ternary(prng(o->key, STREAM(1, 0, 0), (u64)k));
}

/* small signed polynomial -> NTT form on global limb ids */
static void small_to_ntt(const orc_t *o, const int *c, const int *limbs, int nl, u32 *out) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < nl; i++) {
        u32 q = o->mod[limbs[i]];
        u32 *dst = out + (size_t)i * o->n;
        for (int k = 0; k < o->n; k++) dst[k] = signed_to_mod(c[k], q);
        ntt_limb(o, limbs[i], dst);
    }
}

/* secret key in NTT form on every limb (Q limbs 0..n_q-1 then P limbs) */
void orc_secret_ntt(void *h, u32 *out) {
    orc_t *o = (orc_t *)h;
    int tot = o->n_q + o->n_p;
    int *s = (int *)malloc(sizeof(int) * o->n);
    int *ids = (int *)malloc(sizeof(int) * tot);
    orc_secret(h, s);
    for (int i = 0; i < tot; i++) ids[i] = i;
    small_to_ntt(o, s, ids, tot, out);
    free(s); free(ids);
}

static void cbd_poly(const orc_t *o, u64 stream, int *c) {
    for (int k = 0; k < o->n; k++) c[k] = cbd21(prng(o->key, stream, (u64)k));
}

/* public key (b, a) over Q limbs 0..n_q-1: b = -a*s + e */
void orc_gen_pk(void *h, u32 *out) {
    orc_t *o = (orc_t *)h;
    int n = o->n, nq = o->n_q, tot = o->n_q + o->n_p;
    u32 *s = (u32 *)malloc(sizeof(u32) * (size_t)tot * n);
    orc_secret_ntt(h, s);
    int *e = (int *)malloc(sizeof(int) * n), *ids = (int *)malloc(sizeof(int) * nq);
    for (int i = 0; i < nq; i++) ids[i] = i;
    cbd_poly(o, STREAM(3, 0, 0), e);
    u32 *b = out, *a = out + (size_t)nq * n;
    small_to_ntt(o, e, ids, nq, b);
    for (int i = 0; i < nq; i++) {
        u32 q = o->mod[i];
        for (int k = 0; k < n; k++) {
            u32 av = (u32)(prng(o->key, STREAM(2, 0, 0), (u64)i * n + k) % q);
            a[(size_t)i * n + k] = av;
            b[(size_t)i * n + k] = subm(b[(size_t)i * n + k], mulm(av, s[(size_t)i * n + k], q), q);
        }
    }
    free(s); free(e); free(ids);
}

/* automorphism X -> X^g on one NTT-form limb, computed in the coefficient domain */
static void automorph_limb(const orc_t *o, int li, u64 g, const u32 *in, u32 *out) {
    int n = o->n;
    u32 q = o->mod[li];
    u32 *c = (u32 *)malloc(sizeof(u32) * n);
    memcpy(c, in, sizeof(u32) * n);
    intt_limb(o, li, c);
    u64 twon = 2ull * n;
    for (int k = 0; k < n; k++) {
        u64 e = (u64)k * g % twon;
        if (e < (u64)n) out[e] = c[k];
        else out[e - n] = c[k] ? q - c[k] : 0;
    }
    ntt_limb(o, li, out);
    free(c);
}

/* key-switching key for s' -> s, s' = s^2 (g == 0), s(X^g) (g < 2N), or s(X^g')^2 for the tag
 * g = 4N + g' (the conjugation / rotation of a 3-polynomial tensor) */
void orc_gen_ksk(void *h, u64 g, u32 *out) {
    orc_t *o = (orc_t *)h;
    int n = o->n, tot = o->n_q + o->n_p, next = o->n_ks + o->n_p;
    u32 *s = (u32 *)malloc(sizeof(u32) * (size_t)tot * n);
    orc_secret_ntt(h, s);
    int *ids = (int *)malloc(sizeof(int) * next);
    for (int i = 0; i < next; i++) ids[i] = i < o->n_ks ? i : o->n_q + (i - o->n_ks);
    /* s' on Q limbs 0..n_ks-1 */
    u32 *sp = (u32 *)malloc(sizeof(u32) * (size_t)o->n_ks * n);
    for (int i = 0; i < o->n_ks; i++) {
        u32 q = o->mod[i];
        if (g == 0) {
            for (int k = 0; k < n; k++) sp[(size_t)i * n + k] = mulm(s[(size_t)i * n + k], s[(size_t)i * n + k], q);
        } else if (g > 4ull * n && g < 6ull * n) {
            u32 *sq = (u32 *)malloc(sizeof(u32) * n);
            for (int k = 0; k < n; k++) sq[k] = mulm(s[(size_t)i * n + k], s[(size_t)i * n + k], q);
            automorph_limb(o, i, g - 4ull * n, sq, sp + (size_t)i * n);
            free(sq);
        } else {
            automorph_limb(o, i, g, s + (size_t)i * n, sp + (size_t)i * n);
        }
    }
    int *e = (int *)malloc(sizeof(int) * n);
    u32 *eN = (u32 *)malloc(sizeof(u32) * (size_t)next * n);
    for (int j = 0; j < o->dnum; j++) {
        u32 *b = out + (size_t)j * 2 * next * n, *a = b + (size_t)next * n;
        cbd_poly(o, STREAM(5, g, j), e);
        small_to_ntt(o, e, ids, next, eN);
        for (int x = 0; x < next; x++) {
            int li = ids[x];
            u32 q = o->mod[li];
            u32 pmod = 1; /* P mod q */
            for (int k = 0; k < o->n_p; k++) pmod = mulm(pmod, o->mod[o->n_q + k] % q, q);
            int in_digit = (x < o->n_ks) && (x / o->alpha == j);
            for (int k = 0; k < n; k++) {
                u32 av = (u32)(prng(o->key, STREAM(4, g, j), (u64)li * n + k) % q);
                u32 v = subm(eN[(size_t)x * n + k], mulm(av, s[(size_t)li * n + k], q), q);
                if (in_digit) v = addm(v, mulm(pmod, sp[(size_t)x * n + k], q), q);
                a[(size_t)x * n + k] = av;
                b[(size_t)x * n + k] = v;
            }
        }
    }
    free(s); free(ids); free(sp); free(e); free(eN);
}

/* ------------------------------------------------------------------ */
/* rescale: drop the last limb with rounding          */
/* in: npoly x (l+2) limbs NTT; out: npoly x (l+1) limbs NTT           */
/* ------------------------------------------------------------------ */
void orc_rescale(void *h, int level, int npoly, const u32 *in, u32 *out) {
    orc_t *o = (orc_t *)h;
    int n = o->n, nl = NL(o, level), r = nl - 1;
    u32 qr = o->mod[r];
    for (int p = 0; p < npoly; p++) {
        const u32 *src = in + (size_t)p * nl * n;
        u32 *dst = out + (size_t)p * (nl - 1) * n;
        u32 *last = (u32 *)malloc(sizeof(u32) * n);
        memcpy(last, src + (size_t)r * n, sizeof(u32) * n);
        intt_limb(o, r, last);
#pragma omp parallel for schedule(static)
        for (int t = 0; t < r; t++) {
            u32 q = o->mod[t];
            u32 *v = (u32 *)malloc(sizeof(u32) * n);
            for (int k = 0; k < n; k++) {
                i64 c = last[k];
                if (c > (i64)(qr >> 1)) c -= qr;
                v[k] = signed_to_mod(c, q);
            }
            ntt_limb(o, t, v);
            u32 qinv = invm(qr % q, q), qinvp = shoup_pre32(qinv, q);
            for (int k = 0; k < n; k++)
                dst[(size_t)t * n + k] = smul(subm(src[(size_t)t * n + k], v[k], q), qinv, qinvp, q);
            free(v);
        }
        free(last);
    }
}

/* ------------------------------------------------------------------ */
/* centred fast base conversion                       */
/* y_i in [0, q_i): u = round(sum_i y_i / q_i) from a 32-bit fixed-point */
/* estimate, mu_i = floor(2^61 / q_i); sum_i y_i qhat_i - u Q is the   */
/* centred representative of the digit (up to rare boundary ties).     */
/* ------------------------------------------------------------------ */
static u32 overflow_count(const u32 *y, size_t stride, int h, const u32 *primes) {
    u64 f = 0;
    for (int i = 0; i < h; i++) {
        u64 mu = (1ull << 61) / primes[i];
        f += ((u64)y[(size_t)i * stride] * mu) >> 29;
    }
    return (u32)((f + (1ull << 31)) >> 32);
}
/* the same for every coefficient k < n, the mu_i hoisted and the coefficients in parallel */
static void overflow_counts(const u32 *y, int n, int h, const u32 *primes, u32 *ucnt) {
    u64 mu[64];
    for (int i = 0; i < h; i++) mu[i] = (1ull << 61) / primes[i];
#pragma omp parallel for schedule(static)
    for (int k = 0; k < n; k++) {
        u64 f = 0;
        for (int i = 0; i < h; i++) f += ((u64)y[(size_t)i * n + k] * mu[i]) >> 29;
        ucnt[k] = (u32)((f + (1ull << 31)) >> 32);
    }
}

/* ------------------------------------------------------------------ */
/* hybrid key switching                               */
/* d: (l+2) limbs NTT form; out: 2 x (l+2) limbs NTT form              */
/* ------------------------------------------------------------------ */
void orc_keyswitch(void *h, int level, const u32 *d, const u32 *ksk, u32 *out) {
    orc_t *o = (orc_t *)h;
    int n = o->n, nl = NL(o, level), np = o->n_p, next_key = o->n_ks + o->n_p;
    int ne = nl + np; /* extended basis: Q limbs 0..nl-1, then P */
    int *gid = (int *)malloc(sizeof(int) * ne);  /* global prime index */
    int *kid = (int *)malloc(sizeof(int) * ne);  /* key limb index */
    for (int x = 0; x < ne; x++) {
        gid[x] = x < nl ? x : o->n_q + (x - nl);
        kid[x] = x < nl ? x : o->n_ks + (x - nl);
    }
    u32 *acc = (u32 *)calloc((size_t)2 * ne * n, sizeof(u32));
    u32 *ext = (u32 *)malloc(sizeof(u32) * (size_t)ne * n);
    u32 *coef = (u32 *)malloc(sizeof(u32) * (size_t)nl * n);
    memcpy(coef, d, sizeof(u32) * (size_t)nl * n);
#pragma omp parallel for schedule(static)
    for (int i = 0; i < nl; i++) intt_limb(o, i, coef + (size_t)i * n);
    int ndig = (nl + o->alpha - 1) / o->alpha;
    for (int j = 0; j < ndig; j++) {
        int lo = j * o->alpha, hi = lo + o->alpha < nl ? lo + o->alpha : nl;
        /* y_i = coef_i * (qhat_i^-1 mod q_i), qhat_i = prod_{k in digit, k != i} q_k */
        u32 *y = (u32 *)malloc(sizeof(u32) * (size_t)(hi - lo) * n);
#pragma omp parallel for schedule(static)
        for (int i = lo; i < hi; i++) {
            u32 q = o->mod[i], qh = 1;
            for (int k = lo; k < hi; k++) if (k != i) qh = mulm(qh, o->mod[k] % q, q);
            u32 qhi = invm(qh, q), qhip = shoup_pre32(qhi, q);
            for (int k = 0; k < n; k++) y[(size_t)(i - lo) * n + k] = smul(coef[(size_t)i * n + k], qhi, qhip, q);
        }
        u32 *ucnt = (u32 *)malloc(sizeof(u32) * n);
        overflow_counts(y, n, hi - lo, o->mod + lo, ucnt);
#pragma omp parallel for schedule(static)
        for (int x = 0; x < ne; x++) {
            u32 *dst = ext + (size_t)x * n;
            if (x >= lo && x < hi) { memcpy(dst, d + (size_t)x * n, sizeof(u32) * n); continue; }
            u32 t = o->mod[gid[x]];
            u32 *qh_t = (u32 *)malloc(sizeof(u32) * (hi - lo));
            for (int i = lo; i < hi; i++) {
                u32 v = 1;
                for (int k = lo; k < hi; k++) if (k != i) v = mulm(v, o->mod[k] % t, t);
                qh_t[i - lo] = v;
            }
            u32 negQ = 1; /* -Q_j mod t */
            for (int k = lo; k < hi; k++) negQ = mulm(negQ, o->mod[k] % t, t);
            negQ = negQ ? t - negQ : 0;
            barrett_t bt = bq_make(t);
            for (int k = 0; k < n; k++) {
                u128 s = (u64)ucnt[k] * negQ;
                for (int i = lo; i < hi; i++) s += (u64)y[(size_t)(i - lo) * n + k] * qh_t[i - lo];
                dst[k] = bred128(s, &bt);
            }
            free(qh_t);
            ntt_limb(o, gid[x], dst);
        }
        free(y); free(ucnt);
        const u32 *kb = ksk + (size_t)j * 2 * next_key * n, *ka = kb + (size_t)next_key * n;
#pragma omp parallel for schedule(static)
        for (int x = 0; x < ne; x++) {
            u32 t = o->mod[gid[x]];
            barrett_t bt = bq_make(t);
            for (int k = 0; k < n; k++) {
                u32 e = ext[(size_t)x * n + k];
                acc[(size_t)x * n + k] = bred64((u64)acc[(size_t)x * n + k] + (u64)e * kb[(size_t)kid[x] * n + k], &bt);
                acc[(size_t)(ne + x) * n + k] = bred64((u64)acc[(size_t)(ne + x) * n + k] + (u64)e * ka[(size_t)kid[x] * n + k], &bt);
            }
        }
    }
    /* ModDown by P */
    for (int p = 0; p < 2; p++) {
        u32 *a = acc + (size_t)p * ne * n;
        u32 *yp = (u32 *)malloc(sizeof(u32) * (size_t)np * n);
#pragma omp parallel for schedule(static)
        for (int k2 = 0; k2 < np; k2++) {
            int g = o->n_q + k2;
            u32 q = o->mod[g], ph = 1;
            for (int m = 0; m < np; m++) if (m != k2) ph = mulm(ph, o->mod[o->n_q + m] % q, q);
            u32 phi = invm(ph, q), phip = shoup_pre32(phi, q);
            memcpy(yp + (size_t)k2 * n, a + (size_t)(nl + k2) * n, sizeof(u32) * n);
            intt_limb(o, g, yp + (size_t)k2 * n);
            for (int k = 0; k < n; k++) yp[(size_t)k2 * n + k] = smul(yp[(size_t)k2 * n + k], phi, phip, q);
        }
        u32 *ucnt = (u32 *)malloc(sizeof(u32) * n);
        overflow_counts(yp, n, np, o->mod + o->n_q, ucnt);
#pragma omp parallel for schedule(static)
        for (int t = 0; t < nl; t++) {
            u32 q = o->mod[t];
            u32 *ph_t = (u32 *)malloc(sizeof(u32) * np);
            u32 pinv = 1;
            for (int k2 = 0; k2 < np; k2++) {
                u32 v = 1;
                for (int m = 0; m < np; m++) if (m != k2) v = mulm(v, o->mod[o->n_q + m] % q, q);
                ph_t[k2] = v;
                pinv = mulm(pinv, o->mod[o->n_q + k2] % q, q);
            }
            u32 negP = pinv ? q - pinv : 0; /* -P mod q */
            pinv = invm(pinv, q);
            barrett_t bt = bq_make(q);
            u32 *conv = (u32 *)malloc(sizeof(u32) * n);
            for (int k = 0; k < n; k++) {
                u128 s = (u64)ucnt[k] * negP;
                for (int k2 = 0; k2 < np; k2++) s += (u64)yp[(size_t)k2 * n + k] * ph_t[k2];
                conv[k] = bred128(s, &bt);
            }
            ntt_limb(o, t, conv);
            u32 *dst = out + (size_t)p * nl * n + (size_t)t * n;
            u32 pinvp = shoup_pre32(pinv, q);
            for (int k = 0; k < n; k++) dst[k] = smul(subm(a[(size_t)t * n + k], conv[k], q), pinv, pinvp, q);
            free(conv); free(ph_t);
        }
        free(yp); free(ucnt);
    }
    free(gid); free(kid); free(acc); free(ext); free(coef);
}

/* ------------------------------------------------------------------ */
/* double-prime rescale (bootstrapping region): divide by  */
/* the two dropped primes at once.  qa = the last limb, qb = the one    */
/* before; X = xa + qa ((xb - xa) qa^-1 mod qb) in [0, qa qb), centred; */
/* out_t = (in_t - X mod q_t) (qa qb)^-1.  in: npoly x nl(l) limbs NTT. */
/* ------------------------------------------------------------------ */
void orc_rescale2(void *h, int level, int npoly, const u32 *in, u32 *out) {
    orc_t *o = (orc_t *)h;
    int n = o->n, nl = NL(o, level), r = nl - 2;
    u32 qa = o->mod[nl - 1], qb = o->mod[nl - 2];
    u32 ainv = invm(qa % qb, qb);
    u64 Q = (u64)qa * qb;
    for (int p = 0; p < npoly; p++) {
        const u32 *src = in + (size_t)p * nl * n;
        u32 *dst = out + (size_t)p * r * n;
        u32 *xa = (u32 *)malloc(sizeof(u32) * n), *xb = (u32 *)malloc(sizeof(u32) * n);
        memcpy(xa, src + (size_t)(nl - 1) * n, sizeof(u32) * n);
        memcpy(xb, src + (size_t)(nl - 2) * n, sizeof(u32) * n);
        intt_limb(o, nl - 1, xa);
        intt_limb(o, nl - 2, xb);
        i64 *X = (i64 *)malloc(sizeof(i64) * n);
        for (int k = 0; k < n; k++) {
            u32 d = subm(xb[k], xa[k] % qb, qb);
            u64 x = (u64)xa[k] + (u64)qa * mulm(d, ainv, qb);
            X[k] = x > Q / 2 ? (i64)x - (i64)Q : (i64)x;
        }
#pragma omp parallel for schedule(static)
        for (int t = 0; t < r; t++) {
            u32 q = o->mod[t];
            u32 *v = (u32 *)malloc(sizeof(u32) * n);
            for (int k = 0; k < n; k++) v[k] = signed_to_mod(X[k], q);
            ntt_limb(o, t, v);
            u32 qinv = invm(mulm(qa % q, qb % q, q), q);
            for (int k = 0; k < n; k++)
                dst[(size_t)t * n + k] = mulm(subm(src[(size_t)t * n + k], v[k], q), qinv, q);
            free(v);
        }
        free(xa); free(xb); free(X);
    }
}

/* ------------------------------------------------------------------ */
/* dense -> sparse key switch of the bootstrap:    */
/* modulus Q0 P' with Q0 = q0 q1 (one digit) and P' = the first np      */
/* special primes.  d: c1 on (q0, q1), NTT form; ksk [2][2 + np][N];    */
/* out [2][2][N] = key-switched (c0', c1') (c0 not added).              */
/* ------------------------------------------------------------------ */
void orc_keyswitch_d2s(void *h, int np, const u32 *d, const u32 *ksk, u32 *out) {
    orc_t *o = (orc_t *)h;
    int n = o->n, nq = 2, ne = nq + np;
    int gid[64];
    for (int x = 0; x < ne; x++) gid[x] = x < nq ? x : o->n_q + (x - nq);
    u32 *coef = (u32 *)malloc(sizeof(u32) * (size_t)nq * n);
    memcpy(coef, d, sizeof(u32) * (size_t)nq * n);
    for (int i = 0; i < nq; i++) intt_limb(o, i, coef + (size_t)i * n);
    u32 *y = (u32 *)malloc(sizeof(u32) * (size_t)nq * n);
    for (int i = 0; i < nq; i++) {
        u32 q = o->mod[i], qh = o->mod[1 - i] % q, qhi = invm(qh, q);
        for (int k = 0; k < n; k++) y[(size_t)i * n + k] = mulm(coef[(size_t)i * n + k], qhi, q);
    }
    u32 *ucnt = (u32 *)malloc(sizeof(u32) * n);
    for (int k = 0; k < n; k++) ucnt[k] = overflow_count(y + k, n, nq, o->mod);
    u32 *ext = (u32 *)malloc(sizeof(u32) * (size_t)ne * n);
    for (int x = 0; x < ne; x++) {
        u32 *dst = ext + (size_t)x * n;
        if (x < nq) { memcpy(dst, d + (size_t)x * n, sizeof(u32) * n); continue; }
        u32 t = o->mod[gid[x]];
        u32 qh0 = o->mod[1] % t, qh1 = o->mod[0] % t;
        u32 negQ = mulm(o->mod[0] % t, o->mod[1] % t, t);
        negQ = negQ ? t - negQ : 0;
        barrett_t bt = bq_make(t);
        for (int k = 0; k < n; k++) {
            u128 s = (u64)ucnt[k] * negQ;
            s += (u64)y[k] * qh0;
            s += (u64)y[(size_t)n + k] * qh1;
            dst[k] = bred128(s, &bt);
        }
        ntt_limb(o, gid[x], dst);
    }
    u32 *acc = (u32 *)calloc((size_t)2 * ne * n, sizeof(u32));
    const u32 *kb = ksk, *ka = ksk + (size_t)ne * n;
    for (int x = 0; x < ne; x++) {
        u32 t = o->mod[gid[x]];
        for (int k = 0; k < n; k++) {
            u32 e = ext[(size_t)x * n + k];
            acc[(size_t)x * n + k] = mulm(e, kb[(size_t)x * n + k], t);
            acc[(size_t)(ne + x) * n + k] = mulm(e, ka[(size_t)x * n + k], t);
        }
    }
    /* ModDown by P' onto (q0, q1) */
    for (int p = 0; p < 2; p++) {
        u32 *a = acc + (size_t)p * ne * n;
        u32 *yp = (u32 *)malloc(sizeof(u32) * (size_t)np * n);
        for (int k2 = 0; k2 < np; k2++) {
            int g = o->n_q + k2;
            u32 q = o->mod[g], ph = 1;
            for (int m = 0; m < np; m++) if (m != k2) ph = mulm(ph, o->mod[o->n_q + m] % q, q);
            u32 phi = invm(ph, q);
            memcpy(yp + (size_t)k2 * n, a + (size_t)(nq + k2) * n, sizeof(u32) * n);
            intt_limb(o, g, yp + (size_t)k2 * n);
            for (int k = 0; k < n; k++) yp[(size_t)k2 * n + k] = mulm(yp[(size_t)k2 * n + k], phi, q);
        }
        u32 *uc = (u32 *)malloc(sizeof(u32) * n);
        overflow_counts(yp, n, np, o->mod + o->n_q, uc);
        for (int t = 0; t < nq; t++) {
            u32 q = o->mod[t], pinv = 1;
            u32 ph_t[16];
            for (int k2 = 0; k2 < np; k2++) {
                u32 v = 1;
                for (int m = 0; m < np; m++) if (m != k2) v = mulm(v, o->mod[o->n_q + m] % q, q);
                ph_t[k2] = v;
                pinv = mulm(pinv, o->mod[o->n_q + k2] % q, q);
            }
            u32 negP = pinv ? q - pinv : 0;
            pinv = invm(pinv, q);
            barrett_t bt = bq_make(q);
            u32 *conv = (u32 *)malloc(sizeof(u32) * n);
            for (int k = 0; k < n; k++) {
                u128 s = (u64)uc[k] * negP;
                for (int k2 = 0; k2 < np; k2++) s += (u64)yp[(size_t)k2 * n + k] * ph_t[k2];
                conv[k] = bred128(s, &bt);
            }
            ntt_limb(o, t, conv);
            u32 *dst = out + (size_t)p * nq * n + (size_t)t * n;
            for (int k = 0; k < n; k++) dst[k] = mulm(subm(a[(size_t)t * n + k], conv[k], q), pinv, q);
            free(conv);
        }
        free(yp); free(uc);
    }
    free(coef); free(y); free(ucnt); free(ext); free(acc);
}

/* ------------------------------------------------------------------ */
/* ciphertext-level primitives                                         */
/* ------------------------------------------------------------------ */
/* (a0,a1) x (b0,b1) -> (d0,d1,d2), level l, NTT form */
void orc_tensor(void *h, int level, const u32 *a, const u32 *b, u32 *out) {
    orc_t *o = (orc_t *)h;
    int n = o->n, nl = NL(o, level);
    size_t P = (size_t)nl * n;
#pragma omp parallel for schedule(static)
    for (int t = 0; t < nl; t++) {
        barrett_t bt = bq_make(o->mod[t]);
        for (int k = 0; k < n; k++) {
            size_t x = (size_t)t * n + k;
            out[x] = bmul(a[x], b[x], &bt);
            out[P + x] = bred64((u64)a[x] * b[P + x] + (u64)a[P + x] * b[x], &bt);
            out[2 * P + x] = bmul(a[P + x], b[P + x], &bt);
        }
    }
}

/* multiply every limb t of npoly polys (nl limbs) by the plaintext polynomial pt (nl limbs), NTT form:
 * a linear transform's diagonal product (the CPU baseline's bootstrap replay, bench.py) */
void orc_mul_poly(void *h, int nl, int npoly, const u32 *pt, const u32 *in, u32 *out) {
    orc_t *o = (orc_t *)h;
    int n = o->n;
#pragma omp parallel for collapse(2) schedule(static)
    for (int p = 0; p < npoly; p++)
        for (int t = 0; t < nl; t++) {
            barrett_t bt = bq_make(o->mod[t]);
            for (int k = 0; k < n; k++) {
                size_t x = ((size_t)p * nl + t) * n + k;
                out[x] = bmul(in[x], pt[(size_t)t * n + k], &bt);
            }
        }
}

/* multiply every limb t of npoly polys by c_t (per-limb constants) */
void orc_mul_limb_consts(void *h, int nl, int npoly, const u32 *c, const u32 *in, u32 *out) {
    orc_t *o = (orc_t *)h;
    int n = o->n;
#pragma omp parallel for collapse(2) schedule(static)
    for (int p = 0; p < npoly; p++)
        for (int t = 0; t < nl; t++) {
            u32 q = o->mod[t], cp = shoup_pre32(c[t], q);
            for (int k = 0; k < n; k++) {
                size_t x = ((size_t)p * nl + t) * n + k;
                out[x] = smul(in[x], c[t], cp, q);
            }
        }
}

/* automorphism of a ciphertext-like array (npoly x (l+2) limbs), NTT form */
void orc_automorph(void *h, int level, u64 g, int npoly, const u32 *in, u32 *out) {
    orc_t *o = (orc_t *)h;
    int n = o->n, nl = NL(o, level);
    for (int p = 0; p < npoly; p++)
#pragma omp parallel for schedule(static)
        for (int t = 0; t < nl; t++)
            automorph_limb(o, t, g, in + ((size_t)p * nl + t) * n, out + ((size_t)p * nl + t) * n);
}

/* public-key encryption at fresh level f: the plaintext is given on
 * limbs 0..f+2 (NTT form, encoded at scale delta[f] * q_{f+2}); the ciphertext is
 * formed at level f+1 and rescaled to level f */
void orc_encrypt(void *h, int f, const u32 *pt, const u32 *pk, u64 ctr, u32 *out) {
    orc_t *o = (orc_t *)h;
    int n = o->n, nq = f + 3, npk = o->n_q;
    if (NL(o, f + 1) != nq) abort();  /* level f + 1 must be single-prime (or the transient L + 1) */
    size_t P = (size_t)nq * n, PK = (size_t)npk * n;
    int *ids = (int *)malloc(sizeof(int) * nq);
    for (int i = 0; i < nq; i++) ids[i] = i;
    int *v = (int *)malloc(sizeof(int) * n), *e = (int *)malloc(sizeof(int) * n);
    u32 *vN = (u32 *)malloc(sizeof(u32) * P), *e0 = (u32 *)malloc(sizeof(u32) * P), *e1 = (u32 *)malloc(sizeof(u32) * P);
    for (int k = 0; k < n; k++) v[k] = ternary(prng(o->key, STREAM(6, 0, ctr), (u64)k));
    small_to_ntt(o, v, ids, nq, vN);
    cbd_poly(o, STREAM(7, 0, ctr), e); small_to_ntt(o, e, ids, nq, e0);
    cbd_poly(o, STREAM(8, 0, ctr), e); small_to_ntt(o, e, ids, nq, e1);
    u32 *tmp = (u32 *)malloc(sizeof(u32) * 2 * P);
    for (int t = 0; t < nq; t++) {
        u32 q = o->mod[t];
        for (int k = 0; k < n; k++) {
            size_t x = (size_t)t * n + k;
            tmp[x] = addm(addm(mulm(vN[x], pk[x], q), e0[x], q), pt[x], q);
            tmp[P + x] = addm(mulm(vN[x], pk[PK + x], q), e1[x], q);
        }
    }
    orc_rescale(h, f + 1, 2, tmp, out);
    free(ids); free(v); free(e); free(vN); free(e0); free(e1); free(tmp);
}

/* decrypt at level l: returns real coefficient vector (message * delta_l, as double) */
void orc_decrypt_coeffs(void *h, int level, int npoly, const u32 *ct, const u32 *s_ntt, double *m_out) {
    orc_t *o = (orc_t *)h;
    int n = o->n, nl = NL(o, level);
    u32 *x = (u32 *)malloc(sizeof(u32) * 2 * n);
    for (int t = 0; t < 2; t++) {
        u32 q = o->mod[t];
        for (int k = 0; k < n; k++) {
            size_t idx = (size_t)t * n + k;
            u32 acc = ct[idx], spow = s_ntt[idx];
            for (int p = 1; p < npoly; p++) {
                acc = addm(acc, mulm(ct[(size_t)p * nl * n + idx], spow, q), q);
                spow = mulm(spow, s_ntt[idx], q);
            }
            x[idx] = acc;
        }
        intt_limb(o, t, x + (size_t)t * n);
    }
    u32 q0 = o->mod[0], q1 = o->mod[1];
    u32 q0inv = invm(q0 % q1, q1);
    u64 Q = (u64)q0 * q1;
    for (int k = 0; k < n; k++) {
        u32 a = x[k], b = x[n + k];
        u64 t = mulm(subm(b, a % q1, q1), q0inv, q1);
        u64 v = (u64)a + t * q0;
        i64 sv = v > Q / 2 ? (i64)v - (i64)Q : (i64)v;
        m_out[k] = (double)sv;
    }
    free(x);
}

/* exact integer constant multiply helpers for tests */
void orc_const_residues(void *h, i64 c, int nl, u32 *out) {
    orc_t *o = (orc_t *)h;
    for (int t = 0; t < nl; t++) out[t] = signed_to_mod(c, o->mod[t]);
}
