/*
 * oracle/sanitize_main.c -- TEST INFRASTRUCTURE: drives every entry point of
 * oracle/ckks_oracle.c once, with the buffer shapes oracle/ckks_cpu.py passes, so that a
 * build under -fsanitize=address,undefined (tests/test_oracle_sanitize.py) checks the
 * oracle's memory accesses and integer arithmetic on the plain chain (N = 2^13, L = 4) and
 * on the bootstrappable chain (L1 = 5, 13 double-prime levels).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32;
typedef uint64_t u64;
typedef int64_t i64;

void *orc_create(int logn, int L, int dnum, u64 seed);
void *orc_create_boot(int logn, int L1, int n_double, int dnum, u64 seed);
void orc_destroy(void *h);
void orc_info(void *h, int *out);
void orc_moduli(void *h, u32 *out);
void orc_deltas(void *h, double *out);
void orc_ntt(void *h, const int *limbs, int nl, u32 *data);
void orc_intt(void *h, const int *limbs, int nl, u32 *data);
void orc_embed_inverse(void *h, const double *zre, const double *zim, double *m_out);
void orc_embed(void *h, const double *m, double *zre, double *zim);
void orc_encode(void *h, const double *zre, const double *zim, double scale, int nl, u32 *out);
void orc_secret(void *h, int *s_out);
void orc_secret_ntt(void *h, u32 *out);
void orc_gen_pk(void *h, u32 *out);
void orc_gen_ksk(void *h, u64 g, u32 *out);
void orc_rescale(void *h, int level, int npoly, const u32 *in, u32 *out);
void orc_keyswitch(void *h, int level, const u32 *d, const u32 *ksk, u32 *out);
void orc_rescale2(void *h, int level, int npoly, const u32 *in, u32 *out);
void orc_keyswitch_d2s(void *h, int np, const u32 *d, const u32 *ksk, u32 *out);
void orc_tensor(void *h, int level, const u32 *a, const u32 *b, u32 *out);
void orc_mul_limb_consts(void *h, int nl, int npoly, const u32 *c, const u32 *in, u32 *out);
void orc_mul_poly(void *h, int nl, int npoly, const u32 *pt, const u32 *in, u32 *out);
void orc_automorph(void *h, int level, u64 g, int npoly, const u32 *in, u32 *out);
void orc_encrypt(void *h, int f, const u32 *pt, const u32 *pk, u64 ctr, u32 *out);
void orc_decrypt_coeffs(void *h, int level, int npoly, const u32 *ct, const u32 *s_ntt, double *m_out);
void orc_const_residues(void *h, i64 c, int nl, u32 *out);

static u64 rs = 0x9E3779B97F4A7C15ull;
static u64 rnd(void) {
    rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17;
    return rs;
}

typedef struct {
    void *h;
    int n, L, L1, n_q, n_ks, n_p, alpha, dnum;
    u32 *mod;
} chain_t;

static int nl_of(const chain_t *c, int l) {
    if (l > c->L) return nl_of(c, c->L) + 1;
    return l <= c->L1 ? l + 2 : c->L1 + 2 + 2 * (l - c->L1);
}

static u32 *xalloc(size_t words) {
    u32 *p = (u32 *)calloc(words, sizeof(u32));
    if (!p) { fprintf(stderr, "out of memory\n"); exit(2); }
    return p;
}

/* npoly polynomials of nl limbs, each limb reduced mod its prime */
static u32 *rand_poly(const chain_t *c, int npoly, int nl) {
    u32 *p = xalloc((size_t)npoly * nl * c->n);
    for (int k = 0; k < npoly; k++)
        for (int t = 0; t < nl; t++)
            for (int i = 0; i < c->n; i++) p[((size_t)k * nl + t) * c->n + i] = (u32)(rnd() % c->mod[t]);
    return p;
}

static void open_chain(chain_t *c, void *h, int L1) {
    int info[8];
    c->h = h;
    orc_info(h, info);
    c->n = info[0]; c->L = info[1]; c->n_q = info[2]; c->n_ks = info[3];
    c->n_p = info[4]; c->alpha = info[5]; c->dnum = info[6]; c->L1 = L1;
    c->mod = xalloc(c->n_q + c->n_p);
    orc_moduli(h, c->mod);
}

static void exercise(chain_t *c) {
    const int n = c->n, ne = c->n_ks + c->n_p, L = c->L;
    double *delta = (double *)calloc(L + 1, sizeof(double));
    orc_deltas(c->h, delta);
    /* transforms on every prime */
    int *ids = (int *)calloc(c->n_q + c->n_p, sizeof(int));
    for (int t = 0; t < c->n_q + c->n_p; t++) ids[t] = t;
    u32 *all = rand_poly(c, 1, c->n_q + c->n_p);
    orc_ntt(c->h, ids, c->n_q + c->n_p, all);
    orc_intt(c->h, ids, c->n_q + c->n_p, all);
    /* encoding */
    double *zr = (double *)calloc(n / 2, sizeof(double)), *zi = (double *)calloc(n / 2, sizeof(double));
    double *m = (double *)calloc(n, sizeof(double));
    for (int i = 0; i < n / 2; i++) { zr[i] = (double)(rnd() % 1000) / 1000.0; zi[i] = -zr[i]; }
    orc_embed_inverse(c->h, zr, zi, m);
    orc_embed(c->h, m, zr, zi);
    const int f = c->L1 < L ? c->L1 - 2 : L;  /* the engine's fresh level on a bootstrappable chain */
    u32 *pt = xalloc((size_t)nl_of(c, f + 1) * n);
    orc_encode(c->h, zr, zi, delta[f] * (double)c->mod[nl_of(c, f)], nl_of(c, f + 1), pt);
    /* keys */
    int *s = (int *)calloc(n, sizeof(int));
    orc_secret(c->h, s);
    u32 *sn = xalloc((size_t)(c->n_q + c->n_p) * n);
    orc_secret_ntt(c->h, sn);
    u32 *pk = xalloc((size_t)2 * c->n_q * n);
    orc_gen_pk(c->h, pk);
    u32 *ksk = xalloc((size_t)c->dnum * 2 * ne * n);
    orc_gen_ksk(c->h, 0, ksk);
    /* encrypt at f, decrypt */
    u32 *ct = xalloc((size_t)2 * nl_of(c, f) * n);
    orc_encrypt(c->h, f, pt, pk, 1, ct);
    orc_decrypt_coeffs(c->h, f, 2, ct, sn, m);
    /* per level: key switch, tensor, automorphism, constant and polynomial products, rescale (single or double prime) */
    for (int l = 0; l <= L; l++) {
        const int nl = nl_of(c, l);
        u32 *a = rand_poly(c, 2, nl), *b = rand_poly(c, 2, nl);
        u32 *o3 = xalloc((size_t)3 * nl * n), *o2 = xalloc((size_t)2 * nl * n);
        orc_keyswitch(c->h, l, a + (size_t)nl * n, ksk, o2);
        orc_tensor(c->h, l, a, b, o3);
        orc_automorph(c->h, l, 5, 2, a, o2);
        u32 *cs = xalloc(nl);
        orc_const_residues(c->h, -12345, nl, cs);
        orc_mul_limb_consts(c->h, nl, 2, cs, a, o2);
        orc_mul_poly(c->h, nl, 2, b, a, o2);
        if (l >= 1 && l <= c->L1) orc_rescale(c->h, l, 2, a, o2);
        if (l > c->L1) orc_rescale2(c->h, l, 2, a, o2);
        free(a); free(b); free(o3); free(o2); free(cs);
    }
    free(delta); free(ids); free(all); free(zr); free(zi); free(m); free(pt); free(s); free(sn); free(pk);
    free(ksk); free(ct);
}

int main(void) {
    chain_t c;
    open_chain(&c, orc_create(13, 4, 3, 7), 4);
    exercise(&c);
    orc_destroy(c.h);
    free(c.mod);

    const int L1 = 5, nd = 13, npd = 2;
    open_chain(&c, orc_create_boot(13, L1, nd, 5, 7), L1);
    exercise(&c);
    u32 *key = xalloc((size_t)2 * (2 + npd) * c.n);
    for (int k = 0; k < 2; k++)
        for (int t = 0; t < 2 + npd; t++) {
            const u32 q = c.mod[t < 2 ? t : c.n_q + (t - 2)];
            for (int i = 0; i < c.n; i++) key[((size_t)k * (2 + npd) + t) * c.n + i] = (u32)(rnd() % q);
        }
    u32 *d = rand_poly(&c, 1, 2), *out = xalloc((size_t)4 * c.n);
    orc_keyswitch_d2s(c.h, npd, d, key, out);
    free(key); free(d); free(out);
    orc_destroy(c.h);
    free(c.mod);
    printf("oracle sanitize run ok\n");
    return 0;
}
