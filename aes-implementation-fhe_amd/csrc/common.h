// common.h -- shared types and 32-bit modular arithmetic for the MI355X CKKS engine.
//
// Every RNS prime q lies in (2^29, 2^30), which lets all modular
// products run on 32-bit VALU multiplies (v_mul_lo_u32 / v_mul_hi_u32) with no 64-bit
// emulation:
//   * Shoup    (constant operand w, w' = floor(w*2^32/q)):  3 multiplies, result < 2q
//   * Barrett  (two variable operands, mu = floor(2^61/q)): 4 multiplies, result < 3q
// 4q < 2^32, so the wrapped 32-bit differences below are exact, and the NTT keeps its
// residues lazily in [0, 4q) between butterflies (Harvey; ntt.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

typedef uint32_t u32;
typedef uint64_t u64;
typedef int64_t i64;

#define HD __host__ __device__ __forceinline__

HD u32 mulhi32(u32 a, u32 b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umulhi(a, b);
#else
    return (u32)(((u64)a * b) >> 32);
#endif
}

HD u32 csub(u32 x, u32 q) { return x >= q ? x - q : x; }
HD u32 add_mod(u32 a, u32 b, u32 q) { return csub(a + b, q); }
HD u32 sub_mod(u32 a, u32 b, u32 q) { return csub(a + q - b, q); }

// a * w mod q, w' = floor(w * 2^32 / q) precomputed; a < 2^32 (any), result in [0, q)
HD u32 shoup_mul(u32 a, u32 w, u32 wp, u32 q) {
    u32 qh = mulhi32(a, wp);
    u32 r = a * w - qh * q;
    return csub(r, q);
}
HD u32 shoup_pre(u32 w, u32 q) { return (u32)(((u64)w << 32) / q); }
// the same floor(w 2^32 / q) for w < q without a 64-bit division: mu = floor(2^61 / q) gives an
// estimate at most 3 below (w mu / 2^29 = w 2^32 / q - w eps / 2^29, w < 2^30, eps < 1, plus the
// shift's floor), then exact corrections
HD u32 shoup_pre_mu(u32 w, u32 q, u32 mu) {
    u32 est = (u32)(((u64)w * mu) >> 29);
    u64 r = ((u64)w << 32) - (u64)est * q;
#pragma unroll
    for (int i = 0; i < 3; ++i)
        if (r >= q) r -= q, ++est;
    return est;
}

// a * b mod q for a, b < q; mu = floor(2^61 / q) (fits 32 bits since q > 2^29)
HD u32 barrett_mul(u32 a, u32 b, u32 q, u32 mu) {
    u32 lo = a * b, hi = mulhi32(a, b);
    u32 t = (hi << 3) | (lo >> 29);          // floor(a*b / 2^29) < 2^31
    u32 qh = mulhi32(t, mu);                  // within 2 of floor(a*b/q)
    u32 r = lo - qh * q;                      // < 3q < 2^32
    r = csub(r, q);
    return csub(r, q);
}
HD u32 barrett_pre(u32 q) { return (u32)((1ull << 61) / q); }

// ---------------------------------------------------------------------------------
// Randomness: ChaCha20 (Bernstein 2008; 20 rounds, 64-bit block counter and
// 64-bit nonce) as a counter-mode PRF.  A sample is the first 64 bits of the block with
// key = the context's 256-bit key, counter = the sample index, nonce = the stream id (what is
// sampled: secret, pk, key-switch key g/digit, encryption counter, ...); every coefficient is
// an independent block, so any thread computes its own sample with no state.
// ---------------------------------------------------------------------------------
struct PrngKey {
    u32 w[8];
};
HD u32 rotl32(u32 x, int r) { return (x << r) | (x >> (32 - r)); }
HD void chacha_qr(u32& a, u32& b, u32& c, u32& d) {
    a += b; d ^= a; d = rotl32(d, 16);
    c += d; b ^= c; b = rotl32(b, 12);
    a += b; d ^= a; d = rotl32(d, 8);
    c += d; b ^= c; b = rotl32(b, 7);
}
HD u64 chacha_u64(const PrngKey& k, u64 stream, u64 ctr) {
    u32 x[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, k.w[0], k.w[1], k.w[2], k.w[3],
                 k.w[4],      k.w[5],      k.w[6],      k.w[7],      (u32)ctr, (u32)(ctr >> 32), (u32)stream,
                 (u32)(stream >> 32)};
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        chacha_qr(x[0], x[4], x[8], x[12]);
        chacha_qr(x[1], x[5], x[9], x[13]);
        chacha_qr(x[2], x[6], x[10], x[14]);
        chacha_qr(x[3], x[7], x[11], x[15]);
        chacha_qr(x[0], x[5], x[10], x[15]);
        chacha_qr(x[1], x[6], x[11], x[12]);
        chacha_qr(x[2], x[7], x[8], x[13]);
        chacha_qr(x[3], x[4], x[9], x[14]);
    }
    return (u64)(x[0] + 0x61707865u) | ((u64)(x[1] + 0x3320646eu) << 32);
}

// reduce a 64-bit accumulator (x < 2^61) with the Barrett constant
HD u32 barrett_reduce64(u64 x, u32 q, u32 mu) {
    u32 lo = (u32)x, hi = (u32)(x >> 32);
    u32 t = (hi << 3) | (lo >> 29);
    u32 qh = mulhi32(t, mu);
    u32 r = lo - qh * q;
    r = csub(r, q);
    return csub(r, q);
}

// fold a full 64-bit accumulator below 2^61 (x mod q unchanged); r32 = 2^32 mod q.
// hi < 2^32 < 8q -> hi < 2q after two steps; 2q r32 + 2^32 < 1.6 * 2^60 + 2^32 for every
// q in (2^29, 2^30) (r32 = 2^32 - 4q < 0.8 * 2^30 when q > 0.8 * 2^30, else r32 < q)
HD u64 fold64(u64 x, u32 q, u32 r32) {
    u32 hi = (u32)(x >> 32);
    hi = hi >= 4 * q ? hi - 4 * q : hi;
    hi = hi >= 2 * q ? hi - 2 * q : hi;
    return (u64)hi * r32 + (u32)x;
}
// any 64-bit x mod q
HD u32 reduce64(u64 x, u32 q, u32 mu, u32 r32) { return barrett_reduce64(fold64(x, q, r32), q, mu); }

// 16-byte vector store of a kernel's output.  With AESFHE_WT (a build flag, A/B) it is WRITE-THROUGH
// (`global_store_dwordx4 ... sc1`, MI355X_MICROARCH.md: the line leaves the XCD's L2 with the store):
// a dependent kernel boundary costs ~1.7-1.9 us + B / 6 TB/s for the B bytes the predecessor left
// dirty in L2, so outputs stored through are not written back at the boundary.  The asm store is
// outside hipcc's wait-count bookkeeping: use it only for a kernel's final stores (nothing in the
// kernel reads them back); `s_nop 1` pads the store-data hazard.
#ifndef AESFHE_WT
#define AESFHE_WT 0
#endif
typedef __attribute__((ext_vector_type(4))) unsigned aesfhe_v4u;
__device__ __forceinline__ void st_out16(void* p, uint4 v) {
#if AESFHE_WT && defined(__HIP_DEVICE_COMPILE__)
    const aesfhe_v4u d = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(d) : "memory");
#else
    *reinterpret_cast<uint4*>(p) = v;
#endif
}

// per-prime constant table kept in device memory
struct PrimeConst {
    u32 q;       // modulus
    u32 mu;      // floor(2^61 / q)
    u32 ninv;    // N^{-1} mod q
    u32 ninv_p;  // Shoup companion
    u32 im;      // psi^{N/2}: the "imaginary unit" of Z_q (X^{N/2} at psi)
    u32 im_p;
    u32 r32;     // 2^32 mod q
    u32 pad1;
};

// limb -> prime map of an RNS polynomial: limbs [0, n1) use primes off1 + l,
// limbs [n1, ...) use primes off2 + (l - n1)  (a Q-prefix followed by the P block)
struct LimbMap {
    int n1, off1, off2;
    HD int prime(int l) const { return l < n1 ? off1 + l : off2 + (l - n1); }
};
