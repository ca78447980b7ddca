// params.h -- RNS-CKKS parameter set for the MI355X engine.
//
// Limb layout: Q limbs 0..n_q-1 = [2 base][rescaling primes][1 encryption prime], then the
// n_p special (key-switching) primes.  Levels 0..L1 drop one prime per rescale (scale
// delta ~ 0.9 * 2^30); levels L1+1..L drop two primes per rescale (scale ~ 2^59.7, the
// bootstrapping region).  A ciphertext at level l lives on Q limbs
// 0..nl(l)-1; level -1 (one limb, q0) exists only inside bootstrapping.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "common.h"

struct HostParams {
    int logn = 16, n = 1 << 16;
    int L = 17;        // top level
    int L1 = 17;       // top level of the single-prime region (== L without bootstrapping)
    int dnum = 3;      // key-switching digits
    int alpha = 7;     // limbs per digit
    int n_q = 20;      // Q limbs incl. the encryption limb
    int n_ks = 19;     // limbs reachable by key switching
    int n_p = 8;       // special primes (alpha + 1)
    int fresh = 17;    // level of fresh encryptions (<= L1)
    uint32_t key[8] = {};  // 256-bit ChaCha20 key of the context's randomness

    std::vector<u32> mod;        // n_q + n_p primes
    std::vector<double> delta;   // delta[l], l = 0..L
    std::vector<double> ptscale; // ptscale[l]: plaintext scale so that ct x pt -> rescale lands on delta[l-1]
    std::vector<int> nl_of;      // limbs at level l, stored at index l + 1 for l = -1..L+1
    std::vector<u32> psi;        // primitive 2N-th root per prime

    int n_tot() const { return n_q + n_p; }
    int p_off() const { return n_q; }        // global index of the first special prime
    int enc_limb() const { return n_q - 1; }
    int nl(int level) const { return nl_of[level + 1]; }
    // Delta_l^2 / Q_drop(l) == Delta_{l-1}: ct x ct products may be rescaled directly
    bool homogeneous(int level) const;

    // builds the prime chain and scales; returns "" or an error message
    std::string build(int logn, int L1, int n_double, int dnum, const uint32_t key[8]);
};

// host modular helpers (64-bit, used for table generation only)
u32 hpowm(u32 a, uint64_t e, u32 q);
u32 hinvm(u32 a, u32 q);
u32 hbitrev(u32 x, int bits);
