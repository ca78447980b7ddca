// params.h -- RNS-CKKS parameter set for the MI355X engine.
//
// Limb layout: Q limbs 0..n_q-1 = [2 base][L rescaling primes][1 encryption prime],
// followed by the n_p special (key-switching) primes.  A ciphertext at level l lives
// on Q limbs 0..l+1; level l rescales by dropping limb l+1.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "common.h"

struct HostParams {
    int logn = 16, n = 1 << 16;
    int L = 17;       // top user level (fresh ciphertexts)
    int dnum = 3;     // key-switching digits
    int alpha = 7;    // limbs per digit (= special primes)
    int n_q = 20;     // L + 3
    int n_ks = 19;    // L + 2 (limbs reachable by key switching)
    int n_p = 8;
    int fresh = 17;   // level of fresh encryptions (<= L)
    uint64_t seed = 0;

    std::vector<u32> mod;       // n_q + n_p primes
    std::vector<double> delta;  // delta[l], l = 0..L
    std::vector<u32> psi;       // primitive 2N-th root per prime

    int n_tot() const { return n_q + n_p; }
    int p_off() const { return n_q; }     // global index of the first special prime
    int enc_limb() const { return n_q - 1; }

    // builds the prime chain and scales; returns "" or an error message
    std::string build(int logn, int L, int dnum, uint64_t seed);
};

// host modular helpers (64-bit, used for table generation only)
u32 hpowm(u32 a, uint64_t e, u32 q);
u32 hinvm(u32 a, u32 q);
u32 hbitrev(u32 x, int bits);
