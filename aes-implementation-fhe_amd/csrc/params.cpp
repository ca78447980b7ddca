// params.cpp -- prime chain, scales and 2N-th roots.
#include "params.h"

#include <algorithm>
#include <cmath>
#include <set>

u32 hpowm(u32 a, uint64_t e, u32 q) {
    uint64_t r = 1, b = a % q;
    for (; e; e >>= 1) {
        if (e & 1) r = r * b % q;
        b = b * b % q;
    }
    return (u32)r;
}
u32 hinvm(u32 a, u32 q) { return hpowm(a, q - 2, q); }
u32 hbitrev(u32 x, int bits) {
    u32 r = 0;
    for (int i = 0; i < bits; ++i, x >>= 1) r = (r << 1) | (x & 1);
    return r;
}

// deterministic Miller-Rabin, exact for 32-bit n (bases 2, 7, 61)
static bool prime32(u32 n) {
    if (n < 2) return false;
    for (u32 p : {2u, 3u, 5u, 7u, 11u, 13u, 17u, 19u, 23u, 29u, 31u, 37u}) {
        if (n == p) return true;
        if (n % p == 0) return false;
    }
    u32 d = n - 1;
    int s = 0;
    while (!(d & 1)) d >>= 1, ++s;
    for (u32 a : {2u, 7u, 61u}) {
        uint64_t x = hpowm(a, d, n);
        if (x == 1 || x == n - 1) continue;
        bool witness = true;
        for (int r = 1; r < s && witness; ++r) {
            x = x * x % n;
            if (x == n - 1) witness = false;
        }
        if (witness) return false;
    }
    return true;
}

// first c = x^((q-1)/2N), x = 2, 3, ... with c^N = -1
static u32 root_2n(u32 q, int logn) {
    uint64_t two_n = 2ull << logn;
    for (u32 x = 2;; ++x) {
        u32 c = hpowm(x, (q - 1) / two_n, q);
        if (hpowm(c, two_n / 2, q) == q - 1) return c;
    }
}

bool HostParams::homogeneous(int level) const { return !(L > L1 && level == L1 + 1); }

std::string HostParams::build(int logn_, int L1_, int n_double, int dnum_, const uint32_t key_[8]) {
    if (logn_ < 13 || logn_ > 16) return "log_n must lie in [13, 16] (NTT kernels, ntt.hip)";
    if (L1_ < 1 || L1_ > 60 || n_double < 0 || n_double > 30) return "max_level must lie in [1, 60]";
    if (dnum_ < 1) return "dnum must be >= 1";
    logn = logn_; n = 1 << logn; L1 = L1_; L = L1 + n_double; dnum = dnum_;
    for (int i = 0; i < 8; ++i) key[i] = key_[i];
    nl_of.assign(L + 3, 0);
    nl_of[0] = 1;  // level -1: q0 only
    for (int l = 0; l <= L; ++l) nl_of[l + 1] = l <= L1 ? l + 2 : L1 + 2 + 2 * (l - L1);
    nl_of[L + 2] = nl_of[L + 1] + 1;  // transient level of a top-level encryption
    n_ks = nl(L);
    n_q = n_ks + 1;
    alpha = (n_ks + dnum - 1) / dnum;
    n_p = alpha + 1;  // P exceeds every digit modulus by one prime
    fresh = L1;
    mod.assign(n_tot(), 0);

    const uint64_t kMax = 1ull << 30;     // q < 2^30: 4q < 2^32 (lazy NTT butterflies in [0, 4q))
    const uint64_t kMin = 1ull << 29;     // q > 2^29: Barrett mu = 2^61 / q fits 32 bits
    const uint64_t two_n = 2ull << logn;
    std::set<u32> taken;

    // largest admissible primes: 2 base, n_p special, 1 encryption
    std::vector<u32> top;
    for (uint64_t c = (kMax - 1) / two_n * two_n + 1; top.size() < (size_t)(2 + n_p + 1); c -= two_n) {
        if (c <= kMin) return "ran out of NTT-friendly primes";
        if (c < kMax && prime32((u32)c)) top.push_back((u32)c);
    }
    mod[0] = top[0];
    mod[1] = top[1];
    for (int k = 0; k < n_p; ++k) mod[n_q + k] = top[2 + k];
    mod[n_q - 1] = top[2 + n_p];
    taken.insert(top.begin(), top.end());

    // unused admissible prime closest to `want` (ties -> smaller)
    auto closest = [&](double want) -> u32 {
        const int64_t centre = (int64_t)((want - 1.0) / (double)two_n + 0.5) * (int64_t)two_n + 1;
        u32 best = 0;
        double best_d = 1e300;
        for (int64_t s = 0; s < 100000; ++s) {
            for (int sg : {-1, 1}) {
                int64_t c = centre + sg * s * (int64_t)two_n;
                if (c <= (int64_t)kMin || c >= (int64_t)kMax) continue;
                if (!prime32((u32)c) || taken.count((u32)c)) continue;
                double d = std::fabs((double)c - want);
                if (d < best_d || (d == best_d && (u32)c < best)) { best_d = d; best = (u32)c; }
            }
            if (best && (double)s * (double)two_n > best_d + (double)two_n) break;
        }
        if (best) taken.insert(best);
        return best;
    };

    const double kT = 966367641.6;  // 0.9 * 2^30: the scale target, inside the prime range
    delta.assign(L + 1, 0.0);
    // single-prime region: delta_L1 = T; limb nl(l)-1 = l+1 is the prime closest to delta_l^2 / T
    delta[L1] = kT;
    for (int l = L1; l >= 1; --l) {
        const u32 q = closest(delta[l] * delta[l] / kT);
        if (!q) return "could not place a rescaling prime";
        mod[l + 1] = q;
        delta[l - 1] = delta[l] * delta[l] / (double)q;
    }
    // double-prime region: delta_L = T^2; levels L..L1+2 drop the pair (qa, qb) closest to
    // sqrt(delta_l^2 / T^2) and its cofactor
    if (L > L1) {
        delta[L] = kT * kT;
        for (int l = L; l >= L1 + 2; --l) {
            const double want = delta[l] * delta[l] / (kT * kT);
            const u32 qa = closest(std::sqrt(want));
            const u32 qb = qa ? closest(want / (double)qa) : 0;
            if (!qa || !qb) return "could not place a rescaling prime pair";
            mod[nl(l) - 1] = qa;
            mod[nl(l) - 2] = qb;
            delta[l - 1] = delta[l] * delta[l] / ((double)qa * (double)qb);
        }
        // transition level L1+1 -> L1: a pair near T, crossed only by plaintext products
        const u32 qa = closest(kT), qb = closest(kT);
        if (!qa || !qb) return "could not place the transition primes";
        mod[nl(L1 + 1) - 1] = qa;
        mod[nl(L1 + 1) - 2] = qb;
    }
    ptscale.assign(L + 1, 0.0);
    for (int l = 1; l <= L; ++l) {
        double qd = 1.0;
        for (int t = nl(l - 1); t < nl(l); ++t) qd *= (double)mod[t];
        ptscale[l] = delta[l - 1] * qd / delta[l];
    }
    psi.resize(n_tot());
    for (int i = 0; i < n_tot(); ++i) psi[i] = root_2n(mod[i], logn);
    return "";
}
