// bootstrap.cpp -- host-side planning of CKKS bootstrapping (see bootstrap.h).
#include "bootstrap.h"

#include <cmath>
#include <cstdlib>
#include <map>

namespace {

using Diags = std::map<int, std::vector<cplx>>;  // offset (mod M) -> diagonal

// butterfly stage s (lenh = 2^(s-1)) of the special FFT, or its inverse
Diags stage(int logn, int s, bool inverse) {
    const int M = 1 << (logn - 1);
    const long two_n = 2L << logn;
    const int lenh = 1 << (s - 1), len = 2 * lenh;
    const long lenq = 4L * len;
    Diags D;
    auto at = [&](int off) -> std::vector<cplx>& {
        int o = ((off % M) + M) % M;
        auto it = D.find(o);
        if (it == D.end()) it = D.emplace(o, std::vector<cplx>(M, 0.0)).first;
        return it->second;
    };
    long g = 1;  // 5^j mod 2N
    std::vector<long> rot(lenh);
    for (int j = 0; j < lenh; ++j) rot[j] = g, g = g * 5 % two_n;
    for (int i = 0; i < M; i += len)
        for (int j = 0; j < lenh; ++j) {
            const long k = (rot[j] % lenq) * (two_n / lenq);
            const cplx xi = std::polar(1.0, 2.0 * M_PI * (double)k / (double)two_n);
            const int p = i + j;
            if (!inverse) {
                at(0)[p] += 1.0;
                at(lenh)[p] += xi;
                at(-lenh)[p + lenh] += 1.0;
                at(0)[p + lenh] += -xi;
            } else {
                at(0)[p] += 0.5;
                at(lenh)[p] += 0.5;
                at(-lenh)[p + lenh] += 0.5 / xi;
                at(0)[p + lenh] += -0.5 / xi;
            }
        }
    return D;
}

// A after B: (A o B)[a + b][p] += A[a][p] * B[b][p + a]
Diags compose(const Diags& A, const Diags& B, int M) {
    Diags C;
    for (const auto& a : A)
        for (const auto& b : B) {
            const int o = (a.first + b.first) % M;
            auto it = C.find(o);
            if (it == C.end()) it = C.emplace(o, std::vector<cplx>(M, 0.0)).first;
            auto& c = it->second;
            for (int p = 0; p < M; ++p) c[p] += a.second[p] * b.second[(p + a.first) % M];
        }
    return C;
}

std::vector<cplx> rotl(const std::vector<cplx>& v, long k) {
    const long M = (long)v.size();
    std::vector<cplx> out(M);
    for (long p = 0; p < M; ++p) out[p] = v[(((p + k) % M) + M) % M];
    return out;
}

LinGroup layout(const Diags& D, int h, int M) {
    LinGroup g;
    g.h = h;
    std::map<int, const std::vector<cplx>*> by_i;  // signed offset / h -> diagonal
    int R = 0;
    for (const auto& kv : D) {
        int so = kv.first <= M / 2 ? kv.first : kv.first - M;
        int i = so / h;
        by_i[i] = &kv.second;
        R = std::max(R, std::abs(i));
    }
    const int n = 2 * R + 1;
    // baby steps are hoisted (one ModUp for all of them, no ModDown each) and cost a key
    // inner product; giant steps are full key switches: about 2 sqrt(n) babies, a power of
    // two (<= 16), and offsets starting at a multiple of B so that one giant step is 0
    static const int bmax = std::getenv("AESFHE_BOOT_BMAX") ? std::atoi(std::getenv("AESFHE_BOOT_BMAX")) : 16;
    int B = 1;
    while (B < bmax && B < 2.0 * std::sqrt((double)n)) B *= 2;
    const int R0 = (R + B - 1) / B * B;
    g.R = R0;
    g.B = B;
    g.G = (R + R0 + 1 + B - 1) / B;
    g.giant.resize(g.G);
    g.diag.assign(g.G, std::vector<std::vector<cplx>>(g.B));
    for (int gg = 0; gg < g.G; ++gg) {
        const long sg = (long)h * (gg * g.B - R0);
        g.giant[gg] = (int)sg;
        for (int b = 0; b < g.B; ++b) {
            const int i = gg * g.B + b - R0;
            auto it = by_i.find(i);
            if (it == by_i.end()) continue;
            g.diag[gg][b] = rotl(*it->second, -sg);
        }
    }
    return g;
}

}  // namespace

std::vector<cplx> apply_group_plain(const LinGroup& g, const std::vector<cplx>& v) {
    const int M = (int)v.size();
    std::vector<std::vector<cplx>> baby(g.B);
    for (int b = 0; b < g.B; ++b) baby[b] = rotl(v, (long)g.h * b);
    std::vector<cplx> out(M, 0.0);
    for (int gg = 0; gg < g.G; ++gg) {
        std::vector<cplx> inner(M, 0.0);
        for (int b = 0; b < g.B; ++b) {
            if (g.diag[gg][b].empty()) continue;
            for (int p = 0; p < M; ++p) inner[p] += g.diag[gg][b][p] * baby[b][p];
        }
        inner = rotl(inner, g.giant[gg]);
        for (int p = 0; p < M; ++p) out[p] += inner[p];
    }
    return out;
}

BootPlan make_boot_plan(int logn, int n_groups_cts, int n_groups_stc, double cts_scale, double stc_scale, int K, int r, int deg,
                        double stc_boost) {
    BootPlan P;
    P.logn = logn;
    P.M = 1 << (logn - 1);
    P.K = K;
    P.r = r;
    P.deg = deg;
    const int M = P.M, logm = logn - 1;

    auto split = [&](int groups) {
        std::vector<std::vector<int>> out(groups);
        for (int s = 1; s <= logm; ++s) out[(long)(s - 1) * groups / logm].push_back(s);
        return out;
    };
    // SlotToCoeff: stages 1..logm in order (input bit-reversed w, output natural slots)
    auto sg = split(n_groups_stc);
    for (size_t gi = 0; gi < sg.size(); ++gi) {
        Diags D;
        D[0] = std::vector<cplx>(M, 1.0);
        for (int s : sg[gi]) D = compose(stage(logn, s, false), D, M);
        // the gain goes into the FIRST group: the signal is smallest right after EvalMod,
        // where SlotToCoeff crosses into the single-prime (2^30-scale) region.  stc_boost
        // also lifts the intermediate groups' signal (undone by the LAST group): the
        // butterfly stages grow the signal ~sqrt(2) each, so without it the first groups'
        // outputs sit far below 1 at a 2^30 scale and their rescale noise (absolute, 2^-16)
        // is amplified by every later group -- the bootstrap's noise floor
        if (gi == 0)
            for (auto& kv : D)
                for (auto& x : kv.second) x *= stc_scale * (sg.size() > 1 ? stc_boost : 1.0);
        if (gi + 1 == sg.size() && sg.size() > 1)
            for (auto& kv : D)
                for (auto& x : kv.second) x /= stc_boost;
        P.stc.push_back(layout(D, 1 << (sg[gi].front() - 1), M));
    }
    // CoeffToSlot: inverse stages logm..1 (output bit-reversed w)
    auto cg = split(n_groups_cts);
    for (int gi = (int)cg.size() - 1; gi >= 0; --gi) {
        Diags D;
        D[0] = std::vector<cplx>(M, 1.0);
        for (int k = (int)cg[gi].size() - 1; k >= 0; --k) D = compose(stage(logn, cg[gi][k], true), D, M);
        if (gi == (int)cg.size() - 1)
            for (auto& kv : D)
                for (auto& x : kv.second) x *= cts_scale;
        P.cts.push_back(layout(D, 1 << (cg[gi].front() - 1), M));
    }
    // Chebyshev interpolation of cos(2 pi (K y - 1/4) / 2^r) at the deg+1 Chebyshev nodes
    const int n = deg + 1;
    std::vector<double> f(n);
    for (int j = 0; j < n; ++j) {
        const double y = std::cos(M_PI * (j + 0.5) / n);
        f[j] = std::cos(2.0 * M_PI * (K * y - 0.25) / std::ldexp(1.0, r));
    }
    P.cheb.assign(n, 0.0);
    for (int k = 0; k < n; ++k) {
        double s = 0.0;
        for (int j = 0; j < n; ++j) s += f[j] * std::cos(M_PI * k * (j + 0.5) / n);
        P.cheb[k] = (k == 0 ? 1.0 : 2.0) * s / n;
    }
    return P;
}

// ---------------------------------------------------------------------------------------
// self-check of the factorisation against the canonical embedding (no GPU needed)
// ---------------------------------------------------------------------------------------
#include <random>

#include "encoder.h"

extern "C" int aesfhe_debug_bootplan(int logn, double* err) {
    const int n = 1 << logn, M = n / 2;
    BootPlan P = make_boot_plan(logn, 3, 3, 1.0, 1.0, 12, 3, 27, 32.0);  // with the engine's SlotToCoeff boost
    Embedding emb(logn);
    std::mt19937_64 rng(1);
    std::normal_distribution<double> nd;
    std::vector<double> m(n), re(M), im(M);
    for (auto& x : m) x = nd(rng);
    emb.forward(m.data(), re.data(), im.data());
    int lb = 0;
    while ((1 << lb) < M) ++lb;
    auto brv = [lb](int x) {
        int r = 0;
        for (int i = 0; i < lb; ++i) r = (r << 1) | ((x >> i) & 1);
        return r;
    };
    std::vector<cplx> w(M), z(M), wb(M);
    for (int k = 0; k < M; ++k) w[k] = cplx(m[k], m[k + M]);
    for (int j = 0; j < M; ++j) z[j] = cplx(re[j], im[j]);
    for (int k = 0; k < M; ++k) wb[k] = w[brv(k)];
    std::vector<cplx> v = wb;
    for (const auto& g : P.stc) v = apply_group_plain(g, v);
    double e1 = 0, e2 = 0;
    for (int j = 0; j < M; ++j) e1 = std::max(e1, std::abs(v[j] - z[j]));
    v = z;
    for (const auto& g : P.cts) v = apply_group_plain(g, v);
    for (int k = 0; k < M; ++k) e2 = std::max(e2, std::abs(v[k] - wb[k]));
    err[0] = e1;
    err[1] = e2;
    // Chebyshev approximation error of the EvalMod kernel on [-1, 1]
    double e3 = 0;
    for (int i = 0; i <= 2000; ++i) {
        const double y = -1.0 + i / 1000.0;
        double t0 = 1, t1 = y, s = P.cheb[0] + P.cheb[1] * y;
        for (int k = 2; k <= P.deg; ++k) {
            const double t2 = 2 * y * t1 - t0;
            s += P.cheb[k] * t2;
            t0 = t1, t1 = t2;
        }
        e3 = std::max(e3, std::abs(s - std::cos(2 * M_PI * (P.K * y - 0.25) / std::ldexp(1.0, P.r))));
    }
    err[2] = e3;
    return 0;
}
