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

// The packed real form of a sparse plan (pack = true).  CoeffToSlot's last group
// also multiplies its output by a (2n-periodic), so w' + conj(w') holds 2 Re w on the first half
// of every 2n block and 2 Im w on the second (the unpacked path's re / im): ONE EvalMod instead of two.  SlotToCoeff's first
// group reads the halves back, u = s b1 + rot_n(s) b2, folded into its diagonals:
//   sum_o d_o rot_o(u) = sum_o (d_o rot_o(b1)) rot_o(s) + sum_o (d_o rot_o(b2)) rot_{o+n}(s).
// n-space offsets are taken signed (|o| <= n/2), valid for the n-periodic vectors they act on.
Diags lift_out(const Diags& D, int n, const std::vector<cplx>& a) {
    Diags L;
    const int n2 = (int)a.size();  // 2n (single packing) or 4n (pair packing)
    for (const auto& kv : D) {
        const int o = kv.first <= n / 2 ? kv.first : kv.first - n;
        std::vector<cplx> v(n2);
        for (int p = 0; p < n2; ++p) v[p] = a[p] * kv.second[p % n];
        L[((o % n2) + n2) % n2] = v;
    }
    return L;
}
Diags lift_in(const Diags& D, int n, const std::vector<cplx>& b1, const std::vector<cplx>& b2) {
    Diags L;
    const int n2 = 2 * n;
    auto add = [&](int off, const std::vector<cplx>& v) {
        const int k = ((off % n2) + n2) % n2;
        auto it = L.find(k);
        if (it == L.end()) {
            L.emplace(k, v);
        } else {
            for (int p = 0; p < n2; ++p) it->second[p] += v[p];
        }
    };
    for (const auto& kv : D) {
        const int o = kv.first <= n / 2 ? kv.first : kv.first - n;
        std::vector<cplx> v1(n2), v2(n2);
        for (int p = 0; p < n2; ++p) {
            const cplx d = kv.second[p % n];
            const int q = (((p + o) % n2) + n2) % n2;
            v1[p] = d * b1[q];
            v2[p] = d * b2[q];
        }
        add(o, v1);
        add(o + n, v2);
    }
    return L;
}

// Pair packing (pack = 2): the hi / lo members of a pair bootstrap share ONE EvalMod.
// CoeffToSlot's last group multiplies by a4 = (1 | -i | 0 | 0) per 4n block (both members,
// shared diagonals); the engine adds the lo member rotated right by 2n and w'' + conj(w'')
// holds (2 Re hi | 2 Im hi | 2 Re lo | 2 Im lo).  SlotToCoeff's first group then comes in two
// forms reading block pair `which` (0: hi, 1: lo) back into an n-periodic u:
//   u[p] = s[(p mod n) + 2n which] + i s[(p mod n) + 2n which + n]
// folded into its diagonals: for q = (p + o) mod 4n in block t, rot_o(u)[p] reads s at
// p + o - t n + 2n which (and + n, times i).
Diags lift_in4(const Diags& D, int n, int which) {
    Diags L;
    const int n4 = 4 * n, base = 2 * n * which;
    const cplx I(0.0, 1.0);
    auto add = [&](int off, int p, cplx v) {
        const int k = ((off % n4) + n4) % n4;
        auto it = L.find(k);
        if (it == L.end()) it = L.emplace(k, std::vector<cplx>(n4, 0.0)).first;
        it->second[p] += v;
    };
    for (const auto& kv : D) {
        const int o = kv.first <= n / 2 ? kv.first : kv.first - n;
        for (int p = 0; p < n4; ++p) {
            const cplx d = kv.second[p % n];
            if (d == 0.0) continue;
            const int q = (((p + o) % n4) + n4) % n4, t = q / n;
            add(o - t * n + base, p, d);
            add(o - t * n + base + n, p, I * d);
        }
    }
    return L;
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
                        double stc_boost, int pack) {
    BootPlan P;
    P.logn = logn;
    P.M = 1 << (logn - 1);
    P.K = K;
    P.r = r;
    P.deg = deg;
    const int M = P.M, logm = logn - 1;
    // packed real form: the 2M-periodic half masks (first half of every 2M block)
    std::vector<cplx> pa, pb1, pb2, pa4;
    if (pack == 2) {
        pa4.assign(4 * M, 0.0);
        for (int p = 0; p < M; ++p) pa4[p] = 1.0, pa4[p + M] = cplx(0.0, -1.0);
    }
    if (pack == 1) {
        const cplx I(0.0, 1.0);
        pa.resize(2 * M), pb1.resize(2 * M), pb2.resize(2 * M);
        for (int p = 0; p < 2 * M; ++p) {
            const double m = p < M ? 1.0 : 0.0;
            pa[p] = m - I * (1.0 - m);  // w' + conj(w') = (2 Re w | 2 Im w): the unpacked re / im halves
            pb1[p] = m + I * (1.0 - m);
            pb2[p] = I * m + (1.0 - m);
        }
    }

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
        if (pack == 2 && gi == 0) {
            const int h = 1 << (sg[gi].front() - 1);
            P.stc.push_back(layout(lift_in4(D, M, 0), h, 4 * M));
            P.stc_lo = layout(lift_in4(D, M, 1), h, 4 * M);
        } else if (pack == 1 && gi == 0) {
            D = lift_in(D, M, pb1, pb2);
            P.stc.push_back(layout(D, 1 << (sg[gi].front() - 1), 2 * M));
        } else {
            P.stc.push_back(layout(D, 1 << (sg[gi].front() - 1), M));
        }
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
        if (pack == 2 && gi == 0) {  // the last group applied
            D = lift_out(D, M, pa4);  // lift_out tiles to the mask's length (4 M here)
            P.cts.push_back(layout(D, 1 << (cg[gi].front() - 1), 4 * M));
        } else if (pack == 1 && gi == 0) {
            D = lift_out(D, M, pa);
            P.cts.push_back(layout(D, 1 << (cg[gi].front() - 1), 2 * M));
        } else {
            P.cts.push_back(layout(D, 1 << (cg[gi].front() - 1), M));
        }
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

// self-check of a sparse (small-ring, M = n slots) plan: random subring coefficients t (2n
// reals) -> slots z; CoeffToSlot then w' + conj(w') (pack 1: the 2n-periodic (2 Re | 2 Im) of
// the bit-reversed coefficient halves; pack 2: two inputs, the lo one rotated right by 2n, the
// 4n-periodic (2 Re hi | 2 Im hi | 2 Re lo | 2 Im lo); unpacked: w itself), SlotToCoeff of the
// same (EvalMod taken as the identity) -> z (2z packed; pack 2: stc[0] -> 2 z_hi, stc_lo ->
// 2 z_lo).  err: [StC error, CtS error]
extern "C" int aesfhe_debug_sparseplan(int n, int pack, double* err) {
    int logm = 0;
    while ((1 << logm) < n) ++logm;
    const int groups = std::max(1, (logm + 4) / 5);
    BootPlan P = make_boot_plan(logm + 1, groups, groups, 1.0, 1.0, 12, 3, 27, 1.0, pack);
    Embedding emb(logm + 1);
    std::mt19937_64 rng(2);
    std::normal_distribution<double> nd;
    const int M = n;
    auto brv = [logm](int x) {
        int r = 0;
        for (int i = 0; i < logm; ++i) r = (r << 1) | ((x >> i) & 1);
        return r;
    };
    auto tile = [](const std::vector<cplx>& v, int len) {
        std::vector<cplx> o(len);
        for (int p = 0; p < len; ++p) o[p] = v[p % v.size()];
        return o;
    };
    auto glen = [](const LinGroup& g, size_t cur) {
        for (const auto& row : g.diag)
            for (const auto& d : row)
                if (!d.empty()) return d.size();
        return cur;
    };
    struct In {
        std::vector<cplx> z, wb;
    };
    auto draw = [&]() {
        std::vector<double> m(2 * M), re(M), im(M);
        for (auto& x : m) x = nd(rng);
        emb.forward(m.data(), re.data(), im.data());
        In r{std::vector<cplx>(M), std::vector<cplx>(M)};
        for (int j = 0; j < M; ++j) r.z[j] = cplx(re[j], im[j]);
        for (int k = 0; k < M; ++k) r.wb[k] = cplx(m[brv(k)], m[brv(k) + M]);
        return r;
    };
    auto cts = [&](const std::vector<cplx>& z) {
        std::vector<cplx> v = z;
        for (const auto& g : P.cts) v = apply_group_plain(g, tile(v, (int)glen(g, v.size())));
        return v;
    };
    auto stc = [&](std::vector<cplx> u, bool lo) {
        for (size_t k = 0; k < P.stc.size(); ++k) {
            const LinGroup& g = (k == 0 && lo) ? P.stc_lo : P.stc[k];
            u = apply_group_plain(g, tile(u, (int)glen(g, u.size())));
        }
        return u;
    };
    double e1 = 0, e2 = 0;
    In a = draw();
    if (pack == 2) {
        In b = draw();
        const int n4 = 4 * M;
        std::vector<cplx> wa = cts(a.z), wb = cts(b.z), w(n4), v(n4);
        for (int p = 0; p < n4; ++p) w[p] = wa[p] + wb[((p - 2 * M) % n4 + n4) % n4];  // lo rotated right by 2n
        for (int p = 0; p < n4; ++p) v[p] = w[p] + std::conj(w[p]);
        for (int p = 0; p < n4; ++p) {
            const int blk = p / M, k = p % M;
            const In& src = blk < 2 ? a : b;
            const double want = (blk % 2 == 0) ? 2 * src.wb[k].real() : 2 * src.wb[k].imag();
            e2 = std::max(e2, std::abs(v[p] - want));
        }
        std::vector<cplx> uh = stc(v, false), ul = stc(v, true);
        for (size_t j = 0; j < uh.size(); ++j) e1 = std::max(e1, std::abs(uh[j] - 2.0 * a.z[j % M]));
        for (size_t j = 0; j < ul.size(); ++j) e1 = std::max(e1, std::abs(ul[j] - 2.0 * b.z[j % M]));
    } else {
        std::vector<cplx> v = cts(a.z), s(v.size());
        for (size_t p = 0; p < v.size(); ++p) s[p] = v[p] + std::conj(v[p]);
        if (pack) {
            for (int p = 0; p < 2 * M; ++p) {
                const cplx want = p < M ? cplx(2 * a.wb[p].real(), 0) : cplx(2 * a.wb[p - M].imag(), 0);
                e2 = std::max(e2, std::abs(s[p] - want));
            }
        } else {
            for (int p = 0; p < M; ++p) e2 = std::max(e2, std::abs(v[p] - a.wb[p]));
            s = v;  // the unpacked path recombines re + i im = w itself
        }
        std::vector<cplx> u = stc(s, false);
        const double gain = pack ? 2.0 : 1.0;
        for (size_t j = 0; j < u.size(); ++j) e1 = std::max(e1, std::abs(u[j] - gain * a.z[j % M]));
    }
    err[0] = e1;
    err[1] = e2;
    return 0;
}
