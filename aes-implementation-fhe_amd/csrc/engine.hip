// engine.hip -- host orchestration of the MI355X RNS-CKKS engine + the C ABI
// declared in include/aesfhe.h.
//
// One Engine = one HIP device + one stream.  Ciphertexts live in HBM as
// [poly][limb][N] uint32 (NTT form unless to_intt was requested); all device work is
// stream-ordered, so temporaries go back to the pool as soon as their last kernel has
// been enqueued.  Conventions (primes, NTT order, key layout, PRNG streams, scales) are
// fixed in DESIGN.md §3 and restated independently by oracle/ckks_oracle.c.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/aesfhe.h"
#include "encoder.h"
#include "kernels.h"
#include "params.h"

namespace {

#define HIP_OK(expr)                                                                                      \
    do {                                                                                                  \
        hipError_t e_ = (expr);                                                                           \
        if (e_ != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_) + \
                                                       " at " #expr);                                      \
    } while (0)

inline u64 stream_id(u64 kind, u64 a, u64 b) { return (kind << 56) | (a << 16) | b; }

// ---------------------------------------------------------------------------------
// device memory pool: exact-size free lists (ciphertext sizes repeat constantly)
// ---------------------------------------------------------------------------------
class Pool {
public:
    u32* get(size_t words) {
        auto& fl = free_[words];
        if (!fl.empty()) {
            u32* p = fl.back();
            fl.pop_back();
            return p;
        }
        void* p = nullptr;
        HIP_OK(hipMalloc(&p, words * sizeof(u32)));
        bytes_ += words * sizeof(u32);
        return (u32*)p;
    }
    void put(u32* p, size_t words) {
        if (p) free_[words].push_back(p);
    }
    void release_all() {
        for (auto& kv : free_)
            for (u32* p : kv.second) (void)hipFree(p);
        free_.clear();
    }
    size_t bytes() const { return bytes_; }

private:
    std::unordered_map<size_t, std::vector<u32*>> free_;
    size_t bytes_ = 0;
};

struct Ct {
    u32* data = nullptr;
    size_t words = 0;
    int level = 0;
    int npoly = 2;
    bool ntt = true;
    bool pending = false;  // tensor product awaiting rescale (scale delta_level^2)
};

struct Pt {
    std::vector<double> re, im;
    bool constant = false;
    std::map<int, u32*> enc;  // level -> NTT-form encoding at scale delta[level]
};

enum Counter { C_MUL, C_RELIN, C_ROT, C_CONJ, C_PTMUL, C_SCALAR, C_RESCALE, C_NTT_ROWS, C_KS, C_ENC, C_DEC, C_BOOT, C_ADD, C_N };

class Engine {
public:
    Engine(int logn, int L, int dnum, int device, u64 seed) : emb_(logn) {
        std::string err = hp_.build(logn, L, dnum, seed);
        if (!err.empty()) throw std::runtime_error(err);
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
            throw std::runtime_error("no HIP device visible: the MI355X engine has no CPU fallback");
        if (device < 0 || device >= ndev) throw std::runtime_error("device_id out of range");
        device_ = device;
        HIP_OK(hipSetDevice(device_));
        HIP_OK(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
        build_tables();
    }
    ~Engine() {
        (void)hipSetDevice(device_);
        (void)hipStreamSynchronize(st_);
        for (auto& kv : cts_) pool_.put(kv.second.data, kv.second.words);
        for (auto& kv : pts_)
            for (auto& e : kv.second.enc) pool_.put(e.second, (size_t)(e.first + 2) * hp_.n);
        pool_.release_all();
        for (void* p : owned_) (void)hipFree(p);
        for (auto& kv : ksk_) (void)hipFree(kv.second);
        if (ring_host_) (void)hipHostFree(ring_host_);
        (void)hipStreamDestroy(st_);
    }

    const HostParams& hp() const { return hp_; }
    void set_fresh(int level) {
        if (level < 0 || level > hp_.L) throw std::runtime_error("fresh level must lie in [0, max_level]");
        hp_.fresh = level;
    }
    int slot_count() const { return hp_.n / 2; }
    void sync() { HIP_OK(hipStreamSynchronize(st_)); }

    // ------------------------------------------------------------------ handles
    aesfhe_handle put_ct(Ct c) {
        aesfhe_handle h = next_++;
        cts_[h] = c;
        return h;
    }
    const Ct& ct(aesfhe_handle h) const {
        auto it = cts_.find(h);
        if (it == cts_.end()) throw std::runtime_error("invalid ciphertext handle");
        return it->second;
    }
    Pt& pt(aesfhe_handle h) {
        auto it = pts_.find(h);
        if (it == pts_.end()) throw std::runtime_error("invalid plaintext handle");
        return it->second;
    }
    void free_handle(aesfhe_handle h) {
        auto it = cts_.find(h);
        if (it != cts_.end()) {
            pool_.put(it->second.data, it->second.words);
            cts_.erase(it);
            return;
        }
        auto ip = pts_.find(h);
        if (ip != pts_.end()) {
            for (auto& e : ip->second.enc) pool_.put(e.second, (size_t)(e.first + 2) * hp_.n);
            pts_.erase(ip);
        }
    }
    aesfhe_handle new_pt(const double* re, const double* im, int n) {
        Pt p;
        const int s = slot_count();
        p.re.assign(s, 0.0);
        p.im.assign(s, 0.0);
        for (int j = 0; j < s && j < n; ++j) p.re[j] = re[j], p.im[j] = im ? im[j] : 0.0;
        p.constant = (n >= s);
        for (int j = 1; j < s && p.constant; ++j) p.constant = (p.re[j] == p.re[0] && p.im[j] == p.im[0]);
        aesfhe_handle h = next_++;
        pts_[h] = std::move(p);
        return h;
    }

    Ct alloc_ct(int level, int npoly) {
        Ct c;
        c.level = level;
        c.npoly = npoly;
        c.words = (size_t)npoly * (level + 2) * hp_.n;
        c.data = pool_.get(c.words);
        return c;
    }
    u32* tmp(size_t rows) { return pool_.get(rows * hp_.n); }
    void untmp(u32* p, size_t rows) { pool_.put(p, rows * hp_.n); }

    // ------------------------------------------------------------------ maps
    static LimbMap qmap() { return LimbMap{1 << 30, 0, 0}; }
    LimbMap extmap(int nl) const { return LimbMap{nl, 0, hp_.p_off()}; }
    static LimbMap single(int prime) { return LimbMap{1, prime, 0}; }

    void ntt(u32* d, int rows, int nl, LimbMap m) {
        launch_ntt_fwd(st_, T_, d, rows, nl, m);
        cnt_[C_NTT_ROWS] += rows;
    }
    void intt(u32* d, int rows, int nl, LimbMap m) {
        launch_ntt_inv(st_, T_, d, rows, nl, m);
        cnt_[C_NTT_ROWS] += rows;
    }

    // ------------------------------------------------------------------ keys
    void keygen() {
        const int n = hp_.n, nt = hp_.n_tot();
        if (!d_s_) {
            d_s_ = dev_alloc((size_t)nt * n);
            launch_sample_small(st_, T_, d_s_, nt, qmap(), hp_.seed, stream_id(1, 0, 0), 0);
            ntt(d_s_, nt, nt, qmap());
        }
        if (!d_pk_) {
            const int nq = hp_.n_q;
            d_pk_ = dev_alloc((size_t)2 * nq * n);
            u32* e = tmp(nq);
            launch_sample_uniform(st_, T_, d_pk_ + (size_t)nq * n, nq, qmap(), hp_.seed, stream_id(2, 0, 0));
            launch_sample_small(st_, T_, e, nq, qmap(), hp_.seed, stream_id(3, 0, 0), 1);
            ntt(e, nq, nq, qmap());
            launch_keygen_combine(st_, T_, d_pk_, d_pk_ + (size_t)nq * n, d_s_, e, nullptr, nullptr, nq, qmap(), 0, 0);
            untmp(e, nq);
        }
        ksk(0);
        ksk(conj_galois());
        sync();
    }
    u64 conj_galois() const { return 2ull * hp_.n - 1; }
    u64 rot_galois(int steps) const {
        const long s = slot_count();
        long k = ((-(long)steps) % s + s) % s;  // np.roll(slots, steps) = left rotation by -steps
        u64 g = 1, b = 5, m = 2ull * hp_.n;
        for (; k; k >>= 1) {
            if (k & 1) g = g * b % m;
            b = b * b % m;
        }
        return g;
    }
    size_t ksk_words() const { return (size_t)hp_.dnum * 2 * (hp_.n_ks + hp_.n_p) * hp_.n; }
    const u32* ksk(u64 g) {
        auto it = ksk_.find(g);
        if (it != ksk_.end()) return it->second;
        if (!d_s_) throw std::runtime_error("keys not generated");
        const int n = hp_.n, nks = hp_.n_ks, np = hp_.n_p, nkey = nks + np;
        void* raw = nullptr;
        HIP_OK(hipMalloc(&raw, ksk_words() * sizeof(u32)));
        u32* key = (u32*)raw;
        u32* sp = tmp(nks);
        if (g == 0) launch_square(st_, T_, sp, d_s_, nks, nks, qmap());
        else launch_automorph(st_, T_, sp, d_s_, g, nks);
        u32* e = tmp(nkey);
        const LimbMap em = extmap(nks);
        for (int j = 0; j < hp_.dnum; ++j) {
            u32* b = key + (size_t)j * 2 * nkey * n;
            u32* a = b + (size_t)nkey * n;
            launch_sample_uniform(st_, T_, a, nkey, em, hp_.seed, stream_id(4, g, j));
            launch_sample_small(st_, T_, e, nkey, em, hp_.seed, stream_id(5, g, j), 1);
            ntt(e, nkey, nkey, em);
            const int lo = j * hp_.alpha, hi = std::min(nks, lo + hp_.alpha);
            launch_keygen_combine(st_, T_, b, a, d_s_, e, sp, d_gadget_, nkey, em, lo, hi);
        }
        untmp(e, nkey);
        untmp(sp, nks);
        ksk_[g] = key;
        return key;
    }

    // ------------------------------------------------------------------ codec
    // host: slots -> residues on limbs 0..nl-1 at `scale` (coefficient form)
    void encode_host(const double* re, const double* im, double scale, int nl, std::vector<u32>& out) {
        const int n = hp_.n;
        std::vector<double> m(n);
        emb_.inverse(re, im, m.data());
        out.assign((size_t)nl * n, 0);
        for (int k = 0; k < n; ++k) {
            const double x = m[k] * scale;
            __int128 v = std::fabs(x) < 4503599627370496.0 ? (__int128)std::llround(x) : (__int128)x;
            for (int t = 0; t < nl; ++t) {
                __int128 r = v % (__int128)hp_.mod[t];
                if (r < 0) r += hp_.mod[t];
                out[(size_t)t * n + k] = (u32)r;
            }
        }
    }
    u32* upload_ntt(const std::vector<u32>& host, int nl) {
        u32* d = tmp(nl);
        HIP_OK(hipMemcpyAsync(d, host.data(), host.size() * sizeof(u32), hipMemcpyHostToDevice, st_));
        HIP_OK(hipStreamSynchronize(st_));  // host vector may die after return
        ntt(d, nl, nl, qmap());
        return d;
    }

    aesfhe_handle encrypt(const double* re, const double* im) {
        if (!d_pk_) throw std::runtime_error("keys not generated");
        // encode at delta_f * q_{f+2} on limbs 0..f+2, encrypt at level f+1, rescale to f
        const int n = hp_.n, f = hp_.fresh, nq = f + 3;
        const int L = f;
        std::vector<u32> host;
        encode_host(re, im, hp_.delta[f] * (double)hp_.mod[f + 2], nq, host);
        u32* m = upload_ntt(host, nq);
        u32* v = tmp(nq);
        u32* e = tmp(2 * nq);
        const u64 ctr = enc_ctr_++;
        launch_sample_small(st_, T_, v, nq, qmap(), hp_.seed, stream_id(6, 0, ctr), 0);
        launch_sample_small(st_, T_, e, nq, qmap(), hp_.seed, stream_id(7, 0, ctr), 1);
        launch_sample_small(st_, T_, e + (size_t)nq * n, nq, qmap(), hp_.seed, stream_id(8, 0, ctr), 1);
        ntt(v, nq, nq, qmap());
        ntt(e, 2 * nq, nq, qmap());
        Ct top = alloc_ct(L + 1, 2);
        launch_add(st_, T_, e, e, m, nq, nq, qmap());  // e0 + m
        launch_fma_poly(st_, T_, top.data, e, d_pk_, v, nq, nq, qmap());
        launch_fma_poly(st_, T_, top.data + (size_t)nq * n, e + (size_t)nq * n, d_pk_ + (size_t)hp_.n_q * n, v, nq, nq, qmap());
        untmp(m, nq);
        untmp(v, nq);
        untmp(e, 2 * nq);
        Ct out = rescale(top);
        release(top);
        cnt_[C_ENC]++;
        return put_ct(out);
    }

    // decryption to real coefficients (message * delta_level)
    int decrypt_coeffs(const Ct& c_in, std::vector<double>& m) {
        const int n = hp_.n;
        Ct c = ensure_ntt(c_in);
        const int level = c.level;
        const int nl = c.level + 2;
        u32* x = tmp(2);
        HIP_OK(hipMemcpyAsync(x, c.data, sizeof(u32) * 2 * n, hipMemcpyDeviceToDevice, st_));
        u32* spow = nullptr;
        for (int p = 1; p < c.npoly; ++p) {
            const u32* s_use = d_s_;
            if (p == 2) {
                spow = tmp(2);
                launch_square(st_, T_, spow, d_s_, 2, 2, qmap());
                s_use = spow;
            }
            launch_fma_poly(st_, T_, x, x, c.data + (size_t)p * nl * n, s_use, 2, 2, qmap());
        }
        intt(x, 2, 2, qmap());
        std::vector<u32> h((size_t)2 * n);
        HIP_OK(hipMemcpyAsync(h.data(), x, sizeof(u32) * 2 * n, hipMemcpyDeviceToHost, st_));
        HIP_OK(hipStreamSynchronize(st_));
        untmp(x, 2);
        if (spow) untmp(spow, 2);
        if (c.data != c_in.data) release(c);
        const u32 q0 = hp_.mod[0], q1 = hp_.mod[1];
        const u64 q0inv = hinvm(q0 % q1, q1);
        const u64 Q = (u64)q0 * q1;
        m.resize(n);
        for (int k = 0; k < n; ++k) {
            const u64 a = h[k], b = h[(size_t)n + k];
            const u64 t = ((b + q1 - a % q1) % q1) * q0inv % q1;
            const u64 v = a + t * q0;
            const i64 sv = v > Q / 2 ? (i64)v - (i64)Q : (i64)v;
            m[k] = (double)sv;
        }
        cnt_[C_DEC]++;
        return level;
    }
    void decrypt(aesfhe_handle h, double* re, double* im) {
        std::vector<double> m;
        const int level = decrypt_coeffs(ct(h), m);
        const double inv = 1.0 / hp_.delta[level];
        for (double& v : m) v *= inv;
        emb_.forward(m.data(), re, im);
    }

    // ------------------------------------------------------------------ basic ops
    void release(const Ct& c) { pool_.put(c.data, c.words); }
    Ct copy(const Ct& c) {
        Ct o = alloc_ct(c.level, c.npoly);
        o.ntt = c.ntt;
        o.pending = c.pending;
        HIP_OK(hipMemcpyAsync(o.data, c.data, c.words * sizeof(u32), hipMemcpyDeviceToDevice, st_));
        return o;
    }
    // returns c itself (same data) when already in NTT form, else a converted copy
    Ct ensure_ntt(const Ct& c, bool resolve_pending = true) {
        Ct o = c;
        if (!c.ntt) {
            o = copy(c);
            ntt(o.data, o.npoly * (o.level + 2), o.level + 2, qmap());
            o.ntt = true;
        }
        if (resolve_pending && o.pending) {
            Ct r = rescale(o);
            if (o.data != c.data) release(o);
            o = r;
        }
        return o;
    }
    Ct to_intt(const Ct& c) {
        Ct o = copy(c);
        if (c.ntt) intt(o.data, o.npoly * (o.level + 2), o.level + 2, qmap());
        o.ntt = false;
        return o;
    }
    Ct to_ntt(const Ct& c) {
        Ct o = copy(c);
        if (!c.ntt) ntt(o.data, o.npoly * (o.level + 2), o.level + 2, qmap());
        o.ntt = true;
        return o;
    }

    // rescale by the last limb: level l -> l-1
    Ct rescale(const Ct& c) {
        if (c.level < 1) throw std::runtime_error("cannot rescale: ciphertext is at level 0 (not enough level)");
        const int n = hp_.n, nl = c.level + 2, r = nl - 1, np = c.npoly;
        u32* last = tmp(np);
        for (int p = 0; p < np; ++p)
            HIP_OK(hipMemcpyAsync(last + (size_t)p * n, c.data + ((size_t)p * nl + r) * n, sizeof(u32) * n, hipMemcpyDeviceToDevice, st_));
        intt(last, np, 1, single(r));
        u32* v = tmp((size_t)np * r);
        launch_rescale_spread(st_, T_, v, last, np, r, hp_.mod[r]);
        ntt(v, np * r, r, qmap());
        Ct o = alloc_ct(c.level - 1, np);
        o.pending = false;
        launch_rescale_finish(st_, T_, o.data, c.data, v, d_rescale_qinv_ + rescale_off_[c.level], np, r, nl);
        untmp(last, np);
        untmp(v, (size_t)np * r);
        cnt_[C_RESCALE]++;
        return o;
    }

    // per-limb constant residues (Shoup pairs, lo/hi halves) on limbs 0..nl-1
    u32* const_half(const std::vector<u32>& lo, const std::vector<u32>& hi) {
        const int nl = (int)lo.size();
        std::vector<u32> h(4 * (size_t)nl);
        for (int t = 0; t < nl; ++t) {
            const u32 q = hp_.mod[t];
            h[4 * t] = lo[t];
            h[4 * t + 1] = shoup_pre(lo[t], q);
            h[4 * t + 2] = hi[t];
            h[4 * t + 3] = shoup_pre(hi[t], q);
        }
        return upload_small(h);
    }
    u32* upload_small(const std::vector<u32>& h) {
        // small constant buffers: pinned host ring -> device ring; on wrap-around the
        // stream is drained so no in-flight kernel still reads a recycled slot
        const size_t words = (h.size() + 63) & ~size_t(63);
        if (ring_off_ + words > kRingWords) {
            HIP_OK(hipStreamSynchronize(st_));
            ring_off_ = 0;
        }
        u32* d = ring_ + ring_off_;
        std::memcpy(ring_host_ + ring_off_, h.data(), h.size() * sizeof(u32));
        HIP_OK(hipMemcpyAsync(d, ring_host_ + ring_off_, h.size() * sizeof(u32), hipMemcpyHostToDevice, st_));
        ring_off_ += words;
        return d;
    }
    static u32 mod_i64(i64 v, u32 q) {
        i64 r = v % (i64)q;
        return (u32)(r < 0 ? r + q : r);
    }

    // X^0 coefficient A, X^{N/2} coefficient B -> NTT-domain values A +/- B*I
    void scalar_residues(i64 A, i64 B, int nl, std::vector<u32>& lo, std::vector<u32>& hi) {
        lo.resize(nl);
        hi.resize(nl);
        for (int t = 0; t < nl; ++t) {
            const u32 q = hp_.mod[t];
            const u64 a = mod_i64(A, q), b = mod_i64(B, q);
            const u64 bi = b * im_[t] % q;
            lo[t] = (u32)((a + bi) % q);
            hi[t] = (u32)((a + q - bi) % q);
        }
    }

    Ct level_down(const Ct& c_in, int level) {
        if (level == c_in.level) return copy(c_in);
        if (level > c_in.level) throw std::runtime_error("level_down: target level above ciphertext level");
        Ct c = ensure_ntt(c_in);
        const int n = hp_.n, nl_mid = level + 3;
        // keep limbs 0..level+2, multiply by round(delta_b q_{b+2} / delta_a), rescale
        Ct mid = alloc_ct(level + 1, c.npoly);
        for (int p = 0; p < c.npoly; ++p)
            HIP_OK(hipMemcpyAsync(mid.data + (size_t)p * nl_mid * n, c.data + (size_t)p * (c.level + 2) * n, sizeof(u32) * nl_mid * n,
                                  hipMemcpyDeviceToDevice, st_));
        const i64 cst = std::llround(hp_.delta[level] * (double)hp_.mod[level + 2] / hp_.delta[c.level]);
        std::vector<u32> r(nl_mid);
        for (int t = 0; t < nl_mid; ++t) r[t] = mod_i64(cst, hp_.mod[t]);
        u32* d = const_half(r, r);
        launch_mul_const_half(st_, T_, mid.data, mid.data, d, c.npoly * nl_mid, nl_mid, qmap());
        Ct o = rescale(mid);
        release(mid);
        if (c.data != c_in.data) release(c);
        return o;
    }
    // two ciphertexts at a common level (copies only when a level change is needed)
    std::pair<Ct, Ct> align(const Ct& a, const Ct& b, bool& fa, bool& fb) {
        const int lv = std::min(a.level - (a.pending ? 1 : 0), b.level - (b.pending ? 1 : 0));
        Ct x = ensure_ntt(a), y = ensure_ntt(b);
        fa = x.data != a.data;
        fb = y.data != b.data;
        if (x.level != lv) {
            Ct t = level_down(x, lv);
            if (fa) release(x);
            x = t, fa = true;
        }
        if (y.level != lv) {
            Ct t = level_down(y, lv);
            if (fb) release(y);
            y = t, fb = true;
        }
        return {x, y};
    }

    Ct add_sub(const Ct& a, const Ct& b, bool sub) {
        bool fa, fb;
        auto xy = align(a, b, fa, fb);
        const Ct &x = xy.first, &y = xy.second;
        const int nl = x.level + 2;
        const int np = std::max(x.npoly, y.npoly);
        Ct o = alloc_ct(x.level, np);
        const int common = std::min(x.npoly, y.npoly) * nl;
        if (sub) launch_sub(st_, T_, o.data, x.data, y.data, common, nl, qmap());
        else launch_add(st_, T_, o.data, x.data, y.data, common, nl, qmap());
        if (x.npoly > y.npoly)
            HIP_OK(hipMemcpyAsync(o.data + (size_t)common * hp_.n, x.data + (size_t)common * hp_.n, sizeof(u32) * nl * hp_.n,
                                  hipMemcpyDeviceToDevice, st_));
        else if (y.npoly > x.npoly) {
            if (sub) launch_neg(st_, T_, o.data + (size_t)common * hp_.n, y.data + (size_t)common * hp_.n, nl, nl, qmap());
            else HIP_OK(hipMemcpyAsync(o.data + (size_t)common * hp_.n, y.data + (size_t)common * hp_.n, sizeof(u32) * nl * hp_.n,
                                       hipMemcpyDeviceToDevice, st_));
        }
        if (fa) release(x);
        if (fb) release(y);
        cnt_[C_ADD]++;
        return o;
    }

    Ct add_scalar(const Ct& c_in, double re, double im) {
        Ct c = ensure_ntt(c_in);
        const int nl = c.level + 2;
        std::vector<u32> lo, hi;
        scalar_residues(std::llround(re * hp_.delta[c.level]), std::llround(im * hp_.delta[c.level]), nl, lo, hi);
        std::vector<u32> h(2 * (size_t)nl);
        for (int t = 0; t < nl; ++t) h[2 * t] = lo[t], h[2 * t + 1] = hi[t];
        u32* d = upload_small(h);
        Ct o = copy(c);
        launch_add_const_half(st_, T_, o.data, c.data, d, nl, nl, qmap());
        if (c.data != c_in.data) release(c);
        return o;
    }

    Ct mul_scalar(const Ct& c_in, double re, double im) {
        Ct c = ensure_ntt(c_in);
        const int nl = c.level + 2;
        Ct o;
        cnt_[C_SCALAR]++;
        if (re == std::floor(re) && im == std::floor(im) && std::fabs(re) < 1048576.0 && std::fabs(im) < 1048576.0) {
            // Gaussian integer a + b i: exact multiplication by a + b X^{N/2}, no level consumed
            std::vector<u32> lo, hi;
            scalar_residues((i64)re, (i64)im, nl, lo, hi);
            u32* d = const_half(lo, hi);
            o = alloc_ct(c.level, c.npoly);
            launch_mul_const_half(st_, T_, o.data, c.data, d, c.npoly * nl, nl, qmap());
        } else {
            if (c.level < 1) throw std::runtime_error("not enough level to multiply by a scalar (level 0)");
            std::vector<u32> lo, hi;
            scalar_residues(std::llround(re * hp_.delta[c.level]), std::llround(im * hp_.delta[c.level]), nl, lo, hi);
            u32* d = const_half(lo, hi);
            Ct t = alloc_ct(c.level, c.npoly);
            launch_mul_const_half(st_, T_, t.data, c.data, d, c.npoly * nl, nl, qmap());
            o = rescale(t);
            release(t);
        }
        if (c.data != c_in.data) release(c);
        return o;
    }

    // plaintext encoded at (level, delta_level), NTT form, cached on the plaintext
    u32* pt_at(Pt& p, int level) {
        auto it = p.enc.find(level);
        if (it != p.enc.end()) return it->second;
        std::vector<u32> host;
        encode_host(p.re.data(), p.im.data(), hp_.delta[level], level + 2, host);
        u32* d = upload_ntt(host, level + 2);
        p.enc[level] = d;
        return d;
    }

    Ct mul_pt(const Ct& c_in, aesfhe_handle hp) {
        Pt& p = pt(hp);
        if (p.constant) return mul_scalar(c_in, p.re[0], p.im[0]);
        if (c_in.level < 1) throw std::runtime_error("not enough level to multiply by a plaintext (level 0)");
        Ct c = ensure_ntt(c_in);
        const int nl = c.level + 2;
        u32* e = pt_at(p, c.level);
        Ct t = alloc_ct(c.level, c.npoly);
        launch_mul_poly(st_, T_, t.data, c.data, e, c.npoly, nl, qmap());
        Ct o = rescale(t);
        release(t);
        if (c.data != c_in.data) release(c);
        cnt_[C_PTMUL]++;
        return o;
    }

    Ct add_pt(const Ct& c_in, aesfhe_handle hp) {
        Pt& p = pt(hp);
        if (p.constant) return add_scalar(c_in, p.re[0], p.im[0]);
        Ct c = ensure_ntt(c_in);
        const int nl = c.level + 2;
        u32* e = pt_at(p, c.level);
        Ct o = copy(c);
        launch_add(st_, T_, o.data, c.data, e, nl, nl, qmap());
        if (c.data != c_in.data) release(c);
        return o;
    }

    // ------------------------------------------------------------------ key switching
    // returns (c0', c1') with c0' + c1' s = d s' (+ add0/add1 folded in); d NTT, level l
    Ct keyswitch(const u32* d, int level, const u32* key, const u32* add0, const u32* add1) {
        const int n = hp_.n, nl = level + 2, np = hp_.n_p, ne = nl + np, alpha = hp_.alpha;
        const int nd = (nl + alpha - 1) / alpha;
        const LimbMap em = extmap(nl);
        u32* coef = tmp(nl);
        HIP_OK(hipMemcpyAsync(coef, d, sizeof(u32) * nl * n, hipMemcpyDeviceToDevice, st_));
        intt(coef, nl, nl, qmap());
        u32* ext = tmp((size_t)nd * ne);
        const size_t* toff = &modup_off_[(size_t)level * hp_.dnum];
        for (int j = 0; j < nd; ++j) {
            const int lo = j * alpha, h = std::min(alpha, nl - lo);
            u32* ej = ext + (size_t)j * ne * n;
            HIP_OK(hipMemcpyAsync(ej + (size_t)lo * n, d + (size_t)lo * n, sizeof(u32) * h * n, hipMemcpyDeviceToDevice, st_));
            launch_base_convert(st_, T_, ej, coef + (size_t)lo * n, h, lo, ne, em, lo, d_modup_ + toff[j],
                                d_modup_ + toff[j] + (size_t)2 * h * ne, d_modup_ + toff[j] + (size_t)2 * h * ne + 2 * h);
            if (lo > 0) ntt(ej, lo, lo, qmap());
            const int rest = ne - (lo + h);
            if (rest > 0) ntt(ej + (size_t)(lo + h) * n, rest, rest, LimbMap{nl - (lo + h), lo + h, hp_.p_off()});
        }
        u32* acc = tmp(2 * (size_t)ne);
        launch_key_inner(st_, T_, acc, ext, key, nd, ne, nl, hp_.n_ks + np, hp_.n_ks, em);
        untmp(ext, (size_t)nd * ne);
        untmp(coef, nl);
        // ModDown by P
        u32* yp = tmp(2 * (size_t)np);
        for (int p = 0; p < 2; ++p)
            HIP_OK(hipMemcpyAsync(yp + (size_t)p * np * n, acc + ((size_t)p * ne + nl) * n, sizeof(u32) * np * n, hipMemcpyDeviceToDevice, st_));
        intt(yp, 2 * np, np, LimbMap{np, hp_.p_off(), 0});
        u32* conv = tmp(2 * (size_t)nl);
        const size_t doff = moddown_off_[level];
        for (int p = 0; p < 2; ++p)
            launch_base_convert(st_, T_, conv + (size_t)p * nl * n, yp + (size_t)p * np * n, np, hp_.p_off(), nl, qmap(), 1 << 30,
                                d_moddown_ + doff, d_moddown_phinv_, d_negp_);
        ntt(conv, 2 * nl, nl, qmap());
        Ct o = alloc_ct(level, 2);
        launch_moddown_finish(st_, T_, o.data, acc, conv, d_pinv_ + (size_t)2 * 0, add0, add1, nl, ne);
        untmp(yp, 2 * (size_t)np);
        untmp(conv, 2 * (size_t)nl);
        untmp(acc, 2 * (size_t)ne);
        cnt_[C_KS]++;
        return o;
    }

    Ct mul(const Ct& a, const Ct& b, bool relin) {
        if (a.npoly != 2 || b.npoly != 2) throw std::runtime_error("multiply expects 2-polynomial ciphertexts");
        if (a.level < 1 || b.level < 1) throw std::runtime_error("not enough level to multiply (level 0)");
        bool fa, fb;
        auto xy = align(a, b, fa, fb);
        const Ct &x = xy.first, &y = xy.second;
        const int nl = x.level + 2, n = hp_.n;
        Ct d = alloc_ct(x.level, 3);
        launch_tensor(st_, T_, d.data, x.data, y.data, nl, qmap());
        if (fa) release(x);
        if (fb) release(y);
        cnt_[C_MUL]++;
        if (!relin) {
            d.pending = true;
            return d;
        }
        Ct r = keyswitch(d.data + (size_t)2 * nl * n, d.level, ksk(0), d.data, d.data + (size_t)nl * n);
        release(d);
        cnt_[C_RELIN]++;
        Ct o = rescale(r);
        release(r);
        return o;
    }

    Ct relinearize(const Ct& c_in) {
        if (c_in.npoly != 3) throw std::runtime_error("relinearize: ciphertext should have 3 polynomials");
        Ct c = ensure_ntt(c_in, false);
        const int nl = c.level + 2, n = hp_.n;
        Ct r = keyswitch(c.data + (size_t)2 * nl * n, c.level, ksk(0), c.data, c.data + (size_t)nl * n);
        if (c.data != c_in.data) release(c);
        cnt_[C_RELIN]++;
        if (!c_in.pending) return r;
        Ct o = rescale(r);
        release(r);
        return o;
    }

    Ct galois(const Ct& c_in, u64 g) {
        if (c_in.npoly != 2) throw std::runtime_error("rotation/conjugation expects a 2-polynomial ciphertext");
        Ct c = ensure_ntt(c_in);
        const int nl = c.level + 2, n = hp_.n;
        const u32* key = ksk(g);
        u32* perm = tmp(2 * (size_t)nl);
        launch_automorph(st_, T_, perm, c.data, g, 2 * nl);
        Ct o = keyswitch(perm + (size_t)nl * n, c.level, key, perm, nullptr);
        untmp(perm, 2 * (size_t)nl);
        if (c.data != c_in.data) release(c);
        return o;
    }
    Ct rotate(const Ct& c, int steps) {
        const long s = slot_count();
        if (((long)steps % s + s) % s == 0) return copy(c);
        cnt_[C_ROT]++;
        return galois(c, rot_galois(steps));
    }
    Ct conjugate(const Ct& c) {
        cnt_[C_CONJ]++;
        return galois(c, conj_galois());
    }

    // x^k at depth ceil(log2 k): x^(2^i) by squaring, x^k = x^(2^t) x^(k - 2^t)
    void power_basis(aesfhe_handle h, int degree, aesfhe_handle* out) {
        const Ct& x = ct(h);
        if (degree < 1) throw std::runtime_error("power basis degree must be >= 1");
        int depth = 0;
        while ((1 << depth) < degree) ++depth;
        if (x.level < depth)
            throw std::runtime_error("not enough level for make_power_basis: need " + std::to_string(depth) + ", have level " +
                                     std::to_string(x.level));
        std::vector<aesfhe_handle> pw(degree + 1, 0);
        pw[1] = put_ct(copy(x));
        for (int k = 2; k <= degree; ++k) {
            int t = 1;
            while ((t << 1) <= k) t <<= 1;
            if (t == k) pw[k] = put_ct(mul(ct(pw[t / 2]), ct(pw[t / 2]), true));
            else pw[k] = put_ct(mul(ct(pw[t]), ct(pw[k - t]), true));
        }
        for (int k = 1; k <= degree; ++k) out[k - 1] = pw[k];
    }

    // secret-key Zeta16 renorm of a state pair (REF/pipeline.py:65-69, REF/state_encoder.py:17-38)
    void renorm_pair(aesfhe_handle hh, aesfhe_handle hl, aesfhe_handle* oh, aesfhe_handle* ol) {
        const int s = slot_count(), stride = s / 16, n = hp_.n;
        std::vector<double> re(s), im(s), m;
        int nib[2][16];
        aesfhe_handle in[2] = {hh, hl};
        for (int w = 0; w < 2; ++w) {
            const int level = decrypt_coeffs(ct(in[w]), m);
            const double inv = 1.0 / hp_.delta[level];
            for (int k = 0; k < n; ++k) m[k] *= inv;
            emb_.forward(m.data(), re.data(), im.data());
            for (int i = 0; i < 16; ++i) {
                const double ang = std::atan2(im[(size_t)i * stride], re[(size_t)i * stride]);
                const double k = std::nearbyint(-ang * 16.0 / (2.0 * M_PI));
                nib[w][i] = (int)(((long)k % 16 + 16) % 16);
            }
        }
        aesfhe_handle outs[2];
        for (int w = 0; w < 2; ++w) {
            std::fill(re.begin(), re.end(), 1.0);
            std::fill(im.begin(), im.end(), 0.0);
            for (int i = 0; i < 16; ++i) {
                const double a = -2.0 * M_PI * nib[w][i] / 16.0;
                re[(size_t)i * stride] = std::cos(a);
                im[(size_t)i * stride] = std::sin(a);
            }
            outs[w] = encrypt(re.data(), im.data());
        }
        *oh = outs[0];
        *ol = outs[1];
    }

    // ------------------------------------------------------------------ raw access
    void export_ct(aesfhe_handle h, u32* out, u64 words) {
        const Ct& c0 = ct(h);
        Ct c = ensure_ntt(c0, false);
        if (words < c.words) throw std::runtime_error("export buffer too small");
        HIP_OK(hipMemcpyAsync(out, c.data, c.words * sizeof(u32), hipMemcpyDeviceToHost, st_));
        HIP_OK(hipStreamSynchronize(st_));
        if (c.data != c0.data) release(c);
    }
    aesfhe_handle import_ct(int level, int npoly, const u32* data) {
        if (level < 0 || level > hp_.L + 1 || npoly < 1 || npoly > 3) throw std::runtime_error("import: bad level/npoly");
        Ct c = alloc_ct(level, npoly);
        HIP_OK(hipMemcpyAsync(c.data, data, c.words * sizeof(u32), hipMemcpyHostToDevice, st_));
        HIP_OK(hipStreamSynchronize(st_));
        return put_ct(c);
    }
    void export_dev(const u32* d, size_t words, u32* out) {
        HIP_OK(hipMemcpyAsync(out, d, words * sizeof(u32), hipMemcpyDeviceToHost, st_));
        HIP_OK(hipStreamSynchronize(st_));
    }
    void export_secret(u32* out) {
        if (!d_s_) throw std::runtime_error("keys not generated");
        export_dev(d_s_, (size_t)hp_.n_tot() * hp_.n, out);
    }
    void export_pk(u32* out) {
        if (!d_pk_) throw std::runtime_error("keys not generated");
        export_dev(d_pk_, (size_t)2 * hp_.n_q * hp_.n, out);
    }
    void export_ksk(u64 g, u32* out) { export_dev(ksk(g), ksk_words(), out); }
    void debug_ntt(u32* data, int rows, int first_prime, int inverse) {
        u32* d = tmp(rows);
        HIP_OK(hipMemcpyAsync(d, data, sizeof(u32) * rows * hp_.n, hipMemcpyHostToDevice, st_));
        LimbMap m{rows, first_prime, 0};
        if (inverse) intt(d, rows, rows, m);
        else ntt(d, rows, rows, m);
        export_dev(d, (size_t)rows * hp_.n, data);
        untmp(d, rows);
    }
    void debug_keyswitch(int level, u64 g, const u32* d_host, u32* out) {
        const int nl = level + 2;
        u32* d = tmp(nl);
        HIP_OK(hipMemcpyAsync(d, d_host, sizeof(u32) * nl * hp_.n, hipMemcpyHostToDevice, st_));
        Ct o = keyswitch(d, level, ksk(g), nullptr, nullptr);
        export_dev(o.data, o.words, out);
        release(o);
        untmp(d, nl);
    }
    u64 counter(int i) const { return i < C_N ? cnt_[i] : 0; }
    void reset_counters() { std::memset(cnt_, 0, sizeof(cnt_)); }

private:
    u32* dev_alloc(size_t words) {
        void* p = nullptr;
        HIP_OK(hipMalloc(&p, words * sizeof(u32)));
        owned_.push_back(p);
        return (u32*)p;
    }
    template <class T>
    T* dev_upload(const std::vector<T>& h) {
        void* p = nullptr;
        HIP_OK(hipMalloc(&p, h.size() * sizeof(T)));
        owned_.push_back(p);
        HIP_OK(hipMemcpy(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
        return (T*)p;
    }

    void build_tables() {
        const int n = hp_.n, nt = hp_.n_tot(), logn = hp_.logn;
        std::vector<PrimeConst> pc(nt);
        std::vector<u32> psi((size_t)nt * n), psip((size_t)nt * n), ipsi((size_t)nt * n), ipsip((size_t)nt * n);
        im_.resize(nt);
        for (int i = 0; i < nt; ++i) {
            const u32 q = hp_.mod[i], w = hp_.psi[i], iw = hinvm(w, q);
            pc[i].q = q;
            pc[i].mu = barrett_pre(q);
            pc[i].ninv = hinvm((u32)n % q, q);
            pc[i].ninv_p = shoup_pre(pc[i].ninv, q);
            pc[i].im = hpowm(w, n / 2, q);
            pc[i].im_p = shoup_pre(pc[i].im, q);
            im_[i] = pc[i].im;
            u64 p = 1, ip = 1;
            for (int k = 0; k < n; ++k) {
                const u32 r = hbitrev((u32)k, logn);
                const size_t at = (size_t)i * n + r;
                psi[at] = (u32)p;
                psip[at] = shoup_pre((u32)p, q);
                ipsi[at] = (u32)ip;
                ipsip[at] = shoup_pre((u32)ip, q);
                p = p * w % q;
                ip = ip * iw % q;
            }
        }
        T_.pc = dev_upload(pc);
        T_.psi = dev_upload(psi);
        T_.psip = dev_upload(psip);
        T_.ipsi = dev_upload(ipsi);
        T_.ipsip = dev_upload(ipsip);
        T_.logn = logn;

        const auto& q = hp_.mod;
        auto mulm = [](u64 a, u64 b, u32 m) { return (u32)(a % m * (b % m) % m); };
        // rescale: per level l >= 1, q_{l+1}^{-1} mod q_t for t <= l
        std::vector<u32> rq;
        rescale_off_.assign(hp_.L + 2, 0);
        for (int l = 1; l <= hp_.L + 1; ++l) {
            rescale_off_[l] = rq.size();
            const u32 qr = q[l + 1];
            for (int t = 0; t <= l; ++t) {
                const u32 v = hinvm(qr % q[t], q[t]);
                rq.push_back(v);
                rq.push_back(shoup_pre(v, q[t]));
            }
        }
        d_rescale_qinv_ = dev_upload(rq);

        // gadget: P mod q_t on Q limbs 0..n_ks-1 (Shoup pairs), indexed by ext row
        std::vector<u32> gad(2 * (size_t)(hp_.n_ks + hp_.n_p), 0);
        for (int t = 0; t < hp_.n_ks; ++t) {
            u32 v = 1;
            for (int k = 0; k < hp_.n_p; ++k) v = mulm(v, q[hp_.p_off() + k], q[t]);
            gad[2 * t] = v;
            gad[2 * t + 1] = shoup_pre(v, q[t]);
        }
        d_gadget_ = dev_upload(gad);

        // ModUp tables per (level, digit): [h][ne] Shoup pairs of qhat_i mod target, then [h] qhat_i^{-1} mod q_i
        std::vector<u32> mu;
        modup_off_.assign((size_t)(hp_.L + 1) * hp_.dnum, 0);
        for (int l = 0; l <= hp_.L; ++l) {
            const int nl = l + 2, ne = nl + hp_.n_p;
            for (int j = 0; j < hp_.dnum; ++j) {
                const int lo = j * hp_.alpha;
                modup_off_[(size_t)l * hp_.dnum + j] = mu.size();
                if (lo >= nl) continue;
                const int h = std::min(hp_.alpha, nl - lo);
                for (int i = 0; i < h; ++i)
                    for (int x = 0; x < ne; ++x) {
                        const u32 tq = x < nl ? q[x] : q[hp_.p_off() + x - nl];
                        u32 v = 1;
                        for (int k = 0; k < h; ++k)
                            if (k != i) v = mulm(v, q[lo + k], tq);
                        mu.push_back(v);
                        mu.push_back(shoup_pre(v, tq));
                    }
                for (int i = 0; i < h; ++i) {
                    const u32 qi = q[lo + i];
                    u32 v = 1;
                    for (int k = 0; k < h; ++k)
                        if (k != i) v = mulm(v, q[lo + k], qi);
                    const u32 inv = hinvm(v, qi);
                    mu.push_back(inv);
                    mu.push_back(shoup_pre(inv, qi));
                }
                for (int x = 0; x < ne; ++x) {  // -Q_digit mod target
                    const u32 tq = x < nl ? q[x] : q[hp_.p_off() + x - nl];
                    u32 v = 1;
                    for (int k = 0; k < h; ++k) v = mulm(v, q[lo + k], tq);
                    mu.push_back(v ? tq - v : 0);
                }
            }
        }
        d_modup_ = dev_upload(mu);  // per (level, digit): [h][ne] qhat pairs, [h] qhat^-1 pairs, [ne] -Q

        // ModDown tables per level: [np][nl] Shoup pairs of phat_k mod q_t; phat_k^{-1} mod p_k; P^{-1} mod q_t
        std::vector<u32> md;
        moddown_off_.assign(hp_.L + 2, 0);
        const int np = hp_.n_p;
        for (int l = 0; l <= hp_.L; ++l) {
            const int nl = l + 2;
            moddown_off_[l] = md.size();
            for (int k = 0; k < np; ++k)
                for (int t = 0; t < nl; ++t) {
                    u32 v = 1;
                    for (int m2 = 0; m2 < np; ++m2)
                        if (m2 != k) v = mulm(v, q[hp_.p_off() + m2], q[t]);
                    md.push_back(v);
                    md.push_back(shoup_pre(v, q[t]));
                }
        }
        d_moddown_ = dev_upload(md);
        std::vector<u32> phinv;
        for (int k = 0; k < np; ++k) {
            const u32 pk = q[hp_.p_off() + k];
            u32 v = 1;
            for (int m2 = 0; m2 < np; ++m2)
                if (m2 != k) v = mulm(v, q[hp_.p_off() + m2], pk);
            const u32 inv = hinvm(v, pk);
            phinv.push_back(inv);
            phinv.push_back(shoup_pre(inv, pk));
        }
        d_moddown_phinv_ = dev_upload(phinv);
        std::vector<u32> pinv, negp;
        for (int t = 0; t < hp_.n_q; ++t) {
            u32 v = 1;
            for (int k = 0; k < np; ++k) v = mulm(v, q[hp_.p_off() + k], q[t]);
            const u32 inv = hinvm(v, q[t]);
            pinv.push_back(inv);
            pinv.push_back(shoup_pre(inv, q[t]));
            negp.push_back(v ? q[t] - v : 0);
        }
        d_pinv_ = dev_upload(pinv);
        d_negp_ = dev_upload(negp);

        void* r = nullptr;
        HIP_OK(hipMalloc(&r, kRingWords * sizeof(u32)));
        owned_.push_back(r);
        ring_ = (u32*)r;
        void* rh = nullptr;
        HIP_OK(hipHostMalloc(&rh, kRingWords * sizeof(u32), hipHostMallocDefault));
        ring_host_ = (u32*)rh;
    }

    HostParams hp_;
    Embedding emb_;
    DevTables T_;
    hipStream_t st_ = nullptr;
    int device_ = 0;
    Pool pool_;
    std::vector<void*> owned_;
    std::unordered_map<aesfhe_handle, Ct> cts_;
    std::unordered_map<aesfhe_handle, Pt> pts_;
    aesfhe_handle next_ = 1;
    u32* d_s_ = nullptr;
    u32* d_pk_ = nullptr;
    std::map<u64, u32*> ksk_;
    u64 enc_ctr_ = 0;
    std::vector<u32> im_;
    u32* d_rescale_qinv_ = nullptr;
    std::vector<size_t> rescale_off_;
    u32* d_gadget_ = nullptr;
    u32* d_modup_ = nullptr;
    std::vector<size_t> modup_off_;
    u32* d_moddown_ = nullptr;
    u32* d_moddown_phinv_ = nullptr;
    std::vector<size_t> moddown_off_;
    u32* d_pinv_ = nullptr;
    u32* d_negp_ = nullptr;
    static constexpr size_t kRingWords = 1 << 20;
    u32* ring_ = nullptr;
    u32* ring_host_ = nullptr;
    size_t ring_off_ = 0;
    u64 cnt_[C_N] = {};

public:
    KernelProfiler prof_;
    void activate() { prof_set(&prof_); }
};

}  // namespace

// =====================================================================================
// C ABI
// =====================================================================================
struct aesfhe_ctx {
    std::unique_ptr<Engine> eng;
    std::string err;
};

#define API_BEGIN                          \
    if (!ctx) return -2;                   \
    if (ctx->eng) ctx->eng->activate();    \
    try {
#define API_END                         \
    return 0;                           \
    }                                   \
    catch (const std::exception& e) {   \
        ctx->err = e.what();            \
        return -1;                      \
    }

extern "C" {

int aesfhe_create(aesfhe_ctx** out, int log_n, int max_level, int dnum, int device_id, uint64_t seed) {
    static thread_local std::string create_err;
    *out = nullptr;
    auto* c = new aesfhe_ctx();
    try {
        c->eng.reset(new Engine(log_n, max_level, dnum, device_id, seed));
    } catch (const std::exception& e) {
        c->err = e.what();
        *out = c;
        return -1;
    }
    *out = c;
    return 0;
}
int aesfhe_destroy(aesfhe_ctx* ctx) {
    delete ctx;
    return 0;
}
const char* aesfhe_last_error(aesfhe_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }
int aesfhe_keygen(aesfhe_ctx* ctx) {
    API_BEGIN ctx->eng->keygen();
    API_END
}
int aesfhe_slot_count(aesfhe_ctx* ctx) { return ctx && ctx->eng ? ctx->eng->slot_count() : -1; }
int aesfhe_max_level(aesfhe_ctx* ctx) { return ctx && ctx->eng ? ctx->eng->hp().L : -1; }
int aesfhe_set_fresh_level(aesfhe_ctx* ctx, int level) {
    API_BEGIN ctx->eng->set_fresh(level);
    API_END
}
int aesfhe_info(aesfhe_ctx* ctx, int32_t* info) {
    API_BEGIN const HostParams& p = ctx->eng->hp();
    int32_t v[8] = {p.n, p.L, p.n_q, p.n_ks, p.n_p, p.alpha, p.dnum, p.logn};
    std::memcpy(info, v, sizeof(v));
    API_END
}
int aesfhe_moduli(aesfhe_ctx* ctx, uint32_t* out) {
    API_BEGIN const auto& m = ctx->eng->hp().mod;
    std::memcpy(out, m.data(), m.size() * sizeof(u32));
    API_END
}
int aesfhe_scales(aesfhe_ctx* ctx, double* out) {
    API_BEGIN const auto& d = ctx->eng->hp().delta;
    std::memcpy(out, d.data(), d.size() * sizeof(double));
    API_END
}
int aesfhe_sync(aesfhe_ctx* ctx) {
    API_BEGIN ctx->eng->sync();
    API_END
}
int aesfhe_free(aesfhe_ctx* ctx, aesfhe_handle h) {
    API_BEGIN ctx->eng->free_handle(h);
    API_END
}
int aesfhe_level(aesfhe_ctx* ctx, aesfhe_handle h, int32_t* level, int32_t* npoly) {
    API_BEGIN const Ct& c = ctx->eng->ct(h);
    *level = c.level;
    *npoly = c.npoly;
    API_END
}
int aesfhe_plaintext(aesfhe_ctx* ctx, const double* re, const double* im, int n, aesfhe_handle* out) {
    API_BEGIN* out = ctx->eng->new_pt(re, im, n);
    API_END
}
int aesfhe_encrypt(aesfhe_ctx* ctx, const double* re, const double* im, int n, aesfhe_handle* out) {
    API_BEGIN Engine& e = *ctx->eng;
    const int s = e.slot_count();
    std::vector<double> r(s, 0.0), i(s, 0.0);
    for (int j = 0; j < s && j < n; ++j) r[j] = re[j], i[j] = im ? im[j] : 0.0;
    *out = e.encrypt(r.data(), i.data());
    API_END
}
int aesfhe_decrypt(aesfhe_ctx* ctx, aesfhe_handle ct, double* re, double* im, int n) {
    API_BEGIN Engine& e = *ctx->eng;
    if (n < e.slot_count()) throw std::runtime_error("decrypt: output buffers shorter than slot_count");
    e.decrypt(ct, re, im);
    API_END
}
#define CT_OP(expr)         \
    API_BEGIN Engine& e = *ctx->eng; \
    *out = e.put_ct(expr);  \
    API_END

int aesfhe_add(aesfhe_ctx* ctx, aesfhe_handle a, aesfhe_handle b, aesfhe_handle* out) { CT_OP(e.add_sub(e.ct(a), e.ct(b), false)) }
int aesfhe_sub(aesfhe_ctx* ctx, aesfhe_handle a, aesfhe_handle b, aesfhe_handle* out) { CT_OP(e.add_sub(e.ct(a), e.ct(b), true)) }
int aesfhe_add_pt(aesfhe_ctx* ctx, aesfhe_handle c, aesfhe_handle p, aesfhe_handle* out) { CT_OP(e.add_pt(e.ct(c), p)) }
int aesfhe_add_scalar(aesfhe_ctx* ctx, aesfhe_handle c, double re, double im, aesfhe_handle* out) {
    CT_OP(e.add_scalar(e.ct(c), re, im))
}
int aesfhe_mul_scalar(aesfhe_ctx* ctx, aesfhe_handle c, double re, double im, aesfhe_handle* out) {
    CT_OP(e.mul_scalar(e.ct(c), re, im))
}
int aesfhe_mul_pt(aesfhe_ctx* ctx, aesfhe_handle c, aesfhe_handle p, aesfhe_handle* out) { CT_OP(e.mul_pt(e.ct(c), p)) }
int aesfhe_mul(aesfhe_ctx* ctx, aesfhe_handle a, aesfhe_handle b, int relin, aesfhe_handle* out) {
    CT_OP(e.mul(e.ct(a), e.ct(b), relin != 0))
}
int aesfhe_relinearize(aesfhe_ctx* ctx, aesfhe_handle c, aesfhe_handle* out) { CT_OP(e.relinearize(e.ct(c))) }
int aesfhe_rescale(aesfhe_ctx* ctx, aesfhe_handle c, aesfhe_handle* out) {
    API_BEGIN Engine& e = *ctx->eng;
    Ct x = e.ensure_ntt(e.ct(c));
    Ct o = e.rescale(x);
    if (x.data != e.ct(c).data) e.release(x);
    *out = e.put_ct(o);
    API_END
}
int aesfhe_level_down(aesfhe_ctx* ctx, aesfhe_handle c, int level, aesfhe_handle* out) { CT_OP(e.level_down(e.ct(c), level)) }
int aesfhe_rotate(aesfhe_ctx* ctx, aesfhe_handle c, int steps, aesfhe_handle* out) { CT_OP(e.rotate(e.ct(c), steps)) }
int aesfhe_conjugate(aesfhe_ctx* ctx, aesfhe_handle c, aesfhe_handle* out) { CT_OP(e.conjugate(e.ct(c))) }
int aesfhe_power_basis(aesfhe_ctx* ctx, aesfhe_handle c, int degree, aesfhe_handle* out) {
    API_BEGIN ctx->eng->power_basis(c, degree, out);
    API_END
}
int aesfhe_to_ntt(aesfhe_ctx* ctx, aesfhe_handle c, aesfhe_handle* out) { CT_OP(e.to_ntt(e.ct(c))) }
int aesfhe_to_intt(aesfhe_ctx* ctx, aesfhe_handle c, aesfhe_handle* out) { CT_OP(e.to_intt(e.ct(c))) }
int aesfhe_bootstrap(aesfhe_ctx* ctx, aesfhe_handle, aesfhe_handle*) {
    if (!ctx) return -2;
    ctx->err = "bootstrap is not available in this build (use_bootstrap parameter set pending)";
    return -1;
}
int aesfhe_renorm_pair(aesfhe_ctx* ctx, aesfhe_handle hi, aesfhe_handle lo, aesfhe_handle* out_hi, aesfhe_handle* out_lo) {
    API_BEGIN ctx->eng->renorm_pair(hi, lo, out_hi, out_lo);
    API_END
}
int aesfhe_export(aesfhe_ctx* ctx, aesfhe_handle c, uint32_t* out, uint64_t words) {
    API_BEGIN ctx->eng->export_ct(c, out, words);
    API_END
}
int aesfhe_import(aesfhe_ctx* ctx, int level, int npoly, const uint32_t* data, aesfhe_handle* out) {
    API_BEGIN* out = ctx->eng->import_ct(level, npoly, data);
    API_END
}
int aesfhe_export_secret(aesfhe_ctx* ctx, uint32_t* out) {
    API_BEGIN ctx->eng->export_secret(out);
    API_END
}
int aesfhe_export_pk(aesfhe_ctx* ctx, uint32_t* out) {
    API_BEGIN ctx->eng->export_pk(out);
    API_END
}
int aesfhe_export_ksk(aesfhe_ctx* ctx, uint64_t g, uint32_t* out) {
    API_BEGIN ctx->eng->export_ksk(g, out);
    API_END
}
int aesfhe_debug_ntt(aesfhe_ctx* ctx, uint32_t* data, int rows, int first_prime, int inverse) {
    API_BEGIN ctx->eng->debug_ntt(data, rows, first_prime, inverse);
    API_END
}
int aesfhe_debug_keyswitch(aesfhe_ctx* ctx, int level, uint64_t g, const uint32_t* d, uint32_t* out) {
    API_BEGIN ctx->eng->debug_keyswitch(level, g, d, out);
    API_END
}
int aesfhe_counters(aesfhe_ctx* ctx, uint64_t* out, int n) {
    API_BEGIN for (int i = 0; i < n; ++i) out[i] = ctx->eng->counter(i);
    API_END
}
int aesfhe_profile(aesfhe_ctx* ctx, uint32_t mask) {
    API_BEGIN ctx->eng->prof_.flush();
    ctx->eng->prof_.mask = mask;
    API_END
}
int aesfhe_kernel_stats(aesfhe_ctx* ctx, double* out, int n, int reset) {
    API_BEGIN KernelProfiler& p = ctx->eng->prof_;
    p.flush();
    for (int k = 0; k < n && k < KID_N; ++k) {
        out[3 * k] = (double)p.launches[k];
        out[3 * k + 1] = p.ms[k];
        out[3 * k + 2] = p.bytes[k];
    }
    if (reset) p.reset();
    API_END
}
int aesfhe_reset_counters(aesfhe_ctx* ctx) {
    API_BEGIN ctx->eng->reset_counters();
    API_END
}

}  // extern "C"
