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
#include <cstdlib>
#include <deque>
#include <functional>
#include <chrono>
#include <map>
#include <mutex>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/aesfhe.h"
#include "bootstrap.h"
#include "encoder.h"
#include "kernels.h"
#include "launch.h"
#include "params.h"

namespace {

#define HIP_OK(expr)                                                                                      \
    do {                                                                                                  \
        hipError_t e_ = (expr);                                                                           \
        if (e_ != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_) + \
                                                       " at " #expr);                                      \
    } while (0)

inline u64 stream_id(u64 kind, u64 a, u64 b) { return (kind << 56) | (a << 16) | b; }

// 256-bit key of a 64-bit seed (test / parity contexts): the seed in key words 0, 1
inline void seed_key(u64 seed, u32 key[8]) {
    for (int i = 0; i < 8; ++i) key[i] = 0;
    key[0] = (u32)seed;
    key[1] = (u32)(seed >> 32);
}

// ---------------------------------------------------------------------------------
// device memory pool: exact-size free lists (ciphertext sizes repeat constantly)
// ---------------------------------------------------------------------------------
// Out of memory: a failed hipMalloc releases the cached free lists (the
// engine's on_oom hook: every pool that no branch thread is using), after a device sync so no
// queued kernel still reads a freed buffer, and retries once; only a second failure throws.
// AESFHE_POOL_LIMIT_MB caps the bytes a pool may hold (a simulated smaller HBM: tests force the
// release-and-retry path with it).
class Pool {
public:
    std::function<void()> on_oom;  // set by the engine: release the free lists it may release
    u32* try_get(size_t words) {
        auto it = free_.find(words);
        if (it == free_.end() || it->second.empty()) return nullptr;
        u32* p = it->second.back();
        it->second.pop_back();
        return p;
    }
    // moves every free buffer of `o` into this pool
    void absorb(Pool& o) {
        for (auto& kv : o.free_) {
            auto& fl = free_[kv.first];
            fl.insert(fl.end(), kv.second.begin(), kv.second.end());
        }
        o.free_.clear();
        bytes_ += o.bytes_;
        o.bytes_ = 0;
    }
    u32* get(size_t words) {
        if (u32* p = try_get(words)) return p;
        const size_t b = words * sizeof(u32);
        void* p = nullptr;
        hipError_t e = raw_alloc(&p, b);
        if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) {
            (void)hipGetLastError();  // not sticky, but leave no error for the next launch check
            ++oom_retries_;
            if (on_oom) on_oom();
            else trim();
            e = raw_alloc(&p, b);
        }
        if (e != hipSuccess)
            throw std::runtime_error(std::string("device memory exhausted after releasing the cached buffers: ") + hipGetErrorString(e));
        bytes_ += b;
        return (u32*)p;
    }
    void put(u32* p, size_t words) {
        if (p) free_[words].push_back(p);
    }
    // frees every cached (free-list) buffer; the caller has synchronised the device
    size_t trim() {
        size_t freed = 0;
        for (auto& kv : free_)
            for (u32* p : kv.second) {
                (void)hipFree(p);
                freed += kv.first * sizeof(u32);
            }
        free_.clear();
        bytes_ = bytes_ > freed ? bytes_ - freed : 0;
        return freed;
    }
    void release_all() { trim(); }
    size_t bytes() const { return bytes_; }
    unsigned long long oom_retries() const { return oom_retries_; }

private:
    hipError_t raw_alloc(void** p, size_t b) {
        if (limit_ && bytes_ + b > limit_) return hipErrorOutOfMemory;
        return hipMalloc(p, b);
    }
    // read when the context is created (a test sets it for one context only)
    size_t limit_ = std::getenv("AESFHE_POOL_LIMIT_MB") ? (size_t)std::atoll(std::getenv("AESFHE_POOL_LIMIT_MB")) << 20 : (size_t)0;
    std::unordered_map<size_t, std::vector<u32*>> free_;
    size_t bytes_ = 0;
    unsigned long long oom_retries_ = 0;
};

// A ciphertext tensor.  `level` is the DATA level (nl(level) limbs per polynomial); `pend`
// rescales are still owed, so the logical level is level - pend and the raw scale is
// raw_scale(level, pend).  `lazy` marks work the engine deferred on its own
// (relinearisation of a product, rescales of scalar products): the API shows such a
// ciphertext as 2 polynomials at its logical level.  `zero`: an exact encryption of 0.
struct Ct {
    u32* data = nullptr;
    size_t words = 0;
    int level = 0;
    int npoly = 2;          // polynomials in data, all batched ciphertexts together
    int nb = 1;             // batched ciphertexts stacked in data: [m][npoly / nb][nl] (bootstrap_pair)
    bool ntt = true;
    int pend = 0;
    bool lazy = false;
    bool zero = false;
    int sid = 0;            // stream of the call that stored the handle
    unsigned epoch = 0;     // fork section it was stored in (0: outside any)
};

// coefficient set of a fused LUT evaluation: C[n_a][n_b] (n_b = 1: univariate)
struct Lut {
    int n_a = 0, n_b = 0;
    std::vector<double> re, im;
    double c0_re = 0.0, c0_im = 0.0;
    std::map<std::string, std::pair<u32*, size_t>> cst;  // (output level, element levels) -> constants
};

struct Pt {
    std::vector<double> re, im;
    bool constant = false;
    std::map<int, std::pair<u32*, size_t>> enc;  // 2*level + mult -> (NTT-form encoding, words)
};

enum Counter { C_MUL, C_RELIN, C_ROT, C_CONJ, C_PTMUL, C_SCALAR, C_RESCALE, C_NTT_ROWS, C_KS, C_ENC, C_DEC, C_BOOT, C_ADD, C_LUT, C_N };

class Engine {
public:
    static constexpr int kStreams = 3;  // see fork() / join()
    PrngKey pkey() const {
        PrngKey k;
        for (int i = 0; i < 8; ++i) k.w[i] = hp_.key[i];
        return k;
    }
    Engine(int logn, int L1, int n_double, int dnum, int device, const u32 key[8]) : emb_(logn) {
        std::string err = hp_.build(logn, L1, n_double, dnum, key);
        if (!err.empty()) throw std::runtime_error(err);
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
            throw std::runtime_error("no HIP device visible: the MI355X engine has no CPU fallback");
        if (device < 0 || device >= ndev) throw std::runtime_error("device_id out of range");
        device_ = device;
        HIP_OK(hipSetDevice(device_));
        for (int k = 0; k < kStreams; ++k) {
            HIP_OK(hipStreamCreateWithFlags(&streams_[k], hipStreamNonBlocking));
            HIP_OK(hipEventCreateWithFlags(&fj_ev_[k], hipEventDisableTiming));
        }
        build_tables();
        for (int k = 0; k < kStreams; ++k)
            pools_[k].on_oom = [this, k] {
                // queued kernels may still read cached buffers; after the device sync none does.  Every
                // pool's cache goes, also inside fork/join: API calls serialise on ctx->mu, so no other
                // thread is allocating, and a branch allocating from pools_[0] must still be able to
                // reclaim what pools_[1..] hold
                (void)hipDeviceSynchronize();
                (void)k;
                for (int j = 0; j < kStreams; ++j) pools_[j].trim();
            };
    }
    unsigned long long oom_retries() const {
        unsigned long long n = 0;
        for (const auto& pl : pools_) n += pl.oom_retries();
        return n;
    }
    size_t pool_bytes() const {
        size_t n = 0;
        for (const auto& pl : pools_) n += pl.bytes();
        return n;
    }
    ~Engine() {
        (void)hipSetDevice(device_);
        (void)hipDeviceSynchronize();
        for (auto& kv : cts_) pools_[0].put(kv.second.data, kv.second.words);
        for (auto& kv : pts_)
            for (auto& e : kv.second.enc) pools_[0].put(e.second.first, e.second.second);
        for (auto& d : deferred_) pools_[0].put(d.first, d.second);
        for (auto& pl : pools_) pl.release_all();
        for (void* p : owned_) (void)hipFree(p);
        for (auto& kv : ksk_) (void)hipFree(kv.second);
        for (int k = 0; k < kStreams; ++k) {
            (void)hipEventDestroy(fj_ev_[k]);
            (void)hipStreamDestroy(streams_[k]);
        }
    }

    const HostParams& hp() const { return hp_; }
    void set_fresh(int level) {
        if (level < 0 || level > hp_.L1 || (hp_.L > hp_.L1 && level >= hp_.L1))
            throw std::runtime_error("fresh level must lie in the single-prime region below its top");
        hp_.fresh = level;
    }
    int slot_count() const { return hp_.n / 2; }
    void sync() {
        for (int k = 0; k < kStreams; ++k) HIP_OK(hipStreamSynchronize(streams_[k]));
    }

    // ------------------------------------------------------------------ streams (fork / join)
    // the calling host thread's stream and buffer pool: 0 unless bound to a branch stream
    static thread_local int t_sidx;
    hipStream_t S() const { return streams_[t_sidx]; }
    Pool& pool() { return pools_[t_sidx]; }
    // allocation on the calling thread's stream: its own pool, then (branch streams) buffers
    // stream 0 released before the fork -- ordered before every branch by the fork event
    u32* alloc_words(size_t words) {
        if (t_sidx != 0) {
            if (u32* p = pools_[t_sidx].try_get(words)) return p;
            if (no_share_) return pools_[t_sidx].get(words);
        }
        return pools_[0].get(words);
    }
    bool no_share_ = std::getenv("AESFHE_NO_POOL_SHARE") != nullptr;  // debug switch
    bool fj_active_ = false;
    unsigned fj_epoch_ = 0;
    static int streams() { return kStreams; }
    void bind_stream(int k) {
        if (k < 0 || k >= kStreams) throw std::runtime_error("bind_stream: stream index out of range");
        t_sidx = k;
    }
    // branch streams start after everything already queued on stream 0
    void fork() {
        if (t_sidx != 0) throw std::runtime_error("fork must be called from the main stream");
        HIP_OK(hipEventRecord(fj_ev_[0], streams_[0]));
        for (int k = 1; k < kStreams; ++k) HIP_OK(hipStreamWaitEvent(streams_[k], fj_ev_[0], 0));
        fj_active_ = true;
        ++fj_epoch_;
    }
    // stream 0 continues after every branch; handles the branch threads dropped go back to
    // stream 0's pool only now (another stream may have read them until here)
    void join() {
        if (t_sidx != 0) throw std::runtime_error("join must be called from the main stream");
        for (int k = 1; k < kStreams; ++k) {
            HIP_OK(hipEventRecord(fj_ev_[k], streams_[k]));
            HIP_OK(hipStreamWaitEvent(streams_[0], fj_ev_[k], 0));
        }
        for (auto& d : deferred_) pools_[0].put(d.first, d.second);
        deferred_.clear();
        for (int k = 1; k < kStreams; ++k) pools_[0].absorb(pools_[k]);  // stream 0 is after them now
        fj_active_ = false;
    }
    void give_back(u32* p, size_t words) {
        if (t_sidx != 0 || fj_active_) deferred_.push_back({p, words});
        else pools_[0].put(p, words);
    }

    // ------------------------------------------------------------------ handles
    aesfhe_handle put_ct(Ct c) {
        aesfhe_handle h = next_++;
        c.sid = t_sidx;
        c.epoch = fj_active_ ? fj_epoch_ : 0;
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
            give_back(it->second.data, it->second.words);
            cts_.erase(it);
            return;
        }
        auto il = luts_.find(h);
        if (il != luts_.end()) {
            for (auto& e : il->second.cst) give_back(e.second.first, e.second.second);
            luts_.erase(il);
            return;
        }
        auto ip = pts_.find(h);
        if (ip != pts_.end()) {
            for (auto& e : ip->second.enc) give_back(e.second.first, e.second.second);
            pts_.erase(ip);
        }
    }
    void free_lut(aesfhe_handle h) {
        if (!luts_.count(h)) throw std::runtime_error("aesfhe_lut_free: not a LUT handle");
        free_handle(h);
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

    Ct alloc_ct(int level, int npoly, int nb = 1) {
        Ct c;
        c.level = level;
        c.npoly = npoly;
        c.nb = nb;
        c.words = (size_t)npoly * hp_.nl(level) * hp_.n;
        c.data = alloc_words(c.words);
        return c;
    }
    u32* tmp(size_t rows) { return alloc_words(rows * hp_.n); }
    void untmp(u32* p, size_t rows) { pool().put(p, rows * hp_.n); }

    // ------------------------------------------------------------------ maps
    static LimbMap qmap() { return LimbMap{1 << 30, 0, 0}; }
    LimbMap extmap(int nl) const { return LimbMap{nl, 0, hp_.p_off()}; }
    static LimbMap single(int prime) { return LimbMap{1, prime, 0}; }

    void ntt(u32* d, int rows, int nl, LimbMap m) {
        launch_ntt_fwd(S(), T_, d, rows, nl, m);
        cnt_[C_NTT_ROWS] += rows;
    }
    void intt(u32* d, int rows, int nl, LimbMap m) {
        launch_ntt_inv(S(), T_, d, rows, nl, m);
        cnt_[C_NTT_ROWS] += rows;
    }
    // out-of-place forms (dense rows unless a RowMap is given)
    void ntt(u32* dst, const u32* src, int rows, RowMap rm, LimbMap m) {
        launch_ntt_fwd(S(), T_, dst, src, rows, rm, m);
        cnt_[C_NTT_ROWS] += rows;
    }
    void intt(u32* dst, const u32* src, int rows, RowMap rm, LimbMap m, const u32* post = nullptr) {
        launch_ntt_inv(S(), T_, dst, src, rows, rm, m, post);
        cnt_[C_NTT_ROWS] += rows;
    }
    // a base conversion and the forward NTT of its output: one fused pass-1 launch when the ring
    // has it (the INTT that made cb's sources then carried the qhat^{-1} factors), else
    // k_base_convert into cb.dst and the NTT of those rows
    bool fused_conv(bool up) const { return (ntt_conv_fused_mask(T_) >> (up ? 0 : 1)) & 1; }

    // ------------------------------------------------------------------ keys
    void keygen() {
        const int n = hp_.n, nt = hp_.n_tot();
        if (!d_s_) {
            d_s_ = dev_alloc((size_t)nt * n);
            launch_sample_small(S(), T_, d_s_, nt, qmap(), pkey(), stream_id(1, 0, 0), 0);
            ntt(d_s_, nt, nt, qmap());
        }
        if (!d_pk_) {
            const int nq = hp_.n_q;
            d_pk_ = dev_alloc((size_t)2 * nq * n);
            u32* e = tmp(nq);
            launch_sample_uniform(S(), T_, d_pk_ + (size_t)nq * n, nq, qmap(), pkey(), stream_id(2, 0, 0));
            launch_sample_small(S(), T_, e, nq, qmap(), pkey(), stream_id(3, 0, 0), 1);
            ntt(e, nq, nq, qmap());
            launch_keygen_combine(S(), T_, d_pk_, d_pk_ + (size_t)nq * n, d_s_, e, nullptr, nullptr, nq, qmap(), 0, 0);
            untmp(e, nq);
        }
        ksk(0);
        ksk(conj_galois());
        sync();
    }
    u64 conj_galois() const { return 2ull * hp_.n - 1; }
    // key tag of sigma_g(s)^2 -> s (g odd, < 2N): the third polynomial of a deferred tensor read
    // through X -> X^g (galois_lazy)
    u64 tag_sq(u64 g) const { return 4ull * hp_.n + g; }
    bool is_tag_sq(u64 t) const { return t > 4ull * hp_.n && t < 6ull * hp_.n; }
    // sigma_g(s_sp) -> s: the sparse -> dense switch read through the first trace step's automorphism g
    u64 tag_s2d_rot(u64 g) const { return 8ull * hp_.n + g; }
    bool is_tag_s2d_rot(u64 t) const { return t > 8ull * hp_.n && t < 10ull * hp_.n; }
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
    // The dense -> sparse key of the bootstrap (step 2) is an RLWE sample under
    // the h = 32 sparse secret, so its modulus must stay small: it lives modulo
    // Q0 * P' only -- Q0 = q0 q1, the two base limbs of level 0 the bootstrap starts from, P' =
    // the first kD2sP special primes (~120 bits) -- not on all n_ks + n_p limbs (~1,700 bits,
    // where a sparse secret is recoverable and with it the dense secret).
    // Layout [2][kD2sQ + kD2sP][N].
    static constexpr int kD2sP = 2, kD2sQ = 2;
    int d2s_np() const { return std::min(kD2sP, hp_.n_p); }
    size_t ksk_words(u64 g) const {
        if (g == tag_d2s()) return (size_t)2 * (kD2sQ + d2s_np()) * hp_.n;
        return (size_t)hp_.dnum * 2 * (hp_.n_ks + hp_.n_p) * hp_.n;
    }
    double d2s_modulus_bits() const {
        double b = 0;
        for (int t = 0; t < kD2sQ; ++t) b += std::log2((double)hp_.mod[t]);
        for (int k = 0; k < d2s_np(); ++k) b += std::log2((double)hp_.mod[hp_.p_off() + k]);
        return b;
    }
    const u32* ksk_d2s() {
        const u64 g = tag_d2s();
        const int n = hp_.n, ne = kD2sQ + d2s_np();
        void* raw = nullptr;
        HIP_OK(hipMalloc(&raw, ksk_words(g) * sizeof(u32)));
        u32* b = (u32*)raw;
        u32* a = b + (size_t)ne * n;
        const LimbMap em = extmap(kD2sQ);  // rows 0, 1: q0, q1; then the first special primes
        u32* e = tmp(ne);
        launch_sample_uniform(S(), T_, a, ne, em, pkey(), stream_id(4, g, 0));
        launch_sample_small(S(), T_, e, ne, em, pkey(), stream_id(5, g, 0), 1);
        ntt(e, ne, ne, em);
        // b = -a s_sp + e + (P' mod q_t) s on the q0, q1 rows
        launch_keygen_combine(S(), T_, b, a, sparse_secret(), e, d_s_, d_d2s_ + d2s_off_.gad, ne, em, 0, kD2sQ);
        untmp(e, ne);
        ksk_[g] = b;
        HIP_OK(hipStreamSynchronize(S()));
        return b;
    }
    const u32* ksk(u64 g) {
        auto it = ksk_.find(g);
        if (it != ksk_.end()) return it->second;
        if (!d_s_) throw std::runtime_error("keys not generated");
        if (g == tag_d2s()) return ksk_d2s();
        const int n = hp_.n, nks = hp_.n_ks, np = hp_.n_p, nkey = nks + np;
        void* raw = nullptr;
        HIP_OK(hipMalloc(&raw, ksk_words(g) * sizeof(u32)));
        u32* key = (u32*)raw;
        // source secret s' (Q limbs 0..n_ks-1) and target secret (all primes) of the key
        u32* sp = tmp(nks);
        const u32* target = d_s_;
        if (g == 0) {
            launch_square(S(), T_, sp, d_s_, nks, nks, qmap());
        } else if (g == tag_s2d()) {  // sparse s_sp -> dense s
            launch_copy_rows(S(), T_, sp, sparse_secret(), nks);
        } else if (is_tag_s2d_rot(g)) {  // sigma_g'(s_sp) -> dense s
            launch_automorph(S(), T_, sp, sparse_secret(), g - 8ull * n, nks);
        } else if (is_tag_sq(g)) {    // sigma_g'(s)^2 -> s: the automorphism of a 3-polynomial tensor
            u32* s2 = tmp(nks);
            launch_square(S(), T_, s2, d_s_, nks, nks, qmap());
            launch_automorph(S(), T_, sp, s2, g - 4ull * n, nks);
            untmp(s2, nks);
        } else {
            launch_automorph(S(), T_, sp, d_s_, g, nks);
        }
        u32* e = tmp(nkey);
        const LimbMap em = extmap(nks);
        for (int j = 0; j < hp_.dnum; ++j) {
            u32* b = key + (size_t)j * 2 * nkey * n;
            u32* a = b + (size_t)nkey * n;
            launch_sample_uniform(S(), T_, a, nkey, em, pkey(), stream_id(4, g, j));
            launch_sample_small(S(), T_, e, nkey, em, pkey(), stream_id(5, g, j), 1);
            ntt(e, nkey, nkey, em);
            const int lo = j * hp_.alpha, hi = std::min(nks, lo + hp_.alpha);
            launch_keygen_combine(S(), T_, b, a, target, e, sp, d_gadget_, nkey, em, lo, hi);
        }
        untmp(e, nkey);
        untmp(sp, nks);
        ksk_[g] = key;
        HIP_OK(hipStreamSynchronize(S()));  // shared by every stream from now on
        return key;
    }

    // ------------------------------------------------------------------ codec
    // host: slots -> residues on limbs 0..nl-1 at `scale` (coefficient form)
    // residues on limbs 0..nl-1 (primes q_0..), then `np` limbs of the P block when np > 0
    void encode_host(const double* re, const double* im, double scale, int nl, std::vector<u32>& out, int np = 0) {
        const int n = hp_.n;
        std::vector<double> m(n);
        emb_.inverse(re, im, m.data());
        const int nr = nl + np;
        out.assign((size_t)nr * n, 0);
        // residues of the integer-valued double x = round(m_k scale): with k = floor(x / q)
        // the remainder fma(-q, k, x) is exact (it is small), one correction step fixes the
        // quotient's rounding; identical to the 128-bit integer reduction, ~20x cheaper
        std::vector<double> qd(nr), qinv(nr);
        for (int t = 0; t < nr; ++t) qd[t] = (double)hp_.mod[t < nl ? t : hp_.p_off() + t - nl], qinv[t] = 1.0 / qd[t];
        for (int k = 0; k < n; ++k) {
            const double y = m[k] * scale;
            const double x = std::fabs(y) < 4503599627370496.0 ? (double)std::llround(y) : y;
            for (int t = 0; t < nr; ++t) {
                double r = std::fma(-qd[t], std::floor(x * qinv[t]), x);
                if (r < 0) r += qd[t];
                if (r >= qd[t]) r -= qd[t];
                out[(size_t)t * n + k] = (u32)r;
            }
        }
    }
    u32* upload_ntt(const std::vector<u32>& host, int nl) {
        u32* d = tmp(nl);
        HIP_OK(hipMemcpyAsync(d, host.data(), host.size() * sizeof(u32), hipMemcpyHostToDevice, S()));
        HIP_OK(hipStreamSynchronize(S()));  // host vector may die after return
        ntt(d, nl, nl, qmap());
        return d;
    }

    aesfhe_handle encrypt(const double* re, const double* im) {
        if (!d_pk_) throw std::runtime_error("keys not generated");
        // encode at delta_f * q_{f+2} on limbs 0..f+2, encrypt at level f+1, rescale to f
        const int f = hp_.fresh, nq = hp_.nl(f) + 1;
        std::vector<u32> host;
        encode_host(re, im, hp_.delta[f] * (double)hp_.mod[hp_.nl(f)], nq, host);
        u32* m = upload_ntt(host, nq);
        Ct out = encrypt_ntt(m);
        untmp(m, nq);
        return put_ct(out);
    }
    // public-key encryption of an encoded message m (NTT form on nl(f) + 1 limbs, scale
    // delta_f q_{nl(f)}): c = (v pk0 + e0 + m, v pk1 + e1) at level f + 1, rescaled to f;
    // level < 0: the fresh level; any level 0..fresh works the same way (the public key
    // restricted to the first nl(f) + 1 limbs)
    // Encryption randomness (v, e0, e1) is drawn under its OWN key: the context key with the
    // per-process 64-bit nonce folded into key words 6-7 (aesfhe_set_enc_nonce).  Ranks of a
    // multi-GPU job share the context key (identical key sets) but not the nonce, so their i-th
    // encryptions never reuse (v, e) -- a reuse would make c_r - c_0 a noiseless encoding of
    // m_r - m_0.  Nonce 0 (the default of the C ABI) leaves the context key unchanged.
    PrngKey enc_key() const {
        PrngKey k = pkey();
        k.w[6] ^= (u32)enc_nonce_;
        k.w[7] ^= (u32)(enc_nonce_ >> 32);
        return k;
    }
    void set_enc_nonce(u64 nonce) { enc_nonce_ = nonce; }
    Ct encrypt_ntt(const u32* m, int level = -1) {
        const int f = level < 0 ? hp_.fresh : level;
        const int n = hp_.n, nq = hp_.nl(f) + 1;
        const int L = f;
        u32* v = tmp(nq);
        u32* e = tmp(2 * nq);
        const u64 ctr = enc_ctr_++;
        const PrngKey ek = enc_key();
        launch_sample_small(S(), T_, v, nq, qmap(), ek, stream_id(6, 0, ctr), 0);
        launch_sample_small(S(), T_, e, nq, qmap(), ek, stream_id(7, 0, ctr), 1);
        launch_sample_small(S(), T_, e + (size_t)nq * n, nq, qmap(), ek, stream_id(8, 0, ctr), 1);
        ntt(v, nq, nq, qmap());
        ntt(e, 2 * nq, nq, qmap());
        Ct top = alloc_ct(L + 1, 2);
        launch_add(S(), T_, e, e, m, nq, nq, qmap());  // e0 + m
        launch_fma_poly(S(), T_, top.data, e, d_pk_, v, nq, nq, qmap());
        launch_fma_poly(S(), T_, top.data + (size_t)nq * n, e + (size_t)nq * n, d_pk_ + (size_t)hp_.n_q * n, v, nq, nq, qmap());
        untmp(v, nq);
        untmp(e, 2 * nq);
        Ct out = rescale(top);
        release(top);
        cnt_[C_ENC]++;
        return out;
    }

    // B <= kEncMax messages (NTT form, member m at m + b m_ms words, nl(f) + 1 limbs each, scale
    // delta_f q_{nl(f)}) encrypted together: ONE sampling launch for every v, e0, e1, ONE NTT of
    // all of them, ONE combine, ONE rescale of the stacked result (nb = B) -- the same residues as
    // B encrypt_ntt calls (same PRNG streams, same arithmetic), 8 launches instead of 14 B
    // m_coef: m is in coefficient form and rides in e0 through the samples' NTT (launch_sample_enc),
    // the same residues as NTT(m) added in the combine
    Ct encrypt_many(const u32* m, int B, size_t m_ms, int level = -1, bool m_coef = false) {
        if (B < 1 || B > kEncMax) throw std::runtime_error("encrypt_many: batch too large");
        const int f = level < 0 ? hp_.fresh : level;
        const int nq = hp_.nl(f) + 1;
        u32* vee = tmp((size_t)B * 3 * nq);
        EncCtrs ec;
        ec.base = enc_ctr_;  // member b: counter base + b, as B single encryptions in a row
        enc_ctr_ += B;
        launch_sample_enc(S(), T_, vee, nq, B, enc_key(), ec, m_coef ? m : nullptr, m_ms);
        ntt(vee, B * 3 * nq, nq, qmap());
        Ct top = alloc_ct(f + 1, 2 * B, B);
        launch_enc_combine(S(), T_, top.data, vee, m_coef ? nullptr : m, m_ms, d_pk_, hp_.n_q, nq, B);
        untmp(vee, (size_t)B * 3 * nq);
        Ct out = rescale(top);
        release(top);
        cnt_[C_ENC] += B;
        return out;
    }

    // decryption to real coefficients (message * delta_level)
    // decryption works on the raw tensor: a deferred third polynomial is decrypted with s^2
    // and owed rescales are folded into the returned scale raw_scale(level, pend); the CRT
    // uses the fewest limbs (2..4) whose product exceeds that scale by 2^26
    double decrypt_coeffs(const Ct& c_in, std::vector<double>& m) {
        const int n = hp_.n;
        Ct c = ensure_ntt(c_in);
        const int nl = hp_.nl(c.level);
        const double need = c.level >= 0 ? std::log2(raw_scale(c.level, c.pend)) + 26.0 : 0.0;
        int kd = std::min(2, nl);
        double have = 0.0;
        for (int i = 0; i < kd; ++i) have += std::log2((double)hp_.mod[i]);
        while (have < need && kd < std::min(4, nl)) have += std::log2((double)hp_.mod[kd++]);
        if (have < need && c.pend > 0) {  // too large for 128-bit CRT: apply the owed work first
            Ct nc = normalize(c, true);
            if (c.data != c_in.data) release(c);
            std::vector<double> mm;
            const double sc = decrypt_coeffs(nc, mm);
            if (nc.data != c_in.data) release(nc);
            m.swap(mm);
            return sc;
        }
        const double scale = c.level >= 0 ? raw_scale(c.level, c.pend) : (bs_.ready ? bs_.s_bt : 1.0);
        u32* x = tmp(kd);
        launch_copy_rows(S(), T_, x, c.data, kd);
        u32* spow = nullptr;
        for (int p = 1; p < c.npoly; ++p) {
            const u32* s_use = d_s_;
            if (p == 2) {
                spow = tmp(kd);
                launch_square(S(), T_, spow, d_s_, kd, kd, qmap());
                s_use = spow;
            }
            launch_fma_poly(S(), T_, x, x, c.data + (size_t)p * nl * n, s_use, kd, kd, qmap());
        }
        intt(x, kd, kd, qmap());
        std::vector<u32> h((size_t)kd * n);
        HIP_OK(hipMemcpyAsync(h.data(), x, sizeof(u32) * kd * n, hipMemcpyDeviceToHost, S()));
        HIP_OK(hipStreamSynchronize(S()));
        untmp(x, kd);
        if (spow) untmp(spow, kd);
        if (c.data != c_in.data) release(c);
        // Garner mixed-radix CRT in 128-bit integers, centred
        typedef unsigned __int128 u128;
        std::vector<u64> minv(kd, 0);
        u128 Qall = 1;
        for (int i = 0; i < kd; ++i) {
            if (i) minv[i] = hinvm((u32)(Qall % hp_.mod[i]), hp_.mod[i]);
            Qall *= hp_.mod[i];
        }
        m.resize(n);
        for (int k = 0; k < n; ++k) {
            u128 v = h[k], M = hp_.mod[0];
            for (int i = 1; i < kd; ++i) {
                const u64 qi = hp_.mod[i];
                const u64 vi = (u64)(v % qi);
                const u64 t = ((h[(size_t)i * n + k] + qi - vi) % qi) * minv[i] % qi;
                v += (u128)t * M;
                M *= qi;
            }
            m[k] = v > Qall / 2 ? -(double)(Qall - v) : (double)v;
        }
        cnt_[C_DEC]++;
        return scale;
    }
    void decrypt(aesfhe_handle h, double* re, double* im) {
        if (ct(h).nb != 1) throw std::runtime_error("decrypt: a stacked ciphertext (unstack it first)");
        std::vector<double> m;
        const double inv = 1.0 / decrypt_coeffs(ct(h), m);
        for (double& v : m) v *= inv;
        emb_.forward(m.data(), re, im);
    }

    // ------------------------------------------------------------------ basic ops
    void release(const Ct& c) { pool().put(c.data, c.words); }
    static void copy_meta(Ct& o, const Ct& c) {
        o.ntt = c.ntt, o.pend = c.pend, o.lazy = c.lazy, o.zero = c.zero, o.nb = c.nb;
    }
    Ct copy(const Ct& c) {
        Ct o = alloc_ct(c.level, c.npoly);
        copy_meta(o, c);
        launch_copy_rows(S(), T_, o.data, c.data, c.words / hp_.n);
        return o;
    }
    // returns c itself (same data) when already in NTT form, else a converted copy
    Ct ensure_ntt(const Ct& c) {
        if (c.ntt) return c;
        Ct o = alloc_ct(c.level, c.npoly);
        copy_meta(o, c);
        const int nl = hp_.nl(o.level);
        ntt(o.data, c.data, o.npoly * nl, rows_dense(nl), qmap());
        o.ntt = true;
        return o;
    }
    Ct to_intt(const Ct& c) {
        if (!c.ntt) return copy(c);
        Ct o = alloc_ct(c.level, c.npoly);
        copy_meta(o, c);
        const int nl = hp_.nl(o.level);
        intt(o.data, c.data, o.npoly * nl, rows_dense(nl), qmap());
        o.ntt = false;
        return o;
    }
    Ct to_ntt(const Ct& c) {
        if (c.ntt) return copy(c);
        Ct o = alloc_ct(c.level, c.npoly);
        copy_meta(o, c);
        const int nl = hp_.nl(o.level);
        ntt(o.data, c.data, o.npoly * nl, rows_dense(nl), qmap());
        o.ntt = true;
        return o;
    }

    // ------------------------------------------------------------------ deferred work
    // product of the primes a rescale at level l drops
    double qdrop(int l) const {
        double d = 1.0;
        for (int i = hp_.nl(l - 1); i < hp_.nl(l); ++i) d *= (double)hp_.mod[i];
        return d;
    }
    // raw scale of a tensor at data level l owing p rescales: delta_{l-p} * Q_drop(l) ... Q_drop(l-p+1)
    double raw_scale(int l, int p) const {
        double sc = hp_.delta[l - p];
        for (int j = 0; j < p; ++j) sc *= qdrop(l - j);
        return sc;
    }
    double log2q(int l) const {
        double b = 0.0;
        for (int i = 0; i < hp_.nl(l); ++i) b += std::log2((double)hp_.mod[i]);
        return b;
    }
    // a message of magnitude <= 2^kMsgBits times `mag` fits below Q_l / 2 at raw scale (l, p)
    static constexpr double kMsgBits = 20.0;
    bool headroom(int l, int p, double mag) const {
        if (l - p < 0) return false;
        return std::log2(raw_scale(l, p)) + std::log2(std::max(1.0, mag)) + kMsgBits < log2q(l) - 1.0;
    }
    static int vis_npoly(const Ct& c) { return c.lazy ? 2 : c.npoly / c.nb; }
    static int pm(const Ct& c) { return c.npoly / c.nb; }  // polynomials per batched ciphertext

    // key switch of the third polynomial at the data level; keeps pend
    Ct relin_raw(const Ct& c) {
        const int nl = hp_.nl(c.level), n = hp_.n;
        const size_t ms = (size_t)3 * nl * n;  // member stride of a batched tensor
        Ct r = keyswitch(c.data + (size_t)2 * nl * n, c.level, ksk(0), c.data, c.data + (size_t)nl * n, c.nb, ms, ms);
        r.pend = c.pend;
        r.lazy = c.lazy && c.pend > 0;
        cnt_[C_RELIN]++;
        return r;
    }
    // canonical form: every owed rescale applied and (need2) relinearised; c itself when
    // nothing is owed.  The caller releases the result when its data differs from c's.
    // A 3-polynomial tensor is only rescaled while its scale stays >= 2^50 (pend 2 -> 1):
    // below that the rounding term r2 s^2 / q (|s^2| ~ 2^14 per coefficient for a dense
    // ternary s) would show in the message, so it is relinearised first.
    Ct normalize(const Ct& c_in, bool need2 = true) {
        Ct cur = ensure_ntt(c_in);
        bool own = cur.data != c_in.data;
        while (pm(cur) == 3 && cur.pend >= 2) {
            Ct r = rescale(cur);
            if (own) release(cur);
            cur = r, own = true;
        }
        if (pm(cur) == 3 && (need2 || cur.pend > 0)) {
            Ct r = fused_relin_rescale_ok(cur) ? relin_rescale(cur) : relin_raw(cur);
            if (own) release(cur);
            cur = r, own = true;
        }
        while (cur.pend > 0) {
            Ct r = rescale(cur);
            if (own) release(cur);
            cur = r, own = true;
        }
        cur.lazy = false;
        return cur;
    }
    // stored ciphertext in canonical form; the table entry is replaced so that deferred work
    // is done once however often the handle is used
    // Inside a fork/join section another stream may read the same handle, so the table entry
    // is left alone and a private canonical copy (released when the API call ends) is used --
    // unless the calling branch itself stored the handle in this section.
    const Ct& canon(aesfhe_handle h) {
        auto it = cts_.find(h);
        if (it == cts_.end()) throw std::runtime_error("invalid ciphertext handle");
        Ct& c = it->second;
        if (!c.lazy) return c;
        Ct nc = normalize(c, true);
        if (nc.data == c.data) {  // nothing was owed: only the flag changes
            c.lazy = false;
            return c;
        }
        // a handle this branch stored in this fork section is invisible to the other branches
        // until the join, so it is memoized like outside a section
        if (fj_active_ && !(c.sid == t_sidx && c.epoch == fj_epoch_)) {
            scratch_.push_back(nc);
            return scratch_.back();
        }
        if (nc.data != c.data) release(c);
        nc.sid = c.sid, nc.epoch = c.epoch;
        c = nc;
        return c;
    }
    std::deque<Ct> scratch_;
    void end_call() {
        for (const Ct& c : scratch_) release(c);
        scratch_.clear();
    }
    Ct zero_ct(int level, int nb = 1) {
        Ct z = alloc_ct(level, 2 * nb, nb);
        HIP_OK(hipMemsetAsync(z.data, 0, z.words * sizeof(u32), S()));
        z.zero = true;
        return z;
    }

    // drop the last k limbs of an npoly x nl tensor, dividing by each dropped prime with
    // rounding; returns a pool buffer of npoly x (nl - k) rows
    // x: np polys of nl limbs each (poly stride `stride` limbs, default nl) -> the first nl - k limbs,
    // divided by the k dropped primes.  cc (nullable, [nl] Shoup pairs): x is first multiplied by a
    // constant (Engine::convert's exact-scale factor) -- folded into the dropped limbs' INTT (post)
    // and the finish's cur read (cmul), no separate multiply launch and no multiplied copy
    u32* drop_limbs(const u32* x, int np, int nl, int k, int stride = 0, const u32* cc = nullptr) {
        const int n = hp_.n;
        if (stride <= 0) stride = nl;
        if (k == 2 && nl >= 3) {
            // both primes at once: INTT of the two dropped rows per poly, then one fused
            // CRT-spread -> NTT -> (cur - v) (q_a q_b)^{-1} pass over the r = nl - 2 kept limbs
            const int r = nl - 2;
            const u32 qa = hp_.mod[r], qb = hp_.mod[r + 1];
            const u32 ainv = hinvm(qa % qb, qb);
            u32* last = tmp(2 * (size_t)np);
            intt(last, x, 2 * np, RowMap{2, stride, 2, r, 0}, LimbMap{2, r, 0}, cc ? cc + 2 * (size_t)r : nullptr);
            u32* v = tmp((size_t)np * r);
            u32* o = tmp((size_t)np * r);
            launch_rescale2_ntt(S(), T_, o, x, last, v, d_rescale2_qinv_ + rescale2_off_[r], np, r, stride, qa, qb, ainv,
                                shoup_pre(ainv, qb), cc);
            cnt_[C_NTT_ROWS] += (size_t)np * r;
            untmp(last, 2 * (size_t)np);
            untmp(v, (size_t)np * r);
            return o;
        }
        const u32* cur = x;
        u32* owned = nullptr;
        for (int step = 0; step < k; ++step) {
            const int r = nl - 1 - step;  // limb dropped now; cur has r + 1 limbs per poly
            const int cs = step ? r + 1 : stride;
            const u32* c0 = step ? nullptr : cc;  // the constant rides on the first drop only
            // coefficients of the dropped limb (one row per poly, read in place), then the
            // fused spread -> NTT -> (cur - v) q_r^{-1} on the r remaining limbs
            u32* last = tmp(np);
            intt(last, cur, np, RowMap{1, cs, 1, r, 0}, single(r), c0 ? c0 + 2 * (size_t)r : nullptr);
            u32* v = tmp((size_t)np * r);
            u32* o = tmp((size_t)np * r);
            launch_rescale_ntt(S(), T_, o, cur, last, v, d_rescale_qinv_ + rescale_off_[r], np, r, cs, hp_.mod[r], c0);
            cnt_[C_NTT_ROWS] += (size_t)np * r;
            untmp(last, np);
            untmp(v, (size_t)np * r);
            if (owned) untmp(owned, (size_t)np * (r + 1));
            owned = o;
            cur = o;
        }
        return owned;
    }

    // rescale: level l -> l-1, dropping nl(l) - nl(l-1) limbs (1 or 2)
    Ct rescale(const Ct& c, bool into_base = false) {
        if (c.level < (into_base ? 0 : 1)) throw std::runtime_error("cannot rescale: ciphertext is at level 0 (not enough level)");
        const int nl = hp_.nl(c.level), nlo = hp_.nl(c.level - 1);
        Ct o;
        o.level = c.level - 1;
        o.npoly = c.npoly;
        o.nb = c.nb;
        o.words = (size_t)c.npoly * nlo * hp_.n;
        o.data = drop_limbs(c.data, c.npoly, nl, nl - nlo);
        o.pend = c.pend > 0 ? c.pend - 1 : 0;
        o.lazy = c.lazy && (o.pend > 0 || pm(o) == 3);
        o.zero = c.zero;
        cnt_[C_RESCALE]++;
        return o;
    }

    // per-limb constant residues (Shoup pairs, lo/hi halves) on limbs 0..nl-1
    LimbConsts const_half(const std::vector<u32>& lo, const std::vector<u32>& hi) {
        const int nl = (int)lo.size();
        if (nl > kMaxConstLimbs) throw std::runtime_error("const_half: too many limbs");
        LimbConsts h{};
        for (int t = 0; t < nl; ++t) {
            const u32 q = hp_.mod[t];
            h.v[4 * t] = lo[t];
            h.v[4 * t + 1] = shoup_pre(lo[t], q);
            h.v[4 * t + 2] = hi[t];
            h.v[4 * t + 3] = shoup_pre(hi[t], q);
        }
        return h;
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

    // exact-scale change of representation: re-express a tensor at
    // (data level t, owing p rescales), logical level t - p <= the input's.  Owed rescales
    // are applied first down to the target data level; the rest is one exact-scale step:
    // keep nl(t) + k limbs, multiply by c = round(S(t,p) q_{nl(t)} ... q_{nl(t)+k-1} / S(l,q))
    // and divide the k limbs away, k the smallest count keeping c >= 2^24 (2^51 on the
    // double-prime levels).  Always returns a
    // new buffer.
    Ct convert(const Ct& c_in, int t, int p) {
        if (p < 0 || t > c_in.level || t - p > c_in.level - c_in.pend)
            throw std::runtime_error("level_down: target level above ciphertext level");
        Ct c = ensure_ntt(c_in);
        bool own = c.data != c_in.data;
        if (c.level == t && c.pend == p) return own ? c : copy(c);
        const int n = hp_.n, nb = hp_.nl(t), na = hp_.nl(c.level);
        int k = 0;
        double ratio = raw_scale(t, p) / raw_scale(c.level, c.pend);
        // the constant's rounding is a relative scale error of up to 0.5 / c: 2^-25 is far below
        // the noise at the single-prime scale (~2^30), but on the double-prime levels (scale
        // ~2^60: CoeffToSlot, EvalMod) it would dominate -- EvalMod's T_k recurrences align
        // operands across levels and its double angles amplify the error 4^r-fold -- so there c
        // keeps ~51 bits (one more limb kept and divided away)
        const double need = t > hp_.L1 ? 2251799813685248.0 : 16777216.0;  // 2^51 : 2^24
        while (ratio < need && nb + k < na) ratio *= (double)hp_.mod[nb + k], ++k;
        if (!(ratio >= 0.999999 && ratio < 9.0e18)) throw std::runtime_error("level_down: scale ratio out of range");
        if (pm(c) == 3 && k > 0 && raw_scale(t, p) < 1.0e15) {  // see normalize()
            Ct r = relin_raw(c);
            if (own) release(c);
            Ct o = convert(r, t, p);
            release(r);
            return o;
        }
        const int nk = nb + k;
        const i64 cst = std::llround(ratio);
        if (k > 0 && fused_convert_) {  // the constant folded into the drop (drop_limbs cc): one launch and one copy fewer
            Ct o;
            o.level = t, o.npoly = c.npoly, o.nb = c.nb, o.pend = p, o.lazy = c.lazy || p > 0, o.zero = c.zero;
            o.words = (size_t)c.npoly * nb * n;
            o.data = drop_limbs(c.data, c.npoly, nk, k, na, conv_consts(cst, nk));
            if (own) release(c);
            return o;
        }
        u32* mid = tmp((size_t)c.npoly * nk);
        std::vector<u32> r(nk);
        for (int i = 0; i < nk; ++i) r[i] = mod_i64(cst, hp_.mod[i]);
        // the first nk limbs of every poly, times the constant (copy fused into the multiply)
        launch_mul_const_half(S(), T_, mid, c.data, const_half(r, r), c.npoly * nk, nk, qmap(), na);
        Ct o;
        o.level = t, o.npoly = c.npoly, o.nb = c.nb, o.pend = p, o.lazy = c.lazy || p > 0, o.zero = c.zero;
        o.words = (size_t)c.npoly * nb * n;
        if (k == 0) {
            o.data = mid;
        } else {
            o.data = drop_limbs(mid, c.npoly, nk, k);
            untmp(mid, (size_t)c.npoly * nk);
        }
        if (own) release(c);
        return o;
    }
    // AESFHE_FUSED_CONVERT=0: the conversion's constant as its own launch (A/B, bit-identity test)
    bool fused_convert_ = !(std::getenv("AESFHE_FUSED_CONVERT") && std::atoi(std::getenv("AESFHE_FUSED_CONVERT")) == 0);
    // [nk] Shoup pairs of cst mod q_i on the device, cached per (constant, limb count): the same
    // conversions recur every round
    std::map<std::pair<i64, int>, u32*> conv_cst_;
    const u32* conv_consts(i64 cst, int nk) {
        auto it = conv_cst_.find({cst, nk});
        if (it != conv_cst_.end()) return it->second;
        std::vector<u32> h(2 * (size_t)nk);
        for (int i = 0; i < nk; ++i) {
            const u32 v = mod_i64(cst, hp_.mod[i]);
            h[2 * i] = v, h[2 * i + 1] = shoup_pre(v, hp_.mod[i]);
        }
        u32* d = dev_alloc(h.size());
        HIP_OK(hipMemcpyAsync(d, h.data(), h.size() * sizeof(u32), hipMemcpyHostToDevice, S()));
        HIP_OK(hipStreamSynchronize(S()));
        return conv_cst_[{cst, nk}] = d;
    }
    // logical level drop of a canonical (pend 0) tensor
    Ct level_down(const Ct& c_in, int level) {
        if (c_in.pend > 0) {
            Ct nc = normalize(c_in, false);
            Ct o = level_down(nc, level);
            if (nc.data != c_in.data) release(nc);
            return o;
        }
        if (level > c_in.level) throw std::runtime_error("level_down: target level above ciphertext level");
        return convert(c_in, level, 0);
    }
    // two canonical ciphertexts at a common level (copies only when a level change is needed)
    std::pair<Ct, Ct> align(const Ct& a, const Ct& b, bool& fa, bool& fb, bool for_mul = false) {
        int lv = std::min(a.level - a.pend, b.level - b.pend);
        if (for_mul && !hp_.homogeneous(lv)) --lv;  // never square across the region boundary
        Ct x = ensure_ntt(a), y = ensure_ntt(b);
        fa = x.data != a.data;
        fb = y.data != b.data;
        if (x.level != lv || x.pend) {
            Ct t = level_down(x, lv);
            if (fa) release(x);
            x = t, fa = true;
        }
        if (y.level != lv || y.pend) {
            Ct t = level_down(y, lv);
            if (fb) release(y);
            y = t, fb = true;
        }
        return {x, y};
    }

    // a + b / a - b.  Operands owing the same work at the same data level combine directly;
    // otherwise both are re-expressed at data level t = min(l_a, l_b, m + 2) owing t - m
    // rescales (m = the lower logical level), falling back to canonical form when the raw
    // scale would not fit
    Ct add_sub(const Ct& a, const Ct& b, bool sub) {
        cnt_[C_ADD]++;
        if (a.nb != b.nb) throw std::runtime_error("add_sub: batched operands of different sizes");
        if (sub && a.data == b.data) return zero_ct(a.level - a.pend, a.nb);
        if (b.zero) return copy(a);
        if (a.zero && !sub) return copy(b);
        Ct x = ensure_ntt(a), y = ensure_ntt(b);
        bool fa = x.data != a.data, fb = y.data != b.data;
        if (x.level != y.level || x.pend != y.pend) {
            const int m = std::min(x.level - x.pend, y.level - y.pend);
            int t = std::min(std::min(x.level, y.level), m + 2), p = t - m;
            if (p > 0 && !headroom(t, p, 1.0)) t = m, p = 0;
            if (x.level != t || x.pend != p) {
                Ct c = convert(x, t, p);
                if (fa) release(x);
                x = c, fa = true;
            }
            if (y.level != t || y.pend != p) {
                Ct c = convert(y, t, p);
                if (fb) release(y);
                y = c, fb = true;
            }
        }
        const int nl = hp_.nl(x.level);
        const int np = std::max(x.npoly, y.npoly);
        Ct o = alloc_ct(x.level, np, x.nb);
        o.pend = x.pend;
        o.lazy = x.lazy || y.lazy;
        if (x.nb > 1 && x.npoly != y.npoly) {  // stacks of a deferred tensor and a ciphertext: per member
            const int px = pm(x), py = pm(y), po = pm(o);
            const size_t rw = (size_t)nl * hp_.n;
            for (int m = 0; m < x.nb; ++m)
                launch_addsub_tail(S(), T_, o.data + m * po * rw, x.data + m * px * rw, y.data + m * py * rw, std::min(px, py) * nl, po * nl,
                                   px > py, sub, nl, qmap());
            if (fa) release(x);
            if (fb) release(y);
            return o;
        }
        const int common = std::min(x.npoly, y.npoly) * nl;
        if (x.zero && x.npoly == y.npoly) {
            launch_neg(S(), T_, o.data, y.data, common, nl, qmap());
        } else if (x.npoly == y.npoly) {
            if (sub) launch_sub(S(), T_, o.data, x.data, y.data, common, nl, qmap());
            else launch_add(S(), T_, o.data, x.data, y.data, common, nl, qmap());
        } else {  // the third polynomial of a deferred tensor comes along in the same launch
            launch_addsub_tail(S(), T_, o.data, x.data, y.data, common, np * nl, x.npoly > y.npoly, sub, nl, qmap());
        }
        if (fa) release(x);
        if (fb) release(y);
        return o;
    }

    // + constant at the tensor's raw scale: round(c delta_m) times the primes the owed
    // rescales will divide out (m = logical level), so nothing has to be applied first
    LimbConsts add_consts(int level, int pend, double re, double im) {
        const int nl = hp_.nl(level), m = level - pend;
        std::vector<u32> lo, hi;
        scalar_residues(std::llround(re * hp_.delta[m]), std::llround(im * hp_.delta[m]), nl, lo, hi);
        if (pend > 0)
            for (int t = 0; t < nl; ++t) {
                u64 f = 1;
                for (int i = hp_.nl(m); i < nl; ++i) f = f * (hp_.mod[i] % hp_.mod[t]) % hp_.mod[t];
                lo[t] = (u32)((u64)lo[t] * f % hp_.mod[t]);
                hi[t] = (u32)((u64)hi[t] * f % hp_.mod[t]);
            }
        if (nl > 2 * kMaxConstLimbs) throw std::runtime_error("add_scalar: too many limbs");
        LimbConsts d{};
        for (int t = 0; t < nl; ++t) d.v[2 * t] = lo[t], d.v[2 * t + 1] = hi[t];
        return d;
    }
    Ct add_scalar(const Ct& c_in, double re, double im) { return lincomb(c_in, 1, nullptr, 0, re, im); }
    // k a + s b + c in ONE launch (k a Gaussian integer, s = +1 / -1 / 0 for no b, c a complex
    // constant): b is first re-expressed at a's (data level, owed rescales) when they differ (a's
    // logical level not above b's), else the general add_sub path.  EvalMod's recurrences
    // 2 T_a T_b - T_(a-b) and 2 T^2 - 1, and add_scalar (k = 1, no b)
    Ct lincomb(const Ct& a_in, i64 k, const Ct* b_in, int s, double cre, double cim) {
        Ct a = ensure_ntt(a_in);
        const bool own_a = a.data != a_in.data;
        Ct b;
        bool own_b = false;
        if (b_in && s) {
            b = ensure_ntt(*b_in);
            own_b = b.data != b_in->data;
            const bool same = b.level == a.level && b.pend == a.pend && b.npoly == a.npoly && b.nb == a.nb && !b.zero;
            if (!same) {
                const bool can = b.nb == a.nb && pm(b) == pm(a) && !b.zero && a.level <= b.level && a.level - a.pend <= b.level - b.pend;
                if (!can) {  // the general path
                    if (own_b) release(b);
                    Ct ka = k == 1 ? copy(a) : mul_scalar(a, (double)k, 0.0);
                    if (own_a) release(a);
                    Ct t = add_sub(ka, *b_in, s < 0);
                    release(ka);
                    if (cre == 0.0 && cim == 0.0) return t;
                    Ct o = lincomb(t, 1, nullptr, 0, cre, cim);
                    release(t);
                    return o;
                }
                Ct cb = convert(b, a.level, a.pend);
                if (own_b) release(b);
                b = cb, own_b = true;
            }
        }
        const int nl = hp_.nl(a.level);
        std::vector<u32> lo, hi;
        scalar_residues(k, 0, nl, lo, hi);
        const bool has_c = cre != 0.0 || cim != 0.0;
        LimbConsts cadd{};
        if (has_c) cadd = add_consts(a.level, a.pend, cre, cim);
        Ct o = alloc_ct(a.level, a.npoly, a.nb);
        copy_meta(o, a);
        o.zero = a.zero && !(b_in && s) && !has_c && k != 0;
        o.lazy = a.lazy || (b_in && s && b.lazy);
        launch_lincomb(S(), T_, o.data, a.data, const_half(lo, hi), (b_in && s) ? b.data : nullptr, s, has_c ? &cadd : nullptr, pm(a),
                       a.npoly * nl, nl, qmap());
        if (own_a) release(a);
        if (own_b) release(b);
        if (b_in && s) cnt_[C_ADD]++;
        return o;
    }

    // applies owed rescales until at most one is left (before one more deferred product)
    Ct upto_one_pend(const Ct& c_in, bool& own) {
        Ct c = ensure_ntt(c_in);
        own = c.data != c_in.data;
        while (c.pend >= 2) {
            Ct r = rescale(c);
            if (own) release(c);
            c = r, own = true;
        }
        return c;
    }

    // ct x scalar.  Gaussian integers multiply exactly (no level).  Otherwise the product
    // consumes one level: eagerly (x round(c ptscale_l), rescale) or, when allow_lazy and the
    // raw scale fits, deferred (x round(c S(l,p+1)/S(l,p)), one more owed rescale)
    Ct mul_scalar(const Ct& c_in, double re, double im, bool allow_lazy = false) {
        cnt_[C_SCALAR]++;
        const bool gauss = re == std::floor(re) && im == std::floor(im) && std::fabs(re) < 1048576.0 && std::fabs(im) < 1048576.0;
        if (!gauss && c_in.level - c_in.pend < 1) throw std::runtime_error("not enough level to multiply by a scalar (level 0)");
        if (c_in.zero) return gauss ? copy(c_in) : zero_ct(c_in.level - c_in.pend - 1, c_in.nb);
        if (gauss) {
            Ct c = ensure_ntt(c_in);
            const int nl = hp_.nl(c.level);
            std::vector<u32> lo, hi;
            scalar_residues((i64)re, (i64)im, nl, lo, hi);
            Ct o = alloc_ct(c.level, c.npoly);
            copy_meta(o, c);
            o.zero = re == 0.0 && im == 0.0;
            launch_mul_const_half(S(), T_, o.data, c.data, const_half(lo, hi), c.npoly * nl, nl, qmap());
            if (c.data != c_in.data) release(c);
            return o;
        }
        bool own;
        Ct c = upto_one_pend(c_in, own);
        const double mag = std::hypot(re, im);
        Ct o;
        if (allow_lazy && headroom(c.level, c.pend + 1, mag)) {
            const int nl = hp_.nl(c.level);
            const double f = raw_scale(c.level, c.pend + 1) / raw_scale(c.level, c.pend);
            std::vector<u32> lo, hi;
            scalar_residues(std::llround(re * f), std::llround(im * f), nl, lo, hi);
            o = alloc_ct(c.level, c.npoly, c.nb);
            o.pend = c.pend + 1;
            o.lazy = true;
            launch_mul_const_half(S(), T_, o.data, c.data, const_half(lo, hi), c.npoly * nl, nl, qmap());
        } else {
            Ct nc = normalize(c, false);
            const int nl = hp_.nl(nc.level);
            std::vector<u32> lo, hi;
            const double sc = hp_.ptscale[nc.level];
            scalar_residues(std::llround(re * sc), std::llround(im * sc), nl, lo, hi);
            Ct t = alloc_ct(nc.level, nc.npoly, nc.nb);
            launch_mul_const_half(S(), T_, t.data, nc.data, const_half(lo, hi), nc.npoly * nl, nl, qmap());
            o = rescale(t);
            o.lazy = c_in.lazy && pm(o) == 3;
            release(t);
            if (nc.data != c.data) release(nc);
        }
        if (own) release(c);
        return o;
    }

    // plaintext encoded on nl(level) limbs, NTT form, cached on the plaintext.  kind 0:
    // additive (delta_level); 1: multiplicative, ptscale[level] (the product rescales onto
    // delta_{level-1}); 2: multiplicative on a tensor owing one rescale, ptscale[level-1]
    u32* pt_at(Pt& p, int level, int kind) {
        const int key = 4 * level + kind;
        auto it = p.enc.find(key);
        if (it != p.enc.end()) return it->second.first;
        std::vector<u32> host;
        const int nl = hp_.nl(level);
        const double sc = kind == 0 ? hp_.delta[level] : kind == 1 ? hp_.ptscale[level] : hp_.ptscale[level - 1];
        encode_host(p.re.data(), p.im.data(), sc, nl, host);
        u32* d = upload_ntt(host, nl);
        HIP_OK(hipStreamSynchronize(S()));  // cached for every stream
        p.enc[key] = {d, (size_t)nl * hp_.n};
        return d;
    }

    Ct mul_pt(const Ct& c_in, aesfhe_handle hp, bool allow_lazy = false) {
        Pt& p = pt(hp);
        if (p.constant) return mul_scalar(c_in, p.re[0], p.im[0], allow_lazy);
        if (c_in.level - c_in.pend < 1) throw std::runtime_error("not enough level to multiply by a plaintext (level 0)");
        cnt_[C_PTMUL]++;
        if (c_in.zero) return zero_ct(c_in.level - c_in.pend - 1, c_in.nb);
        bool own;
        Ct c = upto_one_pend(c_in, own);
        Ct o;
        if (allow_lazy && headroom(c.level, c.pend + 1, 1.0)) {
            const int nl = hp_.nl(c.level);
            u32* e = pt_at(p, c.level, 1 + c.pend);
            o = alloc_ct(c.level, c.npoly, c.nb);
            o.pend = c.pend + 1;
            o.lazy = true;
            launch_mul_poly(S(), T_, o.data, c.data, e, c.npoly, nl, qmap());
        } else {
            Ct nc = normalize(c, false);
            const int nl = hp_.nl(nc.level);
            u32* e = pt_at(p, nc.level, 1);
            Ct t = alloc_ct(nc.level, nc.npoly, nc.nb);
            launch_mul_poly(S(), T_, t.data, nc.data, e, nc.npoly, nl, qmap());
            o = rescale(t);
            o.lazy = c_in.lazy && pm(o) == 3;
            release(t);
            if (nc.data != c.data) release(nc);
        }
        if (own) release(c);
        return o;
    }

    // sum_i c_i (.) p_i over n <= kMaxMembers (ciphertext, plaintext) pairs (aesfhe_mul_pt_sum): the
    // operands at their common logical level (exact drops), ONE k_mul_poly_sum launch, the rescale owed
    // as mul_pt's lazy form -- the same value as the n lazy products summed (MixColFinal.sr_entry)
    Ct mul_pt_sum(const std::vector<const Ct*>& C, const std::vector<aesfhe_handle>& P) {
        const int n = (int)C.size();
        if (n < 1 || n > kMaxMembers || (int)P.size() != n) throw std::runtime_error("mul_pt_sum: 1..8 (ciphertext, plaintext) pairs");
        int l = 1 << 30;
        const int nb = C[0]->nb;  // stacks of one size: every member times the same plaintext
        for (const Ct* c : C) {
            if (c->nb != nb || vis_npoly(*c) != 2 || c->zero) throw std::runtime_error("mul_pt_sum: nonzero 2-polynomial ciphertexts of one stack size");
            l = std::min(l, c->level - c->pend);
        }
        if (l < 1) throw std::runtime_error("not enough level to multiply by a plaintext (level 0)");
        for (aesfhe_handle h : P)
            if (pt(h).constant) throw std::runtime_error("mul_pt_sum: constant plaintexts take mul_scalar");
        std::vector<Ct> own;
        PtSumArgs a;
        for (int i = 0; i < n; ++i) {
            // canonical (NTT, two polynomials, nothing owed), then the exact drop to l
            Ct x = (pm(*C[i]) != 2 || C[i]->pend || !C[i]->ntt) ? normalize(*C[i], true) : *C[i];
            if (x.level != l) {
                Ct t = level_down(x, l);
                if (x.data != C[i]->data) release(x);
                x = t;
            }
            if (x.data != C[i]->data) own.push_back(x);
            a.in[i] = x.data;
            a.pt[i] = pt_at(pt(P[i]), l, 1);
            cnt_[C_PTMUL]++;
        }
        Ct o = alloc_ct(l, 2 * nb, nb);
        launch_mul_poly_sum(S(), T_, o.data, a, n, 2 * nb, hp_.nl(l), qmap());
        for (const Ct& x : own) release(x);
        o.pend = 1;
        o.lazy = true;
        if (!headroom(l, 1, 1.0)) {
            Ct r = rescale(o);
            release(o);
            return r;
        }
        return o;
    }

    Ct add_pt(const Ct& c_in, aesfhe_handle hp) {
        Pt& p = pt(hp);
        if (p.constant) return add_scalar(c_in, p.re[0], p.im[0]);
        Ct c = normalize(c_in, false);
        const int nl = hp_.nl(c.level);
        u32* e = pt_at(p, c.level, 0);
        Ct o = copy(c);
        o.zero = false;
        o.lazy = c_in.lazy && pm(o) == 3;
        for (int m = 0; m < c.nb; ++m) {  // c0 of every stacked member
            const size_t off = (size_t)m * pm(c) * nl * hp_.n;
            launch_add(S(), T_, o.data + off, c.data + off, e, nl, nl, qmap());
        }
        if (c.data != c_in.data) release(c);
        return o;
    }

    // ------------------------------------------------------------------ fused LUT evaluation
    aesfhe_handle lut_create(int n_a, int n_b, const double* re, const double* im, double c0_re, double c0_im) {
        if (n_a < 1 || n_b < 1 || (n_b > 1 && (n_a > kLutMax || n_b > kLutMax)))
            throw std::runtime_error("lut_create: bad shape (bivariate LUTs are at most 16 x 16)");
        Lut L;
        L.n_a = n_a, L.n_b = n_b;
        L.re.assign(re, re + (size_t)n_a * n_b);
        L.im.assign(im, im + (size_t)n_a * n_b);
        L.c0_re = c0_re, L.c0_im = c0_im;
        const aesfhe_handle h = next_++;
        luts_.emplace(h, std::move(L));
        return h;
    }
    Lut& lut(aesfhe_handle h) {
        auto it = luts_.find(h);
        if (it == luts_.end()) throw std::runtime_error("invalid LUT handle");
        return it->second;
    }
    // Shoup pairs of the integer constants round(c_j f_j), per term j, limb t < nl, slot half
    const u32* lut_consts(Lut& L, const std::string& key, const std::vector<std::pair<int, double>>& terms, int nl) {
        auto it = L.cst.find(key);
        if (it != L.cst.end()) return it->second.first;
        std::vector<u32> h(terms.size() * (size_t)nl * 4);
        std::vector<u32> lo, hi;
        for (size_t j = 0; j < terms.size(); ++j) {
            const int c = terms[j].first;
            const double f = terms[j].second;
            const double a = L.re[c] * f, b = L.im[c] * f;
            if (std::fabs(a) > 9.0e18 || std::fabs(b) > 9.0e18) throw std::runtime_error("level: LUT constant out of range");
            scalar_residues(std::llround(a), std::llround(b), nl, lo, hi);
            for (int t = 0; t < nl; ++t) {
                u32* e = &h[(j * nl + t) * 4];
                e[0] = lo[t], e[1] = shoup_pre(lo[t], hp_.mod[t]);
                e[2] = hi[t], e[3] = shoup_pre(hi[t], hp_.mod[t]);
            }
        }
        const size_t words = (h.size() + (size_t)hp_.n - 1) / hp_.n * hp_.n;
        u32* d = alloc_words(words);
        HIP_OK(hipMemcpyAsync(d, h.data(), h.size() * sizeof(u32), hipMemcpyHostToDevice, S()));
        HIP_OK(hipStreamSynchronize(S()));  // cached for every stream; host vector dies here
        L.cst[key] = {d, words};
        return d;
    }
    // sum_{p,q} C_pq A_p B_q (n_b > 1) or sum_p C_p A_p + c0 (n_b = 1), as a deferred tensor at
    // the lowest data level l of the elements used: (l, 2 owed rescales, 3 polys) or
    // (l, 1 owed rescale, 2 polys) -- the same logical level as the per-term products
    Ct lut_eval(aesfhe_handle hl, const aesfhe_handle* A, const aesfhe_handle* B) {
        Lut& L = lut(hl);
        const bool bi = L.n_b > 1;
        if (!A || (bi && !B)) throw std::runtime_error("lut_eval: missing element handles");
        std::vector<const Ct*> ea(L.n_a, nullptr), eb(bi ? L.n_b : 0, nullptr);
        double mag = std::hypot(L.c0_re, L.c0_im);
        for (int p = 0; p < L.n_a; ++p)
            for (int q = 0; q < L.n_b; ++q) {
                const size_t c = (size_t)p * L.n_b + q;
                if (L.re[c] == 0.0 && L.im[c] == 0.0) continue;
                mag += std::hypot(L.re[c], L.im[c]);
                if (!ea[p]) ea[p] = &canon(A[p]);
                if (bi && !eb[q]) eb[q] = &canon(B[q]);
            }
        int l = 1 << 30;
        for (auto* e : ea) if (e) l = std::min(l, e->level);
        for (auto* e : eb) if (e) l = std::min(l, e->level);
        if (l == (1 << 30)) throw std::runtime_error("lut_eval: all coefficients are zero");
        int members = 0;  // stacked elements: every element a stack of the same member count
        for (auto* e : ea) if (e) members = members ? members : e->nb;
        for (auto* e : ea) if (e && (pm(*e) != 2 || e->nb != members)) throw std::runtime_error("lut_eval expects 2-polynomial ciphertexts (stacks of one size)");
        for (auto* e : eb) if (e && (pm(*e) != 2 || e->nb != members)) throw std::runtime_error("lut_eval expects 2-polynomial ciphertexts (stacks of one size)");
        const int pend = bi ? 2 : 1;
        if (l - pend < 0 || !headroom(l, pend, mag)) throw std::runtime_error("not enough level for the fused LUT (level)");
        const int nl = hp_.nl(l);
        const double S_out = raw_scale(l, pend);
        std::string key = std::to_string(l) + ":";
        for (auto* e : ea) key += (e ? std::to_string(e->level) : "-") + ",";
        for (auto* e : eb) key += (e ? std::to_string(e->level) : "-") + ",";
        Ct o;
        if (bi) {
            LutOperands op{};
            std::vector<std::pair<int, double>> terms;
            int j = 0;
            for (int p = 0; p < L.n_a; ++p) {
                op.p_start[p] = j;
                for (int q = 0; q < L.n_b; ++q) {
                    const size_t c = (size_t)p * L.n_b + q;
                    if (L.re[c] == 0.0 && L.im[c] == 0.0) continue;
                    op.q_of[j++] = q;
                    terms.push_back({(int)c, S_out / (hp_.delta[ea[p]->level] * hp_.delta[eb[q]->level])});
                }
                op.a[p] = ea[p] ? ea[p]->data : nullptr;
                op.na[p] = ea[p] ? hp_.nl(ea[p]->level) : 0;
            }
            for (int p = L.n_a; p <= kLutMax; ++p) op.p_start[p] = j;
            for (int q = 0; q < L.n_b; ++q) op.b[q] = eb[q] ? eb[q]->data : nullptr, op.nb[q] = eb[q] ? hp_.nl(eb[q]->level) : 0;
            const u32* cst = lut_consts(L, key, terms, nl);
            o = alloc_ct(l, 3 * members, members);
            launch_lut_bivariate(S(), T_, o.data, op, L.n_a, cst, nl, members);
        } else {
            std::vector<std::pair<int, double>> terms;
            std::vector<int> idx;
            for (int p = 0; p < L.n_a; ++p)
                if (ea[p]) terms.push_back({p, S_out / hp_.delta[ea[p]->level]}), idx.push_back(p);
            const u32* cst = lut_consts(L, key, terms, nl);
            o = alloc_ct(l, 2 * members, members);
            for (size_t c0 = 0; c0 < idx.size(); c0 += kLutChunk) {
                LutChunk ch{};
                const int n = (int)std::min<size_t>(kLutChunk, idx.size() - c0);
                for (int j = 0; j < n; ++j) ch.x[j] = ea[idx[c0 + j]]->data, ch.nx[j] = hp_.nl(ea[idx[c0 + j]]->level);
                launch_lut_univariate(S(), T_, o.data, c0 ? o.data : nullptr, ch, n, cst + c0 * (size_t)nl * 4, 2, nl, members);
            }
        }
        o.pend = pend;
        o.lazy = true;
        cnt_[C_LUT]++;
        if (!bi && (L.c0_re != 0.0 || L.c0_im != 0.0)) {
            Ct r = add_scalar(o, L.c0_re, L.c0_im);
            release(o);
            o = r;
        }
        return o;
    }

    // ------------------------------------------------------------------ key switching
    // returns (c0', c1') with c0' + c1' s = d s' (+ add0/add1 folded in); d NTT, level l
    // ModUp: coefficient form of d, every digit converted to all other limbs of Q*P in one
    // launch, one NTT launch over all converted rows (own limbs skipped: key_inner reads
    // those straight from d).  Returns nd x ne rows (tmp; the caller untmps).
    // nb > 1: the d polynomials of nb batched ciphertexts (d + m d_ms words), one launch per
    // stage for all of them; ext = [m][nd][ne]
    // tp (tensor mode, relin_rescale_tensor): member m's source rows are the products tp->a[m] (.) tp->b[m],
    // formed inside the inverse NTT (d unused)
    // rev: the source rows read in reversed coefficient order (the conjugation's permutation, galois)
    // cols_only: the extended rows' forward NTT stops after its column pass (the row pass runs inside
    // the fused key-switch core, ki_core)
    u32* modup(const u32* d, int level, int nb = 1, size_t d_ms = 0, const TensorPtrs* tp = nullptr, bool rev = false,
               bool cols_only = false) {
        const int n = hp_.n, nl = hp_.nl(level), np = hp_.n_p, ne = nl + np, alpha = hp_.alpha;
        const int nd = (nl + alpha - 1) / alpha;
        if (alpha > kMaxConvH || np > kMaxConvH || nb * nd > kMaxConvGroups) throw std::runtime_error("keyswitch: digit too large");
        const LimbMap em = extmap(nl);
        const bool fz = fused_conv(true);
        if ((tp || rev) && fz) throw std::runtime_error("modup: the tensor / reversed form needs the separate conversion");
        u32* coef = tmp((size_t)nb * nl);
        // k_bx_cols: the INTT's row pass here, its column pass + the conversion + the ext rows'
        // forward column pass in one launch
        const bool bx = bx_ok() && alpha <= kBxMaxH;
        const u32* up_post = conv_pre_ && !bx ? d_modup_qh_ + modup_qh_off_[nl] : nullptr;
        if (bx) {
            const RowMap rm{nl, nb > 1 ? (int)(d_ms / n) : nl, nl, 0, 0};
            if (rev) launch_ntt_inv_rows(S(), T_, coef, d, nb * nl, rm, qmap(), nullptr, true);
            else if (tp) launch_ntt_inv_rows(S(), T_, coef, nullptr, nb * nl, RowMap{nl, nl, nl, 0, 0}, qmap(), tp, false);
            else launch_ntt_inv_rows(S(), T_, coef, d, nb * nl, rm, qmap());
            cnt_[C_NTT_ROWS] += nb * nl;
        } else if (rev) {
            launch_ntt_inv_rev(S(), T_, coef, d, nb * nl, RowMap{nl, nb > 1 ? (int)(d_ms / n) : nl, nl, 0, 0}, qmap(), up_post);
            cnt_[C_NTT_ROWS] += nb * nl;
        } else if (tp) {
            launch_ntt_inv_prod(S(), T_, coef, *tp, nb * nl, RowMap{nl, nl, nl, 0, 0}, qmap(), up_post);
            cnt_[C_NTT_ROWS] += nb * nl;
        } else {
            intt(coef, d, nb * nl, RowMap{nl, nb > 1 ? (int)(d_ms / n) : nl, nl, 0, 0}, qmap(), fz ? d_modup_qh_ + modup_qh_off_[nl] : up_post);
        }
        u32* ext = tmp((size_t)nb * nd * ne);
        const size_t* toff = &modup_off_[(size_t)nl * hp_.dnum];
        ConvBatch up;
        up.n = nb * nd;
        up.pre = up_post != nullptr;
        for (int m = 0; m < nb; ++m)
            for (int j = 0; j < nd; ++j) {
                const int lo = j * alpha, h = std::min(alpha, nl - lo), gi = m * nd + j;
                up.h[gi] = h, up.d0[gi] = lo, up.skip0[gi] = lo;
                up.src[gi] = coef + ((size_t)m * nl + lo) * n;
                up.dst[gi] = ext + (size_t)gi * ne * n;
                up.tab[gi] = d_modup_ + toff[j];
                up.qhinv[gi] = up.tab[gi] + (size_t)2 * h * ne;
                up.negq[gi] = up.qhinv[gi] + 2 * h;
            }
        RowMap xr = rows_dense(ne);
        xr.skip_alpha = alpha, xr.skip_nl = nl, xr.skip_groups = nd;
        if (bx) {
            launch_bx_cols(S(), T_, up, ne, em);
            if (!cols_only) launch_ntt_fwd_rows(S(), T_, ext, nb * nd * ne, xr, em);
            cnt_[C_NTT_ROWS] += nb * nd * ne;
        } else if (fz) {
            if (cols_only) throw std::runtime_error("modup: the fused conversion has no column-pass-only form");
            launch_ntt_fwd_conv(S(), T_, ext, up, nb * nd * ne, xr, em);
            cnt_[C_NTT_ROWS] += nb * nd * ne;
        } else {
            launch_base_convert(S(), T_, up, ne, em);
            if (cols_only) {
                launch_ntt_fwd_cols(S(), T_, ext, ext, nb * nd * ne, xr, em);
                cnt_[C_NTT_ROWS] += nb * nd * ne;
            } else {
                ntt(ext, ext, nb * nd * ne, xr, em);
            }
        }
        untmp(coef, (size_t)nb * nl);
        return ext;
    }
    // ------------------------------------------------------------------ fused key-switch core
    // launch_ntt_ki: the ModUp's row pass, the key inner product and the ModDown
    // INTT's row pass in ONE launch.  acc rows x < kept are written ([m][2][ne], the finish's cur);
    // rows x >= kept go to ys ([m][2][ne - kept]) transformed by the inverse row pass -- the
    // ModDown then runs only its INTT column pass on ys.  AESFHE_FUSED_KI=0: the separate launches
    // (C2 62.1-62.5 -> 64.8-64.9 rounds/s, 11,762 -> 10,670 launches per encrypt, same box:
    // profiles/r4_ab_fused_ki_wt_ct8_auto.txt).
    bool fused_ki_ = std::getenv("AESFHE_FUSED_KI") == nullptr || std::getenv("AESFHE_FUSED_KI")[0] != '0';
    // the base conversions' qhat_i^{-1} factors folded into the N^{-1} scaling of the INTT that makes
    // their sources (launch_ntt_inv's post; ConvBatch::pre): k_base_convert is VALU-bound and every
    // target chunk of a block redid those H multiplies (AESFHE_CONV_PRE=0: multiplied in the conversion)
    bool conv_pre_ = !(std::getenv("AESFHE_CONV_PRE") && std::atoi(std::getenv("AESFHE_CONV_PRE")) == 0);
    bool fused_ki_ok() const { return fused_ki_ && !fused_conv(true) && !fused_conv(false); }
    // k_bx_cols for the ModUp / ModDown middles (AESFHE_BX_COLS=1, N = 2^16; groups of at most
    // kBxMaxH sources: the kernel keeps them in VGPRs -- 242 at 12, 2 waves / SIMD; the double-prime
    // levels' ModDown + rescale (13 sources) keeps the separate launches)
    static constexpr int kBxMaxH = 12;
    bool bx_cols_ = std::getenv("AESFHE_BX_COLS") != nullptr && std::atoi(std::getenv("AESFHE_BX_COLS")) != 0;
    bool bx_ok() const { return bx_cols_ && bx_cols_on(T_) && !fused_conv(true) && !fused_conv(false); }
    struct KiSrc {
        const u32* ext;
        const u32* d;
        const u32* key;
    };
    void ki_core(u32* acc, u32* ys, int level, int kept, int nb, const KiSrc* src, int nsrc, size_t d_ms, KsFold fold) {
        const int nl = hp_.nl(level), np = hp_.n_p, ne = nl + np, n = hp_.n;
        KiArgs a;
        for (int i = 0; i < nsrc; ++i) a.ext[i] = src[i].ext, a.d[i] = src[i].d, a.key[i] = src[i].key;
        a.nsrc = nsrc;
        a.nd = (nl + hp_.alpha - 1) / hp_.alpha, a.ne = ne, a.nl = nl, a.alpha = hp_.alpha;
        a.nkey = hp_.n_ks + np, a.nks = hp_.n_ks;
        a.kept = kept, a.ys_rows = ne - kept, a.nb = nb;
        a.ext_ms = (size_t)a.nd * ne * n, a.d_ms = d_ms, a.acc_ms = (size_t)2 * ne * n, a.ys_ms = (size_t)2 * (ne - kept) * n;
        a.acc = acc, a.ys = ys, a.fold = fold;
        launch_ntt_ki(S(), T_, a, extmap(nl));  // its row passes are counted with the column passes they pair with
    }
    int ext_rows(int level) const { return (hp_.nl(level) + hp_.alpha - 1) / hp_.alpha * (hp_.nl(level) + hp_.n_p); }
    // acc (2 x ne rows, Q*P) = sum_j ext_j * key_j; g != 0 reads ext and d through X -> X^g
    // nb batched ciphertexts (ext = [m][nd][ne], d + m d_ms, acc = [m][2][ne]) share the key reads
    void key_inner(u32* acc, const u32* ext, const u32* d, const u32* key, int level, u64 g, int nb = 1, size_t d_ms = 0,
                   KsFold fold = {}, bool accum = false) {
        const int nl = hp_.nl(level), np = hp_.n_p, ne = nl + np, n = hp_.n;
        const int nd = (nl + hp_.alpha - 1) / hp_.alpha;
        launch_key_inner(S(), T_, acc, ext, d, key, nd, ne, nl, hp_.alpha, hp_.n_ks + np, hp_.n_ks, extmap(nl), g, nb,
                         (size_t)nd * ne * n, d_ms, (size_t)2 * ne * n, fold, accum);
    }
    // ModDown by P: coefficients of the P rows (read in place from acc), conversion of both
    // polys in one launch, NTT fused with (acc_Q - conv) P^{-1} (+ add)
    // nb batched ciphertexts: acc = [m][2][ne]; member m adds add0/add1 + m add_ms words
    // dst: write the result there (member stride 2 nl N; the caller owns it) instead of a new buffer
    // outm: member m's result into outm[m] (nb <= 8; the returned Ct then carries no data)
    // add_rev: add0 read in reversed coefficient order (the conjugation's c0, galois)
    // ys_in: the P rows already through the INTT's row pass (ki_core, [m][2][np]): only its column pass runs here
    Ct moddown(const u32* acc, int level, const u32* add0, const u32* add1, int nb = 1, size_t add_ms = 0, u32* dst = nullptr,
               u32* const* outm = nullptr, bool add_rev = false, u32* ys_in = nullptr) {
        const int n = hp_.n, nl = hp_.nl(level), np = hp_.n_p, ne = nl + np, npl = 2 * nb;
        if (npl > kMaxConvGroups) throw std::runtime_error("moddown: batch too large");
        const bool fz = fused_conv(false);
        u32* yp = ys_in ? ys_in : tmp((size_t)npl * np);
        const bool bx = bx_ok() && np <= kBxMaxH;
        if (bx) {  // the P rows through the INTT's row pass only (k_bx_cols runs the rest)
            if (!ys_in) launch_ntt_inv_rows(S(), T_, yp, acc, npl * np, RowMap{np, ne, np, nl, 0}, LimbMap{np, hp_.p_off(), 0});
            cnt_[C_NTT_ROWS] += (size_t)npl * np;
        } else if (ys_in) {
            if (fz) throw std::runtime_error("moddown: a fused-core input needs the separate conversion");
            launch_ntt_inv_cols(S(), T_, yp, npl * np, rows_dense(np), LimbMap{np, hp_.p_off(), 0}, conv_pre_ ? d_moddown_phinv_ : nullptr);
            cnt_[C_NTT_ROWS] += (size_t)npl * np;
        } else {
            intt(yp, acc, npl * np, RowMap{np, ne, np, nl, 0}, LimbMap{np, hp_.p_off(), 0}, fz || conv_pre_ ? d_moddown_phinv_ : nullptr);
        }
        u32* conv = tmp((size_t)npl * nl);
        const size_t doff = moddown_off_[nl];
        ConvBatch dn;
        dn.n = npl;
        dn.pre = conv_pre_ && !bx;
        for (int p = 0; p < npl; ++p) {
            dn.h[p] = np, dn.d0[p] = hp_.p_off(), dn.skip0[p] = 1 << 30;
            dn.src[p] = yp + (size_t)p * np * n;
            dn.dst[p] = conv + (size_t)p * nl * n;
            dn.tab[p] = d_moddown_ + doff;
            dn.qhinv[p] = d_moddown_phinv_;
            dn.negq[p] = d_negp_;
        }
        if (bx) launch_bx_cols(S(), T_, dn, nl, qmap());
        else if (!fz) launch_base_convert(S(), T_, dn, nl, qmap());
        Ct o;
        if (dst || outm) {
            o.level = level, o.npoly = npl, o.nb = nb, o.words = (size_t)npl * nl * n, o.data = dst;
        } else {
            o = alloc_ct(level, npl, nb);
        }
        if (fz && add_rev) throw std::runtime_error("moddown: the reversed addend needs the separate conversion");
        if (bx)
            launch_ntt_finish_rows(S(), T_, o.data, conv, acc, ne, d_pinv_, add0, add1, npl, nl, add_ms, outm, add_rev);
        else if (fz)
            launch_ntt_finish_conv(S(), T_, o.data, conv, dn, acc, ne, d_pinv_, add0, add1, npl, nl, add_ms, outm);
        else
            launch_ntt_finish(S(), T_, o.data, conv, acc, ne, d_pinv_, add0, add1, npl, nl, add_ms, outm, 0u, nullptr, add_rev);
        cnt_[C_NTT_ROWS] += (size_t)npl * nl;
        if (!ys_in) untmp(yp, (size_t)npl * np);
        untmp(conv, (size_t)npl * nl);
        return o;
    }
    // key switch of d (nl rows); nb > 1: the d polynomials of nb batched ciphertexts (d + m d_ms
    // words, add0 / add1 + m add_ms), one key read for all of them -> (c0', c1') per member
    // A stack of more members than one batched key switch carries (ks_chunk) goes through in
    // chunks, each chunk's ModDown writing its rows of the one stacked result.
    Ct keyswitch(const u32* d, int level, const u32* key, const u32* add0, const u32* add1, int nb = 1, size_t d_ms = 0,
                 size_t add_ms = 0, u32* dst = nullptr) {
        const int ne = hp_.nl(level) + hp_.n_p, ch = ks_chunk(level);
        if (nb > ch) {
            Ct o;
            if (dst) {
                o.level = level, o.npoly = 2 * nb, o.nb = nb, o.words = (size_t)2 * nb * hp_.nl(level) * hp_.n, o.data = dst;
            } else {
                o = alloc_ct(level, 2 * nb, nb);
            }
            const size_t oms = (size_t)2 * hp_.nl(level) * hp_.n;
            for (int m0 = 0; m0 < nb; m0 += ch) {
                const int c = std::min(ch, nb - m0);
                keyswitch(d + m0 * d_ms, level, key, add0 ? add0 + m0 * add_ms : nullptr, add1 ? add1 + m0 * add_ms : nullptr, c, d_ms, add_ms,
                          o.data + m0 * oms);
            }
            return o;
        }
        if (fused_ki_ok()) {
            const int np = hp_.n_p;
            u32* ext = modup(d, level, nb, d_ms, nullptr, false, true);
            u32* acc = tmp(2 * (size_t)ne * nb);
            u32* ys = tmp(2 * (size_t)np * nb);
            const KiSrc src{ext, d, key};
            ki_core(acc, ys, level, hp_.nl(level), nb, &src, 1, d_ms, KsFold{});
            untmp(ext, (size_t)nb * ext_rows(level));
            Ct o = moddown(acc, level, add0, add1, nb, add_ms, dst, nullptr, false, ys);
            untmp(ys, 2 * (size_t)np * nb);
            untmp(acc, 2 * (size_t)ne * nb);
            cnt_[C_KS] += nb;
            tally(LV_KS, level, nb);
            return o;
        }
        u32* ext = modup(d, level, nb, d_ms);
        u32* acc = tmp(2 * (size_t)ne * nb);
        key_inner(acc, ext, d, key, level, 0, nb, d_ms);
        untmp(ext, (size_t)nb * ext_rows(level));
        Ct o = moddown(acc, level, add0, add1, nb, add_ms, dst);
        untmp(acc, 2 * (size_t)ne * nb);
        cnt_[C_KS] += nb;
        tally(LV_KS, level, nb);
        return o;
    }
    // bootstrapping step 2: the single-limb (q0) ciphertexts' d = c1 switched to the sparse
    // secret with ksk_d2s (modulus q0 * P', P' = d2s_np() special primes); (c0', c1') with
    // c0' = add0 + ...; nb members at d + m ms / add0 + m ms
    // d: c1 of nb members (NTT form, the two base limbs q0, q1, member stride ms words);
    // returns the key-switched (c0', c1') over (q0, q1) with add0 (c0) added to c0'
    Ct keyswitch_d2s(const u32* d, const u32* add0, int nb, size_t ms) {
        const int n = hp_.n, nq = kD2sQ, np = d2s_np(), ne = nq + np, npl = 2 * nb;
        if (npl > kMaxConvGroups || nb > kMaxKsBatch) throw std::runtime_error("keyswitch_d2s: batch too large");
        const LimbMap em = extmap(nq);
        const u32* key = ksk(tag_d2s());
        // ModUp Q0 -> P' (the own limbs q0, q1 are read from d by the key inner product)
        const bool fz = fused_conv(true), fzd = fused_conv(false);
        u32* coef = tmp((size_t)nb * nq);
        intt(coef, d, nb * nq, RowMap{nq, (int)(ms / n), nq, 0, 0}, qmap(), fz || conv_pre_ ? d_d2s_ + d2s_off_.up_qhinv : nullptr);
        u32* ext = tmp((size_t)nb * ne);
        ConvBatch up;
        up.n = nb;
        up.pre = conv_pre_;
        for (int m = 0; m < nb; ++m) {
            up.h[m] = nq, up.d0[m] = 0, up.skip0[m] = 0;
            up.src[m] = coef + (size_t)m * nq * n;
            up.dst[m] = ext + (size_t)m * ne * n;
            up.tab[m] = d_d2s_ + d2s_off_.up_tab;      // [nq][ne] pairs: (Q0 / q_i) mod target
            up.qhinv[m] = d_d2s_ + d2s_off_.up_qhinv;  // [nq] pairs: (Q0 / q_i)^-1 mod q_i
            up.negq[m] = d_d2s_ + d2s_off_.up_negq;    // [ne]: -Q0 mod target
        }
        RowMap xr = rows_dense(ne);
        xr.skip_alpha = hp_.alpha, xr.skip_nl = nq, xr.skip_groups = 1;
        if (fz) {
            launch_ntt_fwd_conv(S(), T_, ext, up, nb * ne, xr, em);
            cnt_[C_NTT_ROWS] += nb * ne;
        } else {
            launch_base_convert(S(), T_, up, ne, em);
            ntt(ext, ext, nb * ne, xr, em);
        }
        untmp(coef, (size_t)nb * nq);
        u32* acc = tmp((size_t)npl * ne);
        launch_key_inner(S(), T_, acc, ext, d, key, 1, ne, nq, hp_.alpha, ne, nq, em, 0, nb, (size_t)ne * n, ms, (size_t)2 * ne * n);
        untmp(ext, (size_t)nb * ne);
        // ModDown by P' onto (q0, q1), + add0
        u32* yp = tmp((size_t)npl * np);
        intt(yp, acc, npl * np, RowMap{np, ne, np, nq, 0}, LimbMap{np, hp_.p_off(), 0}, fzd || conv_pre_ ? d_d2s_ + d2s_off_.dn_qhinv : nullptr);
        u32* conv = tmp((size_t)npl * nq);
        ConvBatch dn;
        dn.n = npl;
        dn.pre = conv_pre_;
        for (int p = 0; p < npl; ++p) {
            dn.h[p] = np, dn.d0[p] = hp_.p_off(), dn.skip0[p] = 1 << 30;
            dn.src[p] = yp + (size_t)p * np * n;
            dn.dst[p] = conv + (size_t)p * nq * n;
            dn.tab[p] = d_d2s_ + d2s_off_.dn_tab;      // [np][nq] pairs: (P' / p_k) mod q_t
            dn.qhinv[p] = d_d2s_ + d2s_off_.dn_qhinv;  // [np] pairs: (P' / p_k)^-1 mod p_k
            dn.negq[p] = d_d2s_ + d2s_off_.dn_negq;    // [nq]: -P' mod q_t
        }
        if (!fzd) launch_base_convert(S(), T_, dn, nq, qmap());
        Ct o = alloc_ct(0, npl, nb);
        if (fzd)
            launch_ntt_finish_conv(S(), T_, o.data, conv, dn, acc, ne, d_d2s_ + d2s_off_.pinv, add0, nullptr, npl, nq, ms);
        else
            launch_ntt_finish(S(), T_, o.data, conv, acc, ne, d_d2s_ + d2s_off_.pinv, add0, nullptr, npl, nq, ms);
        untmp(yp, (size_t)npl * np);
        cnt_[C_NTT_ROWS] += (size_t)npl * nq;
        untmp(conv, (size_t)npl * nq);
        untmp(acc, (size_t)npl * ne);
        cnt_[C_KS] += nb;
        tally(LV_KS, 0, nb);
        return o;
    }

    // relinearisation fused with the rescale that follows it: one ModDown by
    // Q' = P * (the dropped limbs of level l).  key_inner folds P (c0, c1) into acc's Q rows, so
    // acc = P * (relinearised ciphertext); the dropped and P rows (contiguous in acc) go to
    // coefficients together, one conversion to the r kept limbs, and the NTT finish computes
    // (acc - conv) Q'^{-1}.  Saves the separate rescale's INTT + spread + NTT of 2 r rows.
    // members one batched key switch at `level` can carry: the key inner product's batch and the
    // ModUp conversion's groups (members x digits) both bound it
    int ks_chunk(int level) const {
        const int nd = (hp_.nl(level) + hp_.alpha - 1) / hp_.alpha;
        return std::max(1, std::min(kMaxKsBatch, kMaxConvGroups / nd));
    }
    bool fused_relin_rescale_ok(const Ct& c) const {
        if (!fuse_rr_ || pm(c) != 3 || c.pend < 1 || c.level < 1 || c.zero) return false;
        return mdr_off_[c.level] != SIZE_MAX && 2 * ks_chunk(c.level) <= kMaxConvGroups;
    }
    // a stack of more than ks_chunk members in chunks, each chunk's ModDown writing its rows of
    // the one stacked result
    // outm (nb <= ks_chunk): member m's result straight into outm[m]; the returned Ct has no data
    Ct relin_rescale(const Ct& c, u32* const* outm = nullptr) {
        const int l = c.level, n = hp_.n, nl = hp_.nl(l), ne = nl + hp_.n_p, nb = c.nb, ch = ks_chunk(l);
        if (outm && nb > ch) throw std::runtime_error("relin_rescale: per-member outputs need one chunk");
        const size_t ms = (size_t)3 * nl * n;
        Ct o;
        if (nb > ch) {
            o = alloc_ct(l - 1, 2 * nb, nb);
            const size_t oms = (size_t)2 * hp_.nl(l - 1) * n;
            for (int m0 = 0; m0 < nb; m0 += ch) {
                const int k = std::min(ch, nb - m0);
                const u32* base = c.data + m0 * ms;
                const KsFold fold{base, base + (size_t)nl * n, ms, d_gadget_};
                if (fused_ki_ok()) {
                    const int h = ne - hp_.nl(l - 1);
                    u32* ext = modup(base + (size_t)2 * nl * n, l, k, ms, nullptr, false, true);
                    u32* acc = tmp(2 * (size_t)ne * k);
                    u32* ys = tmp(2 * (size_t)h * k);
                    const KiSrc src{ext, base + (size_t)2 * nl * n, ksk(0)};
                    ki_core(acc, ys, l, hp_.nl(l - 1), k, &src, 1, ms, fold);
                    untmp(ext, (size_t)k * ext_rows(l));
                    moddown_rescale(acc, l, k, o.data + m0 * oms, nullptr, nullptr, ys);
                    untmp(ys, 2 * (size_t)h * k);
                    untmp(acc, 2 * (size_t)ne * k);
                    continue;
                }
                u32* ext = modup(base + (size_t)2 * nl * n, l, k, ms);
                u32* acc = tmp(2 * (size_t)ne * k);
                key_inner(acc, ext, base + (size_t)2 * nl * n, ksk(0), l, 0, k, ms, fold);
                untmp(ext, (size_t)k * ext_rows(l));
                moddown_rescale(acc, l, k, o.data + m0 * oms);
                untmp(acc, 2 * (size_t)ne * k);
            }
        } else {
            const u32* d2 = c.data + (size_t)2 * nl * n;
            const KsFold fold{c.data, c.data + (size_t)nl * n, ms, d_gadget_};
            if (fused_ki_ok()) {
                const int h = ne - hp_.nl(l - 1);
                u32* ext = modup(d2, l, nb, ms, nullptr, false, true);
                u32* acc = tmp(2 * (size_t)ne * nb);
                u32* ys = tmp(2 * (size_t)h * nb);
                const KiSrc src{ext, d2, ksk(0)};
                ki_core(acc, ys, l, hp_.nl(l - 1), nb, &src, 1, ms, fold);
                untmp(ext, (size_t)nb * ext_rows(l));
                o = moddown_rescale(acc, l, nb, nullptr, outm, nullptr, ys);
                untmp(ys, 2 * (size_t)h * nb);
                untmp(acc, 2 * (size_t)ne * nb);
            } else {
                u32* ext = modup(d2, l, nb, ms);
                u32* acc = tmp(2 * (size_t)ne * nb);
                key_inner(acc, ext, d2, ksk(0), l, 0, nb, ms, fold);
                untmp(ext, (size_t)nb * ext_rows(l));
                o = moddown_rescale(acc, l, nb, nullptr, outm);
                untmp(acc, 2 * (size_t)ne * nb);
            }
        }
        o.pend = c.pend - 1;
        o.lazy = c.lazy && o.pend > 0;
        cnt_[C_KS] += nb;
        tally(LV_KS, l, nb);
        cnt_[C_RELIN]++;
        return o;
    }
    // the 2 x - c epilogue per member of a relinearisation + rescale (EvalMod's 2 T^2 - 1, the
    // residues of lincomb(P, 2, nullptr, 0, -c, 0)): dbl bit m doubles member m, cst[m] its constant
    struct Affine {
        unsigned dbl = 0;
        const u32* cst[kMaxKsBatch] = {};
        bool any() const { return dbl != 0; }
    };
    // relin_rescale of the products a[m] * b[m] (2-polynomial ciphertexts at one level, NTT form,
    // pend 0; nb <= ks_chunk) without materialising their tensors: the ModUp's inverse NTT forms
    // c2 = a1 (.) b1 on load, k_key_inner forms the own digit's c2 and the fold's (c0, c1) -- the
    // residues k_tensor_ptrs would have written, so the result is the same bit for bit, one launch
    // and 3 written + 3 re-read tensor rows per limb fewer (AESFHE_FUSED_TENSOR=0: tensor first)
    void relin_rescale_tensor(const TensorPtrs& tp, int l, int nb, u32* const* outm, const Affine* af = nullptr) {
        const int n = hp_.n, nl = hp_.nl(l), ne = nl + hp_.n_p;
        if (nb > ks_chunk(l) || nb > kMaxKsBatch) throw std::runtime_error("relin_rescale_tensor: more members than one chunk");
        TensorPtrs t1;  // a1, b1
        KsFold f{nullptr, nullptr, 0, d_gadget_};
        f.tnl = nl;
        for (int m = 0; m < nb; ++m) {
            t1.a[m] = tp.a[m] + (size_t)nl * n, t1.b[m] = tp.b[m] + (size_t)nl * n;
            f.ta[m] = tp.a[m], f.tb[m] = tp.b[m];
        }
        if (fused_ki_ok()) {
            const int h = ne - hp_.nl(l - 1);
            u32* ext = modup(nullptr, l, nb, 0, &t1, false, true);
            u32* acc = tmp(2 * (size_t)ne * nb);
            u32* ys = tmp(2 * (size_t)h * nb);
            const KiSrc src{ext, nullptr, ksk(0)};
            ki_core(acc, ys, l, hp_.nl(l - 1), nb, &src, 1, 0, f);
            untmp(ext, (size_t)nb * ext_rows(l));
            moddown_rescale(acc, l, nb, nullptr, outm, af, ys);
            untmp(ys, 2 * (size_t)h * nb);
            untmp(acc, 2 * (size_t)ne * nb);
            cnt_[C_KS] += nb;
            tally(LV_KS, l, nb);
            cnt_[C_RELIN]++;
            return;
        }
        u32* ext = modup(nullptr, l, nb, 0, &t1);
        u32* acc = tmp(2 * (size_t)ne * nb);
        key_inner(acc, ext, nullptr, ksk(0), l, 0, nb, 0, f);
        untmp(ext, (size_t)nb * ext_rows(l));
        Ct o = moddown_rescale(acc, l, nb, nullptr, outm, af);
        (void)o;
        untmp(acc, 2 * (size_t)ne * nb);
        cnt_[C_KS] += nb;
        tally(LV_KS, l, nb);
        cnt_[C_RELIN]++;
    }
    // device residues of the constant -c at (level, pend 0), [limb][lo, hi] (k_lincomb's cadd), cached
    const u32* affine_const(int level, double c) {
        const auto key = std::make_pair(level, c);
        auto it = affine_cst_.find(key);
        if (it != affine_cst_.end()) return it->second;
        const LimbConsts lc = add_consts(level, 0, -c, 0.0);
        const int nl = hp_.nl(level);
        u32* d = dev_alloc((size_t)2 * nl);
        HIP_OK(hipMemcpy(d, lc.v, sizeof(u32) * 2 * nl, hipMemcpyHostToDevice));
        return affine_cst_[key] = d;
    }
    std::map<std::pair<int, double>, const u32*> affine_cst_;
    // acc = [m][2][ne] in Q*P, NTT form, already holding P * (the ciphertext) -> the ciphertext
    // divided by the dropped limbs of level l, at level l - 1 (one ModDown by Q' = P * D)
    // ys_in: the dropped + P rows already through the INTT's row pass (ki_core, [m][2][h]): only its column pass runs here
    Ct moddown_rescale(const u32* acc, int l, int nb, u32* dst = nullptr, u32* const* outm = nullptr, const Affine* af = nullptr,
                       u32* ys_in = nullptr) {
        const int n = hp_.n, nl = hp_.nl(l), r = hp_.nl(l - 1), k = nl - r, np = hp_.n_p, ne = nl + np;
        const int npl = 2 * nb, h = k + np;
        if (mdr_off_[l] == SIZE_MAX || npl > kMaxConvGroups) throw std::runtime_error("moddown_rescale: unsupported level or batch");
        const bool fz = fused_conv(false);
        if (fz && af && af->any()) throw std::runtime_error("moddown_rescale: the epilogue needs the separate conversion");
        const size_t off = mdr_off_[l];
        u32* ys = ys_in ? ys_in : tmp((size_t)npl * h);
        const bool bx = bx_ok() && h <= kBxMaxH;
        if (bx) {  // the dropped + P rows through the INTT's row pass only (k_bx_cols runs the rest)
            if (!ys_in) launch_ntt_inv_rows(S(), T_, ys, acc, npl * h, RowMap{h, ne, h, r, 0}, LimbMap{k, r, hp_.p_off()});
            cnt_[C_NTT_ROWS] += (size_t)npl * h;
        } else if (ys_in) {
            if (fz) throw std::runtime_error("moddown_rescale: a fused-core input needs the separate conversion");
            launch_ntt_inv_cols(S(), T_, ys, npl * h, rows_dense(h), LimbMap{k, r, hp_.p_off()}, conv_pre_ ? d_mdr_ + off + 2 * (size_t)h * r : nullptr);
            cnt_[C_NTT_ROWS] += (size_t)npl * h;
        } else {
            intt(ys, acc, npl * h, RowMap{h, ne, h, r, 0}, LimbMap{k, r, hp_.p_off()}, fz || conv_pre_ ? d_mdr_ + off + 2 * (size_t)h * r : nullptr);
        }
        u32* conv = tmp((size_t)npl * r);
        ConvBatch cb;
        cb.n = npl;
        cb.pre = conv_pre_ && !bx;
        for (int p = 0; p < npl; ++p) {
            cb.h[p] = h, cb.d0[p] = r, cb.split[p] = k, cb.d1[p] = hp_.p_off(), cb.skip0[p] = 1 << 30;
            cb.src[p] = ys + (size_t)p * h * n;
            cb.dst[p] = conv + (size_t)p * r * n;
            cb.tab[p] = d_mdr_ + off;                           // [h][r] pairs
            cb.qhinv[p] = d_mdr_ + off + 2 * (size_t)h * r;     // [h] pairs
            cb.negq[p] = d_mdr_ + off + 2 * (size_t)h * (r + 1);  // [r]
        }
        if (bx) launch_bx_cols(S(), T_, cb, r, qmap());
        else if (!fz) launch_base_convert(S(), T_, cb, r, qmap());
        Ct o;
        if (dst || outm) {
            o.level = l - 1, o.npoly = npl, o.nb = nb, o.words = (size_t)npl * r * n, o.data = dst;
        } else {
            o = alloc_ct(l - 1, npl, nb);
        }
        const u32* qinv = d_mdr_ + off + 2 * (size_t)h * (r + 1) + r;
        if (bx)
            launch_ntt_finish_rows(S(), T_, o.data, conv, acc, ne, qinv, nullptr, nullptr, npl, r, 0, outm, false, af ? af->dbl : 0u,
                                   af && af->any() ? af->cst : nullptr);
        else if (fz)
            launch_ntt_finish_conv(S(), T_, o.data, conv, cb, acc, ne, qinv, nullptr, nullptr, npl, r, 0, outm);
        else
            launch_ntt_finish(S(), T_, o.data, conv, acc, ne, qinv, nullptr, nullptr, npl, r, 0, outm, af ? af->dbl : 0u,
                              af && af->any() ? af->cst : nullptr);
        if (!ys_in) untmp(ys, (size_t)npl * h);
        cnt_[C_NTT_ROWS] += (size_t)npl * r;
        untmp(conv, (size_t)npl * r);
        cnt_[C_RESCALE]++;
        return o;
    }

    // ct x ct.  Inputs are brought to canonical form; the tensor owes one rescale.  relin:
    // key switch now (eager) or leave it to the first consumer that needs two polynomials
    // (lazy)
    // aff (relin, not lazy): the product's 2 P - 1 (EvalMod's 2 T^2 - 1) instead of P -- in the
    // relinearisation's finish when it is fused (Affine), else one lincomb after it
    Ct mul(const Ct& a_in, const Ct& b_in, bool relin, bool lazy = false, bool aff = false) {
        if (vis_npoly(a_in) != 2 || vis_npoly(b_in) != 2) throw std::runtime_error("multiply expects 2-polynomial ciphertexts");
        if (a_in.level - a_in.pend < 1 || b_in.level - b_in.pend < 1)
            throw std::runtime_error("not enough level to multiply (level 0)");
        Ct a = normalize(a_in);
        Ct b = b_in.data == a_in.data ? a : normalize(b_in);
        const bool oa = a.data != a_in.data, ob = b.data != b_in.data && b.data != a.data;
        bool fa, fb;
        auto xy = align(a, b, fa, fb, true);
        const Ct &x = xy.first, &y = xy.second;
        const int nl = hp_.nl(x.level);
        if (x.nb != y.nb) throw std::runtime_error("multiply: batched operands of different sizes");
        if (relin && !lazy && fused_tensor_ && !fused_conv(true) && x.nb <= std::min(ks_chunk(x.level), kMaxKsBatch)) {
            Ct probe;
            probe.level = x.level, probe.npoly = 3 * x.nb, probe.nb = x.nb, probe.pend = 1, probe.ntt = true;
            if (fused_relin_rescale_ok(probe)) {  // relinearised and rescaled straight from the factors (relin_rescale_tensor)
                Ct o = alloc_ct(x.level - 1, 2 * x.nb, x.nb);
                o.ntt = true, o.pend = 0, o.lazy = false;
                TensorPtrs tp;
                u32* om[kMaxKsBatch];
                const size_t ms = (size_t)2 * nl * hp_.n, oms = (size_t)2 * hp_.nl(x.level - 1) * hp_.n;
                Affine af;
                for (int m = 0; m < x.nb; ++m) {
                    tp.a[m] = x.data + m * ms, tp.b[m] = y.data + m * ms, om[m] = o.data + m * oms;
                    if (aff) af.dbl |= 1u << m, af.cst[m] = affine_const(x.level - 1, 1.0);
                }
                relin_rescale_tensor(tp, x.level, x.nb, om, aff ? &af : nullptr);
                cnt_[C_MUL]++;
                tally(LV_MUL, o.level + 1, o.nb);
                if (fa) release(x);
                if (fb && y.data != x.data) release(y);
                if (oa) release(a);
                if (ob) release(b);
                return o;
            }
        }
        Ct d = alloc_ct(x.level, 3 * x.nb, x.nb);
        d.pend = 1;
        launch_tensor(S(), T_, d.data, x.data, y.data, nl, qmap(), x.nb);
        if (fa) release(x);
        if (fb && y.data != x.data) release(y);
        if (oa) release(a);
        if (ob) release(b);
        cnt_[C_MUL]++;
        tally(LV_MUL, d.level, d.nb);
        if (!relin) return d;
        if (lazy) {
            d.lazy = true;
            return d;
        }
        Ct o;
        if (fused_relin_rescale_ok(d)) {
            o = relin_rescale(d);
            release(d);
        } else {
            Ct r = relin_raw(d);
            release(d);
            o = rescale(r);
            release(r);
        }
        if (!aff) return o;
        Ct t = lincomb(o, 2, nullptr, 0, -1.0, 0.0);
        release(o);
        return t;
    }

    // n independent products a_i b_i, relinearised and rescaled, batched:
    // pairs whose aligned operands sit at one level share ONE tensor launch and one fused
    // relinearisation + rescale per chunk of kMaxKsBatch members (each key residue read once
    // per chunk, every launch carrying the chunk's rows); the results equal n mul() calls
    // aff (nullable, one flag per pair): that product's 2 P - 1 (mul's aff)
    std::vector<Ct> mul_many(const std::vector<const Ct*>& A, const std::vector<const Ct*>& B, const std::vector<char>* aff = nullptr) {
        const int n = (int)A.size();
        std::vector<Ct> out(n);
        auto affi = [&](int i) { return aff && (*aff)[i]; };
        bool batch = batch_ops_ && n >= 2;
        for (int i = 0; i < n; ++i) {
            if (vis_npoly(*A[i]) != 2 || vis_npoly(*B[i]) != 2) throw std::runtime_error("multiply expects 2-polynomial ciphertexts");
            if (A[i]->level - A[i]->pend < 1 || B[i]->level - B[i]->pend < 1)
                throw std::runtime_error("not enough level to multiply (level 0)");
            batch = batch && A[i]->nb == 1 && B[i]->nb == 1;
        }
        if (!batch) {
            for (int i = 0; i < n; ++i) out[i] = mul(*A[i], *B[i], true, false, affi(i));
            return out;
        }
        struct Prep {
            Ct a, b, x, y;
        };
        std::vector<Prep> pr(n);
        std::vector<Ct> owned;  // normalised inputs and level-aligned copies, released after the tensors
        for (int i = 0; i < n; ++i) {
            Prep& P = pr[i];
            P.a = normalize(*A[i]);
            if (P.a.data != A[i]->data) owned.push_back(P.a);
            P.b = B[i]->data == A[i]->data ? P.a : normalize(*B[i]);
            if (P.b.data != B[i]->data && P.b.data != P.a.data) owned.push_back(P.b);
        }
        // level alignment of every pair (as align(..., for_mul)), the exact-scale drops of inputs at one
        // (level, owed rescales) to one target batched: ONE copy-and-scale launch and ONE limb drop
        // for the group (convert_many) instead of one convert each
        struct Need {
            const Ct* src;
            int t;
            Ct res;
        };
        std::vector<Need> needs;
        auto want = [&](const Ct& c, int t) -> int {
            if (c.level == t && !c.pend) return -1;
            for (size_t j = 0; j < needs.size(); ++j)
                if (needs[j].src->data == c.data && needs[j].t == t) return (int)j;
            needs.push_back({&c, t, Ct{}});
            return (int)needs.size() - 1;
        };
        std::vector<int> wa(n), wb(n);
        for (int i = 0; i < n; ++i) {
            int lv = std::min(pr[i].a.level - pr[i].a.pend, pr[i].b.level - pr[i].b.pend);
            if (!hp_.homogeneous(lv)) --lv;
            wa[i] = want(pr[i].a, lv);
            wb[i] = want(pr[i].b, lv);
        }
        std::vector<bool> conv_done(needs.size(), false);
        for (size_t j = 0; j < needs.size(); ++j) {
            if (conv_done[j]) continue;
            const Ct& c = *needs[j].src;
            std::vector<size_t> grp{j};
            for (size_t k = j + 1; k < needs.size() && (int)grp.size() < kMaxMembers; ++k) {
                const Ct& d = *needs[k].src;
                if (!conv_done[k] && needs[k].t == needs[j].t && d.level == c.level && d.pend == c.pend && d.npoly == c.npoly &&
                    d.nb == 1 && c.nb == 1 && d.ntt && c.ntt)
                    grp.push_back(k);
            }
            for (size_t k : grp) conv_done[k] = true;
            if (grp.size() == 1) {
                needs[j].res = level_down(c, needs[j].t);
                owned.push_back(needs[j].res);
                continue;
            }
            std::vector<const Ct*> srcs;
            for (size_t k : grp) srcs.push_back(needs[k].src);
            Ct st;
            if (!convert_many(srcs, needs[j].t, 0, st)) {  // no batched form: one convert each
                for (size_t k : grp) {
                    needs[k].res = level_down(*needs[k].src, needs[k].t);
                    owned.push_back(needs[k].res);
                }
                continue;
            }
            owned.push_back(st);
            const size_t per = st.words / grp.size();
            for (size_t m = 0; m < grp.size(); ++m) {
                Ct v = st;
                v.data = st.data + m * per, v.words = per, v.npoly = st.npoly / (int)grp.size(), v.nb = 1;
                needs[grp[m]].res = v;
            }
        }
        for (int i = 0; i < n; ++i) {
            pr[i].x = wa[i] < 0 ? pr[i].a : needs[wa[i]].res;
            pr[i].y = wb[i] < 0 ? pr[i].b : needs[wb[i]].res;
        }
        std::vector<bool> done(n, false);
        for (int i = 0; i < n; ++i) {
            if (done[i]) continue;
            std::vector<int> grp;  // members at the same level, up to kMaxMembers
            for (int j = i; j < n && (int)grp.size() < kMaxMembers; ++j)
                if (!done[j] && pr[j].x.level == pr[i].x.level) grp.push_back(j), done[j] = true;
            const int g = (int)grp.size(), L = pr[i].x.level, nl = hp_.nl(L), nn = hp_.n;
            TensorPtrs tp;
            for (int m = 0; m < g; ++m) tp.a[m] = pr[grp[m]].x.data, tp.b[m] = pr[grp[m]].y.data;
            const int chunk = ks_chunk(L);
            {  // every chunk relinearised and rescaled straight from its factors (relin_rescale_tensor)
                Ct probe;
                probe.level = L, probe.npoly = 3 * std::min(chunk, g), probe.nb = std::min(chunk, g), probe.pend = 1, probe.ntt = true;
                if (fused_tensor_ && !fused_conv(true) && fused_relin_rescale_ok(probe)) {
                    cnt_[C_MUL] += g;
                    tally(LV_MUL, L, g);
                    for (int m0 = 0; m0 < g; m0 += chunk) {
                        const int c = std::min(chunk, g - m0);
                        TensorPtrs sub;
                        u32* om[kMaxKsBatch];
                        Affine af;
                        for (int m = 0; m < c; ++m) {
                            sub.a[m] = tp.a[m0 + m], sub.b[m] = tp.b[m0 + m];
                            Ct& r = out[grp[m0 + m]];
                            r = alloc_ct(L - 1, 2);
                            r.ntt = true, r.pend = 0, r.lazy = false;
                            om[m] = r.data;
                            if (affi(grp[m0 + m])) af.dbl |= 1u << m, af.cst[m] = affine_const(L - 1, 1.0);
                        }
                        relin_rescale_tensor(sub, L, c, om, af.any() ? &af : nullptr);
                    }
                    continue;
                }
            }
            Ct d = alloc_ct(L, 3 * g, g);
            d.pend = 1;
            launch_tensor_ptrs(S(), T_, d.data, tp, g, nl, qmap());
            cnt_[C_MUL] += g;
            tally(LV_MUL, L, g);
            for (int m0 = 0; m0 < g; m0 += chunk) {
                const int c = std::min(chunk, g - m0);
                Ct v = d;  // view of members m0 .. m0 + c - 1 (not released on its own)
                v.data = d.data + (size_t)m0 * 3 * nl * nn, v.npoly = 3 * c, v.nb = c, v.words = (size_t)3 * c * nl * nn;
                if (fused_relin_rescale_ok(v)) {
                    // each member's ModDown finish writes its own output buffer: no unstack copy
                    u32* om[kMaxKsBatch];
                    for (int m = 0; m < c; ++m) {
                        Ct& r = out[grp[m0 + m]];
                        r = alloc_ct(L - 1, 2);
                        r.ntt = true, r.pend = 0, r.lazy = false;
                        om[m] = r.data;
                    }
                    Ct o = relin_rescale(v, om);
                    (void)o;
                } else {
                    Ct r = relin_raw(v);
                    Ct o = rescale(r);
                    release(r);
                    unstack(o, &out[0], grp.data() + m0);
                    release(o);
                }
            }
            release(d);
            for (int m = 0; m < g; ++m)  // the tensor-first form: 2 P - 1 as its own launch
                if (affi(grp[m])) {
                    Ct t = lincomb(out[grp[m]], 2, nullptr, 0, -1.0, 0.0);
                    release(out[grp[m]]);
                    out[grp[m]] = t;
                }
        }
        for (const Ct& c : owned) release(c);  // stream-ordered: the tensors above were queued first
        return out;
    }
    // convert(c, t, p) of several ciphertexts at one (data level, owed rescales, polys): ONE
    // copy-and-scale launch into a stack and ONE limb drop for all of them.  st: the stack (nb =
    // members, member m = S[m] converted, the same residues as convert(S[m], t, p)).  false when
    // the conversion needs the relinearise-first path of convert()
    bool convert_many(const std::vector<const Ct*>& Sv, int t, int p, Ct& st) {
        const Ct& c = *Sv[0];
        const int m = (int)Sv.size();
        if (m > kMaxMembers || p < 0 || t > c.level || t - p > c.level - c.pend) return false;
        const int n = hp_.n, nb = hp_.nl(t), na = hp_.nl(c.level);
        int k = 0;
        double ratio = raw_scale(t, p) / raw_scale(c.level, c.pend);
        const double need = t > hp_.L1 ? 2251799813685248.0 : 16777216.0;  // as convert()
        while (ratio < need && nb + k < na) ratio *= (double)hp_.mod[nb + k], ++k;
        if (!(ratio >= 0.999999 && ratio < 9.0e18)) return false;
        if (pm(c) == 3 && k > 0 && raw_scale(t, p) < 1.0e15) return false;
        const int nk = nb + k, np = c.npoly;
        u32* mid = tmp((size_t)m * np * nk);
        const i64 cst = std::llround(ratio);
        std::vector<u32> r(nk);
        for (int i = 0; i < nk; ++i) r[i] = mod_i64(cst, hp_.mod[i]);
        MemberPtrs mp;
        for (int i = 0; i < m; ++i) mp.src[i] = Sv[i]->data;
        launch_mul_const_half_members(S(), T_, mid, mp, m, const_half(r, r), np * nk, nk, qmap(), na);
        st = Ct{};
        st.level = t, st.npoly = m * np, st.nb = m, st.pend = p, st.lazy = c.lazy || p > 0, st.zero = false;
        st.words = (size_t)m * np * nb * n;
        if (k == 0) {
            st.data = mid;
        } else {
            st.data = drop_limbs(mid, m * np, nk, k);
            untmp(mid, (size_t)m * np * nk);
        }
        return true;
    }
    // members of a stacked canonical ciphertext -> separate ciphertexts out[idx[m]]
    void unstack(const Ct& o, Ct* out, const int* idx) {
        const int c = o.nb, nlo = hp_.nl(o.level), nn = hp_.n, per = o.npoly / c;
        MemberPtrs mp;
        for (int m = 0; m < c; ++m) {
            Ct r = alloc_ct(o.level, per);
            copy_meta(r, o);
            r.nb = 1;
            mp.src[m] = o.data + (size_t)m * per * nlo * nn;
            mp.dst[m] = r.data;
            out[idx[m]] = r;
        }
        launch_copy_members(S(), T_, mp, c, per * nlo);
    }
    // ------------------------------------------------------------------ stacked ciphertexts (multi-pair batches)
    // n single ciphertexts -> ONE stacked ciphertext (nb = n members, [m][2][nl] rows): canonical
    // form, dropped to the lowest member level.  Every op then treats the stack as one operand:
    // element-wise launches cover all members' rows, key switches read each key once per chunk
    // of ks_chunk members, LUT sums take a member grid dimension.
    Ct stack(const std::vector<const Ct*>& C) {
        const int n = (int)C.size();
        if (n < 1) throw std::runtime_error("stack: no ciphertexts");
        std::vector<Ct> cn(n);
        std::vector<bool> own(n);
        int lv = 1 << 30;
        for (int i = 0; i < n; ++i) {
            if (C[i]->nb != 1) throw std::runtime_error("stack: members must be single ciphertexts");
            cn[i] = normalize(*C[i]);
            own[i] = cn[i].data != C[i]->data;
            if (pm(cn[i]) != 2) throw std::runtime_error("stack: 2-polynomial ciphertexts expected");
            lv = std::min(lv, cn[i].level);
        }
        for (int i = 0; i < n; ++i)
            if (cn[i].level != lv) {
                Ct t = level_down(cn[i], lv);
                if (own[i]) release(cn[i]);
                cn[i] = t, own[i] = true;
            }
        const int nl = hp_.nl(lv), nn = hp_.n;
        Ct st = alloc_ct(lv, 2 * n, n);
        st.ntt = true;
        for (int m0 = 0; m0 < n; m0 += kMaxMembers) {
            const int c = std::min(kMaxMembers, n - m0);
            MemberPtrs mp;
            for (int m = 0; m < c; ++m) mp.src[m] = cn[m0 + m].data, mp.dst[m] = st.data + (size_t)(m0 + m) * 2 * nl * nn;
            launch_copy_members(S(), T_, mp, c, 2 * nl);
        }
        for (int i = 0; i < n; ++i)
            if (own[i]) release(cn[i]);
        return st;
    }
    // the members of a stack as single canonical ciphertexts
    std::vector<Ct> unstack_all(const Ct& c_in) {
        Ct c = normalize(c_in);
        const int nb = c.nb, per = pm(c), nl = hp_.nl(c.level), nn = hp_.n;
        std::vector<Ct> out(nb);
        for (int m0 = 0; m0 < nb; m0 += kMaxMembers) {
            const int k = std::min(kMaxMembers, nb - m0);
            MemberPtrs mp;
            for (int m = 0; m < k; ++m) {
                Ct r = alloc_ct(c.level, per);
                copy_meta(r, c);
                r.nb = 1;
                mp.src[m] = c.data + (size_t)(m0 + m) * per * nl * nn;
                mp.dst[m] = r.data;
                out[m0 + m] = r;
            }
            launch_copy_members(S(), T_, mp, k, per * nl);
        }
        if (c.data != c_in.data) release(c);
        return out;
    }
    // rows [m0, m0 + cnt) of a canonical stack as a stack of their own (a copy)
    Ct members_of(const Ct& c, int m0, int cnt) {
        const int per = pm(c), nl = hp_.nl(c.level);
        Ct o = alloc_ct(c.level, per * cnt, cnt);
        copy_meta(o, c);
        o.nb = cnt;
        launch_copy_rows(S(), T_, o.data, c.data + (size_t)m0 * per * nl * hp_.n, (size_t)cnt * per * nl);
        return o;
    }

    // X -> X^g of n independent ciphertexts: canonical inputs at one level are stacked and key
    // switched together (chunks of kMaxKsBatch); results equal n galois() calls
    std::vector<Ct> galois_many(const std::vector<const Ct*>& C, u64 g) {
        const int n = (int)C.size();
        std::vector<Ct> out(n);
        std::vector<Ct> cn(n);
        std::vector<bool> own(n), done(n, false);
        for (int i = 0; i < n; ++i) {
            if (vis_npoly(*C[i]) != 2) throw std::runtime_error("rotation/conjugation expects a 2-polynomial ciphertext");
            cn[i] = normalize(*C[i]);
            own[i] = cn[i].data != C[i]->data;
        }
        for (int i = 0; i < n; ++i) {
            if (done[i]) continue;
            std::vector<int> grp;
            for (int j = i; j < n && (int)grp.size() < ks_chunk(cn[i].level); ++j)
                if (!done[j] && batch_ops_ && cn[j].level == cn[i].level && cn[j].nb == 1 && cn[i].nb == 1) grp.push_back(j), done[j] = true;
            if (grp.size() < 2) {
                done[i] = true;
                out[i] = galois(cn[i], g);
                for (int j : grp) if (j != i) done[j] = false;
                continue;
            }
            const int c = (int)grp.size(), nl = hp_.nl(cn[i].level), nn = hp_.n;
            Ct st = alloc_ct(cn[i].level, 2 * c, c);
            copy_meta(st, cn[i]);
            st.nb = c;
            MemberPtrs mp;
            for (int m = 0; m < c; ++m) mp.src[m] = cn[grp[m]].data, mp.dst[m] = st.data + (size_t)m * 2 * nl * nn;
            launch_copy_members(S(), T_, mp, c, 2 * nl);
            Ct o = galois(st, g);
            release(st);
            unstack(o, &out[0], grp.data());
            release(o);
        }
        for (int i = 0; i < n; ++i)
            if (own[i]) release(cn[i]);
        return out;
    }

    // ------------------------------------------------------------------ heterogeneous batched key switch
    // n automorphisms X -> X^G[i] of possibly different ciphertexts (rotations by different steps,
    // conjugations, or a mix), each followed by its key switch.  Inputs are brought to canonical
    // form first -- deferred scalar / plaintext products owing ONE rescale at a common level are
    // stacked and rescaled together (one INTT + one spread-NTT-finish for all of them).  Items at
    // one level then form ONE batched key switch per chunk: one ModUp per distinct source (a
    // source's several automorphisms read its extension through X -> X^g: hoisted), ONE key inner
    // product launch with a key and a Galois element per member, ONE automorphism launch for the
    // c0s and ONE stacked ModDown.  Results equal galois(C[i], G[i]) bit for bit.
    struct KsSrc {
        const u32* c0;
        const u32* c1;
        int level;
    };
    std::vector<Ct> galois_multi(const std::vector<const Ct*>& C, const std::vector<u64>& G) {
        const int n = (int)C.size(), nn = hp_.n;
        if ((int)G.size() != n) throw std::runtime_error("galois_multi: one Galois element per ciphertext");
        const u64 two_n = 2ull * nn;
        for (u64 g : G)
            if (!(g & 1) || g >= two_n) throw std::runtime_error("galois_multi: Galois elements must be odd and below 2N");
        std::vector<Ct> out(n);
        bool stacked = false;
        for (const Ct* c : C) stacked = stacked || c->nb != 1;
        if (stacked) {  // stacks: one galois() each (every member of a stack in one key switch)
            for (int i = 0; i < n; ++i) {
                if (G[i] == 1) { Ct cn = normalize(*C[i]); out[i] = cn.data != C[i]->data ? cn : copy(cn); continue; }
                out[i] = galois(*C[i], G[i]);
            }
            return out;
        }
        std::vector<Ct> owned;                      // buffers released at the end
        std::map<const u32*, KsSrc> src_of;         // input data -> canonical source
        // 1. canonical sources; lazy 2-polynomial tensors owing one rescale, grouped by level, are
        //    stacked and rescaled together
        std::map<int, std::vector<const Ct*>> lazy1;
        std::vector<bool> done(n, false);
        for (int i = 0; i < n; ++i) {
            const Ct& c = *C[i];
            if (vis_npoly(c) != 2) throw std::runtime_error("rotation/conjugation expects a 2-polynomial ciphertext");
            // conjugations of deferred tensors stay deferred, exactly as conjugate() does them (§3.14)
            if (G[i] == conj_galois() && lazy_galois_ok(c)) {
                out[i] = galois_lazy(c, G[i]);
                done[i] = true;
                continue;
            }
            if (src_of.count(c.data)) continue;
            if (c.lazy && c.pend == 1 && pm(c) == 2 && c.nb == 1 && c.ntt && !c.zero) {
                auto& v = lazy1[c.level];
                if (std::find(v.begin(), v.end(), &c) == v.end()) v.push_back(&c);
                src_of[c.data] = KsSrc{nullptr, nullptr, -1};  // filled below
                continue;
            }
            Ct cn = normalize(c);
            if (cn.data != c.data) owned.push_back(cn);
            src_of[c.data] = KsSrc{cn.data, cn.data + (size_t)hp_.nl(cn.level) * nn, cn.level};
        }
        for (auto& kv : lazy1) {
            const auto& v = kv.second;
            for (size_t m0 = 0; m0 < v.size(); m0 += kMaxMembers) {
                const int cnt = (int)std::min<size_t>(kMaxMembers, v.size() - m0), l = kv.first, nl = hp_.nl(l);
                if (cnt == 1) {
                    Ct cn = normalize(*v[m0]);
                    owned.push_back(cn);
                    src_of[v[m0]->data] = KsSrc{cn.data, cn.data + (size_t)hp_.nl(cn.level) * nn, cn.level};
                    continue;
                }
                Ct st = alloc_ct(l, 2 * cnt, cnt);
                MemberPtrs mp;
                for (int m = 0; m < cnt; ++m) mp.src[m] = v[m0 + m]->data, mp.dst[m] = st.data + (size_t)m * 2 * nl * nn;
                launch_copy_members(S(), T_, mp, cnt, 2 * nl);
                st.pend = 1;
                st.lazy = true;
                Ct rs = rescale(st);  // one rescale of all members (rescale handles npoly = 2 cnt)
                release(st);
                owned.push_back(rs);
                const int nlo = hp_.nl(rs.level);
                for (int m = 0; m < cnt; ++m) {
                    const u32* c0 = rs.data + (size_t)m * 2 * nlo * nn;
                    src_of[v[m0 + m]->data] = KsSrc{c0, c0 + (size_t)nlo * nn, rs.level};
                }
            }
        }
        // 2. items by level, chunked: members <= kMaxMembers, sources x digits <= kMaxConvGroups
        std::map<int, std::vector<int>> by_level;
        for (int i = 0; i < n; ++i) {
            if (done[i]) continue;
            const KsSrc& s = src_of.at(C[i]->data);
            if (G[i] == 1) {  // identity: a copy of the canonical source
                Ct o = alloc_ct(s.level, 2);
                launch_copy_rows(S(), T_, o.data, s.c0, 2 * (size_t)hp_.nl(s.level));
                out[i] = o;
                continue;
            }
            by_level[s.level].push_back(i);
        }
        for (auto& kv : by_level) {
            const int l = kv.first, nl = hp_.nl(l), ne = nl + hp_.n_p, nd = (nl + hp_.alpha - 1) / hp_.alpha;
            const auto& items = kv.second;
            const int max_src = std::max(1, kMaxConvGroups / nd);
            size_t pos = 0;
            while (pos < items.size()) {
                std::vector<int> chunk;
                std::vector<KsSrc> srcs;  // distinct sources, in first-use order
                auto src_index = [&](const KsSrc& s) {
                    for (size_t j = 0; j < srcs.size(); ++j)
                        if (srcs[j].c0 == s.c0) return (int)j;
                    return -1;
                };
                while (pos < items.size() && (int)chunk.size() < kMaxMembers) {
                    const KsSrc& s = src_of.at(C[items[pos]]->data);
                    const bool known = src_index(s) >= 0;
                    if (!known && (int)srcs.size() >= max_src) break;
                    if (!known) srcs.push_back(s);
                    chunk.push_back(items[pos++]);
                }
                const int nm = (int)chunk.size(), ns = (int)srcs.size();
                // c1 of every source, stacked: used in place when the sources already sit at a
                // member stride of 2 nl N (e.g. one stack rescaled above), else gathered
                const u32* c1s = srcs[0].c1;
                size_t d_ms = 0;
                u32* c1buf = nullptr;
                if (ns > 1) {
                    const size_t stride = (size_t)2 * nl * nn;
                    bool regular = true;
                    for (int j = 0; j < ns; ++j) regular = regular && srcs[j].c1 == srcs[0].c1 + j * stride;
                    if (regular) {
                        d_ms = stride;
                    } else {
                        std::vector<const u32*> c1v(ns);
                        for (int j = 0; j < ns; ++j) c1v[j] = srcs[j].c1;
                        c1buf = tmp((size_t)ns * nl);
                        MemberPtrs mp;
                        for (int j = 0; j < ns; ++j) mp.src[j] = c1v[j], mp.dst[j] = c1buf + (size_t)j * nl * nn;
                        launch_copy_members(S(), T_, mp, ns, nl);
                        c1s = c1buf, d_ms = (size_t)nl * nn;
                    }
                }
                u32* ext = modup(c1s, l, ns, d_ms);
                u32* acc = tmp((size_t)nm * 2 * ne);
                KsMultiArgs ka;
                AutoMulti am;
                for (int m = 0; m < nm; ++m) {
                    const int i = chunk[m];
                    const KsSrc& s = src_of.at(C[i]->data);
                    ka.key[m] = ksk(G[i]);
                    ka.g[m] = G[i];
                    ka.src[m] = src_index(s);
                    am.src[m] = s.c0;
                    am.g[m] = G[i];
                }
                launch_key_inner_multi(S(), T_, acc, ext, c1s, ka, nm, ns, nd, ne, nl, hp_.alpha, hp_.n_ks + hp_.n_p, hp_.n_ks, extmap(nl),
                                       (size_t)ext_rows(l) * nn, d_ms, (size_t)2 * ne * nn);
                untmp(ext, (size_t)ns * ext_rows(l));
                if (c1buf) untmp(c1buf, (size_t)ns * nl);
                const size_t ms = (size_t)2 * nl * nn;
                u32* c0p = tmp((size_t)nm * 2 * nl);  // member stride 2 nl N (moddown's add stride), first nl rows used
                launch_automorph_multi(S(), T_, c0p, ms, am, nm, nl);
                u32* om[kMaxMembers];  // each member's ModDown finish writes its own buffer: no unstack copy
                for (int m = 0; m < nm; ++m) {
                    Ct& r = out[chunk[m]];
                    r = alloc_ct(l, 2);
                    r.ntt = true, r.pend = 0, r.lazy = false;
                    om[m] = r.data;
                }
                moddown(acc, l, c0p, nullptr, nm, ms, nullptr, om);
                untmp(acc, (size_t)nm * 2 * ne);
                untmp(c0p, (size_t)nm * 2 * nl);
                cnt_[C_KS] += nm;
                tally(LV_KS, l, nm);
            }
        }
        for (const Ct& c : owned) release(c);
        return out;
    }

    void count_conj() { cnt_[C_CONJ]++; }
    void count_rot() { cnt_[C_ROT]++; }
    std::vector<Ct> conjugate_many(const std::vector<const Ct*>& C) {
        cnt_[C_CONJ] += C.size();
        // deferred inputs (a LUT sum owing its relinearisation and rescales) are conjugated as they
        // are (galois_lazy), the rest batched as before
        std::vector<Ct> out(C.size());
        std::vector<const Ct*> canon_in;
        std::vector<size_t> idx;
        for (size_t i = 0; i < C.size(); ++i) {
            if (lazy_galois_ok(*C[i])) out[i] = galois_lazy(*C[i], conj_galois());
            else canon_in.push_back(C[i]), idx.push_back(i);
        }
        if (!canon_in.empty()) {
            std::vector<Ct> r = galois_many(canon_in, conj_galois());
            for (size_t j = 0; j < idx.size(); ++j) out[idx[j]] = r[j];
        }
        return out;
    }

    // ------------------------------------------------------------------ automorphism of a deferred tensor
    // X -> X^g of a tensor that still owes work, WITHOUT resolving it: c0' = sigma(d0), plus the key
    // switch of sigma(d1) (sigma(s) -> s) and, for a 3-polynomial tensor, of sigma(d2) with the key
    // sigma(s)^2 -> s (tag_sq), both inner products summed in Q*P and ONE ModDown by P.  The owed
    // rescales stay owed (same data level, pend, raw scale): the caller's sum S1 + conj(S2) of two
    // deferred LUT tensors is then one addition at the same (level, pend), and a renorm reads it
    // raw -- no relinearisation, no rescale of either part (the conjugate-split LUTs of XOR4, the GF
    // multipliers and SubBytes).  Key-switching noise is added at the raw scale
    // S(l, pend) >= Delta^2 q, far below the message.
    bool lazy_galois_ok(const Ct& c) const {
        if (!lazy_galois_ || !c.ntt || c.zero || c.nb != 1) return false;
        return pm(c) == 3 ? c.lazy : (pm(c) == 2 && c.pend > 0);  // an explicit 3-polynomial product stays an error
    }
    bool lazy_galois_ = std::getenv("AESFHE_LAZY_GALOIS") == nullptr || std::getenv("AESFHE_LAZY_GALOIS")[0] != '0';
    Ct galois_lazy(const Ct& c, u64 g) {
        const int l = c.level, nl = hp_.nl(l), np = hp_.n_p, ne = nl + np, n = hp_.n, k = pm(c);
        if (g == conj_galois() && conj_rev_ && !fused_conv(true) && !fused_conv(false)) {
            // the conjugation (X -> X^(2N-1)) is the index reversal i -> N - 1 - i in this NTT order:
            // read reversed where the permuted copy was read -- the ModUp's inverse NTT, the own
            // digit's key inner product and the ModDown finish's c0 -- no k_automorph, same residues
            const int nsrc = k - 1;
            KsFold fr{};
            fr.rev_d = 1;
            if (fused_ki_ok()) {
                u32* ext = modup(c.data + (size_t)nl * n, l, nsrc, (size_t)nl * n, nullptr, true, true);
                u32* acc = tmp(2 * (size_t)ne);
                u32* ys = tmp(2 * (size_t)np);
                const KiSrc src[2] = {{ext, c.data + (size_t)nl * n, ksk(g)},
                                      {ext + (size_t)ext_rows(l) * n, c.data + (size_t)2 * nl * n, nsrc == 2 ? ksk(tag_sq(g)) : nullptr}};
                ki_core(acc, ys, l, nl, 1, src, nsrc, 0, fr);
                untmp(ext, (size_t)nsrc * ext_rows(l));
                Ct o = moddown(acc, l, c.data, nullptr, 1, 0, nullptr, nullptr, true, ys);
                untmp(ys, 2 * (size_t)np);
                untmp(acc, 2 * (size_t)ne);
                o.pend = c.pend;
                o.lazy = c.pend > 0;
                cnt_[C_KS] += nsrc;
                tally(LV_KS, l, nsrc);
                return o;
            }
            u32* ext = modup(c.data + (size_t)nl * n, l, nsrc, (size_t)nl * n, nullptr, true);
            u32* acc = tmp(2 * (size_t)ne);
            key_inner(acc, ext, c.data + (size_t)nl * n, ksk(g), l, 0, 1, 0, fr);
            if (nsrc == 2)
                key_inner(acc, ext + (size_t)ext_rows(l) * n, c.data + (size_t)2 * nl * n, ksk(tag_sq(g)), l, 0, 1, 0, fr, true);
            untmp(ext, (size_t)nsrc * ext_rows(l));
            Ct o = moddown(acc, l, c.data, nullptr, 1, 0, nullptr, nullptr, true);
            untmp(acc, 2 * (size_t)ne);
            o.pend = c.pend;
            o.lazy = c.pend > 0;
            cnt_[C_KS] += nsrc;
            tally(LV_KS, l, nsrc);
            return o;
        }
        u32* perm = tmp((size_t)k * nl);
        launch_automorph(S(), T_, perm, c.data, g, k * nl);
        // d1 (and d2) of the permuted tensor are consecutive rows: ONE ModUp for both sources
        const int nsrc = k - 1;
        u32* ext = modup(perm + (size_t)nl * n, l, nsrc, (size_t)nl * n);
        u32* acc = tmp(2 * (size_t)ne);
        key_inner(acc, ext, perm + (size_t)nl * n, ksk(g), l, 0);
        if (nsrc == 2)
            key_inner(acc, ext + (size_t)ext_rows(l) * n, perm + (size_t)2 * nl * n, ksk(tag_sq(g)), l, 0, 1, 0, KsFold{}, true);
        untmp(ext, (size_t)nsrc * ext_rows(l));
        Ct o = moddown(acc, l, perm, nullptr);
        untmp(acc, 2 * (size_t)ne);
        untmp(perm, (size_t)k * nl);
        o.pend = c.pend;
        o.lazy = c.pend > 0;
        cnt_[C_KS] += nsrc;
        tally(LV_KS, l, nsrc);
        return o;
    }

    Ct relinearize(const Ct& c_in) {
        if (vis_npoly(c_in) != 3) throw std::runtime_error("relinearize: ciphertext should have 3 polynomials");
        Ct c = ensure_ntt(c_in);
        Ct r = relin_raw(c);
        if (c.data != c_in.data) release(c);
        Ct o = normalize(r, true);
        if (o.data != r.data) release(r);
        return o;
    }

    Ct galois(const Ct& c_in, u64 g) {
        if (vis_npoly(c_in) != 2) throw std::runtime_error("rotation/conjugation expects a 2-polynomial ciphertext");
        Ct c = normalize(c_in);
        const int nl = hp_.nl(c.level), n = hp_.n;
        const u32* key = ksk(g);
        if (g == conj_galois() && conj_rev_ && c.nb == 1 && !fused_conv(true) && !fused_conv(false)) {
            // the conjugation as reversed reads (galois_lazy): no permuted copy
            const int ne = nl + hp_.n_p;
            KsFold fr{};
            fr.rev_d = 1;
            if (fused_ki_ok()) {
                const int np = hp_.n_p;
                u32* ext = modup(c.data + (size_t)nl * n, c.level, 1, 0, nullptr, true, true);
                u32* acc = tmp(2 * (size_t)ne);
                u32* ys = tmp(2 * (size_t)np);
                const KiSrc src{ext, c.data + (size_t)nl * n, key};
                ki_core(acc, ys, c.level, nl, 1, &src, 1, 0, fr);
                untmp(ext, (size_t)ext_rows(c.level));
                Ct o = moddown(acc, c.level, c.data, nullptr, 1, 0, nullptr, nullptr, true, ys);
                untmp(ys, 2 * (size_t)np);
                untmp(acc, 2 * (size_t)ne);
                cnt_[C_KS]++;
                tally(LV_KS, c.level, 1);
                if (c.data != c_in.data) release(c);
                return o;
            }
            u32* ext = modup(c.data + (size_t)nl * n, c.level, 1, 0, nullptr, true);
            u32* acc = tmp(2 * (size_t)ne);
            key_inner(acc, ext, c.data + (size_t)nl * n, key, c.level, 0, 1, 0, fr);
            untmp(ext, (size_t)ext_rows(c.level));
            Ct o = moddown(acc, c.level, c.data, nullptr, 1, 0, nullptr, nullptr, true);
            untmp(acc, 2 * (size_t)ne);
            cnt_[C_KS]++;
            tally(LV_KS, c.level, 1);
            if (c.data != c_in.data) release(c);
            return o;
        }
        u32* perm = tmp(2 * (size_t)nl * c.nb);
        launch_automorph(S(), T_, perm, c.data, g, 2 * nl * c.nb);
        const size_t ms = (size_t)2 * nl * n;  // member stride of a batched ciphertext
        Ct o = keyswitch(perm + (size_t)nl * n, c.level, key, perm, nullptr, c.nb, ms, ms);
        untmp(perm, 2 * (size_t)nl * c.nb);
        if (c.data != c_in.data) release(c);
        return o;
    }
    // several rotations of ONE ciphertext, hoisted: c1 is ModUp'ed once, each step is a key
    // inner product read through its automorphism plus a ModDown adding the permuted c0
    // (the same arithmetic as rotate(): ModUp commutes with the automorphism)
    std::vector<Ct> rotate_hoisted(const Ct& c_in, const std::vector<int>& steps) {
        std::vector<Ct> out(steps.size());
        if (vis_npoly(c_in) != 2) throw std::runtime_error("rotation/conjugation expects a 2-polynomial ciphertext");
        Ct c = normalize(c_in);
        const long sc = slot_count();
        int nrot = 0;
        for (int st : steps) nrot += (((long)st % sc + sc) % sc) != 0;
        if (c.nb != 1 || nrot < 2 || !batch_ops_) {
            for (size_t i = 0; i < steps.size(); ++i) out[i] = rotate(c, steps[i]);
            if (c.data != c_in.data) release(c);
            return out;
        }
        const int l = c.level, nl = hp_.nl(l), ne = nl + hp_.n_p, n = hp_.n;
        const u32* c1 = c.data + (size_t)nl * n;
        u32* ext = modup(c1, l, 1, 0);
        for (size_t i = 0; i < steps.size(); ++i) {
            if ((((long)steps[i] % sc + sc) % sc) == 0) {
                out[i] = copy(c);
                continue;
            }
            const u64 g = rot_galois(steps[i]);
            u32* acc = tmp(2 * (size_t)ne);
            key_inner(acc, ext, c1, ksk(g), l, g);
            u32* p0 = tmp(nl);
            launch_automorph(S(), T_, p0, c.data, g, nl);
            out[i] = moddown(acc, l, p0, nullptr);
            untmp(p0, nl);
            untmp(acc, 2 * (size_t)ne);
            cnt_[C_ROT]++;
            cnt_[C_KS]++;
            tally(LV_KS, l, 1);
        }
        untmp(ext, ext_rows(l));
        if (c.data != c_in.data) release(c);
        return out;
    }
    Ct rotate(const Ct& c, int steps) {
        const long s = slot_count();
        if (((long)steps % s + s) % s == 0) return copy(c);
        cnt_[C_ROT]++;
        return galois(c, rot_galois(steps));
    }
    Ct conjugate(const Ct& c) {
        cnt_[C_CONJ]++;
        if (lazy_galois_ok(c)) return galois_lazy(c, conj_galois());
        return galois(c, conj_galois());
    }

    // x^k at depth ceil(log2 k): x^(2^i) by squaring, x^k = x^(2^t) x^(k - 2^t)
    void power_basis(aesfhe_handle h, int degree, aesfhe_handle* out) {
        const Ct& x = canon(h);
        if (pm(x) != 2) throw std::runtime_error("make_power_basis expects a 2-polynomial ciphertext");
        if (degree < 1) throw std::runtime_error("power basis degree must be >= 1");
        int depth = 0;
        while ((1 << depth) < degree) ++depth;
        if (x.level < depth)
            throw std::runtime_error("not enough level for make_power_basis: need " + std::to_string(depth) + ", have level " +
                                     std::to_string(x.level));
        std::vector<aesfhe_handle> pw(degree + 1, 0);
        pw[1] = put_ct(copy(x));
        // x^k = x^h x^(k - h), h the largest power of two below k; the products of one depth
        // (k in (h, 2h]) only read lower depths, so each depth is one mul_many batch
        for (int h = 1; h < degree; h *= 2) {
            const int hi = std::min(2 * h, degree);
            for (int k0 = h + 1; k0 <= hi; k0 += kMaxMembers) {
                std::vector<const Ct*> A, B;
                const int k1 = std::min(hi, k0 + kMaxMembers - 1);
                for (int k = k0; k <= k1; ++k) {
                    A.push_back(&ct(pw[h]));
                    B.push_back(&ct(pw[k - h]));
                }
                std::vector<Ct> r = mul_many(A, B);
                for (int k = k0; k <= k1; ++k) pw[k] = put_ct(r[k - k0]);
            }
        }
        for (int k = 1; k <= degree; ++k) out[k - 1] = pw[k];
    }

    // CRT limbs (2..4) covering raw_scale * 2^26, or 0 when 4 are not enough
    int crt_limbs(const Ct& c) const {
        const int nl = hp_.nl(c.level);
        const double need = c.level >= 0 ? std::log2(raw_scale(c.level, c.pend)) + 26.0 : 0.0;
        int kd = std::min(2, nl);
        double have = 0.0;
        for (int i = 0; i < kd; ++i) have += std::log2((double)hp_.mod[i]);
        while (have < need && kd < std::min(4, nl)) have += std::log2((double)hp_.mod[kd++]);
        return have >= need ? kd : 0;
    }
    const CrtConsts& crt_consts(int kd) {
        CrtConsts& cc = crt_[kd - 1];
        if (cc.q[0]) return cc;
        double P = 1.0;
        for (int i = 0; i < kd; ++i) {
            const u32 qi = hp_.mod[i];
            cc.q[i] = qi;
            cc.pd[i] = P;
            u64 pm = 1;
            for (int j = 0; j < i; ++j) {
                cc.p_mod[i][j] = (u32)pm;
                pm = pm * (hp_.mod[j] % qi) % qi;
            }
            cc.minv[i] = i ? hinvm((u32)pm, qi) : 1;
            P *= (double)qi;
        }
        return cc;
    }
    // s^2 on the first four limbs (NTT form), for decrypting deferred 3-polynomial tensors
    const u32* s_sq4() {
        if (!d_s2_) {
            d_s2_ = dev_alloc((size_t)4 * hp_.n);
            launch_square(S(), T_, d_s2_, d_s_, std::min(4, hp_.n_tot()), 4, qmap());
            HIP_OK(hipStreamSynchronize(S()));
        }
        return d_s2_;
    }

    // secret-key Zeta16 renorm of a state pair (REF/pipeline.py:65-69, REF/state_encoder.py:17-38),
    // entirely on the device: raw decryption of both tensors on 2..4 limbs, mixed-radix CRT,
    // the 16 state slots evaluated directly, snap to the nearest zeta16 power, closed-form
    // re-encoding (every other slot 1) and fresh encryption -- no host round trip
    //
    // states > 1 is the slot-packed layout: state b of the
    // batch holds byte i in slot i * stride + b, so every slot with (j mod stride) < states is
    // snapped and the rest are reset to 1.  The whole slot vector is decoded and re-encoded
    // with a device fp64 FFT (launch_fft2); states == 1 keeps the 16-slot direct evaluation.
    //
    // level >= 0 re-encrypts at min(level, fresh) instead of the fresh level:
    // callers that know what the next step needs save the limbs
    void renorm_pair(aesfhe_handle hh, aesfhe_handle hl, aesfhe_handle* oh, aesfhe_handle* ol) { renorm_states(hh, hl, 1, oh, ol); }
    // period > 0: the periodic layout (slot j == slot j mod period, state_encoder.SlotLayout):
    // period 16 decodes / re-encodes its 16 slots directly (5^i positions), other periods snap
    // every slot (states = slot_count / 16)
    //
    // unpack = n > 0: hh is a packed state (hi | lo halves of every 2n-slot block, the
    // pipeline's packed XOR stage) and hl must be hh; oh / ol get its hi / lo halves as
    // n-periodic states.  single: hh == hl, one output (ol untouched) with every slot snapped.
    // single with packed_period = 32 (the packed XOR stage's hi | lo form, period 2 x 16): the
    // 32 slots are decoded / re-encoded directly (decode32 / encode32, no FFT); unpack = 16 likewise
    // hc (packed / single renorms): the renorm of hh + conj(hc) -- a conjugate-split LUT's S1 + conj(S2)
    //  renormalised without its conjugation key switch: both are decrypted in the
    // one raw-decryption launch and conj(m2) is the automorphism X -> X^-1 of the NTT-form m2, added
    // on the CRT limbs before the codec.  Inputs that do not share (level, owed rescales, shape) are
    // summed homomorphically first (same result).
    // hcl: the lo channel's partner of a pair renorm (hl + conj(hcl)), hc then the hi channel's.
    // pack_out (pair, period 16): ONE output, the snapped hi | lo pair in the packed period-32 form
    // (StateEncoder.pack's layout) -- the decode's two 16-slot channels are the 32 packed slots in
    // order, so the encode is the packed renorm's (no mask products, no level for the pack).
    void renorm_states(aesfhe_handle hh, aesfhe_handle hl, int states, aesfhe_handle* oh, aesfhe_handle* ol, int level = -1,
                       int period = 0, int unpack = 0, bool single = false, int packed_period = 0, aesfhe_handle hc = 0,
                       aesfhe_handle hcl = 0, bool pack_out = false, const int* slot_perm = nullptr) {
        if (!d_pk_) throw std::runtime_error("keys not generated");
        // slot_perm (pair, period 16): output slot i takes input slot slot_perm[i] -- a byte
        // permutation such as ShiftRows folded into the renorm: the decode reads each output slot's
        // value through the permuted root table, the encode writes slot i (no rotation, no level)
        if (slot_perm) {  // a period-16 pair, or the unpacking renorm of one packed period-16 pair
            const bool pair16 = !unpack && !single && period == 16, unpack16 = unpack == 16 && !single;
            if (!(pair16 || unpack16) || ct(hh).nb > 1 || ct(hl).nb > 1)
                throw std::runtime_error("renorm: a slot permutation needs a single period-16 state pair");
            for (int i = 0; i < 16; ++i)
                if (slot_perm[i] < 0 || slot_perm[i] > 15) throw std::runtime_error("renorm: slot permutation entries must lie in [0, 16)");
            // checked before any temporary is taken or launch issued
            if (unpack16 && !direct32_) throw std::runtime_error("renorm: a slot permutation needs the direct period-32 codec");
        }
        if (pack_out && (unpack || single || period != 16 || ct(hh).nb > 1 || ct(hl).nb > 1))
            throw std::runtime_error("renorm: the packed output needs a single period-16 state pair");
        if (hc || hcl) {
            const bool one = unpack || single;
            if (one ? (hl != hh || hcl) : (!hc || !hcl)) throw std::runtime_error("renorm: conjugate partners: one per input channel");
            auto same = [&](const Ct& a, const Ct& b) {
                return a.nb == 1 && b.nb == 1 && a.level == b.level && a.pend == b.pend && vis_npoly(a) == vis_npoly(b) && a.npoly == b.npoly &&
                       a.lazy == b.lazy && !a.zero && !b.zero;
            };
            if (!same(ct(hh), ct(hc)) || (!one && !same(ct(hl), ct(hcl)))) {
                auto summed = [&](aesfhe_handle a, aesfhe_handle b) {
                    Ct cj = conjugate(ct(b));
                    Ct sm = add_sub(ct(a), cj, false);
                    release(cj);
                    return put_ct(sm);
                };
                const aesfhe_handle th = summed(hh, hc), tl = one ? th : summed(hl, hcl);
                try {
                    renorm_states(th, tl, states, oh, ol, level, period, unpack, single, packed_period, 0, 0, pack_out, slot_perm);
                } catch (...) {
                    free_handle(th);
                    if (tl != th) free_handle(tl);
                    throw;
                }
                free_handle(th);
                if (tl != th) free_handle(tl);
                return;
            }
        }
        if (unpack || single) {
            if (hl != hh) throw std::runtime_error("renorm: a packed / single renorm reads one ciphertext");
            if (unpack && (unpack & (unpack - 1) || unpack < 16 || 2 * unpack > slot_count()))
                throw std::runtime_error("renorm: bad packed period");
            period = 0;
            states = slot_count() / 16;  // every slot snapped (FFT codec)
        }
        if (period > 0) {
            if (period & (period - 1) || period < 16 || period > slot_count()) throw std::runtime_error("renorm: bad period");
            states = period == 16 ? 1 : slot_count() / 16;
        }
        const bool per16 = period == 16;
        if (level > hp_.fresh) level = hp_.fresh;  // never above a fresh encryption
        const int n = hp_.n, s = slot_count(), stride = s / 16;
        if (states < 1 || states > stride)
            throw std::runtime_error("renorm: states per ciphertext must be in [1, slot_count / 16]");
        if (states > 1 || ct(hh).nb > 1) ensure_slot_pos();
        if (slots_.e[1] == 0) {
            const u64 two_n = 2ull * n;
            u64 e = 1;
            for (int j = 0; j < s; ++j) {
                if (j % stride == 0) slots_.e[j / stride] = (u32)e;
                if (j < 16) slots_p_.e[j] = (u32)e;
                if (j < 32) slots32_.e[j] = (u32)e;
                e = e * 5 % two_n;
            }
            for (int k = 0; k < kStreams; ++k) {
                d_codec_[k] = (double*)dev_alloc(2 * 64 * 2);  // two accumulators acc[64], or acc + w (AESFHE_SNAP_ENCODE=0)
                // zeroed on the stream the codec launches run on, ordered before the first decode
                // (hipMemset on the null stream does not order a hipStreamNonBlocking stream); from
                // then on each snapping encode zeroes the other accumulator (kernels.h launch_decode16 / 32)
                HIP_OK(hipMemsetAsync(d_codec_[k], 0, 2 * 64 * sizeof(double), S()));
                HIP_OK(hipStreamSynchronize(S()));
                d_nib_[k] = (int*)dev_alloc(32);
            }
        }
        const int P = ct(hh).nb;
        if (P > 1 || ct(hl).nb > 1) {
            if (ct(hl).nb != P) throw std::runtime_error("renorm: hi and lo stacks of different sizes");
            renorm_stacked(hh, hl, period == 16 ? stride : states, oh, ol, level, unpack, single);
            return;
        }
        u32* x = tmp(8);  // [2][4][N]
        int kd[2];
        CrtConsts cc[2];
        double isc[2];
        const aesfhe_handle in[2] = {hh, (hc && (unpack || single)) ? hc : hl};
        // unpack / single read ONE ciphertext: it is decrypted once and the codec runs on one input
        // channel (k_snap_slots' unpack gathers both outputs from channel 0; single has one output);
        // a conjugate partner is decrypted as the second channel and folded into the first
        const int n_in = (unpack || single) ? 1 : 2, n_out = (single || pack_out) ? 1 : 2, n_dec = (hc && n_in == 1) ? 2 : n_in;
        kd[1] = 0;
        // raw decryption of the inputs: ONE launch forms c0 + c1 s (+ c2 s^2) on the CRT limbs of
        // both, one inverse NTT when their limb counts agree
        DecRaw dr;
        Ct dc[2];
        bool down[2] = {false, false};
        bool need_s2 = false;
        for (int w = 0; w < n_dec; ++w) {
            Ct c = ensure_ntt(ct(in[w]));
            bool own = c.data != ct(in[w]).data;
            kd[w] = crt_limbs(c);
            if (!kd[w]) {
                Ct nc = normalize(c, true);
                if (own) release(c);
                c = nc, own = nc.data != ct(in[w]).data;
                kd[w] = crt_limbs(c);
            }
            dc[w] = c, down[w] = own;
            dr.ct[w] = c.data, dr.npoly[w] = c.npoly, dr.nlc[w] = hp_.nl(c.level), dr.kd[w] = kd[w];
            need_s2 = need_s2 || c.npoly == 3;
            cc[w] = crt_consts(kd[w]);
            isc[w] = 1.0 / (c.level >= 0 ? raw_scale(c.level, c.pend) : 1.0);
            cnt_[C_DEC]++;
        }
        // the sparse decryption (round 6, AESFHE_SPARSE_DEC, default on with the pool): the packed period-32
        // renorm and the periodic pair renorm decode only the D subring coefficients the snapped message can
        // have (launch_renorm_sparse: block sums of c0 + c1 s, a D-point inverse transform, the CRT, the
        // slots, the snap and the message's NTT table in TWO launches), then the pooled re-encryption: three
        // launches for the whole renorm instead of six (dec_raw, the INTT's two passes, decode, table, combine)
        {
            const int fs = level < 0 ? hp_.fresh : level;
            const bool one = direct32_ && single && packed_period == 32 && n_in == 1 && n_out == 1;
            const bool two = states == 1 && per16 && !pack_out && !unpack && !single && n_in == 2 && n_out == 2;
            if (sparse_dec_ && pool_k_ > 0 && !hc && !slot_perm && hp_.nl(fs) <= kRenormMaxLimbs && (one || two)) {
                SparseDec sd;
                for (int w = 0; w < n_in; ++w) sd.kd[w] = kd[w], sd.cc[w] = cc[w];
                u32* W = renorm_w();
                launch_renorm_sparse(S(), T_, W, renorm_b(), dr, n_in, sd, slots32_, slots_p_, hp_.delta[fs], hp_.nl(fs), gtab(one ? 64 : 32), d_s_,
                                     need_s2 ? s_sq4() : d_s_);
                for (int w = 0; w < n_dec; ++w)
                    if (down[w]) release(dc[w]);
                RenormOut ro;
                Ct outs[2];
                for (int c = 0; c < n_out; ++c) {
                    outs[c] = alloc_ct(fs, 2);
                    ro.pool[c] = zero_enc(fs);
                    ro.out[c] = outs[c].data;
                }
                launch_renorm_combine(S(), T_, ro, n_out, W, hp_.nl(fs), one ? 6 : 5);
                retire_pools();
                cnt_[C_ENC] += n_out;
                *oh = put_ct(outs[0]);
                if (n_out == 2) *ol = put_ct(outs[1]);
                untmp(x, 8);
                return;
            }
        }
        launch_dec_raw(S(), T_, x, dr, n_dec, d_s_, need_s2 ? s_sq4() : d_s_);
        if (hc && n_in == 1) {
            if (kd[1] != kd[0] || isc[1] != isc[0]) throw std::runtime_error("renorm: conjugate partner at another scale");
            u32* cj = tmp(kd[0]);
            launch_automorph(S(), T_, cj, x + (size_t)4 * n, conj_galois(), kd[0]);
            launch_add(S(), T_, x, x, cj, kd[0], kd[0], qmap());
            untmp(cj, kd[0]);
            cnt_[C_CONJ]++;
        } else if (hc) {  // pair: the partners of both channels in a second raw decryption
            DecRaw d2;
            Ct pc[2];
            bool pown[2] = {false, false}, ps2 = false;
            const aesfhe_handle ph[2] = {hc, hcl};
            for (int w = 0; w < 2; ++w) {
                Ct c = ensure_ntt(ct(ph[w]));
                bool own = c.data != ct(ph[w]).data;
                if (!crt_limbs(c)) {
                    Ct nc = normalize(c, true);
                    if (own) release(c);
                    c = nc, own = nc.data != ct(ph[w]).data;
                }
                if (crt_limbs(c) != kd[w] || 1.0 / (c.level >= 0 ? raw_scale(c.level, c.pend) : 1.0) != isc[w])
                    throw std::runtime_error("renorm: conjugate partner at another scale");
                pc[w] = c, pown[w] = own;
                d2.ct[w] = c.data, d2.npoly[w] = c.npoly, d2.nlc[w] = hp_.nl(c.level), d2.kd[w] = kd[w];
                ps2 = ps2 || c.npoly == 3;
            }
            u32* xc = tmp(8);
            launch_dec_raw(S(), T_, xc, d2, 2, d_s_, ps2 ? s_sq4() : d_s_);
            u32* cj = tmp(std::max(kd[0], kd[1]));
            for (int w = 0; w < 2; ++w) {
                launch_automorph(S(), T_, cj, xc + (size_t)w * 4 * n, conj_galois(), kd[w]);
                launch_add(S(), T_, x + (size_t)w * 4 * n, x + (size_t)w * 4 * n, cj, kd[w], kd[w], qmap());
                cnt_[C_CONJ]++;
            }
            untmp(cj, std::max(kd[0], kd[1]));
            untmp(xc, 8);
            for (int w = 0; w < 2; ++w)
                if (pown[w]) release(pc[w]);
        }
        if (n_in == 2 && kd[0] == kd[1]) {
            intt(x, x, 2 * kd[0], RowMap{kd[0], 4, 4, 0, 0}, qmap());
        } else {
            for (int w = 0; w < n_in; ++w) intt(x + (size_t)w * 4 * n, kd[w], kd[w], qmap());
        }
        for (int w = 0; w < n_dec; ++w)
            if (down[w]) release(dc[w]);
        const int f = level < 0 ? hp_.fresh : level, nq = hp_.nl(f) + 1;
        const double enc_scale = hp_.delta[f] * (double)hp_.mod[hp_.nl(f)];
        const bool direct32 = direct32_ && ((unpack == 16) || (single && packed_period == 32));
        // the re-encryption from this stream's pool of zero encryptions (zero_enc) where the snapped
        // message is sparse: the direct period-32 / period-16 codecs (pooled_ok)
        const bool pooled = pool_k_ > 0 && hp_.nl(f) <= kRenormMaxLimbs && (direct32 || (states == 1 && (pack_out || per16)));
        u32* m = pooled ? nullptr : tmp(2 * (size_t)nq);
        u32* W = pooled ? renorm_w() : nullptr;
        int ld = 0;  // log2 D of the pooled message
        // the snap inside the encode (AESFHE_SNAP_ENCODE, default on): the two accumulators of this
        // stream alternate -- this renorm decodes into one, its encode snaps from it and zeroes the other
        double* acc = d_codec_[t_sidx] + (snap_encode_ ? 64 * codec_flip_[t_sidx] : 0);
        double* zacc = snap_encode_ ? d_codec_[t_sidx] + 64 * (1 - codec_flip_[t_sidx]) : nullptr;
        double* wv = snap_encode_ ? acc : d_codec_[t_sidx] + 64;
        if (slot_perm && unpack && !direct32) throw std::runtime_error("renorm: a slot permutation needs the direct period-32 codec");
        // the message's NTT table instead of its coefficients (pooled): 32 slots of one channel (D = 64),
        // or 16 periodic slots of each of two channels (D = 32)
        auto wtab = [&](bool one32, const Slot16& s16) {
            if (one32) launch_renorm_wtab32(S(), T_, W, wv, zacc, slots32_, hp_.delta[f], hp_.nl(f), gtab(64)), ld = 6;
            else launch_renorm_wtab16(S(), T_, W, wv, zacc, s16, hp_.delta[f], hp_.nl(f), gtab(32)), ld = 5;
        };
        if (direct32) {
            // the 32 slots of the packed period-32 state: one direct decode, the snap as 2 x 16, and
            // either the two 16-periodic halves (unpack) or the 32-periodic whole (single); a slot
            // permutation applies within each 16-slot half (hi, lo)
            Slot32 sp32 = slots32_;
            if (slot_perm)
                for (int j = 0; j < 32; ++j) sp32.e[j] = slots32_.e[16 * (j / 16) + slot_perm[j % 16]];
            launch_decode32(S(), T_, x, kd[0], cc[0], sp32, isc[0], acc);
            if (!snap_encode_) launch_snap16(S(), acc, wv, d_nib_[t_sidx]);
            if (pooled) wtab(!unpack, slots_p_);
            else if (unpack) launch_encode16(S(), T_, m, wv, slots_p_, enc_scale, nq, true, zacc);
            else launch_encode32(S(), T_, m, wv, slots32_, enc_scale, nq, zacc);
            if (snap_encode_) codec_flip_[t_sidx] ^= 1;
        } else if (states == 1) {
            const Slot16& sl = per16 ? slots_p_ : slots_;
            Slot16 sp = sl;
            if (slot_perm)
                for (int i = 0; i < 16; ++i) sp.e[i] = sl.e[slot_perm[i]];
            launch_decode16(S(), T_, x, kd, cc, sp, isc, acc);
            if (!snap_encode_) launch_snap16(S(), acc, wv, d_nib_[t_sidx]);
            if (pooled) wtab(pack_out, sl);
            else if (pack_out) launch_encode32(S(), T_, m, wv, slots32_, enc_scale, nq, zacc);  // acc[c][i] = packed slot 16 c + i
            else launch_encode16(S(), T_, m, wv, sl, enc_scale, nq, per16, zacc);
            if (snap_encode_) codec_flip_[t_sidx] ^= 1;
        } else {
            double*& zbuf = d_fft_[t_sidx];
            if (!zbuf) zbuf = (double*)dev_alloc((size_t)2 * 2 * 2 * 2 * n);  // 2 buffers x [2][N] complex double
            double* z = zbuf;
            double* w = zbuf + (size_t)2 * 2 * n;
            if (n_in == 1) cc[1] = cc[0], isc[1] = isc[0];
            launch_decode_twist(S(), T_, x, kd, cc, isc, z, n_in);
            launch_fft2(S(), T_, z, 1, n_in);
            launch_snap_slots(S(), T_, z, w, d_slot_pos_, states, unpack, n_out);
            launch_fft2(S(), T_, w, -1, n_out);
            launch_encode_untwist(S(), T_, m, w, enc_scale, nq, n_out);
        }
        if (pooled) {
            // out_c = a pooled encryption of zero at level f + the message's NTT (one launch for both)
            RenormOut ro;
            Ct outs[2];
            for (int c = 0; c < n_out; ++c) {
                outs[c] = alloc_ct(f, 2);
                ro.pool[c] = zero_enc(f);
                ro.out[c] = outs[c].data;
            }
            launch_renorm_combine(S(), T_, ro, n_out, W, hp_.nl(f), ld);
            retire_pools();
            cnt_[C_ENC] += n_out;
            *oh = put_ct(outs[0]);
            if (n_out == 2) *ol = put_ct(outs[1]);
            untmp(x, 8);
            return;
        }
        // both re-encryptions in one set of launches, the coefficient-form message added to e0
        Ct enc = encrypt_many(m, n_out, (size_t)nq * n, f, true);
        if (n_out == 1) {
            enc.nb = 1;
            *oh = put_ct(enc);
        } else {
            Ct parts[2];
            const int idx[2] = {0, 1};
            unstack(enc, parts, idx);
            release(enc);
            *oh = put_ct(parts[0]);
            *ol = put_ct(parts[1]);
        }
        untmp(m, 2 * (size_t)nq);
        untmp(x, 8);
    }

    // ---- pooled zero encryptions for the renorm (AESFHE_RENORM_POOL = K per refill, default 16; 0: every
    // renorm encrypts its own message, the round-5 path).  A refill is ONE encrypt_many of K zero
    // messages at level f (the same sampling, NTT, combine and rescale launches as one renorm's
    // encryption, K members wide); each member is handed out once (its own PRNG counter: fresh v, e0, e1),
    // and the renorm adds its message's NTT (k_renorm_combine).  Pools are per stream (the refill, the
    // consumers and the slab's release stay stream-ordered) and per level; aesfhe_renorm_pool resets them
    // (bench.py empties them before its timed region: every encryption used there is made there).
    int pool_k_ = env_int("AESFHE_RENORM_POOL", 16);
    struct ZPool {
        Ct slab;
        int next = 0;
    };
    std::map<int, ZPool> zpool_[kStreams];
    std::vector<Ct> zretired_[kStreams];
    std::map<int, u32*> gtab_;
    u32* renorm_w_[kStreams] = {};
    u32* renorm_b_[kStreams] = {};
    bool sparse_dec_ = env_int("AESFHE_SPARSE_DEC", 1) != 0;
    u32* renorm_b() {  // [2][4][64] block sums of the sparse decryption
        u32*& b = renorm_b_[t_sidx];
        if (!b) b = dev_alloc((size_t)2 * 4 * 64);
        return b;
    }
    u32* renorm_w() {
        u32*& w = renorm_w_[t_sidx];
        if (!w) w = dev_alloc((size_t)2 * kRenormMaxLimbs * 64);
        return w;
    }
    // [t][e] = g_t^e, g_t = psi_t^(N / D) (a primitive 2D-th root mod q_t), e < 2D, every Q prime
    const u32* gtab(int D) {
        auto it = gtab_.find(D);
        if (it != gtab_.end()) return it->second;
        const int nq = hp_.n_q;
        std::vector<u32> h((size_t)nq * 2 * D);
        for (int t = 0; t < nq; ++t) {
            const u64 q = hp_.mod[t];
            u64 g = 1, b = hp_.psi[t];
            for (u64 e = (u64)hp_.n / D; e; e >>= 1, b = b * b % q)
                if (e & 1) g = g * b % q;
            u64 v = 1;
            for (int e = 0; e < 2 * D; ++e, v = v * g % q) h[(size_t)t * 2 * D + e] = (u32)v;
        }
        u32* d = dev_alloc(h.size());
        HIP_OK(hipMemcpy(d, h.data(), sizeof(u32) * h.size(), hipMemcpyHostToDevice));
        return gtab_[D] = d;
    }
    const u32* zero_enc(int f) {
        ZPool& zp = zpool_[t_sidx][f];
        if (!zp.slab.data || zp.next >= zp.slab.nb) {
            if (zp.slab.data) zretired_[t_sidx].push_back(zp.slab);  // released after this renorm's launches
            zp.slab = encrypt_many(nullptr, pool_k_, 0, f, true);
            zp.next = 0;
        }
        return zp.slab.data + (size_t)(zp.next++) * 2 * hp_.nl(f) * hp_.n;
    }
    void retire_pools() {
        for (const Ct& c : zretired_[t_sidx]) release(c);
        zretired_[t_sidx].clear();
    }
    void renorm_pool(int k) {  // k < 0: keep the size, empty the pools
        if (k > 4096) throw std::runtime_error("renorm_pool: size above 4096");
        HIP_OK(hipDeviceSynchronize());
        for (int s = 0; s < kStreams; ++s) {
            for (auto& kv : zpool_[s])
                if (kv.second.slab.data) pools_[s].put(kv.second.slab.data, kv.second.slab.words);
            zpool_[s].clear();
            for (const Ct& c : zretired_[s]) pools_[s].put(c.data, c.words);
            zretired_[s].clear();
        }
        if (k >= 0) pool_k_ = k;
    }

    // NTT position of every slot (5^j mod 2N -> (e - 1) / 2), for the FFT codec
    void ensure_slot_pos() {
        if (d_slot_pos_) return;
        const int n = hp_.n, s = slot_count();
        std::vector<u32> pos(s);
        const u64 two_n = 2ull * n;
        u64 e = 1;
        for (int j = 0; j < s; ++j) pos[j] = (u32)((e - 1) / 2), e = e * 5 % two_n;
        d_slot_pos_ = dev_alloc(s);
        HIP_OK(hipMemcpy(d_slot_pos_, pos.data(), sizeof(u32) * s, hipMemcpyHostToDevice));
    }
    // the renorm of P stacked state pairs (multi-pair batches): every member's
    // channels in ONE set of launches -- one raw decryption, one inverse NTT, the fp64 FFT codec
    // over all n_in P channels (states = the slots snapped per 16-slot row, as renorm_states), one
    // encryption of all n_out P messages -- and the outputs as stacks again (hi = members
    // [0, P), lo = [P, 2P) of the encryption).  Same snapped values as P single renorms.
    void renorm_stacked(aesfhe_handle hh, aesfhe_handle hl, int states, aesfhe_handle* oh, aesfhe_handle* ol, int level, int unpack,
                        bool single) {
        const int n = hp_.n, P = ct(hh).nb;
        const int n_in = (unpack || single) ? 1 : 2, n_out = single ? 1 : 2;
        int kd[2] = {0, 0};
        CrtConsts cc[2];
        double isc[2] = {1.0, 1.0};
        DecRaw dr;
        dr.members = P;
        Ct dc[2];
        bool down[2] = {false, false}, need_s2 = false;
        const aesfhe_handle in[2] = {hh, hl};
        for (int w = 0; w < n_in; ++w) {
            Ct c = ensure_ntt(ct(in[w]));
            bool own = c.data != ct(in[w]).data;
            kd[w] = crt_limbs(c);
            if (!kd[w]) {
                Ct nc = normalize(c, true);
                if (own) release(c);
                c = nc, own = nc.data != ct(in[w]).data;
                kd[w] = crt_limbs(c);
            }
            dc[w] = c, down[w] = own;
            dr.ct[w] = c.data, dr.npoly[w] = pm(c), dr.nlc[w] = hp_.nl(c.level), dr.kd[w] = kd[w];
            dr.ms[w] = (size_t)pm(c) * hp_.nl(c.level) * n;
            need_s2 = need_s2 || pm(c) == 3;
            cc[w] = crt_consts(kd[w]);
            isc[w] = 1.0 / (c.level >= 0 ? raw_scale(c.level, c.pend) : 1.0);
            cnt_[C_DEC] += P;
        }
        if (n_in == 1) kd[1] = kd[0], cc[1] = cc[0], isc[1] = isc[0];
        const int chin = n_in * P, chout = n_out * P;
        u32* x = tmp((size_t)4 * chin);  // [channel][4][N]
        launch_dec_raw(S(), T_, x, dr, n_in, d_s_, need_s2 ? s_sq4() : d_s_);
        if (kd[0] == kd[1] || n_in == 1) {
            intt(x, x, chin * kd[0], RowMap{kd[0], 4, 4, 0, 0}, qmap());
        } else {
            for (int w = 0; w < n_in; ++w) intt(x + (size_t)w * P * 4 * n, x + (size_t)w * P * 4 * n, P * kd[w], RowMap{kd[w], 4, 4, 0, 0}, qmap());
        }
        for (int w = 0; w < n_in; ++w)
            if (down[w]) release(dc[w]);
        ensure_slot_pos();
        const int f = level < 0 ? hp_.fresh : level, nq = hp_.nl(f) + 1;
        const double enc_scale = hp_.delta[f] * (double)hp_.mod[hp_.nl(f)];
        // fp64 codec buffers: a complex double is 4 words, so a channel of N values is 4 rows
        u32* zb = tmp((size_t)4 * chin);
        u32* wb = tmp((size_t)4 * chout);
        double* z = (double*)zb;
        double* wv = (double*)wb;
        launch_decode_twist(S(), T_, x, kd, cc, isc, z, chin, P);
        launch_fft2(S(), T_, z, 1, chin);
        launch_snap_slots(S(), T_, z, wv, d_slot_pos_, states, unpack, chout, P);
        launch_fft2(S(), T_, wv, -1, chout);
        u32* m = tmp((size_t)chout * nq);
        launch_encode_untwist(S(), T_, m, wv, enc_scale, nq, chout);
        untmp(zb, (size_t)4 * chin);
        untmp(wb, (size_t)4 * chout);
        untmp(x, (size_t)4 * chin);
        Ct enc = encrypt_many(m, chout, (size_t)nq * n, f, true);
        untmp(m, (size_t)chout * nq);
        if (n_out == 1) {
            *oh = put_ct(enc);
            return;
        }
        *oh = put_ct(members_of(enc, 0, P));
        *ol = put_ct(members_of(enc, P, P));
        release(enc);
    }

    // ------------------------------------------------------------------ bootstrapping
    static constexpr int kBootStc = 3, kSparseH = 32;
    // EvalMod: range K (|I| < K), r double angles, Chebyshev degree (AESFHE_BOOT_K / _R / _DEG
    // override, for sweeps; read once per process).  Degree 23 (27 until round 5): the same depth and
    // the same measured error (full-slot 2.1-2.5e-4 max against 2.2-2.8e-4; the interpolation error
    // 5e-15 against 3e-15) with fewer leaf terms, C2 +1.8 % (profiles/r5_boot_deg_ab.txt); 19 was 10x
    // less accurate, 15 failed
    static int env_int(const char* name, int dflt) {
        const char* e = std::getenv(name);
        return e ? std::atoi(e) : dflt;
    }
    static int boot_k() { static const int v = env_int("AESFHE_BOOT_K", 12); return v; }
    static int boot_r() { static const int v = env_int("AESFHE_BOOT_R", 4); return v; }
    static int boot_deg() { static const int v = env_int("AESFHE_BOOT_DEG", 23); return v; }
    // CoeffToSlot groups (one double-prime level each; AESFHE_BOOT_CTS overrides, for sweeps)
    static int boot_cts() {
        static const int v = std::getenv("AESFHE_BOOT_CTS") ? std::atoi(std::getenv("AESFHE_BOOT_CTS")) : 3;
        return v;
    }
    // message bits b: s_bt = Q0 / 2^b (AESFHE_BOOT_MSG_BITS overrides, for accuracy sweeps)
    int boot_msg_bits_ = std::getenv("AESFHE_BOOT_MSG_BITS") ? std::atoi(std::getenv("AESFHE_BOOT_MSG_BITS")) : 9;
    // depth of cheb_eval for a degree-d series: baby T_k at ceil(log2 k), a leaf one more
    // (its scalar products), giant T_m at log2 m, p = q + T_m r at max(q, 1 + max(T_m, r))
    static int cheb_depth(int d) {
        auto clog2 = [](int k) { int e = 0; while ((1 << e) < k) ++e; return e; };
        if (d <= kBabyDeg) return clog2(std::max(d, 1)) + 1;
        int m = kBabyDeg;
        while (2 * m <= d) m *= 2;
        return std::max(cheb_depth(m - 1), 1 + std::max(clog2(m), cheb_depth(d - m)));
    }
    static int boot_evalmod_depth() { return cheb_depth(boot_deg()) + boot_r(); }
    static int boot_depth() { return boot_cts() + boot_evalmod_depth() + kBootStc; }
    // double-prime levels: CoeffToSlot + EvalMod + the region-crossing first SlotToCoeff group
    static int boot_double_levels() { return boot_cts() + boot_evalmod_depth() + 1; }
    u64 tag_d2s() const { return 2ull * hp_.n + 1; }
    u64 tag_s2d() const { return 2ull * hp_.n + 3; }

    // ephemeral sparse ternary secret (h = 32): positions and signs from PRNG stream 9 (host)
    std::vector<int> sparse_coeffs() const {
        std::vector<int> s(hp_.n, 0);
        int cnt = 0;
        for (u64 ctr = 0; cnt < kSparseH; ++ctr) {
            const u64 r = chacha_u64(pkey(), stream_id(9, 0, 0), ctr);
            const u64 pos = r % (u64)hp_.n;
            if (s[pos] == 0) {
                s[pos] = (r >> 63) ? -1 : 1;
                ++cnt;
            }
        }
        return s;
    }
    const u32* sparse_secret() {
        if (d_ssp_) return d_ssp_;
        const int n = hp_.n, nt = hp_.n_tot();
        const std::vector<int> s = sparse_coeffs();
        std::vector<u32> h((size_t)nt * n);
        for (int t = 0; t < nt; ++t)
            for (int k = 0; k < n; ++k) h[(size_t)t * n + k] = s[k] >= 0 ? (u32)s[k] : hp_.mod[t] - 1;
        d_ssp_ = dev_alloc((size_t)nt * n);
        HIP_OK(hipMemcpy(d_ssp_, h.data(), h.size() * sizeof(u32), hipMemcpyHostToDevice));
        ntt(d_ssp_, nt, nt, qmap());
        HIP_OK(hipStreamSynchronize(S()));
        return d_ssp_;
    }

    struct BootGroupDev {
        const LinGroup* g = nullptr;
        std::map<int, std::vector<std::vector<u32*>>> pts;  // level -> [giant][baby] encoded diagonals
        // compact diagonals (group_pts): log2 of the run length s of equal NTT values and of the
        // 2 dn values per limb; 0 = full rows
        int c_shift = 0, c_logc = 0;
    };
    struct BootState {
        bool ready = false;
        BootPlan plan;
        int top = 0;
        double s_bt = 0.0;  // message scale of the level-0 (mod Q0 = q0 q1) ciphertext
        i64 k1 = 0;         // integer factor taking delta_0 to s_bt
        std::vector<BootGroupDev> cts, stc;
    } bs_;
    // sparse-slot bootstrap of an n-periodic message (slot j == slot j mod n):
    // the message lies in the subring Z[X^(N/2n)], the ring of dimension 2n with n slots, so
    // after ModRaise a trace (log2(M/n) rotations by n 2^i, summed) removes the overflow's
    // components outside that subring and CoeffToSlot / SlotToCoeff are the small ring's
    // transforms (log2 n stages), their diagonals tiled with period n
    struct SparseBoot {
        int n = 0, top = 0, out_level = 0;
        bool packed = false;  // real / imaginary halves in one 2n-periodic ciphertext (one EvalMod)
        bool pair4 = false;   // pair bootstraps: hi and lo as well, 4n-periodic (one EvalMod for both)
        BootPlan plan;
        std::vector<BootGroupDev> cts, stc;
        BootGroupDev stc_lo;  // pair4: the lo member's form of stc[0]
    };
    std::map<int, SparseBoot> sparse_;  // key n (single / unpacked pair), -n (pair4)
    bool trace4_ = std::getenv("AESFHE_TRACE4") ? std::atoi(std::getenv("AESFHE_TRACE4")) != 0 : true;
    // x + rot(x, -a) + rot(x, -2a) + rot(x, -3a) for the nb members of x: the three rotations
    // hoisted (one ModUp of c1, key inner products read through each automorphism) and summed
    // in Q*P (one ModDown adding c0 + the permuted c0s and c1) -- two trace doublings for ~1.5
    // rotations' work
    Ct trace4(const Ct& x_in, int a) {
        if (vis_npoly(x_in) != 2) throw std::runtime_error("trace4: 2-polynomial ciphertext expected");
        Ct x = normalize(x_in);
        const int l = x.level, nl = hp_.nl(l), ne = nl + hp_.n_p, n = hp_.n, nb = x.nb;
        const size_t qs = (size_t)2 * nl * n;
        const u32* c1 = x.data + (size_t)nl * n;
        u32* ext = modup(c1, l, nb, qs);
        u32* acc = tmp(2 * (size_t)ne * nb);
        // the three rotations' key inner products summed in one launch, c0 + its three
        // automorphisms in another (bit for bit the separate launches' sums)
        KsSumArgs ka;
        ka.J = 3;
        for (int j = 1; j <= 3; ++j) ka.g[j - 1] = rot_galois(-j * a), ka.key[j - 1] = ksk(ka.g[j - 1]);
        const int nd = (nl + hp_.alpha - 1) / hp_.alpha;
        launch_key_inner_sum(S(), T_, acc, ext, c1, ka, nb, nd, ne, nl, hp_.alpha, hp_.n_ks + hp_.n_p, hp_.n_ks, extmap(nl),
                             (size_t)ext_rows(l) * n, qs, (size_t)2 * ne * n);
        untmp(ext, (size_t)nb * ext_rows(l));
        u32* c0s = tmp(2 * (size_t)nl * nb);  // member stride qs, first nl rows used (moddown's add0)
        launch_automorph_sum(S(), T_, c0s, x.data, ka, nb, nl, qs, qmap());
        Ct o = moddown(acc, l, c0s, c1, nb, qs);
        o.ntt = x.ntt;
        untmp(acc, 2 * (size_t)ne * nb);
        untmp(c0s, 2 * (size_t)nl * nb);
        if (x.data != x_in.data) release(x);
        cnt_[C_ROT] += 3 * nb;
        cnt_[C_KS] += 3 * nb;
        tally(LV_KS, l, 3 * nb);
        return o;
    }
    // The sparse -> dense switch fused into the first trace step (AESFHE_S2D_TRACE, default on):
    // raised (under s_sp) -> x + rot(x, -a) + rot(x, -2a) + rot(x, -3a) with x = raised switched to s.
    // The automorphism of raised decrypts under sigma(s_sp), so each of the four terms is ONE key
    // inner product from the same hoisted ModUp of raised's c1 (keys s_sp -> s and sigma_j(s_sp) -> s,
    // tag_s2d_rot) and the four share one ModDown: one ModUp and one ModDown at the top level fewer
    // than keyswitch(s2d) followed by trace4.  Same plaintext; the key-switch noise terms differ.
    bool s2d_trace_ = env_int("AESFHE_S2D_TRACE", 1) != 0;
    Ct s2d_trace4(const Ct& raised, int a) {
        const int l = raised.level, nl = hp_.nl(l), ne = nl + hp_.n_p, n = hp_.n, nb = raised.nb;
        const size_t qs = (size_t)2 * nl * n;
        const u32* c1 = raised.data + (size_t)nl * n;
        u32* ext = modup(c1, l, nb, qs);
        u32* acc = tmp(2 * (size_t)ne * nb);
        KsSumArgs ka;
        ka.J = 4;
        ka.g[0] = 1, ka.key[0] = ksk(tag_s2d());
        for (int j = 1; j <= 3; ++j) ka.g[j] = rot_galois(-j * a), ka.key[j] = ksk(tag_s2d_rot(ka.g[j]));
        const int nd = (nl + hp_.alpha - 1) / hp_.alpha;
        launch_key_inner_sum(S(), T_, acc, ext, c1, ka, nb, nd, ne, nl, hp_.alpha, hp_.n_ks + hp_.n_p, hp_.n_ks, extmap(nl),
                             (size_t)ext_rows(l) * n, qs, (size_t)2 * ne * n);
        untmp(ext, (size_t)nb * ext_rows(l));
        KsSumArgs kc;  // c0 + its three automorphisms
        kc.J = 3;
        for (int j = 1; j <= 3; ++j) kc.g[j - 1] = ka.g[j];
        u32* c0s = tmp(2 * (size_t)nl * nb);  // member stride qs, first nl rows used (moddown's add0)
        launch_automorph_sum(S(), T_, c0s, raised.data, kc, nb, nl, qs, qmap());
        Ct o = moddown(acc, l, c0s, nullptr, nb, qs);
        o.ntt = raised.ntt;
        untmp(acc, 2 * (size_t)ne * nb);
        untmp(c0s, 2 * (size_t)nl * nb);
        cnt_[C_ROT] += 3 * nb;
        cnt_[C_KS] += 4 * nb;
        tally(LV_KS, l, 4 * nb);
        return o;
    }
    SparseBoot& sparse_variant(int n, bool pair = false) {
        const char* p4 = std::getenv("AESFHE_SPARSE_PAIR4");  // "0": the pair keeps two EvalMod members (A/B)
        pair = pair && n <= 32 && !(p4 && std::atoi(p4) == 0);
        auto it = sparse_.find(pair ? -n : n);
        if (it != sparse_.end()) return it->second;
        const int M = slot_count();
        int logm = 0;
        while ((1 << logm) < n) ++logm;
        if ((1 << logm) != n || n < 16 || n >= M) throw std::runtime_error("sparse bootstrap: period must be a power of two in [16, slot_count)");
        SparseBoot& sv = sparse_[pair ? -n : n];
        sv.n = n;
        const int groups = std::max(1, (logm + 4) / 5);  // <= 5 butterfly stages per group, like the full plan
        // StC's first group crosses the single / double-prime transition (plaintext products only)
        sv.top = hp_.L1 + 1 + groups + boot_evalmod_depth();
        sv.out_level = hp_.L1 + 1 - groups;
        if (sv.top > hp_.L) throw std::runtime_error("sparse bootstrap: chain too short");
        const double Q0 = (double)hp_.mod[0] * (double)hp_.mod[1];
        // the trace multiplies by M / n: folded into CoeffToSlot
        const double cts_scale = hp_.delta[sv.top] / (2.0 * Q0 * boot_k() * ((double)M / n));
        const double stc_scale = Q0 / (2.0 * M_PI * bs_.s_bt);
        const int later = logm - (logm + groups - 1) / groups;
        const double boost = groups > 1 ? std::ldexp(1.0, later / 2) : 1.0;
        // packed form while the half-folded SlotToCoeff group stays small (offsets up to n + R)
        const char* pk = std::getenv("AESFHE_SPARSE_PACK");  // "0": two EvalMods (A/B)
        sv.packed = n <= 64 && !(pk && std::atoi(pk) == 0);
        sv.pair4 = pair && sv.packed;
        sv.plan = make_boot_plan(logm + 1, groups, groups, cts_scale, stc_scale, boot_k(), boot_r(), boot_deg(), boost,
                                 sv.pair4 ? 2 : sv.packed ? 1 : 0);
        sv.cts.assign(sv.plan.cts.size(), {});
        sv.stc.assign(sv.plan.stc.size(), {});
        for (size_t i = 0; i < sv.cts.size(); ++i) sv.cts[i].g = &sv.plan.cts[i];
        for (size_t i = 0; i < sv.stc.size(); ++i) sv.stc[i].g = &sv.plan.stc[i];
        sv.stc_lo.g = &sv.plan.stc_lo;
        return sv;
    }

    void boot_setup() {
        if (bs_.ready) return;
        if (hp_.L - hp_.L1 != boot_double_levels() || hp_.L - hp_.fresh < boot_depth())
            throw std::runtime_error("bootstrap needs the bootstrappable parameter set (use_bootstrap=True): chain has " +
                                     std::to_string(hp_.L - hp_.fresh) + " spare levels, need " + std::to_string(boot_depth()));
        bs_.top = hp_.L;
        // the bootstrap starts modulo Q0 = q0 q1 (level 0) with the message at s_bt = Q0 / 2^b
        const double Q0 = (double)hp_.mod[0] * (double)hp_.mod[1];
        bs_.k1 = std::llround(Q0 / std::ldexp(1.0, boot_msg_bits_) / hp_.delta[0]);
        bs_.s_bt = hp_.delta[0] * (double)bs_.k1;
        const double cts_scale = hp_.delta[bs_.top] / (2.0 * Q0 * boot_k());
        const double stc_scale = Q0 / (2.0 * M_PI * bs_.s_bt);
        // intermediate SlotToCoeff signal lifted by the later groups' butterfly gain,
        // 2^(stages after the first group / 2) (AESFHE_STC_BOOST overrides; 1 = off)
        const int later = (hp_.logn - 1) - (hp_.logn - 1 + kBootStc - 1) / kBootStc;
        const double boost = std::getenv("AESFHE_STC_BOOST") ? std::atof(std::getenv("AESFHE_STC_BOOST")) : std::ldexp(1.0, later / 2);
        bs_.plan = make_boot_plan(hp_.logn, boot_cts(), kBootStc, cts_scale, stc_scale, boot_k(), boot_r(), boot_deg(), boost);
        bs_.cts.assign(bs_.plan.cts.size(), {});
        bs_.stc.assign(bs_.plan.stc.size(), {});
        for (size_t i = 0; i < bs_.cts.size(); ++i) bs_.cts[i].g = &bs_.plan.cts[i];
        for (size_t i = 0; i < bs_.stc.size(); ++i) bs_.stc[i].g = &bs_.plan.stc[i];
        ksk(tag_d2s());
        ksk(tag_s2d());
        bs_.ready = true;
    }

    Ct rotl(const Ct& c, long k) { return rotate(c, (int)(-k)); }
    // debug: apply CoeffToSlot group `which` (0..2) or SlotToCoeff group (3..5)
    BootGroupDev& debug_group(int which) {
        boot_setup();
        if (which < 0 || which >= boot_cts() + kBootStc) throw std::runtime_error("debug_lin_group: no such group");
        return which < boot_cts() ? bs_.cts[which] : bs_.stc[which - boot_cts()];
    }
    Ct debug_lin_group(const Ct& c, int which) { return lin_group(c, debug_group(which)); }
    // the same for the sparse-slot plan of period n: CoeffToSlot groups first,
    // then SlotToCoeff (stc[0..], then -- pair4 plans -- stc_lo last)
    BootGroupDev& debug_sparse_group(int period, int which, bool pair = false) {
        boot_setup();
        SparseBoot& sv = sparse_variant(period, pair);
        const int nc = (int)sv.cts.size(), ns = (int)sv.stc.size();
        if (which < 0 || which >= nc + ns + (sv.pair4 ? 1 : 0)) throw std::runtime_error("debug_sparse_group: no such group");
        return which < nc ? sv.cts[which] : which < nc + ns ? sv.stc[which - nc] : sv.stc_lo;
    }
    // the group applied on the host: the plan is the small ring's (its diagonals one period dn
    // long), so it acts on the first dn slots of the (dn-periodic) input and the result is tiled
    // over all slots -- the model of debug_sparse_group on a periodic message
    void debug_sparse_group_plain(int period, int which, bool pair, const double* re, const double* im, double* ore, double* oim,
                                  int* info) {
        const LinGroup& g = *debug_sparse_group(period, which, pair).g;
        const SparseBoot& sv = sparse_variant(period, pair);
        info[1] = (int)sv.cts.size();
        info[2] = (int)(sv.cts.size() + sv.stc.size() + (sv.pair4 ? 1 : 0));
        int dn = 0;
        for (const auto& row : g.diag)
            for (const auto& d : row)
                if (!d.empty()) dn = (int)d.size();
        const int M = slot_count();
        if (dn <= 0 || M % dn) throw std::runtime_error("debug_sparse_group_plain: bad diagonal period");
        std::vector<cplx> v(dn);
        for (int j = 0; j < dn; ++j) v[j] = cplx(re[j], im[j]);
        v = apply_group_plain(g, v);
        for (int j = 0; j < M; ++j) ore[j] = v[j % dn].real(), oim[j] = v[j % dn].imag();
        info[0] = dn;
    }
    // the same group applied to slot values on the host (bootstrap.cpp apply_group_plain): the
    // model debug_lin_group's decryption is checked against
    void debug_lin_group_plain(int which, const double* re, const double* im, double* ore, double* oim) {
        const LinGroup& g = *debug_group(which).g;
        const int M = slot_count();
        std::vector<cplx> v(M);
        for (int j = 0; j < M; ++j) v[j] = cplx(re[j], im[j]);
        v = apply_group_plain(g, v);
        for (int j = 0; j < M; ++j) ore[j] = v[j].real(), oim[j] = v[j].imag();
    }
    void boot_info(double* out) const {
        out[0] = bs_.s_bt;
        out[1] = (double)bs_.k1;
        out[2] = bs_.top;
        out[3] = boot_k();
        out[4] = boot_r();
        out[5] = boot_deg();
        out[6] = d2s_modulus_bits();
        out[7] = kSparseH;
        out[8] = d2s_np();
        out[9] = kD2sQ;
        out[10] = boot_msg_bits_;
    }

    // diagonals of one group encoded at `level` (scale ptscale_level) on the Q limbs AND the
    // P block (nl + n_p rows): the hoisted baby steps are summed in Q*P (lin_group); cached
    std::vector<std::vector<u32*>>& group_pts(BootGroupDev& G, int level) {
        auto it = G.pts.find(level);
        if (it != G.pts.end()) return it->second;
        const LinGroup& g = *G.g;
        const int M = slot_count(), n = hp_.n;
        std::vector<std::vector<u32*>> P(g.G, std::vector<u32*>(g.B, nullptr));
        std::vector<double> re(M), im(M);
        std::vector<u32> host;
        // a sparse plan's diagonals are dn-periodic slot vectors (dn < M), i.e. elements of the
        // subring Z[X^s], s = N / (2 dn): their coefficients off the multiples of s are exactly 0
        // (the fp64 embedding leaves rounding noise there -- ~Delta 2^-52 -- which the projection
        // below removes).  In NTT form such an element takes the value p(psi^(s (2 brv(i) + 1))),
        // which depends on i only through its top log2(2 dn) bits: runs of s equal residues.
        // k_lin_mac then reads 2 dn words per limb (LinMacArgs::pt_shift) instead of N
        size_t dn0 = 0;
        bool same = true;
        for (int gg = 0; gg < g.G; ++gg)
            for (int b = 0; b < g.B; ++b)
                if (!g.diag[gg][b].empty()) {
                    if (!dn0) dn0 = g.diag[gg][b].size();
                    same = same && g.diag[gg][b].size() == dn0;
                }
        const bool tiled = same && dn0 && dn0 < (size_t)M && M % dn0 == 0, compact = tiled && compact_diag_;
        const size_t sr = tiled ? (size_t)n / (2 * dn0) : 1;
        if (compact) {
            int a = 0, c = 0;
            while (((size_t)1 << a) < sr) ++a;
            while (((size_t)1 << c) < 2 * dn0) ++c;
            G.c_shift = a, G.c_logc = c;
        }
        for (int gg = 0; gg < g.G; ++gg)
            for (int b = 0; b < g.B; ++b) {
                const auto& d = g.diag[gg][b];
                if (d.empty()) continue;
                const size_t dn = d.size();  // M, or n for a sparse plan (tiled with period n)
                for (int p = 0; p < M; ++p) re[p] = d[p % dn].real(), im[p] = d[p % dn].imag();
                const int nl = hp_.nl(level), ne = nl + hp_.n_p;
                encode_host(re.data(), im.data(), hp_.ptscale[level], nl, host, hp_.n_p);
                if (tiled)  // project onto the subring Z[X^s]
                    for (size_t x = 0; x < host.size(); ++x)
                        if ((x & (size_t)(n - 1)) % sr) host[x] = 0;
                u32* dv = tmp(ne);
                HIP_OK(hipMemcpyAsync(dv, host.data(), host.size() * sizeof(u32), hipMemcpyHostToDevice, S()));
                HIP_OK(hipStreamSynchronize(S()));
                ntt(dv, ne, ne, extmap(nl));
                if (compact) {  // one residue per run: [ne][2 dn]
                    u32* cv = dev_alloc((size_t)ne * 2 * dn0);
                    HIP_OK(hipMemcpy2DAsync(cv, sizeof(u32), dv, sr * sizeof(u32), sizeof(u32), (size_t)ne * 2 * dn0,
                                            hipMemcpyDeviceToDevice, S()));
                    HIP_OK(hipStreamSynchronize(S()));
                    untmp(dv, ne);
                    dv = cv;
                }
                P[gg][b] = dv;
            }
        HIP_OK(hipStreamSynchronize(S()));  // cached for every stream
        return G.pts.emplace(level, std::move(P)).first->second;
    }

    // one merged butterfly group, baby-step giant-step (bootstrap.h) with hoisted baby steps
    // (DESIGN.md §4): c1 is ModUp'ed ONCE; every baby rotation b is only a key inner product
    // read through X -> X^{g_b} (u_b, in Q*P) plus the automorphism of c0 (a_b).  Each giant
    // step sums its diagonals in Q*P and pays ONE ModDown:
    //   inner = ModDown(sum_b P_b u_b) + (sum_b P_b a_b, P_0 c1),  a_0 = c0,
    // then rescales and takes its giant rotation (a full key switch).
    Ct lin_group(const Ct& in, BootGroupDev& G) {
        const LinGroup& g = *G.g;
        const int l = in.level, nl = hp_.nl(l), np = hp_.n_p, ne = nl + np, n = hp_.n;
        if (g.B > kMacMax) throw std::runtime_error("lin_group: more than 16 baby steps");
        auto& P = group_pts(G, l);
        // nb batched ciphertexts (bootstrap_pair): member m at + m qs words; every Q-side
        // buffer below uses the same member stride qs, the Q*P ones ps, so k_lin_mac reads the
        // diagonals once for all members
        const int nb = in.nb;
        const size_t qs = (size_t)2 * nl * n, ps = (size_t)2 * ne * n;
        const u32* c0 = in.data;
        const u32* c1 = in.data + (size_t)nl * n;
        std::vector<u32*> u(g.B, nullptr);
        std::vector<u64> gals(g.B, 0);
        bool any_baby = false;
        for (int b = 1; b < g.B; ++b)
            for (int gg = 0; gg < g.G; ++gg) any_baby = any_baby || P[gg][b];
        // baby steps' key inner products inside k_lin_mac when every giant step fits one pass
        // (each is then computed once), else materialised by k_key_inner
        const bool fused_baby = fused_baby_ && g.G <= kLinG;
        std::vector<const u32*> bkey(g.B, nullptr);
        u32* ext = nullptr;
        if (any_baby) {
            ext = modup(c1, l, nb, qs);
            for (int b = 1; b < g.B; ++b) {
                bool used = false;
                for (int gg = 0; gg < g.G; ++gg) used = used || P[gg][b];
                if (!used) continue;
                const u64 gal = rot_galois(-(int)((long)g.h * b));  // left rotation by h b
                if (fused_baby) {
                    bkey[b] = ksk(gal);
                } else {
                    u[b] = tmp(2 * (size_t)ne * nb);
                    key_inner(u[b], ext, c1, ksk(gal), l, gal, nb, qs);
                }
                gals[b] = gal;  // c0's automorphism is read inside k_lin_mac
                cnt_[C_ROT] += nb;
                tally(LV_KS, l, nb);  // a baby-step rotation: one key switch per member (hoisted ModUp)
            }
            if (!fused_baby) {
                untmp(ext, (size_t)nb * ext_rows(l));
                ext = nullptr;
            }
        }
        Ct out;
        bool have = false;
        // double hoisting: the rotated giant steps' key inner products are summed in Q*P and
        // share ONE ModDown (their permuted c0 summed beside), the unrotated step folded in
        const bool dh = double_hoist_;
        u32* dh_acc = nullptr;
        u32* dh_c0 = nullptr;
        // the fused-core form's P rows (after the ModDown INTT's row pass), owned by THIS call: an
        // exception between giant_accumulate_many and the ModDown below cannot leave it to a later
        // group (it was Engine-wide state that a later call would have taken as its own)
        u32* dh_ys = nullptr;
        int dh_n = 0;
        bool continue_giant = false;
        // all giant steps' diagonal sums in one pass per chunk of kLinG giant steps (k_lin_mac):
        // every baby-step residue is read once instead of once per giant step
        for (int g0 = 0; g0 < g.G; g0 += kLinG) {
            const int gn = std::min(kLinG, g.G - g0);
            LinMacArgs m{};
            m.B = g.B, m.G = gn, m.c1 = c1;
            m.pt_shift = G.c_shift, m.pt_logc = G.c_logc;
            m.nb = nb, m.q_ms = qs, m.p_ms = ps;
            // rotated giant steps: P (out0, out1) folded into outp, ModDown fused with the rescale
            const bool fold = fuse_rr_ && l >= 1 && mdr_off_[l] != SIZE_MAX;
            m.gad = fold ? d_gadget_ : nullptr;
            for (int b = 0; b < g.B; ++b)
                m.a[b] = (b == 0 || u[b] || bkey[b]) ? c0 : nullptr, m.u[b] = b ? u[b] : nullptr, m.gal[b] = gals[b], m.key[b] = bkey[b];
            if (ext) {
                m.ks_ext = ext, m.ks_d = c1, m.ext_ms = (size_t)ext_rows(l) * n, m.d_ms = qs;
                m.nd = (nl + hp_.alpha - 1) / hp_.alpha, m.alpha = hp_.alpha, m.nkey = hp_.n_ks + np, m.nks = hp_.n_ks;
            }
            bool any[kLinG] = {}, rot[kLinG] = {};
            for (int j = 0; j < gn; ++j)
                for (int b = 0; b < g.B; ++b) {
                    m.pt[j][b] = P[g0 + j][b];
                    any[j] = any[j] || P[g0 + j][b];
                    rot[j] = rot[j] || (b && P[g0 + j][b]);
                }
            // rotated giant steps of a double-hoisted group: their Q*P sums side by side in one
            // block (stacked members [j][b]) -> ONE ModDown + rescale, stacked ModUps
            std::vector<int> bj;
            if (dh && fold && giant_batch_)
                for (int j = 0; j < gn; ++j)
                    if (any[j] && rot[j] && g.giant[g0 + j]) bj.push_back(j);
            if ((int)bj.size() < 2 || 2 * nb * (int)bj.size() > kMaxConvGroups) bj.clear();
            u32* blk = bj.empty() ? nullptr : tmp(bj.size() * 2 * (size_t)ne * nb);
            bool in_blk[kLinG] = {};
            for (size_t i = 0; i < bj.size(); ++i) in_blk[bj[i]] = true;
            for (int j = 0, i = 0; j < gn; ++j) {
                const bool folded = fold && rot[j];
                m.out0[j] = folded ? nullptr : tmp(2 * (size_t)nl * nb);  // member stride qs, first nl rows used
                m.out1[j] = (P[g0 + j][0] && !folded) ? tmp(2 * (size_t)nl * nb) : nullptr;
                m.outp[j] = in_blk[j] ? blk + (size_t)(i++) * nb * ps : rot[j] ? tmp(2 * (size_t)ne * nb) : nullptr;
            }
            launch_lin_mac(S(), T_, m, nl, ne, extmap(nl));
            for (int j = 0; j < gn; ++j)
                for (int b = 0; b < g.B; ++b)
                    if (P[g0 + j][b]) tally(LV_PTMUL, l, nb);  // one diagonal product per member
            if (!bj.empty()) {
                Ct rs = moddown_rescale(blk, l, nb * (int)bj.size());
                std::vector<u64> gs;
                for (int j : bj) gs.push_back(rot_galois(-(int)g.giant[g0 + j]));
                // the only accumulation of the group: one chunk, and no other giant step of it rotated
                bool sole = g.G <= kLinG && dh_n == 0;
                for (int j = 0; j < gn && sole; ++j)
                    if (!in_blk[j] && any[j] && dh && g.giant[g0 + j]) sole = false;
                giant_accumulate_many(rs, gs, nb, dh_acc, dh_c0, dh_n, dh_ys, sole);
                release(rs);
                untmp(blk, bj.size() * 2 * (size_t)ne * nb);
            }
            for (int j = 0; j < gn; ++j) {
                const int gg = g0 + j;
                if (in_blk[j]) {
                    if (m.out0[j]) untmp(m.out0[j], 2 * (size_t)nl * nb);
                    if (m.out1[j]) untmp(m.out1[j], 2 * (size_t)nl * nb);
                    continue;
                }
                if (any[j]) {
                    Ct inner, rs;
                    if (rot[j] && fold) {
                        rs = moddown_rescale(m.outp[j], l, nb);
                    } else if (rot[j]) {
                        inner = moddown(m.outp[j], l, m.out0[j], m.out1[j], nb, qs);
                    } else {  // only the unrotated diagonal
                        inner = alloc_ct(l, 2 * nb, nb);
                        for (int mb = 0; mb < nb; ++mb) {
                            launch_copy_rows(S(), T_, inner.data + mb * qs, m.out0[j] + mb * qs, nl);
                            launch_copy_rows(S(), T_, inner.data + mb * qs + (size_t)nl * n, m.out1[j] + mb * qs, nl);
                        }
                    }
                    if (!(rot[j] && fold)) {
                        rs = rescale(inner);
                        release(inner);
                    }
                    if (dh && g.giant[gg]) {
                        giant_accumulate(rs, rot_galois(-(int)g.giant[gg]), dh_acc, dh_c0, dh_n);
                        release(rs);
                        continue_giant = true;
                    }
                    Ct part;
                    if (!continue_giant) {
                        part = g.giant[gg] ? rotl(rs, g.giant[gg]) : rs;
                        if (g.giant[gg]) release(rs);
                    }
                    if (continue_giant) {
                        continue_giant = false;
                    } else if (!have) {
                        out = part, have = true;
                    } else {
                        Ct s2 = add_sub(out, part, false);
                        release(out);
                        release(part);
                        out = s2;
                    }
                }
                if (m.out0[j]) untmp(m.out0[j], 2 * (size_t)nl * nb);
                if (m.out1[j]) untmp(m.out1[j], 2 * (size_t)nl * nb);
                if (m.outp[j]) untmp(m.outp[j], 2 * (size_t)ne * nb);
            }
        }
        for (int b = 1; b < g.B; ++b) {
            if (u[b]) untmp(u[b], 2 * (size_t)ne * nb);
        }
        if (ext) untmp(ext, (size_t)nb * ext_rows(l));
        if (dh_n > 0) {
            const int lv = l - 1, r = hp_.nl(lv), ne2 = r + np;
            const size_t ms = (size_t)2 * r * n;
            const u32* add1 = nullptr;
            if (have) {  // the unrotated giant step: c0 into the sum, c1 as the second addend
                if (out.level != lv || pm(out) != 2 || out.pend) throw std::runtime_error("lin_group: unrotated part off level");
                for (int mb = 0; mb < nb; ++mb) launch_add(S(), T_, dh_c0 + mb * ms, dh_c0 + mb * ms, out.data + mb * ms, r, r, qmap());
                add1 = out.data + (size_t)r * n;
            }
            Ct res = moddown(dh_acc, lv, dh_c0, add1, nb, ms, nullptr, nullptr, false, dh_ys);
            if (dh_ys) untmp(dh_ys, 2 * (size_t)np * nb), dh_ys = nullptr;
            if (have) release(out);
            untmp(dh_acc, 2 * (size_t)ne2 * nb);
            untmp(dh_c0, 2 * (size_t)r * nb);
            out = res;
        }
        return out;
    }
    // K rotated giant steps at once: rs holds K x nb stacked members ([j][b]), step j permuted
    // by X -> X^gals[j]; their c1 ModUp'ed together (chunks within kMaxConvGroups), each key
    // inner product accumulated into acc, the permuted c0 summed into c0sum per member
    // sole: no other giant step of the group is accumulated (lin_group): the fused-core form may run.
    // AESFHE_FUSED_GIANT=0 turns it off: the full-slot bootstrap's groups take it (batch leg 11,551 ->
    // 11,407 launches per step, 4,984-5,000 -> 5,055-5,056 blocks/s, profiles/r4_ab_giant_batch.txt),
    // C2's sparse plans do not; bit-identical (tests/test_gpu_fused_giant.py)
    bool fused_giant_ = !(std::getenv("AESFHE_FUSED_GIANT") && std::atoi(std::getenv("AESFHE_FUSED_GIANT")) == 0);
    int test_fail_giant_ = env_int("AESFHE_TEST_FAIL_GIANT", 0);
    // ys (out): set by the fused form to the P rows after the INTT row pass, for the caller's ModDown
    void giant_accumulate_many(const Ct& rs, const std::vector<u64>& gals, int nb, u32*& acc, u32*& c0sum, int& count, u32*& ys,
                               bool sole = false) {
        const int K = (int)gals.size(), lv = rs.level, r = hp_.nl(lv), ne2 = r + hp_.n_p, n = hp_.n;
        const size_t ms = (size_t)2 * r * n;
        if (rs.nb != K * nb || K > kMaxMembers) throw std::runtime_error("giant_accumulate_many: batch shape");
        // test hook (tests/test_gpu_flag_identity.py): the k-th call of the process fails, after
        // its group allocated its accumulators -- the next bootstrap must not see any of that group's state
        if (test_fail_giant_ > 0 && --test_fail_giant_ == 0) throw std::runtime_error("giant_accumulate_many: test failure (AESFHE_TEST_FAIL_GIANT)");
        u32* perm = tmp(2 * (size_t)r * nb * K);
        for (int j = 0; j < K; ++j) launch_automorph(S(), T_, perm + (size_t)j * nb * ms, rs.data + (size_t)j * nb * ms, gals[j], 2 * r * nb);
        if (!acc) acc = tmp(2 * (size_t)ne2 * nb);
        const int nd = (r + hp_.alpha - 1) / hp_.alpha;
        const int per = std::max(1, std::min(kMaxConvGroups / (nd * nb), kMaxKsBatch));  // steps per ModUp
        if (sole && count == 0 && fused_ki_ok() && fused_giant_ && K <= kMaxKiSrc && per >= K) {
            // the group's only accumulation: the K key inner products summed in ONE fused-core launch
            // (multi-source k_ntt2_ki: each step's ModUp row pass in registers, no ext written), the P
            // rows through the ModDown INTT's row pass into ys for lin_group's ModDown
            const u32* c1 = perm + (size_t)r * n;
            u32* ext = modup(c1, lv, nb * K, ms, nullptr, false, true);
            const size_t er = (size_t)ext_rows(lv) * n;
            KiSrc src[kMaxKiSrc];
            for (int j = 0; j < K; ++j) src[j] = KiSrc{ext + (size_t)j * nb * er, perm + (size_t)j * nb * ms + (size_t)r * n, ksk(gals[j])};
            ys = tmp(2 * (size_t)hp_.n_p * nb);
            ki_core(acc, ys, lv, r, nb, src, K, ms, KsFold{});
            untmp(ext, (size_t)nb * K * ext_rows(lv));
        }
        for (int j0 = 0; j0 < K && !ys; j0 += per) {
            const int k = std::min(per, K - j0);
            const u32* c1 = perm + (size_t)j0 * nb * ms + (size_t)r * n;
            u32* ext = modup(c1, lv, nb * k, ms);
            const size_t er = (size_t)ext_rows(lv) * n;
            for (int j = j0; j < j0 + k; ++j) {
                key_inner(acc, ext + (size_t)(j - j0) * nb * er, perm + (size_t)j * nb * ms + (size_t)r * n, ksk(gals[j]), lv, 0, nb, ms, KsFold{},
                          count > 0 || j > 0);
            }
            untmp(ext, (size_t)nb * k * ext_rows(lv));
        }
        const bool fresh = c0sum == nullptr;
        if (fresh) c0sum = tmp(2 * (size_t)r * nb);
        for (int b = 0; b < nb; ++b) {
            MemberPtrs mp;
            for (int j = 0; j < K; ++j) mp.src[j] = perm + ((size_t)j * nb + b) * ms;
            launch_add_members(S(), T_, c0sum + (size_t)b * ms, mp, K, r, qmap(), !fresh);
        }
        untmp(perm, 2 * (size_t)r * nb * K);
        count += K;
        cnt_[C_ROT] += K * nb;
        cnt_[C_KS] += K * nb;
        tally(LV_KS, lv, K * nb);
    }
    // one rotated giant step of a double-hoisted group: rs permuted by X -> X^gal, its c1
    // key switched into the running Q*P sum acc (allocated on the first call), its c0 summed
    // into c0sum (the first permuted buffer, member stride 2 r N)
    void giant_accumulate(const Ct& rs, u64 gal, u32*& acc, u32*& c0sum, int& count) {
        if (vis_npoly(rs) != 2 || rs.pend || rs.lazy) throw std::runtime_error("giant_accumulate: canonical input expected");
        const int lv = rs.level, r = hp_.nl(lv), ne2 = r + hp_.n_p, nb = rs.nb, n = hp_.n;
        const size_t ms = (size_t)2 * r * n;
        u32* perm = tmp(2 * (size_t)r * nb);
        launch_automorph(S(), T_, perm, rs.data, gal, 2 * r * nb);
        const u32* p1 = perm + (size_t)r * n;
        u32* ext = modup(p1, lv, nb, ms);
        if (!acc) acc = tmp(2 * (size_t)ne2 * nb);
        key_inner(acc, ext, p1, ksk(gal), lv, 0, nb, ms, KsFold{}, count > 0);
        untmp(ext, (size_t)nb * ext_rows(lv));
        if (count == 0) {
            c0sum = perm;
        } else {
            for (int mb = 0; mb < nb; ++mb) launch_add(S(), T_, c0sum + mb * ms, c0sum + mb * ms, perm + mb * ms, r, r, qmap());
            untmp(perm, 2 * (size_t)r * nb);
        }
        ++count;
        cnt_[C_ROT] += nb;
        cnt_[C_KS] += nb;
        tally(LV_KS, lv, nb);
    }

    Ct lin_transform(const Ct& in, std::vector<BootGroupDev>& groups) {
        Ct cur = in;
        bool own = false;
        for (auto& G : groups) {
            Ct nx = lin_group(cur, G);
            if (own) release(cur);
            cur = nx, own = true;
        }
        return cur;
    }

    // sum_{k <= deg} c_k T_k from the baby table T[1..8] (T_0 = 1): scalar products deferred
    // (one rescale for the whole leaf), constant term added at the raw scale
    // c_0 + sum_k c_k T_k as ONE fused kernel (k_lut_univariate): integer constants
    // round(c_k S_out / delta_{level(T_k)}) at the output's raw scale S_out = raw_scale(l, 1),
    // l = the lowest level of the terms (their first nl(l) limbs are read); cached per
    // coefficient vector and level signature.  Returns false when the scale has no headroom.
    bool cheb_leaf_fused(const std::vector<Ct>& T, const std::vector<double>& c, Ct& out) {
        std::vector<int> ks;
        double mag = std::fabs(c[0]);
        int l = 1 << 30;
        for (size_t k = 1; k < c.size(); ++k) {
            if (c[k] == 0.0) continue;
            const Ct& t = T[k];
            if (pm(t) != 2 || t.nb != T[1].nb || t.pend != 0 || t.lazy || !t.ntt) return false;
            ks.push_back((int)k);
            mag += std::fabs(c[k]);
            l = std::min(l, t.level);
        }
        if (ks.empty() || (int)ks.size() > kLutChunk || !headroom(l, 1, mag)) return false;
        const int nl = hp_.nl(l);
        const double S_out = raw_scale(l, 1);
        std::string key = std::to_string(l) + ":";
        for (int k : ks) key += std::to_string(k) + "@" + std::to_string(T[k].level) + "=" + std::to_string(c[k]) + ",";
        auto it = leaf_cst_.find(key);
        if (it == leaf_cst_.end()) {
            std::vector<u32> h(ks.size() * (size_t)nl * 4), lo, hi;
            for (size_t j = 0; j < ks.size(); ++j) {
                scalar_residues(std::llround(c[ks[j]] * S_out / hp_.delta[T[ks[j]].level]), 0, nl, lo, hi);
                for (int t = 0; t < nl; ++t) {
                    u32* e = &h[(j * nl + t) * 4];
                    e[0] = lo[t], e[1] = shoup_pre(lo[t], hp_.mod[t]);
                    e[2] = hi[t], e[3] = shoup_pre(hi[t], hp_.mod[t]);
                }
            }
            const size_t words = (h.size() + (size_t)hp_.n - 1) / hp_.n * hp_.n;
            u32* d = dev_alloc(words);  // lives with the context (one per leaf and level signature)
            HIP_OK(hipMemcpyAsync(d, h.data(), h.size() * sizeof(u32), hipMemcpyHostToDevice, S()));
            HIP_OK(hipStreamSynchronize(S()));
            it = leaf_cst_.emplace(key, d).first;
        }
        LutChunk ch{};
        for (size_t j = 0; j < ks.size(); ++j) ch.x[j] = T[ks[j]].data, ch.nx[j] = hp_.nl(T[ks[j]].level);
        const int nb = T[ks[0]].nb;
        Ct o = alloc_ct(l, 2 * nb, nb);
        // c_0 added in the same launch (the add_scalar lincomb's constants at the sum's level and owed rescale)
        LimbConsts cadd{};
        if (c[0] != 0.0) cadd = add_consts(l, 1, c[0], 0.0);
        launch_lut_univariate(S(), T_, o.data, nullptr, ch, (int)ks.size(), it->second, 2, nl, nb, c[0] != 0.0 ? &cadd : nullptr);
        o.pend = 1;
        o.lazy = true;
        out = normalize(o, true);
        if (out.data != o.data) release(o);
        return true;
    }
    std::map<std::string, u32*> leaf_cst_;

    Ct cheb_leaf(const std::vector<Ct>& T, const std::vector<double>& c) {
        Ct fused;
        if (cheb_leaf_fused(T, c, fused)) return fused;
        Ct acc;
        bool have = false;
        for (size_t k = 1; k < c.size(); ++k) {
            if (c[k] == 0.0) continue;
            Ct t = mul_scalar(T[k], c[k], 0.0, true);
            if (!have) {
                acc = t, have = true;
            } else {
                Ct s = add_sub(acc, t, false);
                release(acc);
                release(t);
                acc = s;
            }
        }
        if (!have) throw std::runtime_error("EvalMod: empty Chebyshev leaf");
        if (c[0] != 0.0) {
            Ct s = add_scalar(acc, c[0], 0.0);
            release(acc);
            acc = s;
        }
        Ct o = normalize(acc, true);
        if (o.data != acc.data) release(acc);
        return o;
    }
    // p = q + T_m r with q_i = c_i - c_{2m-i} (i < m), r_0 = c_m, r_j = 2 c_{m+j}; recurse
    // until the degree is within the baby table (Paterson-Stockmeyer in the Chebyshev basis)
    // Paterson-Stockmeyer style split c = q + T_m r (m the largest power-of-two giant step <= d),
    // applied to several polynomials at once: the giant-step products of one recursion depth are
    // independent, so they run as ONE batched multiply (mul_many, bit-exact with mul); the sums
    // are the same as the one-polynomial recursion's
    // applied to several polynomials at once, item i on input in[i] (its T / giant sets): the
    // giant-step products of one recursion depth are independent, so they run as ONE batched
    // multiply (mul_many, bit-exact with mul); the sums are the one-polynomial recursion's
    std::vector<Ct> cheb_eval_many(const std::vector<std::vector<Ct>>& T, const std::vector<std::map<int, Ct>>& giant,
                                   const std::vector<int>& in, const std::vector<std::vector<double>>& cs) {
        std::vector<Ct> out(cs.size());
        std::vector<std::vector<double>> sub;  // q_0, r_0, q_1, r_1, ...
        std::vector<int> idx, ms, sub_in;
        for (size_t i = 0; i < cs.size(); ++i) {
            const auto& c = cs[i];
            const int d = (int)c.size() - 1;
            if (d <= kBabyDeg) {
                out[i] = cheb_leaf(T[in[i]], c);
                continue;
            }
            int m = kBabyDeg;
            while (2 * m <= d) m *= 2;
            std::vector<double> q(m), r(d - m + 1);
            for (int k = 0; k < m; ++k) q[k] = c[k] - (2 * m - k <= d ? c[2 * m - k] : 0.0);
            r[0] = c[m];
            for (int j = 1; j <= d - m; ++j) r[j] = 2.0 * c[m + j];
            idx.push_back((int)i), ms.push_back(m);
            sub.push_back(std::move(q)), sub.push_back(std::move(r));
            sub_in.push_back(in[i]), sub_in.push_back(in[i]);
        }
        if (idx.empty()) return out;
        std::vector<Ct> v = cheb_eval_many(T, giant, sub_in, sub);
        std::vector<const Ct*> A, B;
        for (size_t j = 0; j < idx.size(); ++j) A.push_back(&giant[in[idx[j]]].at(ms[j])), B.push_back(&v[2 * j + 1]);
        std::vector<Ct> P = mul_list(A, B);
        for (size_t j = 0; j < idx.size(); ++j) {
            release(v[2 * j + 1]);
            out[idx[j]] = add_sub(v[2 * j], P[j], false);
            release(v[2 * j]);
            release(P[j]);
        }
        return out;
    }
    // The same series as cheb_eval_many with its split tree flattened into a product schedule:
    // each product T_m r is issued as soon as r's value exists, not after q's subtree.  In the
    // degree-23 series (q' + T_8 r') + T_16 r both r' and r are leaves, so T_8 r' and T_16 r run as
    // ONE batched multiply (same level) and the series takes one product round per level of depth
    // (EvalMod: 10 -> 9 rounds).  Leaves, products and sums are the recursion's own operations on the
    // same operands, so the result is bit-identical (AESFHE_CHEB_SCHED=0: the recursion, A/B).
    std::vector<Ct> cheb_eval_sched(const std::vector<std::vector<Ct>>& T, const std::vector<std::map<int, Ct>>& giant,
                                    const std::vector<int>& in, const std::vector<std::vector<double>>& cs) {
        struct Node {
            int in = 0, m = 0, q = -1, r = -1;  // m > 0: value = q + T_m r
            std::vector<double> c;              // m == 0: a leaf's coefficients
            Ct val, prod;
            bool has = false, has_prod = false;
        };
        std::vector<Node> nd;  // parents before children (indices only: the vector grows)
        std::function<int(int, const std::vector<double>&)> build = [&](int i, const std::vector<double>& c) -> int {
            const int d = (int)c.size() - 1, id = (int)nd.size();
            nd.emplace_back();
            nd[id].in = i;
            if (d <= kBabyDeg) {
                nd[id].c = c;
                return id;
            }
            int m = kBabyDeg;
            while (2 * m <= d) m *= 2;
            std::vector<double> q(m), r(d - m + 1);
            for (int k = 0; k < m; ++k) q[k] = c[k] - (2 * m - k <= d ? c[2 * m - k] : 0.0);
            r[0] = c[m];
            for (int j = 1; j <= d - m; ++j) r[j] = 2.0 * c[m + j];
            const int qi = build(i, q), ri = build(i, r);
            nd[id].m = m, nd[id].q = qi, nd[id].r = ri;
            return id;
        };
        std::vector<int> root(cs.size());
        for (size_t i = 0; i < cs.size(); ++i) root[i] = build(in[i], cs[i]);
        for (auto& x : nd)
            if (x.m == 0) x.val = cheb_leaf(T[x.in], x.c), x.has = true;
        for (;;) {
            bool all = true;
            for (int id : root) all = all && nd[id].has;
            if (all) break;
            std::vector<const Ct*> A, B;
            std::vector<int> ids;
            for (int k = 0; k < (int)nd.size(); ++k)
                if (nd[k].m > 0 && !nd[k].has_prod && nd[nd[k].r].has)
                    A.push_back(&giant[nd[k].in].at(nd[k].m)), B.push_back(&nd[nd[k].r].val), ids.push_back(k);
            bool moved = !ids.empty();
            if (moved) {
                std::vector<Ct> P = mul_list(A, B);
                for (size_t j = 0; j < ids.size(); ++j) {
                    Node& x = nd[ids[j]];
                    x.prod = P[j], x.has_prod = true;
                    release(nd[x.r].val);
                }
            }
            for (int k = (int)nd.size() - 1; k >= 0; --k) {  // children first: a finished sum may finish its parent
                Node& x = nd[k];
                if (x.m == 0 || x.has || !x.has_prod || !nd[x.q].has) continue;
                x.val = add_sub(nd[x.q].val, x.prod, false);
                release(nd[x.q].val);
                release(x.prod);
                x.has = moved = true;
            }
            if (!moved) throw std::runtime_error("EvalMod: Chebyshev schedule stalled");
        }
        std::vector<Ct> out(cs.size());
        for (size_t i = 0; i < cs.size(); ++i) out[i] = nd[root[i]].val;
        return out;
    }
    bool cheb_sched_ = env_int("AESFHE_CHEB_SCHED", 1) != 0;
    // products of a list of pairs: one batched multiply (AESFHE_EVALMOD_BATCH=0: one at a time)
    std::vector<Ct> mul_list(const std::vector<const Ct*>& A, const std::vector<const Ct*>& B, const std::vector<char>* aff = nullptr) {
        static const bool batch = env_int("AESFHE_EVALMOD_BATCH", 1) != 0;
        if (batch) return mul_many(A, B, aff);
        std::vector<Ct> P(A.size());
        for (size_t j = 0; j < A.size(); ++j) P[j] = mul(*A[j], *B[j], true, false, aff && (*aff)[j]);
        return P;
    }
    static constexpr int kBabyDeg = 8;

    // EvalMod: sin(2 pi K y) via the Chebyshev interpolant of cos(2 pi (K y - 1/4) / 2^r)
    // (baby T_1..T_8, giant T_8, T_16, ...) and r double angles
    Ct eval_mod(const Ct& y) { return std::move(eval_mod_many({&y})[0]); }
    // EvalMod of several ciphertexts at once (the bootstrap's re / im halves): every product of
    // one step -- a baby-step depth group, a giant step, a Chebyshev recursion depth, a double
    // angle -- for all inputs as ONE batched multiply.  Baby steps by depth: T_k = 2 T_a T_b -
    // T_{a-b} (a = ceil(k/2), b = floor(k/2)) needs only T_1 .. T_{lo-1}, so T_lo .. T_{2 lo - 2}
    // are independent -- T_2, then T_3..T_4, then T_5..T_8
    std::vector<Ct> eval_mod_many(const std::vector<const Ct*>& ys) {
        const auto& c = bs_.plan.cheb;
        const int d = (int)c.size() - 1, ni = (int)ys.size();
        std::vector<std::vector<Ct>> T(ni, std::vector<Ct>(kBabyDeg + 1));
        for (int i = 0; i < ni; ++i) T[i][1] = *ys[i];  // read only (the caller owns it): no copy, not released below
        static const bool batch_baby = env_int("AESFHE_EVALMOD_BATCH", 1) != 0;
        for (int lo = 2; lo <= kBabyDeg;) {
            const int hi = batch_baby ? std::min(kBabyDeg, 2 * lo - 2) : lo;
            std::vector<const Ct*> A, B;
            std::vector<char> aff;  // 2 T_a^2 - 1 in the product's own relinearisation (fused_affine_)
            for (int i = 0; i < ni; ++i)
                for (int k = lo; k <= hi; ++k)
                    A.push_back(&T[i][(k + 1) / 2]), B.push_back(&T[i][k / 2]), aff.push_back(fused_affine_ && (k + 1) / 2 == k / 2);
            std::vector<Ct> P = mul_list(A, B, &aff);
            int j = 0;
            for (int i = 0; i < ni; ++i)
                for (int k = lo; k <= hi; ++k, ++j) {
                    const int a = (k + 1) / 2, b = k / 2;
                    // 2 T_a T_b - T_(a-b) (a > b) / 2 T_a^2 - 1, one launch each (none for the latter when fused)
                    if (aff[j]) {
                        T[i][k] = P[j];
                        continue;
                    }
                    T[i][k] = (a == b) ? lincomb(P[j], 2, nullptr, 0, -1.0, 0.0) : lincomb(P[j], 2, &T[i][a - b], -1, 0.0, 0.0);
                    release(P[j]);
                }
            lo = hi + 1;
        }
        std::vector<std::map<int, Ct>> giant(ni);
        for (int i = 0; i < ni; ++i) giant[i][kBabyDeg] = T[i][kBabyDeg];
        for (int m = 2 * kBabyDeg; m <= d; m *= 2) {
            std::vector<const Ct*> A;
            for (int i = 0; i < ni; ++i) A.push_back(&giant[i].at(m / 2));
            const std::vector<char> aff(ni, fused_affine_ ? 1 : 0);
            std::vector<Ct> P = mul_list(A, A, &aff);
            for (int i = 0; i < ni; ++i) {
                if (fused_affine_) {
                    giant[i][m] = P[i];
                    continue;
                }
                giant[i][m] = lincomb(P[i], 2, nullptr, 0, -1.0, 0.0);  // 2 T^2 - 1, one launch
                release(P[i]);
            }
        }
        std::vector<int> in(ni);
        for (int i = 0; i < ni; ++i) in[i] = i;
        const std::vector<std::vector<double>> cs(ni, c);
        std::vector<Ct> g = cheb_sched_ ? cheb_eval_sched(T, giant, in, cs) : cheb_eval_many(T, giant, in, cs);
        for (int i = 0; i < ni; ++i) {
            for (int k = 2; k <= kBabyDeg; ++k) release(T[i][k]);
            for (auto& kv : giant[i])
                if (kv.first != kBabyDeg) release(kv.second);
        }
        for (int it = 0; it < bs_.plan.r; ++it) {
            std::vector<const Ct*> A;
            for (int i = 0; i < ni; ++i) A.push_back(&g[i]);
            const std::vector<char> aff(ni, fused_affine_ ? 1 : 0);
            std::vector<Ct> P = mul_list(A, A, &aff);
            for (int i = 0; i < ni; ++i) {
                release(g[i]);
                if (fused_affine_) {
                    g[i] = P[i];
                    continue;
                }
                g[i] = lincomb(P[i], 2, nullptr, 0, -1.0, 0.0);  // double angle 2 g^2 - 1, one launch
                release(P[i]);
            }
        }
        return g;
    }

    // stop_after (debug): 1 q0-only, 2 after SSE, 3 ModRaise, 4 back to dense, 5 CoeffToSlot,
    // 6 real part, 7 imaginary part, 8 EvalMod(real), 9 EvalMod(imag), 10 recombined, 11 output
    // gain: the output carries gain * message (folded into the level-0 scaling integer k1,
    // relative precision 2^-k1bits; the true-FHE snap's kappa, zeta16_noise_reducer.py)
    // level-0 stack z (nb members, consumed) -> the bootstrapped stack, in chunks of two members
    // (the pair bootstrap's batch: every key and diagonal read once per chunk)
    // members per chunk (AESFHE_BOOT_CHUNK, default 4: a 16-pair stack's final bootstraps 98.1 -> 86.4 ms
    // per round against chunks of 2, profiles/r4_stack16_chunk{2,4}_step_profile.json; every member's
    // bytes are the same at any chunk size, tests/test_gpu_boot_chunk.py)
    int boot_chunk_ = std::max(1, env_int("AESFHE_BOOT_CHUNK", 4));
    Ct boot_stack(Ct z, double gain, SparseBoot* sv) {
        const int P = z.nb, B = boot_chunk_;
        if (P <= B) return bootstrap_l0(z, 99, gain, sv);
        Ct out;
        for (int m0 = 0; m0 < P; m0 += B) {
            const int c = std::min(B, P - m0);
            Ct r = bootstrap_l0(members_of(z, m0, c), 99, gain, sv);
            if (m0 == 0) {
                out = alloc_ct(r.level, pm(r) * P, P);
                copy_meta(out, r);
                out.nb = P;
            }
            if (r.level != out.level || pm(r) != pm(out)) throw std::runtime_error("bootstrap: stack chunks at different levels");
            launch_copy_rows(S(), T_, out.data + (size_t)m0 * pm(r) * hp_.nl(r.level) * hp_.n, r.data, r.words / hp_.n);
            release(r);
        }
        release(z);
        return out;
    }
    Ct bootstrap(const Ct& in, int stop_after = 99, double gain = 1.0, int period = 0) {
        boot_setup();
        if (vis_npoly(in) != 2) throw std::runtime_error("bootstrap expects a 2-polynomial ciphertext");
        SparseBoot* sv = (period > 0 && period < slot_count()) ? &sparse_variant(period) : nullptr;
        if (in.nb > 1) {  // a stack (multi-pair batch): chunks of two members
            if (stop_after != 99) throw std::runtime_error("bootstrap: debug stages take a single ciphertext");
            Ct c = normalize(in);
            Ct z = level_down(c, 0);
            if (c.data != in.data) release(c);
            if (period > 0 && stack_pack_ > 1 && in.nb % 2 == 0 && 2 * period <= slot_count()) return boot_stack_packed(z, gain, period);
            return boot_stack(z, gain, sv);
        }
        Ct c = normalize(in);
        Ct z = level_down(c, 0);
        if (c.data != in.data) release(c);
        return bootstrap_l0(z, stop_after, gain, sv);
    }
    // the hi / lo bootstraps of an AES step (MixColumns' final bootstrap) as ONE batched
    // bootstrap of two stacked ciphertexts: every key switch reads its key, and every linear
    // transform its diagonals, once for both; half the launches
    void bootstrap_pair(const Ct& a_in, const Ct& b_in, aesfhe_handle* oa, aesfhe_handle* ob, double gain = 1.0, int period = 0) {
        boot_setup();
        if (vis_npoly(a_in) != 2 || vis_npoly(b_in) != 2 || a_in.nb != b_in.nb)
            throw std::runtime_error("bootstrap expects a 2-polynomial ciphertext");
        if (period > 0 && 2 * period <= slot_count() && mono_pair_) return bootstrap_pair_mono(a_in, b_in, oa, ob, gain, period);
        if (a_in.nb > 1) {  // stacks: a's and b's members bootstrapped in chunks of two
            *oa = put_ct(bootstrap(a_in, 99, gain, period));
            *ob = put_ct(bootstrap(b_in, 99, gain, period));
            return;
        }
        SparseBoot* sv = (period > 0 && period < slot_count()) ? &sparse_variant(period, true) : nullptr;
        const int n = hp_.n, nl0 = hp_.nl(0);
        Ct z = alloc_ct(0, 4, 2);
        const Ct* in[2] = {&a_in, &b_in};
        for (int m = 0; m < 2; ++m) {
            Ct c = normalize(*in[m]);
            Ct zm = level_down(c, 0);
            if (c.data != in[m]->data) release(c);
            launch_copy_rows(S(), T_, z.data + (size_t)m * 2 * nl0 * n, zm.data, 2 * nl0);
            release(zm);
        }
        Ct out = bootstrap_l0(z, 99, gain, sv);
        const int nlo = hp_.nl(out.level);
        aesfhe_handle* dst[2] = {oa, ob};
        for (int m = 0; m < 2; ++m) {
            Ct o = alloc_ct(out.level, 2);
            o.ntt = out.ntt;
            launch_copy_rows(S(), T_, o.data, out.data + (size_t)m * 2 * nlo * n, 2 * nlo);
            *dst[m] = put_ct(o);
        }
        release(out);
    }
    // The pair of n-periodic messages a, b (2n <= slots) as ONE 2n-periodic message
    // (DESIGN.md §4b): a, b lie in the subring Z[X^2k], k = N / 4n, so z = a + X^k b lies in
    // Z[X^k] -- the 2n-periodic messages -- exactly (a monomial product only permutes and
    // negates coefficients).  One bootstrap at period 2n (the full-slot one when 2n = slots)
    // with gain / 2 (|z| <= |a| + |b|) refreshes both; the rotation by n slots is
    // X -> X^(4n+1) (5^n = 4n + 1 mod 8n), which fixes X^2k and negates X^k, so with
    // m = gain z / 2 and r = rot_n(m):  gain a = m + r,  gain b = X^-k (m - r).
    int z_members_ = 1;
    bool mono_pair_ = !(std::getenv("AESFHE_PAIR_MONO") && std::atoi(std::getenv("AESFHE_PAIR_MONO")) == 0);
    // z = a + X^k b at level 0 (k = N / 4 period): exact, one fused multiply-add with the NTT form
    // of the monomial
    Ct mono_pack(const Ct& a_in, const Ct& b_in, int period) {
        const int n = hp_.n, k = n / (4 * period), nl0 = hp_.nl(0);
        if (period < 1 || 2 * period > slot_count() || n % (4 * period)) throw std::runtime_error("mono_pack: bad period");
        Ct z0[2];
        const Ct* in[2] = {&a_in, &b_in};
        for (int m = 0; m < 2; ++m) {
            Ct c = normalize(*in[m]);
            z0[m] = level_down(c, 0);
            if (c.data != in[m]->data) release(c);
        }
        if (z0[0].nb != z0[1].nb) throw std::runtime_error("mono_pack: stacks of different sizes");
        Ct z = alloc_ct(0, z0[0].npoly, z0[0].nb);
        launch_fma_poly(S(), T_, z.data, z0[0].data, z0[1].data, monomial(k), z0[0].npoly * nl0, nl0, qmap());
        release(z0[0]);
        release(z0[1]);
        return z;
    }
    // m = (a + X^k b) / 2 -> (a, b): r = rot_period(m) fixes X^2k and negates X^k, so a = m + r and
    // b = X^-k (m - r)
    void mono_split(const Ct& mz, int period, Ct& hi, Ct& lo) {
        const int n = hp_.n, k = n / (4 * period);
        Ct r = rotate(mz, period);
        hi = add_sub(mz, r, false);
        Ct d = add_sub(mz, r, true);
        release(r);
        Ct dn = ensure_ntt(d);
        if (dn.data != d.data) release(d);
        lo = alloc_ct(dn.level, dn.npoly, dn.nb);
        copy_meta(lo, dn);
        launch_mul_poly(S(), T_, lo.data, dn.data, monomial(2 * n - k), dn.npoly, hp_.nl(dn.level), qmap());
        release(dn);
    }
    void bootstrap_pair_mono(const Ct& a_in, const Ct& b_in, aesfhe_handle* oa, aesfhe_handle* ob, double gain, int period) {
        Ct z = mono_pack(a_in, b_in, period);
        z_members_ = z.nb;
        SparseBoot* sv = 2 * period < slot_count() ? &sparse_variant(2 * period) : nullptr;
        Ct mz = boot_stack(z, 0.5 * gain, sv);  // a stack of P packed pairs: chunks of two
        Ct hi, lo;
        mono_split(mz, period, hi, lo);
        release(mz);
        cnt_[C_BOOT] += z_members_;  // bootstrap_l0 counted one per packed pair: two messages each
        *oa = put_ct(hi);
        *ob = put_ct(lo);
    }
    // four n-periodic messages (4n <= slots) as ONE 4n-periodic message:
    // the pairs (a, b) and (c, d) packed as above into the 2n-periodic z1, z2, then
    // z = z1 + X^(N/8n) z2 in Z[X^(N/8n)] (exact again).  One bootstrap at period 4n with
    // gain / 4 refreshes all four; rotations by 2n then n slots split it back (mono_split twice)
    void bootstrap_quad_mono(const Ct* const in[4], aesfhe_handle* out[4], double gain, int period) {
        boot_setup();
        for (int m = 0; m < 4; ++m)
            if (vis_npoly(*in[m]) != 2 || in[m]->nb != in[0]->nb)
                throw std::runtime_error("bootstrap_quad: four 2-polynomial ciphertexts of one stack size expected");
        const int n = hp_.n, nl0 = hp_.nl(0);
        if (period < 1 || 4 * period > slot_count() || n % (8 * period))
            throw std::runtime_error("bootstrap_quad: the period must satisfy 4 period <= slots");
        Ct z1 = mono_pack(*in[0], *in[1], period);
        Ct z2 = mono_pack(*in[2], *in[3], period);
        Ct z = alloc_ct(0, z1.npoly, z1.nb);
        launch_fma_poly(S(), T_, z.data, z1.data, z2.data, monomial(n / (8 * period)), z1.npoly * nl0, nl0, qmap());
        release(z1);
        release(z2);
        z_members_ = z.nb;
        SparseBoot* sv = 4 * period < slot_count() ? &sparse_variant(4 * period) : nullptr;
        Ct mz = boot_stack(z, 0.25 * gain, sv);
        Ct h[2], o[4];
        mono_split(mz, 2 * period, h[0], h[1]);
        release(mz);
        for (int j = 0; j < 2; ++j) {
            mono_split(h[j], period, o[2 * j], o[2 * j + 1]);
            release(h[j]);
        }
        cnt_[C_BOOT] += 3 * z_members_;  // four messages per packed quad
        for (int m = 0; m < 4; ++m) *out[m] = put_ct(o[m]);
    }
    // a stack of M period-P members bootstrapped G members per bootstrap:
    // the monomial pair packing applied log2 G times over the stack's halves -- members [0, m/2)
    // + X^(N/4p) members [m/2, m), exact, one launch per level -- so M / G members of period P G
    // go through boot_stack with gain / G, then log2 G mono_split levels (one batched rotation of
    // the stack each) unpack them in the original member order.  G: the largest power of two
    // <= stack_pack_ dividing M with P G <= slots.  The members' bootstrap errors grow ~G x (the
    // packed message is G x smaller against the same bootstrap error); stack_pack_ = 1: off
    // (16: C3 stacks of 64 pairs 78 -> 50 ms per pair, precision margin 121x; profiles/r6_stack_pack_ab.txt)
    int stack_pack_ = env_int("AESFHE_STACK_PACK", 16);
    Ct boot_stack_packed(Ct z, double gain, int period) {
        const int M = z.nb, n = hp_.n, nl0 = hp_.nl(0), per = pm(z);
        int G = 1;
        while (2 * G <= stack_pack_ && M % (2 * G) == 0 && 2 * G * period <= slot_count()) G *= 2;
        Ct cur = z;
        int p = period, m = M;
        for (int g = 1; g < G; g *= 2, p *= 2, m /= 2) {
            const int h = m / 2;
            Ct nz = alloc_ct(0, per * h, h);
            copy_meta(nz, cur);
            nz.nb = h;
            launch_fma_poly(S(), T_, nz.data, cur.data, cur.data + (size_t)h * per * nl0 * n, monomial(n / (4 * p)), per * h * nl0, nl0,
                            qmap());
            release(cur);
            cur = nz;
        }
        SparseBoot* sv = p < slot_count() ? &sparse_variant(p) : nullptr;
        Ct out = boot_stack(cur, gain / G, sv);  // consumes cur
        cnt_[C_BOOT] += M - M / G;               // boot_stack counted one per packed member
        for (; m < M; m *= 2) {
            p /= 2;
            Ct hi, lo;
            mono_split(out, p, hi, lo);
            release(out);
            const int nlo = hp_.nl(hi.level), ph = pm(hi);
            Ct cat = alloc_ct(hi.level, ph * 2 * m, 2 * m);
            copy_meta(cat, hi);
            cat.nb = 2 * m;
            const size_t half = (size_t)m * ph * nlo;
            launch_copy_rows(S(), T_, cat.data, hi.data, half);
            launch_copy_rows(S(), T_, cat.data + half * n, lo.data, half);
            release(hi);
            release(lo);
            out = cat;
        }
        return out;
    }
    // NTT form of the monomial X^e (X^N = -1, e in [0, 2N)) on every Q limb: the product by
    // it is exact (coefficients shifted, the wrapped ones negated; no level, no noise)
    std::map<int, u32*> mono_;
    const u32* monomial(int e) {
        auto it = mono_.find(e);
        if (it != mono_.end()) return it->second;
        const int n = hp_.n, nq = hp_.n_q;
        std::vector<u32> h((size_t)nq * n, 0u);
        for (int t = 0; t < nq; ++t) h[(size_t)t * n + e % n] = (e / n) % 2 ? hp_.mod[t] - 1 : 1u;
        u32* d = dev_alloc((size_t)nq * n);
        HIP_OK(hipMemcpy(d, h.data(), h.size() * sizeof(u32), hipMemcpyHostToDevice));
        ntt(d, nq, nq, qmap());
        HIP_OK(hipStreamSynchronize(S()));
        mono_[e] = d;
        return d;
    }
    // z: level-0 ciphertext(s), nb batched members, consumed here
    Ct bootstrap_l0(Ct z, int stop_after, double gain = 1.0, SparseBoot* sv = nullptr) {
        const int n = hp_.n, top = sv ? sv->top : bs_.top, nb = z.nb;
        // 1. scale delta_0 -> s_bt = Q0 / 2^b (an exact integer product) on the two
        // base limbs: the ciphertext stays modulo Q0 = q0 q1 (no rescale, no rounding noise)
        const int nq = kD2sQ;
        if (hp_.nl(0) != nq) throw std::runtime_error("bootstrap: level 0 must hold the two base limbs");
        std::vector<u32> r(nq);
        if (!(gain > 0.0 && gain <= 1.0)) throw std::runtime_error("bootstrap: gain must lie in (0, 1]");
        const i64 k1 = gain == 1.0 ? bs_.k1 : std::llround(gain * (double)bs_.k1);
        for (int t = 0; t < nq; ++t) r[t] = mod_i64(k1, hp_.mod[t]);
        launch_mul_const_half(S(), T_, z.data, z.data, const_half(r, r), z.npoly * nq, nq, qmap());
        if (stop_after == 1) return z;
        // 2. sparse-secret encapsulation: dense s -> sparse s_sp at modulus Q0
        Ct sp = keyswitch_d2s(z.data + (size_t)nq * n, z.data, nb, (size_t)2 * nq * n);
        release(z);
        if (stop_after == 2) return sp;
        // 3. ModRaise: centred CRT lift of both polynomials to every limb of the top level
        intt(sp.data, 2 * nb * nq, nq, qmap());
        Ct raised = alloc_ct(top, 2 * nb, nb);
        launch_crt2_spread(S(), T_, raised.data, sp.data, 2 * nb, hp_.nl(top), hp_.mod[0], hp_.mod[1]);
        release(sp);
        const int nlt = hp_.nl(top);
        ntt(raised.data, 2 * nb * nlt, nlt, qmap());
        if (stop_after == 3) return raised;
        // 4. back to the dense secret (sparse: fused into the first trace step, s2d_trace4)
        const size_t tms = (size_t)2 * nlt * n;
        const bool fuse_s2d = sv && s2d_trace_ && trace4_ && 4 * sv->n <= slot_count() && stop_after != 12;
        Ct u = fuse_s2d ? s2d_trace4(raised, sv->n)
                        : keyswitch(raised.data + (size_t)nlt * n, top, ksk(tag_s2d()), raised.data, nullptr, nb, tms, tms);
        release(raised);
        if (stop_after == 12) return u;  // debug: back on the dense secret, before the sparse trace
        // 4b. sparse: the trace to the subring, x += rot(x, n 2^i) for 2^i < M / n (the overflow's
        // components outside the subring cancel, the rest is multiplied by M / n)
        if (sv)
            for (int st = fuse_s2d ? 4 * sv->n : sv->n; st < slot_count();) {
                if (trace4_ && 4 * st <= slot_count()) {  // two doublings at once (hoisted)
                    Ct s4 = trace4(u, st);
                    release(u);
                    u = s4;
                    st *= 4;
                    continue;
                }
                Ct r = rotate(u, -st);
                Ct s2 = add_sub(u, r, false);
                release(r);
                release(u);
                u = s2;
                st *= 2;
            }
        if (stop_after == 4) return u;
        // 5. CoeffToSlot (bit-reversed coefficient halves / (2 q0 K))
        Ct w = lin_transform(u, sv ? sv->cts : bs_.cts);
        release(u);
        if (stop_after == 5) return w;
        if (sv && sv->pair4 && nb == 2) {
            // pair-packed sparse form: lo rotated right by 2n beside hi, w'' + conj(w'') =
            // (2 Re hi | 2 Im hi | 2 Re lo | 2 Im lo) per 4n block, ONE EvalMod for both, and
            // SlotToCoeff's first group in its hi / lo forms
            const int lv = w.level, nlw = hp_.nl(lv);
            Ct half[2];
            for (int m = 0; m < 2; ++m) {
                half[m] = alloc_ct(lv, 2);
                copy_meta(half[m], w);
                half[m].nb = 1;
                launch_copy_rows(S(), T_, half[m].data, w.data + (size_t)m * 2 * nlw * n, 2 * nlw);
            }
            release(w);
            Ct wr = rotate(half[1], 2 * sv->n);
            release(half[1]);
            Ct ws = add_sub(half[0], wr, false);
            release(half[0]);
            release(wr);
            Ct cj = conjugate(ws);
            Ct v = add_sub(ws, cj, false);
            release(ws);
            release(cj);
            Ct f = eval_mod(v);
            release(v);
            Ct oh = lin_group(f, sv->stc[0]), ol = lin_group(f, sv->stc_lo);
            release(f);
            const int nlo = hp_.nl(oh.level);
            Ct st = alloc_ct(oh.level, 4, 2);
            copy_meta(st, oh);
            st.nb = 2;
            launch_copy_rows(S(), T_, st.data, oh.data, 2 * nlo);
            launch_copy_rows(S(), T_, st.data + (size_t)2 * nlo * n, ol.data, 2 * nlo);
            release(oh);
            release(ol);
            for (size_t k = 1; k < sv->stc.size(); ++k) {
                Ct nx = lin_group(st, sv->stc[k]);
                release(st);
                st = nx;
            }
            cnt_[C_BOOT] += nb;
            if (st.level > hp_.fresh) {
                Ct o = level_down(st, hp_.fresh);
                release(st);
                st = o;
            }
            return st;
        }
        if (sv && sv->packed) {
            // packed sparse form: w' + conj(w') = (Re w | Im w) per 2n block, one EvalMod, and
            // SlotToCoeff's first group recombines the halves
            Ct cj = conjugate(w);
            Ct v = add_sub(w, cj, false);
            release(w);
            release(cj);
            if (stop_after <= 9) return v;
            Ct f = eval_mod(v);
            release(v);
            if (stop_after == 10) return f;
            Ct out = lin_transform(f, sv->stc);
            release(f);
            cnt_[C_BOOT] += nb;
            if (out.level > hp_.fresh) {
                Ct o = level_down(out, hp_.fresh);
                release(out);
                out = o;
            }
            return out;
        }
        // 6. real / imaginary parts (exact: conjugation, add, multiply by -i)
        Ct cj = conjugate(w);
        Ct re = add_sub(w, cj, false);
        Ct dif = add_sub(w, cj, true);
        release(w);
        release(cj);
        Ct im = mul_scalar(dif, 0.0, -1.0);
        release(dif);
        if (stop_after == 6) return release(im), re;
        if (stop_after == 7) return release(re), im;
        // 7. EvalMod on both halves: stacked into ONE batched ciphertext (2 nb members) so
        // every key switch of the polynomial evaluation reads its key once for both halves
        Ct fre, fim;
        // (eval_mod_many({re, im}) is bit-exact with the stacked form below but measured no faster:
        // the stacked halves already share every key read; profiles/r2_evalmod_batch_ab.json)
        if (stop_after > 9 && stack_evalmod_ && 2 * nb <= std::min(4, ks_chunk(re.level)) && re.level == im.level && re.pend == im.pend &&
            !re.lazy && !im.lazy && pm(re) == 2 && pm(im) == 2 && re.ntt == im.ntt) {
            Ct st = alloc_ct(re.level, re.npoly + im.npoly, 2 * nb);
            st.ntt = re.ntt, st.pend = re.pend;
            launch_copy_rows(S(), T_, st.data, re.data, re.words / n);
            launch_copy_rows(S(), T_, st.data + re.words, im.data, im.words / n);
            release(re);
            release(im);
            Ct f = eval_mod(st);
            release(st);
            Ct* half[2] = {&fre, &fim};
            for (int h = 0; h < 2; ++h) {
                Ct& o = *half[h];
                o = alloc_ct(f.level, f.npoly / 2, nb);
                copy_meta(o, f);
                o.nb = nb;
                launch_copy_rows(S(), T_, o.data, f.data + h * o.words, o.words / n);
            }
            release(f);
        } else {
            fre = eval_mod(re);
            release(re);
            if (stop_after == 8) return release(im), fre;
            fim = eval_mod(im);
            release(im);
            if (stop_after == 9) return release(fre), fim;
        }
        Ct ifim = mul_scalar(fim, 0.0, 1.0);
        release(fim);
        Ct wp = add_sub(fre, ifim, false);
        release(fre);
        release(ifim);
        if (stop_after == 10) return wp;
        // 8. SlotToCoeff (scaled back to the message)
        Ct out = lin_transform(wp, sv ? sv->stc : bs_.stc);
        release(wp);
        cnt_[C_BOOT] += nb;
        if (out.level > hp_.fresh) {  // a sparse plan's SlotToCoeff ends above the fresh level
            Ct o = level_down(out, hp_.fresh);
            release(out);
            out = o;
        }
        return out;
    }

    // ------------------------------------------------------------------ raw access
    void export_ct(aesfhe_handle h, u32* out, u64 words) {
        const Ct& c0 = canon(h);
        Ct c = ensure_ntt(c0);
        if (words < c.words) throw std::runtime_error("export buffer too small");
        HIP_OK(hipMemcpyAsync(out, c.data, c.words * sizeof(u32), hipMemcpyDeviceToHost, S()));
        HIP_OK(hipStreamSynchronize(S()));
        if (c.data != c0.data) release(c);
    }
    aesfhe_handle import_ct(int level, int npoly, const u32* data) {
        if (level < -1 || level > hp_.L || npoly < 1 || npoly > 3) throw std::runtime_error("import: bad level/npoly");
        Ct c = alloc_ct(level, npoly);
        HIP_OK(hipMemcpyAsync(c.data, data, c.words * sizeof(u32), hipMemcpyHostToDevice, S()));
        HIP_OK(hipStreamSynchronize(S()));
        return put_ct(c);
    }
    void export_dev(const u32* d, size_t words, u32* out) {
        HIP_OK(hipMemcpyAsync(out, d, words * sizeof(u32), hipMemcpyDeviceToHost, S()));
        HIP_OK(hipStreamSynchronize(S()));
    }
    void export_secret(u32* out) {
        if (!d_s_) throw std::runtime_error("keys not generated");
        export_dev(d_s_, (size_t)hp_.n_tot() * hp_.n, out);
    }
    void export_pk(u32* out) {
        if (!d_pk_) throw std::runtime_error("keys not generated");
        export_dev(d_pk_, (size_t)2 * hp_.n_q * hp_.n, out);
    }
    void export_ksk(u64 g, u32* out) { export_dev(ksk(g), ksk_words(g), out); }
    void debug_ntt(u32* data, int rows, int first_prime, int inverse) {
        u32* d = tmp(rows);
        HIP_OK(hipMemcpyAsync(d, data, sizeof(u32) * rows * hp_.n, hipMemcpyHostToDevice, S()));
        LimbMap m{rows, first_prime, 0};
        if (inverse) intt(d, rows, rows, m);
        else ntt(d, rows, rows, m);
        export_dev(d, (size_t)rows * hp_.n, data);
        untmp(d, rows);
    }
    void debug_keyswitch(int level, u64 g, const u32* d_host, u32* out) {
        const int nl = hp_.nl(level);
        u32* d = tmp(nl);
        HIP_OK(hipMemcpyAsync(d, d_host, sizeof(u32) * nl * hp_.n, hipMemcpyHostToDevice, S()));
        Ct o = keyswitch(d, level, ksk(g), nullptr, nullptr);
        export_dev(o.data, o.words, out);
        release(o);
        untmp(d, nl);
    }
    // micro-benchmark of one engine primitive, back to back on the engine stream (HIP events
    // around the loop: device time incl. launch gaps).  op 0: NTT of arg rows, 1: inverse
    // NTT of arg rows, 2: key switch (relinearisation key) at level arg, 3: rescale of a
    // 2-poly ciphertext at level arg, 4: ct x ct + relinearise + rescale at level arg
    double bench_host_us_ = 0.0;  // host enqueue time per iteration of the last bench_op
    double bench_op(int op, int arg, int iters) {
        if (iters <= 0) throw std::runtime_error("bench_op: iters must be positive");
        const int n = hp_.n;
        if ((op == 0 || op == 1) && (arg <= 0 || arg > 4 * hp_.n_tot())) throw std::runtime_error("bench_op: bad row count");
        if (op >= 2 && (arg < 1 || arg > hp_.L)) throw std::runtime_error("bench_op: bad level");
        if (op > 4 || op < 0) throw std::runtime_error("bench_op: unknown op");
        const int rows = op <= 1 ? arg : 3 * hp_.nl(arg);
        u32* buf = tmp(rows);
        HIP_OK(hipMemsetAsync(buf, 0, sizeof(u32) * rows * n, S()));
        const int nl = op <= 1 ? std::min(arg, hp_.n_q) : hp_.nl(arg);
        Ct c;
        c.data = buf, c.level = op <= 1 ? 0 : arg, c.npoly = 2, c.ntt = true, c.words = (size_t)2 * nl * n;
        auto run = [&]() {
            if (op == 0) ntt(buf, buf, arg, rows_dense(nl), qmap());
            else if (op == 1) intt(buf, buf, arg, rows_dense(nl), qmap());
            else if (op == 2) release(keyswitch(buf + (size_t)2 * nl * n, arg, ksk(0), buf, buf + (size_t)nl * n));
            else if (op == 3) release(rescale(c));
            else release(mul(c, c, true));
        };
        run();
        hipEvent_t a, b;
        HIP_OK(hipEventCreate(&a));
        HIP_OK(hipEventCreate(&b));
        HIP_OK(hipEventRecord(a, S()));
        const auto h0 = std::chrono::steady_clock::now();
        for (int i = 0; i < iters; ++i) run();
        bench_host_us_ = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count() / iters;
        HIP_OK(hipEventRecord(b, S()));
        HIP_OK(hipEventSynchronize(b));
        float ms = 0.f;
        HIP_OK(hipEventElapsedTime(&ms, a, b));
        (void)hipEventDestroy(a);
        (void)hipEventDestroy(b);
        untmp(buf, rows);
        return 1000.0 * ms / iters;
    }
    u64 counter(int i) const { return i < C_N ? cnt_[i] : 0; }
    bool lazy() const { return lazy_; }
    void prof_every(int every) {
        if (every < 1) throw std::runtime_error("profile_every must be >= 1");
        prof_.every = (unsigned)every;
    }
    void set_lazy(bool on) { lazy_ = on; }
    void reset_counters() {
        std::memset(cnt_, 0, sizeof(cnt_));
        std::memset(lvl_cnt_, 0, sizeof(lvl_cnt_));
    }
    // per-level work tallies (aesfhe_level_counters): the CPU baseline replays a bootstrap's key
    // switches, ct x ct products and diagonal products on the C oracle at the levels they ran at
    enum LevelTally { LV_KS, LV_MUL, LV_PTMUL, LV_N };
    static constexpr int kLvMax = 64;
    u64 level_counter(int kind, int level) const { return kind >= 0 && kind < LV_N && level >= 0 && level < kLvMax ? lvl_cnt_[kind][level] : 0; }

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
        std::vector<uint2> tw((size_t)nt * n), itw((size_t)nt * n);
        im_.resize(nt);
        for (int i = 0; i < nt; ++i) {
            const u32 q = hp_.mod[i], w = hp_.psi[i], iw = hinvm(w, q);
            pc[i].q = q;
            pc[i].mu = barrett_pre(q);
            pc[i].ninv = hinvm((u32)n % q, q);
            pc[i].ninv_p = shoup_pre(pc[i].ninv, q);
            pc[i].im = hpowm(w, n / 2, q);
            pc[i].im_p = shoup_pre(pc[i].im, q);
            pc[i].r32 = (u32)((1ull << 32) % q);
            im_[i] = pc[i].im;
            u64 p = 1, ip = 1;
            for (int k = 0; k < n; ++k) {
                const u32 r = hbitrev((u32)k, logn);
                const size_t at = (size_t)i * n + r;
                tw[at] = make_uint2(0u - (u32)p, shoup_pre((u32)p, q));  // -w mod 2^32 (ntt.hip ct_bfly)
                itw[at] = make_uint2((u32)ip, shoup_pre((u32)ip, q));
                p = p * w % q;
                ip = ip * iw % q;
            }
        }
        // the inverse pass 2's factored twiddles (ntt.hip k_ntt2_inv): stage s, row R, word
        // offset t: psi^-(2^(7-s) (2 brv(R) + 1)) * psi^-((N / 2^s) brv_s(t)) = itw[2^(logn-8+s) + R 2^s + t]
        const int r1 = n >> 8, logr1 = logn - 8;
        std::vector<uint2> irow((size_t)nt * r1 * 4, make_uint2(0u, 0u)), igam((size_t)nt * 256, make_uint2(0u, 0u));
        for (int i = 0; i < nt; ++i) {
            const u32 q = hp_.mod[i], iw = hinvm(hp_.psi[i], q);
            for (int R = 0; R < r1; ++R)
                for (int s = 5; s <= 7; ++s) {
                    const u32 v = hpowm(iw, (uint64_t)(1u << (7 - s)) * (2u * hbitrev((u32)R, logr1) + 1u), q);
                    irow[((size_t)i * r1 + R) * 4 + (s - 5)] = make_uint2(v, shoup_pre(v, q));
                }
            for (int s = 5; s <= 7; ++s)
                for (int t = 0; t < (1 << s); ++t) {
                    const u32 v = hpowm(iw, (uint64_t)(n >> s) * hbitrev((u32)t, s), q);
                    igam[(size_t)i * 256 + (1 << s) + t] = make_uint2(v, shoup_pre(v, q));
                }
        }
        T_.pc = dev_upload(pc);
        T_.tw = dev_upload(tw);
        T_.itw = dev_upload(itw);
        T_.irow = dev_upload(irow);
        T_.igam = dev_upload(igam);
        T_.logn = logn;

        const auto& q = hp_.mod;
        auto mulm = [](u64 a, u64 b, u32 m) { return (u32)(a % m * (b % m) % m); };
        // rescale: per dropped limb r >= 1, q_r^{-1} mod q_t for t < r
        std::vector<u32> rq;
        rescale_off_.assign(hp_.n_q, 0);
        for (int r = 1; r < hp_.n_q; ++r) {
            rescale_off_[r] = rq.size();
            const u32 qr = q[r];
            for (int t = 0; t < r; ++t) {
                const u32 v = hinvm(qr % q[t], q[t]);
                rq.push_back(v);
                rq.push_back(shoup_pre(v, q[t]));
            }
        }
        d_rescale_qinv_ = dev_upload(rq);
        // double rescale: dropping limbs r and r + 1 at once, (q_r q_{r+1})^{-1} mod q_t, t < r
        rq.clear();
        rescale2_off_.assign(hp_.n_q, 0);
        for (int r = 1; r + 1 < hp_.n_q; ++r) {
            rescale2_off_[r] = rq.size();
            for (int t = 0; t < r; ++t) {
                const u32 v = hinvm(mulm(q[r], q[r + 1], q[t]), q[t]);
                rq.push_back(v);
                rq.push_back(shoup_pre(v, q[t]));
            }
        }
        d_rescale2_qinv_ = dev_upload(rq);

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
        modup_off_.assign((size_t)(hp_.n_ks + 1) * hp_.dnum, 0);  // indexed by limb count nl = 1..n_ks
        for (int nl = 1; nl <= hp_.n_ks; ++nl) {
            const int ne = nl + hp_.n_p;
            for (int j = 0; j < hp_.dnum; ++j) {
                const int lo = j * hp_.alpha;
                modup_off_[(size_t)nl * hp_.dnum + j] = mu.size();
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
        // the same qhat^-1 pairs per limb count, limb by limb across the digits (the ModUp INTT's
        // post factors when the conversion is fused into the NTT: ntt.hip k_ntt1_fwd_conv)
        std::vector<u32> mq;
        modup_qh_off_.assign((size_t)hp_.n_ks + 1, 0);
        for (int nl = 1; nl <= hp_.n_ks; ++nl) {
            modup_qh_off_[nl] = mq.size();
            for (int j = 0; j * hp_.alpha < nl; ++j) {
                const int lo = j * hp_.alpha, h = std::min(hp_.alpha, nl - lo), ne = nl + hp_.n_p;
                const size_t at = modup_off_[(size_t)nl * hp_.dnum + j] + (size_t)2 * h * ne;
                for (int i = 0; i < 2 * h; ++i) mq.push_back(mu[at + i]);
            }
        }
        d_modup_qh_ = dev_upload(mq);

        // ModDown tables per level: [np][nl] Shoup pairs of phat_k mod q_t; phat_k^{-1} mod p_k; P^{-1} mod q_t
        std::vector<u32> md;
        moddown_off_.assign(hp_.n_ks + 1, 0);  // indexed by limb count nl = 1..n_ks
        const int np = hp_.n_p;
        for (int nl = 1; nl <= hp_.n_ks; ++nl) {
            moddown_off_[nl] = md.size();
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

        // ModDown fused with the rescale, per level l (sources: the k = nl(l) - nl(l-1) dropped
        // limbs, then P; Q' their product; r = nl(l-1) targets): [h][r] pairs of Q'/s_i mod q_t,
        // [h] pairs of (Q'/s_i)^{-1} mod s_i, [r] values of -Q' mod q_t, [r] pairs of Q'^{-1} mod q_t
        std::vector<u32> mdr;
        mdr_off_.assign(hp_.L + 1, SIZE_MAX);
        for (int l = 1; l <= hp_.L; ++l) {
            const int nl = hp_.nl(l), r = hp_.nl(l - 1), k = nl - r, h = k + np;
            if (nl > hp_.n_ks || k < 1 || h > kMaxConvH) continue;
            std::vector<u32> src;
            for (int i = 0; i < k; ++i) src.push_back(q[r + i]);
            for (int i = 0; i < np; ++i) src.push_back(q[hp_.p_off() + i]);
            mdr_off_[l] = mdr.size();
            for (int i = 0; i < h; ++i)
                for (int t = 0; t < r; ++t) {
                    u32 v = 1;
                    for (int m2 = 0; m2 < h; ++m2)
                        if (m2 != i) v = mulm(v, src[m2], q[t]);
                    mdr.push_back(v);
                    mdr.push_back(shoup_pre(v, q[t]));
                }
            for (int i = 0; i < h; ++i) {
                u32 v = 1;
                for (int m2 = 0; m2 < h; ++m2)
                    if (m2 != i) v = mulm(v, src[m2], src[i]);
                const u32 inv = hinvm(v, src[i]);
                mdr.push_back(inv);
                mdr.push_back(shoup_pre(inv, src[i]));
            }
            std::vector<u32> all(r);
            for (int t = 0; t < r; ++t) {
                u32 v = 1;
                for (int m2 = 0; m2 < h; ++m2) v = mulm(v, src[m2], q[t]);
                all[t] = v;
                mdr.push_back(v ? q[t] - v : 0);
            }
            for (int t = 0; t < r; ++t) {
                const u32 inv = hinvm(all[t], q[t]);
                mdr.push_back(inv);
                mdr.push_back(shoup_pre(inv, q[t]));
            }
        }
        d_mdr_ = dev_upload(mdr);

        // dense -> sparse key switch over q0 * P' (ksk_d2s): [P' mod q0 pair][np pairs P'/p_k mod q0]
        // [np pairs (P'/p_k)^-1 mod p_k][-P' mod q0][P'^-1 mod q0 pair]
        {  // dense -> sparse key switch over Q0 * P' (keyswitch_d2s): offsets in d2s_off_
            const int nq = kD2sQ, npd = d2s_np(), ne = nq + npd;
            auto tq = [&](int x) { return x < nq ? q[x] : q[hp_.p_off() + x - nq]; };
            std::vector<u32> t;
            auto pair_ = [&](u32 v, u32 m) { t.push_back(v), t.push_back(shoup_pre(v, m)); };
            d2s_off_.gad = t.size();  // [nq] pairs: P' mod q_t (the key's gadget)
            for (int x = 0; x < nq; ++x) {
                u32 v = 1;
                for (int k = 0; k < npd; ++k) v = mulm(v, q[hp_.p_off() + k], q[x]);
                pair_(v, q[x]);
            }
            d2s_off_.up_tab = t.size();  // [nq][ne] pairs: (Q0 / q_i) mod target x
            for (int i = 0; i < nq; ++i)
                for (int x = 0; x < ne; ++x) {
                    u32 v = 1;
                    for (int k = 0; k < nq; ++k)
                        if (k != i) v = mulm(v, q[k], tq(x));
                    pair_(v, tq(x));
                }
            d2s_off_.up_qhinv = t.size();  // [nq] pairs: (Q0 / q_i)^-1 mod q_i
            for (int i = 0; i < nq; ++i) {
                u32 v = 1;
                for (int k = 0; k < nq; ++k)
                    if (k != i) v = mulm(v, q[k], q[i]);
                pair_(hinvm(v, q[i]), q[i]);
            }
            d2s_off_.up_negq = t.size();  // [ne]: -Q0 mod target x
            for (int x = 0; x < ne; ++x) {
                u32 v = 1;
                for (int k = 0; k < nq; ++k) v = mulm(v, q[k], tq(x));
                t.push_back(v ? tq(x) - v : 0);
            }
            d2s_off_.dn_tab = t.size();  // [np][nq] pairs: (P' / p_k) mod q_t
            for (int k = 0; k < npd; ++k)
                for (int x = 0; x < nq; ++x) {
                    u32 v = 1;
                    for (int m2 = 0; m2 < npd; ++m2)
                        if (m2 != k) v = mulm(v, q[hp_.p_off() + m2], q[x]);
                    pair_(v, q[x]);
                }
            d2s_off_.dn_qhinv = t.size();  // [np] pairs: (P' / p_k)^-1 mod p_k
            for (int k = 0; k < npd; ++k) {
                const u32 pk = q[hp_.p_off() + k];
                u32 v = 1;
                for (int m2 = 0; m2 < npd; ++m2)
                    if (m2 != k) v = mulm(v, q[hp_.p_off() + m2], pk);
                pair_(hinvm(v, pk), pk);
            }
            d2s_off_.dn_negq = t.size();  // [nq]: -P' mod q_t
            for (int x = 0; x < nq; ++x) {
                u32 v = 1;
                for (int k = 0; k < npd; ++k) v = mulm(v, q[hp_.p_off() + k], q[x]);
                t.push_back(v ? q[x] - v : 0);
            }
            d2s_off_.pinv = t.size();  // [nq] pairs: P'^-1 mod q_t
            for (int x = 0; x < nq; ++x) {
                u32 v = 1;
                for (int k = 0; k < npd; ++k) v = mulm(v, q[hp_.p_off() + k], q[x]);
                pair_(hinvm(v, q[x]), q[x]);
            }
            d_d2s_ = dev_upload(t);
        }

    }

    HostParams hp_;
    Embedding emb_;
    DevTables T_;
    // stream 0 carries the caller's work; streams 1..kStreams-1 carry the branches of a
    // fork/join section (aesfhe_fork / aesfhe_join), each bound to one host thread
    hipStream_t streams_[kStreams] = {};
    hipEvent_t fj_ev_[kStreams] = {};
    Pool pools_[kStreams];
    std::vector<std::pair<u32*, size_t>> deferred_;  // handle frees from branch threads
    int device_ = 0;

    std::vector<void*> owned_;
    std::unordered_map<aesfhe_handle, Ct> cts_;
    std::unordered_map<aesfhe_handle, Pt> pts_;
    aesfhe_handle next_ = 1;
    u32* d_s_ = nullptr;
    u32* d_pk_ = nullptr;
    u32* d_ssp_ = nullptr;
    std::map<u64, u32*> ksk_;
    u64 enc_ctr_ = 0;
    u64 enc_nonce_ = 0;  // see enc_key()
    std::vector<u32> im_;
    u32* d_rescale_qinv_ = nullptr;
    u32* d_rescale2_qinv_ = nullptr;
    std::vector<size_t> rescale2_off_;
    std::vector<size_t> rescale_off_;
    u32* d_gadget_ = nullptr;
    u32* d_modup_ = nullptr;
    std::vector<size_t> modup_off_;
    u32* d_modup_qh_ = nullptr;
    std::vector<size_t> modup_qh_off_;
    u32* d_moddown_ = nullptr;
    u32* d_moddown_phinv_ = nullptr;
    std::vector<size_t> moddown_off_;
    u32* d_mdr_ = nullptr;       // ModDown fused with the rescale, per level (see build_tables)
    u32* d_d2s_ = nullptr;       // dense -> sparse key switch constants over Q0 * P' (see build_tables)
    struct { size_t gad, up_tab, up_qhinv, up_negq, dn_tab, dn_qhinv, dn_negq, pinv; } d2s_off_{};
    std::vector<size_t> mdr_off_;
    bool batch_ops_ = std::getenv("AESFHE_BATCH_OPS") == nullptr || std::getenv("AESFHE_BATCH_OPS")[0] != '0';
    bool stack_evalmod_ = std::getenv("AESFHE_STACK_EVALMOD") == nullptr || std::getenv("AESFHE_STACK_EVALMOD")[0] != '0';
    bool fused_baby_ = std::getenv("AESFHE_FUSED_BABY") == nullptr || std::getenv("AESFHE_FUSED_BABY")[0] != '0';
    bool giant_batch_ = std::getenv("AESFHE_GIANT_BATCH") == nullptr || std::getenv("AESFHE_GIANT_BATCH")[0] != '0';
    bool double_hoist_ = std::getenv("AESFHE_DOUBLE_HOIST") == nullptr || std::getenv("AESFHE_DOUBLE_HOIST")[0] != '0';
    // sparse-plan diagonals as 2 dn residues per limb (group_pts; AESFHE_COMPACT_DIAG=0: full rows of
    // the same projected diagonals -- bit-identical results, the A/B and the check of the run structure)
    bool compact_diag_ = std::getenv("AESFHE_COMPACT_DIAG") == nullptr || std::getenv("AESFHE_COMPACT_DIAG")[0] != '0';
    // mul_many: products relinearised straight from their factors (relin_rescale_tensor; AESFHE_FUSED_TENSOR=0: tensor first)
    bool fused_tensor_ = std::getenv("AESFHE_FUSED_TENSOR") == nullptr || std::getenv("AESFHE_FUSED_TENSOR")[0] != '0';
    // EvalMod's 2 T^2 - 1 in the product's relinearisation finish (AESFHE_FUSED_AFFINE=0: one lincomb each)
    bool fused_affine_ = std::getenv("AESFHE_FUSED_AFFINE") == nullptr || std::getenv("AESFHE_FUSED_AFFINE")[0] != '0';
    // conjugations as reversed reads, no permuted copy (galois / galois_lazy; AESFHE_CONJ_REV=0: k_automorph first)
    bool conj_rev_ = std::getenv("AESFHE_CONJ_REV") == nullptr || std::getenv("AESFHE_CONJ_REV")[0] != '0';
    bool fuse_rr_ = std::getenv("AESFHE_FUSED_RESCALE") == nullptr || std::getenv("AESFHE_FUSED_RESCALE")[0] != '0';
    u32* d_pinv_ = nullptr;
    u32* d_negp_ = nullptr;
    u64 cnt_[C_N] = {};
    u64 lvl_cnt_[LV_N][kLvMax] = {};
    void tally(int kind, int level, u64 n) {
        if (level >= 0 && level < kLvMax) lvl_cnt_[kind][level] += n;
    }
    CrtConsts crt_[4] = {};
    std::unordered_map<aesfhe_handle, Lut> luts_;
    Slot16 slots_ = {};    // the reference layout's 16 state slots, 5^(i N/32)
    Slot32 slots32_ = {};  // the first 32 slots, 5^j (the packed period-32 form)
    // AESFHE_RENORM_DIRECT32=0: the packed renorms through the FFT codec (A/B runs)
    bool direct32_ = !(std::getenv("AESFHE_RENORM_DIRECT32") && std::atoi(std::getenv("AESFHE_RENORM_DIRECT32")) == 0);
    Slot16 slots_p_ = {};  // the 16-periodic layout's, 5^i
    double* d_codec_[kStreams] = {};
    int codec_flip_[kStreams] = {};  // which of the stream's two accumulators the next decode uses
    bool snap_encode_ = !(std::getenv("AESFHE_SNAP_ENCODE") && std::atoi(std::getenv("AESFHE_SNAP_ENCODE")) == 0);
    int* d_nib_[kStreams] = {};
    double* d_fft_[kStreams] = {};  // slot-packed renorm: [2 buffers][2 cts][N] complex double
    u32* d_slot_pos_ = nullptr;     // (5^j mod 2N - 1) / 2 for slot j < N/2
    u32* d_s2_ = nullptr;
    bool lazy_ = true;  // defer relinearisation / rescales of API-level products

public:
    KernelProfiler prof_;
    void activate() { prof_set(&prof_); }
};
thread_local int Engine::t_sidx = 0;

}  // namespace

// =====================================================================================
// C ABI
// =====================================================================================
// One engine may be driven by several host threads (one per stream, aesfhe_bind_stream):
// every call holds the context mutex while it queues work; errors are per thread.
struct aesfhe_ctx {
    std::unique_ptr<Engine> eng;
    std::recursive_mutex mu;
};
static thread_local std::string t_err;

#define API_BEGIN                                      \
    if (!ctx) return -2;                               \
    g_census_op = __func__;                            \
    std::lock_guard<std::recursive_mutex> lock_(ctx->mu); \
    if (ctx->eng) ctx->eng->activate();                \
    try {
#define API_END                                        \
    if (ctx->eng) ctx->eng->end_call();                \
    return 0;                                          \
    }                                                  \
    catch (const std::exception& e) {                  \
        t_err = e.what();                              \
        if (ctx->eng) ctx->eng->end_call();            \
        return -1;                                     \
    }

extern "C" {

static int create_keyed(aesfhe_ctx** out, int log_n, int max_level, int dnum, int device_id, const u32 key[8], int boot) {
    *out = nullptr;
    auto* c = new aesfhe_ctx();
    *out = c;
    try {
        if (boot) {
            const int L1 = max_level + Engine::kBootStc - 1;
            c->eng.reset(new Engine(log_n, L1, Engine::boot_double_levels(), dnum, device_id, key));
            c->eng->set_fresh(max_level);
        } else {
            c->eng.reset(new Engine(log_n, max_level, 0, dnum, device_id, key));
        }
    } catch (const std::exception& e) {
        t_err = e.what();
        return -1;
    }
    return 0;
}
int aesfhe_create(aesfhe_ctx** out, int log_n, int max_level, int dnum, int device_id, uint64_t seed) {
    u32 key[8];
    seed_key(seed, key);
    return create_keyed(out, log_n, max_level, dnum, device_id, key, 0);
}
int aesfhe_create_boot(aesfhe_ctx** out, int log_n, int fresh_level, int dnum, int device_id, uint64_t seed) {
    u32 key[8];
    seed_key(seed, key);
    return create_keyed(out, log_n, fresh_level, dnum, device_id, key, 1);
}
int aesfhe_create_keyed(aesfhe_ctx** out, int log_n, int max_level, int dnum, int device_id, const uint8_t* key, int bootstrappable) {
    u32 k[8];
    for (int i = 0; i < 8; ++i)
        k[i] = (u32)key[4 * i] | ((u32)key[4 * i + 1] << 8) | ((u32)key[4 * i + 2] << 16) | ((u32)key[4 * i + 3] << 24);
    return create_keyed(out, log_n, max_level, dnum, device_id, k, bootstrappable);
}
int aesfhe_level_limbs(aesfhe_ctx* ctx, int32_t* out) {
    API_BEGIN const HostParams& p = ctx->eng->hp();
    for (int l = 0; l <= p.L; ++l) out[l] = p.nl(l);
    API_END
}
int aesfhe_destroy(aesfhe_ctx* ctx) {
    delete ctx;
    return 0;
}
const char* aesfhe_last_error(aesfhe_ctx* ctx) { return ctx ? t_err.c_str() : "null context"; }
int aesfhe_streams(aesfhe_ctx* ctx) { return ctx && ctx->eng ? Engine::streams() : -1; }
int aesfhe_bind_stream(aesfhe_ctx* ctx, int index) {
    API_BEGIN ctx->eng->bind_stream(index);
    API_END
}
int aesfhe_settle(aesfhe_ctx* ctx, aesfhe_handle c) {
    API_BEGIN(void) ctx->eng->canon(c);
    API_END
}
int aesfhe_fork(aesfhe_ctx* ctx) {
    API_BEGIN ctx->eng->fork();
    API_END
}
int aesfhe_join(aesfhe_ctx* ctx) {
    API_BEGIN ctx->eng->join();
    API_END
}
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
    // deferred work is invisible: a lazy tensor shows its logical level and 2 polynomials;
    // an explicitly unrelinearised product shows its data level and 3 polynomials
    *level = c.lazy ? c.level - c.pend : c.level;
    *npoly = c.lazy ? 2 : c.npoly;
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
    CT_OP(e.mul_scalar(e.ct(c), re, im, e.lazy()))
}
int aesfhe_mul_pt(aesfhe_ctx* ctx, aesfhe_handle c, aesfhe_handle p, aesfhe_handle* out) { CT_OP(e.mul_pt(e.ct(c), p, e.lazy())) }
int aesfhe_mul(aesfhe_ctx* ctx, aesfhe_handle a, aesfhe_handle b, int relin, aesfhe_handle* out) {
    CT_OP(e.mul(e.canon(a), e.canon(b), relin != 0, e.lazy()))
}
int aesfhe_lut_create(aesfhe_ctx* ctx, int n_a, int n_b, const double* re, const double* im, double c0_re, double c0_im,
                      aesfhe_handle* out) {
    API_BEGIN* out = ctx->eng->lut_create(n_a, n_b, re, im, c0_re, c0_im);
    API_END
}
int aesfhe_lut_eval(aesfhe_ctx* ctx, aesfhe_handle lut, const aesfhe_handle* a, const aesfhe_handle* b, aesfhe_handle* out) {
    CT_OP(e.lut_eval(lut, a, b))
}
int aesfhe_lut_free(aesfhe_ctx* ctx, aesfhe_handle lut) {
    API_BEGIN ctx->eng->free_lut(lut);
    API_END
}
int aesfhe_set_enc_nonce(aesfhe_ctx* ctx, uint64_t nonce) {
    API_BEGIN ctx->eng->set_enc_nonce(nonce);
    API_END
}
int aesfhe_set_lazy(aesfhe_ctx* ctx, int on) {
    API_BEGIN ctx->eng->set_lazy(on != 0);
    API_END
}
int aesfhe_relinearize(aesfhe_ctx* ctx, aesfhe_handle c, aesfhe_handle* out) { CT_OP(e.relinearize(e.ct(c))) }
int aesfhe_rescale(aesfhe_ctx* ctx, aesfhe_handle c, aesfhe_handle* out) {
    API_BEGIN Engine& e = *ctx->eng;
    const Ct& c0 = e.canon(c);
    Ct x = e.normalize(c0, false);
    Ct o = e.rescale(x);
    if (x.data != c0.data) e.release(x);
    *out = e.put_ct(o);
    API_END
}
int aesfhe_level_down(aesfhe_ctx* ctx, aesfhe_handle c, int level, aesfhe_handle* out) { CT_OP(e.level_down(e.canon(c), level)) }
int aesfhe_rotate(aesfhe_ctx* ctx, aesfhe_handle c, int steps, aesfhe_handle* out) { CT_OP(e.rotate(e.canon(c), steps)) }
int aesfhe_conjugate(aesfhe_ctx* ctx, aesfhe_handle c, aesfhe_handle* out) { CT_OP(e.conjugate(e.ct(c))) }
int aesfhe_rotate_hoisted(aesfhe_ctx* ctx, aesfhe_handle c, int n, const int* steps, aesfhe_handle* out) {
    API_BEGIN Engine& e = *ctx->eng;
    if (n < 0 || (n > 0 && (!steps || !out))) throw std::runtime_error("rotate_hoisted: bad arguments");
    std::vector<Ct> r = e.rotate_hoisted(e.canon(c), std::vector<int>(steps, steps + n));
    for (int i = 0; i < n; ++i) out[i] = e.put_ct(r[i]);
    API_END
}
int aesfhe_mul_many(aesfhe_ctx* ctx, int n, const aesfhe_handle* a, const aesfhe_handle* b, aesfhe_handle* out) {
    API_BEGIN Engine& e = *ctx->eng;
    if (n < 0 || (n > 0 && (!a || !b || !out))) throw std::runtime_error("mul_many: bad arguments");
    std::vector<const Ct*> A(n), B(n);
    for (int i = 0; i < n; ++i) A[i] = &e.canon(a[i]), B[i] = &e.canon(b[i]);
    std::vector<Ct> r = e.mul_many(A, B);
    for (int i = 0; i < n; ++i) out[i] = e.put_ct(r[i]);
    API_END
}
int aesfhe_renorm_pool(aesfhe_ctx* ctx, int size) {
    API_BEGIN ctx->eng->renorm_pool(size);
    API_END
}
int aesfhe_set_stack_pack(aesfhe_ctx* ctx, int members) {
    API_BEGIN if (members < 1) throw std::runtime_error("set_stack_pack: members >= 1");
    ctx->eng->stack_pack_ = members;
    API_END
}
int aesfhe_mul_pt_sum(aesfhe_ctx* ctx, int n, const aesfhe_handle* cts, const aesfhe_handle* pts, aesfhe_handle* out) {
    API_BEGIN Engine& e = *ctx->eng;
    if (n < 1 || !cts || !pts || !out) throw std::runtime_error("mul_pt_sum: bad arguments");
    std::vector<const Ct*> C(n);
    const std::vector<aesfhe_handle> P(pts, pts + n);
    for (int i = 0; i < n; ++i) C[i] = &e.ct(cts[i]);
    *out = e.put_ct(e.mul_pt_sum(C, P));
    API_END
}
int aesfhe_stack(aesfhe_ctx* ctx, int n, const aesfhe_handle* in, aesfhe_handle* out) {
    API_BEGIN Engine& e = *ctx->eng;
    if (n < 1 || !in || !out) throw std::runtime_error("stack: bad arguments");
    std::vector<const Ct*> C(n);
    for (int i = 0; i < n; ++i) C[i] = &e.ct(in[i]);
    *out = e.put_ct(e.stack(C));
    API_END
}
int aesfhe_unstack(aesfhe_ctx* ctx, aesfhe_handle in, int n, aesfhe_handle* out) {
    API_BEGIN Engine& e = *ctx->eng;
    const Ct& c = e.ct(in);
    if (!out || n != c.nb) throw std::runtime_error("unstack: n must equal the stack's member count");
    std::vector<Ct> r = e.unstack_all(c);
    for (int i = 0; i < n; ++i) out[i] = e.put_ct(r[i]);
    API_END
}
int aesfhe_members(aesfhe_ctx* ctx, aesfhe_handle h, int* members) {
    API_BEGIN Engine& e = *ctx->eng;
    if (!members) throw std::runtime_error("members: null output");
    *members = e.ct(h).nb;
    API_END
}
int aesfhe_galois_multi(aesfhe_ctx* ctx, int n, const aesfhe_handle* in, const uint64_t* galois, aesfhe_handle* out) {
    API_BEGIN Engine& e = *ctx->eng;
    if (n < 0 || (n > 0 && (!in || !galois || !out))) throw std::runtime_error("galois_multi: bad arguments");
    std::vector<const Ct*> C(n);
    std::vector<u64> G(galois, galois + n);
    for (int i = 0; i < n; ++i) C[i] = &e.ct(in[i]);  // deferred work is resolved inside (batched)
    std::vector<Ct> r = e.galois_multi(C, G);
    for (int i = 0; i < n; ++i) {
        if (G[i] == e.conj_galois()) e.count_conj();
        else if (G[i] != 1) e.count_rot();
        out[i] = e.put_ct(r[i]);
    }
    API_END
}
int aesfhe_conjugate_many(aesfhe_ctx* ctx, int n, const aesfhe_handle* in, aesfhe_handle* out) {
    API_BEGIN Engine& e = *ctx->eng;
    if (n < 0 || (n > 0 && (!in || !out))) throw std::runtime_error("conjugate_many: bad arguments");
    std::vector<const Ct*> C(n);
    for (int i = 0; i < n; ++i) C[i] = &e.ct(in[i]);  // deferred work resolved inside, where needed
    std::vector<Ct> r = e.conjugate_many(C);
    for (int i = 0; i < n; ++i) out[i] = e.put_ct(r[i]);
    API_END
}
int aesfhe_power_basis(aesfhe_ctx* ctx, aesfhe_handle c, int degree, aesfhe_handle* out) {
    API_BEGIN ctx->eng->power_basis(c, degree, out);
    API_END
}
int aesfhe_to_ntt(aesfhe_ctx* ctx, aesfhe_handle c, aesfhe_handle* out) { CT_OP(e.to_ntt(e.canon(c))) }
int aesfhe_to_intt(aesfhe_ctx* ctx, aesfhe_handle c, aesfhe_handle* out) { CT_OP(e.to_intt(e.canon(c))) }
int aesfhe_bootstrap(aesfhe_ctx* ctx, aesfhe_handle c, aesfhe_handle* out) { CT_OP(e.bootstrap(e.canon(c))) }
int aesfhe_bootstrap_pair(aesfhe_ctx* ctx, aesfhe_handle a, aesfhe_handle b, aesfhe_handle* out_a, aesfhe_handle* out_b) {
    API_BEGIN Engine& e = *ctx->eng;
    const Ct& ca = e.canon(a);
    const Ct& cb = e.canon(b);
    e.bootstrap_pair(ca, cb, out_a, out_b);
    API_END
}
int aesfhe_bootstrap_scaled(aesfhe_ctx* ctx, aesfhe_handle c, double gain, aesfhe_handle* out) {
    CT_OP(e.bootstrap(e.canon(c), 99, gain))
}
int aesfhe_bootstrap_pair_scaled(aesfhe_ctx* ctx, aesfhe_handle a, aesfhe_handle b, double gain, aesfhe_handle* out_a,
                                 aesfhe_handle* out_b) {
    API_BEGIN Engine& e = *ctx->eng;
    const Ct& ca = e.canon(a);
    const Ct& cb = e.canon(b);
    e.bootstrap_pair(ca, cb, out_a, out_b, gain);
    API_END
}
int aesfhe_bootstrap_sparse(aesfhe_ctx* ctx, aesfhe_handle c, int period, double gain, aesfhe_handle* out) {
    CT_OP(e.bootstrap(e.canon(c), 99, gain, period))
}
int aesfhe_bootstrap_pair_sparse(aesfhe_ctx* ctx, aesfhe_handle a, aesfhe_handle b, int period, double gain, aesfhe_handle* out_a,
                                 aesfhe_handle* out_b) {
    API_BEGIN Engine& e = *ctx->eng;
    const Ct& ca = e.canon(a);
    const Ct& cb = e.canon(b);
    e.bootstrap_pair(ca, cb, out_a, out_b, gain, period);
    API_END
}
int aesfhe_bootstrap_quad_sparse(aesfhe_ctx* ctx, const aesfhe_handle* in, int period, double gain, aesfhe_handle* out) {
    API_BEGIN Engine& e = *ctx->eng;
    if (!in || !out) throw std::runtime_error("bootstrap_quad: null handle array");
    const Ct* c[4];
    for (int m = 0; m < 4; ++m) c[m] = &e.canon(in[m]);
    aesfhe_handle* o[4] = {out, out + 1, out + 2, out + 3};
    e.bootstrap_quad_mono(c, o, gain, period);
    API_END
}
int aesfhe_bootstrap_depth(void) { return Engine::boot_depth(); }
int aesfhe_debug_boot_stage(aesfhe_ctx* ctx, aesfhe_handle c, int stage, aesfhe_handle* out) {
    // AESFHE_DEBUG_PERIOD: the stages of the sparse-slot bootstrap of that period (profiling)
    static const int period = std::getenv("AESFHE_DEBUG_PERIOD") ? std::atoi(std::getenv("AESFHE_DEBUG_PERIOD")) : 0;
    CT_OP(e.bootstrap(e.canon(c), stage, 1.0, period))
}
int aesfhe_debug_boot_stage_sparse(aesfhe_ctx* ctx, aesfhe_handle c, int stage, int period, aesfhe_handle* out) {
    CT_OP(e.bootstrap(e.canon(c), stage, 1.0, period))
}
int aesfhe_debug_sparse_group(aesfhe_ctx* ctx, aesfhe_handle c, int period, int which, int pair, aesfhe_handle* out) {
    CT_OP(e.lin_group(e.canon(c), e.debug_sparse_group(period, which, pair != 0)))
}
int aesfhe_debug_sparse_group_plain(aesfhe_ctx* ctx, int period, int which, int pair, const double* re, const double* im,
                                    double* out_re, double* out_im, int* info3) {
    API_BEGIN if (!re || !im || !out_re || !out_im || !info3) throw std::runtime_error("debug_sparse_group_plain: null buffer");
    ctx->eng->debug_sparse_group_plain(period, which, pair != 0, re, im, out_re, out_im, info3);
    API_END
}
int aesfhe_debug_mono_pack(aesfhe_ctx* ctx, aesfhe_handle a, aesfhe_handle b, int period, aesfhe_handle* out) {
    CT_OP(e.mono_pack(e.canon(a), e.canon(b), period))
}
int aesfhe_debug_mono_split(aesfhe_ctx* ctx, aesfhe_handle m, int period, aesfhe_handle* out_hi, aesfhe_handle* out_lo) {
    API_BEGIN Engine& e = *ctx->eng;
    Ct hi, lo;
    e.mono_split(e.canon(m), period, hi, lo);
    *out_hi = e.put_ct(hi);
    *out_lo = e.put_ct(lo);
    API_END
}
int aesfhe_debug_lin_group(aesfhe_ctx* ctx, aesfhe_handle c, int which, aesfhe_handle* out) {
    CT_OP(e.debug_lin_group(e.canon(c), which))
}
int aesfhe_debug_lin_group_plain(aesfhe_ctx* ctx, int which, const double* re, const double* im, double* out_re, double* out_im) {
    API_BEGIN if (!re || !im || !out_re || !out_im) throw std::runtime_error("debug_lin_group_plain: null buffer");
    ctx->eng->debug_lin_group_plain(which, re, im, out_re, out_im);
    API_END
}
int aesfhe_export_sparse(aesfhe_ctx* ctx, uint32_t* out) {
    API_BEGIN Engine& e = *ctx->eng;
    e.export_dev(e.sparse_secret(), (size_t)e.hp().n_tot() * e.hp().n, out);
    API_END
}
int aesfhe_boot_info(aesfhe_ctx* ctx, double* out) {
    API_BEGIN Engine& e = *ctx->eng;
    e.boot_setup();
    e.boot_info(out);
    API_END
}
int aesfhe_renorm_pair(aesfhe_ctx* ctx, aesfhe_handle hi, aesfhe_handle lo, aesfhe_handle* out_hi, aesfhe_handle* out_lo) {
    API_BEGIN ctx->eng->renorm_pair(hi, lo, out_hi, out_lo);
    API_END
}
int aesfhe_renorm_periodic(aesfhe_ctx* ctx, aesfhe_handle hi, aesfhe_handle lo, int period, int level, aesfhe_handle* out_hi,
                           aesfhe_handle* out_lo) {
    API_BEGIN ctx->eng->renorm_states(hi, lo, 1, out_hi, out_lo, level, period);
    API_END
}
int aesfhe_renorm_unpack(aesfhe_ctx* ctx, aesfhe_handle packed, int period, int level, aesfhe_handle* out_hi, aesfhe_handle* out_lo) {
    API_BEGIN ctx->eng->renorm_states(packed, packed, 1, out_hi, out_lo, level, 0, period);
    API_END
}
int aesfhe_renorm_unpack_perm(aesfhe_ctx* ctx, aesfhe_handle packed, aesfhe_handle packed_conj, const int32_t* perm16, int period, int level,
                              aesfhe_handle* out_hi, aesfhe_handle* out_lo) {
    API_BEGIN if (!perm16) throw std::runtime_error("renorm_unpack_perm: no permutation");
    int p[16];
    for (int i = 0; i < 16; ++i) p[i] = perm16[i];
    ctx->eng->renorm_states(packed, packed, 1, out_hi, out_lo, level, 0, period, false, 0, packed_conj, 0, false, p);
    API_END
}
int aesfhe_renorm_periodic_perm(aesfhe_ctx* ctx, aesfhe_handle hi, aesfhe_handle lo, aesfhe_handle hi_conj, aesfhe_handle lo_conj,
                                const int32_t* perm16, int pack_out, int period, int level, aesfhe_handle* out_hi, aesfhe_handle* out_lo) {
    API_BEGIN if ((hi_conj != 0) != (lo_conj != 0)) throw std::runtime_error("renorm_periodic_perm: give both conjugate partners or none");
    if (!perm16) throw std::runtime_error("renorm_periodic_perm: no permutation");
    int p[16];
    for (int i = 0; i < 16; ++i) p[i] = perm16[i];
    ctx->eng->renorm_states(hi, lo, 1, out_hi, pack_out ? nullptr : out_lo, level, period, 0, false, 0, hi_conj, lo_conj, pack_out != 0, p);
    API_END
}
int aesfhe_renorm_pack(aesfhe_ctx* ctx, aesfhe_handle hi, aesfhe_handle lo, aesfhe_handle hi_conj, aesfhe_handle lo_conj, int period, int level,
                       aesfhe_handle* out) {
    API_BEGIN if ((hi_conj != 0) != (lo_conj != 0)) throw std::runtime_error("renorm_pack: give both conjugate partners or none");
    ctx->eng->renorm_states(hi, lo, 1, out, nullptr, level, period, 0, false, 0, hi_conj, lo_conj, true);
    API_END
}
int aesfhe_renorm_periodic_conj(aesfhe_ctx* ctx, aesfhe_handle hi, aesfhe_handle lo, aesfhe_handle hi_conj, aesfhe_handle lo_conj, int period,
                                int level, aesfhe_handle* out_hi, aesfhe_handle* out_lo) {
    API_BEGIN ctx->eng->renorm_states(hi, lo, 1, out_hi, out_lo, level, period, 0, false, 0, hi_conj, lo_conj);
    API_END
}
int aesfhe_renorm_packed_conj(aesfhe_ctx* ctx, aesfhe_handle c, aesfhe_handle c_conj, int period, int level, aesfhe_handle* out) {
    API_BEGIN if (period < 16 || (period & (period - 1))) throw std::runtime_error("renorm_packed: period must be a power of two >= 16");
    ctx->eng->renorm_states(c, c, 1, out, nullptr, level, 0, 0, true, period, c_conj);
    API_END
}
int aesfhe_renorm_unpack_conj(aesfhe_ctx* ctx, aesfhe_handle packed, aesfhe_handle packed_conj, int period, int level, aesfhe_handle* out_hi,
                              aesfhe_handle* out_lo) {
    API_BEGIN ctx->eng->renorm_states(packed, packed, 1, out_hi, out_lo, level, 0, period, false, 0, packed_conj);
    API_END
}
int aesfhe_renorm_single(aesfhe_ctx* ctx, aesfhe_handle c, int level, aesfhe_handle* out) {
    API_BEGIN ctx->eng->renorm_states(c, c, 1, out, nullptr, level, 0, 0, true);
    API_END
}
int aesfhe_renorm_packed(aesfhe_ctx* ctx, aesfhe_handle c, int period, int level, aesfhe_handle* out) {
    API_BEGIN
    if (period < 16 || (period & (period - 1))) throw std::runtime_error("renorm_packed: period must be a power of two >= 16");
    ctx->eng->renorm_states(c, c, 1, out, nullptr, level, 0, 0, true, period);
    API_END
}
int aesfhe_renorm_states(aesfhe_ctx* ctx, aesfhe_handle hi, aesfhe_handle lo, int states, aesfhe_handle* out_hi,
                         aesfhe_handle* out_lo) {
    API_BEGIN ctx->eng->renorm_states(hi, lo, states, out_hi, out_lo);
    API_END
}
int aesfhe_renorm_at(aesfhe_ctx* ctx, aesfhe_handle hi, aesfhe_handle lo, int states, int level, aesfhe_handle* out_hi,
                     aesfhe_handle* out_lo) {
    API_BEGIN ctx->eng->renorm_states(hi, lo, states, out_hi, out_lo, level);
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
int aesfhe_bench_op(aesfhe_ctx* ctx, int op, int arg, int iters, double* us) {
    API_BEGIN * us = ctx->eng->bench_op(op, arg, iters);
    if (std::getenv("AESFHE_BENCH_HOST")) std::fprintf(stderr, "bench_op %d %d: gpu %.2f us, host enqueue %.2f us\n", op, arg, *us, ctx->eng->bench_host_us_);
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
int aesfhe_profile_every(aesfhe_ctx* ctx, int every) {
    API_BEGIN ctx->eng->prof_every(every);
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
int aesfhe_kernel_work(aesfhe_ctx* ctx, double* out, int n) {
    API_BEGIN KernelProfiler& p = ctx->eng->prof_;
    p.flush();
    for (int k = 0; k < n && k < KID_N; ++k) out[k] = p.work[k];
    API_END
}
int aesfhe_pool_stats(aesfhe_ctx* ctx, uint64_t* out) {
    API_BEGIN out[0] = ctx->eng->pool_bytes();
    out[1] = ctx->eng->oom_retries();
    API_END
}
int aesfhe_kernel_gaps(aesfhe_ctx* ctx, double* out, int n) {
    API_BEGIN KernelProfiler& p = ctx->eng->prof_;
    p.flush();
    for (int k = 0; k < n && k < KID_N; ++k) {
        out[2 * k] = (double)p.gap_n[k];
        out[2 * k + 1] = p.gap_ms[k];
    }
    API_END
}
uint64_t aesfhe_launch_count(void) { return g_launches.load(std::memory_order_relaxed); }
uint64_t aesfhe_launch_census(char* buf, uint64_t cap, int reset) { return census_dump(buf, (size_t)cap, reset != 0); }
int aesfhe_alg_bytes(double* bytes, uint64_t* launches, int n) {
    if (!bytes || !launches) return -2;
    for (int k = 0; k < n && k < KID_N; ++k) {
        bytes[k] = (double)g_alg_bytes[k].load(std::memory_order_relaxed);
        launches[k] = g_alg_launches[k].load(std::memory_order_relaxed);
    }
    return 0;
}
int aesfhe_level_counters(aesfhe_ctx* ctx, int kind, uint64_t* out, int n) {
    API_BEGIN if (kind < 0 || kind >= Engine::LV_N) throw std::runtime_error("level_counters: no such kind");
    for (int l = 0; l < n; ++l) out[l] = ctx->eng->level_counter(kind, l);
    API_END
}
int aesfhe_reset_counters(aesfhe_ctx* ctx) {
    API_BEGIN ctx->eng->reset_counters();
    API_END
}

}  // extern "C"
