// encoder.cpp -- canonical embedding via one length-N complex FFT.
//
// m(zeta^{2t+1}) = sum_k (m_k zeta^k) e^{2 pi i t k / N}, so the values at all N odd
// powers are a DFT of the twisted coefficients; slot j is the value at t = (5^j - 1)/2
// and its conjugate sits at t = (2N - 5^j - 1)/2.
#include "encoder.h"

#include <cmath>

Embedding::Embedding(int logn) : logn_(logn), n_(1 << logn) {
    const int s = n_ / 2;
    const long two_n = 2L * n_;
    slot_pos_.resize(s);
    conj_pos_.resize(s);
    long e = 1;
    for (int j = 0; j < s; ++j) {
        slot_pos_[j] = (int)((e - 1) / 2);
        conj_pos_[j] = (int)((two_n - e - 1) / 2);
        e = e * 5 % two_n;
    }
    twist_.resize(n_);
    roots_.resize(n_ / 2);
    for (int k = 0; k < n_; ++k) twist_[k] = std::polar(1.0, M_PI * k / n_);
    for (int k = 0; k < n_ / 2; ++k) roots_[k] = std::polar(1.0, -2.0 * M_PI * k / n_);
}

// iterative radix-2; forward sign e^{-2 pi i}, inverse_sign -> e^{+2 pi i} (unnormalised)
void Embedding::fft(std::vector<std::complex<double>>& a, bool inverse_sign) const {
    const int n = n_;
    for (int i = 1, j = 0; i < n; ++i) {
        int bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) std::swap(a[i], a[j]);
    }
    for (int len = 2; len <= n; len <<= 1) {
        const int step = n / len;
        for (int i = 0; i < n; i += len)
            for (int k = 0; k < len / 2; ++k) {
                std::complex<double> w = roots_[k * step];
                if (inverse_sign) w = std::conj(w);
                std::complex<double> u = a[i + k], v = a[i + k + len / 2] * w;
                a[i + k] = u + v;
                a[i + k + len / 2] = u - v;
            }
    }
}

void Embedding::inverse(const double* re, const double* im, double* m) const {
    std::vector<std::complex<double>> v(n_);
    for (int j = 0; j < n_ / 2; ++j) {
        v[slot_pos_[j]] = {re[j], im[j]};
        v[conj_pos_[j]] = {re[j], -im[j]};
    }
    fft(v, false);
    const double inv_n = 1.0 / n_;
    for (int k = 0; k < n_; ++k) m[k] = (v[k] * inv_n * std::conj(twist_[k])).real();
}

void Embedding::forward(const double* m, double* re, double* im) const {
    std::vector<std::complex<double>> v(n_);
    for (int k = 0; k < n_; ++k) v[k] = m[k] * twist_[k];
    fft(v, true);
    for (int j = 0; j < n_ / 2; ++j) {
        re[j] = v[slot_pos_[j]].real();
        im[j] = v[slot_pos_[j]].imag();
    }
}
