// encoder.h -- CKKS canonical embedding on the host.
//
// Slot j <-> evaluation at zeta^{5^j}, zeta = e^{i pi / N}.  embed_inverse returns the
// real coefficients m_k of the polynomial whose slots are z; embed is its inverse.
#pragma once
#include <complex>
#include <vector>

class Embedding {
public:
    explicit Embedding(int logn);
    // z: slot_count complex values -> N real coefficients (unscaled)
    void inverse(const double* re, const double* im, double* m) const;
    // N real coefficients -> slot_count complex values
    void forward(const double* m, double* re, double* im) const;
    int n() const { return n_; }

private:
    void fft(std::vector<std::complex<double>>& a, bool inverse_sign) const;
    int logn_, n_;
    std::vector<int> slot_pos_;                    // (5^j mod 2N - 1) / 2
    std::vector<int> conj_pos_;                    // (2N - 5^j - 1) / 2
    std::vector<std::complex<double>> twist_;      // zeta^k
    std::vector<std::complex<double>> roots_;      // e^{-2 pi i k / N}
};
