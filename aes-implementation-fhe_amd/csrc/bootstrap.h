// bootstrap.h -- host-side planning of CKKS bootstrapping.
//
// The slot <-> coefficient maps are the special FFT z = V w, V[j][k] = zeta^{k 5^j}
// (w = coefficient halves t_lo + i t_hi), factored into log2(M) radix-2 butterfly stages
// acting on bit-reversed w.  Each stage is a 3-diagonal map (offsets 0, +-lenh); stages are
// merged into a few groups (one level each) and every group is evaluated with the
// baby-step / giant-step diagonal method.  Offsets follow out[p] = sum_o d_o[p] in[p + o],
// i.e. a LEFT rotation by o (rotate(ct, -o) in the np.roll convention of the C ABI).
#pragma once
#include <complex>
#include <vector>

using cplx = std::complex<double>;

struct LinGroup {
    int h = 1;                 // offset quantum of the group (smallest lenh)
    int B = 1, G = 1, R = 0;   // baby steps, giant steps, offset radius (in units of h)
    std::vector<int> giant;    // left-rotation applied after giant step g: h (g B - R)
    // diag[g][b]: pre-rotated diagonal for offset h (g B + b - R); empty when absent
    std::vector<std::vector<std::vector<cplx>>> diag;
};

struct BootPlan {
    int logn = 16, M = 1 << 15;
    int K = 12;     // EvalMod range: |t / q0| < K
    int r = 3;      // double-angle iterations
    int deg = 27;   // Chebyshev degree of cos(2 pi (K y - 1/4) / 2^r) on [-1, 1]
    std::vector<double> cheb;
    std::vector<LinGroup> cts, stc;  // in application order
    LinGroup stc_lo;                 // pack 2: the lo member's form of stc[0]
};

// cts_scale multiplies CoeffToSlot (folded into its first group), stc_scale multiplies
// SlotToCoeff (folded into its first group)
// stc_boost: intermediate SlotToCoeff groups carry the signal times stc_boost (first group
// x stc_boost, last group / stc_boost; same transform)
// pack (sparse plans): 1 = CoeffToSlot's last group and SlotToCoeff's first work on 2M-periodic
// vectors so that the real and imaginary halves share ONE EvalMod; 2 = 4M-periodic, the hi / lo
// members of a pair bootstrap also share it (stc[0] reads the hi blocks, stc_lo the lo blocks)
BootPlan make_boot_plan(int logn, int n_groups_cts, int n_groups_stc, double cts_scale, double stc_scale, int K, int r, int deg,
                        double stc_boost = 1.0, int pack = 0);

// reference evaluation of the planned transforms on plain vectors (self-check)
std::vector<cplx> apply_group_plain(const LinGroup& g, const std::vector<cplx>& v);
