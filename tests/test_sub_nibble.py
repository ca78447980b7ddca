"""The nibble-bivariate SubBytes form (sub_bytes_lut.nibble_matrix, round 5): the 16 x 16 matrices
derived from the reference's own 8 -> 4 coefficient files (REF/gen/coeff/mod256_to_16_*.json,
REF/sub_bytes_lut.py:46-73) equal coeffgen.lut_bivariate of the AES S-box nibble tables, and
sum_{p,q} C[p,q] ζ16^(hp + lq) gives ζ16 of the S-box (InvS-box) output nibble for all 256 bytes."""
import numpy as np
import pytest

import coeffgen
from aes_keyschedule import load_all_coeffs
from sub_bytes_lut import nibble_matrix


@pytest.mark.parametrize("name", ["sub", "inv_sub"])
@pytest.mark.parametrize("which", ["hi", "lo"])
def test_nibble_matrix_is_the_sbox_table(name, which):
    sbox, inv_sbox = coeffgen._sboxes()
    tab = sbox if name == "sub" else inv_sbox
    nib = (lambda y: y >> 4) if which == "hi" else (lambda y: y & 15)
    C = nibble_matrix(load_all_coeffs()[f"{name}_{which}"])
    assert np.abs(C - coeffgen.lut_bivariate(lambda h, l: nib(tab[16 * h + l]))).max() < 1e-12
    z = np.exp(-2j * np.pi / 16)
    h, l = np.meshgrid(np.arange(16), np.arange(16), indexing="ij")
    P, Q = np.arange(16)[:, None, None, None], np.arange(16)[None, :, None, None]
    val = (C[:, :, None, None] * z ** (P * h + Q * l)).sum(axis=(0, 1))
    want = z ** np.vectorize(lambda a, b: nib(tab[16 * a + b]))(h, l)
    assert np.abs(val - want).max() < 1e-12
