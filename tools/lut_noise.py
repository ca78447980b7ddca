"""Slot error of the fused LUT op vs the per-term loop, against the ideal Zeta16 outputs
(SubBytes, XOR4, GF x2): prints max / rms angular error of the 16 state slots."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from aes_keyschedule import load_all_coeffs  # noqa: E402
from engine_context import EngineContext  # noqa: E402
from lut import ensure_coeffs  # noqa: E402
from mixcol_final import MixColFinal  # noqa: E402
from oracle import aes_plain  # noqa: E402
from state_encoder import StateEncoder  # noqa: E402
from sub_bytes_lut import SubBytesLUT  # noqa: E402
from xor4_lut import XOR4LUT  # noqa: E402


def err(ctx, ct, nib):
    sc = ctx.engine.slot_count
    z = ctx.decrypt(ct)[: 16 * (sc // 16): sc // 16]
    ref = np.exp(-2j * np.pi * nib / 16)
    a = np.abs(np.angle(z / ref))
    return float(a.max()), float(np.sqrt((a ** 2).mean())), float(np.abs(np.abs(z) - np.abs(z).mean()).max())


def main():
    co = load_all_coeffs(ensure_coeffs())
    ctx = EngineContext(signature=2, max_level=17, log_n=16)
    enc = StateEncoder(ctx)
    rng = np.random.default_rng(1)
    st = rng.integers(0, 256, 16).astype(np.uint8)
    k = rng.integers(0, 256, 16).astype(np.uint8)
    hi, lo = enc.encode(st)
    kh, kl = enc.encode(k)
    sb = SubBytesLUT(ctx, co["sub_hi"], co["sub_lo"])
    x = XOR4LUT(ctx, co["xor4"])
    mc = MixColFinal(ctx, x)
    out = aes_plain.SBOX[st]
    g2 = aes_plain.GF_MUL[2][st]
    for fused in (True, False):
        ctx.fused_luts = fused
        tag = "fused" if fused else "loop "
        h, l = sb.apply(hi, lo)
        print(tag, "subbytes hi", err(ctx, h, out >> 4), "lo", err(ctx, l, out & 15), "levels", h.level, l.level)
        print(tag, "xor4", err(ctx, x.apply(hi, kh), (st ^ k) >> 4))
        a, b = mc.gf_mult_2(hi, lo)
        print(tag, "gf2", err(ctx, a, g2 >> 4), err(ctx, b, g2 & 15))
    # statistics of the SubBytes error over several states (the 128th power amplifies any
    # difference in the lifted input, so single runs differ by noise realisation)
    for fused in (True, False):
        ctx.fused_luts = fused
        ang = []
        for t in range(6):
            s2 = np.random.default_rng(100 + t).integers(0, 256, 16).astype(np.uint8)
            h, l = sb.apply(*enc.encode(s2))
            o = aes_plain.SBOX[s2]
            for ct, nib in ((h, o >> 4), (l, o & 15)):
                sc = ctx.engine.slot_count
                z = ctx.decrypt(ct)[: 16 * (sc // 16): sc // 16]
                ang.append(np.abs(np.angle(z / np.exp(-2j * np.pi * nib / 16))))
        ang = np.concatenate(ang)
        print("fused" if fused else "loop ", "subbytes over 6 states: max %.5f rms %.5f" % (ang.max(), np.sqrt((ang ** 2).mean())))


if __name__ == "__main__":
    main()
