"""StateEncoder: 16-byte AES state <-> (ct_hi, ct_lo) (REF/state_encoder.py:9-38).

Byte i (column-first order, REF/README.md:103-104) goes to slot i*stride with
stride = slot_count/16; every other slot holds 1+0j.
"""
from typing import Any, Tuple

import numpy as np

from utils import ZetaEncoder


class StateEncoder:
    def __init__(self, ctx):
        self.ctx = ctx
        self.sc = ctx.engine.slot_count
        self.stride = self.sc // 16

    def _pack(self, nibbles: np.ndarray) -> np.ndarray:
        vec = np.ones(self.sc, dtype=np.complex128)
        vec[0:16 * self.stride:self.stride] = ZetaEncoder.to_zeta(nibbles.astype(np.uint8), 16)
        return vec

    def encode(self, state: np.ndarray) -> Tuple[Any, Any]:
        state = np.asarray(state, dtype=np.uint8)
        assert state.shape == (16,)
        return self.ctx.encrypt(self._pack(state >> 4)), self.ctx.encrypt(self._pack(state & 0x0F))

    def decode(self, ct_hi, ct_lo) -> np.ndarray:
        take = slice(0, 16 * self.stride, self.stride)
        hi = ZetaEncoder.from_zeta(self.ctx.decrypt(ct_hi)[take], 16)
        lo = ZetaEncoder.from_zeta(self.ctx.decrypt(ct_lo)[take], 16)
        return ((hi << 4) | lo).astype(np.uint8)

    def renorm(self, ct_hi, ct_lo) -> Tuple[Any, Any]:
        """decode -> re-encode (REF/pipeline.py:65-69), done on the device when available."""
        fast = getattr(self.ctx, "renorm_pair", None)
        if fast is not None:
            return fast(ct_hi, ct_lo)
        return self.encode(self.decode(ct_hi, ct_lo))
