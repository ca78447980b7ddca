"""Per-step slot error trace of a slot-packed true-FHE encrypt (AESPipeline(true_fhe=True)):
max / 99.9th percentile / rms distance of every state slot from its ideal Zeta16 codeword after
each step, and the level.  Usage: python3 tools/fhe_trace.py [states]  (default 256)."""
import json, sys
from pathlib import Path
import numpy as np
ROOT = Path.cwd()
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]
from engine_context import EngineContext
from aes_keyschedule import expand_aes128_key, load_all_coeffs
from pipeline import AESPipeline
from oracle import aes_plain as A
from utils import NEED_SUBBYTES, NEED_SR_MIX, NEED_SR_ARK
ctx = EngineContext(signature=1, max_level=17, seed=0xB007)
co = load_all_coeffs()
rng = np.random.default_rng(53)
rks = expand_aes128_key(rng.integers(0, 256, 16).astype(np.uint8))
S = ctx.engine.slot_count; stride = S // 16
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
pipe = AESPipeline(ctx, co, states=B, true_fhe=True)
enc = pipe.encoder
def errs(pair_ct, byt):
    out = []
    for ct, nib in ((pair_ct[0], byt >> 4), (pair_ct[1], byt & 15)):
        v = ctx.decrypt(ct)[:16 * stride].reshape(16, stride)[:, :B].T
        out.append(np.abs(v - np.exp(-2j * np.pi * nib / 16)))
    e = np.maximum(*out)
    return "max %.2e p99.9 %.2e rms %.2e L%d" % (e.max(), np.quantile(e, 0.999), np.sqrt((e**2).mean()), pair_ct[0].level)
pts = rng.integers(0, 256, (B, 16)).astype(np.uint8)
rk = pipe._prepare_round_keys(rks)
s = pts ^ rks[0]
ct = pipe.ark(*enc.encode(pts), *rk[0], out_level=1); print("r0.ark", errs(ct, s), flush=True)
ct = pipe._renorm_pair(*ct, level=NEED_SUBBYTES); print("r0.renorm", errs(ct, s), flush=True)
for r in range(1, 10):
    ct = pipe.sub.apply(*ct, out_level=1); s = A.SBOX[s]; print(f"r{r}.sb", errs(ct, s), flush=True)
    ct = pipe._renorm_pair(*ct, level=NEED_SR_ARK); print(f"r{r}.sb.renorm", errs(ct, s), flush=True)
    ct = pipe.shift_rows(*ct); s = np.stack([A.shift_rows(x) for x in s]); print(f"r{r}.sr", errs(ct, s), flush=True)
    ct = pipe.mix(*ct); s = np.stack([A.ref_mix_columns(x) for x in s]); print(f"r{r}.mc", errs(ct, s), flush=True)
    ct = pipe.ark(*ct, *rk[r], out_level=1); s = s ^ rks[r]; print(f"r{r}.ark", errs(ct, s), flush=True)
    ct = pipe._renorm_pair(*ct, level=NEED_SUBBYTES); print(f"r{r}.ark.renorm", errs(ct, s), flush=True)
