"""Generate tests/golden/stages.json: per-stage AES state bytes for seeds {0, 7, 42}.

Inputs follow the reference harness: np.random.seed(seed), then the master key, then the
plaintext, 16 random bytes each (REF/test/test_aes_pipeline_roundtrip.py:136-140;
REF/main.py:44-46 draws state then key for config 1).  Expected bytes come from the byte-level
restatement oracle/aes_plain.py, which follows the reference's step order and MixColumns
orientation (REF/pipeline.py:123-254, REF/mixcol_final.py:169-221) and is pinned to FIPS-197
(tests/test_oracle_golden.py).  Run:  python tests/golden/make_stage_fixture.py
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from aes_keyschedule import expand_aes128_key  # noqa: E402
from oracle import aes_plain as A  # noqa: E402


def stages_for(seed: int) -> dict:
    np.random.seed(seed)
    key = np.random.randint(0, 256, 16, dtype=np.uint8)
    pt = np.random.randint(0, 256, 16, dtype=np.uint8)
    rks = expand_aes128_key(key)
    st = {}
    s = pt ^ rks[0]
    st["r0.ark"] = s
    for r in range(1, 10):
        s = A.SBOX[s]; st[f"r{r}.sb"] = s
        s = A.shift_rows(s); st[f"r{r}.sr"] = s
        s = A.ref_mix_columns(s); st[f"r{r}.mc"] = s
        s = s ^ rks[r]; st[f"r{r}.ark"] = s
    s = A.SBOX[s]; st["r10.sb"] = s
    s = A.shift_rows(s); st["r10.sr"] = s
    s = s ^ rks[10]; st["r10.ark"] = s
    return {"seed": seed, "key": key.tolist(), "plaintext": pt.tolist(),
            "round_keys": [k.tolist() for k in rks], "ciphertext": s.tolist(),
            "stages": {k: v.tolist() for k, v in st.items()}}


def config1() -> dict:
    """BASELINE config 1: np.random.seed(0); state, then key (REF/main.py:44-46); ARK only."""
    np.random.seed(0)
    state = np.random.randint(0, 256, 16, dtype=np.uint8)
    key = np.random.randint(0, 256, 16, dtype=np.uint8)
    return {"state": state.tolist(), "key": key.tolist(), "ark": (state ^ key).tolist()}


def main():
    out = {"generator": "tests/golden/make_stage_fixture.py", "seeds": [stages_for(s) for s in (0, 7, 42)],
           "config1": config1()}
    path = Path(__file__).with_name("stages.json")
    path.write_text(json.dumps(out, indent=1))
    print("wrote", path)


if __name__ == "__main__":
    main()
