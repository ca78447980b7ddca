"""Calibration workload for FETCH_SIZE on the NTT passes: plain forward NTTs of 160 rows
(bench parameter set), so the bytes each pass must move are known exactly (read + write of
160 x 256 KiB; pass 2 adds its twiddle pairs).  Run under rocprofv3 --pmc FETCH_SIZE and
WRITE_SIZE passes; compare raw FETCH per launch with WRITE per launch (exact for wide stores)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from engine_context import EngineContext  # noqa: E402

if __name__ == "__main__":
    E = EngineContext(signature=1, max_level=17).engine
    print(E.bench_op("ntt", 160, 50), flush=True)
