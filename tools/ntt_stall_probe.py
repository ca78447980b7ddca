"""A forward-NTT-only workload (160 rows x 200 iterations, bench parameter set) for rocprofv3
SQ counter passes: where the NTT passes' waves spend their cycles."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from engine_context import EngineContext  # noqa: E402


def main():
    E = EngineContext(signature=1, max_level=17, seed=1).engine
    print(E.bench_op("ntt", int(sys.argv[1]) if len(sys.argv) > 1 else 160, 200), flush=True)


if __name__ == "__main__":
    main()
