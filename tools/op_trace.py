"""One engine primitive repeated (aesfhe_bench_op) for rocprofv3 --kernel-trace: which kernels
a primitive launches and what each costs.  usage: op_trace.py <op> <arg> [iters]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "aes-implementation-fhe_amd")]

from engine_context import EngineContext  # noqa: E402

if __name__ == "__main__":
    E = EngineContext(signature=1, max_level=17).engine
    op, arg = sys.argv[1], int(sys.argv[2])
    it = int(sys.argv[3]) if len(sys.argv) > 3 else 100
    E.bench_op(op, arg, 5)
    print(op, arg, "us", E.bench_op(op, arg, it))
