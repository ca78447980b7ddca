"""bench.py's stdout line stays parseable by the driver (VERDICT r4 'do this' 1): the full record
of round 4's final bench (profiles/r4_bench_final.json, 83 KB, every leg with per-class rooflines)
goes through the same compact_line / emit_line the bench prints with, and must come out as ONE
JSON line under 12 KB that keeps every contract key and each leg's number."""
import json
import sys

from conftest import ROOT

sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

FULL = ROOT / "profiles" / "r4_bench_final.json"


def _full():
    return json.loads(FULL.read_text())


def test_line_under_limit_and_round_trips(tmp_path):
    full = _full()
    assert len(json.dumps(full)) > 60_000  # the record that did not parse
    detail = tmp_path / "detail.json"
    s = bench.emit_line(full, str(detail))
    assert "\n" not in s
    assert len(s) < 12_000
    line = json.loads(s)
    assert json.loads(detail.read_text()) == full  # nothing lost: the detail file holds the whole record
    assert line["detail_file"] == str(detail)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "roofline_step", "cpu_baseline"):
        assert k in line, k
    assert line["config"]["workload"].startswith("C2")
    assert abs(line["value"] - full["value"]) / full["value"] < 1e-5
    r = line["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r
    assert abs(r["frac"] - full["roofline"]["frac"]) < 1e-4
    cb = line["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cb
    for leg in ("batch", "batch_pairs", "batch_packed_pairs", "true_fhe", "eager_ref_calls"):
        assert leg in line and line[leg]["roofline_step"]["frac"] > 0
    assert line["batch"]["roundtrip"]["roundtrip_blocks_per_s"] > 0
    # per-class entries are numeric arrays in the documented field order
    cls = line["roofline_step"]["classes"]["ntt_rows_fwd"]
    assert len(cls) == len(bench.CLASS_FIELDS) and all(isinstance(x, (int, float)) or x is None for x in cls)
    # the prose appears once, in notes
    assert s.count("dispatch-inclusive duration") == 1
    assert line["roofline_step"]["traffic_over_algorithmic"]["ntt_rows_fwd"] > 0.5


def test_line_without_detail_file_and_oversize_fallback():
    full = _full()
    s = bench.emit_line(full, None)
    assert len(s) < 12_000 and "detail_file" not in json.loads(s)
    # a record with many more legs still fits: the per-class arrays of secondary legs are dropped first
    for i in range(6):
        full[f"extra_{i}"] = full["batch"]
    saved = bench.LEG_KEYS
    try:
        bench.LEG_KEYS = saved + tuple(f"extra_{i}" for i in range(6))
        s = bench.emit_line(full, None)
    finally:
        bench.LEG_KEYS = saved
    assert len(s) < 12_000
    json.loads(s)


def test_sig_rounding():
    assert bench._sig(0.362346652, 3) == 0.362
    assert bench._sig(47095808.0, 4) == 47100000.0
    assert bench._sig(5) == 5 and bench._sig(None) is None and bench._sig(True) is True
