"""bench.py's stdout line stays parseable by the round-end driver.

Round 5's line grew to 23 KB and the driver's bounded tail cut it
(BENCH_r05 parsed: null).  The compact line is built here from recorded full
results (every line the bench measures) and must fit LINE_LIMIT, round-trip
through json, and carry the contract's keys plus roofline and cpu_baseline.
"""
import glob
import json
import os

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")


def recorded():
    out = []
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "round5_bench_r5*.json"))):
        with open(p) as f:
            try:
                d = json.load(f)
            except ValueError:
                continue
        if isinstance(d, dict) and "metric" in d and "roofline" in d:
            out.append((os.path.basename(p), d))
    return out


@pytest.mark.parametrize("name,full", recorded(), ids=[n for n, _ in recorded()])
def test_compact_line_fits_and_round_trips(name, full):
    full = json.loads(json.dumps(full))
    big = len(json.dumps(full))
    line = bench.compact_line(full, "gpurun_out/bench_detail.json")
    s = json.dumps(line)
    assert len(s) <= bench.LINE_LIMIT, (name, len(s))
    assert "\n" not in s
    back = json.loads(s)
    for k in CONTRACT:
        assert k in back, k
    assert back["value"] == full["value"]
    assert back["ms_per_step"] == full["ms_per_step"]
    assert back["roofline"]["frac"] == full["roofline"]["frac"]
    assert back["roofline"]["traffic"] == full["roofline"]["traffic"]
    assert back["cpu_baseline"]["value"] == full["cpu_baseline"]["value"]
    assert back["detail_file"] == "gpurun_out/bench_detail.json"
    assert big > len(s)


def test_compact_line_bounded_even_with_huge_extras():
    full = {"metric": "m", "value": 1.0, "unit": "u", "n_gpus": 1, "steps": 1, "warmup": 0,
            "ms_per_step": 1.0, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u32", "data": "synthetic", "config": {"workload": "C2"},
            "roofline": {"bound": "valu", "frac": 0.3, "traffic": None},
            "cpu_baseline": {"value": 1.0, "lines": [{"impl": "x", "value": 1.0}] * 3},
            "sha256_stage": {"pad": "x" * 20000},
            "go_wiring_latency": {"pad": "y" * 50000}}
    s = json.dumps(bench.compact_line(full, None))
    assert len(s) <= bench.LINE_LIMIT
    assert json.loads(s)["value"] == 1.0


def test_detail_file_written(tmp_path):
    full = {"metric": "m", "value": 2.0, "nested": {"a": [1, 2, 3]}}
    p = str(tmp_path / "sub" / "d.json")
    got = bench.write_detail(full, p)
    assert got == p
    with open(p) as f:
        assert json.load(f) == full
