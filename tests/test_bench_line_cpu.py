"""bench.py's stdout contract: the driver parses the LAST stdout line, and
r05's 18,962-byte line was not parsed.  The full result of a
real run (profiles/r05/bench_final.log, every informational leg included)
goes through bench.emit(): the printed line must be the last stdout line,
parse as JSON, stay <= 4 KB and carry the contract keys, the roofline and the
cpu_baseline; the full result must land in the side file."""
import io
import json
import os
import sys
from contextlib import redirect_stdout

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config")


def _full_result():
    with open(os.path.join(ROOT, "profiles", "r05", "bench_final.log")) as f:
        return json.loads(f.read().strip().splitlines()[-1])


def test_compact_line_parses_and_fits(tmp_path):
    full = _full_result()
    assert len(json.dumps(full)) > 3 * bench.STDOUT_LIMIT  # the stub really is the oversized line
    side = tmp_path / "detail.json"
    buf = io.StringIO()
    with redirect_stdout(buf):
        bench.emit(full, str(side))
    lines = buf.getvalue().strip().splitlines()
    line = lines[-1]
    assert len(line.encode()) <= bench.STDOUT_LIMIT
    d = json.loads(line)
    for k in CONTRACT:
        assert k in d, k
    assert d["value"] == full["value"] and d["ms_per_step"] == full["ms_per_step"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "bytes_per_launch_algorithmic"):
        assert k in d["roofline"], k
    assert d["roofline"]["frac"] == full["roofline"]["frac"]
    for k in ("value", "unit", "cores", "kind", "sample", "parity_bit_exact_on_sample"):
        assert k in d["cpu_baseline"], k
    assert "n11" in d["perf_mode"] and "Mpatches_per_s" in d["perf_mode"]["n11"]
    assert d["scaling_leg"]["fast"]["ranks_store_equal"] is True
    # the side file holds everything
    assert json.loads(side.read_text()) == full


def test_compact_sheds_legs_before_exceeding_limit(tmp_path):
    full = _full_result()
    full["config"]["workload"] = "x" * 5000  # pathological: the contract part alone is large
    buf = io.StringIO()
    with redirect_stdout(buf):
        bench.emit(full, None)
    line = buf.getvalue().strip().splitlines()[-1]
    d = json.loads(line)
    assert "value" in d and "roofline" in d and "cpu_baseline" in d
    assert "perf_mode" not in d and "seed_generation" not in d
