"""bench.py keeps the driver's JSON-line contract (one line on rank 0, the BASELINE metric, the
roofline and CPU-baseline objects) and its full-size parity spot check holds -- run on the small
C2 workload so it finishes in seconds."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("workload", ["c2", "c3"])
def test_bench_json_line_contract(workload):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--workload", workload,
                          "--steps", "2", "--warmup", "1", "--cpu-seconds", "1"],
                         capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [x for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["metric"].startswith("routing-table build time") and d["unit"] == "node-pairs/s"
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["value"] > 0
    rf = d["roofline"]
    assert rf["bound"] in ("hbm", "mfma") and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    cb = d["cpu_baseline"]
    assert cb["kind"] in ("port", "reference") and cb["cores"] == 1 and cb["value"] > 0
    assert cb["all_cores"]["cores"] >= 1 and cb["all_cores"]["value"] > 0
    assert d["parity"]["lat_bit_exact"] is True
    assert d["parity"]["rel_max_rel_err"] <= 1e-12
    assert d["parity"]["rows_checked"] >= 4 and d["parity"]["tied_pairs"] >= 0
    assert 0.0 <= d["parity"]["tied_frac"] < 0.5
