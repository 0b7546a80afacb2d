"""bench.py contract on one GPU: one JSON line with the driver's keys, the
roofline and cpu_baseline objects, and a passing y check (short run)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]


@pytest.mark.gpu
def test_bench_json_line_contract():
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    out = subprocess.run([sys.executable, str(REPO / "bench.py"), "--steps", "20", "--warmup", "3",
                          "--cold-steps", "2", "--cpu-seconds", "0.5"],
                         cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 20 and d["warmup"] == 3
    assert d["unit"] == "GFLOP/s" and d["value"] > 0 and d["higher_is_better"] is True
    assert d["dtype"] == "f64" and d["config"]["workload"].startswith("c2")
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert 0 < r["frac"] < 1 and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    c = d["cpu_baseline"]
    assert c["kind"] == "port" and c["cores"] >= 1 and c["value"] > 0
    ref = c["reference_f32"]  # the reference's own program, when oracle/_ref was built
    if (REPO / "oracle" / "_ref" / "libref_spmvcsr.so").exists():
        assert ref["kind"] == "reference" and ref["value"] > 0 and ref["time_avg_s"] > 0
    assert d["check"]["pass"] is True
