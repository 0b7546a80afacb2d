#!/usr/bin/env python3
"""A/B of the CPU baseline's process settings on the bench's C3 matrix
(oracle/cpu_bench.py in a process of its own per variant): OpenMP wait
policy (libgomp default / active) x thread placement (one per L3 domain /
unbound) x team size, each variant --reps times, interleaved; with the
cgroup's throttling counters of every leg.  One JSON line per run.

    python heterogeneous-spmv_amd/tools/cpu_baseline_ab.py --out F.jsonl [--budget 6]
"""
import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
sys.path.insert(0, str(HERE.parent))
from hspmv import dist as hdist  # noqa: E402
from hspmv import gen  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--budget", type=float, default=6.0)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--threads", default="15,12,8", help="team sizes to try (0: the quota minus one)")
    a = ap.parse_args()
    a.threads = [int(t) for t in a.threads.split(",")]
    sh = hdist.build_shard(a.config, 0, 1)
    A = sh.A
    d = Path(tempfile.mkdtemp(prefix="hspmv_cpuab_", dir="/dev/shm"))
    np.save(d / "row_ptr.npy", A.row_ptr)
    np.save(d / "col_idx.npy", A.col_idx)
    np.save(d / "val.npy", A.val)
    np.save(d / "x.npy", gen.rand_x(A.n, 42, dtype=A.val.dtype))
    variants = [(pol, bind, th) for pol, bind in ((None, True), ("active", True), (None, False))
                for th in a.threads]
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    with open(a.out, "w") as f:
        for rep in range(a.reps):
            for pol, bind, th in variants:
                env = {k: v for k, v in os.environ.items() if not k.startswith(("OMP_", "GOMP_"))}
                env["OMP_SCHEDULE"] = "static"
                if pol:
                    env["OMP_WAIT_POLICY"] = pol
                dump = Path(a.out).with_suffix("").as_posix() + f"_r{rep}_{pol or 'default'}_{'b' if bind else 'u'}{th}.npy"
                cmd = [sys.executable, str(REPO / "oracle" / "cpu_bench.py"), "--dir", str(d),
                       "--dump-samples", dump,
                       "--budget", str(a.budget), "--no-tried", "--threads", str(th)] + ([] if bind else ["--no-bind"])
                out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
                r = json.loads(out.stdout.strip().splitlines()[-1]) if out.returncode == 0 else {}
                rec = {"config": a.config, "rep": rep, "wait_policy": pol or "default", "bind": bind,
                       "rc": out.returncode, "err": out.stderr[-300:] if out.returncode else ""}
                for k in ("value", "gflops_from_median", "gflops_from_avg", "avg_over_min", "cores",
                          "cgroup_throttling", "runs_within_10pct_of_min", "runs_within_50pct_of_min"):
                    rec[k] = r.get(k)
                ref = r.get("reference_f32") or {}
                rec["ref_value"], rec["ref_avg_over_min"] = ref.get("value"), ref.get("avg_over_min")
                print(json.dumps(rec), flush=True)
                f.write(json.dumps(rec) + "\n")
    shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
