#!/usr/bin/env python3
"""oracle/cpu_bench.py -- TEST INFRASTRUCTURE ONLY: the CPU baseline legs of
bench.py, run in a process of their own.

bench.py writes the matrix and x (``np.save``) into a scratch directory and
starts this script; it prints ONE JSON object.  A separate process keeps the
timed OpenMP team alone in its process: no torch or HIP runtime threads, and
a libgomp initialised with this process's OMP_* environment (the wait policy
is read once, at load).

Legs (spmv-csr/spmv.c:164-185 protocol: 5 warm-ups + N timed runs, each
bracketed by omp_get_wtime; value = 2 nnz / TimeMin as run_norm.py records
it, the median and TimeAvg beside it):

* ``port``  the oracle's omp_spmv restatement (oracle/spmv_oracle.c) on the
  matrix's own dtype;
* ``reference_f32``  the reference's own omp_spmv (spmv-csr/spmv.c compiled
  unmodified into oracle/_ref) on the fp32 copy, when that library exists;
* ``threads_tried``  the full-quota and all-core team sizes, unbound, as
  bursts (never reported as value).

Threads: one fewer than the cgroup CPU quota (cpu.max), so the process's
other threads keep a CPU and the team is never throttled; without a quota,
the physical cores.  The team is spread one thread per L3 domain
(OMP_PROC_BIND=spread over ll_caches places; run_scripts/run_cuda_new.py:75-79
binds as well) and the matrix is first-touch copied in omp_spmv's static
row partition, so each thread streams its rows from its own NUMA node.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent))
import oracle  # noqa: E402


def host_cpu_info() -> dict:
    """Physical cores from lscpu (Core(s) per socket x Socket(s)), the CPUs
    this process may run on, and the cgroup CPU quota (cpu.max), if any."""
    info = {"physical_cores": None, "affinity_cpus": len(os.sched_getaffinity(0)),
            "cgroup_cpu_quota": None, "model": None}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=20).stdout
        kv = {}
        for line in out.splitlines():
            k, _, v = line.partition(":")
            kv[k.strip()] = v.strip()
        cps, sock = int(kv.get("Core(s) per socket", "0")), int(kv.get("Socket(s)", "0"))
        if cps and sock:
            info["physical_cores"] = cps * sock
        info["model"] = kv.get("Model name")
    except Exception:
        pass
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            info["cgroup_cpu_quota"] = float(q) / float(per)
    except Exception:
        pass
    return info


def l3_places(cpus) -> list:
    """One place per L3 domain (an EPYC CCD) of the given CPUs, physical cores
    only (the first SMT sibling of each core), ordered so that consecutive
    places alternate between sockets: what OMP_PLACES=ll_caches +
    OMP_PROC_BIND=spread give.  [] when sysfs lacks the cache topology."""
    def rd(c, f):
        return Path(f"/sys/devices/system/cpu/cpu{c}/{f}").read_text().strip()
    dom = {}
    try:
        for c in sorted(cpus):
            sib = rd(c, "topology/thread_siblings_list").replace("-", ",").split(",")
            if int(sib[0]) != c and int(sib[0]) in cpus:
                continue  # not the first hardware thread of its core
            key = (int(rd(c, "topology/physical_package_id")), int(rd(c, "cache/index3/id")))
            dom.setdefault(key, []).append(c)
    except (OSError, ValueError):
        return []
    by_pkg = {}
    for (pkg, _l3), cs in sorted(dom.items()):
        by_pkg.setdefault(pkg, []).append(cs)
    out = []
    for i in range(max((len(v) for v in by_pkg.values()), default=0)):
        for pkg in sorted(by_pkg):
            if i < len(by_pkg[pkg]):
                out.append(by_pkg[pkg][i])
    return out


def cpu_stat() -> dict:
    """The cgroup's CPU accounting (cpu.stat): throttled periods and time."""
    out = {}
    try:
        for line in Path("/sys/fs/cgroup/cpu.stat").read_text().splitlines():
            k, v = line.split()
            out[k] = int(v)
    except (OSError, ValueError):
        pass
    return out


def throttled(before: dict, after: dict) -> dict:
    return {k: after.get(k, 0) - before.get(k, 0)
            for k in ("nr_periods", "nr_throttled", "throttled_usec") if k in after}


def timing(nnz: int, samples: np.ndarray) -> dict:
    tmin, tmax = float(samples.min()), float(samples.max())
    tavg, tmed = float(samples.mean()), float(np.median(samples))
    g = lambda t: round(2.0 * nnz / t * 1e-9, 3)  # noqa: E731
    return {"time_min_s": tmin, "time_avg_s": tavg, "time_max_s": tmax, "median_s": tmed,
            "avg_over_min": round(tavg / tmin, 3), "gflops_from_min": g(tmin),
            "gflops_from_median": g(tmed), "gflops_from_avg": g(tavg), "runs": int(samples.size)}


def reference_leg(rp, ci, val32, x32, nnz: int, threads: int, budget_s: float):
    """The reference's own omp_spmv (spmv-csr/spmv.c:92-114, oracle/_ref) on the
    fp32 copy, called once per timed run (its only dtype)."""
    import ctypes as C
    if not oracle.ref_available():
        return None
    R = oracle.ref()
    oracle.set_schedule("static", threads)
    y = np.zeros(rp.shape[0] - 1, np.float32)
    args = (C.c_int(rp.shape[0] - 1), C.c_int(x32.shape[0]), C.c_int(nnz), rp.ctypes.data,
            ci.ctypes.data, val32.ctypes.data, x32.ctypes.data, y.ctypes.data)
    for _ in range(5):
        R.omp_spmv(*args)
    ts = []
    t_end = time.perf_counter() + budget_s
    while len(ts) < 20 or (time.perf_counter() < t_end and len(ts) < 20000):
        t0 = time.perf_counter()
        R.omp_spmv(*args)
        ts.append(time.perf_counter() - t0)
    tm = timing(nnz, np.array(ts))
    return {"kind": "reference", "dtype": "f32", "cores": threads, "value": tm["gflops_from_min"],
            "unit": "GFLOP/s", **{k: tm[k] for k in ("avg_over_min", "gflops_from_avg",
                                                      "gflops_from_median", "median_s", "time_min_s",
                                                      "time_avg_s", "time_max_s", "runs")},
            "sample": (f"the reference's omp_spmv (oracle/_ref, built from spmv-csr/spmv.c) on the "
                       f"same matrix in fp32, OMP_SCHEDULE=static, {threads} threads, 5 warm-ups + "
                       f"{tm['runs']} timed calls, value = 2 nnz / TimeMin")}


def run(d: Path, budget_s: float, threads: int = 0, bind: bool = True, tried: bool = True,
        reference: bool = True, dump: str = "") -> dict:
    rp = np.load(d / "row_ptr.npy", mmap_mode="r")
    ci = np.load(d / "col_idx.npy", mmap_mode="r")
    val = np.load(d / "val.npy", mmap_mode="r")
    x = np.ascontiguousarray(np.load(d / "x.npy"))
    m, nnz = rp.shape[0] - 1, ci.shape[0]
    hw = host_cpu_info()
    phys = hw["physical_cores"] or hw["affinity_cpus"]
    avail = max(1, min(phys, hw["affinity_cpus"]))
    quota = hw["cgroup_cpu_quota"]
    if threads <= 0:
        threads = max(1, min(avail, int(math.floor(quota)) - 1)) if quota else avail
    legs = {}
    if tried:
        full = min(avail, int(math.floor(quota))) if quota else avail
        for t in sorted({full, avail} - {threads}):
            oracle.set_schedule("static", t)
            tm = timing(nnz, oracle.time_spmv_samples(rp, ci, val, x, 5, 20))
            tm["within_quota"] = bool(not quota or t <= quota)
            tm["note"] = ("burst: above the cgroup CPU quota, throttled on average" if quota and t > quota
                          else "no CPU left for the process's other threads")
            legs[int(t)] = tm
    oracle.set_schedule("static", threads)
    places = l3_places(os.sched_getaffinity(0)) if bind else []
    bound = oracle.bind_threads(threads, places) if places else 0
    lrp, lci, lval = oracle.localize(rp, ci, val)
    per = max(float(np.median(oracle.time_spmv_samples(lrp, lci, lval, x, 2, 5))), 1e-6)
    runs = int(max(20, min(20000, 0.35 * budget_s / per)))
    res = {}
    for sched in ("static", "guided"):  # run_norm.py:18,66 / run_cuda_new.py:79
        oracle.set_schedule(sched, threads)
        c0 = cpu_stat()
        smp = oracle.time_spmv_samples(lrp, lci, lval, x, 5, runs)
        if dump and sched == "static":  # every run's seconds, in order (A/B diagnosis)
            np.save(dump, smp)
        res[sched] = timing(nnz, smp)
        res[sched]["cgroup_throttling"] = throttled(c0, cpu_stat())
        # share of runs within 10 % / 50 % of TimeMin
        res[sched]["runs_within_10pct_of_min"] = round(float(np.mean(smp <= 1.1 * smp.min())), 3)
        res[sched]["runs_within_50pct_of_min"] = round(float(np.mean(smp <= 1.5 * smp.min())), 3)
    st = res["static"]
    legs[int(threads)] = dict(st, within_quota=True, note="reported leg")
    dt = "fp64" if val.dtype == np.float64 else "fp32"
    policy = os.environ.get("OMP_WAIT_POLICY", "(libgomp default)")
    placement = (f"one thread per L3 domain ({len(places)} domains, {bound} threads bound)"
                 if bound else "unbound")
    out = {"value": st["gflops_from_min"], "unit": "GFLOP/s", "cores": int(threads), "kind": "port",
           "cores_note": ((f"{threads} OpenMP threads = the cgroup quota of {quota} CPUs minus one "
                           f"for the process's other threads" if quota else
                           f"{threads} OpenMP threads = the physical cores (no cgroup quota)")
                          + f" ({phys} physical cores, {hw['affinity_cpus']} CPUs in the affinity "
                          f"mask); {placement}; OMP_WAIT_POLICY={policy}; a process of its own "
                          f"(oracle/cpu_bench.py)"),
           "cgroup_cpu_quota": quota,
           "sample": (f"the same matrix as the GPU line (m={m}, nnz={nnz}, {dt}, CSR), omp_spmv "
                      f"restatement (oracle/spmv_oracle.c), OMP_SCHEDULE=static, {threads} threads, "
                      f"5 warm-ups + {runs} timed runs (spmv-csr/spmv.c:164-185 protocol), "
                      f"value = 2 nnz / TimeMin"),
           **{k: st[k] for k in ("time_min_s", "time_avg_s", "time_max_s", "median_s", "avg_over_min",
                                 "gflops_from_median", "gflops_from_avg", "cgroup_throttling",
                                 "runs_within_10pct_of_min", "runs_within_50pct_of_min")},
           "host": hw, "wait_policy": policy, "threads_tried": legs,
           "guided": {"gflops": res["guided"]["gflops_from_min"],
                      "gflops_from_median": res["guided"]["gflops_from_median"],
                      "gflops_from_avg": res["guided"]["gflops_from_avg"],
                      "time_min_s": res["guided"]["time_min_s"],
                      "time_max_s": res["guided"]["time_max_s"],
                      "time_avg_s": res["guided"]["time_avg_s"],
                      "median_s": res["guided"]["median_s"], "runs": runs}}
    if reference:
        v32 = np.ascontiguousarray(val, np.float32)
        r32, c32, l32 = oracle.localize(rp, ci, v32)
        out["reference_f32"] = reference_leg(r32, c32, l32, np.ascontiguousarray(x, np.float32), nnz,
                                             threads, 0.5 * budget_s)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True, help="row_ptr.npy, col_idx.npy, val.npy, x.npy")
    ap.add_argument("--budget", type=float, default=10.0, help="seconds of timed runs (about)")
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--no-bind", action="store_true")
    ap.add_argument("--no-tried", action="store_true")
    ap.add_argument("--no-reference", action="store_true")
    ap.add_argument("--dump-samples", default="", help=".npy of the static leg's run times")
    a = ap.parse_args()
    out = run(Path(a.dir), a.budget, a.threads, not a.no_bind, not a.no_tried, not a.no_reference,
              a.dump_samples)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
