#!/usr/bin/env python3
"""bench.py -- SpMV GFLOP/s and achieved HBM GB/s (fp64) on 1..8 MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1
launched with torch.distributed.run, one rank per GPU.  A "step" is one SpMV
y = A x over every rank's row-range shard of the workload (inputs resident in
HBM; no data-path collective -- rows are independent).
W untimed steps, then exactly K steps bracketed by barrier + synchronize; the
max over ranks is the step time; rank 0 prints ONE JSON line.

Workload (default ``--config c2``): BASELINE configs[1], CSR fp64 on the 2-D
5-point Laplacian 1000 x 1000 (m = 1e6, nnz = 4,996,000) per GPU; at N GPUs
the global grid is 1000 x 1000N, row-range partitioned (weak scaling).
``--config c4``: the 2e7-row banded matrix split over N GPUs (strong).

Extra fields on the line:
  roofline     dominant kernel, algorithmic bytes per launch / event-timed
               average launch duration on the launch stream, vs 8 TB/s HBM
  cold         the same SpMV with the 256 MiB Infinity Cache flushed before
               every launch (the C2 matrix, 80 MB, is MALL-resident when warm)
  comm         RCCL x broadcast / y all-gather / halo-exchange times (N > 1),
               timed separately, and the end-to-end rates they imply:
               2 nnz / (step + y all-gather), and the iterative form
               2 nnz / (step + halo exchange) where x is distributed like y
  cpu_baseline the oracle's OpenMP restatement of spmv-csr's omp_spmv on the
               host cores, rank 0 at N = 1 only (bounded sample); beside it,
               reference_f32: the reference's own spmv-csr program (fp32)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

os.environ.setdefault("OMP_SCHEDULE", "static")  # before any libgomp loads

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "heterogeneous-spmv_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402  (device memory, streams, torch.distributed: plumbing)
import torch.distributed as dist  # noqa: E402

import hspmv  # noqa: E402
from hspmv import dist as hdist  # noqa: E402
from hspmv import gen  # noqa: E402

METRIC = "SpMV GFLOP/s and achieved HBM GB/s (fp64) per matrix, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c2", choices=["c2", "c4"])
    ap.add_argument("--kernel", default="auto", choices=["auto", "stream", "vector"])
    ap.add_argument("--lanes", type=int, default=0)
    ap.add_argument("--nt", action="store_true", help="non-temporal matrix loads")
    ap.add_argument("--cold-steps", type=int, default=20)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="budget of the CPU-baseline sample (rank 0, N=1)")
    ap.add_argument("--no-cpu", action="store_true")
    return ap.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a HIP GPU")
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return rank, world, local


def barrier(world):
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(v: float, world: int) -> float:
    if world == 1:
        return v
    t = torch.tensor([v], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(v: float, world: int) -> float:
    if world == 1:
        return v
    t = torch.tensor([v], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def load_traffic(workload_key: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary
    (profiles/*_pmc.json, written by heterogeneous-spmv_amd/tools/pmc_summary.py),
    or None when no summary for this workload exists."""
    best = None
    for p in sorted((REPO / "profiles").glob("*_pmc.json")):
        try:
            d = json.loads(p.read_text())
        except Exception:
            continue
        if d.get("workload") == workload_key and d.get("hbm_bytes_per_launch"):
            best = d
    return best


def cpu_baseline(A, x, budget_s: float):
    """Oracle OpenMP restatement of omp_spmv (spmv-csr/spmv.c:92-114) timed with
    the reference protocol (5 warm-ups + timed runs), on this host's cores."""
    sys.path.insert(0, str(REPO / "oracle"))
    import oracle  # test infrastructure: the CPU baseline leg only
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    threads = min(threads, os.cpu_count() or threads)
    res = {}
    for sched in ("static", "guided"):  # run_norm.py:18,66 / run_cuda_new.py:79
        oracle.set_schedule(sched, threads)
        tmin, tmax, tavg, used = oracle.time_spmv(A.row_ptr, A.col_idx, A.val, x, warmup=5, runs=20)
        runs = int(max(20, min(20000, budget_s / max(tavg, 1e-6))))
        tmin, tmax, tavg, used = oracle.time_spmv(A.row_ptr, A.col_idx, A.val, x, warmup=5,
                                                  runs=runs)
        res[sched] = (tmin, tmax, tavg, int(used), runs)
    tmin, tmax, tavg, used, runs = res["static"]
    g = res["guided"]
    return {"value": round(2.0 * A.nnz / tavg * 1e-9, 3), "unit": "GFLOP/s", "cores": used,
            "kind": "port",
            "sample": (f"full C2 matrix (m={A.m}, nnz={A.nnz}) fp64, omp_spmv restatement "
                       f"(oracle/spmv_oracle.c), OMP_SCHEDULE=static, 5 warm-ups + {runs} timed "
                       f"runs (spmv-csr/spmv.c:164-185 protocol), value from TimeAvg"),
            "time_min_s": tmin, "time_avg_s": tavg, "time_max_s": tmax,
            "gflops_from_min": round(2.0 * A.nnz / tmin * 1e-9, 3),
            "guided": {"gflops": round(2.0 * A.nnz / g[2] * 1e-9, 3),
                       "gflops_from_min": round(2.0 * A.nnz / g[0] * 1e-9, 3),
                       "time_avg_s": g[2], "runs": g[4]}}


def reference_cpu(A, runs: int = 200):
    """The reference's own spmv-csr program (spmv-csr/spmv.c main, built
    unmodified from /root/reference into oracle/_ref by oracle/Makefile) on
    the fp32 version of the workload, run in a child process exactly as
    `spmv.exe file.csr runs`: its reader, x = 1, `runs` serial test_spmv
    calls, 5 warm-ups and `runs` timed omp_spmv calls (OMP_SCHEDULE=static,
    run_norm.py:18).  Returns its TimeMin/TimeAvg, or None when the library
    was not built (no /root/reference where build() ran)."""
    import subprocess
    import tempfile
    lib = REPO / "oracle" / "_ref" / "libref_spmvcsr.so"
    if not lib.exists():
        return None
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "c2.mtx.rcm.csr")
        hspmv.write_csr(path, A.astype(np.float32))  # the reference's text format (A15)
        code = ("import ctypes, sys; L = ctypes.CDLL(sys.argv[1]); "
                "a = (ctypes.c_char_p * 3)(b'spmv.exe', sys.argv[2].encode(), sys.argv[3].encode()); "
                "L.ref_main(3, a)")
        env = dict(os.environ, OMP_NUM_THREADS=str(threads), OMP_SCHEDULE="static")
        try:
            out = subprocess.run([sys.executable, "-c", code, str(lib), path, str(runs)], env=env,
                                 capture_output=True, text=True, timeout=180)
        except subprocess.TimeoutExpired:
            return None
    vals = {}
    for line in out.stdout.splitlines():  # parsed like run_norm.py:94-107
        for key in ("TimeMin:", "TimeMax:", "TimeAvg:"):
            if line.startswith(key):
                vals[key[:-1]] = float(line[len(key):].strip())
    if out.returncode != 0 or "TimeAvg" not in vals:
        return None
    return {"kind": "reference", "dtype": "f32", "cores": threads,
            "value": round(2.0 * A.nnz / vals["TimeAvg"] * 1e-9, 3), "unit": "GFLOP/s",
            "gflops_from_min": round(2.0 * A.nnz / vals["TimeMin"] * 1e-9, 3),
            "time_min_s": vals["TimeMin"], "time_avg_s": vals["TimeAvg"],
            "time_max_s": vals.get("TimeMax"),
            "sample": (f"the reference's spmv-csr main (oracle/_ref, built from spmv-csr/spmv.c) on "
                       f"the C2 matrix in fp32 (its only dtype), x = 1, num_runs = {runs}, "
                       f"OMP_SCHEDULE=static")}


def main():
    args = parse()
    rank, world, local = dist_setup(args)
    dtype = np.float64
    shard = hdist.build_shard(args.config, rank, world, dtype)
    A = shard.A
    # one non-default stream for everything: the SpMV launches (through the C
    # ABI), the flush writes and the timing events all live on it
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    op = hspmv.SpMV(A, device=local, stream=stream.cuda_stream, kernel=args.kernel,
                    lanes=args.lanes, nontemporal=args.nt)
    info = op.info

    # x: generated on rank 0, broadcast over RCCL (the path's exchange step)
    x = torch.empty(shard.n_global, dtype=torch.float64, device="cuda")
    if rank == 0:
        x.copy_(torch.from_numpy(gen.rand_x(shard.n_global, 42)))
    barrier(world)
    t0 = time.perf_counter()
    if world > 1:
        hdist.broadcast_x(x)
    barrier(world)
    bcast_ms = (time.perf_counter() - t0) * 1e3
    y = torch.empty(A.m, dtype=torch.float64, device="cuda")
    op.bind_x_device(x.data_ptr())
    op.bind_y_device(y.data_ptr())

    # warmup
    for _ in range(args.warmup):
        op.spmv()
    barrier(world)

    # timed region: exactly K steps
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(world)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        op.spmv()
    ev1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    barrier(world)
    step_s = max_over_ranks(wall / args.steps, world)
    ev_launch_s = ev0.elapsed_time(ev1) * 1e-3 / args.steps  # avg launch on this stream

    # cold: evict the 256 MiB Infinity Cache before every launch by READING a
    # 512 MiB buffer (a read leaves no dirty lines whose write-back the SpMV
    # would then pay for)
    flush = torch.ones(64 << 20, dtype=torch.float64, device="cuda")
    sink = torch.empty(1, dtype=torch.float64, device="cuda")
    cold = []
    for _ in range(args.cold_steps):
        torch.sum(flush, dim=0, out=sink)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        op.spmv()
        b.record(stream)
        torch.cuda.synchronize()
        cold.append(a.elapsed_time(b) * 1e-3)
    del flush, sink
    cold_s = max_over_ranks(float(np.median(cold)), world)

    # correctness property on the last y (no oracle in the product bench)
    y_host = y.cpu().numpy()
    ok, rel = hdist.checksum_ok(A, x.cpu().numpy(), y_host)
    ok_all = sum_over_ranks(1.0 if ok else 0.0, world) == world

    # exchange step costs (reported, not in the step): y all-gather over RCCL,
    # and the halo exchange that replaces the x broadcast when x is
    # distributed like y (iterative use; point-to-point RCCL send/recv)
    gather_ms = halo_ms = None
    halo_b = 0
    if world > 1:
        times = []
        for _ in range(5):
            barrier(world)
            t0 = time.perf_counter()
            yfull = hdist.gather_y(y, shard.splits)
            barrier(world)
            times.append((time.perf_counter() - t0) * 1e3)
            del yfull
        gather_ms = max_over_ranks(float(np.median(times)), world)
        halo = hdist.plan_halo(A, shard.splits, rank, world)
        xw = x[halo.lo:halo.hi].clone()
        times = []
        for _ in range(20):
            barrier(world)
            t0 = time.perf_counter()
            hdist.halo_exchange(xw, halo)
            torch.cuda.synchronize()
            times.append((time.perf_counter() - t0) * 1e3)
        halo_ms = max_over_ranks(float(np.median(times)), world)
        halo_b = int(max_over_ranks(float(hdist.halo_bytes(halo)), world))
        halo_ok = bool(torch.equal(xw, x[halo.lo:halo.hi]))
        ok_all = ok_all and sum_over_ranks(1.0 if halo_ok else 0.0, world) == world
        del xw

    flops_step = 2.0 * shard.nnz_global
    alg_local = info["alg_bytes"]  # x counted as the distinct columns this shard reads
    alg_total = sum_over_ranks(alg_local, world)
    gflops = flops_step / step_s * 1e-9
    achieved = alg_local / ev_launch_s * 1e-9
    workload_key = f"{args.config}-w{world}-r0-{info['kernel_name']}"
    traffic = load_traffic(workload_key) if rank == 0 else None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(A, x.cpu().numpy(), args.cpu_seconds)
        cpu["reference_f32"] = reference_cpu(A)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(gflops, 3),
            "unit": "GFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(step_s * 1e3, 6),
            "higher_is_better": True,
            "scaling": shard.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded generator, hspmv.gen); x = rand_x(n, 42)",
            "config": {"workload": f"{args.config}: {shard.name}", "m": shard.m_global,
                       "nnz": shard.nnz_global, "rows_per_gpu": int(A.m),
                       "kernel": info["kernel_name"], "lanes": info["lanes"],
                       "nontemporal": bool(args.nt), "parallelism": f"row-range x{world}",
                       "workload_key": workload_key, "col16": info["col16"]},
            "gbps_alg": round(alg_total / step_s * 1e-9, 2),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": (traffic["hbm_bytes_per_launch"] if traffic else None),
                         "kernel": f"hspmv_csr_{info['kernel_name']}<double>",
                         "alg_bytes_per_launch": alg_local,
                         "format_bytes_per_launch": info["format_bytes"],
                         "launch_us_events": round(ev_launch_s * 1e6, 3),
                         "traffic_source": (traffic["source"] if traffic else None)},
            "cold": {"launch_us": round(cold_s * 1e6, 3),
                     "gbps_alg": round(alg_local / cold_s * 1e-9, 2),
                     "gflops": round(flops_step / cold_s * 1e-9, 3),
                     "note": "a 512 MiB read before each launch evicts the Infinity Cache"},
            "comm": {"bcast_x_ms": round(bcast_ms, 3) if world > 1 else None,
                     "gather_y_ms": round(gather_ms, 3) if gather_ms is not None else None,
                     "halo_x_ms": round(halo_ms, 4) if halo_ms is not None else None,
                     "x_bytes": shard.n_global * 8, "y_bytes": shard.m_global * 8,
                     "halo_bytes_per_rank": halo_b if world > 1 else None,
                     "end_to_end_gflops": (round(flops_step / (step_s + gather_ms * 1e-3) * 1e-9, 3)
                                           if gather_ms is not None else round(gflops, 3)),
                     "iterative_gflops": (round(flops_step / (step_s + halo_ms * 1e-3) * 1e-9, 3)
                                          if halo_ms is not None else round(gflops, 3))},
            "check": {"pass": bool(ok_all), "checksum_rel": rel},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    op.close()
    if world > 1:
        dist.destroy_process_group()
    if not ok_all:
        sys.exit(3)


if __name__ == "__main__":
    main()
