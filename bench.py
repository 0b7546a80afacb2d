#!/usr/bin/env python3
"""bench.py -- SpMV GFLOP/s and achieved HBM GB/s (fp64) on 1..8 MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1
launched with torch.distributed.run, one rank per GPU -- or, when no launcher
set WORLD_SIZE, bench.py starts that launcher itself as a child process (the
parent touches no GPU, relays rank 0's line and exits with the child's code;
``self_launch``).  A "step" is one SpMV
y = A x over every rank's row-range shard of the workload (inputs resident in
HBM; no data-path collective -- rows are independent).
W untimed steps, then exactly K steps bracketed by barrier + synchronize; the
max over ranks is the step time; rank 0 prints ONE JSON line.

Workload (``--config``, default by world size; hspmv.dist.default_config):
  N = 1  c3: BASELINE configs[2], the largest single-GPU configuration --
         CSR-3 fp64 on the 27-point 125^3 stencil, RCM-permuted
         (m = 1,953,125, nnz = 51,895,117), maps (ssrs, srs) = (20, 10) from
         the .csr3 writer heuristic; the hspmv_csr3 kernel.
  N > 1  c4: BASELINE configs[3], the 2e7-row banded matrix (~200 M nnz)
         row-range partitioned over the N GPUs, nnz-balanced (strong scaling).
  Also: c2 (configs[1], weak scaling: 1000 x 1000 rows per GPU), c3h (the
  hugebubbles-00000 stand-in), c5 (configs[4], CSR-3 fp32 power-law) and c5r
  (the same matrix RCM-permuted, the reference's input ordering).
``--dry-run`` prints the partition plan without touching a GPU.

Extra fields on the line:
  roofline     one SpMV (the kernel launch(es) of a step), algorithmic bytes
               per SpMV / HIP-event-timed average over the timed region on
               the launch stream, vs 8 TB/s HBM; traffic from the committed
               rocprofv3 PMC summary for this workload (profiles/*_pmc.json).
               Every leg runs inside a roctx range (bench:headline,
               bench:headline_cold, bench:plan_packed, bench:plan_ssr,
               bench:n1_<cfg>[_cold]): rocprofv3 --kernel-trace --marker-trace
               --kernel-rename --stats then reports each leg's kernels apart
  cold         the same SpMV with the 256 MiB Infinity Cache evicted before
               every launch (a 512 MiB read)
  comm         RCCL x broadcast / y all-gather / halo-exchange times (N > 1),
               timed separately, and the end-to-end rates they imply; plus the
               y all-gather OVERLAPPED with the SpMV (rows in K chunks, chunk k
               gathered while chunks k+1.. compute; hspmv.dist.OverlappedGather)
  csr3_maps_plans  (CSR-3 workloads) the same SpMV under the two maps-driven
               CSR-3 plans, timed in the same process: "packed" (whole
               super-rows of the inner map packed into <= 64-row wave tasks)
               and "ssr" (one workgroup per super-super-row of the outer map,
               the reference's cuSpMV_3 mapping, csrk.cu:245-319); the
               headline times config.csr3_plan ("aligned": 64-row tasks)
  scaling_reference  (N = 1) the N > 1 default workload, C4, timed on this
               one GPU: the same-matrix N = 1 point for the strong-scaling
               curve, its y checked like the headline's
  strong_scaling (N > 1) the same workload timed on rank 0's GPU alone in
               the same job: n1_gflops, efficiency = value / (N n1), and the
               cold (Infinity-Cache-evicted) pair cold_gflops /
               cold_efficiency, so a warm shard that fits the cache cannot
               read as super-linear scaling
  cpu_baseline the oracle's OpenMP restatement of spmv-csr's omp_spmv on the
               host cores, on the SAME matrix (rank 0 at N = 1 only, bounded
               sample, a process of its own: oracle/cpu_bench.py), value from
               TimeMin as run_norm.py records it (median and TimeAvg beside
               it), on the cgroup CPU quota minus one thread, one per L3
               domain, matrix first-touched per thread; beside it
               reference_f32: the reference's own omp_spmv (spmv-csr/spmv.c,
               built unmodified into oracle/_ref) on the fp32 copy
  cpu_c1       BASELINE configs[0] itself: the same OpenMP restatement on the
               1000 x 1000 5-point Laplacian (m = 1e6, nnz = 4,996,000) in
               fp64, x = 1 (the reference CLI's x) and x = rand:42, under
               OMP_SCHEDULE static and guided (run_norm.py:18,65-66,
               run_cuda_new.py:79), 5 warm-ups + timed runs, TimeMin / TimeMax
               / TimeAvg and GFLOP/s from TimeMin (rank 0 at N = 1 only)
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import time
from pathlib import Path

# before any libgomp loads: the CPU baseline's schedule (run_norm.py:18,66).
# OMP_PROC_BIND / OMP_PLACES are NOT set: libgomp then pins
# the main thread to one core at load, which shrinks the affinity mask the
# baseline reads its thread count from to that core (r02x: 2 threads,
# 11.5 GFLOP/s instead of 128 threads, 144 GFLOP/s).
os.environ.setdefault("OMP_SCHEDULE", "static")

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "heterogeneous-spmv_amd"))

import numpy as np  # noqa: E402

METRIC = "SpMV GFLOP/s and achieved HBM GB/s (fp64) per matrix, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="auto", choices=["auto", "c2", "c3", "c3h", "c4", "c5", "c5r"],
                    help="auto: c3 at N = 1, c4 at N > 1")
    ap.add_argument("--kernel", default="auto", choices=["auto", "stream", "vector", "csr3"])
    ap.add_argument("--lanes", type=int, default=0)
    ap.add_argument("--nt", action="store_true", help="non-temporal matrix loads")
    ap.add_argument("--xcd-chunk", type=int, default=0,
                    help="workgroups per XCD turn (0 = the planner's choice, 1 = dispatch order)")
    ap.add_argument("--cold-steps", type=int, default=20)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="budget of the CPU-baseline sample (rank 0, N=1)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-plans", action="store_true",
                    help="skip the csr3_maps_plans legs (maps-driven CSR-3 plans)")
    ap.add_argument("--no-scaling-ref", action="store_true",
                    help="skip the one-GPU reference point (N = 1: C4 on this GPU; N > 1: "
                         "the run's workload on rank 0's GPU)")
    ap.add_argument("--dry-run", action="store_true",
                    help="print the workload and partition plan, touch no GPU")
    # rehearsal of the N > 1 path on a one-GPU box: every rank on device 0,
    # gloo for the exchanges (RCCL allows one rank per device); never the
    # driver's configuration
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"], help=argparse.SUPPRESS)
    ap.add_argument("--same-device", action="store_true", help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.gpus < 1:
        ap.error("--gpus must be >= 1")
    if a.steps < 1 or a.warmup < 0:
        ap.error("--steps must be >= 1 and --warmup >= 0")
    return a


def resolve_config(args) -> str:
    from hspmv import dist as hdist
    return hdist.default_config(args.gpus) if args.config == "auto" else args.config


def dry_run(args) -> None:
    """CPU-side plan: the configuration and the nnz-balanced row partition the
    run would use (closed-form row lengths; no matrix is built)."""
    from hspmv import dist as hdist
    cfg = resolve_config(args)
    out = {"dry_run": True, "n_gpus": args.gpus, "steps": args.steps, "warmup": args.warmup,
           "config": cfg, "metric": METRIC}
    try:
        out["plan"] = hdist.plan_splits(cfg, args.gpus)
    except ValueError:
        out["plan"] = {"config": cfg, "world": args.gpus, "scaling": "strong",
                       "note": "row lengths known only after generating the matrix"}
    print(json.dumps(out), flush=True)


# ------------------------------------------------------------------ trace ranges

class _Roctx:
    """roctx ranges around the bench's legs, so that a rocprofv3 run of this
    script with ``--kernel-trace --marker-trace --kernel-rename --stats``
    reports each leg's kernels under the leg's name (the headline's aligned
    CSR-3 launches apart from the packed / ssr legs, which launch the same
    kernel template).  Loaded from ROCm's roctx library through ctypes; a
    no-op when it is absent.  Outside a profiler the calls cost nothing
    measurable and sit outside every timed region."""

    def __init__(self):
        self.lib = None
        self.tried = False  # loaded on first use: the self-launching parent never loads it

    def load(self):
        self.tried = True
        import ctypes
        for name in ("librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1"):
            try:
                self.lib = ctypes.CDLL(name)
                self.lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                break
            except OSError:
                continue

    def push(self, name: str) -> None:
        if not self.tried:
            self.load()
        if self.lib is not None:
            self.lib.roctxRangePushA(name.encode())

    def pop(self) -> None:
        if self.lib is not None:
            self.lib.roctxRangePop()


ROCTX = _Roctx()


class leg_range:
    """``with leg_range("bench:headline"): ...`` -- one roctx range."""

    def __init__(self, name: str):
        self.name = name

    def __enter__(self):
        ROCTX.push(self.name)
        return self

    def __exit__(self, *exc):
        ROCTX.pop()
        return False


# ------------------------------------------------------------------ torch plumbing

def dist_setup(args):
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a HIP GPU")
    if args.same_device:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    return rank, world, local


def barrier(world):
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def reduce_over_ranks(v: float, world: int, op: str) -> float:
    if world == 1:
        return v
    import torch
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return float(t.item())


def round_order(p: Path):
    """Sort key of a profile name 'r<round><pass letters>_...': round, then
    pass (a..z, then aa..zz), then the name."""
    m = re.match(r"r(\d+)([a-z]*)_", p.name)
    if not m:
        return (-1, 0, "", p.name)
    return (int(m.group(1)), len(m.group(2)), m.group(2), p.name)


def load_traffic(workload_key: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary
    (profiles/*_pmc.json, written by heterogeneous-spmv_amd/tools/pmc_summary.py),
    or None when no summary for this workload exists.  The newest file wins
    (profiles are named per round and pass: r01_ < r02_ < r02a < r02z <
    r02aa ..., by round_order)."""
    best = None
    for p in sorted((REPO / "profiles").glob("*_pmc.json"), key=round_order):
        try:
            d = json.loads(p.read_text())
        except Exception:
            continue
        if d.get("workload") == workload_key and d.get("hbm_bytes_per_launch"):
            best = d
            best["file"] = str(p.relative_to(REPO))
    return best


# ------------------------------------------------------------------ CPU baseline

# OpenMP wait policy of the CPU-baseline process (None: libgomp's default,
# spin then sleep).  Measured on the GPU box (profiles/r04b_cpu_baseline_ab.jsonl).
CPU_WAIT_POLICY = None


def cpu_baseline(A, x, budget_s: float, extra_args=()):
    """The CPU legs (oracle/cpu_bench.py: the oracle's omp_spmv restatement,
    spmv-csr/spmv.c:92-114, and the reference's own omp_spmv in fp32) on the
    SAME matrix, in a process of their own: the matrix and x go through a
    scratch directory, the legs' JSON comes back on stdout.  value = 2 nnz /
    TimeMin (run_norm.py records min/max/avg), median and
    TimeAvg beside it; threads = the cgroup CPU quota minus one, one per L3
    domain, matrix first-touched per thread (see oracle/cpu_bench.py)."""
    import shutil
    import tempfile
    d = Path(tempfile.mkdtemp(prefix="hspmv_cpu_", dir="/dev/shm" if Path("/dev/shm").is_dir() else None))
    try:
        np.save(d / "row_ptr.npy", np.ascontiguousarray(A.row_ptr, np.int32))
        np.save(d / "col_idx.npy", np.ascontiguousarray(A.col_idx, np.int32))
        np.save(d / "val.npy", np.ascontiguousarray(A.val))
        np.save(d / "x.npy", np.ascontiguousarray(x, A.val.dtype))
        env = {k: v for k, v in os.environ.items() if not k.startswith(("OMP_", "GOMP_"))}
        env["OMP_SCHEDULE"] = "static"
        if CPU_WAIT_POLICY:
            env["OMP_WAIT_POLICY"] = CPU_WAIT_POLICY
        out = subprocess.run([sys.executable, str(REPO / "oracle" / "cpu_bench.py"), "--dir", str(d),
                              "--budget", str(budget_s), *extra_args], env=env, capture_output=True,
                             text=True, timeout=600)
        if out.returncode != 0:
            raise RuntimeError(f"oracle/cpu_bench.py failed: {out.stderr[-1500:]}")
        return json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    finally:
        shutil.rmtree(d, ignore_errors=True)


def cpu_c1(budget_s: float) -> dict:
    """BASELINE configs[0]: spmv-csr's OpenMP loop (the oracle's omp_spmv
    restatement, oracle/cpu_bench.py) on the 1000 x 1000 5-point Laplacian in
    fp64 on this box's host cores.  Both x the reference CLI knows of -- x = 1
    (spmv-csr/spmv.c:133) and a seeded x = rand:42 -- each under
    OMP_SCHEDULE static and guided (run_norm.py:18,65-66; run_cuda_new.py:79),
    5 warm-ups + timed runs around each call (spmv.c:164-185); TimeMin /
    TimeMax / TimeAvg in seconds and GFLOP/s = 2 nnz / TimeMin."""
    from hspmv import gen
    A = gen.laplace2d(1000, 1000)
    legs, first = {}, None
    for name, x in (("ones", np.ones(A.n)), ("rand:42", gen.rand_x(A.n, 42))):
        c = cpu_baseline(A, x, budget_s, ("--no-tried", "--no-reference"))
        first = first or c
        legs[name] = {
            sched: {"TimeMin": leg["time_min_s"], "TimeMax": leg["time_max_s"],
                    "TimeAvg": leg["time_avg_s"], "gflops": round(2.0 * A.nnz / leg["time_min_s"] * 1e-9, 3),
                    "runs": leg["runs"]}
            for sched, leg in (("static", dict(c, runs=c["guided"]["runs"])), ("guided", c["guided"]))}
    return {"config": "c1: spmv-csr OpenMP fp64, 5-pt Laplacian 1000 x 1000", "m": A.m, "nnz": A.nnz,
            "dtype": "f64", "kind": "port", "cores": first["cores"], "cores_note": first["cores_note"],
            "cgroup_cpu_quota": first["cgroup_cpu_quota"], "x": legs,
            "value": legs["rand:42"]["static"]["gflops"], "unit": "GFLOP/s",
            "sample": (f"gen.laplace2d(1000, 1000): m={A.m}, nnz={A.nnz}, fp64 CSR; omp_spmv restatement "
                       f"(oracle/spmv_oracle.c), {first['cores']} threads, 5 warm-ups + the timed runs "
                       f"in x[x][schedule].runs (a {max(0.2, budget_s):.1f} s budget per x); value = "
                       f"x rand:42, static, 2 nnz / TimeMin")}


def single_gpu_point(args, stream, cfg: str):
    """Workload `cfg` as a world-1 run on THIS GPU, same protocol as the step
    (warm K/10 back-to-back launches, wall-clock per step; the median of
    cold launches, the Infinity Cache evicted before each): the N = 1 point
    of the scaling curve whose N-rank points bench.py --gpus N reports.  Its
    y gets the headline's property check."""
    import torch

    import hspmv
    from hspmv import dist as hdist
    from hspmv import gen
    sh = hdist.build_shard(cfg, 0, 1)
    A = sh.A
    op = hspmv.SpMV(A, sh.maps, device=torch.cuda.current_device(), stream=stream.cuda_stream)
    x = torch.from_numpy(gen.rand_x(sh.n_global, 42, dtype=A.val.dtype)).to("cuda")
    y = torch.empty(A.m, dtype=x.dtype, device="cuda")
    op.bind_x_device(x.data_ptr())
    op.bind_y_device(y.data_ptr())
    for _ in range(max(3, args.warmup // 4)):
        op.spmv()
    steps = max(10, args.steps // 10)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with leg_range(f"bench:n1_{cfg}"):
        t0 = time.perf_counter()
        ev0.record(stream)
        for _ in range(steps):
            op.spmv()
        ev1.record(stream)
        torch.cuda.synchronize()
        step_s = (time.perf_counter() - t0) / steps
    ev_s = ev0.elapsed_time(ev1) * 1e-3 / steps
    flush = torch.ones(64 << 20, dtype=torch.float64, device="cuda")
    cold = []
    for _ in range(max(3, args.cold_steps)):
        flush.sum()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with leg_range(f"bench:n1_{cfg}_cold"):
            a.record(stream)
            op.spmv()
            b.record(stream)
            torch.cuda.synchronize()
        cold.append(a.elapsed_time(b) * 1e-3)
    del flush
    cold_s = float(np.median(cold))
    info = op.info
    op.close()
    # the same property check as the headline's y (no oracle in the bench)
    ok, rel = hdist.checksum_ok(A, x.cpu().numpy(), y.cpu().numpy())
    return {"config": f"{cfg}: {sh.name}", "n_gpus": 1, "m": sh.m_global, "nnz": sh.nnz_global,
            "check": {"pass": bool(ok), "checksum_rel": rel},
            "value": round(2.0 * sh.nnz_global / step_s * 1e-9, 3), "unit": "GFLOP/s",
            "ms_per_step": round(step_s * 1e3, 6), "steps": steps,
            "launch_us_events": round(ev_s * 1e6, 3), "kernel": info["kernel_name"],
            "frac": round(info["alg_bytes"] / ev_s * 1e-9 / HBM_PEAK_GBS, 4),
            "cold_launch_us": round(cold_s * 1e6, 3),
            "cold_gflops": round(2.0 * sh.nnz_global / cold_s * 1e-9, 3)}


def scaling_reference(args, stream):
    """(N = 1) the N > 1 default workload (C4, the whole 200 M-nnz banded
    matrix) on this one GPU (the N = 1 headline is C3, a different matrix)."""
    from hspmv import dist as hdist
    d = single_gpu_point(args, stream, hdist.default_config(2))
    d["note"] = ("the N > 1 default workload on this one GPU: every bench.py --gpus N line "
                 "carries its own strong_scaling block measured the same way")
    return d


def strong_scaling(n1: dict, world: int, gflops: float, cold_gflops):
    """The N-rank point against the same workload on one GPU of this node
    (rank 0's GPU, timed in the same job): efficiency = value / (N * n1),
    warm and cold.  Warm shards of a strong-scaled matrix shrink into the
    256 MiB Infinity Cache (C4 at N = 8: 350 MB per rank, partly resident
    across back-to-back launches) while the whole matrix on one GPU streams
    from HBM, so warm efficiency can read super-linear; the cold ratio evicts
    the cache before every launch on both sides."""
    eff = gflops / (world * n1["value"]) if n1["value"] else None
    ceff = (cold_gflops / (world * n1["cold_gflops"])
            if cold_gflops and n1["cold_gflops"] else None)
    return {"n1_gflops": n1["value"], "efficiency": round(eff, 4) if eff is not None else None,
            "n1_cold_gflops": n1["cold_gflops"], "cold_gflops": round(cold_gflops, 3) if cold_gflops else None,
            "cold_efficiency": round(ceff, 4) if ceff is not None else None,
            "speedup": round(gflops / n1["value"], 3) if n1["value"] else None,
            "n1": n1}


def csr3_maps_plans(args, A, maps, x, y_ref, stream, device):
    """The same CSR-3 SpMV under the two maps-driven plans (hspmv_options
    csr3_plan), in this process, with the headline's protocol: "packed"
    packs whole super-rows of the inner map into <= 64-row wave tasks;
    "ssr" gives each super-super-row of the outer map one workgroup, its
    super-rows split over the waves by nonzeros -- the reference's cuSpMV_3
    mapping (csrk.cu:245-319, launched spmv-auto-mi100.cu:200-236).  The row
    sums are row-local, so y must equal the headline's bit for bit."""
    import torch

    import hspmv
    out = {}
    for plan in ("packed", "ssr"):
        op = hspmv.SpMV(A, maps, device=device, stream=stream.cuda_stream,
                        options={"csr3_plan": plan})
        info = op.info
        y = torch.empty_like(y_ref)
        op.bind_x_device(x.data_ptr())
        op.bind_y_device(y.data_ptr())
        for _ in range(args.warmup):
            op.spmv()
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with leg_range(f"bench:plan_{plan}"):
            ev0.record(stream)
            for _ in range(args.steps):
                op.spmv()
            ev1.record(stream)
            torch.cuda.synchronize()
        s = ev0.elapsed_time(ev1) * 1e-3 / args.steps
        out[plan] = {"launch_us_events": round(s * 1e6, 3),
                     "gflops": round(2.0 * A.nnz / s * 1e-9, 3),
                     "frac": round(info["alg_bytes"] / s * 1e-9 / HBM_PEAK_GBS, 4),
                     "kernel": info["kernel_name"], "wave_tasks": info["wave_tasks"],
                     "waves_per_block": info["waves_per_block"], "blocks": info["blocks"],
                     "x_dict": info["x_dict"], "csr3_plan": info["csr3_plan"],
                     "y_bitwise_equal_to_headline": bool(torch.equal(y, y_ref))}
        op.close()
    return out


def overlapped_gather(args, A, shard, x, y, stream, device, info, world, chunks: int = 4):
    """One SpMV + the y all-gather, overlapped: this rank's rows in `chunks`
    nnz-balanced handles launched back to back on the SpMV stream, each
    chunk's rows all-gathered (async, RCCL's stream) right after its kernel,
    so the exchange of chunk k overlaps chunks k+1..  Timed end to end
    (launch of the first chunk to the assembled full y), max over ranks; y
    checked against the plain gather of the headline y."""
    import torch

    import hspmv
    from hspmv import dist as hdist
    sub = hdist.chunk_splits(A, chunks)
    og = hdist.OverlappedGather(np.diff(sub), device="cuda", dtype=y.dtype)
    ops = []
    for k in range(chunks):
        a, b = int(sub[k]), int(sub[k + 1])
        op = hspmv.SpMV(A.rows(a, b), device=device, stream=stream.cuda_stream)
        op.bind_x_device(x.data_ptr())
        op.bind_y_device(og.buffer(k).data_ptr())
        ops.append(op)

    def once():
        for k, op in enumerate(ops):
            op.spmv()
            og.start(k)
        return og.finish()

    ref = hdist.gather_y(y, shard.splits)
    for _ in range(2):
        yfull = once()
    torch.cuda.synchronize()
    times = []
    for _ in range(5):
        barrier(world)
        t0 = time.perf_counter()
        yfull = once()
        torch.cuda.synchronize()
        times.append((time.perf_counter() - t0) * 1e3)
        barrier(world)
    ms = reduce_over_ranks(float(np.median(times)), world, "max")
    if info["deterministic"]:
        ok = bool(torch.equal(yfull, ref))
    else:  # csort shards: the same y within the summation order -- and, with
        # fp32 row partials per column part, within an fp32 rounding of each
        # part's sum, which on a row whose parts cancel is absolute, not
        # relative to that row's y (hence the atol on the largest |y|)
        tol = 1e-5 if y.dtype == torch.float32 else 1e-12
        ok = bool(torch.allclose(yfull, ref, rtol=tol, atol=tol * float(ref.abs().max())))
    ok = reduce_over_ranks(1.0 if ok else 0.0, world, "sum") == world
    for op in ops:
        op.close()
    return ({"chunks": chunks, "ms": round(ms, 4),
             "end_to_end_overlapped_gflops": round(2.0 * shard.nnz_global / (ms * 1e-3) * 1e-9, 3),
             "y_equal_to_plain_gather": ok}, ok)


# ------------------------------------------------------------------ main

# Environment the ranks of a self-launched run get when the caller left it
# unset.  HSA_ENABLE_IPC_MODE_LEGACY=0: the box's driver only supports dmabuf
# IPC, and RCCL's peer setup fails with hipIpcGetMemHandle: invalid argument
# without it.
RANK_ENV = {"HSA_ENABLE_IPC_MODE_LEGACY": "0"}


def launch_command(argv, gpus: int, port: int) -> list:
    """torch.distributed.run over this script with the same arguments: one
    rank per GPU of this node, rendezvous on 127.0.0.1."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), str(Path(__file__).resolve()),
            *argv]


def self_launch(args, argv) -> int:
    """``bench.py --gpus N`` (N > 1) with no launcher around it: start the
    launcher as a CHILD process (never exec: this process must not replace
    itself, and it touches no GPU -- torch is not even imported here), relay
    the ranks' stdout (rank 0's one JSON line), return the child's exit code.
    The reference's harness runs its binaries directly (run_norm.py:73-76);
    this keeps the same one-command shape for the N-GPU runs."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    for k, v in RANK_ENV.items():
        env.setdefault(k, v)
    import signal
    proc = subprocess.Popen(launch_command(argv, args.gpus, port), env=env, stdout=subprocess.PIPE,
                            text=True, bufsize=1)

    def stop(signum, _frame):  # a timeout's SIGTERM reaches the ranks too
        proc.send_signal(signum)

    signal.signal(signal.SIGTERM, stop)
    try:
        for line in proc.stdout:
            sys.stdout.write(line)
            sys.stdout.flush()
    except KeyboardInterrupt:
        proc.send_signal(signal.SIGINT)
    return proc.wait()


def main():
    args = parse()
    if args.dry_run:
        dry_run(args)
        return
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args, sys.argv[1:]))
    import torch  # device memory, streams, torch.distributed: plumbing

    import hspmv
    from hspmv import dist as hdist
    from hspmv import gen

    rank, world, local = dist_setup(args)
    cfg = resolve_config(args)
    shard = hdist.build_shard(cfg, rank, world)
    A, maps = shard.A, shard.maps
    np_dt = A.val.dtype
    tdt = torch.float64 if np_dt == np.float64 else torch.float32
    # one non-default stream for everything: the SpMV launches (through the C
    # ABI), the flush reads and the timing events all live on it
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    op = hspmv.SpMV(A, maps, device=local, stream=stream.cuda_stream, kernel=args.kernel,
                    lanes=args.lanes, nontemporal=args.nt,
                    xcd_remap=(False if args.xcd_chunk == 1 else None),
                    xcd_chunk=(args.xcd_chunk if args.xcd_chunk > 1 else 0))
    info = op.info

    # x: generated on rank 0, broadcast over RCCL (the path's exchange step)
    x = torch.empty(shard.n_global, dtype=tdt, device="cuda")
    if rank == 0:
        x.copy_(torch.from_numpy(gen.rand_x(shard.n_global, 42, dtype=np_dt)))
    barrier(world)
    t0 = time.perf_counter()
    if world > 1:
        hdist.broadcast_x(x)
    barrier(world)
    bcast_ms = (time.perf_counter() - t0) * 1e3
    y = torch.empty(A.m, dtype=tdt, device="cuda")
    op.bind_x_device(x.data_ptr())
    op.bind_y_device(y.data_ptr())

    for _ in range(args.warmup):
        op.spmv()
    barrier(world)

    # timed region: exactly K steps; HIP events on the launch stream bracket
    # the same K SpMVs (the kernel-side time of one SpMV = their average)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(world)
    with leg_range("bench:headline"):  # the K timed launches only
        t0 = time.perf_counter()
        ev0.record(stream)
        for _ in range(args.steps):
            op.spmv()
        ev1.record(stream)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
    barrier(world)
    step_s = reduce_over_ranks(wall / args.steps, world, "max")
    ev_launch_s = ev0.elapsed_time(ev1) * 1e-3 / args.steps

    # cold: evict the 256 MiB Infinity Cache before every launch by READING a
    # 512 MiB buffer (a read leaves no dirty lines whose write-back the SpMV
    # would then pay for)
    flush = torch.ones(64 << 20, dtype=torch.float64, device="cuda")
    cold = []
    for _ in range(args.cold_steps):
        flush.sum()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with leg_range("bench:headline_cold"):
            a.record(stream)
            op.spmv()
            b.record(stream)
            torch.cuda.synchronize()
        cold.append(a.elapsed_time(b) * 1e-3)
    del flush
    cold_s = reduce_over_ranks(float(np.median(cold)), world, "max") if cold else None

    # correctness property on the last y (no oracle in the product bench)
    x_host = x.cpu().numpy()
    ok, rel = hdist.checksum_ok(A, x_host, y.cpu().numpy())
    ok_all = reduce_over_ranks(1.0 if ok else 0.0, world, "sum") == world

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
        gather_ms = reduce_over_ranks(float(np.median(times)), world, "max")
        halo = hdist.plan_halo(A, shard.splits, rank, world)
        xw = x[halo.lo:halo.hi].clone()
        times = []
        for _ in range(20):
            barrier(world)
            t0 = time.perf_counter()
            hdist.halo_exchange(xw, halo)
            torch.cuda.synchronize()
            times.append((time.perf_counter() - t0) * 1e3)
        halo_ms = reduce_over_ranks(float(np.median(times)), world, "max")
        halo_b = int(reduce_over_ranks(float(hdist.halo_bytes(halo, x.element_size())), world, "max"))
        halo_ok = bool(torch.equal(xw, x[halo.lo:halo.hi]))
        ok_all = ok_all and reduce_over_ranks(1.0 if halo_ok else 0.0, world, "sum") == world
        del xw
        overlap, ov_ok = overlapped_gather(args, A, shard, x, y, stream, local, info, world)
        ok_all = ok_all and ov_ok

    flops_step = 2.0 * shard.nnz_global
    alg_local = info["alg_bytes"]  # x counted as the distinct columns this shard reads
    alg_total = reduce_over_ranks(alg_local, world, "sum")
    gflops = flops_step / step_s * 1e-9
    achieved = alg_local / ev_launch_s * 1e-9
    workload_key = f"{cfg}-w{world}-r0-{info['kernel_name']}"
    traffic = load_traffic(workload_key) if rank == 0 else None

    plans = None
    if maps is not None and info["kernel_name"] == "csr3" and not args.no_plans:
        plans = csr3_maps_plans(args, A, maps, x, y, stream, local)
        ok_all = ok_all and reduce_over_ranks(
            1.0 if all(p["y_bitwise_equal_to_headline"] for p in plans.values()) else 0.0,
            world, "sum") == world

    sref = None
    if world == 1 and cfg != hdist.default_config(2) and not args.no_scaling_ref:
        sref = scaling_reference(args, stream)
        ok_all = ok_all and sref["check"]["pass"]

    # N > 1: the same workload on rank 0's GPU alone, timed after the
    # sharded run while the other ranks wait -- every N > 1 line is then a
    # self-contained scaling point (warm and cold efficiency)
    scal = None
    if world > 1 and not args.no_scaling_ref:
        barrier(world)
        n1 = single_gpu_point(args, stream, cfg) if rank == 0 else None
        barrier(world)
        if rank == 0:
            ok_all = ok_all and n1["check"]["pass"]
            cold_g = 2.0 * shard.nnz_global / cold_s * 1e-9 if cold_s else None
            scal = strong_scaling(n1, world, flops_step / step_s * 1e-9, cold_g)
        ok_all = reduce_over_ranks(1.0 if ok_all else 0.0, world, "sum") == world

    cpu = c1 = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(A, x_host, args.cpu_seconds)
        c1 = cpu_c1(max(0.2, 0.25 * args.cpu_seconds))

    if rank == 0:
        ctype = "double" if np_dt == np.float64 else "float"
        kname = {"csr3": "hspmv_csr3", "stream": "hspmv_csr_stream", "csort": "hspmv_csort",
                 "vector": "hspmv_csr_vector"}.get(info["kernel_name"], info["kernel_name"])
        csort = info["kernel_name"] == "csort"
        launches = 1 if csort else (info["x_slabs"] or 1)
        # csort: the finishing pass (column parts / long-row slices) unless the
        # block sums are written to y directly (one part, no long rows)
        extra = (0 if (info["csort_parts"] == 1 and not info["n_split_rows"]) else 1) if csort else \
            (2 if info["n_split_rows"] else 0)
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
            "dtype": "f64" if np_dt == np.float64 else "f32",
            "data": "synthetic (seeded generator, hspmv.gen); x = rand_x(n, 42)",
            "config": {"workload": f"{cfg}: {shard.name}", "m": shard.m_global,
                       "nnz": shard.nnz_global, "rows_per_gpu": int(A.m), "nnz_per_gpu": int(A.nnz),
                       "csr3_maps": ({"n_ssr": maps.n_ssr, "n_sr": maps.n_sr} if maps is not None
                                     else None),
                       "kernel": info["kernel_name"], "chunk_u": info["chunk_u"],
                       "csr3_plan": hspmv._lib.CSR3_PLAN_NAMES[info["csr3_plan"]],
                       "deterministic": bool(info["deterministic"]),
                       "xcd_chunk": info["xcd_remap"],
                       "x_dict": info["x_dict"], "x_windows": info["x_windows"],
                       "x_slabs": info["x_slabs"], "col16": info["col16"],
                       "nontemporal": bool(args.nt), "parallelism": f"row-range x{world}",
                       "workload_key": workload_key},
            "gbps_alg": round(alg_total / step_s * 1e-9, 2),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": (traffic["hbm_bytes_per_launch"] if traffic else None),
                         "kernel": f"{kname}<{ctype},...>",
                         "row_kernel_launches_per_spmv": launches,
                         "split_row_launches_per_spmv": 0 if csort else extra,
                         "finish_launches_per_spmv": extra if csort else 0,
                         "launches_per_spmv": launches + extra,
                         "csort_parts": info["csort_parts"],
                         "alg_bytes_per_launch": alg_local,
                         "format_bytes_per_launch": info["format_bytes"],
                         "launch_us_events": round(ev_launch_s * 1e6, 3),
                         "traffic_source": (traffic["file"] + ": " + traffic["source"]
                                            if traffic else None)},
            "cold": ({"launch_us": round(cold_s * 1e6, 3),
                      "gbps_alg": round(alg_local / cold_s * 1e-9, 2),
                      "frac": round(alg_local / cold_s * 1e-9 / HBM_PEAK_GBS, 4),
                      "gflops": round(2.0 * A.nnz / cold_s * 1e-9, 3),
                      "note": "a 512 MiB read before each launch evicts the Infinity Cache"}
                     if cold_s else None),
            "comm": {"overlap": overlap if world > 1 else None,
                     "bcast_x_ms": round(bcast_ms, 3) if world > 1 else None,
                     "gather_y_ms": round(gather_ms, 3) if gather_ms is not None else None,
                     "halo_x_ms": round(halo_ms, 4) if halo_ms is not None else None,
                     "x_bytes": shard.n_global * x.element_size(),
                     "y_bytes": shard.m_global * x.element_size(),
                     "halo_bytes_per_rank": halo_b if world > 1 else None,
                     "end_to_end_gflops": (round(flops_step / (step_s + gather_ms * 1e-3) * 1e-9, 3)
                                           if gather_ms is not None else round(gflops, 3)),
                     "iterative_gflops": (round(flops_step / (step_s + halo_ms * 1e-3) * 1e-9, 3)
                                          if halo_ms is not None else round(gflops, 3))},
            "check": {"pass": bool(ok_all), "checksum_rel": rel},
            "csr3_maps_plans": plans,
            "scaling_reference": sref,
            "strong_scaling": scal,
            "cpu_baseline": cpu,
            "cpu_c1": c1,
        }
        print(json.dumps(out), flush=True)
    op.close()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    if not ok_all:
        sys.exit(3)


if __name__ == "__main__":
    main()
