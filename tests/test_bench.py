"""bench.py contract: the CPU-side dry run names the configuration each world
size measures (C3 at N = 1, C4 strong scaling at N > 1) and its partition;
on one GPU, one JSON line with the driver's keys, the roofline and
cpu_baseline objects, and a passing y check (short run)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]


def _dry(*args):
    out = subprocess.run([sys.executable, str(REPO / "bench.py"), "--dry-run", *args], cwd=REPO,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    return json.loads(lines[0])


def test_dry_run_n1_is_c3():
    d = _dry()
    assert d["n_gpus"] == 1 and d["config"] == "c3"


@pytest.mark.parametrize("n", [2, 8])
def test_dry_run_multi_gpu_is_c4_strong_nnz_balanced(n):
    d = _dry("--gpus", str(n))
    assert d["config"] == "c4"
    p = d["plan"]
    assert p["scaling"] == "strong" and p["world"] == n and p["m"] == 20_000_000
    assert len(p["splits"]) == n + 1 and p["splits"][0] == 0 and p["splits"][-1] == p["m"]
    assert sum(p["nnz_per_rank"]) == p["nnz"] and 199_999_000 < p["nnz"] <= 200_000_000
    assert max(p["nnz_per_rank"]) - min(p["nnz_per_rank"]) <= 20


def test_bench_rejects_bad_arguments():
    out = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "0", "--dry-run"],
                         cwd=REPO, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "--gpus" in out.stderr


def test_c3_shards_cover_the_matrix_on_ssr_boundaries():
    """A CSR-3 configuration split over ranks keeps whole super-super-rows
    per rank and every row exactly once (what bench.py --config c3 --gpus N
    gives each rank); checked on a small CSR-3 matrix with the same code."""
    from hspmv import dist as hdist
    from hspmv import gen
    import hspmv
    A = gen.laplace2d(40, 30)
    maps = hspmv.build_csr3_maps(A, 7, 8)
    for world in (1, 2, 3, 5):
        splits = hspmv.partition_rows(A.row_ptr, world, maps)
        rows = 0
        for r in range(world):
            A_loc, m_loc = hdist.slice_csr3(A, maps, splits, r)
            assert m_loc.inner[0] == 0 and m_loc.inner[-1] == A_loc.m
            assert m_loc.outer[0] == 0 and m_loc.outer[-1] == m_loc.n_sr
            assert np.array_equal(A_loc.col_idx,
                                  A.col_idx[A.row_ptr[splits[r]]:A.row_ptr[splits[r + 1]]])
            rows += A_loc.m
        assert rows == A.m


_SPAWN_PROBE = r"""
import json, subprocess, sys
sys.argv = ["bench.py", "--gpus", "4", "--steps", "7"]
seen = {}
class FakeProc:
    def __init__(self, cmd, **kw):
        seen["cmd"] = cmd
        seen["env_ipc"] = kw["env"].get("HSA_ENABLE_IPC_MODE_LEGACY")
        seen["torch_loaded"] = sorted(m for m in sys.modules if m == "torch" or m.startswith("torch."))
        seen["hspmv_loaded"] = sorted(m for m in sys.modules if m.startswith("hspmv"))
        self.stdout = iter(['{"value": 1.0}\n'])
    def wait(self):
        return 5
subprocess.Popen = FakeProc
import bench
try:
    bench.main()
except SystemExit as e:
    seen["exit"] = e.code
print("PROBE " + json.dumps(seen))
"""


def test_self_launch_spawns_the_launcher_without_touching_the_gpu():
    """`python bench.py --gpus N` with no WORLD_SIZE: the parent starts
    torch.distributed.run over itself as a child (same arguments, 127.0.0.1
    rendezvous, the RCCL IPC environment), relays its stdout and exits with
    its code -- and has imported neither torch (so no torch.cuda) nor the
    HIP library when it spawns."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "HSA_ENABLE_IPC_MODE_LEGACY")}
    out = subprocess.run([sys.executable, "-c", _SPAWN_PROBE], cwd=REPO, env=env,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    assert '{"value": 1.0}' in out.stdout  # relayed
    seen = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("PROBE ")][0][6:])
    assert seen["torch_loaded"] == [] and seen["hspmv_loaded"] == []
    assert seen["exit"] == 5 and seen["env_ipc"] == "0"
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "7"] and cmd[-5].endswith("bench.py")


def test_cpu_c1_leg_times_configs0():
    """The cpu_c1 leg: configs[0]'s matrix (nnz = 4,996,000), fp64, x = 1 and
    x = rand:42, static and guided, TimeMin/Max/Avg and GFLOP/s from TimeMin."""
    sys.path.insert(0, str(REPO))
    import bench
    c = bench.cpu_c1(0.2)
    assert c["m"] == 1_000_000 and c["nnz"] == 4_996_000 and "nnz=4996000" in c["sample"]
    assert c["dtype"] == "f64" and c["kind"] == "port" and c["cores"] >= 1
    for xname in ("ones", "rand:42"):
        for sched in ("static", "guided"):
            leg = c["x"][xname][sched]
            assert 0 < leg["TimeMin"] <= leg["TimeAvg"] <= leg["TimeMax"]
            assert abs(leg["gflops"] - 2 * c["nnz"] / leg["TimeMin"] * 1e-9) < 1e-2
    assert c["value"] == c["x"]["rand:42"]["static"]["gflops"]


def test_cpu_baseline_runs_in_its_own_process(tmp_path):
    """bench.py's CPU legs (oracle/cpu_bench.py) on a small matrix: a process
    of its own, the reference protocol's min / median / avg, the reported
    team one thread under the cgroup quota (or the physical cores), the
    cgroup's throttling counters, and the reference's own omp_spmv beside
    it when oracle/_ref was built."""
    sys.path.insert(0, str(REPO))
    import bench
    from hspmv import gen
    A = gen.laplace2d(300, 300)
    x = gen.rand_x(A.n, 42)
    c = bench.cpu_baseline(A, x, 0.5)
    assert c["kind"] == "port" and c["unit"] == "GFLOP/s" and c["value"] > 0
    assert abs(c["value"] - 2 * A.nnz / c["time_min_s"] * 1e-9) < 1e-2 * c["value"]
    assert c["time_min_s"] <= c["median_s"] <= c["time_max_s"]
    assert c["threads_tried"][str(c["cores"])]["note"] == "reported leg"
    q = c["cgroup_cpu_quota"]
    assert c["cores"] == (max(1, min(c["host"]["physical_cores"] or c["host"]["affinity_cpus"],
                                     c["host"]["affinity_cpus"], int(q) - 1)) if q else c["cores"])
    assert "a process of its own" in c["cores_note"] and f"nnz={A.nnz}" in c["sample"]
    assert 0.0 <= c["runs_within_10pct_of_min"] <= 1.0
    if (REPO / "oracle" / "_ref" / "libref_spmvcsr.so").exists():
        r = c["reference_f32"]
        assert r["kind"] == "reference" and r["value"] > 0 and r["cores"] == c["cores"]


@pytest.mark.gpu
def test_bench_json_line_contract():
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    out = subprocess.run([sys.executable, str(REPO / "bench.py"), "--steps", "20", "--warmup", "3",
                          "--cold-steps", "2", "--cpu-seconds", "0.5"],
                         cwd=REPO, env=env, capture_output=True, text=True, timeout=400)
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
    assert d["dtype"] == "f64" and d["config"]["workload"].startswith("c3")
    assert d["config"]["kernel"] == "csr3" and d["config"]["nnz"] == 51_895_117
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert 0 < r["frac"] < 1 and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert r["kernel"].startswith("hspmv_csr3<double")
    assert r["launches_per_spmv"] == 1 and r["csort_parts"] == 0
    assert d["config"]["csr3_plan"] == "aligned" and d["config"]["deterministic"] is True
    plans = d["csr3_maps_plans"]  # the maps-driven plans, same process, same y bits
    for p, code in (("packed", 2), ("ssr", 3)):
        assert plans[p]["csr3_plan"] == code and plans[p]["launch_us_events"] > 0
        assert plans[p]["y_bitwise_equal_to_headline"] is True
    c = d["cpu_baseline"]
    assert c["kind"] == "port" and c["cores"] >= 1 and c["value"] > 0
    # the reported leg leaves one CPU of the cgroup quota to the runtime
    if c["cgroup_cpu_quota"]:
        assert c["cores"] <= c["cgroup_cpu_quota"] - 1 or c["cores"] == 1
    assert c["time_min_s"] <= c["median_s"] <= c["time_max_s"]
    assert c["threads_tried"][str(c["cores"])]["note"] == "reported leg"
    assert d["strong_scaling"] is None  # N = 1: scaling_reference instead
    assert abs(c["value"] - 2 * d["config"]["nnz"] / c["time_min_s"] * 1e-9) < 1e-2 * c["value"]
    assert "nnz=51895117" in c["sample"]
    c1 = d["cpu_c1"]  # configs[0] itself on this host
    assert c1["nnz"] == 4_996_000 and "nnz=4996000" in c1["sample"] and c1["dtype"] == "f64"
    for xname in ("ones", "rand:42"):
        for sched in ("static", "guided"):
            leg = c1["x"][xname][sched]
            assert 0 < leg["TimeMin"] <= leg["TimeAvg"] <= leg["TimeMax"] and leg["gflops"] > 0
    ref = c["reference_f32"]  # the reference's own omp_spmv, when oracle/_ref was built
    if (REPO / "oracle" / "_ref" / "libref_spmvcsr.so").exists():
        assert ref["kind"] == "reference" and ref["value"] > 0 and ref["time_min_s"] > 0
    assert d["cold"]["launch_us"] > 0
    assert d["check"]["pass"] is True
    sr = d["scaling_reference"]  # C4 on this one GPU: the N = 1 point of the N > 1 curve
    assert sr["config"].startswith("c4") and sr["nnz"] > 199_999_000 and sr["value"] > 0
    assert sr["check"]["pass"] is True and sr["cold_gflops"] > 0


@pytest.mark.gpu
def test_bench_multi_rank_path_rehearsal_on_one_gpu(tmp_path):
    """bench.py's N > 1 code path (self-launched ranks, shards, x broadcast,
    barriers, max over ranks, y all-gather, halo exchange, rank-0 JSON line)
    run as 2 ranks that
    share device 0 and exchange over gloo -- RCCL allows one rank per device,
    so this is the rehearsal a one-GPU box can do; the driver's N > 1 runs use
    RCCL on one GPU per rank.  C2 (weak scaling) keeps it short."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONUNBUFFERED"] = "1"
    # the plain command: bench.py starts its own launcher (self_launch)
    out = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2",
                          "--backend", "gloo", "--same-device", "--config", "c2",
                          "--steps", "10", "--warmup", "2", "--cold-steps", "2"],
                         cwd=REPO, env=env, capture_output=True, text=True, timeout=400)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["check"]["pass"] is True
    assert d["config"]["m"] == 2_000_000 and d["config"]["parallelism"] == "row-range x2"
    c = d["comm"]
    assert c["bcast_x_ms"] > 0 and c["gather_y_ms"] > 0 and c["halo_x_ms"] > 0
    assert c["halo_bytes_per_rank"] == 1000 * 8   # one grid line from the neighbour
    ov = c["overlap"]  # chunked SpMV with the y all-gather overlapped
    assert ov["chunks"] == 4 and ov["ms"] > 0 and ov["y_equal_to_plain_gather"] is True
    assert d["cpu_baseline"] is None              # rank 0 at N = 1 only
    assert d["scaling_reference"] is None
    sc = d["strong_scaling"]  # the same workload on rank 0's GPU alone, same job
    assert sc["n1"]["config"].startswith("c2") and sc["n1"]["n_gpus"] == 1
    assert sc["n1"]["check"]["pass"] is True and sc["n1_gflops"] > 0
    assert abs(sc["efficiency"] - d["value"] / (2 * sc["n1_gflops"])) < 1e-3
    assert sc["cold_gflops"] > 0 and sc["n1_cold_gflops"] > 0
    assert abs(sc["cold_efficiency"] - sc["cold_gflops"] / (2 * sc["n1_cold_gflops"])) < 1e-3


@pytest.mark.gpu
def test_bench_eight_rank_orchestration_rehearsal_on_one_gpu(tmp_path):
    """The driver's 8-GPU run is the one whose failure would be total, so its
    orchestration is rehearsed whole: plain ``bench.py --gpus 8`` (it
    self-launches 8 ranks) on device 0 over gloo, C2 weak scaling (8 M rows).
    One JSON line, the y check, the halo of an interior rank (a grid line
    from each neighbour), the overlapped gather equal to the plain one, and
    the strong_scaling block."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONUNBUFFERED"] = "1"
    out = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "8",
                          "--backend", "gloo", "--same-device", "--config", "c2",
                          "--steps", "10", "--warmup", "2", "--cold-steps", "2"],
                         cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["scaling"] == "weak" and d["check"]["pass"] is True
    assert d["config"]["m"] == 8_000_000 and d["config"]["parallelism"] == "row-range x8"
    c = d["comm"]
    assert c["bcast_x_ms"] > 0 and c["gather_y_ms"] > 0 and c["halo_x_ms"] > 0
    # the max over ranks: an interior rank receives one grid line (1000
    # fp64) from each of its two neighbours
    assert c["halo_bytes_per_rank"] == 2 * 1000 * 8
    ov = c["overlap"]
    assert ov["chunks"] == 4 and ov["ms"] > 0 and ov["y_equal_to_plain_gather"] is True
    assert d["cpu_baseline"] is None and d["scaling_reference"] is None
    sc = d["strong_scaling"]  # C2 scales weakly: its N = 1 point is one GPU's share
    assert sc["n1"]["check"]["pass"] is True and sc["n1"]["m"] == 1_000_000
    assert abs(sc["efficiency"] - d["value"] / (8 * sc["n1_gflops"])) < 1e-3
    assert sc["cold_gflops"] > 0 and sc["n1_cold_gflops"] > 0
