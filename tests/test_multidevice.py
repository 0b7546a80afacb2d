"""The distinct-device paths of the row-range partition.  The
reference has no multi-device code (cuda-spmv-csrk/cuda/spmv-auto-ampere.cu:
200-203 only prints the device count), so these are the only proof that
the 8-GPU split works.  Each test needs at least two HIP devices and SKIPS
(does not fail) on a one-GPU box; there the same code paths run with
repeated devices and gloo (tests/test_sharded.py, tests/test_bench.py).

* the library's single-process partition: hspmv_create(num_gpus = all
  visible devices) -> one shard per device, ncclCommInitAll over the list,
  ncclBroadcast of x, ncclAllGather of the padded y, unpadded by
  hspmv_get_y; a C4-shaped banded CSR matrix and a CSR-3 matrix whose
  splits fall (unevenly) on super-super-row boundaries;
* plain ``bench.py --gpus 2`` (it starts torch.distributed.run itself) with
  the "nccl" (RCCL) backend, one process per GPU: the driver's N > 1
  command, whose y check must pass.
y is checked against the oracle bit for bit (every row here has <= 40
nonzeros: the ordered sums)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

import hspmv
import oracle
from hspmv import gen

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parents[1]


def need(n):
    have = hspmv.device_count()
    if have < n:
        pytest.skip(f"needs {n} distinct HIP devices, {have} visible")
    return have


def check_bitwise(A, x, y):
    y64 = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
    assert np.diff(A.row_ptr).max() <= 40
    assert np.array_equal(y.view(np.uint64), y64.view(np.uint64))


def test_library_partition_distinct_devices_c4_shaped():
    P = min(need(2), 8)
    A = gen.banded(4_000_000, per_row=10, half=32, seed=11)  # C4's rows, 4e7 nonzeros
    x1, x2 = gen.rand_x(A.n, 7), gen.rand_x(A.n, 8)
    with hspmv.SpMV(A, num_gpus=P) as op:
        info = op.info
        assert info["num_gpus"] == P
        check_bitwise(A, x1, op(x1))
        check_bitwise(A, x2, op(x2))  # x broadcast again from GPU 0
        b, g = op.exchange()
        assert b > 0.0 and g > 0.0
        t = op.run(warmup=2, iters=5)
        assert t["num_gpus"] == P and t["t_min"] > 0
        check_bitwise(A, x2, op.get_y())


def test_library_partition_distinct_devices_csr3_uneven_ssr_splits():
    P = min(need(2), 8)
    A = gen.stencil27(60)
    # coarse, uneven super-super-rows: the shards cannot be equal
    maps = hspmv.build_csr3_maps(A, 200, 7)
    splits = hspmv.partition_rows(A.row_ptr, P, maps)
    firsts = set(int(v) for v in maps.inner[maps.outer[:-1]]) | {A.m}
    assert all(int(s) in firsts for s in splits)
    assert len(set(np.diff(splits).tolist())) > 1
    x = gen.rand_x(A.n, 5)
    with hspmv.SpMV(A, maps, devices=list(range(P))) as op:
        assert op.info["kernel_name"] == "csr3" and op.info["num_gpus"] == P
        check_bitwise(A, x, op(x))
    # fp32 through the same partition: bitwise against the reference's loop
    A32 = A.astype(np.float32)
    x32 = x.astype(np.float32)
    with hspmv.SpMV(A32, maps, devices=list(range(P))) as op:
        y = op(x32)
    y_ref = oracle.spmv(A32.row_ptr, A32.col_idx, A32.val, x32)
    assert np.array_equal(y.view(np.uint32), y_ref.view(np.uint32))


def test_bench_nccl_two_ranks():
    need(2)
    # exactly the driver's command: no launcher, no extra environment
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONUNBUFFERED"] = "1"
    out = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2",
                          "--steps", "20", "--warmup", "3", "--cold-steps", "2"],
                         cwd=REPO, env=env, capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["workload"].startswith("c4")
    assert d["check"]["pass"] is True and d["scaling"] == "strong"
    c = d["comm"]
    assert c["bcast_x_ms"] > 0 and c["gather_y_ms"] > 0 and c["halo_x_ms"] > 0
    assert c["overlap"]["y_equal_to_plain_gather"] is True
    sc = d["strong_scaling"]  # C4 whole on rank 0's GPU, same job
    assert sc["n1"]["config"].startswith("c4") and sc["n1"]["check"]["pass"] is True
    assert abs(sc["efficiency"] - d["value"] / (2 * sc["n1_gflops"])) < 1e-3
    assert sc["cold_efficiency"] > 0
