"""Seeded random shapes through every kernel and plan, against the oracle.

Each case draws a matrix from a mixture the fixed tests cover one at a time:
empty rows, short rows (<= 40 nonzeros, the ordered-sum path), medium rows
(41..4096, cooperative sums), rare split rows (> 4096), uniform / banded /
clustered columns, sorted or unsorted columns with duplicates, exact zeros,
m and n from 1 up, fp32 or fp64.  Every case runs AUTO, STREAM, VECTOR (a
random lane count), CSR3 with freshly built maps under the aligned / packed /
ssr plans, csort (auto, 4 column parts, and reproducible fixed-point sums:
bit-identical on a second launch), AUTO with deterministic = 1, the serial
order (deterministic = 3: AUTO, CSR3 under a random plan, STREAM with split
rows kept whole -- bitwise equal to omp_spmv on EVERY row),
STREAM with split rows kept whole, AUTO over 2 x slabs, and AUTO over three
row-range shards, each twice (two x vectors through one handle: no state may
leak from one launch into the next).

Bars (spmv-csr/spmv.c:92-114 restated by the oracle):
* fp64: |y - y64| <= 1e-6 |y64| + 1e-12 sum|a x| (north star);
* fp32: within omp_spmv's own accumulation error of the fp64 sum;
* STREAM / CSR3 (ordered row sums): bitwise equal to omp_spmv on rows of up
  to 40 nonzeros, in both dtypes.
Parity for these shapes rests on the oracle alone (the reference ships no
such matrices); the seeds are fixed so a failure names its case.
"""
import numpy as np
import pytest

import hspmv
import oracle
from conftest import fp64_tol_ok
from hspmv import gen

pytestmark = pytest.mark.gpu

SERIAL_MAX = 40
N_CASES = 64
SEEN = set()  # kernels the cases ran (test_fuzz_ran_every_kernel)


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    assert hspmv.device_count() >= 1, "no HIP device visible: the gpu tests must run on the MI355X box"


def random_matrix(seed: int):
    """A seeded matrix from the mixture above (<= ~1.5 M nonzeros)."""
    rng = np.random.default_rng(seed)
    m = int(rng.choice([1, 7, 63, 64, 65, 1000, 4097, 20_000, 60_000]))
    n = int(rng.choice([1, 5, 64, 1000, 50_000, 300_000, 300_000, 2_000_000]))
    p = rng.dirichlet([2.0, 6.0, 1.0])  # empty / short / medium
    kind = rng.choice(3, m, p=p)
    lens = np.where(kind == 0, 0, np.where(kind == 1, rng.integers(1, SERIAL_MAX + 1, m),
                                           rng.integers(SERIAL_MAX + 1, 600, m)))
    if rng.random() < 0.3:  # a few split rows
        k = int(rng.integers(1, 4))
        lens[rng.integers(0, m, k)] = rng.integers(4097, 12_000, k)
    cap = 1_500_000
    if lens.sum() > cap:
        lens = (lens * (cap / lens.sum())).astype(np.int64)
    rows = np.repeat(np.arange(m), lens)
    nnz = rows.size
    pattern = rng.choice(["uniform", "banded", "clustered"])
    if pattern == "uniform":
        cols = rng.integers(0, n, nnz)
    elif pattern == "banded":
        centre = (rows.astype(np.float64) * n / max(m, 1)).astype(np.int64)
        cols = np.clip(centre + rng.integers(-300, 301, nnz), 0, n - 1)
    else:  # runs of consecutive columns from a few random starts per row
        start = rng.integers(0, n, m)[rows]
        off = np.arange(nnz) - np.repeat(np.concatenate([[0], np.cumsum(lens)[:-1]]), lens)
        cols = (start + off) % n
    unsorted = rng.random() < 0.25
    if not unsorted:  # sorted within each row (duplicates may remain)
        order = np.lexsort((cols, rows))
        cols = cols[order]
    vals = rng.uniform(-1, 1, nnz)
    vals[rng.random(nnz) < 0.02] = 0.0
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    dtype = np.float64 if rng.random() < 0.5 else np.float32
    A = hspmv.CsrMatrix(m, n, rp, cols.astype(np.int32), vals.astype(dtype))
    return A, {"m": m, "n": n, "nnz": int(nnz), "pattern": str(pattern), "unsorted": bool(unsorted),
               "dtype": np.dtype(dtype).name}


def runs(A, rng):
    """(label, SpMV kwargs) for every kernel / plan of a case."""
    yield "auto", {}
    yield "stream", {"kernel": "stream"}
    yield "vector", {"kernel": "vector", "lanes": int(rng.choice([1, 2, 4, 8, 16, 32, 64]))}
    if A.m >= 1:
        maps = hspmv.build_csr3_maps(A, int(rng.integers(2, 40)), int(rng.integers(2, 12)))
        yield "csr3-aligned", {"maps": maps, "kernel": "csr3"}
        yield "csr3-packed", {"maps": maps, "kernel": "csr3", "options": {"csr3_plan": "packed"}}
        yield "csr3-ssr", {"maps": maps, "kernel": "csr3", "options": {"csr3_plan": "ssr"}}
        yield "csr3-serial", {"maps": maps, "kernel": "csr3",
                              "options": {"csr3_plan": str(rng.choice(["aligned", "packed", "ssr"])),
                                          "deterministic": "serial"}}
    yield "csort", {"kernel": "csort"}
    yield "csort-4parts", {"kernel": "csort", "options": {"csort_parts": 4}}
    yield "csort-repro", {"kernel": "csort", "options": {"deterministic": "reproducible"}}
    yield "auto-det", {"options": {"deterministic": 1}}
    yield "stream-whole-rows", {"kernel": "stream", "split_rows": False}
    yield "auto-serial", {"options": {"deterministic": "serial"}}
    yield "stream-serial-whole-rows", {"kernel": "stream", "split_rows": False,
                                       "options": {"deterministic": "serial"}}
    yield "auto-2slabs", {"options": {"x_slabs": 2}}
    yield "sharded-3", {"devices": [0, 0, 0]}  # row-range shards (one device, repeated)


def fixed_point_term(A, x):
    """Reproducible csort: each product rounded once to 2^-50 of its row's
    largest |value| times max|x| (tests/test_csort.py fixed_bound)."""
    lens = np.diff(A.row_ptr)
    vmax = np.zeros(A.m)
    nz = lens > 0
    if A.nnz:
        vmax[nz] = np.maximum.reduceat(np.abs(A.val.astype(np.float64)), A.row_ptr[:-1][nz])
    xmax = float(np.abs(x.astype(np.float64)).max()) if x.size else 0.0
    return lens * 2.0 ** -48 * vmax * xmax


def check(A, x, y, ordered, what, fixed=False, serial=False):
    y64 = oracle.spmv(A.row_ptr, A.col_idx, A.val.astype(np.float64), x.astype(np.float64))
    absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
    lens = np.diff(A.row_ptr)
    fx = fixed_point_term(A, x) if fixed else 0.0
    err = np.abs(y.astype(np.float64) - y64)
    if A.val.dtype == np.float64:
        tol = 1e-6 * np.abs(y64) + 1e-12 * absrow + fx
        assert np.all(err <= tol), (what, float(err.max()))
    else:
        assert np.all(err <= (lens + 2) * 2.0 ** -23 * absrow + fx + 1e-30), (what, float(err.max()))
    if ordered:  # omp_spmv's bits on the short rows (serial order: on every row)
        yo = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
        short = lens <= (np.iinfo(np.int64).max if serial else SERIAL_MAX)
        u = np.uint64 if y.dtype == np.float64 else np.uint32
        bad = np.flatnonzero(y[short].view(u) != yo[short].view(u))
        assert bad.size == 0, (what, int(np.flatnonzero(short)[bad[0]]))


@pytest.mark.parametrize("seed", range(N_CASES))
def test_fuzz_every_kernel_matches_oracle(seed):
    A, desc = random_matrix(1000 + seed)
    rng = np.random.default_rng(seed)
    xs = [gen.rand_x(A.n, 7 + seed).astype(A.val.dtype),
          rng.uniform(-4, 4, A.n).astype(A.val.dtype)]
    ran = []
    for label, kw in runs(A, rng):
        kw = dict(kw)
        maps = kw.pop("maps", None)
        op = hspmv.SpMV(A, maps, **kw)  # a forced kernel that cannot be built falls back
        with op:
            name = op.info["kernel_name"]
            fixed = op.info["csort_fixed_point"] == 1
            serial = op.info["serial_order"] == 1
            assert serial == ("serial" in label), (desc, label)
            for i, x in enumerate(xs):
                y = op(x)
                check(A, x, y, name in ("stream", "csr3"), (desc, label, name, i), fixed, serial)
                if fixed:  # reproducible: the same bits again
                    assert np.array_equal(op(x).view(np.uint8), y.view(np.uint8)), (desc, label, i)
        if label == "csort-repro" and name == "csort":
            name = "csort-fixed" if fixed else name
        if serial:
            name = name + "-serial"
        ran.append((label, name))
        SEEN.add(name)
    assert len(ran) >= 10, (desc, ran)


def test_fuzz_ran_every_kernel():
    """The forced kernels really ran somewhere in the cases above."""
    if len(SEEN) == 0:
        pytest.skip("run with the fuzz cases")
    assert {"stream", "vector", "csr3", "csort", "csort-fixed", "stream-serial", "csr3-serial"} <= SEEN, SEEN
