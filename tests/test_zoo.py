"""GPU parity on shapes outside the BASELINE configurations, every kernel.

The matrices of tools/auto_regret.py's zoo at test size: uniform random
columns, dense diagonal blocks, an arrowhead (rows long enough to be split),
a wide matrix (n >> m), a tall one over a tiny x (n << m), a diagonal, and
half-empty rows.  AUTO and each forced kernel against the oracle
(spmv-csr/spmv.c:92-114 restated) at the north-star fp64 bar; the row
kernels (STREAM, CSR3) bitwise on rows of <= 40 nonzeros, which they sum in
omp_spmv's order.  Parity for these shapes rests on the oracle alone (the
reference ships no such matrices).
"""
import numpy as np
import pytest

import hspmv
import oracle
from conftest import fp64_tol_ok
from hspmv import gen

pytestmark = pytest.mark.gpu

SERIAL_MAX = 40


def _random_rows(m, n, k, seed):
    rng = np.random.default_rng(seed)
    ci = np.sort(rng.integers(0, n, (m, k), dtype=np.int32), axis=1).reshape(-1)
    rp = np.arange(0, m * k + 1, k, dtype=np.int64).astype(np.int32)
    return hspmv.CsrMatrix(m, n, rp, ci, rng.uniform(-1, 1, m * k))


def _from_coo(m, n, r, c, v):
    import scipy.sparse as sp
    S = sp.csr_matrix((v, (r, c)), shape=(m, n))
    S.sum_duplicates()
    return hspmv.CsrMatrix.from_scipy(S, np.float64)


def zoo(name):
    rng = np.random.default_rng(17)
    if name == "urand":
        return _random_rows(200_000, 200_000, 8, 1)
    if name == "blocks32":
        m, b = 100_000, 32
        ci = ((np.arange(m) // b) * b)[:, None] + np.arange(b)[None, :]
        rp = np.arange(0, m * b + 1, b).astype(np.int32)
        return hspmv.CsrMatrix(m, m, rp, ci.reshape(-1).astype(np.int32), rng.uniform(-1, 1, m * b))
    if name == "arrow":  # banded + 4 rows of 60 K random columns (split rows)
        B = gen.banded(200_000, per_row=8, half=16, seed=4)
        r = np.repeat(np.arange(B.m), np.diff(B.row_ptr))
        heads = rng.choice(B.m, 4, replace=False)
        hr = np.repeat(heads, 60_000)
        return _from_coo(B.m, B.m, np.concatenate([r, hr]),
                         np.concatenate([B.col_idx, rng.integers(0, B.m, hr.size)]),
                         np.concatenate([B.val, rng.uniform(-1, 1, hr.size)]))
    if name == "wide":
        return _random_rows(20_000, 2_000_000, 64, 5)
    if name == "tall":
        return _random_rows(1_000_000, 512, 3, 6)
    if name == "diag":
        m = 2_000_000
        return hspmv.CsrMatrix(m, m, np.arange(m + 1, dtype=np.int32), np.arange(m, dtype=np.int32),
                               rng.uniform(-1, 1, m))
    if name == "half_empty":  # every other row empty at random, the rest 1..100 nonzeros
        m = 300_000
        lens = np.where(rng.random(m) < 0.5, 0, rng.integers(1, 101, m))
        r = np.repeat(np.arange(m), lens)
        return _from_coo(m, m, r, rng.integers(0, m, r.size), rng.uniform(-1, 1, r.size))
    raise ValueError(name)


ZOO = ["urand", "blocks32", "arrow", "wide", "tall", "diag", "half_empty"]
FORCED = [("auto", 0), ("stream", 0), ("vector", 4), ("vector", 64), ("csr3", 0), ("csort", 0)]


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    assert hspmv.device_count() >= 1, "no HIP device visible: the gpu tests must run on the MI355X box"


@pytest.mark.parametrize("name", ZOO)
def test_zoo_every_kernel_matches_oracle(name):
    A = zoo(name)
    x = gen.rand_x(A.n, 3)
    y64 = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
    absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
    short = np.diff(A.row_ptr) <= SERIAL_MAX
    seen = set()
    for kernel, lanes in FORCED:
        with hspmv.SpMV(A, kernel=kernel, lanes=lanes) as op:
            y = op(x)
            info = op.info
        seen.add(info["kernel_name"])
        assert fp64_tol_ok(y, y64, absrow), (name, kernel, lanes, np.abs(y - y64).max())
        if info["kernel_name"] in ("stream", "csr3"):  # ordered sums: omp_spmv's bits
            assert np.array_equal(y[short], y64[short]), (name, kernel, info["kernel_name"])
    # the forced kernels really ran (csort is refused only when its slots
    # cannot fit, which none of these shapes reaches)
    assert {"stream", "vector", "csort"} <= seen, seen
