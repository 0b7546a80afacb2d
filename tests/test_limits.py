"""Index-width limits: the STREAM / CSR3 kernels address x and
the matrix streams as a base pointer plus a 32-bit byte offset, so an x of
4 GiB or more (fp64: n >= 2^29 columns) must go to a kernel that indexes
through pointers (csort when built, else VECTOR) instead of wrapping."""
import numpy as np
import pytest

import hspmv
import oracle
from conftest import fp64_tol_ok

pytestmark = pytest.mark.gpu


def test_x_over_4gib_takes_a_pointer_indexed_kernel():
    if hspmv.device_count() < 1:
        pytest.fail("no HIP device visible")
    n = (1 << 29) + 4096            # fp64 x = 4 GiB + 32 KiB
    m = 3000
    rng = np.random.default_rng(1)
    lens = rng.integers(1, 12, m)
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    # rows in 64-row groups gather from a narrow window, either at the start
    # of x or past 2^29 (where a 32-bit byte offset of an fp64 entry wraps)
    ci = []
    for r, ln in enumerate(lens):
        base = 0 if (r // 64) % 2 == 0 else n - 4000
        ci.append(np.sort(rng.choice(4000, ln, replace=False)) + base)
    ci = np.concatenate(ci).astype(np.int32)
    A = hspmv.CsrMatrix(m, n, rp, ci, rng.uniform(-1, 1, rp[-1]))
    x = np.zeros(n)
    x[:4000] = rng.uniform(-1, 1, 4000)
    x[n - 4000:] = rng.uniform(-1, 1, 4000)
    y_ref = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
    absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
    for kernel, want in (("auto", ("vector", "csort")), ("stream", ("vector",)),
                         ("csort", ("csort",))):
        with hspmv.SpMV(A, kernel=kernel) as op:
            y = op(x)
            assert op.info["kernel_name"] in want, (kernel, op.info["kernel_name"])
        assert fp64_tol_ok(y, y_ref, absrow), kernel
