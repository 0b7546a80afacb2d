"""hipSPARSE as the external comparison point (the
reference's hipsparse-spmv/spmv.cu:151-180 runs hipsparseSpMV with
ALG_DEFAULT in fp32 and fp64): tools/hipsparse_cmp.cpp times libhspmv (the
bench's kernel choice, CSR-3 maps included) beside hipsparseSpMV ALG_DEFAULT /
CSR_ALG1 / CSR_ALG2 on the same device x, warm and cold, and dumps every y.
Both implementations' y are checked against the oracle here; the records go
to $HSPMV_CMP_OUT (a JSON-lines file) when set -- that is how
profiles/r02_hipsparse_cmp.jsonl is produced.  (The small golden matrices
are not run through hipSPARSE: on powerlaw1500 in fp32 hipsparseSpMV
CSR_ALG1 did not return within 90 s on the MI355X box, r02h.)"""
import json
import os
import sys
from pathlib import Path

import numpy as np
import pytest

import oracle
from conftest import GOLDEN, REPO

pytestmark = pytest.mark.gpu

sys.path.insert(0, str(REPO / "heterogeneous-spmv_amd" / "tools"))


def _check(A, x, y, exact):
    y64 = oracle.spmv(A.row_ptr, A.col_idx, A.val.astype(np.float64), x.astype(np.float64))
    absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
    if A.val.dtype == np.float64:
        tol = 1e-6 * np.abs(y64) + 1e-12 * absrow
    else:  # fp32 sums of any order: within the fp32 summation error
        tol = (np.diff(A.row_ptr) + 2) * 2.0 ** -23 * absrow + 1e-30
    err = np.abs(y.astype(np.float64) - y64)
    assert np.all(err <= tol), err.max()
    if exact is not None:
        yr = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
        assert np.array_equal(y[exact], yr[exact])


def _x(n, dtype):
    # hipsparse_cmp.cpp's fill_x: the splitmix64 U(-1, 1) of hspmv.gen.rand_x, seed 42
    from hspmv import gen
    return gen.rand_x(n, 42).astype(dtype)


@pytest.mark.parametrize("cfgs", [["c2", "c3", "c4", "c5"]])
def test_hipsparse_comparison_full_configs(cfgs, tmp_path):
    import hipsparse_cmp as hc
    from sweep import build
    records = []
    for cfg in cfgs:
        A, maps, desc = build(cfg)
        recs = hc.compare(cfg, A, maps, desc, iters=20, cold=10, dump_dir=tmp_path, timeout=150)
        impls = [r["impl"] for r in recs]
        assert impls[0] == "hspmv" and "hipsparse" in impls
        x = _x(A.n, A.val.dtype)
        h = recs[0]
        yh = np.fromfile(tmp_path / f"{cfg}_hspmv.bin", A.val.dtype)
        exact = np.diff(A.row_ptr) <= 40 if h["kernel"] in ("stream", "csr3") else None
        _check(A, x, yh, exact)
        for r in recs[1:]:
            if "t_min_us" not in r:
                continue  # an algorithm this hipSPARSE build refused (recorded)
            ys = np.fromfile(tmp_path / f"{cfg}_{r['alg']}.bin", A.val.dtype)
            _check(A, x, ys, None)
            assert r["hspmv_speedup"] > 0
        records += recs
        for f in tmp_path.glob(f"{cfg}_*.bin"):
            f.unlink()
    out = os.environ.get("HSPMV_CMP_OUT")
    if out:
        Path(out).write_text("".join(json.dumps(d) + "\n" for d in records))
