"""Generates the committed golden fixtures under tests/golden/.

Run in the build container (needs /root/reference for the reference build):
    python tests/golden/make_golden.py

For every input matrix (.csr text in the reference layout, written like
helpers/converter.m:25-33) it records
  * y_ref_f32_ones  -- the REFERENCE's own spmv-csr/spmv.c (my_read_csr +
                       omp_spmv, compiled unmodified into oracle/_ref/) with
                       x = 1, exactly what spmv.exe computes (spmv.c:128-181);
  * y_ref_f32_rand  -- same binary, x = float32(rand_x(n, 42));
  * y_orc_f64_rand  -- the fp64 restatement (oracle/spmv_oracle.c), x = rand_x(n, 42).
and asserts that the fp32 restatement is bitwise equal to the reference
outputs before writing anything.  The .csr3 fixtures are built with the
oracle's restated handCoarsen grouping (the reference reformatter needs Boost,
absent here: unbuildable) and written in the writer layout of
reformat-csr-to-csr3/spmv-auto.cpp:38-62.
"""
from __future__ import annotations

import hashlib
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO / "oracle"))
sys.path.insert(0, str(REPO / "heterogeneous-spmv_amd"))

import oracle  # noqa: E402
from hspmv import gen  # noqa: E402  (synthetic generators; pure numpy/scipy)
from hspmv.api import CsrMatrix  # noqa: E402


def write_csr3_text(path: Path, A: CsrMatrix, outer, inner) -> None:
    with open(path, "w") as f:
        f.write(f"{len(outer) - 1} {len(inner) - 1} {A.m} {A.n} {A.nnz} \n")
        for arr in (outer, inner, A.row_ptr, A.col_idx):
            f.write("".join(f"{int(v)} " for v in arr))
        f.write("".join("%.6f " % v for v in A.val.tolist()))


def rcm(A: CsrMatrix) -> CsrMatrix:
    from scipy.sparse.csgraph import reverse_cuthill_mckee
    S = A.to_scipy()
    p = reverse_cuthill_mckee(S, symmetric_mode=True)
    return CsrMatrix.from_scipy(S[p][:, p], np.float64)


def matrices():
    rng = np.random.default_rng(2024)
    out = {}
    out["lap32.mtx.rcm"] = rcm(gen.laplace2d(32, 32))
    out["powerlaw1500"] = gen.powerlaw(1500, seed=1234, dtype=np.float64)
    out["banded3000"] = gen.banded(3000, per_row=10, half=32, seed=11)
    # edge cases the reference's readers/kernels meet: empty rows (first,
    # last, runs of them), one row, one very long row (> 1024 nnz), rows of
    # every length 0..70 (crosses the 32-lane serial threshold and the 64-row
    # wave tasks).
    import scipy.sparse as sp
    S = sp.random(300, 300, density=0.02, random_state=7, format="csr")
    S = S.tolil()
    for r in (0, 1, 2, 150, 299):
        S.rows[r] = []
        S.data[r] = []
    S = S.tocsr()
    S.data = rng.uniform(-1, 1, S.nnz)
    out["empty_rows"] = CsrMatrix.from_scipy(S)
    one = sp.csr_matrix(rng.uniform(-1, 1, (1, 257)))
    out["single_row"] = CsrMatrix.from_scipy(one)
    n = 2000
    rows = [np.zeros(0, np.int64)] * 0
    indptr = [0]
    cols = []
    for r in range(200):
        ln = 1500 if r == 77 else (r % 71)
        c = np.sort(rng.choice(n, ln, replace=False))
        cols.append(c)
        indptr.append(indptr[-1] + ln)
    ci = np.concatenate(cols)
    out["long_row"] = CsrMatrix(200, n, np.array(indptr), ci, rng.uniform(-1, 1, ci.shape[0]))
    return out


def main():
    oracle.build(ref=True)
    manifest = {"generator": "tests/golden/make_golden.py", "x_seed": 42, "fixtures": {}}
    for name, A in matrices().items():
        path = HERE / f"{name}.csr"
        gen.write_csr_text(str(path), A)
        # what the reference actually computes from the text file
        m, n, rp, ci, v32, v64, base = oracle.read_csr(path)
        assert base == 0 and m == A.m and n == A.n
        x64 = gen.rand_x(n, 42)
        x32 = x64.astype(np.float32)
        y_ref_ones = oracle.ref_spmv_file(path) if m == n else None
        y_ref_rand = oracle.ref_spmv_file(path, x32)
        y_orc32 = oracle.spmv(rp, ci, v32, x32)
        assert np.array_equal(y_orc32.view(np.uint32), y_ref_rand.view(np.uint32)), name
        if y_ref_ones is not None:
            y1 = oracle.spmv(rp, ci, v32, np.ones(n, np.float32))
            assert np.array_equal(y1.view(np.uint32), y_ref_ones.view(np.uint32)), name
        y64 = oracle.spmv(rp, ci, v64, x64)
        arrays = {"y_ref_f32_rand": y_ref_rand, "y_orc_f64_rand": y64}
        if y_ref_ones is not None:
            arrays["y_ref_f32_ones"] = y_ref_ones
        np.savez_compressed(HERE / f"{name}.npz", **arrays)
        entry = {"m": m, "n": n, "nnz": int(rp[-1]),
                 "sha256": hashlib.sha256(path.read_bytes()).hexdigest(),
                 "arrays": sorted(arrays)}
        # CSR-3 fixture with the restated handCoarsen maps (Volta/.csr3-writer
        # parameters, reformat-csr-to-csr3/spmv-auto.cpp:154-173).
        if m == n and m > 1:
            d = rp[-1] / m
            ssrs = int(np.floor(8.89888 - 1.25 * np.log(d) + 0.5))
            srs = int(np.floor(10.14618 - 1.5 * np.log(d) + 0.5))
            if 8.0 < d <= 16.0:
                ssrs = int(np.floor(ssrs * 1.5 + 0.5)); srs = ssrs * 2
            elif 16.0 < d <= 32.0:
                ssrs *= 4; srs = ssrs >> 1
            elif d > 32.0:
                ssrs *= 5; srs = ssrs >> 1
            ssrs, srs = max(ssrs, 1), max(srs, 1)
            outer, inner = oracle.build_maps(rp, ci, ssrs, srs)
            p3 = HERE / f"{name}.csr3"
            A3 = CsrMatrix(m, n, rp, ci, v64)
            write_csr3_text(p3, A3, outer, inner)
            o2, i2, m2, n2, rp2, ci2, v32b, v64b = oracle.read_csr3(p3)
            y3 = oracle.csr3_spmv(o2, i2, rp2, ci2, v64b, x64)
            assert np.array_equal(y3, y64), name
            entry["csr3"] = {"ssrs": ssrs, "srs": srs, "n_ssr": int(len(outer) - 1),
                             "n_sr": int(len(inner) - 1),
                             "sha256": hashlib.sha256(p3.read_bytes()).hexdigest()}
            np.savez_compressed(HERE / f"{name}.maps.npz", outer=outer, inner=inner)
        manifest["fixtures"][name] = entry
        print(f"{name}: m={m} n={n} nnz={rp[-1]} ok")
    # 1-based variant of lap32 (readers of spmv-csrk/spmv.cpp:60,67 subtract 1)
    A = rcm(gen.laplace2d(32, 32))
    gen.write_csr_text(str(HERE / "lap32.onebased.csr"), A, index_base=1)
    manifest["fixtures"]["lap32.onebased"] = {"same_as": "lap32.mtx.rcm", "index_base": 1}
    (HERE / "manifest.json").write_text(json.dumps(manifest, indent=1, sort_keys=True) + "\n")


if __name__ == "__main__":
    main()
