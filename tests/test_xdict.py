"""Block x dictionaries (host planner, hspmv_xdict_plan; CPU only).

The STREAM / CSR3 kernels can stage, per workgroup, the x entries its rows
reference (runs of consecutive columns) in LDS and gather through 16-bit
positions (spmv_device.cuh stage_xdict).  These tests check the format the
host builds: every in-kernel nonzero's position addresses exactly x[col],
runs are sorted, disjoint and at most 63 per workgroup, the per-block
entries respect the cap, and split rows are left out.  The GPU side is
checked bit for bit in tests/test_gpu_parity.py::test_xdict_bitwise_and_fallback.
"""
import numpy as np
import pytest

import hspmv
from hspmv import gen


def _random_rows(m, n, per_row, seed):
    rng = np.random.default_rng(seed)
    cols = np.sort(rng.choice(n, size=(m, per_row), replace=True), axis=1)
    rp = np.arange(0, m * per_row + 1, per_row, dtype=np.int32)
    return hspmv.CsrMatrix(m, n, rp, cols.reshape(-1).astype(np.int32),
                           rng.uniform(-1, 1, m * per_row))


def _long_rows():
    rng = np.random.default_rng(2)
    lens = rng.integers(0, 30, 600)
    lens[[0, 255, 256, 599]] = [5000, 4097, 9000, 4096]
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    ci = np.concatenate([np.sort(rng.choice(20000, ln, replace=False)) for ln in lens]).astype(np.int32)
    return hspmv.CsrMatrix(600, 20000, rp, ci, rng.uniform(-1, 1, rp[-1]))


def block_rows(A, maps, kernel, fill=True):
    """Workgroup row ranges the planner uses (STREAM: 256 rows; CSR3: four
    tasks, 64-row aligned groups by default, or with the packed plan whole
    super-rows packed into <= 64-row tasks; both cut at the budget, and the
    workgroups with the largest dictionaries cut in two)."""
    if maps is None or kernel == "stream":
        return np.append(np.arange(0, A.m, 256), A.m)
    if fill:
        starts = cap_tasks(A, list(range(0, A.m, 64)) + [A.m])
        return cut_blocks(A, starts)
    starts, start = [], 0
    inner = maps.inner
    for sr in range(len(inner) - 1):
        r0, r1 = inner[sr], inner[sr + 1]
        if r1 - start <= 64:
            continue
        if r0 > start:
            starts.append(start)
            start = r0
        while r1 - start > 64:
            starts.append(start)
            start += 64
    if start < A.m or not starts:
        starts.append(start)
    starts.append(A.m)
    starts = cap_tasks(A, starts)
    return cut_blocks(A, starts)


def dict_entries(A, r0, r1, long_t=4096, gap=8):
    """x entries a workgroup over rows [r0, r1) stages: its distinct columns
    as runs, gaps <= gap bridged (doubled until <= 63 runs), split rows out
    (hspmv_api.cpp plan_xdict)."""
    lens = np.diff(A.row_ptr)
    c = np.unique(np.concatenate([A.col_idx[A.row_ptr[r]:A.row_ptr[r + 1]] for r in range(r0, r1)
                                  if lens[r] <= long_t] or [np.zeros(0, np.int32)]))
    if len(c) == 0:
        return 0
    while True:
        brk = np.flatnonzero(np.diff(c) > gap)
        if len(brk) + 1 <= 63:
            break
        gap *= 2
    starts = np.concatenate([[c[0]], c[brk + 1]])
    ends = np.concatenate([c[brk], [c[-1]]])
    return int(np.sum(ends - starts + 1))


def xd_target(dtype):
    """Largest dictionary of a 4-task block sized for 6 workgroups per CU
    (hspmv_api.cpp xd_target_entries: 160 KiB / 6 in 1 KiB granules, minus
    the product staging of U = 4 fp64 / 16 fp32)."""
    sv = np.dtype(dtype).itemsize
    staging = 4 * 64 * (4 if sv == 8 else 16) * sv + 16
    return (160 * 1024 // 6 // 1024 * 1024 - staging) // sv


def cut_blocks(A, starts):
    """Four tasks per workgroup; a workgroup whose dictionary exceeds
    xd_target is cut into two of two tasks each (split_xd_blocks)."""
    target = xd_target(A.val.dtype)
    out = []
    for i in range(0, len(starts) - 1, 4):
        ts = starts[i:i + 5]
        out.append(ts[0])
        if len(ts) - 1 > 2 and dict_entries(A, ts[0], ts[-1]) > target:
            out.append(ts[2])
    return np.array(out + [A.m])


def cap_tasks(A, starts, budget=2048, long_t=4096):
    """Tasks over the nonzero budget are cut at rows (in-kernel rows only:
    split rows count 0), hspmv_api.cpp cap_task_nnz."""
    lens = np.diff(A.row_ptr)
    lens = np.where(lens > long_t, 0, lens)
    out = []
    for a, b in zip(starts[:-1], starts[1:]):
        out.append(a)
        acc = 0
        for r in range(a, b):
            if r > out[-1] and acc + lens[r] > budget:
                out.append(r)
                acc = 0
            acc += lens[r]
    return out + [starts[-1]]


def check_plan(A, plan, bounds, split=True, cap=None):
    blk, runs, pos = plan
    assert len(blk) == len(bounds)
    x = np.arange(A.n, dtype=np.int64) * 7 + 3  # any injective x
    lens = np.diff(A.row_ptr)
    for b in range(len(blk) - 1):
        rec = runs[blk[b]:blk[b + 1]]
        real, sentinel = rec[:-1], rec[-1]
        assert len(real) <= 63
        starts, offs = real[:, 0], real[:, 1]
        total = int(sentinel[1])
        if cap is not None:
            assert total <= cap
        lens_run = np.diff(np.append(offs, total))
        assert np.all(lens_run > 0) and (len(offs) == 0 or offs[0] == 0)
        # runs sorted and disjoint in x
        assert np.all(starts[1:] > starts[:-1] + lens_run[:-1] - 1)
        staged = np.concatenate([x[s:s + ln] for s, ln in zip(starts, lens_run)]) if len(real) else x[:0]
        assert len(staged) == total
        r0, r1 = bounds[b], bounds[b + 1]
        for r in range(r0, r1):
            if split and lens[r] > 4096:
                continue
            k = slice(A.row_ptr[r], A.row_ptr[r + 1])
            assert np.array_equal(staged[pos[k].astype(np.int64)], x[A.col_idx[k]]), (b, r)


@pytest.mark.parametrize("fill", [True, False])
@pytest.mark.parametrize("case", ["lap", "stencil", "banded", "random", "longrows"])
def test_plan_addresses_every_nonzero(case, fill):
    opts = None if fill else {"csr3_plan": "packed"}
    A = {"lap": lambda: gen.laplace2d(120, 90),
         "stencil": lambda: gen.stencil27(14),
         "banded": lambda: gen.banded(5000, per_row=10, half=32, seed=5),
         "random": lambda: _random_rows(1500, 6000, 3, 4),   # many short runs: gaps bridged
         "longrows": _long_rows}[case]()
    for kernel, maps in [("stream", None), ("csr3", hspmv.build_csr3_maps(A, 7, 8))]:
        plan = hspmv.xdict_plan(A, maps, kernel=kernel, cap_entries=65536, options=opts)
        assert plan is not None
        check_plan(A, plan, block_rows(A, maps, kernel, fill))
    if case == "longrows":  # without split rows every row is in the dictionary
        plan = hspmv.xdict_plan(A, None, kernel="stream", cap_entries=65536, split=False)
        check_plan(A, plan, block_rows(A, None, "stream"), split=False)


def test_cap_and_defaults():
    A = gen.stencil27(14)
    plan = hspmv.xdict_plan(A)  # default cap (20 KiB of fp64): a 14^3 stencil fits
    assert plan is not None
    blk, runs, _ = plan
    totals = runs[blk[1:] - 1, 1]
    assert totals.max() <= 20 * 1024 // 8
    # too small a cap: no dictionary
    assert hspmv.xdict_plan(A, cap_entries=totals.max() - 1) is None
    assert hspmv.xdict_plan(A, cap_entries=int(totals.max())) is not None
    # the vector kernel never uses dictionaries
    assert hspmv.xdict_plan(A, kernel="vector") is None
    # fp32 doubles the default cap in entries
    rng = np.random.default_rng(1)  # 24 columns within +-2000 of the row: ~3200 per block
    m = 8000
    cols = np.sort(np.clip(np.arange(m)[:, None] + rng.integers(-2000, 2001, (m, 24)), 0, m - 1), 1)
    A = hspmv.CsrMatrix(m, m, np.arange(0, 24 * m + 1, 24, dtype=np.int32),
                        cols.reshape(-1).astype(np.int32), rng.uniform(-1, 1, 24 * m))
    assert hspmv.xdict_plan(A) is None                          # > 2560 fp64 entries
    assert hspmv.xdict_plan(A.astype(np.float32)) is not None   # <= 5120 fp32 entries


def test_stencil_reuse():
    """On the RCM 27-point stencil a 256-row workgroup references ~5.9 x
    entries per row against 26.6 nonzeros (SURVEY.md C3's structure)."""
    A = gen.stencil27(40)
    blk, runs, _ = hspmv.xdict_plan(A, cap_entries=65536)
    entries = runs[blk[1:] - 1, 1].sum()
    assert entries < 0.35 * A.nnz
    nruns = np.diff(blk) - 1
    assert nruns.mean() < 12


def test_0_1_signature_equals_ex():
    """hspmv_xdict_plan keeps its 0.1 signature (kernel flags as the third
    argument) and plans exactly what hspmv_xdict_plan_ex plans with those
    flags in an hspmv_options."""
    import ctypes as C
    from hspmv import _lib
    A = gen.stencil27(12)
    cs = A.c_struct()
    res = []
    for ex in (False, True):
        nb, nr = C.c_int64(), C.c_int64()
        if ex:
            opt = _lib.make_options(_lib.KERNEL_STREAM, None)
            third = C.byref(opt)
            fn = hspmv.lib().hspmv_xdict_plan_ex
        else:
            third = _lib.KERNEL_STREAM
            fn = hspmv.lib().hspmv_xdict_plan
        assert fn(C.byref(cs), None, third, 0, C.byref(nb), C.byref(nr), None, None, None) == 0
        blk = np.empty(nb.value + 1, np.int32)
        runs = np.empty((nr.value, 2), np.int32)
        pos = np.zeros(A.nnz, np.uint16)
        assert fn(C.byref(cs), None, third, 0, C.byref(nb), C.byref(nr), blk.ctypes.data,
                  runs.ctypes.data, pos.ctypes.data) == 0
        res.append((blk, runs, pos))
    assert res[0][0].size > 1
    for a, b in zip(*res):
        assert np.array_equal(a, b)
