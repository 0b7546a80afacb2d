"""A CPU restatement of the reproducible (fixed-point) column-sorted SpMV
(hspmv_options.deterministic = 2; csrc/csort.hip fix_q, hspmv_csort_xexp,
csrc/hspmv_csort_build.cpp rexp) -- test infrastructure, like oracle/.

Because that path's row sums are integer sums, its y does not depend on the
order in which the GPU adds them, so numpy can state it exactly:

* xexp = the largest frexp exponent of a finite, nonzero |x| over all of x
  (|x| < 2^xexp), floored at -1000; E = 50 - xexp;
* per row r: rexp[r] = -(ilogb max_r|v| + 1) (rows of <= 4096 nonzeros), and
  v' = ldexp(v, rexp[r]) exactly;
* per nonzero: q = rint(v' x 2^E) (half-even) of the EXACT product -- for
  fp32 data the fp64 product is exact; for fp64 data the kernel's one fma
  against a rounding constant rounds the exact product once, which the
  model states with Python integers (exact_q);
* y[r] = T(ldexp(double(sum_r q), -E - rexp[r])): the int64 sum converted to
  fp64 once (correctly rounded), scaled, rounded to the value type.

This is what the kernel gives on rows of <= 4096 nonzeros: each column
part's slot holds that part's sum_r q, the workgroup writes the fp64 value
as a partial (fp32 for fp32 data: part32; fp64 for fp64) or y directly with
one part, and the finishing pass adds the partials in part order in fp64 and
rounds y.  The
parts' boundaries come from the build's cost model; the handle reports them
(hspmv_info.csort_part_begin).
"""
import numpy as np

FIX_BITS = 50


def xexp_of(x: np.ndarray) -> int:
    a = np.abs(x.astype(np.float64))
    a = a[(a != 0) & np.isfinite(a)]
    if a.size == 0:
        return -1000
    e = int(np.frexp(a)[1].max())
    return max(e, -1000)


def row_scales(row_ptr, val) -> np.ndarray:
    lens = np.diff(row_ptr)
    vmax = np.zeros(lens.size)
    nz = lens > 0
    if val.size:
        vmax[nz] = np.maximum.reduceat(np.abs(val.astype(np.float64)), row_ptr[:-1][nz])
    rexp = np.zeros(lens.size, np.int64)
    pos = vmax > 0
    rexp[pos] = -(np.frexp(vmax[pos])[1] - 1 + 1)  # ilogb(m) = frexp exponent - 1
    return rexp


def exact_q(v: np.ndarray, x: np.ndarray, E: int) -> np.ndarray:
    """rint(v * x * 2^E), half-even, of the exact product of two fp64 arrays
    (Python integers: v = mv 2^ev, x = mx 2^ex with 53-bit integer mv, mx)."""
    fv, ev = np.frexp(v)
    fx, ex = np.frexp(x)
    mv = np.ldexp(fv, 53).astype(np.int64).astype(object)
    mx = np.ldexp(fx, 53).astype(np.int64).astype(object)
    k = (ev.astype(np.int64) + ex.astype(np.int64) - 106 + E)
    out = np.empty(v.size, np.int64)
    for i, (a, b, kk) in enumerate(zip(mv, mx, k.tolist())):
        P = a * b
        if kk >= 0:
            q = P << kk
        else:
            sh = -kk
            q = P >> sh  # floor, also for negative P
            rem = P - (q << sh)
            half = 1 << (sh - 1)
            if rem > half or (rem == half and (q & 1)):
                q += 1
        out[i] = q
    return out


def reproducible_csort_y(row_ptr, col_idx, val, x, part_begin=(0,)) -> np.ndarray:
    """y of the fixed-point csort, fp32 or fp64 data (see the module docstring);
    NaN on rows of more than 4096 nonzeros, which the kernel slices (their
    slices add in the finishing pass's shuffle tree).  part_begin: the first
    column of each column part (hspmv_info.csort_part_begin): each part's
    integer row sum becomes an fp64 value, rounded to an fp32 partial, and
    the partials are added in part order in fp64 and rounded to y."""
    assert val.dtype == x.dtype and val.dtype in (np.float32, np.float64)
    T = val.dtype.type
    row_ptr = np.asarray(row_ptr, np.int64)
    lens = np.diff(row_ptr)
    E = FIX_BITS - xexp_of(x)
    rexp = row_scales(row_ptr, val)
    rows = np.repeat(np.arange(lens.size), lens)
    vs = np.ldexp(val, rexp[rows].astype(np.int32))  # exact
    if T is np.float32:
        prod = vs.astype(np.float64) * x[col_idx].astype(np.float64)  # exact
        q = np.rint(np.ldexp(prod, E)).astype(np.int64)
    else:
        q = exact_q(vs, x[col_idx], E)
    bounds = np.asarray(list(part_begin), np.int64)
    part = np.searchsorted(bounds, np.asarray(col_idx, np.int64), side="right") - 1
    acc = np.zeros(lens.size, np.float64)
    for h in range(bounds.size):
        s = np.zeros(lens.size, np.int64)
        sel = part == h
        np.add.at(s, rows[sel], q[sel])
        p = np.ldexp(s.astype(np.float64), (-E - rexp).astype(np.int32)).astype(T)
        acc = acc + p.astype(np.float64) if h else p.astype(np.float64)
    y = acc.astype(T)
    y[lens > 4096] = np.nan
    return y
