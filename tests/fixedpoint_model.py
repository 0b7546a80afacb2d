"""A CPU restatement of the reproducible (fixed-point) column-sorted SpMV
(hspmv_options.deterministic = 2; csrc/csort.hip fix_q, hspmv_csort_xexp,
csrc/hspmv_csort_build.cpp rexp) -- test infrastructure, like oracle/.

Because that path's row sums are integer sums, its y does not depend on the
order in which the GPU adds them, so numpy can state it exactly:

* xexp = the largest frexp exponent of a finite, nonzero |x| over all of x
  (|x| < 2^xexp), floored at -1000; E = 50 - xexp;
* per row r: rexp[r] = -(ilogb max_r|v| + 1) (rows of <= 4096 nonzeros), and
  v' = ldexp(v, rexp[r]) exactly;
* per nonzero: q = rint(v' x 2^E) (half-even) -- the product of two fp32
  values is exact in fp64, and so is the scaling;
* y[r] = T(ldexp(double(sum_r q), -E - rexp[r])): the int64 sum converted to
  fp64 once (correctly rounded), scaled, rounded to the value type.

This is what one column part (csort_parts = 1) gives for fp32 data on rows
of <= 4096 nonzeros: the slot holds sum_r q, the workgroup writes the fp64
value as the fp32 partial (or y directly), and the finishing pass adds one
partial.  With two or more parts each part's sum is rounded on its own and
the parts' boundaries come from the build's cost model, so those handles
are checked against the error bound instead (tests/test_csort.py).
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


def reproducible_csort_y(row_ptr, col_idx, val, x) -> np.ndarray:
    """y of the fixed-point csort with one column part, fp32 data (see the
    module docstring); NaN on rows of more than 4096 nonzeros, which the
    kernel slices (their slices add in the finishing pass's shuffle tree)."""
    assert val.dtype == np.float32 and x.dtype == np.float32
    row_ptr = np.asarray(row_ptr, np.int64)
    lens = np.diff(row_ptr)
    E = FIX_BITS - xexp_of(x)
    rexp = row_scales(row_ptr, val)
    rows = np.repeat(np.arange(lens.size), lens)
    vs = np.ldexp(val, rexp[rows].astype(np.int32))  # fp32, exact
    prod = vs.astype(np.float64) * x[col_idx].astype(np.float64)  # exact
    q = np.rint(np.ldexp(prod, E)).astype(np.int64)
    s = np.zeros(lens.size, np.int64)
    np.add.at(s, rows, q)
    y = np.ldexp(s.astype(np.float64), (-E - rexp).astype(np.int32)).astype(np.float32)
    y[lens > 4096] = np.nan
    return y
