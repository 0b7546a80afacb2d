"""The XCD block order is a bijection on [0, nb) for every chunk size.

Restates xcd_chunk_remap (heterogeneous-spmv_amd/csrc/spmv_device.cuh) in
numpy; a non-bijective order would leave rows of y unwritten, which a parity
test can miss when y's buffer still holds an earlier, equal result.
"""
import numpy as np
import pytest


def xcd_chunk_remap(b, nb, s):
    b = np.asarray(b, dtype=np.int64)
    if s <= 1:
        return b.copy()
    span = 8 * s
    full = (nb // span) * span
    i, x = b // 8, b % 8
    out = (i // s) * span + x * s + (i % s)
    return np.where(b >= full, b, out)


@pytest.mark.parametrize("nb", [1, 7, 8, 9, 63, 64, 65, 1000, 3907, 9766, 40001])
@pytest.mark.parametrize("s", [1, 2, 4, 16, 64, 488])
def test_bijective(nb, s):
    m = xcd_chunk_remap(np.arange(nb), nb, s)
    assert np.array_equal(np.sort(m), np.arange(nb))


def test_full_chunk_gives_contiguous_eighths():
    nb = 8 * 100
    m = xcd_chunk_remap(np.arange(nb), nb, 100)
    for x in range(8):  # blocks dispatched to XCD x (b % 8 == x)
        assert np.array_equal(np.sort(m[x::8]), np.arange(100 * x, 100 * (x + 1)))


def test_small_chunk_keeps_front_compact():
    nb, s = 8 * 16 * 50, 16
    m = xcd_chunk_remap(np.arange(nb), nb, s)
    # any 8*s consecutive dispatch slots cover one 8*s-block logical window
    for g in range(0, nb, 8 * s):
        w = m[g:g + 8 * s]
        assert w.max() - w.min() == 8 * s - 1
