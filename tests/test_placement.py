"""Placement trials (hspmv_options.placement_trials = K, opt-in):
the streamed arrays are copied into K-1 further allocations, each set is
timed and the fastest kept.  Checked here: the trials run on an HBM-resident
matrix (footprint > 192 MiB), the kept set gives y bit for bit equal to a
handle without trials, and a MALL-resident matrix skips them."""
import numpy as np
import pytest

import hspmv
from hspmv import gen

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    assert hspmv.device_count() >= 1, "no HIP device visible: the gpu tests must run on the MI355X box"


def test_trials_keep_y_bitwise():
    # 2.4 M rows x 10 nonzeros fp64: ~320 MB streamed, HBM-resident
    A = gen.banded(2_400_000, per_row=10, half=32, seed=3)
    x = gen.rand_x(A.n, 9)
    with hspmv.SpMV(A) as op:
        y0 = op(x)
        assert op.info["placement_trials"] == 0  # off by default
    with hspmv.SpMV(A, options={"placement_trials": 3}) as op:
        y1 = op(x)
        info = op.info
    assert info["placement_trials"] == 3 and 0 <= info["placement_pick"] < 3
    assert len(info["placement_us"]) == 3 and min(info["placement_us"]) > 0
    assert np.array_equal(y0, y1)


def test_mall_resident_skips_trials():
    A = gen.laplace2d(300, 300)
    with hspmv.SpMV(A, options={"placement_trials": 3}) as op:
        op(gen.rand_x(A.n, 1))
        assert op.info["placement_trials"] == 0
