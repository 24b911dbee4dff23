"""GPU parity tests: the HIP path vs the oracle's golden fixtures, through
the C-ABI.  Run on the MI355X box: pytest -m gpu."""
import numpy as np
import pytest

from golden_util import prehashed_arrays

pytestmark = pytest.mark.gpu


def test_prehashed_golden(gpu_auth):
    xy, e, r, s, exp, labels = prehashed_arrays()
    slots, valid = gpu_auth.register_points(xy)
    assert valid.all()
    st = gpu_auth.verify_prehashed(e, r, s, slots)
    got = (st == 0).astype(np.int64)
    bad = [(labels[i], int(st[i]), int(exp[i])) for i in range(len(exp)) if got[i] != exp[i]]
    assert not bad, bad[:20]
