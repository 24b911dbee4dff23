"""GPU parity tests: the HIP path vs the oracle's golden fixtures, through
the C-ABI.  Run on the MI355X box: pytest -m gpu."""
import numpy as np
import pytest

from golden_util import prehashed_arrays

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("wbits", [16, 8])
def test_prehashed_golden(lib, wbits):
    from minbft_amd.authenticator import Authenticator
    xy, e, r, s, exp, labels = prehashed_arrays()
    with Authenticator(0) as a:
        a.set_key_window(wbits)
        slots, valid = a.register_points(xy)
        assert valid.all()
        st = a.verify_prehashed(e, r, s, slots)
    got = (st == 0).astype(np.int64)
    bad = [(labels[i], int(st[i]), int(exp[i])) for i in range(len(exp)) if got[i] != exp[i]]
    assert not bad, bad[:20]
