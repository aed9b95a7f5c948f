"""CPU: the oracle reproduces the committed golden fixtures (tests/golden/,
made by tests/golden/make_golden.py from the reference's checkasm inputs), so
any drift of the checker itself is caught before it is trusted on the GPU."""
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("bd", [8, 10])
def test_oracle_reproduces_golden(oracle, bd):
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    with np.load(os.path.join(HERE, "golden", f"golden_{bd}.npz"), allow_pickle=False) as z:
        want = {k: z[k] for k in z.files}
    got = mg.compute(bd)
    assert set(got) == set(want)
    for k in sorted(want):
        assert np.array_equal(np.asarray(got[k]), want[k]), k
