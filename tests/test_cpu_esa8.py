"""CPU: the oracle's sub-partition ESA decisions (oracle/oracle.c me_search_esa8, the semantics of
x264hip_*_me_search_esa8; reference encoder/me.c:618-631 for PIXEL_16x8 / 8x16 / 8x8 at the
offsets of analyse.c:1425,1480,1546) against two other restatements: plain Python loops
(tests/esa8_cases.py) and the 16x16 table decision me_esa_argmin applied to tables summed from
the oracle's 8x8 quadrant tables (me_search_full8)."""
import numpy as np
import pytest

import esa8_cases as ec


def _frames(bd, w, h, seed):
    from conftest import load_package
    load_package()
    from x264hip import synth
    return synth.make_sequence(2, w, h, bd, seed=seed)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("limit", [None, 20])
def test_esa8_oracle_vs_python(oracle, bd, limit):
    """every partition of a 3x2-MB frame, me_range 4, windows moved off the MB centre and (limit
    20) clipped by mv_limit_fpel at the frame edges"""
    W, H, me_range = 48, 32, 4
    planes, stride, origin = _frames(bd, W, H, 7)
    mbw, mbh = W // 16, H // 16
    cen, par, ic = ec.jobs(mbw, mbh, me_range, seed=bd + (limit or 0), spread=3, frac=0.6, centre_amp=4,
                           limit=limit)
    cm, c0 = ec.cost_mv()
    f, r = planes[1].ravel(), planes[0].ravel()
    got = oracle.me_search_esa8(bd, f, origin, stride, r, origin, stride, mbw, mbh, me_range, par, ic, cm, c0)
    want = ec.esa8_py(f, origin, stride, r, origin, stride, mbw, me_range, par, ic, cm, c0, range(mbw * mbh))
    for i, v in want.items():
        assert tuple(got[i]) == v, (i, tuple(got[i]), v)
    assert (got[:, 0] < ic).any()                       # the search improved on some predictors


@pytest.mark.parametrize("bd", [8, 10])
def test_esa8_oracle_vs_quadrant_tables(oracle, bd):
    """the partitions' SADs are sums of the MB's 8x8 quadrant SADs at the same mv, so the
    decision over quadrant-summed tables (me_esa_argmin, me.c:618-631 over a table) equals the
    direct one for windows inside the table"""
    W, H, R, me_range = 96, 64, 12, 4
    planes, stride, origin = _frames(bd, W, H, 11)
    mbw, mbh = W // 16, H // 16
    nmb = mbw * mbh
    cen, par, ic = ec.jobs(mbw, mbh, me_range, seed=5, spread=4, frac=0.7, centre_amp=3)
    cm, c0 = ec.cost_mv()
    f, r = planes[1].ravel(), planes[0].ravel()
    got = oracle.me_search_esa8(bd, f, origin, stride, r, origin, stride, mbw, mbh, me_range, par, ic, cm, c0)
    q = oracle.me_search_full8(bd, f, origin, stride, r, origin, stride, mbw, mbh, R).astype(np.int64)
    q = q.reshape(nmb, 4, 2 * R + 1, 2 * R + 1)
    combos = [(0, 1), (2, 3), (0, 2), (1, 3), (0,), (1,), (2,), (3,)]
    w = 2 * R + 1
    pitch = (w + 3) & ~3
    tabs = np.zeros((nmb * 8, w, pitch), np.uint16 if bd == 8 else np.uint32)
    for p, qs in enumerate(combos):
        tabs[p::8, :, :w] = sum(q[:, k] for k in qs)
    want = oracle.me_esa_argmin(bd, tabs, R, me_range, par, ic, cm, c0)
    assert np.array_equal(got, want)
