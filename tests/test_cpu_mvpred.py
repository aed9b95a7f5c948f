"""CPU: the predictor restatement of tests/mvpred_cases.py on the cases mvpred.c distinguishes
(reference common/mvpred.c:129-157, 519-600): the frame's first MB, the top row (A only), the left
column (median with A = 0), the right column (C unavailable -> D), the interior median, the
lowres mv's 16-bit doubling and the temporal scaling's clip."""
import numpy as np

import mvpred_cases as mp


def _field(mbw, mbh, seed=1):
    rs = np.random.default_rng(seed)
    return {(y, x): (int(rs.integers(-99, 99)), int(rs.integers(-99, 99))) for y in range(mbh) for x in range(mbw)}


def test_predict_mv_16x16_cases():
    mbw, mbh = 5, 4
    f = _field(mbw, mbh)
    assert mp.predict_mv_16x16(f, 0, 0, mbw) == (0, 0)                       # nothing available
    assert mp.predict_mv_16x16(f, 3, 0, mbw) == f[(0, 2)]                    # top row: A only
    a, b, c = (0, 0), f[(1, 0)], f[(1, 1)]                                   # left column: A off the frame
    assert mp.predict_mv_16x16(f, 0, 2, mbw) == (mp.median(a[0], b[0], c[0]), mp.median(a[1], b[1], c[1]))
    a, b, d = f[(2, 3)], f[(1, 4)], f[(1, 3)]                                # right column: C -> D
    assert mp.predict_mv_16x16(f, 4, 2, mbw) == (mp.median(a[0], b[0], d[0]), mp.median(a[1], b[1], d[1]))
    a, b, c = f[(2, 1)], f[(1, 2)], f[(1, 3)]                                # interior
    assert mp.predict_mv_16x16(f, 2, 2, mbw) == (mp.median(a[0], b[0], c[0]), mp.median(a[1], b[1], c[1]))


def test_predict_mv_ref16x16_cases():
    mbw, mbh = 4, 3
    f = _field(mbw, mbh, seed=2)
    # spatial only: left, top, top-left, top-right, zeros off the frame
    assert mp.predict_mv_ref16x16(f, 0, 0, mbw, mbh) == [(0, 0)] * 4
    assert mp.predict_mv_ref16x16(f, 3, 1, mbw, mbh) == [f[(1, 2)], f[(0, 3)], f[(0, 2)], (0, 0)]
    # the lowres mv doubled in 16-bit lanes; an invalid field (0x7fff first) adds nothing
    lr = np.zeros((mbw * mbh, 2), np.int16)
    lr[5] = (20000, -20000)
    got = mp.predict_mv_ref16x16(f, 1, 1, mbw, mbh, lowres=lr)
    assert got[0] == (40000 - 65536, -40000 + 65536)
    lr[0, 0] = 0x7fff
    assert len(mp.predict_mv_ref16x16(f, 1, 1, mbw, mbh, lowres=lr)) == 4
    # temporal: colocated, right (not on the last column), below (not on the last row), clipped
    tm = np.zeros((mbw * mbh, 2), np.int16)
    tm[5] = (-30000, 10)
    tm[6] = (100, -3)
    tm[9] = (7, 7)
    got = mp.predict_mv_ref16x16(f, 1, 1, mbw, mbh, tmv=tm, tscale=512)
    assert got[4:] == [(-32768, 20), (200, -6), (14, 14)]
    assert len(mp.predict_mv_ref16x16(f, 3, 2, mbw, mbh, tmv=tm, tscale=256)) == 5


def test_limits_match_search_cases():
    """with an unbounded i_mv_range the limits are search_cases.jobs' (analyse.c:330-349)"""
    lim = mp.limits(2, 1, 6, 4, 1 << 14)
    smin = (4 * (-16 * 2 - 24), 4 * (-16 * 1 - 24))
    smax = (4 * (16 * (6 - 2 - 1) + 24), 4 * (16 * (4 - 1 - 1) + 24))
    assert lim == ((smin[0] >> 2) + 6, (smin[1] >> 2) + 6, (smax[0] >> 2) - 6, (smax[1] >> 2) - 6) + smin + smax
