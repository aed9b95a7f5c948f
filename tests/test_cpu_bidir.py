"""The oracle's x264_me_refine_bidir_satd (oracle.c FN(me_refine_bidir): reference encoder/me.c:
994-1183 with rd = 0, the dia4d passes with the visited bits, mc.avg's rounding / implicit-weight
averages of common/mc.c:49-99, mbcmp + four mv costs) against the literal Python restatement of
tests/bidir_cases.py: every partition 16x16 .. 8x8, SATD and SAD, weights 32 and != 32, 8 and 10
bit, with the reference's mbcmp-call and pass counts."""
import numpy as np
import pytest

import bidir_cases as bc
import refine_cases as rc
import search_cases as sc


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("i_pixel", [0, 1, 2, 3])
@pytest.mark.parametrize("satd", [1, 0])
def test_bidir_oracle_vs_python(oracle, bd, i_pixel, satd):
    W, H, cf = 48, 32, 1
    mr = sc.MultiRef(bd, W, H, cf, seed=21 + bd + i_pixel)
    pos, par, wt = bc.jobs(mr, i_pixel, seed=5 + i_pixel + satd)
    cm, c0 = rc.cost_mv()
    out, cost, ne = oracle.me_refine_bidir(bd, mr.fenc_y, mr.origin, mr.stride, mr.refs[0].luma, mr.refs[1].luma,
                                           mr.origin, mr.stride, i_pixel, satd, pos[:, 1:], par, wt, cm, c0)
    for i in range(len(pos)):
        want, wc, wn = bc.refine_bidir_py(mr.fenc_y, mr.refs[0].luma, mr.refs[1].luma, mr.origin, mr.stride,
                                          int(pos[i, 1]), int(pos[i, 2]), i_pixel, satd, par[i], int(wt[i]), cm, c0, bd)
        assert tuple(out[i]) == want and cost[i] == wc and ne[i] == wn, (i, out[i], want, cost[i], wc, ne[i], wn)
    assert (ne >> 16).max() >= 2                               # some partitions moved
    assert (ne == 0).any()                                     # the guard-band early return ran
