"""The oracle's x264_me_search_ref (oracle.c FN(me_search_ref): reference encoder/me.c:182-798 with
DIA / HEX / UMH, the predictor checks of x264_predictor_clip / _roundclip, the qpel conversion
and refine_subpel) against a literal Python restatement (tests/search_cases.py, over numpy_ref's
SAD / get_ref, then test_cpu_refine_chroma's refine_subpel): every partition size, subme 1 / 2 /
4 / 7 / 9 (both predictor paths, every refine schedule), me_range 16 and 24, unweighted and
weighted references (p_fref_w weighted, COST_MV_HPEL's get_ref weighted), with chroma ME on at
subme >= 5, 8 and 10 bit, with the reference's call counts."""
import numpy as np
import pytest

import refine_cases as rc
import search_cases as sc
from test_cpu_refine_chroma import _weigh, refine_chroma_py


def _case(bd, cf, W, H, fade, seed):
    cc = rc.ChromaCase(bd, W, H, cf, seed=seed, fade=fade)
    weights = rc.FADE_WEIGHTS if fade else (None, None, None)
    fw = cc.luma[0] if weights[0] is None else _weigh(cc.luma[0].astype(np.int64), weights[0], bd).astype(
        cc.luma[0].dtype)
    return cc, weights, fw


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("me_method", [0, 1, 2])
@pytest.mark.parametrize("i_pixel", [0, 1, 2, 3])
@pytest.mark.parametrize("subme,fade,chroma", [(1, 0, 0), (2, 0, 0), (4, 1, 0), (7, 0, 1), (9, 1, 1)])
def test_search_oracle_vs_python(oracle, bd, me_method, i_pixel, subme, fade, chroma):
    W, H, cf = 64, 48, 1
    cc, weights, fw = _case(bd, cf, W, H, fade, seed=bd + i_pixel + 3 * me_method)
    me_range = 24 if subme == 9 else 16
    pos, par, mvc = sc.jobs(W // 16, H // 16, 1, i_pixel, seed=subme * 5 + me_method)
    cm, c0 = rc.cost_mv()
    ext = oracle.refine_ext(chroma, cf, 0, weights)
    got, ne = oracle.me_search_ref(bd, cc.fenc_y, cc.origin, cc.stride, cc.luma, fw, cc.origin, cc.stride, i_pixel,
                                   me_method, subme, me_range, pos[:, 1:], par, mvc, cm, c0, ext=ext,
                                   fenc_c=cc.fenc_c, fc_origin=cc.co, fcs=cc.cs, ref_c=cc.ref_c, rc_origin=cc.co,
                                   rcs=cc.cs)
    for i in range(len(pos)):
        x, y = int(pos[i, 1]), int(pos[i, 2])
        want, wn = sc.search_ref_py(cc.fenc_y, cc.luma, fw, cc.origin, cc.stride, x, y, i_pixel, par[i], mvc[i], cm,
                                    c0, me_method, subme, me_range, weight0=weights[0], bd=bd)
        assert ne[i, 0] == wn[0] | (wn[1] << 16), (i, hex(ne[i, 0]), wn)
        if subme >= 2:
            rpar = (want[1], want[2], par[i, 0], par[i, 1], par[i, 6], par[i, 7], par[i, 8], par[i, 9])
            want, wrn = refine_chroma_py(cc, x, y, i_pixel, rpar, want[0], cm, c0, subme, 0, chroma, weights)
            assert ne[i, 1] == wrn, (i, hex(ne[i, 1]), hex(wrn))
        assert tuple(got[i]) == tuple(want), (i, got[i], want)
