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
@pytest.mark.parametrize("me_method", [0, 1, 2, 3])
@pytest.mark.parametrize("i_pixel", [0, 1, 2, 3, 4, 5, 6])
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


INT_MAX = (1 << 31) - 1


def _chain_py(mr, k, i_pixel, pos, par, mvc, cm, c0, me_method, subme, me_range, thr, rcost, chroma):
    """reference k of analyse.c:1268-1314's loop for every partition, restated: search_ref_py then
    refine_chroma_py with the partition's threshold (thr, rcost as the oracle takes them)"""
    res = []
    for i in range(len(pos)):
        x, y = int(pos[i, 1]), int(pos[i, 2])
        r = mr.refs[k]
        want, _ = sc.search_ref_py(mr.fenc_y, r.luma, r.luma[0], mr.origin, mr.stride, x, y, i_pixel, par[i], mvc[i],
                                   cm, c0, me_method, subme, me_range, bd=mr.bd)
        rpar = (want[1], want[2], par[i, 0], par[i, 1], par[i, 6], par[i, 7], par[i, 8], par[i, 9])
        t = [int(thr[i])]
        cc = _as_case(mr, k)
        want, _ = refine_chroma_py(cc, x, y, i_pixel, rpar, want[0], cm, c0, subme, 0, chroma, (None, None, None),
                                   thresh=t, ref_cost=int(rcost[i]))
        thr[i] = t[0]
        res.append(want)
    return res


def _as_case(mr, k):
    """reference k of a MultiRef in ChromaCase's shape"""
    o = type("Case", (), {})()
    o.bd, o.cf, o.stride, o.origin, o.cs, o.co = mr.bd, mr.cf, mr.stride, mr.origin, mr.cs, mr.co
    o.fenc_y, o.fenc_c, o.luma, o.ref_c = mr.fenc_y, mr.fenc_c, mr.refs[k].luma, mr.refs[k].ref_c
    return o


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("me_method", [1, 2])
@pytest.mark.parametrize("i_pixel", [0, 3])
def test_search_thresh_chain_oracle_vs_python(oracle, bd, me_method, i_pixel):
    """x264's default ref = 3 chain (analyse.c:1260-1314, common/base.c:384): each reference's
    search with p_halfpel_thresh (me.c:931-944) and the i_ref_cost adjustments around it, the
    oracle's me_search_ref_thresh against the Python restatement, threshold by threshold"""
    W, H, cf, subme, me_range = 64, 48, 1, 7, 16
    mr = sc.MultiRef(bd, W, H, cf, seed=3 + bd + i_pixel)
    cm, c0 = rc.cost_mv()
    ext = oracle.refine_ext(1, cf, 0, (None, None, None))
    n = len(mr.jobs(0, i_pixel, 0)[0])
    thr = np.full(n, INT_MAX, np.int32)
    thr_py = thr.copy()
    early = 0
    for k in range(3):
        pos, par, mvc = mr.jobs(k, i_pixel, seed=17 * k + me_method)
        rcost = np.full(n, 40 * (1 if k == 0 else 3), np.int32)
        r = mr.refs[k]
        got, ne = oracle.me_search_ref(bd, mr.fenc_y, mr.origin, mr.stride, r.luma, r.luma[0], mr.origin, mr.stride,
                                       i_pixel, me_method, subme, me_range, pos[:, 1:], par, mvc, cm, c0, ext=ext,
                                       fenc_c=mr.fenc_c, fc_origin=mr.co, fcs=mr.cs, ref_c=r.ref_c, rc_origin=mr.co,
                                       rcs=mr.cs, thresh=thr, ref_cost=rcost, out_fill=-7)
        want = _chain_py(mr, k, i_pixel, pos, par, mvc, cm, c0, me_method, subme, me_range, thr_py, rcost, 1)
        for i, w in enumerate(want):
            assert tuple(got[i, :3]) == tuple(w[:3]), (k, i, got[i], w)
            assert got[i, 3] == (-7 if w[3] is None else w[3]), (k, i, got[i], w)
        assert np.array_equal(thr, thr_py), k
        early += int((got[:, 3] == -7).sum())
        if k == 0:
            assert early == 0                       # INT_MAX - i_ref_cost: never on the first reference
    assert early > 0                                # the exit fired on later references


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("subme", [2, 5, 7, 9])
def test_refdupe_oracle_vs_python(oracle, bd, subme):
    """x264_me_refine_qpel_refdupe (me.c:812-815) after reference 0's search, as analyse.c:1279-1283
    runs it on a reference that duplicates reference 0: start at reference 0's mv, m->cost as the
    reused x264_me_t holds it, with the threshold"""
    W, H, cf, i_pixel = 64, 48, 1, 0
    mr = sc.MultiRef(bd, W, H, cf, seed=9 + bd)
    cm, c0 = rc.cost_mv()
    chroma = int(subme >= 5)
    ext = oracle.refine_ext(chroma, cf, 0, (None, None, None))
    pos, par, mvc = mr.jobs(0, i_pixel, seed=subme)
    n = len(pos)
    thr = np.full(n, INT_MAX, np.int32)
    r = mr.refs[0]
    rc0 = np.full(n, 40, np.int32)
    out0, _ = oracle.me_search_ref(bd, mr.fenc_y, mr.origin, mr.stride, r.luma, r.luma[0], mr.origin, mr.stride,
                                   i_pixel, 1, subme, 16, pos[:, 1:], par, mvc, cm, c0, ext=ext, fenc_c=mr.fenc_c,
                                   fc_origin=mr.co, fcs=mr.cs, ref_c=r.ref_c, rc_origin=mr.co, rcs=mr.cs, thresh=thr,
                                   ref_cost=rc0)
    rc1 = np.full(n, 120, np.int32)
    rpar = np.stack([out0[:, 1], out0[:, 2], par[:, 0] + 4, par[:, 1] - 4, par[:, 6], par[:, 7], par[:, 8], par[:, 9]],
                    1).astype(np.int16)
    init = (out0[:, 0] + rc0).astype(np.int32)
    thr_py = thr.copy()
    got, ne = oracle.me_refine_qpel_refdupe(bd, mr.fenc_y, mr.origin, mr.stride, r.luma, mr.origin, mr.stride, i_pixel,
                                            subme, pos[:, 1:], rpar, init, cm, c0, thresh=thr, ref_cost=rc1,
                                            out_fill=-7, ext=ext, fenc_c=mr.fenc_c, fc_origin=mr.co, fcs=mr.cs,
                                            ref_c=r.ref_c, rc_origin=mr.co, rcs=mr.cs)
    for i in range(n):
        t = [int(thr_py[i])]
        w, wn = refine_chroma_py(_as_case(mr, 0), int(pos[i, 1]), int(pos[i, 2]), i_pixel, rpar[i], init[i], cm, c0,
                                 subme, 0, chroma, (None, None, None), refdupe=True, thresh=t, ref_cost=120)
        thr_py[i] = t[0]
        assert tuple(got[i, :3]) == tuple(w[:3]) and got[i, 3] == (-7 if w[3] is None else w[3]), (i, got[i], w)
        assert ne[i] == wn, (i, hex(ne[i]), hex(wn))
    assert np.array_equal(thr, thr_py)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("i_pixel", [0, 3])
def test_umh_cross_past_limit_oracle_vs_python(oracle, bd, i_pixel):
    """UMH with mv_limit_fpel one pixel short of the true motion: the winners DIA1_ITER finds past
    the limit, and the CROSS around them that range-checks only its moving axis (me.c:146-176)"""
    W, H, cf, subme = 64, 48, 1, 1
    cc, weights, fw = _case(bd, cf, W, H, 0, seed=13 + bd)
    pos, par, mvc = sc.jobs(W // 16, H // 16, 1, i_pixel, seed=4)
    par[:, 4] = np.minimum(par[:, 4], 2)
    par[:, 5] = np.minimum(par[:, 5], 1)
    cm, c0 = rc.cost_mv()
    got, ne = oracle.me_search_ref(bd, cc.fenc_y, cc.origin, cc.stride, cc.luma, fw, cc.origin, cc.stride, i_pixel, 2,
                                   subme, 16, pos[:, 1:], par, mvc, cm, c0)
    for i in range(len(pos)):
        want, wn = sc.search_ref_py(cc.fenc_y, cc.luma, fw, cc.origin, cc.stride, int(pos[i, 1]), int(pos[i, 2]),
                                    i_pixel, par[i], mvc[i], cm, c0, 2, subme, 16, bd=bd)
        assert tuple(got[i]) == tuple(want) and ne[i, 0] == wn[0] | (wn[1] << 16), (i, got[i], want)
    assert ((got[:, 1] == 12) | (got[:, 2] == 8)).any()
