"""GPU parity: x264_me_search_ref at full resolution (x264hip_*_me_search_ref, reference
encoder/me.c:182-798: predictor checks, DIA / HEX / UMH integer search, qpel conversion, then
refine_subpel) against the oracle restatement (pinned by tests/test_cpu_search.py's literal Python
restatement): every partition size, subme 1 / 2 / 4 / 7 / 9, me_range 16 / 24, unweighted and
weighted references, chroma ME at subme >= 5, two frame pairs per launch, with the reference's
call counts; and whole 1080p frames at x264's default settings (HEX, subme 7, chroma ME)."""
import numpy as np
import pytest
import torch

import refine_cases as rc
import search_cases as sc
from test_cpu_refine_chroma import _weigh

pytestmark = pytest.mark.gpu


def _t(a, bd):
    a = np.ascontiguousarray(a)
    return torch.from_numpy(a.view(np.int16) if bd == 10 else a).cuda()


def _run(hip, oracle, bd, cf, W, H, nframes, i_pixel, me_method, subme, me_range, fade, chroma, seed):
    weights = rc.FADE_WEIGHTS if fade else (None, None, None)
    cases = [rc.ChromaCase(bd, W, H, cf, seed=seed + 11 * k, fade=fade) for k in range(nframes)]
    c0_ = cases[0]
    rows = c0_.ref.y.shape[0]
    crows = (c0_.ref.nv if cf in (1, 2) else c0_.ref.u).shape[0]
    fws = [c.luma[0] if not fade else _weigh(c.luma[0].astype(np.int64), weights[0], bd).astype(c.luma[0].dtype)
           for c in cases]
    fenc = _t(np.stack([c.fenc_y.reshape(rows, -1) for c in cases]), bd)
    luma = [_t(np.stack([c.luma[k].reshape(rows, -1) for c in cases]), bd) for k in range(4)]
    fw = _t(np.stack([w.reshape(rows, -1) for w in fws]), bd)
    fenc_c = [_t(np.stack([c.fenc_c[k].reshape(crows, -1) for c in cases]), bd) for k in range(len(c0_.fenc_c))]
    ref_c = [_t(np.stack([c.ref_c[k].reshape(crows, -1) for c in cases]), bd) for k in range(len(c0_.ref_c))]
    pos, par, mvc = sc.jobs(W // 16, H // 16, nframes, i_pixel, seed=seed + subme)
    cm, c0 = rc.cost_mv()
    cmd = torch.from_numpy(cm.view(np.int16)).cuda()
    ext = hip.refine_ext(chroma, cf, 0, weights, fenc_chroma=fenc_c, fenc_chroma_origin=c0_.co,
                         fenc_chroma_stride=c0_.cs, ref_chroma=ref_c, ref_chroma_origin=c0_.co,
                         ref_chroma_stride=c0_.cs)
    ne = torch.full((len(pos), 2), -1, dtype=torch.int32, device="cuda")
    got = hip.me_search_ref(fenc, c0_.origin, c0_.stride, fw, luma, c0_.origin, c0_.stride, i_pixel, me_method, subme,
                            me_range, torch.from_numpy(pos).cuda(), torch.from_numpy(par).cuda(),
                            torch.from_numpy(mvc).cuda(), (cmd, c0), nevals=ne, ext=ext).cpu().numpy()
    ne = ne.cpu().numpy()
    oext = oracle.refine_ext(chroma, cf, 0, weights)
    for f, c in enumerate(cases):
        sel = pos[:, 0] == f
        want, wne = oracle.me_search_ref(bd, c.fenc_y, c.origin, c.stride, c.luma, fws[f].ravel(), c.origin, c.stride,
                                         i_pixel, me_method, subme, me_range, pos[sel, 1:], par[sel], mvc[sel], cm, c0,
                                         ext=oext, fenc_c=c.fenc_c, fc_origin=c.co, fcs=c.cs, ref_c=c.ref_c,
                                         rc_origin=c.co, rcs=c.cs)
        bad = np.argwhere((got[sel] != want).any(1)).ravel()
        assert not len(bad), (f, bad[:4], got[sel][bad[:4]], want[bad[:4]])
        badn = np.argwhere((ne[sel] != wne).any(1)).ravel()
        assert not len(badn), (f, badn[:4], ne[sel][badn[:4]], wne[badn[:4]])
    return got, par, ne


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("me_method", [0, 1, 2, 3])
@pytest.mark.parametrize("i_pixel", [0, 1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("subme,fade,chroma", [(1, 0, 0), (2, 0, 0), (4, 1, 0), (7, 0, 1), (9, 1, 1)])
def test_search_small(hip, oracle, bd, me_method, i_pixel, subme, fade, chroma):
    _run(hip, oracle, bd, 1, 96, 64, 2, i_pixel, me_method, subme, 24 if subme == 9 else 16, fade, chroma,
         seed=bd + 5 * i_pixel + me_method)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("me_method,i_pixel", [(1, 0), (2, 0), (1, 3), (1, 6), (2, 6), (2, 4), (3, 0), (3, 3)])
def test_search_1080p(hip, oracle, bd, me_method, i_pixel):
    """every partition of a 1920x1088 frame pair at x264's default settings (HEX, subme 7, chroma ME
    on P slices) and UMH"""
    got, par, ne = _run(hip, oracle, bd, 1, 1920, 1088, 1, i_pixel, me_method, 7, 16, 0, 1, seed=61 + bd)
    assert (got[:, 1:3] != 0).any(1).mean() > 0.5                       # the searches found the motion


def test_search_args(hip):
    t = torch.zeros(64, dtype=torch.int32, device="cuda")
    p = torch.zeros((2, 160, 256), dtype=torch.uint8, device="cuda")
    pos = torch.zeros((1, 3), dtype=torch.int32, device="cuda")
    par = torch.zeros((1, 12), dtype=torch.int16, device="cuda")
    mvc = torch.zeros((1, 14, 2), dtype=torch.int16, device="cuda")
    for i_pixel, me, subme, rng in ((7, 1, 7, 16), (0, 4, 7, 16), (0, 1, 0, 16), (0, 1, 7, 2), (0, 1, 7, 65)):
        with pytest.raises(RuntimeError):
            hip.me_search_ref(p, 32 * 256 + 32, 256, p, [p, p, p, p], 32 * 256 + 32, 256, i_pixel, me, subme, rng,
                              pos, par, mvc, (t.view(torch.int16), 0))


@pytest.mark.parametrize("bd,me_method", [(8, 1), (10, 2)])
def test_search_2160p(hip, oracle, bd, me_method):
    """every 16x16 partition of a 3840x2160 frame pair (configs[3]'s frame size): HEX at 8 bit,
    UMH at 10 bit, subme 7 with chroma ME"""
    got, par, ne = _run(hip, oracle, bd, 1, 3840, 2160, 1, 0, me_method, 7, 16, 0, 1, seed=71 + bd)
    assert (got[:, 1:3] != 0).any(1).mean() > 0.5


INT_MAX = (1 << 31) - 1


def _chain(hip, oracle, bd, W, H, i_pixel, me_method, subme, seed, nref=3):
    """x264's default ref = 3 loop (analyse.c:1260-1314): one launch per reference with the
    partition's p_halfpel_thresh chained through them and the i_ref_cost adjustments, the HIP
    threshold / outputs / call counts against the oracle's after every reference; returns how
    many partitions took the early exit"""
    cf = 1
    mr = sc.MultiRef(bd, W, H, cf, seed=seed)
    rows = mr.fenc_y.size // mr.stride
    crows = mr.fenc_c[0].size // mr.cs
    fenc = _t(mr.fenc_y.reshape(1, rows, -1), bd)
    fenc_c = [_t(mr.fenc_c[0].reshape(1, crows, -1), bd)]
    cm, c0 = rc.cost_mv()
    cmd = torch.from_numpy(cm.view(np.int16)).cuda()
    oext = oracle.refine_ext(1, cf, 0, (None, None, None))
    n = len(mr.jobs(0, i_pixel, 0)[0])
    thr = np.full(n, INT_MAX, np.int32)
    thr_d = torch.from_numpy(thr.copy()).cuda()
    early = 0
    for k in range(nref):
        r = mr.refs[k]
        luma = [_t(p.reshape(1, rows, -1), bd) for p in r.luma]
        ref_c = [_t(r.ref_c[0].reshape(1, crows, -1), bd)]
        ext = hip.refine_ext(1, cf, 0, (None, None, None), fenc_chroma=fenc_c, fenc_chroma_origin=mr.co,
                             fenc_chroma_stride=mr.cs, ref_chroma=ref_c, ref_chroma_origin=mr.co,
                             ref_chroma_stride=mr.cs)
        pos, par, mvc = mr.jobs(k, i_pixel, seed=seed + 17 * k)
        rcost = np.full(n, 40 if k == 0 else 120, np.int32)
        out = torch.full((n, 4), -7, dtype=torch.int32, device="cuda")
        ne = torch.full((n, 2), -1, dtype=torch.int32, device="cuda")
        hip.me_search_ref(fenc, mr.origin, mr.stride, luma[0], luma, mr.origin, mr.stride, i_pixel, me_method, subme,
                          16, torch.from_numpy(pos).cuda(), torch.from_numpy(par).cuda(), torch.from_numpy(mvc).cuda(),
                          (cmd, c0), out=out, nevals=ne, ext=ext, halfpel_thresh=thr_d,
                          ref_cost=torch.from_numpy(rcost).cuda())
        want, wne = oracle.me_search_ref(bd, mr.fenc_y, mr.origin, mr.stride, r.luma, r.luma[0], mr.origin, mr.stride,
                                         i_pixel, me_method, subme, 16, pos[:, 1:], par, mvc, cm, c0, ext=oext,
                                         fenc_c=mr.fenc_c, fc_origin=mr.co, fcs=mr.cs, ref_c=r.ref_c, rc_origin=mr.co,
                                         rcs=mr.cs, thresh=thr, ref_cost=rcost, out_fill=-7)
        got = out.cpu().numpy()
        bad = np.argwhere((got != want).any(1)).ravel()
        assert not len(bad), (k, bad[:4], got[bad[:4]], want[bad[:4]])
        ne = ne.cpu().numpy()
        badn = np.argwhere((ne != wne).any(1)).ravel()
        assert not len(badn), (k, badn[:4], ne[badn[:4]], wne[badn[:4]])
        assert np.array_equal(thr_d.cpu().numpy(), thr), k
        early += int((want[:, 3] == -7).sum())
    return early, n


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("me_method", [1, 2])
@pytest.mark.parametrize("i_pixel", [0, 3])
def test_search_thresh_chain_small(hip, oracle, bd, me_method, i_pixel):
    early, n = _chain(hip, oracle, bd, 96, 64, i_pixel, me_method, 7, seed=5 + bd + me_method)
    assert early > 0


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("me_method", [1, 2])
def test_search_thresh_chain_1080p(hip, oracle, bd, me_method):
    """x264's default P16x16 path (ref 3, b_early_terminate, HEX or UMH, subme 7, chroma ME) over
    a whole 1920x1088 frame"""
    early, n = _chain(hip, oracle, bd, 1920, 1088, 0, me_method, 7, seed=31 + bd)
    assert 0 < early < 2 * n


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("subme", [2, 5, 7, 9])
def test_refdupe(hip, oracle, bd, subme):
    """x264_me_refine_qpel_refdupe (me.c:812-815) on a reference duplicating reference 0
    (analyse.c:1279-1283), after reference 0's search with the threshold"""
    W, H, cf, i_pixel = 96, 64, 1, 0
    mr = sc.MultiRef(bd, W, H, cf, seed=9 + bd)
    rows, crows = mr.fenc_y.size // mr.stride, mr.fenc_c[0].size // mr.cs
    r = mr.refs[0]
    fenc = _t(mr.fenc_y.reshape(1, rows, -1), bd)
    luma = [_t(p.reshape(1, rows, -1), bd) for p in r.luma]
    chroma = int(subme >= 5)
    ext = hip.refine_ext(chroma, cf, 0, (None, None, None), fenc_chroma=[_t(mr.fenc_c[0].reshape(1, crows, -1), bd)],
                         fenc_chroma_origin=mr.co, fenc_chroma_stride=mr.cs,
                         ref_chroma=[_t(r.ref_c[0].reshape(1, crows, -1), bd)], ref_chroma_origin=mr.co,
                         ref_chroma_stride=mr.cs)
    oext = oracle.refine_ext(chroma, cf, 0, (None, None, None))
    cm, c0 = rc.cost_mv()
    cmd = torch.from_numpy(cm.view(np.int16)).cuda()
    pos, par, mvc = mr.jobs(0, i_pixel, seed=subme)
    n = len(pos)
    thr = np.full(n, INT_MAX, np.int32)
    rc0 = np.full(n, 40, np.int32)
    out0, _ = oracle.me_search_ref(bd, mr.fenc_y, mr.origin, mr.stride, r.luma, r.luma[0], mr.origin, mr.stride,
                                   i_pixel, 1, subme, 16, pos[:, 1:], par, mvc, cm, c0, ext=oext, fenc_c=mr.fenc_c,
                                   fc_origin=mr.co, fcs=mr.cs, ref_c=r.ref_c, rc_origin=mr.co, rcs=mr.cs, thresh=thr,
                                   ref_cost=rc0)
    rpar = np.stack([out0[:, 1], out0[:, 2], par[:, 0] + 4, par[:, 1] - 4, par[:, 6], par[:, 7], par[:, 8], par[:, 9]],
                    1).astype(np.int16)
    init = (out0[:, 0] + rc0).astype(np.int32)
    rc1 = np.full(n, 120, np.int32)
    thr_d = torch.from_numpy(thr.copy()).cuda()
    out = torch.full((n, 4), -7, dtype=torch.int32, device="cuda")
    ne = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    hip.me_refine_qpel_refdupe(fenc, mr.origin, mr.stride, luma, mr.origin, mr.stride, i_pixel, subme,
                               torch.from_numpy(pos).cuda(), torch.from_numpy(rpar).cuda(),
                               torch.from_numpy(init).cuda(), (cmd, c0), halfpel_thresh=thr_d,
                               ref_cost=torch.from_numpy(rc1).cuda(), out=out, nevals=ne, ext=ext)
    want, wne = oracle.me_refine_qpel_refdupe(bd, mr.fenc_y, mr.origin, mr.stride, r.luma, mr.origin, mr.stride,
                                              i_pixel, subme, pos[:, 1:], rpar, init, cm, c0, thresh=thr,
                                              ref_cost=rc1, out_fill=-7, ext=oext, fenc_c=mr.fenc_c, fc_origin=mr.co,
                                              fcs=mr.cs, ref_c=r.ref_c, rc_origin=mr.co, rcs=mr.cs)
    assert np.array_equal(out.cpu().numpy(), want)
    assert np.array_equal(ne.cpu().numpy(), wne)
    assert np.array_equal(thr_d.cpu().numpy(), thr)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("i_pixel", [0, 3])
@pytest.mark.parametrize("subme", [1, 7])
def test_search_umh_cross_past_limit(hip, oracle, bd, i_pixel, subme):
    """UMH's CROSS range-checks only the axis it moves along (me.c:152-176): with mv_limit_fpel's
    max one pixel short of the true motion (3, 2) the predictors clip to the limit, DIA1_ITER
    scores the true match one step past it unchecked (me.c:146-150), and the crosses around that
    winner run at an out-of-range omx / omy -- the reference scores those points"""
    W, H, cf = 96, 64, 1
    cc = rc.ChromaCase(bd, W, H, cf, seed=13 + bd)
    pos, par, mvc = sc.jobs(W // 16, H // 16, 1, i_pixel, seed=3 + subme)
    par[:, 4] = np.minimum(par[:, 4], 2)                     # fpel x max: true 3
    par[:, 5] = np.minimum(par[:, 5], 1)                     # fpel y max: true 2
    rows, crows = cc.ref.y.shape[0], cc.ref.nv.shape[0]
    fenc = _t(cc.fenc_y.reshape(1, rows, -1), bd)
    luma = [_t(p.reshape(1, rows, -1), bd) for p in cc.luma]
    chroma = int(subme >= 5)
    ext = hip.refine_ext(chroma, cf, 0, (None, None, None), fenc_chroma=[_t(cc.fenc_c[0].reshape(1, crows, -1), bd)],
                         fenc_chroma_origin=cc.co, fenc_chroma_stride=cc.cs,
                         ref_chroma=[_t(cc.ref_c[0].reshape(1, crows, -1), bd)], ref_chroma_origin=cc.co,
                         ref_chroma_stride=cc.cs)
    cm, c0 = rc.cost_mv()
    cmd = torch.from_numpy(cm.view(np.int16)).cuda()
    ne = torch.full((len(pos), 2), -1, dtype=torch.int32, device="cuda")
    got = hip.me_search_ref(fenc, cc.origin, cc.stride, luma[0], luma, cc.origin, cc.stride, i_pixel, 2, subme, 16,
                            torch.from_numpy(pos).cuda(), torch.from_numpy(par).cuda(), torch.from_numpy(mvc).cuda(),
                            (cmd, c0), nevals=ne, ext=ext).cpu().numpy()
    want, wne = oracle.me_search_ref(bd, cc.fenc_y, cc.origin, cc.stride, cc.luma, cc.luma[0], cc.origin, cc.stride,
                                     i_pixel, 2, subme, 16, pos[:, 1:], par, mvc, cm, c0,
                                     ext=oracle.refine_ext(chroma, cf, 0, (None, None, None)), fenc_c=cc.fenc_c,
                                     fc_origin=cc.co, fcs=cc.cs, ref_c=cc.ref_c, rc_origin=cc.co, rcs=cc.cs)
    bad = np.argwhere((got != want).any(1)).ravel()
    assert not len(bad), (bad[:4], got[bad[:4]], want[bad[:4]])
    assert np.array_equal(ne.cpu().numpy(), wne)
    if subme == 1:                                           # integer winners past the limit exist
        assert ((want[:, 1] == 12) | (want[:, 2] == 8)).any()
