"""GPU parity: x264's P16x16 reference-0 analysis with the encoder's own predictors
(x264hip_*_me_analyse_p16x16: mvp = x264_mb_predict_mv_16x16, mvc = x264_mb_predict_mv_ref16x16,
the limits of analyse.c:330-349, x264_me_search_ref; reference common/mvpred.c:129-157, 519-600)
against the raster loop of tests/mvpred_cases.py over the oracle's me_search_ref, bit-exact in
results and call counts: the wavefront of MB anti-diagonals must reproduce every MB's predictors
from its decided neighbours."""
import numpy as np
import pytest
import torch

import mvpred_cases as mp
import refine_cases as rc

pytestmark = pytest.mark.gpu


def _t(a, bd):
    a = np.ascontiguousarray(a)
    return torch.from_numpy(a.view(np.int16) if bd == 10 else a).cuda()


def _run(hip, oracle, bd, W, H, nframes, me_method, subme, me_range, chroma, seed, mv_range=512, lowres=False,
         temporal=False):
    cf = 1
    cases = [rc.ChromaCase(bd, W, H, cf, seed=seed + 11 * k) for k in range(nframes)]
    c0_ = cases[0]
    rows = c0_.ref.y.shape[0]
    crows = c0_.ref.nv.shape[0]
    fenc = _t(np.stack([c.fenc_y.reshape(rows, -1) for c in cases]), bd)
    luma = [_t(np.stack([c.luma[k].reshape(rows, -1) for c in cases]), bd) for k in range(4)]
    fenc_c = [_t(np.stack([c.fenc_c[k].reshape(crows, -1) for c in cases]), bd) for k in range(len(c0_.fenc_c))]
    ref_c = [_t(np.stack([c.ref_c[k].reshape(crows, -1) for c in cases]), bd) for k in range(len(c0_.ref_c))]
    mbw, mbh = W // 16, H // 16
    nmb = mbw * mbh
    rs = np.random.default_rng(seed)
    lr = tm = None
    if lowres:
        lr = rs.integers(-200, 200, (nframes, nmb, 2)).astype(np.int16)
        lr[-1, 0, 0] = 0x7fff                           # the last frame has no lowres field
    if temporal:
        tm = rs.integers(-90, 90, (nframes, nmb, 2)).astype(np.int16)
    tscale = 384 if temporal else 0
    cm, c0 = rc.cost_mv()
    cmd = torch.from_numpy(cm.view(np.int16)).cuda()
    ext = hip.refine_ext(chroma, cf, 0, (None, None, None), fenc_chroma=fenc_c, fenc_chroma_origin=c0_.co,
                         fenc_chroma_stride=c0_.cs, ref_chroma=ref_c, ref_chroma_origin=c0_.co,
                         ref_chroma_stride=c0_.cs)
    ne = torch.full((nframes, nmb, 2), -1, dtype=torch.int32, device="cuda")
    got = hip.me_analyse_p16x16(fenc, c0_.origin, c0_.stride, luma[0], luma, c0_.origin, c0_.stride, mbw, mbh, nframes,
                                me_method, subme, me_range, (cmd, c0), mv_range=mv_range,
                                lowres_mv=None if lr is None else torch.from_numpy(lr).cuda(),
                                ref_mv=None if tm is None else torch.from_numpy(tm).cuda(), ref_mv_scale=tscale,
                                nevals=ne, ext=ext).cpu().numpy()
    ne = ne.cpu().numpy()
    oext = oracle.refine_ext(chroma, cf, 0, (None, None, None))
    for f, c in enumerate(cases):
        def search(x, y, par, mvc, c=c):
            o, n = oracle.me_search_ref(bd, c.fenc_y, c.origin, c.stride, c.luma, c.luma[0].ravel(), c.origin,
                                        c.stride, 0, me_method, subme, me_range, np.array([[16 * x, 16 * y]]),
                                        par[None], mvc[None], cm, c0, ext=oext, fenc_c=c.fenc_c, fc_origin=c.co,
                                        fcs=c.cs, ref_c=c.ref_c, rc_origin=c.co, rcs=c.cs)
            return o[0], n[0]
        want, wne = mp.analyse_p16x16(search, mbw, mbh, mv_range, None if lr is None else lr[f],
                                      None if tm is None else tm[f], tscale)
        bad = np.argwhere((got[f] != want).any(1)).ravel()
        assert not len(bad), (f, bad[:4], got[f][bad[:4]], want[bad[:4]])
        badn = np.argwhere((ne[f] != wne).any(1)).ravel()
        assert not len(badn), (f, badn[:4], ne[f][badn[:4]], wne[badn[:4]])
    return got


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("me_method,subme", [(0, 4), (1, 7), (2, 7), (1, 1)])
def test_analyse_p16x16(hip, oracle, bd, me_method, subme):
    got = _run(hip, oracle, bd, 112, 80, 2, me_method, subme, 16, subme >= 5, seed=3 + me_method + bd)
    assert (got[..., 1:3] != 0).any(-1).mean() > 0.5


@pytest.mark.parametrize("lowres,temporal", [(True, False), (False, True), (True, True)])
def test_analyse_p16x16_predictor_sources(hip, oracle, lowres, temporal):
    """the lookahead's lowres mv and the reference's temporal mvs in the candidate list"""
    _run(hip, oracle, 8, 96, 64, 2, 1, 7, 16, 1, seed=17, lowres=lowres, temporal=temporal)


def test_analyse_p16x16_mv_range(hip, oracle):
    """a small i_mv_range clamps the spel limits (analyse.c:336-339) on a wide frame"""
    _run(hip, oracle, 8, 160, 48, 1, 2, 7, 16, 0, seed=23, mv_range=40)


@pytest.mark.parametrize("W,H", [(16, 64), (96, 16), (16, 16)])
def test_analyse_p16x16_degenerate_shapes(hip, oracle, W, H):
    """one MB column (every diagonal a single MB, C always off the frame), one MB row (A only),
    a single MB"""
    _run(hip, oracle, 8, W, H, 2, 1, 7, 16, 0, seed=29 + W + H)
