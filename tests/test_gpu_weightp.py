"""GPU parity: the weighted-prediction analysis (x264hip_*_weight_cost_batch, _frame_pixel_stats,
_weights_analyse; reference encoder/slicetype.c:63-501, encoder/ratecontrol.c:225-257,
406-414) against the oracle: every candidate cost of every kind (luma lowres with and without
lowres mvs, SATD and SAD; 4:2:0 / 4:2:2 asd8 with and without mc_chroma; 4:4:4 with full-pel
copies), the frame statistics in every chroma format (the uint32 sum wrap included), and the
chosen weights -- lookahead and encode modes, subme 2..11 distances, the FAKE cost delta, the
chroma break and the offset clamp -- with the lookahead's weighted lowres plane."""
import numpy as np
import pytest
import torch

import weightp_cases as wc
from test_cpu_weightp import CASES

pytestmark = pytest.mark.gpu


def _dev(a):
    a = np.ascontiguousarray(a)
    return torch.from_numpy(a.view(np.int16) if a.dtype == np.uint16 else a).cuda()


def _u32(t):
    return t.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("kind,cf", [(0, 0), (1, 1), (2, 2), (3, 3)])
@pytest.mark.parametrize("with_mvs", [False, True])
@pytest.mark.parametrize("satd", [True, False])
@pytest.mark.parametrize("size", [(176, 144), (1920, 1088)])
def test_weight_cost_batch(hip, oracle, bd, kind, cf, with_mvs, satd, size):
    if kind in (1, 2) and not satd:
        pytest.skip("asd8 has no mbcmp choice")
    if size[0] > 176 and (not satd or bd == 10):
        pytest.skip("one 1080p pass per kind and mv mode")
    W, H = size
    ref, fenc = wc.make_pair(bd, W, H, cf, (1.1, -6), ((0.9, 4), (1.2, -3)), seed=bd + kind + W)
    an = wc.Analysis(oracle, ref, fenc, satd=satd, search_mvs=False)
    mvs = wc.random_mvs(an.mbw, an.mbh, 5 + kind) if with_mvs else None
    cands = wc.candidates(bd * 10 + kind + W, n=70)                      # two launches of 64 + 6
    dmvs = None if mvs is None else _dev(mvs)
    for plane in ((0, 1) if kind in (1, 2) else (0,)):
        if kind == 0:
            f, r, o, s = an.fenc_lr[0], an.ref_lr, an.lo, an.ls
            got = hip.weight_cost_batch(0, _dev(f), [_dev(p) for p in r], o, s, an.mbw, an.mbh, cands,
                                        intra_cost=_dev(an.intra), mvs=dmvs, satd=satd, lam=3, n_slices=2)
            want = oracle.weight_cost_list(bd, 0, f.ravel(), [p.ravel() for p in r], o, s, an.mbw, an.mbh, cands,
                                           intra=an.intra, mvs=mvs, satd=satd, lam=3, n_slices=2)
        else:
            f, r = (fenc.nv, ref.nv) if kind in (1, 2) else (fenc.u, ref.u)
            s = f.shape[1]
            o = 32 * s + 32
            got = hip.weight_cost_batch(kind, _dev(f), [_dev(r)], o, s, an.mbw, an.mbh, cands, mvs=dmvs, satd=satd,
                                        plane=plane, lam=3, n_slices=2)
            want = oracle.weight_cost_list(bd, kind, f.ravel(), [r.ravel()], o, s, an.mbw, an.mbh, cands, mvs=mvs,
                                           satd=satd, plane=plane, lam=3, n_slices=2)
        got = _u32(got)
        bad = np.flatnonzero(got != want)
        assert not len(bad), (plane, bad[:6], got[bad[:6]], want[bad[:6]], [cands[i] for i in bad[:6]])


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("cf", [0, 1, 2, 3])
@pytest.mark.parametrize("size", [(64, 48), (1920, 1088)])
def test_frame_pixel_stats(hip, oracle, bd, cf, size):
    W, H = size
    ref, fenc = wc.make_pair(bd, W, H, cf, (1.2, 7), ((0.8, 3), (1.1, -2)), seed=cf + W)
    mbw, mbh = W // 16, H // 16
    for fr in (ref, fenc):
        ch = fr.chroma()
        got = hip.frame_pixel_stats(_dev(fr.y), fr.yo, fr.ys, mbw, mbh, cf,
                                    None if ch[0] is None else _dev(ch[0]), None if ch[1] is None else _dev(ch[1]),
                                    fr.co, fr.cs).cpu().numpy().view(np.uint64)
        planes = [fr.y.ravel()] + [None if c is None else c.ravel() for c in ch]
        s, d = oracle.frame_pixel_stats(bd, planes, [fr.yo, fr.co, fr.co], [fr.ys, fr.cs, fr.cs], mbw, mbh, cf)
        assert got[:3].tolist() == s.astype(np.uint64).tolist() and got[3:].tolist() == d.tolist()


def test_frame_pixel_stats_sum_wrap(hip, oracle):
    """10-bit 4096x2176 near-white: the luma sum passes 2^32 and wraps as the uint32 field does"""
    W, H = 4096, 2176
    rs = np.random.default_rng(5)
    ys = W + 64
    y = np.pad(rs.integers(1000, 1024, size=(H, W)), 32, mode="edge").astype(np.uint16)
    got = hip.frame_pixel_stats(_dev(y), 32 * ys + 32, ys, W // 16, H // 16).cpu().numpy().view(np.uint64)
    s, d = oracle.frame_pixel_stats(10, [y.ravel(), None, None], [32 * ys + 32, 0, 0], [ys, 0, 0], W // 16, H // 16,
                                    0)
    assert int(y[32:-32, 32:-32].astype(np.int64).sum()) > 1 << 32
    assert got[:3].tolist() == s.astype(np.uint64).tolist() and got[3:].tolist() == d.tolist()


def _analyse_both(hip, oracle, bd, ref, fenc, an, cf, bl, subme, fake, lam=3, ns=1):
    wl_gpu = torch.zeros_like(_dev(an.ref_lr[0]))
    wl_ora = np.zeros_like(an.ref_lr[0]).ravel()
    fc, rc = fenc.chroma(), ref.chroma()
    got, gdelta = hip.weights_analyse(
        _dev(an.fenc_lr[0]), [_dev(p) for p in an.ref_lr], an.ls, an.mbw, an.mbh, _dev(an.intra), an.fstats,
        an.rstats, mvs=None if an.mvs is None else _dev(an.mvs), chroma_format=cf,
        fenc_chroma=[None if c is None else _dev(c) for c in fc], ref_chroma=[None if c is None else _dev(c) for c in rc],
        chroma_origin=fenc.co, chroma_stride=fenc.cs, b_lookahead=bl, subme=subme, lam=lam, n_slices=ns,
        weightp_fake=fake, weighted_lowres=wl_gpu)
    want, wdelta = oracle.weights_analyse(
        bd, an.fenc_lr[0].ravel(), [p.ravel() for p in an.ref_lr], an.lo, an.ls, an.mbw, an.mbh, an.intra, an.fstats,
        an.rstats, mvs=an.mvs, chroma_format=cf, fenc_c=[None if c is None else c.ravel() for c in fc],
        ref_c=[None if c is None else c.ravel() for c in rc], c_origin=fenc.co, cs=fenc.cs, b_lookahead=bl,
        subme=subme, lam=lam, n_slices=ns, weightp_fake=fake, weighted=wl_ora)
    assert [list(w) for w in got] == want.tolist()
    assert gdelta == wdelta
    g = wl_gpu.cpu().numpy().ravel()
    if bd == 10:
        g = g.view(np.uint16)
    assert np.array_equal(g, wl_ora)
    return got


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_weights_analyse(hip, oracle, bd, case):
    cf, lf, cfs, bl, subme, with_mvs, fake, flat = CASES[case]
    ref, fenc = wc.make_pair(bd, 64, 48, cf, lf, cfs, seed=11 + case, flat_ref_chroma=flat,
                             shift=(3, 2) if with_mvs else (0, 0))
    an = wc.Analysis(oracle, ref, fenc, search_mvs=with_mvs, intra_scale=1 << (bd - 8))
    _analyse_both(hip, oracle, bd, ref, fenc, an, cf, bl, subme, fake)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("bl,subme,cf", [(True, 7, 0), (False, 11, 1), (False, 9, 3)])
def test_weights_analyse_1080p(hip, oracle, bd, bl, subme, cf):
    """a fade over a 1920x1088 pair: the lookahead's luma-only call (slicetype.c:862, which also
    writes fenc->weighted[0]) and the encoder's call with chroma (slicetype.c:1942)"""
    ref, fenc = wc.make_pair(bd, 1920, 1088, cf, (0.85, 12), ((1.1, -4), (0.9, 6)), seed=40 + bd,
                             shift=(0, 0) if bl else (3, 2))
    an = wc.Analysis(oracle, ref, fenc, search_mvs=not bl, intra_scale=1 << (bd - 8))
    got = _analyse_both(hip, oracle, bd, ref, fenc, an, cf, bl, subme, False, ns=4)
    assert got[0][0] == 1                                                 # a luma weight was found


def test_weights_analyse_args(hip, oracle):
    ref, fenc = wc.make_pair(8, 64, 48, 0, (0.8, 10), seed=3, shift=(0, 0))
    an = wc.Analysis(oracle, ref, fenc, search_mvs=False)
    fl, rl, ic = _dev(an.fenc_lr[0]), [_dev(p) for p in an.ref_lr], _dev(an.intra)
    for kw in ({"subme": 12}, {"subme": -1}, {"chroma_format": 4}, {"n_slices": 0}, {"lam": -1},
               {"chroma_format": 1, "b_lookahead": False}):                # chroma planes missing
        with pytest.raises(RuntimeError):
            hip.weights_analyse(fl, rl, an.ls, an.mbw, an.mbh, ic, an.fstats, an.rstats, **kw)
    with pytest.raises(RuntimeError):                                     # denom 8
        hip.weight_cost_batch(0, fl, rl, an.lo, an.ls, an.mbw, an.mbh, [(1, 1, 8, 0)], intra_cost=ic)
    with pytest.raises(RuntimeError):                                     # no intra cost for luma
        hip.weight_cost_batch(0, fl, rl, an.lo, an.ls, an.mbw, an.mbh, [(1, 1, 0, 0)])
