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
@pytest.mark.parametrize("me_method", [0, 1, 2])
@pytest.mark.parametrize("i_pixel", [0, 1, 2, 3])
@pytest.mark.parametrize("subme,fade,chroma", [(1, 0, 0), (2, 0, 0), (4, 1, 0), (7, 0, 1), (9, 1, 1)])
def test_search_small(hip, oracle, bd, me_method, i_pixel, subme, fade, chroma):
    _run(hip, oracle, bd, 1, 96, 64, 2, i_pixel, me_method, subme, 24 if subme == 9 else 16, fade, chroma,
         seed=bd + 5 * i_pixel + me_method)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("me_method,i_pixel", [(1, 0), (2, 0), (1, 3)])
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
    for i_pixel, me, subme, rng in ((4, 1, 7, 16), (0, 3, 7, 16), (0, 1, 0, 16), (0, 1, 7, 2), (0, 1, 7, 65)):
        with pytest.raises(RuntimeError):
            hip.me_search_ref(p, 32 * 256 + 32, 256, p, [p, p, p, p], 32 * 256 + 32, 256, i_pixel, me, subme, rng,
                              pos, par, mvc, (t.view(torch.int16), 0))


@pytest.mark.parametrize("bd,me_method", [(8, 1), (10, 2)])
def test_search_2160p(hip, oracle, bd, me_method):
    """every 16x16 partition of a 3840x2160 frame pair (configs[3]'s frame size): HEX at 8 bit,
    UMH at 10 bit, subme 7 with chroma ME"""
    got, par, ne = _run(hip, oracle, bd, 1, 3840, 2160, 1, 0, me_method, 7, 16, 0, 1, seed=71 + bd)
    assert (got[:, 1:3] != 0).any(1).mean() > 0.5
