"""GPU parity: refine_subpel with chroma ME and weighted references (x264hip_*_me_refine_subpel_ex,
reference encoder/me.c:826-863, 872-875, 925-929; get_ref / mc_chroma / mc_weight common/mc.c:117-137,
221-283) against the oracle restatement (tests/test_cpu_refine_chroma.py pins it to a literal
Python restatement): 4:2:0 / 4:2:2 / 4:4:4, every partition 16x16 .. 8x8, subme 5 / 7 / 9 and
x264_me_refine_qpel's iterations, fpelcmp SAD and SATD (TESA), unweighted, weighted and weighted
with denom 0, 8 and 10 bit, two frame pairs per launch (the chroma frame strides), the
reference's cmp-call counts (chroma calls included), and whole 1080p frames at subme 7 with
b_chroma_me -- x264's default P-slice settings."""
import numpy as np
import pytest
import torch

import refine_cases as rc

pytestmark = pytest.mark.gpu


def _t(a, bd):
    a = np.ascontiguousarray(a)
    return torch.from_numpy(a.view(np.int16) if bd == 10 else a).cuda()


def _run(hip, oracle, bd, cf, W, H, nframes, i_pixel, subme, refine_qpel, b_chroma_me, weights, fpel_satd=0,
         seed=1, cost_scale=1):
    cases = [rc.ChromaCase(bd, W, H, cf, seed=seed + 17 * k, fade=any(w is not None for w in weights))
             for k in range(nframes)]
    c0_ = cases[0]
    rows = c0_.ref.y.shape[0]
    crows = (c0_.ref.nv if cf in (1, 2) else c0_.ref.u).shape[0]
    fenc = _t(np.stack([c.fenc_y.reshape(rows, -1) for c in cases]), bd)
    luma = [_t(np.stack([c.luma[k].reshape(rows, -1) for c in cases]), bd) for k in range(4)]
    fenc_c = [_t(np.stack([c.fenc_c[k].reshape(crows, -1) for c in cases]), bd) for k in range(len(c0_.fenc_c))]
    ref_c = [_t(np.stack([c.ref_c[k].reshape(crows, -1) for c in cases]), bd) for k in range(len(c0_.ref_c))]
    mbw, mbh = W // 16, H // 16
    pos, par, cost = rc.jobs(mbw, mbh, nframes, i_pixel, seed + subme, cost_scale=(1 << (bd - 8)) * cost_scale)
    cm, c0 = rc.cost_mv()
    cmd = torch.from_numpy(cm.view(np.int16)).cuda()
    ext = hip.refine_ext(b_chroma_me, cf, 0, weights, fenc_chroma=fenc_c, fenc_chroma_origin=c0_.co,
                         fenc_chroma_stride=c0_.cs, ref_chroma=ref_c, ref_chroma_origin=c0_.co,
                         ref_chroma_stride=c0_.cs)
    ne = torch.full((len(pos),), -1, dtype=torch.int32, device="cuda")
    got = hip.me_refine_subpel(fenc, c0_.origin, c0_.stride, luma, c0_.origin, c0_.stride, i_pixel, subme,
                               torch.from_numpy(pos).cuda(), torch.from_numpy(par).cuda(),
                               torch.from_numpy(cost).cuda(), (cmd, c0), refine_qpel=refine_qpel,
                               fpel_satd=fpel_satd, nevals=ne, ext=ext).cpu().numpy()
    ne = ne.cpu().numpy()
    oext = oracle.refine_ext(b_chroma_me, cf, 0, weights)
    for f, c in enumerate(cases):
        sel = pos[:, 0] == f
        want, wne = oracle.me_refine_subpel(bd, c.fenc_y, c.origin, c.stride, c.luma, c.origin, c.stride, i_pixel,
                                            subme, pos[sel, 1:], par[sel], cost[sel], cm, c0, refine_qpel, fpel_satd,
                                            counts=True, ext=oext, fenc_c=c.fenc_c, fc_origin=c.co, fcs=c.cs,
                                            ref_c=c.ref_c, rc_origin=c.co, rcs=c.cs)
        bad = np.argwhere((got[sel] != want).any(1)).ravel()
        assert not len(bad), (f, bad[:4], got[sel][bad[:4]], want[bad[:4]])
        badn = np.argwhere(ne[sel] != wne).ravel()
        assert not len(badn), (f, badn[:4], [hex(v) for v in ne[sel][badn[:4]]], [hex(v) for v in wne[badn[:4]]])
    return got, par, ne


W_NONE, W_FADE, W_D0 = (None, None, None), rc.FADE_WEIGHTS, rc.FADE_WEIGHTS_DENOM0


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("cf", [1, 2, 3])
@pytest.mark.parametrize("i_pixel", [0, 1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("subme,refine_qpel,b_chroma_me,wsel,fpel_satd", [
    (7, 0, 1, 0, 0), (5, 0, 1, 1, 0), (9, 0, 1, 2, 0), (5, 1, 1, 1, 0), (7, 0, 0, 1, 0), (7, 0, 1, 0, 1)])
def test_refine_chroma_small(hip, oracle, bd, cf, i_pixel, subme, refine_qpel, b_chroma_me, wsel, fpel_satd):
    weights = (W_NONE, W_FADE, W_D0)[wsel]
    got, par, ne = _run(hip, oracle, bd, cf, 96, 64, 2, i_pixel, subme, refine_qpel, b_chroma_me, weights,
                        fpel_satd=fpel_satd, seed=bd + 3 * i_pixel + cf,
                        cost_scale=16 if refine_qpel else 1)
    if b_chroma_me and (i_pixel <= 3 or cf == 3):           # me.c:872
        assert (ne >> 24).sum() > 0                       # the chroma branch ran
    elif b_chroma_me:
        assert not (ne >> 24).any()                       # sub-8x8 at 4:2:0 / 4:2:2: no chroma ME
    if subme >= 5 and not refine_qpel:
        assert (got[:, 1:3] != par[:, :2]).any(1).mean() > 0.02


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("cf,i_pixel", [(1, 0), (1, 3), (3, 0), (1, 6), (3, 5)])
def test_refine_chroma_1080p(hip, oracle, bd, cf, i_pixel):
    """every partition of a 1920x1088 frame pair at subme 7 with b_chroma_me (x264's default P-slice
    settings), x264_me_search_ref's iterations"""
    _run(hip, oracle, bd, cf, 1920, 1088, 1, i_pixel, 7, 0, 1, W_NONE, seed=41 + bd)


def test_refine_chroma_args(hip):
    t = torch.zeros(64, dtype=torch.int32, device="cuda")
    p = torch.zeros((2, 160, 256), dtype=torch.uint8, device="cuda")
    pos = torch.zeros((1, 3), dtype=torch.int32, device="cuda")
    par = torch.zeros((1, 8), dtype=torch.int16, device="cuda")
    bad = [hip.refine_ext(1, 0, fenc_chroma=[p], ref_chroma=[p]),          # chroma format 0 with chroma ME
           hip.refine_ext(1, 1),                                            # no chroma planes
           hip.refine_ext(1, 3, fenc_chroma=[p, p], ref_chroma=[p] * 4),    # 4:4:4 without V's planes
           hip.refine_ext(0, 1, weights=((1, 9, 0), None, None))]           # denom out of range
    for e in bad:
        with pytest.raises(RuntimeError):
            hip.me_refine_subpel(p, 32 * 256 + 32, 256, [p, p, p, p], 32 * 256 + 32, 256, 0, 7, pos, par,
                                 t[:1], (t.view(torch.int16), 0), ext=e)
