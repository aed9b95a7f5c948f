"""The oracle's refine_subpel with chroma ME and weighted references (oracle.c
FN(me_refine_subpel_ex): COST_MV_SATD's b_chroma_me branch, reference encoder/me.c:826-863,
872-875, 925-929, with get_ref / mc_chroma / mc_weight, common/mc.c:117-137, 221-283) against a
literal Python restatement built from numpy_ref.py's get_ref / SAD / SATD and an independent
numpy mc_chroma: 4:2:0, 4:2:2 and 4:4:4, every partition 16x16 .. 8x8, subme 5 / 7 / 9 (chroma
ME needs subme >= 5, common/macroblock.c:507-509), both iteration sets, unweighted and
weighted (denom 0 too), 8 and 10 bit, with the reference's cmp-call counts."""
import numpy as np
import pytest

import numpy_ref as nr
import refine_cases as rc
from test_cpu_refine import SUBPEL_ITERATIONS, _s32


def _weigh(a, w, bd):
    """mc_weight (mc.c:117-137) of an int64 block; w = (scale, denom, offset) or None"""
    if w is None:
        return a
    s, d, o = w
    o <<= bd - 8
    v = ((a * s + (1 << (d - 1))) >> d) + o if d >= 1 else a * s + o
    return np.clip(v, 0, (1 << bd) - 1)


def _mc_chroma(nv, off, stride, mvx, mvy, w, h):
    """mc_chroma (mc.c:252-283) of the interleaved plane at element offset off: (u, v) int64"""
    dx, dy = mvx & 7, mvy & 7
    base = off + (mvy >> 3) * stride + (mvx >> 3) * 2
    s = nv[base + np.arange(h + 1)[:, None] * stride + np.arange(2 * w + 2)[None, :]].astype(np.int64)
    out = []
    for p in (0, 1):
        a, b = s[:h, p:p + 2 * w:2], s[:h, p + 2:p + 2 * w + 2:2]
        c, d = s[1:, p:p + 2 * w:2], s[1:, p + 2:p + 2 * w + 2:2]
        out.append(((8 - dx) * (8 - dy) * a + dx * (8 - dy) * b + (8 - dx) * dy * c + dx * dy * d + 32) >> 6)
    return out


def refine_chroma_py(cc, x, y, i_pixel, par, cost, cm, c0, subme, refine_qpel, b_chroma_me, weights, mvy_offset=0,
                     refdupe=False, thresh=None, ref_cost=0):
    """refine_subpel (me.c:865-992) with COST_MV_SATD's chroma branch; returns (cost, mvx, mvy,
    cost_mv) and the call counts (sad, satd, chroma).  refdupe: x264_me_refine_qpel_refdupe's
    iterations (me.c:812-815); thresh: a one-element list holding *p_halfpel_thresh (me.c:931-944),
    updated, with ref_cost subtracted around the call as analyse.c:1271 / 1310 do -- on the early
    exit cost_mv is None (m->cost_mv untouched)"""
    bd, cf = cc.bd, cc.cf
    bw, bh = nr.SIZES[i_pixel]
    qsatd = subme > 1
    st, org = cc.stride, cc.origin
    fb = nr.block(cc.fenc_y, org + y * st + x, st, bw, bh)
    n = [0, 0, 0]

    def luma(satd, mx, my):
        r = _weigh(nr.get_ref(cc.luma, org + y * st + x, st, mx, my, bw, bh), weights[0], bd)
        n[1 if satd else 0] += 1
        return nr.satd(fb, r) if satd else nr.sad(fb, r)

    def chroma(mx, my, cost, bcost):
        cmp = nr.satd if qsatd else nr.sad
        if cf == 3:
            for p in (0, 1):
                if not cost < bcost:
                    break
                r = _weigh(nr.get_ref(cc.ref_c[4 * p:4 * p + 4], cc.co + y * cc.cs + x, cc.cs, mx, my, bw, bh),
                           weights[1 + p], bd)
                cost += cmp(nr.block(cc.fenc_c[p], cc.co + y * cc.cs + x, cc.cs, bw, bh), r)
                n[2] += 1
            return cost
        vs = 1 if cf == 1 else 0
        cw, ch = bw >> 1, bh >> vs
        off = cc.co + (y >> vs) * cc.cs + x
        pu_pv = _mc_chroma(cc.ref_c[0], off, cc.cs, mx, (2 * (my + mvy_offset)) >> vs, cw, ch)
        fe = nr.block(cc.fenc_c[0], off, cc.cs, 2 * cw, ch)
        for p in (0, 1):
            if not cost < bcost:
                break
            cost += cmp(fe[:, p::2], _weigh(pu_pv[p], weights[1 + p], bd))
            n[2] += 1
        return cost

    mvp = (int(par[2]), int(par[3]))
    cmx = lambda v: int(cm[c0 + v - mvp[0]])
    cmy = lambda v: int(cm[c0 + v - mvp[1]])

    b_chroma_me = b_chroma_me and (i_pixel <= 3 or cf == 3)          # me.c:872

    def satd_cost(mx, my, bcost):
        c = luma(qsatd, mx, my) + cmx(mx) + cmy(my)
        if b_chroma_me and c < bcost:
            c = chroma(mx, my, c, bcost)
        return c

    mn, mx_ = (int(par[4]), int(par[5])), (int(par[6]), int(par[7]))
    hpel = 0 if refdupe else SUBPEL_ITERATIONS[subme][0 if refine_qpel else 2]
    qpel = min(2, SUBPEL_ITERATIONS[subme][3]) if refdupe else SUBPEL_ITERATIONS[subme][1 if refine_qpel else 3]
    bmx, bmy, bcost = int(par[0]), int(par[1]), int(cost)
    if hpel:
        if subme < 3:                                       # the predictor's subpel component (me.c:889-895)
            px = min(max(mvp[0], mn[0] + 2), mx_[0] - 2)
            py = min(max(mvp[1], mn[1] + 2), mx_[1] - 2)
            if (px - bmx) | (py - bmy):
                c = luma(False, px, py) + cmx(px) + cmy(py)
                if c < bcost:
                    bcost, bmx, bmy = c, px, py
        bcost = _s32(bcost << 6)
        for _ in range(hpel):
            omx, omy = bmx, bmy
            for qx, qy, code in ((omx, omy - 2, 2), (omx, omy + 2, 6), (omx - 2, omy, 16), (omx + 2, omy, 48)):
                c = _s32((luma(False, qx, qy) + cmx(qx) + cmy(qy)) << 6) + code
                if c < bcost:
                    bcost = c
            if not bcost & 63:
                break
            bmx -= _s32((bcost << 26) & 0xFFFFFFFF) >> 29
            bmy -= _s32((bcost << 29) & 0xFFFFFFFF) >> 29
            bcost &= ~63
        bcost >>= 6
    if not refine_qpel and (qsatd or b_chroma_me):
        bcost = satd_cost(bmx, bmy, 1 << 28)
    if thresh is not None:
        t = thresh[0] - ref_cost
        early = (bcost * 7) >> 3 > t
        if not early and bcost < t:
            t = bcost
        thresh[0] = t + ref_cost
        if early:
            return (bcost, bmx, bmy, None), n[0] | (n[1] << 16) | (n[2] << 24)
    bdir = -1
    for _ in range(qpel):
        if bmy <= mn[1] or bmy >= mx_[1] or bmx <= mn[0] or bmx >= mx_[0]:
            break
        odir = bdir
        omx, omy = bmx, bmy
        for d, (dx, dy) in enumerate(((0, -1), (0, 1), (-1, 0), (1, 0))):
            if not refine_qpel and (d ^ 1) == odir:
                continue
            c = satd_cost(omx + dx, omy + dy, bcost)
            if c < bcost:
                bcost, bmx, bmy, bdir = c, omx + dx, omy + dy, d
        if bmx == omx and bmy == omy:
            break
    return (bcost, bmx, bmy, cmx(bmx) + cmy(bmy)), n[0] | (n[1] << 16) | (n[2] << 24)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("cf", [1, 2, 3])
@pytest.mark.parametrize("i_pixel", [0, 1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("subme,refine_qpel,b_chroma_me,wsel", [(7, 0, 1, 0), (5, 0, 1, 1), (9, 0, 1, 2),
                                                                (5, 1, 1, 1), (7, 0, 0, 1)])
def test_refine_chroma_oracle_vs_python(oracle, bd, cf, i_pixel, subme, refine_qpel, b_chroma_me, wsel):
    W, H = 48, 32
    cc = rc.ChromaCase(bd, W, H, cf, seed=bd + cf + i_pixel, fade=wsel > 0)
    weights = (None, None, None) if wsel == 0 else rc.FADE_WEIGHTS if wsel == 1 else rc.FADE_WEIGHTS_DENOM0
    pos, par, cost = rc.jobs(W // 16, H // 16, 1, i_pixel, seed=subme * 7 + bd + cf,
                       cost_scale=(1 << (bd - 8)) * (16 if refine_qpel else 1))
    cm, c0 = rc.cost_mv()
    ext = oracle.refine_ext(b_chroma_me, cf, 0, weights)
    got, ne = oracle.me_refine_subpel(bd, cc.fenc_y, cc.origin, cc.stride, cc.luma, cc.origin, cc.stride, i_pixel,
                                      subme, pos[:, 1:], par, cost, cm, c0, refine_qpel, False, counts=True, ext=ext,
                                      fenc_c=cc.fenc_c, fc_origin=cc.co, fcs=cc.cs, ref_c=cc.ref_c, rc_origin=cc.co,
                                      rcs=cc.cs)
    moved = 0
    for i in range(len(pos)):
        want, wn = refine_chroma_py(cc, int(pos[i, 1]), int(pos[i, 2]), i_pixel, par[i], cost[i], cm, c0, subme,
                                    refine_qpel, b_chroma_me, weights)
        assert tuple(got[i]) == want and ne[i] == wn, (i, got[i], want, hex(ne[i]), hex(wn))
        moved += (want[1], want[2]) != (int(par[i, 0]), int(par[i, 1]))
    if b_chroma_me and (i_pixel <= 3 or cf == 3):            # me.c:872
        assert (ne >> 24).sum() > 0                        # the chroma branch ran
    elif b_chroma_me:
        assert not (ne >> 24).any()                        # sub-8x8 at 4:2:0 / 4:2:2: no chroma ME


def test_refine_chroma_changes_decisions(oracle):
    """chroma ME is not a no-op on this content: some 1080p-shaped partitions end elsewhere (or
    at another cost) with it than without it"""
    bd, cf, W, H = 8, 1, 96, 64
    cc = rc.ChromaCase(bd, W, H, cf, seed=5)
    pos, par, cost = rc.jobs(W // 16, H // 16, 1, 0, seed=11)
    cm, c0 = rc.cost_mv()
    res = []
    for b in (0, 1):
        res.append(oracle.me_refine_subpel(bd, cc.fenc_y, cc.origin, cc.stride, cc.luma, cc.origin, cc.stride, 0, 7,
                                           pos[:, 1:], par, cost, cm, c0, ext=oracle.refine_ext(b, cf),
                                           fenc_c=cc.fenc_c, fc_origin=cc.co, fcs=cc.cs, ref_c=cc.ref_c,
                                           rc_origin=cc.co, rcs=cc.cs))
    assert (res[0][:, 1:3] != res[1][:, 1:3]).any()
