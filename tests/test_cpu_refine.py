"""The oracle's refine_subpel (oracle.c FN(me_refine_subpel)) against a literal Python
restatement of reference encoder/me.c:865-992 built from the numpy get_ref / SAD / SATD of
numpy_ref.py (an independent matrix-form restatement): every partition of small frames over
subme 1..9, both iteration sets, fpelcmp SAD and SATD, 8 and 10 bit."""
import numpy as np
import pytest

import numpy_ref as nr
import refine_cases as rc

SUBPEL_ITERATIONS = [[0, 0, 0, 0], [1, 1, 0, 0], [0, 1, 1, 0], [0, 2, 1, 0], [0, 2, 1, 1], [0, 2, 1, 2],
                     [0, 0, 2, 2], [0, 0, 2, 2], [0, 0, 4, 10], [0, 0, 4, 10], [0, 0, 4, 10], [0, 0, 4, 10]]


def _s32(v):
    """int32 wrap (the reference's int arithmetic on the packed costs)"""
    return (int(v) + (1 << 31)) % (1 << 32) - (1 << 31)


def refine_py(planes, fenc, origin, stride, x, y, bw, bh, par, cost, cm, c0, subme, refine_qpel, fpel_satd):
    fsatd = fpel_satd and subme > 1
    qsatd = subme > 1
    fb = nr.block(fenc, origin + y * stride + x, stride, bw, bh)

    def cmp(satd, mx, my):
        r = nr.get_ref(planes, origin + y * stride + x, stride, mx, my, bw, bh)
        return nr.satd(fb, r) if satd else nr.sad(fb, r)

    mvp = (int(par[2]), int(par[3]))
    cmx = lambda v: int(cm[c0 + v - mvp[0]])
    cmy = lambda v: int(cm[c0 + v - mvp[1]])
    mn, mx_ = (int(par[4]), int(par[5])), (int(par[6]), int(par[7]))
    hpel = SUBPEL_ITERATIONS[subme][0 if refine_qpel else 2]
    qpel = SUBPEL_ITERATIONS[subme][1 if refine_qpel else 3]
    bmx, bmy, bcost = int(par[0]), int(par[1]), int(cost)
    if hpel:
        if subme < 3:
            px = min(max(mvp[0], mn[0] + 2), mx_[0] - 2)
            py = min(max(mvp[1], mn[1] + 2), mx_[1] - 2)
            if (px - bmx) | (py - bmy):
                c = cmp(fsatd, px, py) + cmx(px) + cmy(py)
                if c < bcost:
                    bcost, bmx, bmy = c, px, py
        bcost = _s32(bcost << 6)
        for _ in range(hpel):
            omx, omy = bmx, bmy
            cands = [(omx, omy - 2, 2), (omx, omy + 2, 6), (omx - 2, omy, 16), (omx + 2, omy, 48)]
            for qx, qy, code in cands:
                c = _s32((cmp(fsatd, qx, qy) + cmx(qx) + cmy(qy)) << 6) + code
                if c < bcost:
                    bcost = c
            if not bcost & 63:
                break
            bmx -= _s32((bcost << 26) & 0xFFFFFFFF) >> 29
            bmy -= _s32((bcost << 29) & 0xFFFFFFFF) >> 29
            bcost &= ~63
        bcost >>= 6
    if not refine_qpel and qsatd != fsatd:
        bcost = cmp(qsatd, bmx, bmy) + cmx(bmx) + cmy(bmy)
    if subme != 1:
        bdir = -1
        for _ in range(qpel):
            if bmy <= mn[1] or bmy >= mx_[1] or bmx <= mn[0] or bmx >= mx_[0]:
                break
            odir = bdir
            omx, omy = bmx, bmy
            for d, (dx, dy) in enumerate(((0, -1), (0, 1), (-1, 0), (1, 0))):
                if not refine_qpel and (d ^ 1) == odir:
                    continue
                qx, qy = omx + dx, omy + dy
                c = cmp(qsatd, qx, qy) + cmx(qx) + cmy(qy)
                if c < bcost:
                    bcost, bmx, bmy, bdir = c, qx, qy, d
            if bmx == omx and bmy == omy:
                break
    elif mn[1] < bmy < mx_[1] and mn[0] < bmx < mx_[0]:
        omx, omy = bmx, bmy
        bcost <<= 4
        for qx, qy, code in ((omx, omy - 1, 1), (omx, omy + 1, 3), (omx - 1, omy, 4), (omx + 1, omy, 12)):
            c = ((cmp(fsatd, qx, qy) + cmx(qx) + cmy(qy)) << 4) + code
            if c < bcost:
                bcost = c
        bmx -= _s32((bcost << 28) & 0xFFFFFFFF) >> 30
        bmy -= _s32((bcost << 30) & 0xFFFFFFFF) >> 30
        bcost >>= 4
    return bcost, bmx, bmy, cmx(bmx) + cmy(bmy)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("i_pixel", [0, 1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("subme,refine_qpel,fpel_satd", [(1, 0, 0), (2, 0, 0), (2, 0, 1), (4, 0, 0), (7, 0, 0),
                                                         (7, 1, 0), (7, 0, 1), (9, 0, 0), (3, 1, 0)])
def test_refine_oracle_vs_python(oracle, bd, i_pixel, subme, refine_qpel, fpel_satd):
    from conftest import load_package
    load_package()
    from x264hip import synth
    W, H = 48, 32
    planes, stride, origin = synth.make_sequence(2, W, H, bd, seed=bd + i_pixel)
    ref, fenc = planes[0], planes[1].ravel()
    hv = nr.hpel_planes(ref, 32, W, H, bd)
    pl = [ref.ravel()] + [h.ravel() for h in hv]
    pos, par, cost = rc.jobs(W // 16, H // 16, 1, i_pixel, seed=subme * 7 + bd)
    cm, c0 = rc.cost_mv()
    got = oracle.me_refine_subpel(bd, fenc, origin, stride, pl, origin, stride, i_pixel, subme, pos[:, 1:], par, cost,
                                  cm, c0, refine_qpel, fpel_satd)
    bw, bh = nr.SIZES[i_pixel]
    for i in range(len(pos)):
        want = refine_py(pl, fenc, origin, stride, int(pos[i, 1]), int(pos[i, 2]), bw, bh, par[i], cost[i], cm, c0,
                         subme, refine_qpel, fpel_satd)
        assert tuple(got[i]) == want, (i, got[i], want)
