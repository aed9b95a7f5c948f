"""Python restatement of x264's P16x16 reference-0 predictors and analysis loop (the checker of
x264hip_*_me_analyse_p16x16): x264_mb_predict_mv_16x16 (reference common/mvpred.c:129-157),
x264_mb_predict_mv_ref16x16 (mvpred.c:519-600; P slice, reference 0, no MBAFF), the mv limits of
encoder/analyse.c:330-349, and the raster loop of x264_mb_analyse_inter_p16x16 calling the
oracle's x264_me_search_ref per MB, every MB taken as P_L0 16x16 with its searched mv."""
import numpy as np


def median(a, b, c):
    """x264_median (common/base.h:228-235)"""
    return max(min(a, b), min(max(a, b), c))


def predict_mv_16x16(field, x, y, mbw):
    """mvp from the decided mvs field[(y, x)] (mvpred.c:129-157): A left, B top, C top-right or, off
    the frame, D top-left; unavailable neighbours have ref -2 and mv 0"""
    def nb(nx, ny):
        if nx < 0 or ny < 0 or nx >= mbw:
            return False, (0, 0)
        return True, field[(ny, nx)]
    va, a = nb(x - 1, y)
    vb, b = nb(x, y - 1)
    vc, c = nb(x + 1, y - 1)
    if not vc:
        vc, c = nb(x - 1, y - 1)
    cnt = va + vb + vc
    if cnt > 1:
        return median(a[0], b[0], c[0]), median(a[1], b[1], c[1])
    if cnt == 1:
        return a if va else b if vb else c
    if not vb and not vc and va:
        return a
    return median(a[0], b[0], c[0]), median(a[1], b[1], c[1])


def _s16(v):
    return (int(v) + 32768) % 65536 - 32768


def predict_mv_ref16x16(field, x, y, mbw, mbh, lowres=None, tmv=None, tscale=0):
    """mvc (mvpred.c:519-600): the lowres mv doubled in 16-bit lanes ((M32 * 2) & 0xfffeffff) when
    the lowres field is valid (first entry's x != 0x7fff), the left / top / top-left / top-right
    16x16 mvs (mvr[-1] = 0 off the frame), then the reference's colocated / right / below mvs
    scaled by tscale (clip3((mv * scale + 128) >> 8))"""
    mvc = []
    mb = y * mbw + x
    if lowres is not None and lowres[0, 0] != 0x7fff:
        mvc.append((_s16(2 * int(lowres[mb, 0])), _s16(2 * int(lowres[mb, 1]))))

    def sp(nx, ny):
        if nx < 0 or ny < 0 or nx >= mbw:
            return (0, 0)
        return field[(ny, nx)]
    mvc += [sp(x - 1, y), sp(x, y - 1), sp(x - 1, y - 1), sp(x + 1, y - 1)]
    if tmv is not None:
        def tp(k):
            return tuple(min(max((int(tmv[k, q]) * tscale + 128) >> 8, -32768), 32767) for q in range(2))
        mvc.append(tp(mb))
        if x < mbw - 1:
            mvc.append(tp(mb + 1))
        if y < mbh - 1:
            mvc.append(tp(mb + mbw))
    return mvc


def limits(x, y, mbw, mbh, mv_range):
    """analyse.c:330-349: (fpel min x, y, max x, y, spel min x, y, max x, y)"""
    fmv = 4 * mv_range
    smin = (max(4 * (-16 * x - 24), -fmv), max(4 * (-16 * y - 24), -fmv))
    smax = (min(4 * (16 * (mbw - x - 1) + 24), fmv - 1), min(4 * (16 * (mbh - y - 1) + 24), fmv - 1))
    return ((smin[0] >> 2) + 6, (smin[1] >> 2) + 6, (smax[0] >> 2) - 6, (smax[1] >> 2) - 6) + smin + smax


def analyse_p16x16(search, mbw, mbh, mv_range, lowres=None, tmv=None, tscale=0):
    """the raster loop for one frame: search(x, y, par int16 [12], mvc int16 [14, 2]) -> (out [4],
    nevals [2]) runs x264_me_search_ref on the MB; returns out [mbs, 4], nevals [mbs, 2]"""
    field = {}
    out = np.zeros((mbw * mbh, 4), np.int32)
    nev = np.zeros((mbw * mbh, 2), np.int32)
    for y in range(mbh):
        for x in range(mbw):
            mvp = predict_mv_16x16(field, x, y, mbw)
            mvc = predict_mv_ref16x16(field, x, y, mbw, mbh, lowres, tmv, tscale)
            par = np.array(tuple(mvp) + limits(x, y, mbw, mbh, mv_range) + (len(mvc), 0), np.int16)
            cand = np.zeros((14, 2), np.int16)
            cand[:len(mvc)] = mvc
            o, ne = search(x, y, par, cand)
            out[y * mbw + x], nev[y * mbw + x] = o, ne
            field[(y, x)] = (int(o[1]), int(o[2]))
    return out, nev
