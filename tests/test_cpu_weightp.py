"""CPU: the oracle's weighted-prediction analysis -- x264_weights_analyse (slicetype.c:284-501),
its cost functions (slicetype.c:77-282), mc_chroma (mc.c:252-283) and the frame statistics
(ratecontrol.c:225-257, 406-414) -- against an independent numpy / float32 restatement.
No GPU involved."""
import math

import numpy as np
import pytest

import weightp_cases as wc

H4 = np.array([[1, 1, 1, 1], [1, -1, 1, -1], [1, 1, -1, -1], [1, -1, -1, 1]])


def np_weight(p, w, bd):
    """mc_weight (mc.c:117-137)"""
    _, scale, denom, offset = w
    off = offset << (bd - 8)
    v = (p.astype(np.int64) * scale + ((1 << (denom - 1)) if denom else 0)) >> denom
    return np.clip(v + off, 0, (1 << bd) - 1)


def np_satd8x8(a, b):
    d = a.astype(np.int64) - b.astype(np.int64)
    tot = 0
    for y in (0, 4):
        s = sum(np.abs(H4 @ d[y:y + 4, x:x + 4] @ H4.T).sum() for x in (0, 4))
        tot += s >> 1                                        # pixel_satd_8x4's halving per band
    return int(tot)


def np_mbcmp(a, b, satd):
    h, w = a.shape
    if not satd:
        return int(np.abs(a.astype(np.int64) - b.astype(np.int64)).sum())
    return sum(np_satd8x8(a[y:y + 8, x:x + 8], b[y:y + 8, x:x + 8]) for y in range(0, h, 8) for x in range(0, w, 8))


def ue(v):
    return 2 * int(math.floor(math.log2(v))) + 1 if v else 1


def se(v):
    t = 1 - 2 * v if 1 - 2 * v >= 0 else 2 * v
    return ue(t) if t < 256 else ue(t >> 8) + 16


def header(w, chroma, lam, ns):
    lam = lam * 4 if chroma else lam
    return lam * ns * (10 + ue(w[2] + 1) * (2 - chroma) + 2 * (se(w[1]) + se(w[3])))


def np_get_ref(planes, lo, ls, mvx, mvy, x, y):
    """8x8 lowres get_ref (mc.c:221-249) at block (x, y) + qpel mv"""
    r0 = [0, 1, 1, 1, 0, 1, 1, 1, 2, 3, 3, 3, 0, 1, 1, 1]
    r1 = [0, 0, 1, 0, 2, 2, 3, 2, 2, 2, 3, 2, 2, 2, 3, 2]
    mx, my = mvx + 4 * x, mvy + 4 * y
    q = ((my & 3) << 2) + (mx & 3)
    oy, ox = 32 + (my >> 2), 32 + (mx >> 2)
    a = planes[r0[q]][oy + ((my & 3) == 3):oy + ((my & 3) == 3) + 8, ox:ox + 8].astype(np.int64)
    if q & 5:
        b = planes[r1[q]][oy:oy + 8, ox + ((mx & 3) == 3):ox + ((mx & 3) == 3) + 8].astype(np.int64)
        a = (a + b + 1) >> 1
    return a


def np_mc_chroma(nv, cy, cx, mvx, mvy, w, h):
    """mc_chroma (mc.c:252-283) at interleaved (cy, cx): (u, v)"""
    dx, dy = mvx & 7, mvy & 7
    cA, cB, cC, cD = (8 - dx) * (8 - dy), dx * (8 - dy), (8 - dx) * dy, dx * dy
    y0, x0 = cy + (mvy >> 3), cx + (mvx >> 3) * 2
    s = nv[y0:y0 + h + 1, x0:x0 + 2 * w + 2].astype(np.int64)
    out = []
    for p in (0, 1):
        a, b = s[:h, p:p + 2 * w:2], s[:h, p + 2:p + 2 * w + 2:2]
        c, d = s[1:h + 1, p:p + 2 * w:2], s[1:h + 1, p + 2:p + 2 * w + 2:2]
        out.append((cA * a + cB * b + cC * c + cD * d + 32) >> 6)
    return out


def np_cost(kind, bd, fenc, ref, mbw, mbh, w, intra=None, mvs=None, satd=True, plane=0, lam=1, ns=1, lr=None):
    """weight_cost_luma / _chroma / _chroma444 with w = (weighted, scale, denom, offset).
    kind 0: fenc / ref = lists of bordered lowres planes ((0,0) at (32, 32)); 1 / 2: bordered NV
    planes; 3: bordered 4:4:4 planes"""
    cost = 0
    if kind == 0:
        f = fenc[0]
        for by in range(mbh):
            for bx in range(mbw):
                mb = by * mbw + bx
                if mvs is None:
                    r = ref[0][32 + 8 * by:40 + 8 * by, 32 + 8 * bx:40 + 8 * bx].astype(np.int64)
                else:
                    r = np_get_ref(ref, 32, 0, int(mvs[mb][0]), int(mvs[mb][1]), 8 * bx, 8 * by)
                if w[0]:
                    r = np_weight(r, w, bd)
                c = np_mbcmp(r, f[32 + 8 * by:40 + 8 * by, 32 + 8 * bx:40 + 8 * bx], satd)
                cost += min(c, int(intra[mb]))
    elif kind in (1, 2):
        h = 8 if kind == 1 else 16
        for by in range(mbh):
            for bx in range(mbw):
                mb = by * mbw + bx
                cy, cx = 32 + h * by, 32 + 16 * bx
                if mvs is None:
                    r = ref[cy:cy + h, cx + plane:cx + 16:2].astype(np.int64)
                else:
                    r = np_mc_chroma(ref, cy, cx, int(mvs[mb][0]), (2 * int(mvs[mb][1])) >> (kind == 1), 8, h)[plane]
                if w[0]:
                    r = np_weight(r, w, bd)
                cost += abs(int(r.sum()) - int(fenc[cy:cy + h, cx + plane:cx + 16:2].astype(np.int64).sum()))
    else:
        for by in range(mbh):
            for bx in range(mbw):
                mb = by * mbw + bx
                mx, my = (0, 0) if mvs is None else (int(np.fix(mvs[mb][0] / 2)), int(np.fix(mvs[mb][1] / 2)))
                r = ref[32 + 16 * by + my:48 + 16 * by + my, 32 + 16 * bx + mx:48 + 16 * bx + mx].astype(np.int64)
                if w[0]:
                    r = np_weight(r, w, bd)
                cost += np_mbcmp(r, fenc[32 + 16 * by:48 + 16 * by, 32 + 16 * bx:48 + 16 * bx], satd)
    if w[0]:
        cost += header(w, kind != 0, lam, ns)
    return cost & 0xFFFFFFFF


def _kind_inputs(kind, ref, fenc, an):
    if kind == 0:
        return an.fenc_lr, an.ref_lr
    if kind in (1, 2):
        return fenc.nv, ref.nv
    return fenc.u, ref.u


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("kind,cf", [(0, 0), (1, 1), (2, 2), (3, 3)])
@pytest.mark.parametrize("with_mvs", [False, True])
@pytest.mark.parametrize("satd", [True, False])
def test_weight_cost_vs_numpy(oracle, bd, kind, cf, with_mvs, satd):
    if kind in (1, 2) and not satd:
        pytest.skip("asd8 has no mbcmp choice")
    ref, fenc = wc.make_pair(bd, 64, 48, cf, (1.1, -6), ((0.9, 4), (1.2, -3)), seed=bd + kind)
    an = wc.Analysis(oracle, ref, fenc, satd=satd, search_mvs=False)
    mvs = wc.random_mvs(an.mbw, an.mbh, 5 + kind) if with_mvs else None
    f, r = _kind_inputs(kind, ref, fenc, an)
    cands = wc.candidates(bd * 10 + kind, n=10)
    for plane in ((0, 1) if kind in (1, 2) else (0,)):
        if kind == 0:
            got = oracle.weight_cost_list(bd, 0, f[0].ravel(), [p.ravel() for p in r], an.lo, an.ls, an.mbw, an.mbh,
                                          cands, intra=an.intra, mvs=mvs, satd=satd, lam=3, n_slices=2)
        else:
            stride = f.shape[1]
            got = oracle.weight_cost_list(bd, kind, f.ravel(), [r.ravel()], 32 * stride + 32, stride, an.mbw, an.mbh,
                                          cands, mvs=mvs, satd=satd, plane=plane, lam=3, n_slices=2)
        want = [np_cost(kind, bd, f, r, an.mbw, an.mbh, c, intra=an.intra, mvs=mvs, satd=satd, plane=plane, lam=3,
                        ns=2) for c in cands]
        assert list(got) == want


@pytest.mark.parametrize("bd", [8, 10])
def test_mc_chroma_vs_numpy(oracle, bd):
    rs = np.random.default_rng(bd)
    nv = rs.integers(0, 1 << bd, size=(40, 96)).astype(oracle.pixel_dtype(bd))
    for mvx, mvy in [(0, 0), (3, 5), (-9, 7), (17, -13), (-1, -1)]:
        u, v = oracle.mc_chroma(bd, nv.ravel(), 12 * 96 + 24, 96, mvx, mvy, 8, 8)
        nu, nv_ = np_mc_chroma(nv, 12, 24, mvx, mvy, 8, 8)
        assert np.array_equal(u, nu) and np.array_equal(v, nv_)


def np_stats(f, mbw, mbh):
    """i_pixel_sum / i_pixel_ssd after x264_adaptive_quant_frame"""
    cf, bd = f.cf, f.bd
    planes = [f.y[32:32 + 16 * mbh, 32:32 + 16 * mbw].astype(np.int64)]
    if cf in (1, 2):
        h = 16 * mbh >> (cf == 1)
        planes += [f.nv[32:32 + h, 32 + p:32 + 16 * mbw:2].astype(np.int64) for p in (0, 1)]
    elif cf == 3:
        planes += [p[32:32 + 16 * mbh, 32:32 + 16 * mbw].astype(np.int64) for p in (f.u, f.v)]
    s, d = [0, 0, 0], [0, 0, 0]
    for i, p in enumerate(planes):
        tot = int(p.sum()) & 0xFFFFFFFF
        sq = int((p * p).sum())
        n = p.size
        s[i], d[i] = tot, (sq - (tot * tot + n // 2) // n) & 0xFFFFFFFFFFFFFFFF
    return s, d


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("cf", [0, 1, 2, 3])
def test_frame_pixel_stats_vs_numpy(oracle, bd, cf):
    ref, fenc = wc.make_pair(bd, 80, 64, cf, seed=3 + cf)
    an = wc.Analysis(oracle, ref, fenc, search_mvs=False)
    for fr, got in ((fenc, an.fstats), (ref, an.rstats)):
        s, d = np_stats(fr, an.mbw, an.mbh)
        assert list(map(int, got[0])) == s and list(map(int, got[1])) == d


# ---- the search, restated in float32 (numpy scalars round every operation to float32) ----
F = np.float32


def c_round(x):
    """C round() of a float promoted to double: half away from zero"""
    x = float(x)
    return int(math.floor(abs(x) + 0.5)) * (1 if x >= 0 else -1)


def clip3(v, lo, hi):
    return lo if v < lo else hi if v > hi else v


def py_weights_analyse(bd, cost_of, fstats, rstats, mbw, mbh, cf, b_lookahead, subme, weightp_fake):
    """slicetype.c:284-485 with cost_of(plane, w) = the plane's weight_cost_* (w None = unweighted)"""
    hs, vs = (1, 1) if cf == 1 else (1, 0) if cf == 2 else (0, 0)
    W = [[0, 1, 0, 0] for _ in range(3)]
    gs, fm, rm = [F(1)] * 3, [F(0)] * 3, [F(0)] * 3
    for plane in range(0, 2 * (not b_lookahead) + 1):
        if not plane or cf:
            zb = int(not rstats[1][plane])
            fv, rv = F(int(fstats[1][plane]) + zb), F(int(rstats[1][plane]) + zb)
            npx = (16 * mbh >> (vs if plane else 0)) * (16 * mbw >> (hs if plane else 0))
            gs[plane] = np.sqrt(F(fv / rv), dtype=F)
            fm[plane] = F(F(int(fstats[0][plane]) + zb) / F(npx)) / F(1 << (bd - 8))
            rm[plane] = F(F(int(rstats[0][plane]) + zb) / F(npx)) / F(1 << (bd - 8))
    cd = 7
    if not b_lookahead:
        while cd > 0:
            th = F(F(127) / F(1 << cd))
            if gs[1] < th and gs[2] < th:
                break
            cd -= 1
    dist = [(0, 0), (0, 0), (0, 1), (0, 1), (0, 1), (0, 1), (0, 1), (1, 1), (1, 1), (2, 1), (2, 1), (4, 2)]
    delta = None
    plane = 0
    while plane < (3 if cf else 1) and not (plane and (not W[0][0] or b_lookahead)):
        if abs(F(rm[plane] - fm[plane])) < F(0.5) and abs(F(F(1) - gs[plane])) < F(1 / 128):
            W[plane] = [0, 1, 0, 0]
            plane += 1
            continue
        if plane:
            W[plane][2] = cd
            W[plane][1] = clip3(c_round(F(gs[plane] * F(1 << cd))), 0, 255)
            if W[plane][1] > 127:
                W[1][0] = W[2][0] = 0
                break
        else:
            s, d = c_round(F(gs[0] * F(128))), 7
            while d > 0 and s > 127:
                d -= 1
                s >>= 1
            W[0][1], W[0][2], W[0][3] = min(s, 127), d, 0
        mindenom, minscale, minoff, found = W[plane][2], W[plane][1], 0, 0
        orig = minscore = cost_of(plane, None)
        if not minscore:
            plane += 1
            continue
        sd, od = (0, 0) if b_lookahead else dist[subme]
        for i_scale in range(clip3(minscale - sd, 0, 127), clip3(minscale + sd, 0, 127) + 1):
            cur_scale = i_scale
            cur_off = int(F(F(fm[plane] - F(F(rm[plane] * F(cur_scale)) / F(1 << mindenom))) + F(F(0.5) * F(b_lookahead))))
            if cur_off < -128 or cur_off > 127:
                cur_off = clip3(cur_off, -128, 127)
                v = F(F(F(F(1 << mindenom) * F(fm[plane] - F(cur_off))) / rm[plane]) + F(0.5))
                cur_scale = int(clip3(float(v), 0.0, 127.0))
            so, eo = clip3(cur_off - od, -128, 127), clip3(cur_off + od, -128, 127)
            for i_off in range(so, eo + 1):
                W[plane] = [1, cur_scale, mindenom, i_off]
                s = cost_of(plane, tuple(W[plane]))
                if s < minscore:
                    minscore, minscale, minoff, found = s, cur_scale, i_off, 1
                if minoff == so and i_off != so:
                    break
        if not plane:
            while mindenom > 0 and not (minscale & 1):
                mindenom -= 1
                minscale >>= 1
        if not found or (minscale == 1 << mindenom and minoff == 0) or F(F(minscore) / F(orig)) > F(0.998):
            W[plane] = [0, 1, 0, 0]
        else:
            W[plane] = [1, minscale, mindenom, minoff]
            if weightp_fake and W[0][0] and not plane:
                delta = float(F(F(minscore) / F(orig)))
        plane += 1
    if W[1][0] or W[2][0]:
        den = W[1][2] if W[1][0] else W[2][2]
        both = W[1][0] and W[2][0]
        while (not both and den == 7) or (den > 0 and not (W[1][0] and W[1][1] & 1) and not (W[2][0] and W[2][1] & 1)):
            den -= 1
            for i in (1, 2):
                if W[i][0]:
                    W[i][1] >>= 1
                    W[i][2] = den
    return W, delta


CASES = [  # (cf, luma fade, chroma fades, b_lookahead, subme, mvs, fake, flat ref chroma)
    (0, (1.0, 0.0), ((1, 0), (1, 0)), True, 7, False, False, False),      # no fade: early termination
    (0, (0.8, 10.0), ((1, 0), (1, 0)), True, 7, False, False, False),     # lookahead fade-out
    (1, (1.25, -12.0), ((0.85, 6), (1.15, -5)), False, 7, True, False, False),
    (1, (0.6, 40.0), ((0.7, 20), (1.3, -20)), False, 11, True, True, False),
    (2, (1.1, 3.0), ((1.05, 2), (0.9, 4)), False, 9, False, False, False),
    (3, (0.9, -5.0), ((1.2, -8), (0.8, 9)), False, 10, True, False, False),
    (1, (1.3, -20.0), ((1.0, 0), (1.0, 0)), False, 2, False, True, True),  # chroma scale > 127: the break
    (0, (0.2, 150.0), ((1, 0), (1, 0)), False, 11, False, False, False),   # offset clamp and rescale
]


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_weights_analyse_vs_python(oracle, bd, case):
    cf, lf, cfs, bl, subme, with_mvs, fake, flat = CASES[case]
    ref, fenc = wc.make_pair(bd, 64, 48, cf, lf, cfs, seed=11 + case, flat_ref_chroma=flat,
                             shift=(3, 2) if with_mvs else (0, 0))
    an = wc.Analysis(oracle, ref, fenc, search_mvs=with_mvs, intra_scale=1 << (bd - 8))
    lam, ns = 3, 1

    def cost_of(plane, w):
        ww = w if w is not None else (0, 1, 0, 0)
        if plane == 0:
            return np_cost(0, bd, an.fenc_lr, an.ref_lr, an.mbw, an.mbh, ww, intra=an.intra, mvs=an.mvs, lam=lam,
                           ns=ns)
        if cf == 3:
            f, r = (fenc.u, ref.u) if plane == 1 else (fenc.v, ref.v)
            return np_cost(3, bd, f, r, an.mbw, an.mbh, ww, mvs=an.mvs, lam=lam, ns=ns)
        return np_cost(cf, bd, fenc.nv, ref.nv, an.mbw, an.mbh, ww, mvs=an.mvs, plane=plane - 1, lam=lam, ns=ns)

    want, wdelta = py_weights_analyse(bd, cost_of, an.fstats, an.rstats, an.mbw, an.mbh, cf, bl, subme, fake)
    got, delta = oracle.weights_analyse(bd, an.fenc_lr[0].ravel(), [p.ravel() for p in an.ref_lr], an.lo, an.ls,
                                        an.mbw, an.mbh, an.intra, an.fstats, an.rstats, mvs=an.mvs, chroma_format=cf,
                                        fenc_c=[None if c is None else c.ravel() for c in fenc.chroma()],
                                        ref_c=[None if c is None else c.ravel() for c in ref.chroma()],
                                        c_origin=fenc.co, cs=fenc.cs, b_lookahead=bl, subme=subme, lam=lam,
                                        n_slices=ns, weightp_fake=fake)
    assert got.tolist() == want, (got.tolist(), want)
    assert delta == wdelta
