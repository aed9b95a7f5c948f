"""CPU: the oracle's intra predictors, intra_*_x3 entries and the lookahead's
lowres intra cost (reference common/predict.c, common/pixel.c:518-560,
encoder/slicetype.c:714-757).  The six directional 8x8 modes are pinned to the
reference's own per-pixel assignment lists (tests/golden/intra8x8_golden.npz,
made by tests/golden/make_intra_golden.py); everything else is checked against
a numpy restatement here.  No GPU involved."""
import os

import numpy as np
import pytest

import numpy_ref as nr

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "intra8x8_golden.npz")
FD = 32


@pytest.mark.parametrize("bd", [8, 10])
def test_predict_8x8_directional_golden(oracle, bd):
    g = np.load(GOLDEN)
    edges, pred = g[f"edges_{bd}"], g[f"pred_{bd}"]
    for i in range(edges.shape[0]):
        for k in range(6):
            got = oracle.predict_8x8(bd, 3 + k, edges[i].astype(oracle.pixel_dtype(bd)))
            assert np.array_equal(got, pred[i, k]), (i, 3 + k)


def _np_filter(top, left, lt):
    """predict_8x8_filter with every neighbour present: edge[36] (predict.c:632-676)"""
    f2 = lambda a, b, c: (a + 2 * b + c + 2) >> 2           # noqa: E731
    e = np.zeros(36, np.int64)
    e[15] = f2(top[0], lt, left[0])
    e[14] = f2(lt, left[0], left[1])
    for y in range(1, 7):
        e[14 - y] = f2(left[y - 1], left[y], left[y + 1])
    e[6] = e[7] = (left[6] + 3 * left[7] + 2) >> 2
    t = np.concatenate([[lt], top])                          # t[-1] = lt
    for x in range(15):
        e[16 + x] = f2(t[x], t[x + 1], t[x + 2])
    e[31] = e[32] = (top[14] + 3 * top[15] + 2) >> 2
    return e


def _np_pred(kind, mode, top, left, bd):
    """4x4 / 16x16 (V, H, DC) and 8x8c / 8x16c (DC, H, V, P) predictions"""
    w, h = {0: (4, 4), 1: (8, 8), 2: (8, 16), 3: (16, 16)}[kind]
    if kind in (0, 3):
        if mode == 0:
            return np.tile(top[:w], (h, 1))
        if mode == 1:
            return np.tile(left[:h, None], (1, w))
        return np.full((h, w), (top[:w].sum() + left[:h].sum() + w) >> (3 if w == 4 else 5))
    if mode == 1:
        return np.tile(left[:h, None], (1, 8))
    if mode == 2:
        return np.tile(top[:8], (h, 1))
    if mode == 0:
        out = np.zeros((h, 8), np.int64)
        s0, s1 = top[:4].sum(), top[4:8].sum()
        for q in range(h // 4):
            sl = left[4 * q:4 * q + 4].sum()
            out[4 * q:4 * q + 4, :4] = (s0 + sl + 4) >> 3 if q == 0 else (sl + 2) >> 2
            out[4 * q:4 * q + 4, 4:] = (s1 + 2) >> 2 if q == 0 else (s1 + sl + 4) >> 3
        return out
    # planar 8x8c; top[-1] / left[-1] = lt is passed as the extra last element
    lt = top[-1]
    tt = lambda i: lt if i < 0 else top[i]                  # noqa: E731
    ll = lambda i: lt if i < 0 else left[i]                 # noqa: E731
    H = sum((i + 1) * (tt(4 + i) - tt(2 - i)) for i in range(4))
    V = sum((i + 1) * (ll(4 + i) - ll(2 - i)) for i in range(4))
    a = 16 * (left[7] + top[7])
    b, c = (17 * H + 16) >> 5, (17 * V + 16) >> 5
    y, x = np.mgrid[0:8, 0:8]
    return np.clip((a - 3 * b - 3 * c + 16 + b * x + c * y) >> 5, 0, (1 << bd) - 1)


def _np_cmp(op, a, b):
    return nr.sad(a, b) if op == 0 else nr.sa8d(a, b) if op == 3 else nr.satd(a, b)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("op", [0, 2])
def test_intra_x3(oracle, bd, kind, op):
    """intra_{sad,satd}_x3 (kind 0-3) and intra_{sad,sa8d}_x3_8x8 (kind 4, op 2 -> sa8d)"""
    rs = np.random.default_rng(bd * 100 + kind * 10 + op)
    w, h = oracle.INTRA_SIZES[kind]
    pdt = oracle.pixel_dtype(bd)
    order = (0, 1, 2) if kind in (0, 3, 4) else (0, 1, 2)
    cmp_op = 3 if (kind == 4 and op == 2) else op
    for trial in range(40):
        fenc = rs.integers(0, 1 << bd, size=16 * 16).astype(pdt)
        if trial == 0:
            fenc[:] = (1 << bd) - 1
        fe = fenc.reshape(16, 16)[:h, :w].astype(np.int64)
        if kind == 4:
            edge = rs.integers(0, 1 << bd, size=36).astype(pdt)
            got = oracle.intra_x3(bd, kind, cmp_op, fenc, 0, edge, 0)
            e = edge.astype(np.int64)
            preds = [np.tile(e[16:24], (8, 1)), np.tile(e[14:6:-1][:, None], (1, 8)),
                     np.full((8, 8), (e[7:15].sum() + e[16:24].sum() + 8) >> 4)]
        else:
            fdec = rs.integers(0, 1 << bd, size=17 * FD + 16).astype(pdt)
            if trial == 1:
                fdec[:] = 0
            off = FD + 8
            got = oracle.intra_x3(bd, kind, cmp_op, fenc, 0, fdec, off)
            top = fdec[off - FD:off - FD + 16].astype(np.int64)
            left = fdec[off - 1 + FD * np.arange(16)].astype(np.int64)
            preds = [_np_pred(kind, m, top, left, bd) for m in order]
        want = [_np_cmp(cmp_op, p.astype(np.int64), fe) for p in preds]
        assert list(got) == want, (trial, list(got), want)


def _np_lowres_cost(plane2d, mbw, mbh, bd, satd, all_modes, lam, invq):
    """per-MB composition of slicetype.c:714-757 with the numpy predictors above and the
    golden-pinned directional modes of the oracle"""
    import oracle_lib as orc
    pdt = orc.pixel_dtype(bd)
    cost = np.zeros(mbw * mbh, np.int64)
    rows = np.zeros(mbh, np.int64)
    est = [0, 0]
    op = 2 if satd else 0
    for mby in range(mbh):
        for mbx in range(mbw):
            y0, x0 = 32 + 8 * mby, 32 + 8 * mbx
            fe = plane2d[y0:y0 + 8, x0:x0 + 8].astype(np.int64)
            top = plane2d[y0 - 1, x0:x0 + 16].astype(np.int64)
            left = plane2d[y0:y0 + 8, x0 - 1].astype(np.int64)
            lt = int(plane2d[y0 - 1, x0 - 1])
            c = min(_np_cmp(op, _np_pred(1, m, top, left, bd), fe) for m in range(3))
            if all_modes:
                c = min(c, _np_cmp(op, _np_pred(1, 3, np.concatenate([top, [lt]]), np.concatenate([left, [lt]]), bd), fe))
                e = _np_filter(top, left, lt).astype(pdt)
                for m in range(3, 9):
                    c = min(c, _np_cmp(op, orc.predict_8x8(bd, m, e).astype(np.int64), fe))
            c = ((c + 5 * lam) >> (bd - 8)) + 4
            mb = mbx + mby * mbw
            cost[mb] = c
            aq = (c * int(invq[mb]) + 128) >> 8 if invq is not None else c
            rows[mby] += aq
            if (0 < mbx < mbw - 1 and 0 < mby < mbh - 1) or mbw <= 2 or mbh <= 2:
                est[0] += c
                est[1] += aq
    return cost, rows, est


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("mode", ["satd_all", "sad_dc_h_v", "sad_all_aq"])
@pytest.mark.parametrize("mbs", [(6, 4), (2, 3)])
def test_lowres_intra_cost(oracle, bd, mode, mbs):
    mbw, mbh = mbs
    rs = np.random.default_rng(bd + mbw)
    W, H = 8 * mbw, 8 * mbh
    stride = W + 64
    plane = rs.integers(0, 1 << bd, size=(H + 64, stride)).astype(oracle.pixel_dtype(bd))
    plane[40:48, 40:48] = (1 << bd) - 1
    satd = mode.startswith("satd")
    all_modes = mode.endswith("all") or mode.endswith("aq")
    invq = rs.integers(100, 400, size=mbw * mbh).astype(np.uint16) if mode.endswith("aq") else None
    lam = 11
    got = oracle.lowres_intra_cost(bd, plane.ravel(), 32 * stride + 32, stride, mbw, mbh, satd, all_modes,
                                   lam, invq)
    want = _np_lowres_cost(plane, mbw, mbh, bd, satd, all_modes, lam, invq)
    assert np.array_equal(got[0], want[0])
    assert np.array_equal(got[1], want[1])
    assert list(got[2]) == want[2]
