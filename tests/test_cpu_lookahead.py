"""CPU: the oracle's lookahead lowres motion search (slicetype_mb_cost's P-frame inter
leg, reference encoder/slicetype.c:514-713, 758-791, with x264_me_search_ref /
refine_subpel, encoder/me.c:182-420, 774-790, 865-992).  Parity unpinned (no golden
vectors exist for this path and the reference cannot be built here):
these tests pin properties the reference's definition implies -- identical frames
take the fast skip, integer lowres translations are found exactly, the cost fields
agree with each other, the mv cost table matches analyse.c's formula -- and the GPU
suite then requires bit-exact agreement with this oracle."""
import numpy as np
import pytest

from conftest import load_package

load_package()
from x264hip import synth  # noqa: E402


def _lowres_pair(oracle, bd, W, H, shift=None, seed=3):
    """two frames of a synthetic sequence (or frame 0 and an integer-lowres-pixel shift of it)
    through the oracle's frame_init_lowres; returns (fenc planes, ref planes, origin, stride)."""
    frames, stride, origin = synth.make_sequence(2, W, H, bd, seed=seed)
    if shift is not None:
        dx, dy = shift                              # fenc(x) = ref(x + d) in lowres pixels
        pad = synth.PAD
        core = frames[0][pad:pad + H, pad:pad + W]
        tex = np.pad(core, 64, mode="reflect")
        moved = tex[64 + 2 * dy:64 + 2 * dy + H, 64 + 2 * dx:64 + 2 * dx + W]
        frames[1] = np.pad(moved, ((pad, pad), (pad, stride - W - pad)), mode="edge")
    ls = synth.plane_stride(W // 2)
    out = []
    for f in range(2):
        out.append(oracle.frame_init_lowres(bd, frames[f].ravel(), origin, stride, W, H, ls))
    return out[1], out[0], 32 * ls + 32, ls


def _run(oracle, bd, W, H, **kw):
    shift = kw.pop("shift", None)
    fenc, ref, lo, ls = _lowres_pair(oracle, bd, W, H, shift)
    mbw, mbh = W // 16, H // 16
    intra, _, _ = oracle.lowres_intra_cost(bd, fenc[0].ravel(), lo, ls, mbw, mbh, True, True, 1)
    res = oracle.lowres_inter_cost(bd, fenc[0].ravel(), [p.ravel() for p in ref], lo, ls, mbw, mbh, intra, **kw)
    return res, intra


def test_cost_mv_table(oracle):
    """analyse.c:143-157 at lambda 1: cost_mv[0] = round(0.718) = 1, symmetric, log2-shaped."""
    t, c0 = oracle.cost_mv_table(1, 512)
    assert t[c0] == 1 and t[c0 + 1] == 4 and t[c0 - 1] == 4          # 2*log2(2) + 1.718 = 3.718
    assert np.array_equal(t[c0 + 1:], t[:c0][::-1])
    assert t[c0 + 3] == 6                                                 # 2*log2(4) + 1.718 = 5.718


@pytest.mark.parametrize("bd", [8, 10])
def test_identical_frames_skip(oracle, bd):
    """ref == fenc: every block has mvp 0 and a zero residual, so the fast skip
    (slicetype.c:677-686) keeps mv 0 at cost 0, and the lowres cost is the 4 penalty."""
    W, H = 128, 96
    frames, stride, origin = synth.make_sequence(1, W, H, bd)
    ls = synth.plane_stride(W // 2)
    p = oracle.frame_init_lowres(bd, frames[0].ravel(), origin, stride, W, H, ls)
    mbw, mbh = W // 16, H // 16
    intra, _, _ = oracle.lowres_intra_cost(bd, p[0].ravel(), 32 * ls + 32, ls, mbw, mbh, True, True, 1)
    mvs, mvc, lc, rows, est = oracle.lowres_inter_cost(bd, p[0].ravel(), [q.ravel() for q in p], 32 * ls + 32, ls,
                                                       mbw, mbh, intra)
    assert not mvs.any() and not mvc.any()
    assert (lc == (1 << 14) + 4).all()
    assert (rows == 4 * mbw).all() and est[2] == 0


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("me_method,subme", [(1, 4), (0, 4), (0, 2)])
def test_integer_translation(oracle, bd, me_method, subme):
    """fenc = ref shifted by (3, -2) lowres pixels: interior blocks find mv (12, -8) in qpel."""
    W, H = 256, 192
    (mvs, mvc, lc, rows, est), _ = _run(oracle, bd, W, H, shift=(3, -2), me_method=me_method, subme=subme)
    mbw, mbh = W // 16, H // 16
    m = mvs.reshape(mbh, mbw, 2)[2:-2, 2:-2].reshape(-1, 2)
    hit = ((m[:, 0] == 12) & (m[:, 1] == -8)).mean()
    assert hit > 0.9, hit


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("me_method,subme,satd", [(1, 4, True), (0, 2, False), (1, 2, True)])
def test_cost_fields_consistent(oracle, bd, me_method, subme, satd):
    """lowres_costs = min(inter + penalty, intra) with list_used, row sums and frame sums
    follow from the per-block fields (slicetype.c:758-790, AQ off)."""
    W, H = 192, 128
    (mvs, mvc, lc, rows, est), intra = _run(oracle, bd, W, H, me_method=me_method, subme=subme, satd=satd)
    mbw, mbh = W // 16, H // 16
    inter = (mvc >> (bd - 8)) + 4
    b_intra = intra.astype(np.int64) < inter
    cost = np.where(b_intra, intra, inter)
    assert np.array_equal(lc & 0x3fff, np.minimum(cost, 16383))
    assert np.array_equal(lc >> 14, (~b_intra).astype(np.uint16))
    assert np.array_equal(rows, cost.reshape(mbh, mbw).sum(1))
    fsm = np.zeros((mbh, mbw), bool)
    fsm[1:-1, 1:-1] = True
    assert est[0] == cost.reshape(mbh, mbw)[fsm].sum() == est[1]
    assert est[2] == b_intra.reshape(mbh, mbw)[fsm].sum()
    # searched mvs stay inside the lowres mv limits of slicetype.c:545-557
    xs = np.tile(np.arange(mbw), mbh)
    ys = np.repeat(np.arange(mbh), mbw)
    assert (mvs[:, 0] >= 4 * (-8 * xs - 12)).all() and (mvs[:, 0] <= 4 * (8 * (mbw - xs - 1) + 12)).all()
    assert (mvs[:, 1] >= 4 * (-8 * ys - 12)).all() and (mvs[:, 1] <= 4 * (8 * (mbh - ys - 1) + 12)).all()


@pytest.mark.parametrize("bd", [8])
def test_aq_scaling(oracle, bd):
    """inv_qscale scales the row sums and cost_est_aq, not cost_est (slicetype.c:779-786)."""
    W, H = 128, 96
    fenc, ref, lo, ls = _lowres_pair(oracle, bd, W, H)
    mbw, mbh = W // 16, H // 16
    intra, _, _ = oracle.lowres_intra_cost(bd, fenc[0].ravel(), lo, ls, mbw, mbh, True, True, 1)
    iq = np.random.default_rng(1).integers(128, 512, mbw * mbh).astype(np.uint16)
    a = oracle.lowres_inter_cost(bd, fenc[0].ravel(), [p.ravel() for p in ref], lo, ls, mbw, mbh, intra)
    b = oracle.lowres_inter_cost(bd, fenc[0].ravel(), [p.ravel() for p in ref], lo, ls, mbw, mbh, intra,
                                 inv_qscale=iq)
    assert np.array_equal(a[2], b[2]) and a[4][0] == b[4][0]
    cost = (a[2] & 0x3fff).astype(np.int64)
    aq = (cost * iq + 128) >> 8
    assert np.array_equal(b[3], aq.reshape(mbh, mbw).sum(1))


def _triplet(oracle, bd, W, H, seed=5):
    """p0, b, p1 = frames 0, 1, 2 of a synthetic sequence through frame_init_lowres"""
    frames, stride, origin = synth.make_sequence(3, W, H, bd, seed=seed)
    ls = synth.plane_stride(W // 2)
    lows = [oracle.frame_init_lowres(bd, frames[f].ravel(), origin, stride, W, H, ls) for f in range(3)]
    return lows, 32 * ls + 32, ls


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("me_method,subme,satd", [(1, 4, True), (0, 2, False)])
def test_bidir_lists_match_p_search(oracle, bd, me_method, subme, satd):
    """the B leg's list searches are the P leg's searches against p0 and p1 (same predictors,
    same me_search_ref), a cached second pass gives the same costs, and the block cost is at
    most the better list's (slicetype.c:645-713)."""
    W, H = 192, 128
    lows, lo, ls = _triplet(oracle, bd, W, H)
    mbw, mbh = W // 16, H // 16
    n = mbw * mbh
    z16, z32 = np.zeros((n, 2), np.int16), np.zeros(n, np.int32)
    ic = np.full(n, 16383, np.uint16)
    f = [p.ravel() for p in lows[1]]
    a = [p.ravel() for p in lows[0]]
    b = [p.ravel() for p in lows[2]]
    kw = dict(me_method=me_method, subme=subme, satd=satd)
    p0 = oracle.lowres_inter_cost(bd, f[0], a, lo, ls, mbw, mbh, ic, **kw)
    p1 = oracle.lowres_inter_cost(bd, f[0], b, lo, ls, mbw, mbh, ic, **kw)
    p1mvs = oracle.lowres_inter_cost(bd, b[0], a, lo, ls, mbw, mbh, ic, **kw)[0]
    m0, k0, m1, k1, lc, rows, est = oracle.lowres_bidir_cost(bd, f[0], a, b, lo, ls, mbw, mbh, 3, z16, z32, z16, z32,
                                                              p1mvs=p1mvs, dsf=128, weight=32, **kw)
    assert np.array_equal(m0, p0[0]) and np.array_equal(k0, p0[1])
    assert np.array_equal(m1, p1[0]) and np.array_equal(k1, p1[1])
    again = oracle.lowres_bidir_cost(bd, f[0], a, b, lo, ls, mbw, mbh, 0, m0, k0, m1, k1, p1mvs=p1mvs, dsf=128,
                                     weight=32, **kw)
    assert np.array_equal(again[4], lc) and np.array_equal(again[5], rows)
    cost = (lc & 0x3fff).astype(np.int64)
    used = lc >> 14
    assert set(np.unique(used)) <= {1, 2, 3}
    assert (cost <= (np.minimum(k0, k1) >> (bd - 8)) + 4).all()
    assert np.array_equal(rows, cost.reshape(mbh, mbw).sum(1))


def test_bidir_identical_refs(oracle):
    """p0 == b == p1: the predicted bidir average reproduces fenc, cost 0 + penalty, list 3."""
    W, H = 128, 96
    frames, stride, origin = synth.make_sequence(1, W, H, 8)
    ls = synth.plane_stride(W // 2)
    p = [q.ravel() for q in oracle.frame_init_lowres(8, frames[0].ravel(), origin, stride, W, H, ls)]
    mbw, mbh = W // 16, H // 16
    n = mbw * mbh
    z16, z32 = np.zeros((n, 2), np.int16), np.zeros(n, np.int32)
    r = oracle.lowres_bidir_cost(8, p[0], p, p, 32 * ls + 32, ls, mbw, mbh, 3, z16, z32, z16, z32, weight=43)
    assert (r[4] == (3 << 14) + 4).all()
