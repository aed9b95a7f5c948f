"""CPU: the oracle's x264_frame_init_lowres (mc.c:458-507 + frame.c:627-631)
against a vectorised numpy restatement.  No GPU involved."""
import numpy as np
import pytest


def _np_lowres(core, bd):
    """core: [H, W] frame; returns the 4 bordered lowres planes [(H/2+64), (W/2+64)]."""
    H, W = core.shape
    s = np.pad(core.astype(np.int64), ((0, 1), (0, 1)), mode="edge")      # duplicated last row / column
    a = lambda x, y: (x + y + 1) >> 1                                       # noqa: E731
    f = lambda p, q, r, t: (a(p, q) + a(r, t) + 1) >> 1                     # noqa: E731
    r0, r1, r2 = s[0:H:2], s[1:H + 1:2], s[2:H + 1:2]
    c0, c1, c2 = slice(0, W, 2), slice(1, W + 1, 2), slice(2, W + 1, 2)
    hl = H // 2
    r2 = np.concatenate([r2, s[H:H + 1]])[:hl] if r2.shape[0] < hl else r2
    planes = [f(r0[:, c0], r1[:, c0], r0[:, c1], r1[:, c1]), f(r0[:, c1], r1[:, c1], r0[:, c2], r1[:, c2]),
              f(r1[:, c0], r2[:, c0], r1[:, c1], r2[:, c1]), f(r1[:, c1], r2[:, c1], r1[:, c2], r2[:, c2])]
    return [np.pad(p, 32, mode="edge") for p in planes]


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("size", [(64, 48), (176, 144), (66, 34)])
def test_frame_init_lowres(oracle, bd, size):
    W, H = size
    rs = np.random.default_rng(bd + W)
    stride = (W + 64 + 63) // 64 * 64
    core = rs.integers(0, 1 << bd, size=(H, W))
    # padding deliberately NOT replicated: the reference overwrites column W / row H itself
    full = rs.integers(0, 1 << bd, size=(H + 64, stride))
    full[32:32 + H, 32:32 + W] = core
    full = full.astype(oracle.pixel_dtype(bd)).ravel()
    ls = (W // 2 + 64 + 63) // 64 * 64
    got = oracle.frame_init_lowres(bd, full, 32 * stride + 32, stride, W, H, ls)
    want = _np_lowres(core, bd)
    for g, w in zip(got, want):
        assert np.array_equal(g[:, :W // 2 + 64], w)


def _np_weight(p, scale, denom, offset, bd):
    off = offset << (bd - 8)
    v = p.astype(np.int64) * scale
    v = ((v + (1 << (denom - 1))) >> denom) if denom >= 1 else v
    return np.clip(v + off, 0, (1 << bd) - 1)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("width,height", [(64, 40), (73, 17), (81, 33), (5, 3)])
@pytest.mark.parametrize("w", [(40, 5, -6), (1, 0, 3), (127, 7, 0), (-3, 1, 100)])
def test_weight_scale_plane(oracle, bd, width, height, w):
    """x264_weight_scale_plane (frame.c:825-842) = mc_weight (mc.c:117-137) of every pixel in
    the reference's strip coverage: 16-wide blocks while x < width-8, then one 8-wide block,
    so up to 7 columns past width; nothing else is touched."""
    stride = 128
    rs = np.random.default_rng(width * height + bd)
    src = rs.integers(0, 1 << bd, (height + 2, stride)).astype(np.uint8 if bd == 8 else np.uint16)
    dst = np.full_like(src, 7)
    oracle.weight_scale_plane(bd, src, stride, stride, width, height, *w, dst=dst)
    cov = 0
    while cov < width - 8:
        cov += 16
    cov = cov + 8 if cov < width else cov
    want = np.full_like(src, 7)
    want[1:height + 1, :cov] = _np_weight(src[1:height + 1, :cov], *w, bd)
    assert np.array_equal(dst, want)


@pytest.mark.parametrize("bd", [8, 10])
def test_lowres_weighted_identity(oracle, bd):
    """The weighted-reference search with the identity weight (scale 1 << denom, offset 0) on the
    unweighted plane is the unweighted search; a real weight changes the result."""
    from conftest import load_package
    load_package()
    from x264hip import synth
    W, H = 128, 96
    frames, stride, origin = synth.make_sequence(2, W, H, bd)
    lw, lh = W // 2, H // 2
    ls = synth.plane_stride(lw)
    per = [oracle.frame_init_lowres(bd, frames[f].ravel(), origin, stride, W, H, ls) for f in range(2)]
    lows = [np.stack([per[f][k] for f in range(2)]) for k in range(4)]
    lo = 32 * ls + 32
    mbw, mbh = W // 16, H // 16
    intra = np.full(mbw * mbh, 16383, np.uint16)
    refs = [p[0].ravel() for p in lows]
    base = oracle.lowres_inter_cost(bd, lows[0][1].ravel(), refs, lo, ls, mbw, mbh, intra)
    same = oracle.lowres_inter_cost(bd, lows[0][1].ravel(), refs, lo, ls, mbw, mbh, intra, ref_w=refs[0],
                                    weight=(16, 4, 0))
    for a, b in zip(base, same):
        assert np.array_equal(a, b)
    wt = (23, 5, -9)
    rw = oracle.weight_scale_plane(bd, lows[0][0], 0, ls, lw + 64, lh + 64, *wt)
    other = oracle.lowres_inter_cost(bd, lows[0][1].ravel(), refs, lo, ls, mbw, mbh, intra, ref_w=rw.ravel(),
                                     weight=wt)
    assert not all(np.array_equal(a, b) for a, b in zip(base, other))


@pytest.mark.parametrize("n_slices", [2, 3, 5])
def test_lowres_slices_oracle_properties(oracle, n_slices):
    """Lookahead slices (i_lookahead_threads > 1, slicetype.c:901-918) in the oracle: the bottom
    slice scans exactly as the whole frame does (its row-below predictors exist either way),
    and a slice's results do not depend on the fenc rows of the other slices."""
    from conftest import load_package
    load_package()
    from x264hip import synth
    W, H = 160, 128
    frames, stride, origin = synth.random_planes(2, W, H, 8, seed=n_slices)   # searches that wander
    lw, lh = W // 2, H // 2
    ls = synth.plane_stride(lw)
    per = [oracle.frame_init_lowres(8, frames[f].ravel(), origin, stride, W, H, ls) for f in range(2)]
    lo = 32 * ls + 32
    mbw, mbh = W // 16, H // 16
    intra = np.full(mbw * mbh, 16383, np.uint16)
    refs = [p.ravel() for p in per[0]]
    fenc = per[1][0].copy()
    one = oracle.lowres_inter_cost(8, fenc.ravel(), refs, lo, ls, mbw, mbh, intra)
    sl = oracle.lowres_inter_cost(8, fenc.ravel(), refs, lo, ls, mbw, mbh, intra, n_slices=n_slices)
    bounds = [((mbh * i + n_slices // 2) // n_slices, (mbh * (i + 1) + n_slices // 2) // n_slices)
              for i in range(n_slices)]
    s0, s1 = bounds[-1]
    rows = slice(s0 * mbw, s1 * mbw)
    assert np.array_equal(one[0][rows], sl[0][rows]) and np.array_equal(one[1][rows], sl[1][rows])
    assert np.array_equal(one[3][s0:], sl[3][s0:])
    assert not (np.array_equal(one[0], sl[0]) and np.array_equal(one[1], sl[1]))   # slice ends lost predictors
    for i, (a, b) in enumerate(bounds):
        f2 = fenc.copy()
        keep = np.zeros(f2.shape[0], bool)
        keep[32 + 8 * a:32 + 8 * b] = True
        f2[~keep] = 255 - f2[~keep]                    # the other slices' (and the border) rows
        got = oracle.lowres_inter_cost(8, f2.ravel(), refs, lo, ls, mbw, mbh, intra, n_slices=n_slices)
        r = slice(a * mbw, b * mbw)
        assert np.array_equal(got[0][r], sl[0][r]) and np.array_equal(got[1][r], sl[1][r]), i
