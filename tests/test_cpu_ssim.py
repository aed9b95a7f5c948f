"""CPU: the oracle's SSIM (reference common/pixel.c:627-714: ssim_4x4x2_core, ssim_end1 /
ssim_end4 and x264_pixel_ssim_wxh's ordered float accumulation) against a numpy / float32
restatement.  No GPU involved."""
import numpy as np
import pytest

F = np.float32


def np_end1(bd, s1, s2, ss, s12):
    pmax = (1 << bd) - 1
    if bd > 9:
        c1, c2 = F(.01 * .01 * pmax * pmax * 64), F(.03 * .03 * pmax * pmax * 64 * 63)
        f1, f2, fss, f12 = F(s1), F(s2), F(ss), F(s12)
        var = F(F(F(fss * F(64)) - F(f1 * f1)) - F(f2 * f2))
        cov = F(F(f12 * F(64)) - F(f1 * f2))
        num = F(F(F(F(F(2) * f1) * f2) + c1) * F(F(F(2) * cov) + c2))
        den = F(F(F(F(f1 * f1) + F(f2 * f2)) + c1) * F(var + c2))
        return F(num / den)
    c1, c2 = int(.01 * .01 * pmax * pmax * 64 + .5), int(.03 * .03 * pmax * pmax * 64 * 63 + .5)
    var = ss * 64 - s1 * s1 - s2 * s2
    cov = s12 * 64 - s1 * s2
    return F(F(F(2 * s1 * s2 + c1) * F(2 * cov + c2)) / F(F(s1 * s1 + s2 * s2 + c1) * F(var + c2)))


def np_sums(a, b):
    """per 4x4 block (s1, s2, ss, s12) of two [4h, 4w] planes: [h, w, 4]"""
    h, w = a.shape[0] // 4, a.shape[1] // 4
    A = a[:4 * h, :4 * w].astype(np.int64).reshape(h, 4, w, 4)
    B = b[:4 * h, :4 * w].astype(np.int64).reshape(h, 4, w, 4)
    return np.stack([A.sum((1, 3)), B.sum((1, 3)), (A * A + B * B).sum((1, 3)), (A * B).sum((1, 3))], -1)


def np_ssim_wxh(bd, a, b, width, height):
    W, H = width >> 2, height >> 2
    s = np_sums(a[:4 * H, :4 * W], b[:4 * H, :4 * W])
    tot = F(0)
    for y in range(1, H):
        for x in range(0, W - 1, 4):
            g = F(0)
            for i in range(min(4, W - x - 1)):
                q = s[y, x + i] + s[y, x + i + 1] + s[y - 1, x + i] + s[y - 1, x + i + 1]
                g = F(g + np_end1(bd, *[int(v) for v in q]))
            tot = F(tot + g)
    return tot, (H - 1) * (W - 1)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("size", [(64, 48), (70, 38), (42, 20), (8, 8), (4, 16)])
def test_ssim_wxh_vs_numpy(oracle, bd, size):
    W, H = size
    rs = np.random.default_rng(bd + W)
    a = rs.integers(0, 1 << bd, size=(H, W + 8)).astype(oracle.pixel_dtype(bd))
    b = np.clip(a.astype(np.int64) + rs.integers(-20, 21, size=a.shape), 0, (1 << bd) - 1).astype(a.dtype)
    got = oracle.ssim_wxh(bd, a.ravel(), 0, W + 8, b.ravel(), 0, W + 8, W, H)
    want = np_ssim_wxh(bd, a, b, W, H)
    assert got[1] == want[1] and got[0].tobytes() == want[0].tobytes(), (got, want)


@pytest.mark.parametrize("bd", [8, 10])
def test_ssim_core_end4_vs_numpy(oracle, bd):
    rs = np.random.default_rng(bd)
    pmax = (1 << bd) - 1
    for it in range(20):
        a = rs.integers(0, pmax + 1, size=(4, 16)).astype(oracle.pixel_dtype(bd))
        b = rs.integers(0, pmax + 1, size=(4, 16)).astype(oracle.pixel_dtype(bd))
        if it == 0:
            a[:] = pmax                                           # the 10-bit overflow note's extreme
            b[:] = pmax
        s = oracle.ssim_4x4x2_core(bd, a.ravel(), 3, 16, b.ravel(), 3, 16)
        want = np_sums(a[:, 3:11], b[:, 3:11])[0]
        assert np.array_equal(s, want)
        # sum rows of real 4x4 blocks: 5 blocks of two row bands (the last iteration: all white)
        pa = rs.integers(0, pmax + 1, size=(8, 20)) if it < 19 else np.full((8, 20), pmax)
        pb = np.clip(pa + rs.integers(-40, 41, size=pa.shape), 0, pmax)
        sums = np_sums(pa, pb)
        s0, s1 = sums[0], sums[1]
        for width in (1, 2, 3, 4):
            g = F(0)
            for i in range(width):
                q = s0[i] + s0[i + 1] + s1[i] + s1[i + 1]
                g = F(g + np_end1(bd, *[int(v) for v in q]))
            assert oracle.ssim_end4(bd, s0, s1, width).tobytes() == g.tobytes()


def test_ssim_encoder_bands():
    """fdec_filter_row's SSIM bands (encoder.c:2412-2420, 2490, 2520) for a 1080p frame, one slice
    and two thread slices (b_start / b_end at the slice edges)"""
    from conftest import load_package
    x = load_package()
    b = x.ssim_encoder_bands(68, 1080)
    assert len(b) == 68
    assert tuple(b[0]) == (2, 10) and tuple(b[1]) == (6, 22) and tuple(b[-1]) == (1062, 18)
    s = x.ssim_encoder_bands(68, 1080, [(0, 34), (34, 68)])
    assert len(s) == 68 and tuple(s[33]) == (518, 26) and tuple(s[34]) == (546, 10)


def test_ssim_bands_mt_matches_per_band(oracle):
    """cpubench.c's threaded band driver (bench.py's CPU SSIM anchor) returns each band's
    x264_pixel_ssim_wxh exactly"""
    import conftest
    conftest.load_package()
    from x264hip import synth, ssim_encoder_bands
    W, H = 256, 128
    planes, stride, origin = synth.make_sequence(2, W, H, 8)
    bands = ssim_encoder_bands(H // 16, H)
    a, b = planes[1].ravel(), planes[0].ravel()
    got, cnt = oracle.ssim_bands_mt(a, origin + 2, stride, b, origin + 2, stride, W - 2, bands, 3)
    for k, (y, h) in enumerate(bands):
        want, wc = oracle.ssim_wxh(8, a, origin + 2 + int(y) * stride, stride, b, origin + 2 + int(y) * stride, stride,
                                   W - 2, int(h))
        assert got[k] == want and cnt[k] == wc
