"""CPU: the oracle's x264_pixel_ssd_wxh / x264_pixel_ssd_nv12 restatements (reference
common/pixel.c:112-178) against direct numpy sums -- the tiling must cover every pixel
once, and the nv12 tail must start at pixel offset w&~7 as the reference writes it."""
import numpy as np
import pytest


def _planes(bd, w, h, seed, extra=40):
    rs = np.random.default_rng(seed)
    dt = np.uint8 if bd == 8 else np.uint16
    stride = w + extra
    a = rs.integers(0, 1 << bd, (h + 2) * stride).astype(dt)
    b = rs.integers(0, 1 << bd, (h + 2) * stride).astype(dt)
    return a, b, stride


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("w,h,off", [(64, 48, 0), (61, 43, 0), (7, 5, 3), (16, 16, 1), (33, 17, 16), (200, 9, 5)])
def test_ssd_wxh(oracle, bd, w, h, off):
    a, b, stride = _planes(bd, w, h, w * h + bd)
    got = oracle.ssd_wxh(bd, a, off, stride, b, off, stride, w, h)
    A = a[off:off + h * stride].reshape(h, stride)[:, :w].astype(np.int64)
    B = b[off:off + h * stride].reshape(h, stride)[:, :w].astype(np.int64)
    assert got == int(((A - B) ** 2).sum())


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("w,h", [(32, 16), (29, 11), (5, 3), (960, 4)])
def test_ssd_nv12(oracle, bd, w, h):
    a, b, stride = _planes(bd, 2 * w, h, w + h + bd)
    got = oracle.ssd_nv12(bd, a, 0, stride, b, 0, stride, w, h)
    A = a[:h * stride].reshape(h, stride).astype(np.int64)
    B = b[:h * stride].reshape(h, stride).astype(np.int64)
    d2 = (A - B) ** 2
    w8, w7 = w & ~7, w & 7
    u = int(d2[:, 0:2 * w8:2].sum()) + int(d2[:, w8:w8 + 2 * w7:2].sum())
    v = int(d2[:, 1:2 * w8:2].sum()) + int(d2[:, w8 + 1:w8 + 2 * w7:2].sum())
    assert got == (u, v)
