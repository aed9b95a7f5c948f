"""GPU parity: batched plane SSD (x264hip_*_ssd_plane_batch / _ssd_nv12_batch) against
the oracle's x264_pixel_ssd_wxh / x264_pixel_ssd_nv12 (reference common/pixel.c:112-178):
1080p and 2160p frames, ragged widths / heights (the tiles' tails), tiny planes, maximal
differences, 8 and 10 bit."""
import numpy as np
import pytest

from conftest import load_package as _x
import torch

pytestmark = pytest.mark.gpu


def _frames(bd, n, w, h, seed, kind="random"):
    rs = np.random.default_rng(seed)
    dt = np.uint8 if bd == 8 else np.uint16
    stride = (w + 64 + 63) // 64 * 64
    pmax = (1 << bd) - 1
    if kind == "extreme":
        a = np.full((n, h + 64, stride), pmax, dt)
        b = np.zeros((n, h + 64, stride), dt)
    else:
        a = rs.integers(0, pmax + 1, (n, h + 64, stride)).astype(dt)
        b = rs.integers(0, pmax + 1, (n, h + 64, stride)).astype(dt)
    return a, b, stride, 32 * stride + 32


def _dev(p, bd):
    return torch.from_numpy(p.view(np.int16) if bd == 10 else p).cuda()


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("w,h,n,kind", [(1920, 1080, 3, "random"), (1917, 1083, 2, "random"), (7, 5, 2, "random"),
                                        (3840, 2160, 1, "random"), (1920, 1080, 1, "extreme"), (8, 8, 4, "random"),
                                        (1920, 1088, 2, "shifted"), (2100, 37, 2, "random")])
def test_ssd_plane(hip, oracle, bd, w, h, n, kind):
    a, b, stride, org = _frames(bd, n, w, h, w + h + n, kind)
    if kind == "shifted":
        org += 3                                      # chunks off 16-byte alignment
    got = hip.ssd_plane_batch(_dev(a, bd), org, stride, _dev(b, bd), org, stride, w, h, n).cpu().numpy()
    want = [oracle.ssd_wxh(bd, a[f].ravel(), org, stride, b[f].ravel(), org, stride, w, h) for f in range(n)]
    assert [int(v) for v in got.view(np.uint64)] == want


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("w,h,n", [(960, 540, 2), (957, 541, 2), (5, 3, 2), (1920, 1080, 1)])
def test_ssd_nv12(hip, oracle, bd, w, h, n):
    a, b, stride, org = _frames(bd, n, 2 * w, h, w * 3 + h)
    got = hip.ssd_nv12_batch(_dev(a, bd), org, stride, _dev(b, bd), org, stride, w, h, n).cpu().numpy()
    for f in range(n):
        want = oracle.ssd_nv12(bd, a[f].ravel(), org, stride, b[f].ravel(), org, stride, w, h)
        assert tuple(int(v) for v in got[f].view(np.uint64)) == want, f
