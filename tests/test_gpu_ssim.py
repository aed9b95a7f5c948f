"""GPU parity of SSIM and the NV12 SSD core (reference common/pixel.c:128-151, 627-714):
the table entries ssim_4x4x2_core / ssim_end4 / ssd_nv12_core installed by
x264hip_{8,10}_pixel_init, and the batched x264_pixel_ssim_wxh (bit-identical float: the
reference's accumulation order) on encoder-shaped bands and whole frames."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _p(arr, off=0):
    return ctypes.c_void_p(arr.ctypes.data + int(off) * arr.itemsize)


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int16) if a.dtype == np.uint16 else a).cuda()


def _planes(oracle, bd, W, H, seed, noise=12):
    rs = np.random.default_rng(seed)
    from x264hip import synth
    tex = synth._texture(H + 8, W + 72, bd, seed)
    a = tex[:H + 8, :W + 72].astype(oracle.pixel_dtype(bd))
    b = np.clip(a.astype(np.int64) + rs.integers(-noise, noise + 1, size=a.shape), 0, (1 << bd) - 1)
    return a, b.astype(a.dtype)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("size", [(1918, 1080), (1918, 16), (1918, 22), (70, 38), (4, 16), (44, 8)])
def test_ssim_wxh(hip, oracle, bd, size):
    """(W - 2) x h bands at x = 2 as encoder.c:2517-2528 passes them, and small odd shapes"""
    W, H = size
    a, b = _planes(oracle, bd, W, H, bd + W + H)
    s = a.shape[1]
    got, cnt = hip.ssim_wxh(_dev(a), 2, s, _dev(b), 2, s, W, H)
    want, wcnt = oracle.ssim_wxh(bd, a.ravel(), 2, s, b.ravel(), 2, s, W, H)
    assert cnt == wcnt and np.float32(got).tobytes() == want.tobytes(), (got, want)


@pytest.mark.parametrize("bd", [8, 10])
def test_ssim_wxh_extremes(hip, oracle, bd):
    """white on white (the 10-bit overflow note of pixel.c:656-658), white on black"""
    pmax = (1 << bd) - 1
    dt = oracle.pixel_dtype(bd)
    for va, vb in ((pmax, pmax), (pmax, 0), (0, 0)):
        a = np.full((64, 128), va, dt)
        b = np.full((64, 128), vb, dt)
        got, _ = hip.ssim_wxh(_dev(a), 0, 128, _dev(b), 0, 128, 120, 64)
        want, _ = oracle.ssim_wxh(bd, a.ravel(), 0, 128, b.ravel(), 0, 128, 120, 64)
        assert np.float32(got).tobytes() == want.tobytes(), (va, vb, got, want)


@pytest.mark.parametrize("bd", [8, 10])
def test_table_ssim_entries(hip, oracle, bd):
    pixf = hip.pixel_init(bd)
    assert pixf.ssim_4x4x2_core and pixf.ssim_end4 and pixf.ssd_nv12_core
    a, b = _planes(oracle, bd, 64, 24, 5 + bd, noise=60)
    s = a.shape[1]
    af, bf = a.ravel(), b.ravel()
    for off in (0, 3, 2 * s + 9):
        sums = (ctypes.c_int * 8)()
        pixf.ssim_4x4x2_core(_p(af, off), s, _p(bf, off + 1), s, sums)
        want = oracle.ssim_4x4x2_core(bd, af, off, s, bf, off + 1, s)
        assert list(sums) == want.ravel().tolist()
    rs = np.random.default_rng(bd)
    for width in (1, 2, 3, 4):
        pa = rs.integers(0, 1 << bd, size=(8, 20))
        pb = np.clip(pa + rs.integers(-30, 31, size=pa.shape), 0, (1 << bd) - 1)
        A, B = pa.reshape(2, 4, 5, 4), pb.reshape(2, 4, 5, 4)
        sums = np.stack([A.sum((1, 3)), B.sum((1, 3)), (A * A + B * B).sum((1, 3)), (A * B).sum((1, 3))], -1)
        s0 = np.ascontiguousarray(sums[0], np.int32)
        s1 = np.ascontiguousarray(sums[1], np.int32)
        got = np.float32(pixf.ssim_end4(_p(s0), _p(s1), width))
        assert got.tobytes() == oracle.ssim_end4(bd, s0, s1, width).tobytes()
    # ssd_nv12_core on the width & ~7 core of a 1080p chroma plane pair (encoder.c:2506-2512)
    from x264hip import synth
    cw, chh = 960, 540
    u = synth._texture(chh, 2 * cw + 64, bd, 9).astype(oracle.pixel_dtype(bd))
    v = np.clip(u.astype(np.int64) + rs.integers(-9, 10, size=u.shape), 0, (1 << bd) - 1).astype(u.dtype)
    su, sv = ctypes.c_uint64(), ctypes.c_uint64()
    pixf.ssd_nv12_core(_p(u.ravel()), u.shape[1], _p(v.ravel()), v.shape[1], cw, chh, ctypes.byref(su),
                       ctypes.byref(sv))
    wu, wv = oracle.ssd_nv12(bd, u.ravel(), 0, u.shape[1], v.ravel(), 0, v.shape[1], cw, chh)
    assert (su.value, sv.value) == (int(wu), int(wv))


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("W,H,slices", [(1920, 1080, None), (1920, 1080, [(0, 17), (17, 34), (34, 51), (51, 68)]),
                                        (352, 288, None), (3840, 2160, None)])
def test_ssim_bands(hip, oracle, bd, W, H, slices):
    """every encoder band of two frame pairs in one launch (encoder.c:2412-2420, 2516-2528), each
    band's float bit-identical to the oracle's x264_pixel_ssim_wxh on it, and the frame's double
    sum equal to the encoder's"""
    mbh = (H + 15) // 16
    bands = hip.ssim_encoder_bands(mbh, H, slices)
    pairs = [_planes(oracle, bd, W, H, bd + W + k) for k in range(2)]
    s = pairs[0][0].shape[1]
    a = _dev(np.stack([p[0] for p in pairs]))
    b = _dev(np.stack([p[1] for p in pairs]))
    got = hip.ssim_bands(a, 2, s, b, 2, s, W - 2, torch.from_numpy(bands).cuda()).cpu().numpy()
    for f, (pa, pb) in enumerate(pairs):
        total, wtotal = 0.0, 0.0
        for i, (y, h) in enumerate(bands):
            want, wcnt = oracle.ssim_wxh(bd, pa.ravel(), 2 + int(y) * s, s, pb.ravel(), 2 + int(y) * s, s, W - 2,
                                         int(h))
            assert got[f, i].tobytes() == want.tobytes(), (f, i, y, h, got[f, i], want)
            assert wcnt == (h // 4 - 1) * ((W - 2) // 4 - 1)
            total += float(got[f, i])
            wtotal += float(want)
        assert total == wtotal



@pytest.mark.parametrize("bd", [8, 10])
def test_ssim_bands_max_width(hip, oracle, bd):
    """the widest band x264hip_*_ssim_bands accepts (nx = width / 4 = 2047 4x4 columns,
    two rows of sums in LDS: 65.5 KB of dynamic LDS, inside gfx950's 160 KB per workgroup), each
    band bit-identical to x264_pixel_ssim_wxh; one column more is refused"""
    W, H = 8192, 48
    bands = hip.ssim_encoder_bands(H // 16, H)
    pa, pb = _planes(oracle, bd, W, H, 77 + bd)
    s = pa.shape[1]
    a, b = _dev(pa[None]), _dev(pb[None])
    got = hip.ssim_bands(a, 2, s, b, 2, s, W - 2, torch.from_numpy(bands).cuda()).cpu().numpy()
    for i, (y, h) in enumerate(bands):
        want, _ = oracle.ssim_wxh(bd, pa.ravel(), 2 + int(y) * s, s, pb.ravel(), 2 + int(y) * s, s, W - 2, int(h))
        assert got[0, i].tobytes() == want.tobytes(), (i, got[0, i], want)
    with pytest.raises(RuntimeError):
        hip.ssim_bands(a, 0, s, b, 0, s, 8196, torch.from_numpy(bands).cuda())
