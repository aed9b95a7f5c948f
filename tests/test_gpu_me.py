"""GPU parity: exhaustive 16x16 SAD search tables (x264hip_*_me_search_full)
against the oracle's exhaustive search built from the reference sad
(reference common/pixel.c:55-80, encoder/me.c:618-631)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _frames(synth, bd, w, h, kind, seed=3):
    if kind == "synthetic":
        return synth.make_sequence(3, w, h, bd, seed=seed)
    return synth.random_planes(3, w, h, bd, seed=seed)


@pytest.fixture(params=["default", "1", "2", "3"])
def variant(request, monkeypatch):
    """every kernel variant (X264HIP_ME_VARIANT, read per launch) must be exact"""
    if request.param != "default":
        monkeypatch.setenv("X264HIP_ME_VARIANT", request.param)
    return request.param


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("rng", [4, 8, 16, 24])
@pytest.mark.parametrize("kind", ["synthetic", "random"])
def test_me_full_small(hip, oracle, bd, rng, kind, variant):
    from x264hip import synth
    w, h = 80, 48
    planes, stride, origin = _frames(synth, bd, w, h, kind)
    dev = torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()
    fs = planes[0].size
    nf = 2
    table = hip.me_search_full(dev[1:], origin, stride, dev[:-1], origin, stride, w // 16, h // 16, nf, rng,
                               fenc_frame_stride=fs, ref_frame_stride=fs)
    got = table.cpu().numpy()
    got = (got.view(np.uint16) if bd == 8 else got.view(np.uint32))[..., :2 * rng + 1]
    for f in range(nf):
        want = oracle.me_search_full(bd, planes[f + 1].ravel(), origin, stride, planes[f].ravel(), origin, stride,
                                     w // 16, h // 16, rng)
        assert np.array_equal(got[f], want), f"frame {f}: {np.argwhere(got[f] != want)[:5]}"


@pytest.mark.parametrize("bd", [8, 10])
def test_me_full_extremes(hip, oracle, bd, variant):
    """maximal differences: checkerboards of 0 / PIXEL_MAX give the largest SADs
    (65280 at 8 bit, 261888 at 10 bit) and exercise the table's full range."""
    from x264hip import synth
    w, h, rng = 48, 32, 8
    pmax = (1 << bd) - 1
    stride = synth.plane_stride(w)
    origin = 32 * stride + 32
    yy, xx = np.meshgrid(np.arange(h + 64), np.arange(stride), indexing="ij")
    dt = np.uint8 if bd == 8 else np.uint16
    a = (((yy + xx) & 1) * pmax).astype(dt)
    b = ((((yy + xx) & 1) ^ 1) * pmax).astype(dt)
    planes = np.stack([b, a])
    dev = torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()
    fs = planes[0].size
    table = hip.me_search_full(dev[1:], origin, stride, dev[:1], origin, stride, w // 16, h // 16, 1, rng,
                               fenc_frame_stride=fs, ref_frame_stride=fs)
    got = table.cpu().numpy()
    got = (got.view(np.uint16) if bd == 8 else got.view(np.uint32))[0][..., :2 * rng + 1]
    want = oracle.me_search_full(bd, a.ravel(), origin, stride, b.ravel(), origin, stride, w // 16, h // 16, rng)
    assert np.array_equal(got, want)
    assert got.max() == 256 * pmax


def test_me_full_1080p_properties(hip, oracle, variant):
    """Full 1080p frame at range 16: every table entry of a sampled set of MBs
    equals the oracle, and the zero-MV column equals an independent batched
    sad_16x16 (pixel_cmp_batch) over all 8160 MBs."""
    from x264hip import synth
    W, H, R = 1920, 1088, 16
    planes, stride, origin = synth.make_sequence(2, W, H, 8)
    dev = torch.from_numpy(planes).cuda()
    fs = planes[0].size
    mbw, mbh = W // 16, H // 16
    table = hip.me_search_full(dev[1:], origin, stride, dev[:1], origin, stride, mbw, mbh, 1, R,
                               fenc_frame_stride=fs, ref_frame_stride=fs)
    got = table.cpu().numpy().view(np.uint16)[0][..., :2 * R + 1]
    # sampled MBs (corners, edges, random interior) against the oracle
    rs = np.random.default_rng(5)
    mbs = {(0, 0), (0, mbw - 1), (mbh - 1, 0), (mbh - 1, mbw - 1)}
    mbs |= {(int(rs.integers(mbh)), int(rs.integers(mbw))) for _ in range(24)}
    for (y, x) in sorted(mbs):
        o = origin + 16 * (y * stride + x)
        want = oracle.me_search_full(8, planes[1].ravel(), o, stride, planes[0].ravel(), o, stride, 1, 1, R)
        assert np.array_equal(got[y, x], want[0, 0]), (y, x)
    # zero-MV column vs the generic batched metric
    ys, xs = np.meshgrid(np.arange(mbh), np.arange(mbw), indexing="ij")
    off = (origin + 16 * (ys.ravel() * stride + xs.ravel())).astype(np.int64)
    f_off = torch.from_numpy(off + fs).cuda()
    r_off = torch.from_numpy(off).cuda()
    flat = dev.view(-1)
    sc = hip.pixel_cmp_batch(hip.CMP_SAD, hip.PIXEL_16x16, flat, stride, flat, stride, f_off, r_off)
    assert np.array_equal(sc.cpu().numpy(), got[:, :, R, R].ravel().astype(np.int32))
    # the minimum of every window is no larger than the zero-MV cost (sanity of argmin use)
    assert (got.reshape(mbh * mbw, -1).min(1) <= got[:, :, R, R].ravel()).all()
