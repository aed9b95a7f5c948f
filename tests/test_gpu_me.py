"""GPU parity: exhaustive 16x16 SAD search tables (x264hip_*_me_search_full)
against the oracle's exhaustive search built from the reference sad
(reference common/pixel.c:55-80, encoder/me.c:618-631)."""
import numpy as np
import pytest

from conftest import load_package as _x
import torch

pytestmark = pytest.mark.gpu


def _frames(synth, bd, w, h, kind, seed=3):
    if kind == "synthetic":
        return synth.make_sequence(3, w, h, bd, seed=seed)
    return synth.random_planes(3, w, h, bd, seed=seed)


@pytest.fixture(params=["grouped", "generic"])
def variant(request):
    """the two kernel forms a launch can take: the grouped lanes (dword-aligned planes, the
    default) and the generic one-lane-per-column kernel, which serves planes whose MB rows are
    not dword aligned -- selected here by moving the plane origin one pixel to the right"""
    return request.param


def _shift(variant, origin):
    return origin + 1 if variant == "generic" else origin


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("rng", [4, 8, 16, 24])
@pytest.mark.parametrize("kind", ["synthetic", "random"])
def test_me_full_small(hip, oracle, bd, rng, kind, variant):
    from x264hip import synth
    w, h = 80, 48
    planes, stride, origin = _frames(synth, bd, w, h, kind)
    origin = _shift(variant, origin)
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
    origin = _shift(variant, 32 * stride + 32)
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
    origin = _shift(variant, origin)
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


def _cost_mv(lam=40, span=4096):
    """an x264-shaped mv cost table (analyse.c:143-157): symmetric, lambda * bits."""
    i = np.arange(-span, span + 1)
    logs = np.where(i == 0, 0.718, 2.0 * np.log2(np.abs(i) + 1) + 1.718)
    return np.minimum((lam * logs + 0.5).astype(np.int64), 65535).astype(np.uint16), span


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("rng,me_range", [(16, 16), (24, 16), (8, 4)])
def test_me_esa_argmin(hip, oracle, bd, rng, me_range):
    """ESA decision (encoder/me.c:618-631) over the GPU table: clipped windows, the
    width rounding, mvp-dependent costs, ties and predictor-wins cases."""
    from x264hip import synth
    W, H = 160, 96
    planes, stride, origin = synth.make_sequence(2, W, H, bd, seed=5)
    dev = torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()
    fs = planes[0].size
    mbw, mbh = W // 16, H // 16
    table = hip.me_search_full(dev[1:], origin, stride, dev[:1], origin, stride, mbw, mbh, 1, rng,
                               fenc_frame_stride=fs, ref_frame_stride=fs)
    nmb = mbw * mbh
    rs = np.random.default_rng(rng * 100 + bd)
    slack = rng - me_range - 3 if rng >= me_range + 3 else 0
    par = np.zeros((nmb, 8), np.int16)
    par[:, 0] = rs.integers(-slack, slack + 1, nmb)               # bmx
    par[:, 1] = rs.integers(-slack, slack + 1, nmb)               # bmy
    par[:, 2] = rs.integers(-64, 65, nmb)                         # mvp qpel
    par[:, 3] = rs.integers(-64, 65, nmb)
    lim = rs.integers(0, me_range + 1, (nmb, 4))                  # some windows clipped
    par[:, 4] = np.maximum(par[:, 0] - me_range, -rng + 0) + np.where(rs.random(nmb) < 0.3, lim[:, 0], 0)
    par[:, 5] = np.maximum(par[:, 1] - me_range, -rng) + np.where(rs.random(nmb) < 0.3, lim[:, 1], 0)
    par[:, 6] = np.minimum(par[:, 0] + me_range, rng - 3) - np.where(rs.random(nmb) < 0.3, lim[:, 2], 0)
    par[:, 7] = np.minimum(par[:, 1] + me_range, rng) - np.where(rs.random(nmb) < 0.3, lim[:, 3], 0)
    par[:, 6] = np.maximum(par[:, 6], par[:, 4])
    par[:, 7] = np.maximum(par[:, 7], par[:, 5])
    init = rs.integers(0, 20000, nmb).astype(np.int32)
    init[::7] = 0                                                 # predictor unbeatable
    cost_mv, c0 = _cost_mv()
    cm_dev = torch.from_numpy(cost_mv.view(np.int16)).cuda()
    got = hip.me_esa_argmin(table, rng, me_range, torch.from_numpy(par).cuda(), torch.from_numpy(init).cuda(),
                            (cm_dev, c0)).cpu().numpy()
    tab = table.cpu().numpy()
    tab = (tab.view(np.uint16) if bd == 8 else tab.view(np.uint32))[0].reshape(nmb, 2 * rng + 1, -1)
    want = oracle.me_esa_argmin(bd, tab, rng, me_range, par, init, cost_mv, c0)
    assert np.array_equal(got, want), np.argwhere((got != want).any(1))[:5]
    assert (got[::7, 0] == 0).all() and (got[:, 0] <= init).all()


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("rng", [8, 16, 24])
def test_me_search_centred(hip, oracle, bd, rng, variant):
    """per-MB centres, including ones far enough out that the window is clamped into the
    padding; the whole ESA-window table (2r+1 rows x me_centred_pitch columns) and the origin
    equal the oracle's (both kernel forms)."""
    from x264hip import synth
    W, H = 96, 64
    planes, stride, origin = synth.make_sequence(3, W, H, bd, seed=7)
    origin = _shift(variant, origin)
    dev = torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()
    fs = planes[0].size
    mbw, mbh, nf = W // 16, H // 16, 2
    rs = np.random.default_rng(bd * 31 + rng)
    cen = rs.integers(-48, 49, (nf * mbw * mbh, 2)).astype(np.int16)
    cen[::5] = 0
    table, org = hip.me_search_centred(dev[1:], origin, stride, dev[:-1], origin, stride, mbw, mbh, nf, rng,
                                       torch.from_numpy(cen).cuda(), fenc_frame_stride=fs, ref_frame_stride=fs)
    assert table.shape[-1] == hip.me_centred_pitch(bd, rng)
    got = table.cpu().numpy()
    got = got.view(np.uint16) if bd == 8 else got.view(np.uint32)
    org = org.cpu().numpy()
    n1 = mbw * mbh
    for f in range(nf):
        want, worg = oracle.me_search_centred(bd, planes[f + 1].ravel(), origin, stride, planes[f].ravel(), origin,
                                              stride, mbw, mbh, rng, cen[f * n1:(f + 1) * n1])
        assert np.array_equal(org[f * n1:(f + 1) * n1], worg), f
        assert np.array_equal(got[f], want), f


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("rng,me_range", [(16, 16), (24, 16), (8, 8), (24, 24)])
def test_me_esa_argmin_centred(hip, oracle, bd, rng, me_range):
    """ESA decision around predictor centres (me.c:618-624 centres the window on bmx, bmy):
    the centred table of radius range >= me_range (the ESA window: no slack rows or columns
    beyond the alignment and width rounding) and the origin-aware argmin, vs the oracle and vs
    a plain exhaustive scan over direct SADs."""
    from x264hip import synth
    W, H = 160, 96
    planes, stride, origin = synth.make_sequence(2, W, H, bd, seed=9)
    dev = torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()
    mbw, mbh = W // 16, H // 16
    nmb = mbw * mbh
    rs = np.random.default_rng(bd + 77)
    par = np.zeros((nmb, 8), np.int16)
    par[:, 0] = rs.integers(-12, 13, nmb)
    par[:, 1] = rs.integers(-12, 13, nmb)
    par[:, 2] = rs.integers(-64, 65, nmb)
    par[:, 3] = rs.integers(-64, 65, nmb)
    mbx, mby = np.arange(nmb) % mbw, np.arange(nmb) // mbw
    par[:, 4] = -16 * mbx - 24                                      # mv_limit_fpel-like (analyse.c:330-349)
    par[:, 5] = -16 * mby - 24
    par[:, 6] = 16 * (mbw - 1 - mbx) + 24 - 4
    par[:, 7] = 16 * (mbh - 1 - mby) + 24
    cen = np.ascontiguousarray(par[:, :2])
    table, org = hip.me_search_centred(dev[1:], origin, stride, dev[:1], origin, stride, mbw, mbh, 1, rng,
                                       torch.from_numpy(cen).cuda())
    init = rs.integers(0, 20000, nmb).astype(np.int32)
    cost_mv, c0 = _cost_mv()
    cm_dev = torch.from_numpy(cost_mv.view(np.int16)).cuda()
    got = hip.me_esa_argmin(table, rng, me_range, torch.from_numpy(par).cuda(), torch.from_numpy(init).cuda(),
                            (cm_dev, c0), origin=org).cpu().numpy()
    tab = table.cpu().numpy()
    tab = (tab.view(np.uint16) if bd == 8 else tab.view(np.uint32))[0].reshape(nmb, 2 * rng + 1, -1)
    want = oracle.me_esa_argmin(bd, tab, rng, me_range, par, init, cost_mv, c0, origin=org.cpu().numpy())
    assert np.array_equal(got, want), np.argwhere((got != want).any(1))[:5]
    # every candidate of the rounded, clipped window lay inside the table: the decision equals the
    # plain exhaustive scan over direct SADs (me.c:627-631)
    f1, f0 = planes[1].ravel(), planes[0].ravel()
    for mb in range(0, nmb, 9):
        bmx, bmy = int(par[mb, 0]), int(par[mb, 1])
        x0 = max(bmx - me_range, int(par[mb, 4]))
        y0 = max(bmy - me_range, int(par[mb, 5]))
        x1 = min(bmx + me_range, int(par[mb, 6]))
        y1 = min(bmy + me_range, int(par[mb, 7]))
        wdt = (x1 - x0 + 3) & ~3
        best = (int(init[mb]), bmx, bmy)
        fo = origin + 16 * mby[mb] * stride + 16 * mbx[mb]
        for my in range(y0, y1 + 1):
            for mx in range(x0, x0 + wdt):
                c = oracle.cmp(bd, "sad", 0, f1, fo, stride, f0, fo + my * stride + mx, stride) \
                    + int(cost_mv[c0 + mx * 4 - par[mb, 2]]) + int(cost_mv[c0 + my * 4 - par[mb, 3]])
                if c < best[0]:
                    best = (c, mx, my)
        assert tuple(got[mb]) == best, mb


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("rng,me_range", [(16, 16), (24, 16), (16, 8), (8, 8), (8, 2), (24, 24), (4, 4)])
@pytest.mark.parametrize("W,H", [(160, 96), (1920, 1088)])
def test_me_search_esa_fused(hip, oracle, bd, rng, me_range, W, H):
    """Fused search + ESA decision (x264hip_*_me_search_esa) equals me_search_centred followed by
    me_esa_argmin_at on the GPU, and the oracle's centred table + argmin, over predictor centres,
    clipped windows, mvp-dependent costs and unbeatable predictors; range = me_range is exact."""
    from x264hip import synth
    if W == 1920 and (rng, me_range) not in ((16, 16), (24, 16)):
        pytest.skip("1080p at me_range 16 only")
    planes, stride, origin = synth.make_sequence(3, W, H, bd, seed=rng + me_range)
    dev = torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()
    fs = planes[0].size
    mbw, mbh, nf = W // 16, H // 16, 2
    nmb = mbw * mbh
    rs = np.random.default_rng(rng * 7 + me_range)
    par = np.zeros((nf * nmb, 8), np.int16)
    par[:, 0] = rs.integers(-12, 13, nf * nmb)
    par[:, 1] = rs.integers(-12, 13, nf * nmb)
    par[:, 2] = rs.integers(-64, 65, nf * nmb)
    par[:, 3] = rs.integers(-64, 65, nf * nmb)
    mb = np.arange(nf * nmb) % nmb
    mbx, mby = mb % mbw, mb // mbw
    tight = rs.integers(0, me_range + 1, (nf * nmb, 4)) * (rs.random((nf * nmb, 4)) < 0.3)
    par[:, 4] = np.minimum(-16 * mbx - 24 + tight[:, 0], par[:, 0])
    par[:, 5] = np.minimum(-16 * mby - 24 + tight[:, 1], par[:, 1])
    par[:, 6] = np.maximum(16 * (mbw - 1 - mbx) + 20 - tight[:, 2], par[:, 0])
    par[:, 7] = np.maximum(16 * (mbh - 1 - mby) + 24 - tight[:, 3], par[:, 1])
    init = rs.integers(0, 20000, nf * nmb).astype(np.int32)
    init[::7] = 0
    cost_mv, c0 = _cost_mv(span=8192)
    cm_dev = torch.from_numpy(cost_mv.view(np.int16)).cuda()
    par_d, init_d = torch.from_numpy(par).cuda(), torch.from_numpy(init).cuda()
    got = hip.me_search_esa(dev[1:], origin, stride, dev[:-1], origin, stride, mbw, mbh, nf, rng, me_range, par_d,
                            init_d, (cm_dev, c0), fenc_frame_stride=fs, ref_frame_stride=fs).cpu().numpy()
    cen = torch.from_numpy(np.ascontiguousarray(par[:, :2])).cuda()
    table, org = hip.me_search_centred(dev[1:], origin, stride, dev[:-1], origin, stride, mbw, mbh, nf, rng, cen,
                                       fenc_frame_stride=fs, ref_frame_stride=fs)
    ref_out = hip.me_esa_argmin(table, rng, me_range, par_d, init_d, (cm_dev, c0), origin=org).cpu().numpy()
    assert np.array_equal(got, ref_out), np.argwhere((got != ref_out).any(1))[:5]
    if W == 160:
        for f in range(nf):
            sl = slice(f * nmb, (f + 1) * nmb)
            tab, worg = oracle.me_search_centred(bd, planes[f + 1].ravel(), origin, stride, planes[f].ravel(), origin,
                                                 stride, mbw, mbh, rng, par[sl, :2])
            want = oracle.me_esa_argmin(bd, tab.reshape(nmb, 2 * rng + 1, -1), rng, me_range, par[sl], init[sl],
                                        cost_mv, c0, origin=worg)
            assert np.array_equal(got[sl], want), (f, np.argwhere((got[sl] != want).any(1))[:5])
    assert (got[::7, 0] == 0).all() and (got[:, 0] <= init).all()


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("rng", [4, 8, 16, 24])
@pytest.mark.parametrize("W,H,nf", [(160, 96, 2), (1920, 1088, 1)])
def test_me_search_full8_quadrants(hip, oracle, bd, rng, W, H, nf):
    """8x8 quadrant tables (x264hip_*_me_search_full8, 8 and 10 bit): every quadrant SAD
    equals the oracle's sad_8x8; their sum is the 16x16 table; the 16x8 / 8x16 pair sums equal
    sad_16x8 / sad_8x16 of those partitions at sampled mvs (pixel.c:55-80)."""
    if W == 1920 and rng not in (16,):
        pytest.skip("1080p at range 16 only")
    from x264hip import synth
    planes, stride, origin = synth.make_sequence(nf + 1, W, H, bd, seed=rng)
    dev = torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()
    fs = planes[0].size
    mbw, mbh = W // 16, H // 16
    w = 2 * rng + 1
    t8 = hip.me_search_full8(dev[1:], origin, stride, dev[:-1], origin, stride, mbw, mbh, nf, rng,
                             fenc_frame_stride=fs, ref_frame_stride=fs)
    t16 = hip.me_search_full(dev[1:], origin, stride, dev[:-1], origin, stride, mbw, mbh, nf, rng,
                             fenc_frame_stride=fs, ref_frame_stride=fs)
    g8 = t8.cpu().numpy().view(np.uint16)[..., :w]
    g16 = t16.cpu().numpy()
    g16 = (g16.view(np.uint16) if bd == 8 else g16.view(np.uint32))[..., :w]
    assert np.array_equal(g8.astype(np.int64).sum(3), g16)
    f = nf - 1
    want = oracle.me_search_full8(bd, planes[f + 1].ravel(), origin, stride, planes[f].ravel(), origin, stride, mbw,
                                  mbh, rng)
    assert np.array_equal(g8[f], want), np.argwhere(g8[f] != want)[:4]
    rs = np.random.default_rng(rng + W)
    f1, f0 = planes[f + 1].ravel(), planes[f].ravel()
    for _ in range(40):
        mbx, mby = int(rs.integers(mbw)), int(rs.integers(mbh))
        mx, my = (int(v) for v in rs.integers(-rng, rng + 1, 2))
        q = g8[f, mby, mbx, :, my + rng, mx + rng].astype(np.int64)
        fo = origin + 16 * mby * stride + 16 * mbx
        for i_pixel, parts in ((hip.PIXEL_16x8, ((0, 0, (0, 1)), (0, 8, (2, 3)))),
                               (hip.PIXEL_8x16, ((0, 0, (0, 2)), (8, 0, (1, 3))))):
            for px, py, qs in parts:
                o = fo + py * stride + px
                assert q[list(qs)].sum() == oracle.cmp(bd, "sad", i_pixel, f1, o, stride, f0, o + my * stride + mx,
                                                       stride)


def test_me_search_full8_shape_checks(hip):
    t = torch.empty(10, dtype=torch.int16, device="cuda")
    d = torch.zeros((2, 160, 256), dtype=torch.uint8, device="cuda")
    with pytest.raises(ValueError):
        hip.me_search_full8(d[1:], 32 * 256 + 32, 256, d[:1], 32 * 256 + 32, 256, 4, 4, 1, 8, table8=t)
