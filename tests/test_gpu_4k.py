"""GPU parity at BASELINE.json's large configurations (VERDICT r1 "configs untested"):

* configs[3]: 2160p (3840x2160 = 240x135 MBs, no vertical MB padding: 2160 = 135*16)
  full search range 16 (plain and predictor-centred windows, so the window clamps of
  me.hip run at 4K extents), the ESA decision, the fused 4x4 / 8x8 DCT+quant and the
  half-pel planes -- whole frames, bit-exact against the oracle (the oracle's full
  search runs a 2160p frame in ~2 s);
* configs[4]: 10-bit 1080p full search (the v5 kernel), its ESA decision and DCT8+quant8
  at full size, bit-exact;
* at both: the fused search + ESA decision and TESA (its own centred table) over whole frames.
Size-independent properties are checked beside the exact comparison: the zero-MV column
equals an independent batched sad_16x16, and every window minimum is at most that cost.
Reference semantics: encoder/me.c:618-631 (ESA window), common/pixel.c:55-80 (sad),
common/dct.c:145-205, 332-386 and common/quant.c:50-104 (transform + quant),
common/mc.c:173-196 (hpel filter)."""
import numpy as np
import pytest
import torch

import checkasm_bufs as cb

pytestmark = pytest.mark.gpu

W4K, H4K = 3840, 2160


def _dev(planes, bd):
    return torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()


def _tab(t, bd, rng):
    a = t.cpu().numpy()
    return (a.view(np.uint16) if bd == 8 else a.view(np.uint32))[..., :2 * rng + 1]


@pytest.fixture(scope="module")
def seq4k():
    from x264hip import synth
    planes, stride, origin = synth.make_sequence(2, W4K, H4K, 8)
    return planes, stride, origin


@pytest.fixture(scope="module")
def seq1080_10():
    from x264hip import synth
    planes, stride, origin = synth.make_sequence(2, 1920, 1088, 10)
    return planes, stride, origin


def _zero_mv_property(hip, dev, planes, stride, origin, got, R, mbw, mbh):
    fs = planes[0].size
    ys, xs = np.meshgrid(np.arange(mbh), np.arange(mbw), indexing="ij")
    off = (origin + 16 * (ys.ravel() * stride + xs.ravel())).astype(np.int64)
    flat = dev.view(-1)
    sc = hip.pixel_cmp_batch(hip.CMP_SAD, hip.PIXEL_16x16, flat, stride, flat, stride,
                             torch.from_numpy(off + fs).cuda(), torch.from_numpy(off).cuda())
    zero = got[:, :, R, R].ravel().astype(np.int64)
    assert np.array_equal(sc.cpu().numpy().astype(np.int64), zero)
    assert (got.reshape(mbh * mbw, -1).min(1) <= zero).all()


@pytest.mark.parametrize("bd", [8, 10])
def test_me_full_large_frame(hip, oracle, seq4k, seq1080_10, bd):
    """8 bit: a whole 2160p frame; 10 bit: a whole 1080p frame (configs[4]); R = 16."""
    planes, stride, origin = seq4k if bd == 8 else seq1080_10
    W, H = (W4K, H4K) if bd == 8 else (1920, 1088)
    R = 16
    mbw, mbh = W // 16, H // 16
    dev = _dev(planes, bd)
    fs = planes[0].size
    table = hip.me_search_full(dev[1:], origin, stride, dev[:1], origin, stride, mbw, mbh, 1, R,
                               fenc_frame_stride=fs, ref_frame_stride=fs)
    got = _tab(table, bd, R)[0]
    want = oracle.me_search_full(bd, planes[1].ravel(), origin, stride, planes[0].ravel(), origin, stride,
                                 mbw, mbh, R)
    bad = np.argwhere((got != want).any(axis=(2, 3)))
    assert not len(bad), bad[:8]
    _zero_mv_property(hip, dev, planes, stride, origin, got, R, mbw, mbh)


def _cost_mv(lam=40, span=4096):
    i = np.arange(-span, span + 1)
    logs = np.where(i == 0, 0.718, 2.0 * np.log2(np.abs(i) + 1) + 1.718)
    return np.minimum((lam * logs + 0.5).astype(np.int64), 65535).astype(np.uint16), span


@pytest.mark.parametrize("bd", [8, 10])
def test_me_centred_esa_large_frame(hip, oracle, seq4k, seq1080_10, bd):
    """Predictor-centred windows over a whole 2160p (8 bit) / 1080p (10 bit) frame: centres
    drawn up to +-40 px, so the windows of edge MBs are clamped into the 32-pixel padding
    (me.hip me_window); table + origins equal the oracle, and the origin-aware ESA decision
    (me.c:618-631, mv_limit_fpel-like bounds of analyse.c:330-349) equals the oracle's."""
    planes, stride, origin = seq4k if bd == 8 else seq1080_10
    W, H = (W4K, H4K) if bd == 8 else (1920, 1088)
    rng = me_range = 16                  # the centred table is me.c's window: no slack range
    mbw, mbh = W // 16, H // 16
    nmb = mbw * mbh
    dev = _dev(planes, bd)
    rs = np.random.default_rng(4000 + bd)
    par = np.zeros((nmb, 8), np.int16)
    par[:, 0] = rs.integers(-40, 41, nmb)
    par[:, 1] = rs.integers(-40, 41, nmb)
    par[::11, :2] = 0
    par[:, 2] = rs.integers(-64, 65, nmb)
    par[:, 3] = rs.integers(-64, 65, nmb)
    mbx, mby = np.arange(nmb) % mbw, np.arange(nmb) // mbw
    par[:, 4] = -16 * mbx - 24
    par[:, 5] = -16 * mby - 24
    par[:, 6] = 16 * (mbw - 1 - mbx) + 24 - 4
    par[:, 7] = 16 * (mbh - 1 - mby) + 24
    # keep every clipped window inside the table (me.c centres on bmx/bmy, clipped by mv limits)
    par[:, 0] = np.clip(par[:, 0], par[:, 4], par[:, 6])
    par[:, 1] = np.clip(par[:, 1], par[:, 5], par[:, 7])
    cen = np.ascontiguousarray(par[:, :2])
    table, org = hip.me_search_centred(dev[1:], origin, stride, dev[:1], origin, stride, mbw, mbh, 1, rng,
                                       torch.from_numpy(cen).cuda())
    got = table.cpu().numpy()
    got = (got.view(np.uint16) if bd == 8 else got.view(np.uint32))[0]
    org_h = org.cpu().numpy()
    want, worg = oracle.me_search_centred(bd, planes[1].ravel(), origin, stride, planes[0].ravel(), origin,
                                          stride, mbw, mbh, rng, cen)
    assert np.array_equal(org_h, worg)
    bad = np.argwhere((got != want).any(axis=(2, 3)))
    assert not len(bad), bad[:8]
    # the clamp moved the windows of edge MBs by more than the dword alignment step
    shift = org_h.astype(np.int32) - (cen.astype(np.int32) - rng)
    assert (np.abs(shift) >= 4).any()
    init = rs.integers(0, 30000, nmb).astype(np.int32)
    init[::13] = 0
    cost_mv, c0 = _cost_mv()
    cm_dev = torch.from_numpy(cost_mv.view(np.int16)).cuda()
    dec = hip.me_esa_argmin(table, rng, me_range, torch.from_numpy(par).cuda(), torch.from_numpy(init).cuda(),
                            (cm_dev, c0), origin=org).cpu().numpy()
    tab = table.cpu().numpy()
    tab = (tab.view(np.uint16) if bd == 8 else tab.view(np.uint32))[0].reshape(nmb, 2 * rng + 1, -1)
    wdec = oracle.me_esa_argmin(bd, tab, rng, me_range, par, init, cost_mv, c0, origin=org_h)
    assert np.array_equal(dec, wdec), np.argwhere((dec != wdec).any(1))[:5]
    assert (dec[::13, 0] == 0).all() and (dec[:, 0] <= init).all()
    # the fused search + decision (no table) over the same frame and predictors
    fs = planes[0].size
    fused = hip.me_search_esa(dev[1:], origin, stride, dev[:1], origin, stride, mbw, mbh, 1, rng, me_range,
                              torch.from_numpy(par).cuda(), torch.from_numpy(init).cuda(), (cm_dev, c0),
                              fenc_frame_stride=fs, ref_frame_stride=fs).cpu().numpy()
    assert np.array_equal(fused, wdec), np.argwhere((fused != wdec).any(1))[:5]


@pytest.mark.parametrize("bd", [8, 10])
def test_me_tesa_large_frame(hip, oracle, seq4k, seq1080_10, bd):
    """TESA over a whole 2160p (8 bit) / 1080p (10 bit) frame at me_range 16 with SATD: the
    self-contained call (its own centred table) against the oracle restatement of me.c:653-748."""
    import tesa_cases as tc
    planes, stride, origin = seq4k if bd == 8 else seq1080_10
    W, H = (W4K, H4K) if bd == 8 else (1920, 1088)
    me_range = 16
    mbw, mbh = W // 16, H // 16
    dev = _dev(planes, bd)
    integ = hip.frame_integral(dev[:1], origin, stride, H)
    par, init = tc.params(mbw, mbh, me_range, seed=bd + 70, centre_spread=6)
    cmv, c0 = tc.cost_mv()
    got = hip.me_tesa(dev[1:], origin, stride, dev[:1], origin, stride, integ, mbw, mbh, 1, me_range,
                      torch.from_numpy(par).cuda(), torch.from_numpy(init).cuda(),
                      (torch.from_numpy(cmv.view(np.int16)).cuda(), c0)).cpu().numpy()
    f1, f0 = planes[1].ravel(), planes[0].ravel()
    ih = oracle.frame_integral(bd, f0, origin, stride, H, tc.PAD, False).ravel()
    want = oracle.me_tesa(bd, f1, origin, stride, f0, origin, ih, tc.PAD * stride + tc.PAD, stride, mbw, mbh,
                          me_range, True, par, init, cmv, c0)
    assert np.array_equal(got, want), np.argwhere((got != want).any(1))[:5]


@pytest.mark.parametrize("transform", [4, 8])
def test_mb_dct_quant_2160p(hip, oracle, seq4k, transform):
    """fused residual transform + quant over a whole 2160p frame, QP 26 flat16 inter
    lists; prediction = reference displaced by the sequence's true motion (3, 2)."""
    planes, stride, origin = seq4k
    mbw, mbh = W4K // 16, H4K // 16
    dev = _dev(planes, 8)
    q4m, q4b, q8m, q8b = hip.cqm_init(8, cb.cqm_lists(0, 8))
    mf, bias = (q4m[1, 26], q4b[1, 26]) if transform == 4 else (q8m[1, 26], q8b[1, 26])
    po = origin + 2 * stride + 3
    dct, nz = hip.mb_dct_quant(transform, dev[1:], origin, stride, dev[:1], po, stride, mbw, mbh, 1,
                               torch.from_numpy(mf.copy()).cuda(), torch.from_numpy(bias.copy()).cuda(),
                               fenc_frame_stride=planes[0].size, pred_frame_stride=planes[0].size)
    wd, wn = oracle.mb_dct_quant(8, transform, planes[1].ravel(), origin, stride, planes[0].ravel(), po, stride,
                                 mbw, mbh, mf, bias)
    assert np.array_equal(dct.cpu().numpy(), wd)
    assert np.array_equal(nz.cpu().numpy(), wn)
    assert wn.any() and (wn == 0).any()


def test_mb_dct8_quant8_1080p_10bit(hip, oracle, seq1080_10):
    """configs[4]'s transform leg: dct8x8 + quant_8x8 at 10 bit over a whole 1080p frame."""
    planes, stride, origin = seq1080_10
    mbw, mbh = 1920 // 16, 1088 // 16
    dev = _dev(planes, 10)
    q4m, q4b, q8m, q8b = hip.cqm_init(10, cb.cqm_lists(0, 10))
    qp = 26 + 12
    po = origin + 2 * stride + 3
    dct, nz = hip.mb_dct_quant(8, dev[1:], origin, stride, dev[:1], po, stride, mbw, mbh, 1,
                               torch.from_numpy(q8m[1, qp].copy()).cuda(), torch.from_numpy(q8b[1, qp].copy()).cuda(),
                               fenc_frame_stride=planes[0].size, pred_frame_stride=planes[0].size)
    wd, wn = oracle.mb_dct_quant(10, 8, planes[1].ravel(), origin, stride, planes[0].ravel(), po, stride,
                                 mbw, mbh, q8m[1, qp], q8b[1, qp])
    assert np.array_equal(dct.cpu().numpy(), wd)
    assert np.array_equal(nz.cpu().numpy(), wn)


def test_hpel_filter_2160p(hip, oracle, seq4k):
    """half-pel planes of a whole 2160p frame (with the filtered borders)."""
    planes, stride, origin = seq4k
    dev = _dev(planes[:1].copy(), 8)
    outs = hip.hpel_filter(dev, origin, stride, W4K, H4K)
    want = oracle.frame_filter(8, planes[0].ravel().copy(), origin, stride, W4K, H4K)
    for o, w, name in zip(outs, want, "hvc"):
        got = o.cpu().numpy()[0][:, :W4K + 64]
        w2 = w.reshape(planes[0].shape)[:, :W4K + 64]
        assert np.array_equal(got, w2), (name, np.argwhere(got != w2)[:4])
