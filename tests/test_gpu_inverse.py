"""GPU parity of the inverse path: the dct / quant / zigzag table entries filled by
x264hip_{8,10}_{dct,quant,zigzag}_init(X264HIP_CPU_HIP) called the way
tools/checkasm.c calls them, the batched device entries on random lists, and
the fused frame-level reconstruction on whole frames — bit-exact against the
oracle (oracle/oracle.c, cross-checked in tests/test_cpu_inverse.py)."""
import ctypes

import numpy as np
import pytest

from conftest import load_package as _x
import torch

import checkasm_bufs as cb
import numpy_ref as nr

pytestmark = pytest.mark.gpu

FLAT = [[16] * 16] * 4 + [[16] * 64] * 4


def _p(arr, off=0):
    return ctypes.c_void_p(arr.ctypes.data + int(off) * arr.itemsize)


def _coefs(oracle, bd, qp=20):
    """checkasm.c:979-993 coefficient set (quant + dequant of the sub16x16_dct(8) of pbuf1/pbuf2)."""
    b = cb.Bufs(bd)
    q4m, q4b, q8m, q8b = oracle.cqm_init(bd, FLAT)
    dq4, dq8 = oracle.cqm_dequant(FLAT)
    dct4 = oracle.sub_dct(bd, "sub16x16_dct", b.pbuf1, 0, b.pbuf1, b.pbuf2_off).reshape(16, 16)
    dct8 = oracle.sub_dct(bd, "sub16x16_dct8", b.pbuf1, 0, b.pbuf1, b.pbuf2_off).reshape(4, 64)
    o4 = [oracle.inplace(bd, "dequant_4x4", oracle.quant(bd, "quant_4x4", dct4[i], q4m[0, qp], q4b[0, qp])[0],
                         oracle._addr(dq4[0]), qp)[0] for i in range(16)]
    o8 = [oracle.inplace(bd, "dequant_8x8", oracle.quant(bd, "quant_8x8", dct8[i], q8m[0, qp], q8b[0, qp])[0],
                         oracle._addr(dq8[0]), qp)[0] for i in range(4)]
    return b, np.concatenate(o4), np.concatenate(o8)


def _cd(bd):
    return np.int16 if bd == 8 else np.int32


def _T(a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint16:
        a = a.view(np.int16)
    if a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(a).cuda()


@pytest.fixture(scope="module", params=[8, 10])
def tabs(request, hip):
    bd = request.param
    return bd, hip.dct_init(bd), hip.quant_init(bd), hip.zigzag_init(bd)


def test_table_add_idct_checkasm(oracle, tabs):
    """TEST_IDCT (checkasm.c:995-1025) for all seven entries, plus saturating inputs."""
    bd, dctf, _, _ = tabs
    b, dct4, dct8 = _coefs(oracle, bd)
    pm = (1 << bd) - 1
    cases = [(dct4, dct8)]
    cases.append((nr.wrap(np.full(256, 4 * pm * 16), bd), nr.wrap(np.full(256, pm * 64), bd)))
    cases.append((nr.wrap(np.full(256, -4 * pm * 16), bd), nr.wrap(np.full(256, -pm * 64), bd)))
    for d4, d8 in cases:
        for name in oracle.IDCT_KINDS:
            src = (d8 if "idct8" in name else d4).astype(_cd(bd))
            buf = b.pbuf1[:32 * 32].copy()
            want, _ = oracle.add_idct(bd, name, buf, 0, src)
            dc = src.copy()
            getattr(dctf, name)(_p(buf), _p(dc))
            assert np.array_equal(buf, want), name


def test_table_idct4x4dc(oracle, tabs):
    """TEST_DCTDC( idct4x4dc ) input classes (checkasm.c:1028-1054)."""
    bd, dctf, _, _ = tabs
    pm = (1 << bd) - 1
    rs = np.random.default_rng(5)
    for i in range(16):
        if i == 0:
            d = np.array([pm * 16 if (j ^ j >> 1 ^ j >> 2 ^ j >> 3) & 1 else -pm * 16 for j in range(16)])
        elif i < 8:
            d = np.where(rs.integers(0, 2, 16) > 0, pm * 16, -pm * 16)
        else:
            d = rs.integers(0, 0x2000, 16) - 0x1000
        want, _ = oracle.inplace(bd, "idct4x4dc", d)
        got = np.ascontiguousarray(d, _cd(bd))
        dctf.idct4x4dc(_p(got))
        assert np.array_equal(got, want), i


def test_table_dequant_all_qp(oracle, tabs):
    """dequant_4x4 / 8x8 / 4x4_dc at every qp with a JVT-style CQM (checkasm.c:2100-2180)."""
    bd, _, qf, _ = tabs
    dq4, dq8 = oracle.cqm_dequant(cb.cqm_lists(2, bd))
    rs = np.random.default_rng(bd + 1)
    lim = 1 << (bd + 2)
    for qp in range(0, 52 + 6 * (bd - 8)):
        for name, n, mf in (("dequant_4x4", 16, dq4[1]), ("dequant_8x8", 64, dq8[1]), ("dequant_4x4_dc", 16, dq4[2])):
            c = rs.integers(-lim, lim, n)
            want, _ = oracle.inplace(bd, name, c, oracle._addr(mf), qp)
            got = np.ascontiguousarray(c, _cd(bd))
            getattr(qf, name)(_p(got), _p(np.ascontiguousarray(mf)), qp)
            assert np.array_equal(got, want), (name, qp)


def test_table_idct_dequant_2x4_and_optimize_chroma(oracle, tabs):
    bd, _, qf, _ = tabs
    dq4, _ = oracle.cqm_dequant(FLAT)
    rs = np.random.default_rng(8)
    for qp in range(0, 52, 3):
        d = rs.integers(-300, 300, 8)
        want, _ = oracle.inplace(bd, "idct_dequant_2x4_dconly", d, oracle._addr(dq4[3]), qp)
        got = np.ascontiguousarray(d, _cd(bd))
        qf.idct_dequant_2x4_dconly(_p(got), _p(dq4[3]), qp)
        assert np.array_equal(got, want), qp
        d4w = rs.integers(-9, 9, (8, 16)).astype(_cd(bd))
        d4g = d4w.copy()
        d8 = np.ascontiguousarray(d, _cd(bd))
        oracle.fn(bd, "idct_dequant_2x4_dc")(oracle._addr(d8.copy()), oracle._addr(d4w), oracle._addr(dq4[3]), qp)
        qf.idct_dequant_2x4_dc(_p(d8), _p(d4g), _p(dq4[3]), qp)
        assert np.array_equal(d4g, d4w), qp
        dmf = int(dq4[2, qp % 6, 0]) << (qp // 6)
        for name, n in (("optimize_chroma_2x2_dc", 4), ("optimize_chroma_2x4_dc", 8)):
            for _ in range(6):
                c = rs.integers(-5, 6, n) * (rs.integers(0, 3, n) > 0)
                want, wnz = oracle.inplace(bd, name, c, dmf)
                got = np.ascontiguousarray(c, _cd(bd))
                assert getattr(qf, name)(_p(got), dmf) == wnz and np.array_equal(got, want), (name, qp, list(c))


def test_table_denoise_decimate_last_run(oracle, tabs):
    bd, _, qf, _ = tabs
    rs = np.random.default_rng(21)
    udt = np.uint16 if bd == 8 else np.uint32
    for size in (16, 64):
        d = rs.integers(-400, 400, size)
        off = rs.integers(0, 80, size).astype(udt)
        s0 = rs.integers(0, 1 << 20, size).astype(np.uint32)
        dw, sw = np.ascontiguousarray(d, _cd(bd)), s0.copy()
        oracle.fn(bd, "denoise_dct")(oracle._addr(dw), oracle._addr(sw), oracle._addr(off), size)
        dg, sg = np.ascontiguousarray(d, _cd(bd)), s0.copy()
        qf.denoise_dct(_p(dg), _p(sg), _p(off), size)
        assert np.array_equal(dg, dw) and np.array_equal(sg, sw)
    run_t = np.dtype([("last", np.int32), ("mask", np.int32), ("pad", np.int32, 2), ("level", _cd(bd), 18)],
                     align=True)
    for t in range(200):
        n = (16, 64, 4, 8, 15)[t % 5]
        mag = rs.integers(1, 3 if t % 3 else 6, 64)
        full = np.where(rs.random(64) < 0.25, mag * np.where(rs.random(64) < 0.5, -1, 1), 0).astype(_cd(bd))
        if t % 23 == 0:
            full[:] = 0
            full[rs.integers(0, n)] = 1
        if n in (16, 64):
            name = f"decimate_score{n}"
            assert getattr(qf, name)(_p(full)) == oracle.inplace(bd, name, full)[1], (n, t)
            assert qf.decimate_score15(_p(full)) == oracle.inplace(bd, "decimate_score15", full)[1]
        last = {4: qf.coeff_last4, 8: qf.coeff_last8, 15: qf.coeff_last[1], 16: qf.coeff_last[2],
                64: qf.coeff_last[5]}[n]
        assert last(_p(full)) == oracle.fn(bd, "coeff_last")(oracle._addr(full), n), (n, t)
        if n != 64 and full[:n].any():
            rl = np.zeros(1, run_t)
            fnr = {4: qf.coeff_level_run4, 8: qf.coeff_level_run8, 15: qf.coeff_level_run[1],
                   16: qf.coeff_level_run[2]}[n]
            cnt = fnr(_p(full), ctypes.c_void_p(rl.ctypes.data))
            wc, wl, wm, wlev = oracle.coeff_level_run(bd, full, n)
            assert cnt == wc and rl["last"][0] == wl and rl["mask"][0] == wm
            assert np.array_equal(rl["level"][0][:cnt], wlev)
    # aliased category slots are filled like the reference (quant.c end of x264_quant_init)
    for cat in (0, 1, 2, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13):
        assert qf.coeff_last[cat]
    assert not qf.coeff_last[3]


def test_table_zigzag(oracle, tabs):
    bd, _, _, (zp, zi) = tabs
    rs = np.random.default_rng(22)
    b = cb.Bufs(bd)
    for field, z in ((0, zp), (1, zi)):
        for n in (16, 64):
            d = rs.integers(-999, 999, n).astype(_cd(bd))
            lev = np.zeros(n, _cd(bd))
            (z.scan_8x8 if n == 64 else z.scan_4x4)(_p(lev), _p(d))
            assert np.array_equal(lev, oracle.zigzag_scan(bd, n, field, d)), (field, n)
        for kind, name in ((0, "sub_4x4"), (1, "sub_4x4ac"), (2, "sub_8x8")):
            dst = np.tile(b.pbuf1[b.pbuf2_off:b.pbuf2_off + 32], 16)
            wnz, wlev, wdc, wdst = oracle.zigzag_sub(bd, kind, field, b.pbuf1, 0, 16, dst, 0, 32)
            lev = np.zeros(64 if kind == 2 else 16, _cd(bd))
            gdst = dst.copy()
            if kind == 1:
                dc = np.zeros(1, _cd(bd))
                nz = z.sub_4x4ac(_p(lev), _p(b.pbuf1), _p(gdst), _p(dc))
                assert dc[0] == wdc
            else:
                nz = getattr(z, name)(_p(lev), _p(b.pbuf1), _p(gdst))
            assert nz == wnz and np.array_equal(lev, wlev) and np.array_equal(gdst, wdst), (field, name)
    src = rs.integers(-9, 9, 64).astype(_cd(bd))
    src[::4] = 0
    dw, nw = np.zeros(64, _cd(bd)), np.full(16, 7, np.uint8)
    oracle.fn(bd, "zigzag_interleave_8x8_cavlc")(oracle._addr(dw), oracle._addr(src), oracle._addr(nw))
    dg, ng = np.zeros(64, _cd(bd)), np.full(16, 7, np.uint8)
    zp.interleave_8x8_cavlc(_p(dg), _p(src), _p(ng))
    assert np.array_equal(dg, dw) and np.array_equal(ng, nw)


@pytest.mark.parametrize("bd", [8, 10])
def test_add_idct_batch_random(hip, oracle, bd):
    """every kind over random non-overlapping destinations with random coefficient blocks."""
    rs = np.random.default_rng(30 + bd)
    pdt = np.uint8 if bd == 8 else np.uint16
    stride = 256
    plane = rs.integers(0, 1 << bd, size=stride * 512).astype(pdt)
    b, dct4, dct8 = _coefs(oracle, bd)
    for kind, name in enumerate(oracle.IDCT_KINDS):
        w = oracle.IDCT_W[kind]
        sz = oracle.IDCT_IN[kind]
        # one call per cell of a w-sized grid (never overlapping), shuffled order
        cells = [(y, x) for y in range(0, 512 - w + 1, w) for x in range(0, stride - w + 1, w)]
        pick = rs.permutation(len(cells))[:600]
        offs = np.array([cells[i][0] * stride + cells[i][1] for i in pick], np.int64)
        src = dct8 if "idct8" in name else dct4
        pool = np.concatenate([src, -src, src // 3, rs.integers(-700, 700, 256).astype(np.int64)])
        blocks = np.stack([np.roll(pool, int(rs.integers(0, pool.size)))[:sz] for _ in offs]).astype(_cd(bd))
        want = oracle.add_idct_list(bd, kind, plane, stride, offs, blocks)
        dev = _T(plane.copy())
        hip.add_idct_batch(kind, dev, stride, _T(offs), _T(blocks))
        got = dev.cpu().numpy().view(pdt)
        assert np.array_equal(got, want), name


@pytest.mark.parametrize("bd", [8, 10])
def test_dequant_batch_random(hip, oracle, bd):
    rs = np.random.default_rng(40 + bd)
    dq4, dq8 = oracle.cqm_dequant(cb.cqm_lists(3, bd))
    qmax = 51 + 6 * (bd - 8)
    for kind, name, size, mf in ((0, "dequant_4x4", 16, dq4[0]), (1, "dequant_8x8", 64, dq8[1]),
                                 (2, "dequant_4x4_dc", 16, dq4[1])):
        n = 3000
        c = rs.integers(-(1 << (bd + 1)), 1 << (bd + 1), (n, size)).astype(_cd(bd))
        qp = rs.integers(0, qmax + 1, n).astype(np.int32)
        want = np.stack([oracle.inplace(bd, name, c[i], oracle._addr(mf), int(qp[i]))[0] for i in range(n)])
        dev = _T(c)
        hip.dequant_batch(kind, dev, _T(mf), _T(qp))
        assert np.array_equal(dev.cpu().numpy(), want), name


@pytest.mark.parametrize("bd", [8, 10])
def test_coef_batches_random(hip, oracle, bd):
    """decimate / coeff_last / level_run / zigzag scan / interleave / idct4x4dc / denoise /
    idct_dequant_2x4 / optimize_chroma over random block lists."""
    rs = np.random.default_rng(50 + bd)
    n = 2000
    mag = rs.integers(1, 4, (n, 64))
    c = np.where(rs.random((n, 64)) < 0.15, mag * np.where(rs.random((n, 64)) < 0.5, -1, 1), 0).astype(_cd(bd))
    c[::37] = 0
    dev = _T(c)
    for kind, name, num in ((0, "decimate_score15", 16), (1, "decimate_score16", 16), (2, "decimate_score64", 64)):
        got = hip.coef_stat_batch(kind, dev, 64, n).cpu().numpy()
        want = [oracle.inplace(bd, name, c[i, :num])[1] for i in range(n)]
        assert np.array_equal(got, want), name
    for kind, num in ((3, 4), (4, 8), (5, 15), (6, 16), (7, 64)):
        got = hip.coef_stat_batch(kind, dev, 64, n).cpu().numpy()
        want = [oracle.fn(bd, "coeff_last")(oracle._addr(np.ascontiguousarray(c[i])), num) for i in range(n)]
        assert np.array_equal(got, want), num
    for num in (4, 8, 15, 16):
        sel = np.flatnonzero(c[:, :num].any(1))
        sub = _T(c[sel])
        last, mask, count, level = (t.cpu().numpy() for t in hip.coeff_level_run_batch(num, sub, 64, sel.size))
        for k, i in enumerate(sel):
            wc, wl, wm, wlev = oracle.coeff_level_run(bd, c[i], num)
            assert (count[k], last[k], mask[k]) == (wc, wl, wm) and np.array_equal(level[k, :wc], wlev), (num, i)
    for size in (4, 8):
        for field in (0, 1):
            src = rs.integers(-999, 999, (300, size * size)).astype(_cd(bd))
            got = hip.zigzag_scan_batch(size, field, _T(src)).cpu().numpy()
            want = np.stack([oracle.zigzag_scan(bd, size * size, field, s) for s in src])
            assert np.array_equal(got, want), (size, field)
    src = c[:500].copy()
    dst, nnz = hip.zigzag_interleave_batch(_T(src))
    dst, nnz = dst.cpu().numpy(), nnz.cpu().numpy()
    for i in range(500):
        dw, nw = np.zeros(64, _cd(bd)), np.zeros(16, np.uint8)
        oracle.fn(bd, "zigzag_interleave_8x8_cavlc")(oracle._addr(dw), oracle._addr(np.ascontiguousarray(src[i])),
                                                     oracle._addr(nw))
        assert np.array_equal(dst[i], dw) and np.array_equal(nnz[i], nw), i
    # idct4x4dc via dc_batch kind DC_I4x4
    d = rs.integers(-0x1000, 0x1000, (400, 16)).astype(_cd(bd))
    dd = _T(d)
    hip.dc_batch(hip.DC_I4x4, dd)
    want = np.stack([oracle.inplace(bd, "idct4x4dc", x)[0] for x in d])
    assert np.array_equal(dd.cpu().numpy(), want)
    # denoise over 300 blocks sharing one sum / offset
    udt = np.uint16 if bd == 8 else np.uint32
    for size in (16, 64):
        d = rs.integers(-300, 300, (300, size)).astype(_cd(bd))
        off = rs.integers(0, 60, size).astype(udt)
        sw = rs.integers(0, 1000, size).astype(np.uint32)
        sg = sw.copy()
        dw = d.copy()
        for i in range(300):
            oracle.fn(bd, "denoise_dct")(oracle._addr(dw[i]), oracle._addr(sw), oracle._addr(off), size)
        ddev, sdev = _T(d), torch.from_numpy(sg.view(np.int32)).cuda()
        hip.denoise_dct_batch(ddev, size, sdev, _T(off))
        assert np.array_equal(ddev.cpu().numpy(), dw) and np.array_equal(sdev.cpu().numpy().view(np.uint32), sw)
    # idct_dequant_2x4 (both forms) and optimize_chroma with per-call qp / dmf
    dq4, _ = oracle.cqm_dequant(FLAT)
    m = 500
    d8 = rs.integers(-300, 300, (m, 8)).astype(_cd(bd))
    qp = rs.integers(0, 52, m).astype(np.int32)
    d4x4 = np.zeros((m, 8, 16), _cd(bd))
    hd = _T(d4x4)
    hip.idct_dequant_2x4_batch(0, _T(d8), _T(dq4[3]), _T(qp), dct4x4=hd)
    want = np.zeros((m, 8, 16), _cd(bd))
    for i in range(m):
        oracle.fn(bd, "idct_dequant_2x4_dc")(oracle._addr(d8[i].copy()), oracle._addr(want[i]), oracle._addr(dq4[3]),
                                             int(qp[i]))
    assert np.array_equal(hd.cpu().numpy(), want)
    od = _T(d8)
    hip.idct_dequant_2x4_batch(1, od, _T(dq4[3]), _T(qp))
    want = np.stack([oracle.inplace(bd, "idct_dequant_2x4_dconly", d8[i], oracle._addr(dq4[3]), int(qp[i]))[0]
                     for i in range(m)])
    assert np.array_equal(od.cpu().numpy(), want)
    for c422, name, nc in ((0, "optimize_chroma_2x2_dc", 4), (1, "optimize_chroma_2x4_dc", 8)):
        dc = (rs.integers(-6, 7, (m, nc)) * (rs.integers(0, 3, (m, nc)) > 0)).astype(_cd(bd))
        dmf = np.array([int(dq4[2, q % 6, 0]) << (q // 6) for q in qp], np.int32)
        gd = _T(dc)
        nz = hip.optimize_chroma_dc_batch(c422, gd, _T(dmf)).cpu().numpy()
        for i in range(m):
            wd, wnz = oracle.inplace(bd, name, dc[i], int(dmf[i]))
            assert nz[i] == wnz and np.array_equal(gd[i].cpu().numpy(), wd), (name, i)


@pytest.mark.parametrize("bd", [8, 10])
def test_zigzag_sub_batch_random(hip, oracle, bd):
    rs = np.random.default_rng(60 + bd)
    pdt = np.uint8 if bd == 8 else np.uint16
    stride = 192
    src = rs.integers(0, 1 << bd, size=stride * 200).astype(pdt)
    dst = rs.integers(0, 1 << bd, size=stride * 200).astype(pdt)
    for kind in (0, 1, 2):
        w = 8 if kind == 2 else 4
        for field in (0, 1):
            cells = [(y, x) for y in range(0, 200 - w + 1, w) for x in range(0, stride - w + 1, w)]
            pick = rs.permutation(len(cells))[:400]
            do = np.array([cells[i][0] * stride + cells[i][1] for i in pick], np.int64)
            so = rs.integers(0, stride * 190, do.size).astype(np.int64)
            dd = _T(dst.copy())
            level, dc, nz = hip.zigzag_sub_batch(kind, field, _T(src), stride, dd, stride, _T(so), _T(do))
            level, dc, nz = level.cpu().numpy(), dc.cpu().numpy(), nz.cpu().numpy()
            want_dst = dst.copy()
            for i in range(do.size):
                wnz, wlev, wdc, want_dst = oracle.zigzag_sub(bd, kind, field, src, so[i], stride, want_dst, do[i],
                                                             stride)
                assert nz[i] == wnz and np.array_equal(level[i], wlev), (kind, field, i)
                if kind == 1:
                    assert dc[i] == wdc
            assert np.array_equal(dd.cpu().numpy().view(pdt), want_dst)


@pytest.fixture(params=["default"])
def recon_variant(request):
    """one kernel per transform and bit depth (8 bit: block pairs for 4x4, packed int16 pairs for
    8x8; 10 bit: a lane per block); the sector-aligned wave shift applies to 64-byte strides"""
    return request.param


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("transform", [4, 8])
def test_mb_dequant_idct_add_frames(hip, oracle, bd, transform, recon_variant):
    """forward (mb_dct_quant) then inverse (mb_dequant_idct_add) over 3 frames of 1080p-width
    synthetic video with per-MB qp; recon compared with the oracle's per-MB dequant + add16x16_idct(8)."""
    from x264hip import synth
    W, H, F = 1920, 144, 3
    mbw, mbh = W // 16, H // 16
    planes, stride, origin = synth.make_sequence(F + 1, W, H, bd, start=11)
    dev = _T(planes)
    fs = planes[0].size
    qmax = 51 + 6 * (bd - 8)
    lists = cb.cqm_lists(2, bd)
    q4m, q4b, q8m, q8b = hip.cqm_init(bd, lists)
    dq4, dq8 = hip.cqm_dequant(lists)
    rs = np.random.default_rng(bd * 10 + transform)
    qp = rs.integers(0, qmax + 1, F * mbw * mbh).astype(np.int32)
    qbase = 26 + 6 * (bd - 8)
    mf = (q8m if transform == 8 else q4m)[1, qbase]
    bias = (q8b if transform == 8 else q4b)[1, qbase]
    dct, _ = hip.mb_dct_quant(transform, dev[1:], origin, stride, dev[:-1], origin, stride, mbw, mbh, F, _T(mf),
                              _T(bias), fenc_frame_stride=fs, pred_frame_stride=fs)
    dmf = dq8[1] if transform == 8 else dq4[1]
    recon = torch.zeros_like(dev[:F])
    hip.mb_dequant_idct_add(transform, dct, mbw, mbh, F, _T(dmf), _T(qp), dev[:-1], origin, stride, recon, origin,
                            stride, pred_frame_stride=fs, recon_frame_stride=fs)
    got = recon.cpu().numpy().view(planes.dtype)
    dc = dct.cpu().numpy()
    for f in range(F):
        want = np.zeros_like(planes[0]).ravel()
        sl = slice(f * mbw * mbh, (f + 1) * mbw * mbh)
        oracle.mb_dequant_idct_add(bd, transform, dc[sl], mbw, mbh, dmf, qp[sl], planes[f].ravel(), origin, stride,
                                   want, origin, stride)
        w2, g2 = want.reshape(planes[0].shape), got[f]
        assert np.array_equal(g2[32:32 + H, 32:32 + W], w2[32:32 + H, 32:32 + W]), f


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("transform", [4, 8])
@pytest.mark.parametrize("dmf_kind,crange", [("cqm", "full"), ("huge", "full"), ("cqm", "mid"), ("cqm", "small")])
def test_mb_dequant_idct_add_extremes(hip, oracle, bd, transform, dmf_kind, crange, recon_variant):
    """uniform random coefficients over the whole dctcoef range and per-MB qp 0..max, so the
    dequant products and IDCT intermediates wrap as the reference's int16 / int32 stores do;
    'huge' dequant_mf entries (>= 2^23) take the kernels' full 32-bit multiply, the CQM ones
    the 24-bit one; 'mid' / 'small' levels at qp <= 30 land on both sides of the 8-bit 8x8
    kernel's +-4096 int16-pair bound (column pass packed and row pass int32, or both packed);
    unaligned recon rows (origin + 1)."""
    mbw, mbh, F = 20, 3, 2
    W, H = 16 * mbw, 16 * mbh
    stride = W + 64
    origin = 32 * stride + 32
    rs = np.random.default_rng(bd * 100 + transform * 10 + (dmf_kind == "huge"))
    pdt = np.uint8 if bd == 8 else np.uint16
    pmax = (1 << bd) - 1
    planes = rs.integers(0, pmax + 1, (F, H + 64, stride)).astype(pdt)
    cdt = np.int16 if bd == 8 else np.int32
    lim = {"full": 1 << 15 if bd == 8 else 1 << 20, "mid": 40, "small": 12}[crange]
    dc = rs.integers(-lim, lim, (F * mbw * mbh, 256)).astype(cdt)
    dc[rs.random(dc.shape) < 0.5] = 0
    qmax = 51 + 6 * (bd - 8) if crange == "full" else 30
    qp = rs.integers(0, qmax + 1, F * mbw * mbh).astype(np.int32)
    dq4, dq8 = hip.cqm_dequant(cb.cqm_lists(4, bd))
    dmf = np.ascontiguousarray((dq8[1] if transform == 8 else dq4[1]).astype(np.int32))
    if dmf_kind == "huge":
        dmf = dmf * 4099 + (1 << 23)
    pred = _T(planes)
    recon = torch.zeros_like(pred)
    ro = origin + 1
    hip.mb_dequant_idct_add(transform, _T(dc), mbw, mbh, F, _T(dmf), _T(qp), pred, origin, stride, recon, ro,
                            stride, pred_frame_stride=planes[0].size, recon_frame_stride=planes[0].size)
    got = recon.cpu().numpy().view(pdt)
    for f in range(F):
        want = np.zeros_like(planes[0]).ravel()
        sl = slice(f * mbw * mbh, (f + 1) * mbw * mbh)
        oracle.mb_dequant_idct_add(bd, transform, dc[sl], mbw, mbh, dmf, qp[sl], planes[f].ravel(), origin, stride,
                                   want, ro, stride)
        w2 = want.reshape(planes[0].shape)
        assert np.array_equal(got[f][32:32 + H, 33:33 + W], w2[32:32 + H, 33:33 + W]), f
