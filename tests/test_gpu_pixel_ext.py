"""GPU parity of the further x264_pixel_function_t entries (sa8d, sa8d_satd,
var, var2, hadamard_ac, vsad, asd8, ads) through the table filled by
x264hip_{8,10}_pixel_init(X264HIP_CPU_HIP) on checkasm's patterns, the batched
entries on random lists, and the ESA integral image on whole frames — all
bit-exact against the oracle."""
import ctypes

import numpy as np
import pytest
import torch

import checkasm_bufs as cb
import numpy_ref as nr

pytestmark = pytest.mark.gpu


def _p(arr, off=0):
    return ctypes.c_void_p(arr.ctypes.data + int(off) * arr.itemsize)


@pytest.fixture(scope="module", params=[8, 10])
def setup(request, hip):
    bd = request.param
    b = cb.Bufs(bd)
    b.fill_pixel_overflow()
    return bd, b, hip.pixel_init(bd)


def _dev(plane, bd):
    return torch.from_numpy(plane.view(np.int16) if bd == 10 else plane).cuda()


def test_table_sa8d(oracle, setup):
    """TEST_PIXEL( sa8d, 1 ) (checkasm.c:384-421)."""
    bd, b, pixf = setup
    for i in (0, 3):
        fn = pixf.sa8d[i]
        assert fn
        for j in range(0, 64, 3):
            s1 = 32 if (j & 31) == 31 else 16
            assert fn(_p(b.pbuf1), s1, _p(b.pbuf1, b.pbuf2_off), 64) == \
                oracle.sa8d(bd, i, b.pbuf1, 0, s1, b.pbuf1, b.pbuf2_off, 64)
        for j in range(0, 0x1000, 256):
            assert fn(_p(b.pbuf3, j), 16, _p(b.pbuf4, j), 16) == oracle.sa8d(bd, i, b.pbuf3, j, 16, b.pbuf4, j, 16)


def test_table_sa8d_satd(oracle, setup):
    """checkasm.c:424-460: (cost8, cost4) = (sa8d_16x16, satd_16x16)."""
    bd, b, pixf = setup
    fn = pixf.sa8d_satd[0]
    assert fn
    for j in range(0, 64, 7):
        assert fn(_p(b.pbuf1), 16, _p(b.pbuf1, b.pbuf2_off + j), 64) == \
            oracle.sa8d_satd(bd, b.pbuf1, 0, 16, b.pbuf1, b.pbuf2_off + j, 64)
    for j in range(0, 0x1000, 256):
        assert fn(_p(b.pbuf3, j), 16, _p(b.pbuf4, j), 16) == oracle.sa8d_satd(bd, b.pbuf3, j, 16, b.pbuf4, j, 16)


def test_table_var_hadamard_ac(oracle, setup):
    """TEST_PIXEL_VAR (checkasm.c:503-528) and hadamard_ac (:555-580)."""
    bd, b, pixf = setup
    for i in (0, 2, 3):
        for buf, off in ((b.pbuf1, 0), (b.pbuf1, 77), (b.pbuf3, 256)):
            assert pixf.var[i](_p(buf, off), 16) == oracle.var(bd, i, buf, off, 16), (i, off)
    for i in range(4):
        w, h = nr.SIZES[i]
        for j in range(32):
            buf = b.pbuf1 if j & 16 else b.pbuf3
            off = (j & 15) * 256
            if off + 16 * (h - 1) + w > buf.size:
                continue
            assert pixf.hadamard_ac[i](_p(buf, off), 16) == oracle.hadamard_ac(bd, i, buf, off, 16), (i, j)


def test_table_var2(oracle, setup):
    """TEST_PIXEL_VAR2 (checkasm.c:530-551)."""
    bd, b, pixf = setup
    for i in (2, 3):
        for fo, do in ((0, b.pbuf2_off), (64, b.pbuf2_off + 5)):
            ssd = (ctypes.c_int * 2)()
            r = pixf.var2[i](_p(b.pbuf1, fo), _p(b.pbuf1, do), ssd)
            assert (r, ssd[0], ssd[1]) == oracle.var2(bd, i, b.pbuf1, fo, b.pbuf1, do), (i, fo)


def test_table_vsad_asd8(oracle, setup):
    """vsad heights 2..32 (checkasm.c:582-605), asd8 height 16 (:607-619)."""
    bd, b, pixf = setup
    alt = np.fromfunction(lambda i, j: (((i + j) % 2) * b.pixel_max), (32, 16), dtype=np.int64)
    alt = alt.astype(oracle.pixel_dtype(bd)).ravel()
    for h in range(2, 33, 2):
        for buf in (b.pbuf1, alt):
            assert pixf.vsad(_p(buf), 16, h) == oracle.vsad(bd, buf, 0, 16, h), h
    for off in (0, 3):
        assert pixf.asd8(_p(b.pbuf1, off), 8, _p(b.pbuf1, b.pbuf2_off + off), 8, 16) == \
            oracle.asd8(bd, b.pbuf1, off, 8, b.pbuf1, b.pbuf2_off + off, 8, 16)


def test_table_ads(oracle, setup):
    """esa ads (checkasm.c:823-873), every slot incl. the aliased ones, delta 32, width 28."""
    bd, b, pixf = setup
    pm = b.pixel_max
    cb.srand(777 + bd)
    cost = np.array([cb.rand30() & 0xFFFF for _ in range(32)], np.uint16)
    for i in range(70):
        slot = i % 7
        ns = (4, 2, 2, 1, 2, 2, 1)[slot]
        thresh = (cb.rand() % 257) * pm + (cb.rand30() & 0xFFFF)
        if i < 28:
            sums = np.array([(cb.rand() % 9) * 8 * pm for _ in range(72)], np.int64).astype(np.uint16)
            dc = np.array([(cb.rand() % 9) * 8 * pm for _ in range(4)], np.int32)
        else:
            sums = np.array([cb.rand30() & ((1 << (bd + 6)) - 1) for _ in range(72)], np.uint16)
            dc = np.array([cb.rand30() & ((1 << (bd + 6)) - 1) for _ in range(4)], np.int32)
        mvs = np.zeros(48, np.int16)
        n = pixf.ads[slot](_p(dc), _p(sums), 32, _p(cost), _p(mvs), 28, thresh)
        want = oracle.ads(bd, ns, dc, sums, 0, 32, cost, 0, 28, thresh)
        assert n == len(want) and np.array_equal(mvs[:n], want), (slot, i)


@pytest.mark.parametrize("bd", [8, 10])
def test_cmp_batch_sa8d_random(hip, oracle, bd):
    rs = np.random.default_rng(40 + bd)
    pdt = np.uint8 if bd == 8 else np.uint16
    plane = rs.integers(0, 1 << bd, size=1 << 20).astype(pdt)
    dev = _dev(plane, bd)
    for i_pixel in (0, 3):
        n = 3000
        fs, rsd = int(rs.integers(16, 300)), int(rs.integers(16, 300))
        fo = rs.integers(0, (1 << 20) - 17 * max(fs, rsd), size=n).astype(np.int64)
        ro = rs.integers(0, (1 << 20) - 17 * max(fs, rsd), size=n).astype(np.int64)
        got = hip.pixel_cmp_batch(hip.CMP_SA8D, i_pixel, dev, fs, dev, rsd, torch.from_numpy(fo).cuda(),
                                  torch.from_numpy(ro).cuda()).cpu().numpy()
        want = [oracle.sa8d(bd, i_pixel, plane, a, fs, plane, c, rsd) for a, c in zip(fo, ro)]
        assert np.array_equal(got, np.array(want, np.int32)), i_pixel


@pytest.mark.parametrize("bd", [8, 10])
def test_stat_batch_random(hip, oracle, bd):
    """var / hadamard_ac / sa8d_satd / vsad / asd8 over random block lists (any alignment)."""
    rs = np.random.default_rng(50 + bd)
    pdt = np.uint8 if bd == 8 else np.uint16
    plane = rs.integers(0, 1 << bd, size=1 << 18).astype(pdt)
    plane[:4096] = np.where(rs.integers(0, 2, 4096) > 0, (1 << bd) - 1, 0)     # maxed region
    dev = _dev(plane, bd)
    n = 1500
    s1, s2 = int(rs.integers(16, 200)), int(rs.integers(16, 200))
    o1 = rs.integers(0, (1 << 18) - 34 * max(s1, s2), size=n).astype(np.int64)
    o2 = rs.integers(0, (1 << 18) - 34 * max(s1, s2), size=n).astype(np.int64)
    o1[:50] = rs.integers(0, 2048, 50)
    d1, d2 = torch.from_numpy(o1).cuda(), torch.from_numpy(o2).cuda()

    def run(op, i_pixel, height=0):
        r = hip.pixel_stat_batch(op, i_pixel, dev, s1, d1, dev, s2, d2, height).cpu().numpy()
        return r.view(np.uint64)

    for i in (0, 2, 3):
        want = [oracle.var(bd, i, plane, a, s1) for a in o1]
        assert np.array_equal(run(hip.STAT_VAR, i), np.array(want, np.uint64)), ("var", i)
    for i in range(4):
        want = [oracle.hadamard_ac(bd, i, plane, a, s1) for a in o1]
        assert np.array_equal(run(hip.STAT_HADAMARD_AC, i), np.array(want, np.uint64)), ("hadamard_ac", i)
    want = [oracle.sa8d_satd(bd, plane, a, s1, plane, c, s2) for a, c in zip(o1, o2)]
    assert np.array_equal(run(hip.STAT_SA8D_SATD, 0), np.array(want, np.uint64))
    for h in (2, 9, 32):
        want = [oracle.vsad(bd, plane, a, s1, h) for a in o1]
        assert np.array_equal(run(hip.STAT_VSAD, 0, h), np.array(want, np.uint64)), ("vsad", h)
        want = [oracle.asd8(bd, plane, a, s1, plane, c, s2, h) for a, c in zip(o1, o2)]
        assert np.array_equal(run(hip.STAT_ASD8, 3, h), np.array(want, np.uint64)), ("asd8", h)


@pytest.mark.parametrize("bd", [8, 10])
def test_var2_batch_random(hip, oracle, bd):
    rs = np.random.default_rng(60 + bd)
    pdt = np.uint8 if bd == 8 else np.uint16
    plane = rs.integers(0, 1 << bd, size=1 << 18).astype(pdt)
    dev = _dev(plane, bd)
    n = 2000
    fs, ds = int(rs.integers(24, 100)), int(rs.integers(24, 100))
    fvd, dvd = int(rs.integers(8, 500)), int(rs.integers(8, 500))
    fo = rs.integers(0, (1 << 18) - 17 * max(fs, ds) - 600, size=n).astype(np.int64)
    do = rs.integers(0, (1 << 18) - 17 * max(fs, ds) - 600, size=n).astype(np.int64)
    for i in (2, 3):
        got = hip.var2_batch(i, dev, fs, fvd, dev, ds, dvd, torch.from_numpy(fo).cuda(),
                             torch.from_numpy(do).cuda()).cpu().numpy()
        h = nr.SIZES[i][1]
        want = np.array([oracle.var2_s(bd, h, plane, a, fs, fvd, plane, c, ds, dvd) for a, c in zip(fo, do)],
                        np.int32)
        assert np.array_equal(got, want), i


@pytest.mark.parametrize("bd", [8, 10])
def test_ads_batch_random(hip, oracle, bd):
    """n independent ads calls with per-call offsets, widths (incl. > 64 and 0) and thresholds."""
    rs = np.random.default_rng(70 + bd)
    sums = rs.integers(0, 1 << (bd + 6), size=1 << 16).astype(np.uint16)
    cost = rs.integers(0, 1 << 10, size=4096).astype(np.uint16)
    n = 600
    delta = 1024
    width = rs.integers(0, 200, size=n).astype(np.int32)
    width[:3] = (0, 64, 128)
    so = rs.integers(0, (1 << 16) - delta - 220, size=n).astype(np.int64)
    co = rs.integers(0, 4096 - 220, size=n).astype(np.int64)
    dc = rs.integers(0, 1 << (bd + 6), size=(n, 4)).astype(np.int32)
    thresh = rs.integers(0, 4 << (bd + 6), size=n).astype(np.int32)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    for i_pixel, ns in ((0, 4), (1, 2), (3, 1)):
        mvs, nmv = hip.ads_batch(bd, i_pixel, T(dc.ravel()), T(sums.view(np.int16)), delta, T(so),
                                 T(cost.view(np.int16)), T(co), T(width), T(thresh), mvs_pitch=200)
        mvs, nmv = mvs.cpu().numpy(), nmv.cpu().numpy()
        for k in range(n):
            want = oracle.ads(bd, ns, dc[k], sums, so[k], delta, cost, co[k], int(width[k]), int(thresh[k]))
            assert nmv[k] == len(want) and np.array_equal(mvs[k, :nmv[k]], want), (i_pixel, k)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("sub8x8", [False, True])
@pytest.mark.parametrize("W,H,variant", [(176, 144, None), (176, 144, 1), (1920, 1088, None)])
def test_frame_integral(hip, oracle, bd, sub8x8, W, H, variant):
    """whole padded frames (edge-replicated borders, maxed corner), 3 frames per call, against
    the reference's integral_init loop restated (rows [1-PADV, lines+PADV-8), cols [-PADH, stride-PADH-8));
    the dword-lane kernel (default) and the column-per-lane one (X264HIP_INTEGRAL_VARIANT=1)."""
    from x264hip import synth
    if variant is not None:
        hip.set_variant("X264HIP_INTEGRAL_VARIANT", variant)
    n = 3
    planes, stride, origin = synth.make_sequence(n, W, H, bd, start=5)
    planes[1, 40:60, 40:80] = (1 << bd) - 1
    dev = _dev(planes, bd)
    got = hip.frame_integral(dev, origin, stride, H, sub8x8=sub8x8).cpu().numpy().view(np.uint16)
    r1 = H + 64 - 8
    for f in range(n):
        want = oracle.frame_integral(bd, planes[f].ravel(), origin, stride, H, 32, int(sub8x8))
        assert np.array_equal(got[f, 1:r1, :stride - 8], want[1:r1, :stride - 8]), f
        if sub8x8:
            o = H + 64
            assert np.array_equal(got[f, o + 1:o + r1, :stride - 8], want[o + 1:o + r1, :stride - 8]), f
