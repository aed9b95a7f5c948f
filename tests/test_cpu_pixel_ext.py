"""CPU: the oracle's further x264_pixel_function_t entries (sa8d, sa8d_satd,
hadamard_ac, var, var2, vsad, asd8, ads) and the frame integral image against
the independent numpy restatement, on the reference's checkasm patterns
(tools/checkasm.c:384-417, 424-460, 503-620, 823-873).  No GPU involved."""
import numpy as np
import pytest

import checkasm_bufs as cb
import numpy_ref as nr


@pytest.fixture(scope="module", params=[8, 10])
def bufs(request):
    b = cb.Bufs(request.param)
    b.fill_pixel_overflow()
    return b


def test_sa8d_checkasm(oracle, bufs):
    """TEST_PIXEL( sa8d, 1 ): aligned pbuf2 (stride 64) vs pbuf1, then the overflow patterns."""
    bd, p1 = bufs.bd, bufs.pbuf1
    for i in (0, 3):
        w, h = nr.SIZES[i]
        for j in range(64):
            s1 = 32 if (j & 31) == 31 else 16
            got = oracle.sa8d(bd, i, p1, 0, s1, p1, bufs.pbuf2_off, 64)
            assert got == nr.sa8d(nr.block(p1, 0, s1, w, h), nr.block(p1, bufs.pbuf2_off, 64, w, h)), (i, j)
        for j in range(0, 0x1000, 256):
            got = oracle.sa8d(bd, i, bufs.pbuf3, j, 16, bufs.pbuf4, j, 16)
            assert got == nr.sa8d(nr.block(bufs.pbuf3, j, 16, w, h), nr.block(bufs.pbuf4, j, 16, w, h)), (i, j)
    # unaligned offsets too (the GPU entries take any offset)
    for j in range(64):
        got = oracle.sa8d(bd, 0, p1, j, 16, p1, bufs.pbuf2_off + j, 64)
        assert got == nr.sa8d(nr.block(p1, j, 16, 16, 16), nr.block(p1, bufs.pbuf2_off + j, 64, 16, 16))


def test_sa8d_satd_contract(oracle, bufs):
    """checkasm.c:424-460: low half = sa8d_16x16, high half = satd_16x16."""
    bd, p1 = bufs.bd, bufs.pbuf1
    cases = [(p1, 0, 16, p1, bufs.pbuf2_off + j, 64) for j in range(64)]
    cases += [(bufs.pbuf3, j, 16, bufs.pbuf4, j, 16) for j in range(0, 0x1000, 256)]
    for a, ao, sa, b, bo, sb in cases:
        got = oracle.sa8d_satd(bd, a, ao, sa, b, bo, sb)
        A, B = nr.block(a, ao, sa, 16, 16), nr.block(b, bo, sb, 16, 16)
        assert got & 0xFFFFFFFF == nr.sa8d(A, B) and got >> 32 == nr.satd(A, B)


def test_hadamard_ac_checkasm(oracle, bufs):
    """checkasm.c:555-580: pix = (j&16 ? pbuf1 : pbuf3) + (j&15)*256, stride 16."""
    bd = bufs.bd
    for i in range(4):
        w, h = nr.SIZES[i]
        for j in range(32):
            buf = bufs.pbuf1 if j & 16 else bufs.pbuf3
            off = (j & 15) * 256
            if off + 16 * (h - 1) + w > buf.size:
                continue
            got = oracle.hadamard_ac(bd, i, buf, off, 16)
            assert got == nr.hadamard_ac(nr.block(buf, off, 16, w, h)), (i, j)
    # maxed checkerboards
    pm = bufs.pixel_max
    for pat in range(4):
        p = np.fromfunction(lambda y, x: ((((y >> pat) + (x >> pat)) & 1) * pm), (16, 16), dtype=np.int64)
        p = p.astype(oracle.pixel_dtype(bd)).ravel()
        for i in range(4):
            w, h = nr.SIZES[i]
            assert oracle.hadamard_ac(bd, i, p, 0, 16) == nr.hadamard_ac(nr.block(p, 0, 16, w, h))


def test_var_checkasm(oracle, bufs):
    """TEST_PIXEL_VAR (checkasm.c:503-528) plus all-max blocks."""
    bd = bufs.bd
    pm = np.full(256, bufs.pixel_max, oracle.pixel_dtype(bd))
    for i in (0, 2, 3):
        w, h = nr.SIZES[i]
        for buf, off in ((bufs.pbuf1, 0), (bufs.pbuf1, 77), (bufs.pbuf3, 256), (pm, 0)):
            assert oracle.var(bd, i, buf, off, 16) == nr.var(nr.block(buf, off, 16, w, h)), (i, off)


def test_var2_checkasm(oracle, bufs):
    """TEST_PIXEL_VAR2 (checkasm.c:530-551): var2(pbuf1, pbuf2, ssd), fenc stride 16 / fdec 32."""
    bd, p1 = bufs.bd, bufs.pbuf1
    for i in (2, 3):
        h = nr.SIZES[i][1]
        for fo, do in ((0, bufs.pbuf2_off), (64, bufs.pbuf2_off + 5)):
            got = oracle.var2(bd, i, p1, fo, p1, do)
            want = nr.var2(nr.block(p1, fo, 16, 8, h), nr.block(p1, do, 32, 8, h),
                           nr.block(p1, fo + 8, 16, 8, h), nr.block(p1, do + 16, 32, 8, h), h)
            assert got == want, (i, fo)
        # maximal differences
        a = np.full(16 * 16, bufs.pixel_max, oracle.pixel_dtype(bd))
        z = np.zeros(32 * 16, oracle.pixel_dtype(bd))
        assert oracle.var2(bd, i, a, 0, z, 0) == nr.var2(nr.block(a, 0, 16, 8, h), nr.block(z, 0, 32, 8, h),
                                                          nr.block(a, 8, 16, 8, h), nr.block(z, 16, 32, 8, h), h)


def test_vsad_asd8_checkasm(oracle, bufs):
    """vsad heights 2..32 over pbuf1 and the alternating max pattern (checkasm.c:582-605);
    asd8(pbuf1, 8, pbuf2, 8, 16) (checkasm.c:607-619)."""
    bd = bufs.bd
    alt = np.fromfunction(lambda i, j: (((i + j) % 2) * bufs.pixel_max), (32, 16), dtype=np.int64)
    alt = alt.astype(oracle.pixel_dtype(bd)).ravel()
    for h in range(2, 33, 2):
        for buf in (bufs.pbuf1, alt):
            got = oracle.vsad(bd, buf, 0, 16, h)
            b = nr.block(buf, 0, 16, 16, h)
            assert got == int(np.abs(b[1:] - b[:-1]).sum()), h
    for off in (0, 3):
        got = oracle.asd8(bd, bufs.pbuf1, off, 8, bufs.pbuf1, bufs.pbuf2_off + off, 8, 16)
        want = abs(int((nr.block(bufs.pbuf1, off, 8, 8, 16) - nr.block(bufs.pbuf1, bufs.pbuf2_off + off, 8, 8, 16)).sum()))
        assert got == want


def random_frame(bd, width, lines, seed, pad=32):
    """x264-style padded luma plane (edge replication, frame.c:599-625 semantics), stride
    align64(width + 2*pad); returns (flat plane, stride, origin of (0,0), lines)."""
    stride = (width + 2 * pad + 63) // 64 * 64
    rs = np.random.default_rng(seed)
    core = rs.integers(0, 1 << bd, size=(lines, width))
    full = np.pad(core, ((pad, pad), (pad, stride - width - pad)), mode="edge")
    dt = np.uint8 if bd == 8 else np.uint16
    return full.astype(dt).ravel(), stride, pad * stride + pad, lines


def _np_ads(nsums, dc, sums, s_off, delta, cost, c_off, width, thresh):
    i = np.arange(width)
    s = sums.astype(np.int64)
    a = np.abs(dc[0] - s[s_off + i])
    if nsums == 4:
        a = a + np.abs(dc[1] - s[s_off + i + 8]) + np.abs(dc[2] - s[s_off + i + delta]) \
            + np.abs(dc[3] - s[s_off + i + delta + 8])
    elif nsums == 2:
        a = a + np.abs(dc[1] - s[s_off + i + delta])
    a = a + cost[c_off + i].astype(np.int64)
    return i[a < thresh].astype(np.int16)


@pytest.mark.parametrize("bd", [8, 10])
def test_ads_checkasm_distribution(oracle, bd):
    """esa ads (checkasm.c:823-873): same generator (glibc rand) and value distributions,
    sums[72], delta 32, width 28; ads4 / ads2 / ads1 (table slots 16x16 / 16x8 / 8x8)."""
    pm = (1 << bd) - 1
    cb.srand(4321)
    cost = np.array([cb.rand30() & 0xFFFF for _ in range(32)], np.uint16)
    for i in range(100):
        nsums = (4, 2, 2, 1)[i & 3]
        thresh = (cb.rand() % 257) * pm + (cb.rand30() & 0xFFFF)
        if i < 40:
            sums = np.array([(cb.rand() % 9) * 8 * pm for _ in range(72)], np.int64).astype(np.uint16)
            dc = np.array([(cb.rand() % 9) * 8 * pm for _ in range(4)], np.int32)
        else:
            r = cb.rand30 if bd + 6 > 15 else cb.rand
            sums = np.array([r() & ((1 << (bd + 6)) - 1) for _ in range(72)], np.uint16)
            dc = np.array([r() & ((1 << (bd + 6)) - 1) for _ in range(4)], np.int32)
        got = oracle.ads(bd, nsums, dc, sums, 0, 32, cost, 0, 28, thresh)
        want = _np_ads(nsums, dc, sums, 0, 32, cost, 0, 28, thresh)
        assert np.array_equal(got, want), i


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("sub8x8", [0, 1])
def test_frame_integral_box_sums(oracle, bd, sub8x8):
    """x264_frame_filter's integral (mc.c:748-782): rows [1-PADV, lines+PADV-8) hold 8x8 box sums
    (and 4x4 box sums in the second plane when sub8x8) for columns [-PADH_ALIGN, stride-PADH_ALIGN-8)."""
    plane, stride, origin, lines = random_frame(bd, 64, 48, seed=3 + sub8x8)
    pad, padh = 32, 32
    buf = oracle.frame_integral(bd, plane, origin, stride, lines, padh, sub8x8)
    p2 = plane.reshape(-1, stride).astype(np.int64)           # rows [-32, lines+32), cols [-32, stride-32)
    b8 = nr.box_sums(p2, 8)                                   # top-left (row r, col c) in buffer coords
    r0, r1 = 1, lines + 2 * pad - 8                           # integral rows 1-PADV .. lines+PADV-9
    c1 = stride - 8
    assert np.array_equal(buf[r0:r1, :c1], b8[r0:r1, :c1])
    if sub8x8:
        b4 = nr.box_sums(p2, 4)
        off = lines + 2 * pad
        assert np.array_equal(buf[off + r0:off + r1, :c1], b4[r0:r1, :c1])
