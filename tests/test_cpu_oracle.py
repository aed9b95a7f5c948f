"""CPU: the oracle (reference loops restated in C, oracle/oracle.c) against the
independent numpy matrix-form restatement (tests/numpy_ref.py), on the
reference's own checkasm input patterns (tools/checkasm.c) for 8 and 10 bit.
No GPU involved."""
import numpy as np
import pytest

import checkasm_bufs as cb
import numpy_ref as nr

OPS = {"sad": nr.sad, "ssd": nr.ssd, "satd": nr.satd}


@pytest.fixture(scope="module", params=[8, 10])
def bufs(request):
    b = cb.Bufs(request.param)
    b.fill_pixel_overflow()
    return b


@pytest.mark.parametrize("op", ["sad", "ssd", "satd"])
def test_pixel_metrics_checkasm(oracle, bufs, op):
    """TEST_PIXEL (checkasm.c:384-417): 64 offsets of pbuf2 (stride 64) vs pbuf1
    (stride 16, or 32 every 32nd), then the overflow patterns pbuf3/pbuf4."""
    bd, p1 = bufs.bd, bufs.pbuf1
    for i, (w, h) in enumerate(nr.SIZES):
        for j in range(64):
            s1 = 32 if (j & 31) == 31 else 16
            got = oracle.cmp(bd, op, i, p1, 0, s1, p1, bufs.pbuf2_off + j, 64)
            want = OPS[op](nr.block(p1, 0, s1, w, h), nr.block(p1, bufs.pbuf2_off + j, 64, w, h))
            assert got == want, (op, i, j)
        for j in range(0, 0x1000, 256):
            got = oracle.cmp(bd, op, i, bufs.pbuf3, j, 16, bufs.pbuf4, j, 16)
            want = OPS[op](nr.block(bufs.pbuf3, j, 16, w, h), nr.block(bufs.pbuf4, j, 16, w, h))
            assert got == want, (op, i, "overflow", j)


@pytest.mark.parametrize("op", ["sad", "satd"])
@pytest.mark.parametrize("n", [3, 4])
def test_pixel_x_checkasm(oracle, bufs, op, n):
    """TEST_PIXEL_X (checkasm.c:462-502): refs pix2, pix2+6, pix2+1, pix2+10, stride 64."""
    bd, p1 = bufs.bd, bufs.pbuf1
    for i, (w, h) in enumerate(nr.SIZES[:7]):
        for j in range(64):
            base = bufs.pbuf2_off + j
            offs = [base, base + 6, base + 1, base + 10][:n]
            got = oracle.cmp_x(bd, op, n, i, p1, 0, p1, offs, 64)
            want = [OPS[op](nr.block(p1, 0, 16, w, h), nr.block(p1, o, 64, w, h)) for o in offs]
            assert list(got) == want, (op, n, i, j)


def test_satd_coefficient_parity():
    """Every 4x4 Hadamard coefficient has the parity of the block's difference sum,
    so sum|coef| is even: SATD's >>1 per 8x4 pair equals >>1 per 4x4 tile."""
    rs = np.random.default_rng(0)
    d = rs.integers(-1023, 1024, size=(20000, 4, 4))
    coef = np.einsum("ij,bjk,lk->bil", nr.H4, d, nr.H4)
    assert (np.abs(coef).sum(axis=(1, 2)) % 2 == 0).all()


def _dct_inputs(b):
    """(fenc, fenc_off, fdec, fdec_off) pairs used by TEST_DCT (checkasm.c:930-966)."""
    out = []
    for j in range(5):
        out.append((b.pbuf1, j * 64, b.pbuf1, b.pbuf2_off + j * 64))
        out.append((b.pbuf3, 16 * j * 16, b.pbuf4, 16 * j * 32))
    return out


DCT_SHAPES = {"sub4x4_dct": (4, 4), "sub8x8_dct": (8, 8), "sub16x16_dct": (16, 16), "sub8x8_dct_dc": (8, 8),
              "sub8x16_dct_dc": (8, 16), "sub8x8_dct8": (8, 8), "sub16x16_dct8": (16, 16)}
NP_DCT = {"sub4x4_dct": lambda d, bd: nr.sub4x4_dct(d, bd), "sub8x8_dct": nr.sub8x8_dct,
          "sub16x16_dct": nr.sub16x16_dct, "sub8x8_dct_dc": nr.sub8x8_dct_dc,
          "sub8x16_dct_dc": nr.sub8x16_dct_dc, "sub8x8_dct8": nr.sub8x8_dct8, "sub16x16_dct8": nr.sub16x16_dct8}


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("name", list(DCT_SHAPES))
def test_sub_dct_checkasm(oracle, bd, name):
    b = cb.Bufs(bd)
    b.fill_dct_overflow()
    w, h = DCT_SHAPES[name]
    for (a, ao, d, do) in _dct_inputs(b):
        got = oracle.sub_dct(bd, name, a, ao, d, do)
        diff = nr.block(a, ao, 16, w, h) - nr.block(d, do, 32, w, h)
        want = NP_DCT[name](diff, bd)
        assert np.array_equal(got.astype(np.int64), want.ravel()), (name, ao)


@pytest.mark.parametrize("bd", [8, 10])
def test_dct4x4dc_checkasm(oracle, bd):
    """TEST_DCTDC (checkasm.c:1034-1058): max DC, max elements, general case."""
    b = cb.Bufs(bd)
    pm = (1 << bd) - 1
    p = b.buf1.view(np.uint16)
    k = 0
    for i in range(16):
        d = np.zeros(16, np.int64)
        for j in range(16):
            if i == 0:
                d[j] = pm * 16 if (j ^ j >> 1 ^ j >> 2 ^ j >> 3) & 1 else -pm * 16
            elif i < 8:
                d[j] = pm * 16 if p[k] & 1 else -pm * 16
                k += 1
            else:
                d[j] = (int(p[k]) & 0x1FFF) - 0x1000
                k += 1
        got = oracle.dct4x4dc(bd, d)
        assert np.array_equal(got.astype(np.int64), nr.dct4x4dc(d, bd)[0]), i


@pytest.mark.parametrize("bd", [8, 10])
def test_dct2x4dc(oracle, bd):
    rs = np.random.default_rng(bd)
    pm = (1 << bd) - 1
    for t in range(50):
        src = rs.integers(-pm * 16, pm * 16 + 1, size=(8, 16))
        if t == 0:
            src[:, 0] = pm * 16
        out, zeroed = oracle.dct2x4dc(bd, src)
        a = src[:, 0].astype(np.int64)
        H = np.array([[1, 1, 1, 1, 1, 1, 1, 1], [1, -1, 1, -1, 1, -1, 1, -1], [1, 1, 1, 1, -1, -1, -1, -1],
                      [1, -1, 1, -1, -1, 1, -1, 1], [1, 1, -1, -1, -1, -1, 1, 1], [1, -1, -1, 1, -1, 1, 1, -1],
                      [1, 1, -1, -1, 1, 1, -1, -1], [1, -1, -1, 1, 1, -1, -1, 1]])
        assert np.array_equal(out.astype(np.int64), nr.wrap(H @ a, bd))
        assert (zeroed[:, 0] == 0).all() and np.array_equal(zeroed[:, 1:], src[:, 1:])


@pytest.mark.parametrize("bd", [8, 10])
def test_cqm_init_all_configs(oracle, bd):
    """x264_cqm_init for the six check_quant CQMs (checkasm.c:2098-2140)."""
    cb.srand(cb.SEED)
    for i_cqm in range(6):
        lists = cb.cqm_lists(i_cqm, bd)
        got = oracle.cqm_init(bd, lists)
        want = nr.cqm_init(bd, lists)
        for g, w, name in zip(got, want, ("q4mf", "q4bias", "q8mf", "q8bias")):
            assert np.array_equal(g, w), (i_cqm, name)


@pytest.mark.parametrize("bd", [8, 10])
def test_quant_checkasm(oracle, bd):
    """TEST_QUANT / TEST_QUANT_DC (checkasm.c:2169-2226) over all CQMs and every QP."""
    cb.srand(cb.SEED + bd)
    qmax = 51 + 6 * (bd - 8)
    for i_cqm in range(6):
        q4m, q4b, q8m, q8b = oracle.cqm_init(bd, cb.cqm_lists(i_cqm, bd))
        for qp in range(qmax, -1, -1):
            for lst in (0, 1):                      # CQM_?IY, CQM_?PY
                for j in range(2):
                    c = cb.init_quant8(j, bd)
                    got, nz = oracle.quant(bd, "quant_8x8", c, q8m[lst, qp], q8b[lst, qp])
                    want, wnz = nr.quant(c, q8m[lst, qp], q8b[lst, qp], bd)
                    assert np.array_equal(got, want) and nz == int(wnz), (i_cqm, qp, "8x8")
                    c = cb.init_quant4(j, 16, bd)
                    got, nz = oracle.quant(bd, "quant_4x4", c, q4m[lst, qp], q4b[lst, qp])
                    want, wnz = nr.quant(c, q4m[lst, qp], q4b[lst, qp], bd)
                    assert np.array_equal(got, want) and nz == int(wnz), (i_cqm, qp, "4x4")
                if qp % 7 == 0:
                    for j in range(16):
                        c = cb.init_quant4(j, 64, bd)
                        got, nz = oracle.quant(bd, "quant_4x4x4", c, q4m[lst, qp], q4b[lst, qp])
                        want, wnz = nr.quant(c.reshape(4, 16), q4m[lst, qp], q4b[lst, qp], bd)
                        mask = sum(int(v) << k for k, v in enumerate(wnz))
                        assert np.array_equal(got, want.ravel()) and nz == mask, (i_cqm, qp, "4x4x4", j)
            for name, n, lst in (("quant_4x4_dc", 16, 0), ("quant_2x2_dc", 4, 2)):
                for j in range(2):
                    c = np.array([(cb.rand() & 0x1FFF) - 0xFFF if j else 0 for _ in range(n)])
                    mf, bias = int(q4m[lst, qp, 0]), int(q4b[lst, qp, 0])
                    got, nz = oracle.quant(bd, name, c, mf, bias)
                    want, wnz = nr.quant(c, mf, bias, bd)
                    assert np.array_equal(got, want) and nz == int(wnz), (i_cqm, qp, name)


@pytest.mark.parametrize("bd", [8, 10])
def test_me_search_full_small(oracle, bd):
    """frame-level exhaustive search table vs numpy (every candidate)."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "synth", os.path.join(os.path.dirname(__file__), "..", "x264-i386pic_amd", "synth.py"))
    synth = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(synth)
    planes, stride, origin = synth.random_planes(2, 32, 32, bd, seed=bd)
    r = 6 if bd == 8 else 4
    got = oracle.me_search_full(bd, planes[1].ravel(), origin, stride, planes[0].ravel(), origin, stride, 2, 2, r)
    f = planes[1].ravel()
    g = planes[0].ravel()
    for mby in range(2):
        for mbx in range(2):
            a = nr.block(f, origin + 16 * (mby * stride + mbx), stride, 16, 16)
            for j in range(2 * r + 1):
                for i in range(2 * r + 1):
                    o = origin + (16 * mby + j - r) * stride + 16 * mbx + i - r
                    assert got[mby, mbx, j, i] == nr.sad(a, nr.block(g, o, stride, 16, 16))


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("transform", [4, 8])
def test_mb_dct_quant_small(oracle, bd, transform):
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "synth", os.path.join(os.path.dirname(__file__), "..", "x264-i386pic_amd", "synth.py"))
    synth = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(synth)
    planes, stride, origin = synth.make_sequence(2, 48, 32, bd)
    q4m, q4b, q8m, q8b = oracle.cqm_init(bd, [cb.FLAT16] * 8)
    mf, bias = (q4m[1, 20], q4b[1, 20]) if transform == 4 else (q8m[1, 20], q8b[1, 20])
    dct, nz = oracle.mb_dct_quant(bd, transform, planes[1].ravel(), origin, stride, planes[0].ravel(), origin,
                                  stride, 3, 2, mf, bias)
    f, p = planes[1].ravel(), planes[0].ravel()
    for mby in range(2):
        for mbx in range(3):
            o = origin + 16 * (mby * stride + mbx)
            d = nr.block(f, o, stride, 16, 16) - nr.block(p, o, stride, 16, 16)
            c = nr.sub16x16_dct(d, bd) if transform == 4 else nr.sub16x16_dct8(d, bd)
            if transform == 4:
                q, z = nr.quant(c.reshape(16, 16), mf, bias, bd)
                mask = sum(int(v) << k for k, v in enumerate(z))
            else:
                q, z = nr.quant(c.reshape(4, 64), mf, bias, bd)
                mask = sum(int(v) << k for k, v in enumerate(z))
            mb = mby * 3 + mbx
            assert np.array_equal(dct[mb].astype(np.int64), q.ravel()) and nz[mb] == mask, (mby, mbx)


def _synth():
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "synth", os.path.join(os.path.dirname(__file__), "..", "x264-i386pic_amd", "synth.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("bd", [8, 10])
def test_frame_filter_and_subpel(oracle, bd):
    """half-pel planes (oracle loops vs vectorised numpy) and qpel get_ref costs."""
    synth = _synth()
    W, H = 48, 32
    planes, stride, origin = synth.random_planes(2, W, H, bd, seed=bd)
    p = planes[0]
    hvc = oracle.frame_filter(bd, p.ravel().copy(), origin, stride, W, H)
    want = nr.hpel_planes(p, 32, W, H, bd)
    for a, b in zip(hvc, want):
        assert np.array_equal(a.reshape(p.shape)[:, :W + 64], b[:, :W + 64])
    flat = [p.ravel()] + [x for x in hvc]
    rs = np.random.default_rng(bd)
    for i_pixel in (0, 3, 6):
        w, h = nr.SIZES[i_pixel]
        qxy, fo = [], []
        for _ in range(200):
            bx, by = int(rs.integers(0, W - w + 1)), int(rs.integers(0, H - h + 1))
            qxy.append((4 * bx + int(rs.integers(-40, 41)), 4 * by + int(rs.integers(-40, 41))))
            fo.append(p.size + origin + by * stride + bx)
        for op in ("sad", "satd"):
            got = oracle.subpel_list(bd, op, i_pixel, planes.ravel(), stride, flat, origin, stride, fo, qxy)
            for k, ((qx, qy), f) in enumerate(zip(qxy, fo)):
                r = nr.get_ref(flat, origin, stride, qx, qy, w, h)
                a = nr.block(planes.ravel(), f, stride, w, h)
                assert got[k] == (nr.sad(a, r) if op == "sad" else nr.satd(a, r))


def test_me_esa_argmin_vs_numpy(oracle):
    """oracle ESA decision vs a vectorised numpy restatement (argmin with first-index ties)."""
    rs = np.random.default_rng(3)
    R, me_range, nmb = 16, 12, 200
    W, P = 2 * R + 1, 36
    tab = rs.integers(0, 3000, size=(nmb, W, P)).astype(np.uint16)
    tab[::5] //= 64                                              # many ties
    i = np.arange(-4096, 4097)
    cost_mv = np.minimum(40 * (2 * np.log2(np.abs(i) + 1) + 1.718) + 0.5, 65535).astype(np.uint16)
    par = np.zeros((nmb, 8), np.int16)
    par[:, :2] = rs.integers(-1, 2, (nmb, 2))
    par[:, 2:4] = rs.integers(-40, 41, (nmb, 2))
    par[:, 4:6] = par[:, :2] - me_range + rs.integers(0, 3, (nmb, 2))
    par[:, 6:8] = par[:, :2] + me_range - rs.integers(0, 3, (nmb, 2))
    init = rs.integers(0, 3000, nmb).astype(np.int32)
    got = oracle.me_esa_argmin(8, tab, R, me_range, par, init, cost_mv, 4096)
    for k in range(nmb):
        bmx, bmy, px, py, x0, y0, x1, y1 = [int(v) for v in par[k]]
        mnx, mny = max(bmx - me_range, x0), max(bmy - me_range, y0)
        mxx, mxy = min(bmx + me_range, x1), min(bmy + me_range, y1)
        width = (mxx - mnx + 3) & ~3
        ys, xs = np.meshgrid(np.arange(mny, mxy + 1), np.arange(mnx, mnx + width), indexing="ij")
        cost = (tab[k][ys + R, xs + R].astype(np.int64) + cost_mv[4096 + 4 * xs - px] + cost_mv[4096 + 4 * ys - py])
        j = int(np.argmin(cost.ravel()))
        want = (init[k], bmx, bmy)
        if cost.ravel()[j] < init[k]:
            want = (int(cost.ravel()[j]), int(xs.ravel()[j]), int(ys.ravel()[j]))
        assert tuple(got[k]) == want, k


@pytest.mark.parametrize("bd", [8, 10])
def test_me_search_centred_oracle(oracle, bd):
    from conftest import load_package
    """centred tables: centre (0,0) equals the plain table; shifted centres equal the SADs at
    origin + (i, j) (numpy), with the origin clamped into the 32-pixel padding and aligned."""
    load_package()
    from x264hip import synth
    W, H, R = 96, 64, 8
    planes, stride, origin = synth.make_sequence(2, W, H, bd)
    mbw, mbh = W // 16, H // 16
    f, r = planes[1].ravel(), planes[0].ravel()
    plain = oracle.me_search_full(bd, f, origin, stride, r, origin, stride, mbw, mbh, R)
    tab, org = oracle.me_search_centred(bd, f, origin, stride, r, origin, stride, mbw, mbh, R,
                                        np.zeros((mbw * mbh, 2), np.int16))
    P = (2 * R + (6 if bd == 8 else 4) + 3) & ~3           # the ESA window's columns
    assert tab.shape[-1] == P
    assert np.array_equal(tab[..., :2 * R + 1], plain) and (org == -R).all()
    rs = np.random.default_rng(bd)
    cen = rs.integers(-40, 41, (mbw * mbh, 2)).astype(np.int16)
    tab, org = oracle.me_search_centred(bd, f, origin, stride, r, origin, stride, mbw, mbh, R, cen)
    al = 4 if bd == 8 else 2
    for mb in range(mbw * mbh):
        mbx, mby = mb % mbw, mb // mbw
        ax = min(max(16 * mbx + cen[mb, 0] - R, -32), 16 * mbw + 12 - P) & ~(al - 1)
        ay = min(max(16 * mby + cen[mb, 1] - R, -32), 16 * mbh + 16 - 2 * R)
        assert (org[mb, 0], org[mb, 1]) == (ax - 16 * mbx, ay - 16 * mby)
        fb = nr.block(f, origin + 16 * mby * stride + 16 * mbx, stride, 16, 16)
        for j in (0, R, 2 * R):
            for i in (0, 3, 2 * R, P - 1):
                rb = nr.block(r, origin + (ay + j) * stride + ax + i, stride, 16, 16)
                assert tab[mby, mbx, j, i] == nr.sad(fb, rb), (mb, i, j)


def test_oracle_quadrant_tables_sum_to_16x16(oracle):
    """The oracle's 8x8 quadrant tables (me_search_full8) add up to its 16x16 table: a SAD is
    additive over the four quadrants (pixel.c:55-80)."""
    from conftest import load_package
    load_package()
    from x264hip import synth
    planes, stride, origin = synth.make_sequence(2, 96, 64, 8, seed=4)
    a = oracle.me_search_full8(8, planes[1].ravel(), origin, stride, planes[0].ravel(), origin, stride, 6, 4, 8)
    b = oracle.me_search_full(8, planes[1].ravel(), origin, stride, planes[0].ravel(), origin, stride, 6, 4, 8)
    assert np.array_equal(a.astype(np.int64).sum(2), b)
