"""CPU: the oracle's inverse path (dequant, add*_idct*, idct4x4dc, idct_dequant_2x4,
optimize_chroma_dc, denoise_dct, decimate_score, coeff_last / level_run, zigzag
scan / sub / interleave, dequant tables) against independent numpy / Python
restatements, on checkasm-style inputs (tools/checkasm.c:979-1026, 2180-2330).
No GPU involved."""
import numpy as np
import pytest

import checkasm_bufs as cb
import numpy_ref as nr

FLAT = [[16] * 16] * 4 + [[16] * 64] * 4


def _coefs(oracle, bd, qp=20):
    """checkasm.c:979-993: sub16x16_dct / sub16x16_dct8 of pbuf1 vs pbuf2, quantised and
    dequantised with the flat intra-luma lists at qp 20 (forces the coefs into idct range)."""
    b = cb.Bufs(bd)
    q4m, q4b, q8m, q8b = oracle.cqm_init(bd, FLAT)
    dq4, dq8 = oracle.cqm_dequant(FLAT)
    dct4 = oracle.sub_dct(bd, "sub16x16_dct", b.pbuf1, 0, b.pbuf1, b.pbuf2_off).reshape(16, 16)
    dct8 = oracle.sub_dct(bd, "sub16x16_dct8", b.pbuf1, 0, b.pbuf1, b.pbuf2_off).reshape(4, 64)
    out4, out8 = [], []
    for i in range(16):
        d, _ = oracle.quant(bd, "quant_4x4", dct4[i], q4m[0, qp], q4b[0, qp])
        d, _ = oracle.inplace(bd, "dequant_4x4", d, oracle._addr(dq4[0]), qp)
        out4.append(d)
    for i in range(4):
        d, _ = oracle.quant(bd, "quant_8x8", dct8[i], q8m[0, qp], q8b[0, qp])
        d, _ = oracle.inplace(bd, "dequant_8x8", d, oracle._addr(dq8[0]), qp)
        out8.append(d)
    return b, np.concatenate(out4), np.concatenate(out8), dq4, dq8


@pytest.mark.parametrize("bd", [8, 10])
def test_cqm_dequant_tables(oracle, bd):
    dq4, dq8 = oracle.cqm_dequant(FLAT)
    assert dq4[0, 0, 0] == 10 * 16 and dq4[0, 5, 5] == 29 * 16 and dq8[0, 0, 0] == 20 * 16
    jvt = cb.cqm_lists(2, bd)
    dq4j, dq8j = oracle.cqm_dequant(jvt)
    for l in range(4):
        for q in range(6):
            for i in range(16):
                j = (i & 1) + ((i >> 2) & 1)
                assert dq4j[l, q, i] == [[10, 13, 16], [11, 14, 18], [13, 16, 20], [14, 18, 23], [16, 20, 25],
                                         [18, 23, 29]][q][j] * jvt[l][i]


@pytest.mark.parametrize("bd", [8, 10])
def test_dequant_all_qp(oracle, bd):
    rs = np.random.default_rng(bd)
    dq4, dq8 = oracle.cqm_dequant(cb.cqm_lists(2, bd))
    qmax = 51 + 6 * (bd - 8)
    lim = 1 << (bd + 2)
    for qp in range(qmax + 1):
        c16 = rs.integers(-lim, lim, 16)
        c64 = rs.integers(-lim, lim, 64)
        got, _ = oracle.inplace(bd, "dequant_4x4", c16, oracle._addr(dq4[1]), qp)
        assert np.array_equal(got, nr.wrap(nr.dequant(c16, dq4[1], qp, 4), bd)), qp
        got, _ = oracle.inplace(bd, "dequant_8x8", c64, oracle._addr(dq8[1]), qp)
        assert np.array_equal(got, nr.wrap(nr.dequant(c64, dq8[1], qp, 6), bd)), qp
        got, _ = oracle.inplace(bd, "dequant_4x4_dc", c16, oracle._addr(dq4[1]), qp)
        dc_mf = np.full((6, 16), 0, np.int64)
        dc_mf[:, :] = dq4[1][:, :1]
        assert np.array_equal(got, nr.wrap(nr.dequant(c16, dc_mf, qp, 6), bd)), qp


@pytest.mark.parametrize("bd", [8, 10])
def test_add_idct_checkasm(oracle, bd):
    """TEST_IDCT (checkasm.c:995-1025): pbuf3 = pbuf1 (32x32, stride 32), then each entry."""
    b, dct4, dct8, _, _ = _coefs(oracle, bd)
    pm = (1 << bd) - 1
    base = b.pbuf1[:32 * 32].copy()
    P = base.reshape(32, 32).astype(np.int64)
    # add4x4_idct vs numpy
    got, _ = oracle.add_idct(bd, "add4x4_idct", base, 0, dct4[:16])
    assert np.array_equal(got.reshape(32, 32)[:4, :4], nr.add4x4_idct(P[:4, :4], dct4[:16], bd))
    # add16x16_idct = 16 add4x4 in quadrant order
    got, _ = oracle.add_idct(bd, "add16x16_idct", base, 0, dct4)
    want = P.copy()
    for blk in range(16):
        q, k = blk // 4, blk % 4
        y, x = (q // 2) * 8 + (k // 2) * 4, (q % 2) * 8 + (k % 2) * 4
        want[y:y + 4, x:x + 4] = nr.add4x4_idct(want[y:y + 4, x:x + 4], dct4[16 * blk:16 * blk + 16], bd)
    assert np.array_equal(got.reshape(32, 32), want)
    # add8x8_idct8 / add16x16_idct8 vs numpy
    got, _ = oracle.add_idct(bd, "add16x16_idct8", base, 0, dct8)
    want = P.copy()
    for q in range(4):
        y, x = (q // 2) * 8, (q % 2) * 8
        want[y:y + 8, x:x + 8] = nr.add8x8_idct8(want[y:y + 8, x:x + 8], dct8[64 * q:64 * q + 64], bd)
    assert np.array_equal(got.reshape(32, 32), want)
    # dc forms
    got, _ = oracle.add_idct(bd, "add16x16_idct_dc", base, 0, dct4[:16])
    want = P.copy()
    for i in range(16):
        y, x = (i // 4) * 4, (i % 4) * 4
        want[y:y + 4, x:x + 4] = np.clip(want[y:y + 4, x:x + 4] + ((int(dct4[i]) + 32) >> 6), 0, pm)
    assert np.array_equal(got.reshape(32, 32), want)
    # saturation: max coefficients in both directions
    for sgn in (1, -1):
        d = np.full(64, sgn * (pm * 64), np.int64)
        got, _ = oracle.add_idct(bd, "add8x8_idct8", base, 0, nr.wrap(d, bd))
        want = nr.add8x8_idct8(P[:8, :8], nr.wrap(d, bd), bd)
        assert np.array_equal(got.reshape(32, 32)[:8, :8], want)


@pytest.mark.parametrize("bd", [8, 10])
def test_add_idct_list_matches_table(oracle, bd):
    b, dct4, dct8, _, _ = _coefs(oracle, bd)
    plane = np.tile(b.pbuf1[:1024], 4)
    offs = np.array([0, 33, 32 * 20 + 7, 2048 + 5], np.int64)
    for kind, name in enumerate(oracle.IDCT_KINDS):
        src = dct8 if "idct8" in name else dct4
        sz = oracle.IDCT_IN[kind]
        blocks = np.concatenate([np.roll(src, 7 * k)[:sz] for k in range(len(offs))])
        got = oracle.add_idct_list(bd, kind, plane, 32, offs, blocks)
        want = plane.copy()
        for k, o in enumerate(offs):
            want, _ = oracle.add_idct(bd, name, want, o, blocks[k * sz:(k + 1) * sz])
        assert np.array_equal(got, want), name


@pytest.mark.parametrize("bd", [8, 10])
def test_idct4x4dc_checkasm(oracle, bd):
    """TEST_DCTDC (checkasm.c:1028-1054) input classes: max dc, max elements, general."""
    pm = (1 << bd) - 1
    rs = np.random.default_rng(9)
    for i in range(16):
        if i == 0:
            d = np.array([pm * 16 if (j ^ j >> 1 ^ j >> 2 ^ j >> 3) & 1 else -pm * 16 for j in range(16)])
        elif i < 8:
            d = np.where(rs.integers(0, 2, 16) > 0, pm * 16, -pm * 16)
        else:
            d = rs.integers(0, 0x2000, 16) - 0x1000
        got, _ = oracle.inplace(bd, "idct4x4dc", d)
        D = d.reshape(4, 4)
        tmp = nr.wrap(nr.H4 @ D.T, bd)
        assert np.array_equal(got.reshape(4, 4), nr.wrap(tmp @ nr.H4.T, bd)), i


@pytest.mark.parametrize("bd", [8, 10])
def test_idct_dequant_2x4(oracle, bd):
    dq4, _ = oracle.cqm_dequant(FLAT)
    rs = np.random.default_rng(3)
    for qp in range(0, 52 + 6 * (bd - 8), 5):
        d = rs.integers(-200, 200, 8)
        a = np.array([d[0] + d[1], d[2] + d[3], d[4] + d[5], d[6] + d[7], d[0] - d[1], d[2] - d[3], d[4] - d[5],
                      d[6] - d[7]])
        b0, b1, b2, b3 = a[0] + a[1], a[2] + a[3], a[4] + a[5], a[6] + a[7]
        b4, b5, b6, b7 = a[0] - a[1], a[2] - a[3], a[4] - a[5], a[6] - a[7]
        dmf = int(dq4[3, qp % 6, 0]) << (qp // 6)
        want = nr.wrap((np.array([b0 + b1, b2 + b3, b0 - b1, b2 - b3, b4 - b5, b6 - b7, b4 + b5, b6 + b7]) * dmf + 32)
                       >> 6, bd)
        got, _ = oracle.inplace(bd, "idct_dequant_2x4_dconly", d, oracle._addr(dq4[3]), qp)
        assert np.array_equal(got, want), qp
        d4 = np.zeros((8, 16), oracle.coef_dtype(bd))
        d8 = np.ascontiguousarray(d, oracle.coef_dtype(bd))
        oracle.fn(bd, "idct_dequant_2x4_dc")(oracle._addr(d8), oracle._addr(d4), oracle._addr(dq4[3]), qp)
        assert np.array_equal(d4[:, 0], want) and not d4[:, 1:].any()


def _py_optimize_chroma(dct, dmf, c422):
    def idq(d):
        if c422:
            a = [d[0] + d[1], d[2] + d[3], d[4] + d[5], d[6] + d[7], d[0] - d[1], d[2] - d[3], d[4] - d[5], d[6] - d[7]]
            b = [a[0] + a[1], a[2] + a[3], a[4] + a[5], a[6] + a[7], a[0] - a[1], a[2] - a[3], a[4] - a[5], a[6] - a[7]]
            return [((v * dmf + 2080) >> 6) for v in (b[0] + b[1], b[2] + b[3], b[0] - b[1], b[2] - b[3], b[4] - b[5],
                                                      b[6] - b[7], b[4] + b[5], b[6] + b[7])]
        d0, d1, d2, d3 = d[0] + d[1], d[2] + d[3], d[0] - d[1], d[2] - d[3]
        return [((v * dmf) >> 5) + 32 for v in (d0 + d1, d0 - d1, d2 + d3, d2 - d3)]
    dct = list(dct)
    orig = idq(dct)
    s = 0
    for v in orig:
        s |= v
    if not (s >> 6):
        return 0, dct
    nz = 0
    for c in range(len(dct) - 1, -1, -1):
        level = dct[c]
        sign = -1 if level < 0 else 1
        while level:
            dct[c] = level - sign
            diff = 0
            for a, b in zip(orig, idq(dct)):
                diff |= a ^ b
            if diff >> 6:
                nz = 1
                dct[c] = level
                break
            level -= sign
    return nz, dct


@pytest.mark.parametrize("bd", [8, 10])
def test_optimize_chroma_dc(oracle, bd):
    """checkasm.c:2330-2380 style: random small DC sets at every chroma dmf."""
    rs = np.random.default_rng(11)
    dq4, _ = oracle.cqm_dequant(FLAT)
    for qp in range(0, 52, 3):
        dmf = int(dq4[2, qp % 6, 0]) << (qp // 6)
        for c422, name, n in ((0, "optimize_chroma_2x2_dc", 4), (1, "optimize_chroma_2x4_dc", 8)):
            for _ in range(8):
                d = rs.integers(-6, 7, n) * (rs.integers(0, 3, n) > 0)
                got, nz = oracle.inplace(bd, name, d, dmf)
                wnz, wd = _py_optimize_chroma([int(v) for v in d], dmf, c422)
                assert nz == wnz and list(got) == wd, (qp, name, list(d))


@pytest.mark.parametrize("bd", [8, 10])
def test_denoise_dct(oracle, bd):
    rs = np.random.default_rng(12)
    for size in (16, 64):
        d = rs.integers(-500, 500, size)
        off = rs.integers(0, 60, size).astype(oracle.ucoef_dtype(bd))
        s0 = rs.integers(0, 1000, size).astype(np.uint32)
        dd = np.ascontiguousarray(d, oracle.coef_dtype(bd))
        sm = s0.copy()
        oracle.fn(bd, "denoise_dct")(oracle._addr(dd), oracle._addr(sm), oracle._addr(off), size)
        lvl = np.abs(d)
        assert np.array_equal(sm, s0 + lvl.astype(np.uint32))
        nl = lvl - off.astype(np.int64)
        assert np.array_equal(dd, np.where(nl < 0, 0, np.sign(d) * nl))


@pytest.mark.parametrize("bd", [8, 10])
def test_decimate_last_level_run(oracle, bd):
    """checkasm.c:2180-2276 style sparse inputs."""
    rs = np.random.default_rng(13)
    for t in range(400):
        n = (15, 16, 64, 4, 8)[t % 5]
        mag = rs.integers(1, 3 if t % 3 else 5, n)
        d = np.where(rs.random(n) < 0.2, mag * np.where(rs.random(n) < 0.5, -1, 1), 0)
        if t % 17 == 0:
            d[:] = 0
        if n in (15, 16, 64):
            full = np.concatenate([[rs.integers(-3, 3)], d]) if n == 15 else d
            got, _ = oracle.inplace(bd, f"decimate_score{n}", full)
            assert _ == nr.decimate_score(d), (n, list(d))
        last = oracle.fn(bd, "coeff_last")(oracle._addr(np.ascontiguousarray(d, oracle.coef_dtype(bd))), n)
        nzi = np.flatnonzero(d)
        assert last == (nzi[-1] if len(nzi) else -1)
        if len(nzi) and n != 64:
            cnt, l2, mask, levels = oracle.coeff_level_run(bd, d, n)
            assert cnt == len(nzi) and l2 == nzi[-1] and mask == sum(1 << int(i) for i in nzi)
            assert np.array_equal(levels, d[nzi[::-1]])


@pytest.mark.parametrize("bd", [8, 10])
def test_zigzag(oracle, bd):
    rs = np.random.default_rng(14)
    for n, w in ((16, 4), (64, 8)):
        d = rs.integers(-999, 999, n)
        lev = oracle.zigzag_scan(bd, n, 0, d)
        order = nr.zigzag_frame(w)
        # level[i] = dct[x*w + y] for the i-th (y, x) of the frame zigzag (dct.c:768-826)
        assert np.array_equal(lev, [d[x * w + y] for (y, x) in order])
        lf = oracle.zigzag_scan(bd, n, 1, d)
        assert sorted(lf.tolist()) == sorted(d.tolist()) and lf[0] == d[0]
    b = cb.Bufs(bd)
    for kind, w in ((0, 4), (1, 4), (2, 8)):
        for field in (0, 1):
            dst = np.tile(b.pbuf1[b.pbuf2_off:b.pbuf2_off + 32], 16)
            nz, lev, dc, dst2 = oracle.zigzag_sub(bd, kind, field, b.pbuf1, 0, 16, dst, 0, 32)
            diff = nr.block(b.pbuf1, 0, 16, w, w) - nr.block(dst, 0, 32, w, w)
            # zigzag of the difference with the same order as the scan of a transposed block
            scan = oracle.zigzag_scan(bd, w * w, field, nr.wrap(diff.T.ravel(), bd))
            if kind == 1:
                assert dc == diff[0, 0] and lev[0] == 0 and np.array_equal(lev[1:], scan[1:])
            else:
                assert np.array_equal(lev, scan)
            assert nz == int(bool(np.any(lev)))
            assert np.array_equal(nr.block(dst2, 0, 32, w, w), nr.block(b.pbuf1, 0, 16, w, w))
    src = rs.integers(-99, 99, 64)
    dst = np.zeros(64, oracle.coef_dtype(bd))
    nnz = np.zeros(16, np.uint8)
    oracle.fn(bd, "zigzag_interleave_8x8_cavlc")(oracle._addr(dst), oracle._addr(np.ascontiguousarray(src, oracle.coef_dtype(bd))),
                                                 oracle._addr(nnz))
    assert np.array_equal(dst.reshape(4, 16), src.reshape(16, 4).T)
