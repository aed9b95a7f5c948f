"""GPU parity of the forward transforms and quantisation.

Table entries are called like tools/checkasm.c does (check_dct :878-1084,
check_quant :2059-2226); the batched device entries are checked at scale,
including a full 1080p frame of the fused inter-luma residual path."""
import ctypes

import numpy as np
import pytest

from conftest import load_package as _x
import torch

import checkasm_bufs as cb

pytestmark = pytest.mark.gpu

DCT_NAMES = ["sub4x4_dct", "sub8x8_dct", "sub16x16_dct", "sub8x8_dct_dc", "sub8x16_dct_dc", "sub8x8_dct8",
             "sub16x16_dct8"]


def _p(arr, off=0):
    return ctypes.c_void_p(arr.ctypes.data + off * arr.itemsize)


def _cdt(bd):
    return np.int16 if bd == 8 else np.int32


@pytest.mark.parametrize("bd", [8, 10])
def test_dct_table_checkasm(hip, oracle, bd):
    b = cb.Bufs(bd)
    b.fill_dct_overflow()
    dctf = hip.dct_init(bd)
    for name in DCT_NAMES:
        fn = getattr(dctf, name)
        assert fn, name
        for j in range(5):
            for (a, ao, d, do) in ((b.pbuf1, j * 64, b.pbuf1, b.pbuf2_off + j * 64),
                                   (b.pbuf3, 16 * j * 16, b.pbuf4, 16 * j * 32)):
                want = oracle.sub_dct(bd, name, a, ao, d, do)
                got = np.zeros_like(want)
                fn(_p(got), _p(a, ao), _p(d, do))
                assert np.array_equal(got, want), (name, j, ao)


@pytest.mark.parametrize("bd", [8, 10])
def test_dc_table_checkasm(hip, oracle, bd):
    b = cb.Bufs(bd)
    pm = (1 << bd) - 1
    dctf = hip.dct_init(bd)
    p = b.buf1.view(np.uint16)
    k = 0
    for i in range(16):
        d = np.zeros(16, _cdt(bd))
        for j in range(16):
            if i == 0:
                d[j] = pm * 16 if (j ^ j >> 1 ^ j >> 2 ^ j >> 3) & 1 else -pm * 16
            elif i < 8:
                d[j] = pm * 16 if p[k] & 1 else -pm * 16
                k += 1
            else:
                d[j] = (int(p[k]) & 0x1FFF) - 0x1000
                k += 1
        want = oracle.dct4x4dc(bd, d)
        got = d.copy()
        dctf.dct4x4dc(_p(got))
        assert np.array_equal(got, want), i
        # dct2x4dc on 8 blocks whose DCs follow the same patterns (checkasm.c:1060-1084)
        src = np.zeros((8, 16), _cdt(bd))
        src[:, 0] = d[:8]
        src[:, 1:] = (np.arange(15) - 7)[None, :]
        want_out, want_src = oracle.dct2x4dc(bd, src)
        out = np.zeros(8, _cdt(bd))
        s2 = src.copy()
        dctf.dct2x4dc(_p(out), _p(s2))
        assert np.array_equal(out, want_out) and np.array_equal(s2, want_src), i


@pytest.mark.parametrize("bd", [8, 10])
def test_quant_table_checkasm(hip, oracle, bd):
    quantf = hip.quant_init(bd)
    cb.srand(cb.SEED + bd)
    qmax = 51 + 6 * (bd - 8)
    for i_cqm in range(6):
        q4m, q4b, q8m, q8b = hip.cqm_init(bd, cb.cqm_lists(i_cqm, bd))
        for qp in range(qmax, -1, -4 if i_cqm else -1):
            for lst in (0, 1):
                for j in range(2):
                    for name, c, m, bi in (("quant_8x8", cb.init_quant8(j, bd), q8m[lst, qp], q8b[lst, qp]),
                                           ("quant_4x4", cb.init_quant4(j, 16, bd), q4m[lst, qp], q4b[lst, qp])):
                        want, wnz = oracle.quant(bd, name, c, m, bi)
                        got = c.astype(_cdt(bd))
                        m = np.ascontiguousarray(m)
                        bi = np.ascontiguousarray(bi)
                        nz = getattr(quantf, name)(_p(got), _p(m), _p(bi))
                        assert np.array_equal(got, want) and nz == wnz, (i_cqm, qp, name)
            c = cb.init_quant4(qp % 16, 64, bd)
            m, bi = np.ascontiguousarray(q4m[1, qp]), np.ascontiguousarray(q4b[1, qp])
            want, wnz = oracle.quant(bd, "quant_4x4x4", c, m, bi)
            got = c.astype(_cdt(bd))
            assert quantf.quant_4x4x4(_p(got), _p(m), _p(bi)) == wnz and np.array_equal(got, want)
            for name, n, lst in (("quant_4x4_dc", 16, 0), ("quant_2x2_dc", 4, 2)):
                c = np.array([(cb.rand() & 0x1FFF) - 0xFFF for _ in range(n)])
                mf, bias = int(q4m[lst, qp, 0]), int(q4b[lst, qp, 0])
                want, wnz = oracle.quant(bd, name, c, mf, bias)
                got = c.astype(_cdt(bd))
                assert getattr(quantf, name)(_p(got), mf, bias) == wnz and np.array_equal(got, want), (name, qp)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("kind", range(7))
def test_sub_dct_batch_random(hip, oracle, bd, kind):
    rs = np.random.default_rng(kind + 3 * bd)
    pdt = np.uint8 if bd == 8 else np.uint16
    plane = rs.integers(0, 1 << bd, size=1 << 18).astype(pdt)
    dev = torch.from_numpy(plane.view(np.int16) if bd == 10 else plane).cuda()
    n, fs, ds = 4000, 40, 72
    fo = rs.integers(0, (1 << 18) - 17 * 72, size=n).astype(np.int64)
    do = rs.integers(0, (1 << 18) - 17 * 72, size=n).astype(np.int64)
    got = hip.sub_dct_batch(kind, dev, fs, dev, ds, torch.from_numpy(fo).cuda(), torch.from_numpy(do).cuda())
    want = oracle.sub_dct_list(bd, kind, plane, fs, plane, ds, fo, do)
    assert np.array_equal(got.cpu().numpy(), want)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("kind", [0, 1, 2])
def test_quant_batch_random(hip, oracle, bd, kind):
    rs = np.random.default_rng(kind + 7 * bd)
    q4m, q4b, q8m, q8b = hip.cqm_init(bd, cb.cqm_lists(1, bd))
    n = 3000
    size = 64 if kind in (0, 2) else 16
    pm = (1 << bd) - 1
    coefs = rs.integers(-pm * 36, pm * 36 + 1, size=(n, size))
    coefs[rs.random((n, size)) < 0.5] = 0
    qp = 30
    mf, bias = (q8m[1, qp], q8b[1, qp]) if kind == 0 else (q4m[1, qp], q4b[1, qp])
    dev = torch.from_numpy(coefs.astype(_cdt(bd))).cuda()
    nz = hip.quant_batch(kind, dev, torch.from_numpy(mf.copy()).cuda(), torch.from_numpy(bias.copy()).cuda())
    name = ["quant_8x8", "quant_4x4", "quant_4x4x4"][kind]
    got = dev.cpu().numpy()
    gnz = nz.cpu().numpy()
    for i in range(0, n, 7):
        want, wnz = oracle.quant(bd, name, coefs[i], mf, bias)
        assert np.array_equal(got[i], want) and gnz[i] == wnz, i


@pytest.mark.parametrize("bd", [8, 10])
def test_dc_and_quant_dc_batch(hip, oracle, bd):
    rs = np.random.default_rng(bd)
    pm = (1 << bd) - 1
    n = 2000
    d = rs.integers(-pm * 16, pm * 16 + 1, size=(n, 16)).astype(_cdt(bd))
    dev = torch.from_numpy(d.copy()).cuda()
    hip.dc_batch(hip.DC_4x4, dev)
    got = dev.cpu().numpy()
    for i in range(0, n, 5):
        assert np.array_equal(got[i], oracle.dct4x4dc(bd, d[i]))
    blocks = rs.integers(-pm * 16, pm * 16 + 1, size=(n, 8, 16)).astype(_cdt(bd))
    dct4x4 = torch.from_numpy(blocks.copy()).cuda()
    out = torch.zeros((n, 8), dtype=torch.int16 if bd == 8 else torch.int32, device="cuda")
    hip.dc_batch(hip.DC_2x4, out, dct4x4, n=n)
    go, gs = out.cpu().numpy(), dct4x4.cpu().numpy()
    for i in range(0, n, 5):
        wo, ws = oracle.dct2x4dc(bd, blocks[i])
        assert np.array_equal(go[i], wo) and np.array_equal(gs[i], ws)
    q4m, q4b, _, _ = hip.cqm_init(bd, cb.cqm_lists(0, bd))
    for kind, size, name in ((hip.QUANT_4x4_DC, 16, "quant_4x4_dc"), (hip.QUANT_2x2_DC, 4, "quant_2x2_dc")):
        c = rs.integers(-0xFFF, 0x1000, size=(n, size))
        dv = torch.from_numpy(c.astype(_cdt(bd))).cuda()
        mf, bias = int(q4m[0, 24, 0]) >> 1, int(q4b[0, 24, 0]) << 1
        nz = hip.quant_dc_batch(kind, dv, mf, bias).cpu().numpy()
        g = dv.cpu().numpy()
        for i in range(0, n, 5):
            want, wnz = oracle.quant(bd, name, c[i], mf, bias)
            assert np.array_equal(g[i], want) and nz[i] == wnz, (name, i)


@pytest.fixture(params=["default", "nt", "plain"])
def dq_variant(request):
    """the store policy of the fused kernels (X264HIP_STREAM_NT): the default, nontemporal
    coefficient stores forced on (nt) or off (plain); the kernel itself is fixed per transform
    and bit depth (4x4: half-band strips; 8x8: packed 16-bit pairs at 8 bit, staged one-wave
    strips at 10 bit)."""
    if request.param != "default":
        _x().set_variant("X264HIP_STREAM_NT", 1 if request.param == "nt" else 0)
    return request.param


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("transform", [4, 8])
def test_mb_dct_quant_1080p(hip, oracle, bd, transform, dq_variant):
    """fused residual transform + quant over a whole 1080p frame pair (plus a
    second frame in the same launch) vs the oracle, QP 26 flat16, inter lists.
    The prediction is the reference displaced by the sequence's true motion
    (3, 2), so most residual blocks quantise to zero and the pointer is unaligned."""
    from x264hip import synth
    W, H = 1920, 1088
    planes, stride, origin = synth.make_sequence(3, W, H, bd)
    dev = torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()
    fsz = planes[0].size
    q4m, q4b, q8m, q8b = hip.cqm_init(bd, cb.cqm_lists(0, bd))
    qp = 26 + 6 * (bd - 8)
    mf, bias = (q4m[1, qp], q4b[1, qp]) if transform == 4 else (q8m[1, qp], q8b[1, qp])
    po = origin + 2 * stride + 3
    dct, nz = hip.mb_dct_quant(transform, dev[1:], origin, stride, dev[:-1], po, stride, W // 16, H // 16, 2,
                               torch.from_numpy(mf.copy()).cuda(), torch.from_numpy(bias.copy()).cuda(),
                               fenc_frame_stride=fsz, pred_frame_stride=fsz)
    dct, nz = dct.cpu().numpy(), nz.cpu().numpy()
    nmb = (W // 16) * (H // 16)
    for f in range(2):
        wd, wn = oracle.mb_dct_quant(bd, transform, planes[f + 1].ravel(), origin, stride, planes[f].ravel(), po,
                                     stride, W // 16, H // 16, mf, bias)
        assert np.array_equal(dct[f * nmb:(f + 1) * nmb], wd), f
        assert np.array_equal(nz[f * nmb:(f + 1) * nmb], wn), f
    assert nz.any() and (nz == 0).any()


@pytest.mark.parametrize("variant", ["default", "plain"])
@pytest.mark.parametrize("cqm", [0, 3, 5])
def test_mb_dct8_quant_extremes(hip, oracle, monkeypatch, variant, cqm):
    """8-bit transform 8 at the residual extremes the packed 16-bit kernel's range argument
    covers (checkerboards of +-255, constant +-255, uniform noise) with the largest mf of
    every CQM family (all-ones lists: the uint32 (f + |c|) * mf wraps) at QP 0, 26 and 51;
    20 MBs wide so the last 16-MB strip is partial."""
    if variant != "default":
        _x().set_variant("X264HIP_STREAM_NT", 0)
    mbw, mbh = 20, 3
    W, H = 16 * mbw, 16 * mbh
    stride = W + 64
    origin = 32 * stride + 32
    rng = np.random.default_rng(cqm)
    yy, xx = np.mgrid[0:H + 64, 0:stride]
    cb1 = (((xx + yy) & 1) * 255).astype(np.uint8)
    cb2 = ((((xx >> 1) + (yy >> 2)) & 1) * 255).astype(np.uint8)
    fr = [cb1, 255 - cb1, cb2, np.zeros_like(cb1), np.full_like(cb1, 255),
          rng.integers(0, 256, cb1.shape, dtype=np.uint8), rng.integers(0, 256, cb1.shape, dtype=np.uint8)]
    pairs = [(0, 1), (1, 0), (2, 3), (4, 3), (3, 4), (5, 6), (4, 2)]
    fenc = np.stack([fr[a] for a, _ in pairs])
    pred = np.stack([fr[b] for _, b in pairs])
    q4m, q4b, q8m, q8b = hip.cqm_init(8, cb.cqm_lists(cqm, 8))
    fd, pd = torch.from_numpy(fenc).cuda(), torch.from_numpy(pred).cuda()
    fsz = fenc[0].size
    nmb = mbw * mbh
    for qp in (0, 26, 51):
        for lst in (1, 3):
            mf, bias = q8m[lst, qp], q8b[lst, qp]
            dct, nz = hip.mb_dct_quant(8, fd, origin, stride, pd, origin, stride, mbw, mbh, len(pairs),
                                       torch.from_numpy(mf.copy()).cuda(), torch.from_numpy(bias.copy()).cuda(),
                                       fenc_frame_stride=fsz, pred_frame_stride=fsz)
            dct, nz = dct.cpu().numpy(), nz.cpu().numpy()
            for f in range(len(pairs)):
                wd, wn = oracle.mb_dct_quant(8, 8, fenc[f].ravel(), origin, stride, pred[f].ravel(), origin, stride,
                                             mbw, mbh, mf, bias)
                assert np.array_equal(dct[f * nmb:(f + 1) * nmb], wd), (qp, lst, f)
                assert np.array_equal(nz[f * nmb:(f + 1) * nmb], wn), (qp, lst, f)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("transform", [4, 8])
@pytest.mark.parametrize("dx", [0, 16, 48])
@pytest.mark.parametrize("stream_xcd", [None, 1, 2])
def test_mb_dct_quant_strip_alignment(hip, oracle, bd, transform, dx, stream_xcd):
    """the default fused kernels with their strips shifted onto 64-byte sectors of the source
    (shift 0-3 MBs from the fenc pointer's offset in its sector: dx moves it), with the
    XCD-contiguous strip order (X264HIP_STREAM_XCD=1) and unshifted (=2); a ragged
    20-MB row so the shifted strips begin left of the row and end past it."""
    from x264hip import synth
    if stream_xcd is not None:
        hip.set_variant("X264HIP_STREAM_XCD", stream_xcd)
    W, H = 320, 64
    planes, stride, origin = synth.make_sequence(3, W + 64, H, bd, seed=dx + transform)
    dev = torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()
    fsz = planes[0].size
    q4m, q4b, q8m, q8b = hip.cqm_init(bd, cb.cqm_lists(0, bd))
    qp = 20 + 6 * (bd - 8)
    mf, bias = (q4m[1, qp], q4b[1, qp]) if transform == 4 else (q8m[1, qp], q8b[1, qp])
    fo, po = origin + dx, origin + stride + 5
    dct, nz = hip.mb_dct_quant(transform, dev[1:], fo, stride, dev[:-1], po, stride, W // 16, H // 16, 2,
                               torch.from_numpy(mf.copy()).cuda(), torch.from_numpy(bias.copy()).cuda(),
                               fenc_frame_stride=fsz, pred_frame_stride=fsz)
    dct, nz = dct.cpu().numpy(), nz.cpu().numpy()
    nmb = (W // 16) * (H // 16)
    for f in range(2):
        wd, wn = oracle.mb_dct_quant(bd, transform, planes[f + 1].ravel(), fo, stride, planes[f].ravel(), po,
                                     stride, W // 16, H // 16, mf, bias)
        assert np.array_equal(dct[f * nmb:(f + 1) * nmb], wd), f
        assert np.array_equal(nz[f * nmb:(f + 1) * nmb], wn), f
