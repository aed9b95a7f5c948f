"""GPU parity of the intra cost entries: the pixel table's intra_*_x3 functions
(x264hip_{8,10}_pixel_init, reference common/pixel.c:518-560) on checkasm's
buffers (tools/checkasm.c:619-763), the batched x264hip_*_intra_cmp_x3_batch on
random block lists, and the lookahead's lowres intra estimate
(x264hip_*_lowres_intra_cost, encoder/slicetype.c:714-757) on whole frames —
all bit-exact against the oracle."""
import ctypes

import numpy as np
import pytest

from conftest import load_package as _x
import torch

import checkasm_bufs as cb

pytestmark = pytest.mark.gpu

TABLE = [("intra_satd_x3_16x16", 3, 2), ("intra_satd_x3_8x16c", 2, 2), ("intra_satd_x3_8x8c", 1, 2),
         ("intra_sa8d_x3_8x8", 4, 3), ("intra_satd_x3_4x4", 0, 2), ("intra_sad_x3_16x16", 3, 0),
         ("intra_sad_x3_8x16c", 2, 0), ("intra_sad_x3_8x8c", 1, 0), ("intra_sad_x3_8x8", 4, 0),
         ("intra_sad_x3_4x4", 0, 0)]


def _p(arr, off=0):
    return ctypes.c_void_p(arr.ctypes.data + int(off) * arr.itemsize)


def _dev(a, bd):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int16) if bd == 10 else np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("bd", [8, 10])
def test_table_intra_x3_checkasm(hip, oracle, bd):
    """TEST_INTRA_X3 (checkasm.c:619-635, 752-763): fenc = pbuf1+48, fdec = pbuf3+48 after the
    overflow fill, edge = predict_8x8_filter( pbuf2+40, ALL_NEIGHBORS ) (checkasm.c:366)."""
    b = cb.Bufs(bd)
    edge = oracle.predict_8x8_filter(bd, b.pbuf1, b.pbuf2_off + 40)
    b.fill_pixel_overflow()
    pixf = hip.pixel_init(bd)
    for name, kind, op in TABLE:
        fn = getattr(pixf, name)
        assert fn, name
        for trial in range(3):
            fenc = b.pbuf1 if trial == 0 else b.pbuf3 if trial == 1 else b.pbuf4
            fdec = edge if kind == 4 else (b.pbuf3 if trial != 1 else b.pbuf4)
            foff = 48 + 64 * trial
            doff = 0 if kind == 4 else 48 + 32 * trial
            res = (ctypes.c_int * 3)()
            fn(_p(fenc, foff), _p(fdec, doff), res)
            want = oracle.intra_x3(bd, kind, op, fenc, foff, fdec, doff)
            assert list(res) == list(want), (name, trial)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4])
def test_intra_cmp_x3_batch_random(hip, oracle, bd, kind):
    rs = np.random.default_rng(70 + 10 * bd + kind)
    pdt = oracle.pixel_dtype(bd)
    plane = rs.integers(0, 1 << bd, size=1 << 18).astype(pdt)
    plane[:4096] = (1 << bd) - 1                                  # saturated corner blocks
    dev = _dev(plane, bd)
    ops = (0, 3) if kind == 4 else (0, 2)
    for op in ops:
        n = 1500
        fs, ds = int(rs.integers(16, 200)), int(rs.integers(17, 200))
        fo = rs.integers(0, (1 << 18) - 17 * fs, size=n).astype(np.int64)
        if kind == 4:
            do = rs.integers(0, (1 << 18) - 40, size=n).astype(np.int64)
        else:
            do = rs.integers(ds + 1, (1 << 18) - 17 * ds, size=n).astype(np.int64)
        fo[:8] = np.arange(8) * 16                                # the saturated region
        got = hip.intra_cmp_x3_batch(kind, op, dev, fs, dev, ds, torch.from_numpy(fo).cuda(),
                                     torch.from_numpy(do).cuda()).cpu().numpy()
        w, h = hip.INTRA_SIZES[kind]
        for i in range(n):
            fenc = np.zeros(16 * 16, pdt)
            fenc.reshape(16, 16)[:h, :w] = plane[fo[i] + np.arange(h)[:, None] * fs + np.arange(w)[None, :]]
            if kind == 4:
                want = oracle.intra_x3(bd, kind, op, fenc, 0, plane, do[i])
            else:
                fdec = np.zeros(17 * 32 + 16, pdt)
                idx = do[i] + np.arange(-1, h)[:, None] * ds + np.arange(-1, w)[None, :]
                fdec.reshape(-1)[32 + 8 - 33 + np.arange(h + 1)[:, None] * 32 + np.arange(w + 1)[None, :]] = plane[idx]
                want = oracle.intra_x3(bd, kind, op, fenc, 0, fdec, 32 + 8)
            assert list(got[i]) == list(want), (op, i)


def test_intra_cmp_x3_batch_bad_args(hip):
    dev = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    off = torch.zeros(1, dtype=torch.int64, device="cuda")
    with pytest.raises(RuntimeError):
        hip.intra_cmp_x3_batch(0, hip.CMP_SA8D, dev, 16, dev, 32, off, off)   # sa8d only for the 8x8 kind
    with pytest.raises(RuntimeError):
        hip.intra_cmp_x3_batch(4, hip.CMP_SATD, dev, 16, dev, 32, off, off)
    with pytest.raises(RuntimeError):
        hip.intra_cmp_x3_batch(5, hip.CMP_SAD, dev, 16, dev, 32, off, off)


def _lowres_frames(hip, bd, W, H, n, seed):
    from x264hip import synth
    if W >= 320:
        planes, stride, origin = synth.make_sequence(n, W, H, bd)
    else:
        planes, stride, origin = synth.random_planes(n, W, H, bd, seed=seed)
    outs, ls = hip.frame_init_lowres(_dev(planes, bd), origin, stride, W, H)
    return outs[0], ls


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("size", [(1920, 1088), (352, 288), (32, 48), (64, 16), (8320, 64)])
@pytest.mark.parametrize("mode", ["satd_all", "sad_dc_h_v", "satd_dc_h_v", "sad_all_aq"])
def test_lowres_intra_cost(hip, oracle, bd, size, mode):
    """the lookahead's intra estimate (one workgroup per MB row) vs the oracle"""
    W, H = size
    mbw, mbh = W // 16, H // 16
    n = 2
    low, ls = _lowres_frames(hip, bd, W, H, n, seed=bd + W)
    satd = mode.startswith("satd")
    all_modes = mode.endswith("all") or mode.endswith("aq")
    rs = np.random.default_rng(W + bd)
    invq = rs.integers(64, 1024, size=(n, mbw * mbh)).astype(np.uint16) if mode.endswith("aq") else None
    lam = 1 if W > 1000 else 57
    cost, rows, est = hip.lowres_intra_cost(low, ls, mbw, mbh, satd, all_modes, lam,
                                            None if invq is None else torch.from_numpy(invq.view(np.int16)).cuda())
    cost = cost.cpu().numpy().view(np.uint16)
    rows, est = rows.cpu().numpy(), est.cpu().numpy()
    host = low.cpu().numpy().view(oracle.pixel_dtype(bd))
    for f in range(n):
        want = oracle.lowres_intra_cost(bd, host[f].ravel(), hip.PAD * ls + hip.PAD, ls, mbw, mbh, satd, all_modes,
                                        lam, None if invq is None else invq[f])
        assert np.array_equal(cost[f], want[0]), (f, np.argwhere(cost[f] != want[0])[:4])
        assert np.array_equal(rows[f], want[1]), f
        assert list(est[f]) == list(want[2]), f


def test_lowres_intra_cost_no_outputs(hip, oracle):
    """row_satd / cost_est are optional (NULL) and the per-MB costs do not depend on them."""
    low, ls = _lowres_frames(hip, 8, 176, 144, 1, seed=3)
    a = hip.lowres_intra_cost(low, ls, 11, 9)[0]
    b = hip.lowres_intra_cost(low, ls, 11, 9, with_rows=False)[0]
    assert torch.equal(a, b)
