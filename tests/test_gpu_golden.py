"""GPU against the committed golden fixtures (tests/golden/golden_{8,10}.npz, made by
tests/golden/make_golden.py): the frozen oracle outputs, compared without the live
oracle in the loop."""
import ctypes
import os

import numpy as np
import pytest
import torch

import checkasm_bufs as cb

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _p(arr, off=0):
    return ctypes.c_void_p(arr.ctypes.data + int(off) * arr.itemsize)


def _T(a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint16:
        a = a.view(np.int16)
    if a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(a).cuda()


@pytest.fixture(scope="module", params=[8, 10])
def gold(request):
    bd = request.param
    with np.load(os.path.join(HERE, "golden", f"golden_{bd}.npz"), allow_pickle=False) as z:
        return bd, {k: z[k] for k in z.files}


def test_golden_pixel_tables(hip, gold):
    bd, g = gold
    b = cb.Bufs(bd)
    b.fill_pixel_overflow()
    pixf = hip.pixel_init(bd)
    for k, op in enumerate(("sad", "ssd", "satd")):
        for i in range(8):
            for j in range(64):
                s1 = 32 if (j & 31) == 31 else 16
                assert getattr(pixf, op)[i](_p(b.pbuf1), s1, _p(b.pbuf1, b.pbuf2_off + j), 64) == g["pixel"][k, i, j]
            for t, j in enumerate(range(0, 0x1000, 256)):
                assert getattr(pixf, op)[i](_p(b.pbuf3, j), 16, _p(b.pbuf4, j), 16) == g["pixel"][k, i, 64 + t]
    for k, i in enumerate((0, 3)):
        for j in range(0, 64, 5):
            s1 = 32 if (j & 31) == 31 else 16
            assert pixf.sa8d[i](_p(b.pbuf1), s1, _p(b.pbuf1, b.pbuf2_off + j), 64) == g["sa8d"][k, j]
    for j in range(0, 64, 7):
        assert pixf.sa8d_satd[0](_p(b.pbuf1), 16, _p(b.pbuf1, b.pbuf2_off + j), 64) == g["sa8d_satd"][j]
    for i in range(4):
        for j in range(32):
            buf = b.pbuf1 if j & 16 else b.pbuf3
            if g["hadamard_ac"][i, j]:
                assert pixf.hadamard_ac[i](_p(buf, (j & 15) * 256), 16) == g["hadamard_ac"][i, j]


def test_golden_frames(hip, gold):
    """me_search_full, mb_dct_quant, mb_dequant_idct_add, hpel_filter, frame_init_lowres and
    frame_integral on the fixtures' 64x48 synthetic pair."""
    from x264hip import synth
    bd, g = gold
    planes, stride, origin = synth.make_sequence(2, 64, 48, bd)
    dev = _T(planes)
    fs = planes[0].size
    tab = hip.me_search_full(dev[1:], origin, stride, dev[:-1], origin, stride, 4, 3, 1, 8)
    want = g["me_full_r8"]
    got = tab.cpu().numpy()
    got = got.view(np.uint16) if bd == 8 else got.view(np.uint32)
    assert np.array_equal(got[0][..., :17], want)                 # table pitch 20, 17 live columns
    q4m, q4b, q8m, q8b = hip.cqm_init(bd, [cb.FLAT16] * 8)
    dq4, dq8 = hip.cqm_dequant([cb.FLAT16] * 8)
    qp = 26 + 6 * (bd - 8)
    for t, mf, bias, dq in ((4, q4m, q4b, dq4), (8, q8m, q8b, dq8)):
        dct, nz = hip.mb_dct_quant(t, dev[1:], origin, stride, dev[:-1], origin, stride, 4, 3, 1, _T(mf[1, qp]),
                                   _T(bias[1, qp]), fenc_frame_stride=fs, pred_frame_stride=fs)
        assert np.array_equal(dct.cpu().numpy(), g[f"mb_dct{t}_quant"])
        assert np.array_equal(nz.cpu().numpy(), g[f"mb_dct{t}_nz"])
        rec = torch.zeros_like(dev[:1])
        hip.mb_dequant_idct_add(t, dct, 4, 3, 1, _T(dq[1]), _T(np.full(12, qp, np.int32)), dev[:1], origin, stride,
                                rec, origin, stride)
        r = rec.cpu().numpy()[0]
        r = r.view(np.uint16) if bd == 10 else r
        assert np.array_equal(r[32:80, 32:96], g[f"recon{t}"])
    hv = hip.hpel_filter(dev[:1], origin, stride, 64, 48)
    for k in range(3):
        h = hv[k].cpu().numpy()[0]
        h = h.view(np.uint16) if bd == 10 else h
        assert np.array_equal(h[:, :64 + 64], g["hpel"][k][:, :64 + 64]), k
    outs, ls = hip.frame_init_lowres(dev[:1], origin, stride, 64, 48)
    for k in range(4):
        lo = outs[k].cpu().numpy()[0]
        lo = lo.view(np.uint16) if bd == 10 else lo
        assert np.array_equal(lo[:, :32 + 64], g["lowres"][k][:, :32 + 64]), k
    integ = hip.frame_integral(dev[:1], origin, stride, 48, sub8x8=True).cpu().numpy()[0].view(np.uint16)
    gi = g["integral"]
    r1 = 48 + 64 - 8
    assert np.array_equal(integ[1:r1, :stride - 8], gi[1:r1, :stride - 8])
    o = 48 + 64
    assert np.array_equal(integ[o + 1:o + r1, :stride - 8], gi[o + 1:o + r1, :stride - 8])
