"""GPU parity of the pixel metrics, called exactly the way the reference's
tools/checkasm.c calls them: through the x264_pixel_function_t table filled by
x264hip_{8,10}_pixel_init(X264HIP_CPU_HIP) (TEST_PIXEL checkasm.c:384-423,
TEST_PIXEL_X :462-502), plus the batched device entry at scale."""
import ctypes

import numpy as np
import pytest
import torch

import checkasm_bufs as cb
import numpy_ref as nr

pytestmark = pytest.mark.gpu


def _p(arr, off=0):
    return ctypes.c_void_p(arr.ctypes.data + off * arr.itemsize)


@pytest.fixture(scope="module", params=[8, 10])
def setup(request, hip):
    bd = request.param
    b = cb.Bufs(bd)
    b.fill_pixel_overflow()
    return bd, b, hip.pixel_init(bd)


@pytest.mark.parametrize("name,op,align", [("sad", "sad", 0), ("sad_aligned", "sad", 1), ("ssd", "ssd", 1),
                                           ("satd", "satd", 0)])
def test_table_entries_checkasm(oracle, setup, name, op, align):
    bd, b, pixf = setup
    tab = getattr(pixf, name)
    for i in range(8):
        fn = tab[i]
        assert fn, f"{name}[{i}] not filled"
        for j in range(0, 64, 3 if name != "sad" else 1):
            s1 = 32 if (j & 31) == 31 else 16
            o2 = b.pbuf2_off + (0 if align else j)
            got = fn(_p(b.pbuf1), s1, _p(b.pbuf1, o2), 64)
            assert got == oracle.cmp(bd, op, i, b.pbuf1, 0, s1, b.pbuf1, o2, 64), (name, i, j)
        for j in range(0, 0x1000, 256):
            got = fn(_p(b.pbuf3, j), 16, _p(b.pbuf4, j), 16)
            assert got == oracle.cmp(bd, op, i, b.pbuf3, j, 16, b.pbuf4, j, 16), (name, i, "overflow", j)


@pytest.mark.parametrize("name,op", [("sad_x3", "sad"), ("sad_x4", "sad"), ("satd_x3", "satd"), ("satd_x4", "satd")])
def test_table_x_entries_checkasm(oracle, setup, name, op):
    bd, b, pixf = setup
    n = int(name[-1])
    tab = getattr(pixf, name)
    for i in range(7):
        for j in range(0, 64, 5):
            base = b.pbuf2_off + j
            offs = [base, base + 6, base + 1, base + 10][:n]
            res = (ctypes.c_int * 4)()
            tab[i](_p(b.pbuf1), *[_p(b.pbuf1, o) for o in offs], 64, res)
            want = oracle.cmp_x(bd, op, n, i, b.pbuf1, 0, b.pbuf1, offs, 64)
            assert list(res)[:n] == list(want), (name, i, j)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("op", [0, 1, 2])
def test_cmp_batch_random_lists(hip, oracle, bd, op):
    """batched entry: 20k random (fenc, ref) block pairs of every size, arbitrary
    alignment and strides, against the oracle list form."""
    rs = np.random.default_rng(op * 10 + bd)
    pdt = np.uint8 if bd == 8 else np.uint16
    plane = rs.integers(0, 1 << bd, size=1 << 20).astype(pdt)
    dev = torch.from_numpy(plane.view(np.int16) if bd == 10 else plane).cuda()
    for i_pixel in range(8):
        n = 2500
        fs, rsd = int(rs.integers(16, 300)), int(rs.integers(16, 300))
        fo = rs.integers(0, (1 << 20) - 17 * max(fs, rsd), size=n).astype(np.int64)
        ro = rs.integers(0, (1 << 20) - 17 * max(fs, rsd), size=n).astype(np.int64)
        got = hip.pixel_cmp_batch(op, i_pixel, dev, fs, dev, rsd, torch.from_numpy(fo).cuda(),
                                  torch.from_numpy(ro).cuda()).cpu().numpy()
        want = oracle.cmp_list(bd, op, i_pixel, plane, fs, plane, rsd, fo, ro)
        assert np.array_equal(got, want), (op, i_pixel)


def test_cmp_batch_empty_and_bad_args(hip):
    L = hip.lib()
    dev = torch.zeros(64, dtype=torch.uint8, device="cuda")
    off = torch.zeros(1, dtype=torch.int64, device="cuda")
    sc = torch.zeros(1, dtype=torch.int32, device="cuda")
    p = ctypes.c_void_p(dev.data_ptr())
    assert L.x264hip_8_pixel_cmp_batch(0, 0, p, 16, p, 16, ctypes.c_void_p(off.data_ptr()),
                                       ctypes.c_void_p(off.data_ptr()), 0, ctypes.c_void_p(sc.data_ptr()), None) == 0
    assert L.x264hip_8_pixel_cmp_batch(7, 0, p, 16, p, 16, None, None, 1, None, None) == -1   # bad op
    assert L.x264hip_8_pixel_cmp_batch(3, 1, p, 16, p, 16, None, None, 1, None, None) == -1   # sa8d 16x8
    assert L.x264hip_8_pixel_stat_batch(5, 0, p, 16, p, 16, None, None, 0, 1, None, None) == -1  # bad op
    assert L.x264hip_8_pixel_stat_batch(0, 1, p, 16, p, 16, None, None, 0, 1, None, None) == -1  # var 16x8
    assert L.x264hip_8_var2_batch(0, p, 16, 8, p, 32, 16, None, None, 1, None, None) == -1       # var2 16x16
    assert L.x264hip_8_pixel_cmp_batch(0, 8, p, 16, p, 16, None, None, 1, None, None) == -1   # bad size
    assert L.x264hip_8_me_search_full(p, 16, 0, p, 16, 0, 1, 1, 1, 5, None, None) == -1      # bad range


def test_numpy_ref_matches_gpu_satd(hip):
    """the clean Hadamard form (numpy) equals the GPU SATD on max-difference tiles"""
    pm = 255
    a = np.zeros((16, 16), np.uint8)
    bb = np.full((16, 16), pm, np.uint8)
    a[::2, 1::2] = pm
    pixf = hip.pixel_init(8)
    got = pixf.satd[0](_p(a), 16, _p(bb), 16)
    assert got == nr.satd(a.astype(np.int64), bb.astype(np.int64))
