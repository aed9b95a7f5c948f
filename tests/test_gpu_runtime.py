"""GPU: the runtime around the tables (VERDICT r1 "single-process
multi-device readiness"):

* per-thread device binding: a thread bound with x264hip_set_thread_device runs its table
  entries on that device, on its own stream + staging buffer, concurrently with other
  threads (x264's frame / lookahead threads, reference encoder/encoder.c:1758-1772);
* x264hip_forward_ref: the reconstructed-reference peer copy of the frame-per-GPU pipeline
  (on one GPU it is exercised as a same-device copy);
* x264hip_upload: frame planes from pinned host memory by a PCIe-read kernel;
* the backend banner (reference encoder/encoder.c:1676-1706 analogue) names the device.
"""
import ctypes
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_thread_device_binding_and_concurrent_entries(hip, oracle):
    pixf = hip.pixel_init(8)
    ndev = torch.cuda.device_count()
    errors = []

    def worker(k):
        try:
            dev = k % ndev
            hip.set_thread_device(dev)
            assert hip.thread_device() == dev
            a = np.random.default_rng(100 + k).integers(0, 256, 16 * 16).astype(np.uint8)
            b = np.random.default_rng(200 + k).integers(0, 256, 64 * 16).astype(np.uint8)
            for i in range(20):
                got = pixf.sad[hip.PIXEL_16x16](a.ctypes.data, 16, b[i:].ctypes.data, 64)
                want = oracle.cmp(8, "sad", 0, a, 0, 16, b, i, 64)
                assert got == want, (k, i, got, want)
            hip.set_thread_device(-1)
            assert hip.thread_device() == 0
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append(e)

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=60)
    assert not errors, errors
    with pytest.raises(hip.BackendUnavailable):
        hip.set_thread_device(ndev + 3)


def test_forward_ref_peer_copy(hip):
    src = torch.randint(0, 256, (1152, 1984), dtype=torch.uint8, device="cuda:0")
    dst = torch.zeros_like(src)
    hip.forward_ref(dst, 0, src, 0)
    torch.cuda.synchronize()
    assert torch.equal(src, dst)
    with pytest.raises(ValueError):
        hip.forward_ref(dst[:10], 0, src, 0)


@pytest.mark.parametrize("nbytes,off", [(8682496, 0), (8682496 + 7, 0), (1 << 20, 3), (5, 0), (17, 1), (0, 0)])
def test_upload_from_pinned(hip, nbytes, off):
    """x264hip_upload: the PCIe-read kernel copies page-locked host bytes exactly, in
    16-byte pieces (aligned, ragged tail) or bytewise (misaligned start)."""
    rng = np.random.default_rng(nbytes + off)
    host = torch.from_numpy(rng.integers(0, 256, nbytes + off + 16, dtype=np.uint8)).pin_memory()
    dev = torch.zeros(nbytes + off + 16, dtype=torch.uint8, device="cuda")
    hip.upload(dev[off:off + nbytes], host[off:off + nbytes])
    torch.cuda.synchronize()
    got = dev.cpu()
    assert torch.equal(got[off:off + nbytes], host[off:off + nbytes])
    assert not got[:off].any() and not got[off + nbytes:].any()   # nothing written outside
    with pytest.raises(ValueError):
        hip.upload(dev[:4], host[:5])


def test_upload_registered_and_pageable(hip):
    """x264hip_upload resolves the source's device address
    (hipHostGetDevicePointer) so hipHostRegister'd memory works, and refuses pageable
    memory with X264HIP_EINVAL instead of letting the kernel fault the GPU."""
    L = hip.lib()
    L.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    L.hipHostRegister.restype = ctypes.c_int
    L.hipHostUnregister.argtypes = [ctypes.c_void_p]
    L.hipHostUnregister.restype = ctypes.c_int
    L.x264hip_upload.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    n = 3 << 20
    buf = np.random.default_rng(7).integers(0, 256, n + 4096, dtype=np.uint8)
    base = (buf.ctypes.data + 4095) & ~4095
    arr = np.frombuffer((ctypes.c_uint8 * n).from_address(base), dtype=np.uint8)
    dev = torch.zeros(n, dtype=torch.uint8, device="cuda")
    # pageable: refused, nothing written, no fault
    assert L.x264hip_upload(ctypes.c_void_p(dev.data_ptr()), ctypes.c_void_p(base), n, None) == -1
    assert "page-locked" in L.x264hip_last_error().decode()
    torch.cuda.synchronize()
    assert not dev.any()
    assert L.hipHostRegister(ctypes.c_void_p(base), n, 0) == 0
    try:
        for off, nb in ((0, n), (5, n - 5), (4096 * 3 + 1, 100000)):
            dev.zero_()
            rc = L.x264hip_upload(ctypes.c_void_p(dev.data_ptr()), ctypes.c_void_p(base + off), nb, None)
            assert rc == 0, L.x264hip_last_error().decode()
            torch.cuda.synchronize()
            assert np.array_equal(dev[:nb].cpu().numpy(), arr[off:off + nb])
        # a range running past the registration is refused
        assert L.x264hip_upload(ctypes.c_void_p(dev.data_ptr()), ctypes.c_void_p(base + 16), n, None) == -1
    finally:
        torch.cuda.synchronize()
        L.hipHostUnregister(ctypes.c_void_p(base))


def test_backend_banner(hip):
    hip.pixel_init(8)
    b = hip.backend_banner()
    assert "gfx950" in b and "satd_x3/x4" in b and "kept from the caller" in b


def test_init_hip_overrides_only(hip):
    """With a device, the _init_hip form replaces the entries it implements and keeps the
    rest of a caller-filled table (the never-initialised ssim[7], intra_*_x9, trellis)."""
    tab = hip.PixelFunctions()
    raw = (ctypes.c_uint64 * (ctypes.sizeof(tab) // 8)).from_buffer(tab)
    for i in range(len(raw)):
        raw[i] = 0x5EED0000 + i
    hip.lib().x264hip_8_pixel_init_hip(ctypes.byref(tab))
    keep = [hip.PixelFunctions.ssim, hip.PixelFunctions.intra_sad_x9_8x8, hip.PixelFunctions.mbcmp, hip.PixelFunctions.fpelcmp_x4]
    for f in keep:
        i0 = f.offset // 8
        n = f.size // 8
        assert all(raw[i] == 0x5EED0000 + i for i in range(i0, i0 + n)), f
    for f in (hip.PixelFunctions.sad, hip.PixelFunctions.ssd_nv12_core, hip.PixelFunctions.ssim_4x4x2_core,
              hip.PixelFunctions.ssim_end4):
        i = f.offset // 8
        assert raw[i] != 0x5EED0000 + i, f


@pytest.mark.parametrize("bd", [8, 10])
def test_empty_launches(hip, bd):
    """every hot-path batched entry with no work (0 frames, or a 0-MB-wide frame for the
    MB-grid entries) returns 0 and writes nothing (the sentinel-filled output stays untouched)"""
    L = hip.lib()
    buf = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    out = torch.full((4096,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    P = ctypes.c_void_p(buf.data_ptr())
    O = ctypes.c_void_p(out.data_ptr())
    pre = f"x264hip_{bd}_"
    fn = lambda n: getattr(L, pre + n)
    dst4 = (ctypes.c_void_p * 4)(*([P.value] * 4))
    for nf, mbw in ((0, 4), (2, 0)):
        calls = {
            "me_search_full": lambda: fn("me_search_full")(P, 64, 0, P, 64, 0, mbw, 2, nf, 16, O, None),
            "me_search_full8": lambda: fn("me_search_full8")(P, 64, 0, P, 64, 0, mbw, 2, nf, 16, O, None),
            "me_tesa": lambda: fn("me_tesa")(P, 64, 0, P, 64, 0, P, 0, mbw, 2, nf, 16, 1, None, 0, None, P, P, P,
                                             O, None),
            "hpel_filter": lambda: fn("hpel_filter")(P, O, O, O, 64, 0, 64, 32, 0, None),
            "mb_dct_quant4": lambda: fn("mb_dct_quant")(4, P, 64, 0, P, 64, 0, mbw, 2, nf, P, P, O, O, None),
            "mb_dct_quant8": lambda: fn("mb_dct_quant")(8, P, 64, 0, P, 64, 0, mbw, 2, nf, P, P, O, O, None),
            "frame_init_lowres": lambda: fn("frame_init_lowres")(P, 64, 0, 64, 32, 0, dst4, 64, 0, None),
            "frame_integral": lambda: fn("frame_integral")(P, 64, 0, 32, 32, 0, 0, O, 0, None),
        }
        for name, call in calls.items():
            assert call() == 0, (name, nf, mbw)
    # the TESA scan addresses rows by 24-bit products: a ref stride of 2^18 is refused
    assert fn("me_tesa")(P, 64, 0, P, 1 << 18, 0, P, 0, 1, 1, 1, 16, 1, None, 0, None, P, P, P, O, None) == -1
    torch.cuda.synchronize()
    assert (out == 0x5A5A5A5A).all()


def _expand_ref(plane, pad_x, pad_y, unit):
    """plane_expand_border (reference common/frame.c:535-554) of a picture plane, in numpy: the
    edge element of `unit` bytes repeated over pad_x bytes, then the first / last padded rows"""
    h, wb = plane.shape
    e = plane.reshape(h, wb // unit, unit)
    left = np.repeat(e[:, :1], pad_x // unit, axis=1)
    right = np.repeat(e[:, -1:], pad_x // unit, axis=1)
    rows = np.concatenate([left, e, right], 1).reshape(h, wb + 2 * pad_x)
    return np.concatenate([np.repeat(rows[:1], pad_y, 0), rows, np.repeat(rows[-1:], pad_y, 0)], 0)


@pytest.mark.parametrize("W,H,unit,pad_x,pad_y", [(96, 64, 1, 32, 32), (96, 32, 2, 32, 32), (192, 64, 2, 64, 32),
                                                   (192, 32, 4, 64, 16), (3840, 2160, 1, 32, 32),
                                                   (3840, 1080, 2, 32, 32), (48, 1, 1, 16, 3)])
def test_upload_plane_expands_borders(hip, W, H, unit, pad_x, pad_y):
    """x264hip_upload_plane: a pinned picture plane lands in the padded plane with the borders
    plane_expand_border writes (luma, NV12 per component, 10-bit units), nothing outside them"""
    rng = np.random.default_rng(W + H + unit)
    src_stride = W + 32
    host_np = rng.integers(0, 256, (H, src_stride), dtype=np.uint8)
    host = torch.from_numpy(host_np).pin_memory()
    ds = (W + 2 * pad_x + 64 + 63) // 64 * 64
    rows = H + 2 * pad_y + 2
    dev = torch.full((rows * ds,), 0xA5, dtype=torch.uint8, device="cuda")
    origin = (pad_y + 1) * ds + pad_x
    hip.upload_plane(dev, origin, ds, host[:, :W], unit=unit, pad_x=pad_x, pad_y=pad_y)
    torch.cuda.synchronize()
    got = dev.cpu().numpy().reshape(rows, ds)
    want = _expand_ref(host_np[:, :W], pad_x, pad_y, unit)
    assert np.array_equal(got[1:1 + H + 2 * pad_y, :W + 2 * pad_x], want)
    assert (got[0] == 0xA5).all() and (got[-1] == 0xA5).all() and (got[:, W + 2 * pad_x:] == 0xA5).all()


def test_upload_plane_refuses(hip):
    dev = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    pinned = torch.zeros((16, 64), dtype=torch.uint8).pin_memory()
    L = hip.lib()
    ptr = ctypes.c_void_p(dev.data_ptr() + 32 * 256 + 32)
    # width not a multiple of 16, a pad band not a multiple of 16, a bad unit, pageable memory
    for wb, unit, px in ((40, 1, 32), (64, 1, 24), (64, 3, 32)):
        assert L.x264hip_upload_plane(ptr, 256, ctypes.c_void_p(pinned.data_ptr()), 64, wb, 16, unit, px, 32,
                                      None) != 0
    page = np.zeros((16, 64), np.uint8)
    assert L.x264hip_upload_plane(ptr, 256, ctypes.c_void_p(page.ctypes.data), 64, 64, 16, 1, 32, 32, None) != 0
    torch.cuda.synchronize()
    assert not dev.any()


@pytest.mark.parametrize("bd", [8, 10])
def test_upload_planes_picture(hip, bd):
    """x264hip_upload_planes: a 4:2:0 picture's luma and NV12 planes in one launch, each padded as
    plane_expand_border pads it (x264_frame_expand_border / _chroma)"""
    W, H = 160, 96
    es = 1 if bd == 8 else 2
    dt = np.uint8 if bd == 8 else np.uint16
    rng = np.random.default_rng(bd)
    y = rng.integers(0, 1 << bd, (H, W)).astype(dt)
    c = rng.integers(0, 1 << bd, (H // 2, W)).astype(dt)             # interleaved U, V
    hy, hc = torch.from_numpy(y).pin_memory(), torch.from_numpy(c).pin_memory()
    tdt = torch.uint8 if bd == 8 else torch.int16
    ys, cs = (W + 64 + 63) // 64 * 64, (W + 64 + 63) // 64 * 64
    dy = torch.zeros(((H + 64) * ys,), dtype=tdt, device="cuda")
    dc = torch.zeros(((H // 2 + 32) * cs,), dtype=tdt, device="cuda")
    hip.upload_planes([hip.plane_upload(dy, 32 * ys + 32, ys, hy, unit=es, pad_x=32 * es, pad_y=32),
                       hip.plane_upload(dc, 16 * cs + 32, cs, hc, unit=2 * es, pad_x=32 * es, pad_y=16)])
    torch.cuda.synchronize()
    gy = dy.cpu().numpy().view(dt).reshape(H + 64, ys)[:, :W + 64]
    gc = dc.cpu().numpy().view(dt).reshape(H // 2 + 32, cs)[:, :W + 64]
    assert np.array_equal(gy, np.pad(y, 32, mode="edge"))
    u, v = c[:, 0::2], c[:, 1::2]
    wc = np.zeros((H // 2 + 32, W + 64), dt)
    wc[:, 0::2], wc[:, 1::2] = np.pad(u, 16, mode="edge"), np.pad(v, 16, mode="edge")
    assert np.array_equal(gc, wc)
