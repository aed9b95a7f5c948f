"""Lookup mode of the drop-in 16x16 SAD entries (x264hip_8_me_bind).

A C99 program (tests/c/me_bind_esa.c) runs encoder/me.c's exhaustive integer search
(me.c:618-631 bounds and width rounding, COST_MV over fpelcmp = sad) through the pixel
table for every MB of a 1080p pair, with the pair's GPU full-search table bound.  The
decisions must equal the oracle's (me_esa_argmin over an oracle table wide enough for
every window), the hits must cover every call whose candidate the bound table holds,
and a hit must cost well under 1 us.  Misses (window rows past the table's range) take
the dispatch path and stay exact."""
import os
import subprocess

import numpy as np
import pytest
import torch

from conftest import ROOT, ensure_built

SRC = os.path.join(ROOT, "tests", "c", "me_bind_esa.c")
MAGIC = 0x4d45424e44


def build(tmp):
    ensure_built("hip")
    exe = os.path.join(tmp, "me_bind_esa")
    lib = os.path.join(ROOT, "x264-i386pic_amd")
    cmd = ["gcc", "-std=c99", "-O2", "-Wall", "-Werror", "-D_POSIX_C_SOURCE=199309L", "-I",
           os.path.join(ROOT, "include"), SRC, "-L", lib, "-lx264hip", f"-Wl,-rpath,{lib}", "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def test_me_bind_esa_builds(tmp_path):
    assert os.path.exists(build(str(tmp_path)))


def _cost_mv(lam=40, span=4096):
    i = np.arange(-span, span + 1)
    logs = np.where(i == 0, 0.718, 2.0 * np.log2(np.abs(i) + 1) + 1.718)
    return np.minimum((lam * logs + 0.5).astype(np.int64), 65535).astype(np.uint16), span


def _run(exe, tmp, planes, stride, origin, W, H, R, me_range, table, par, init, cm, c0, step, bind=1):
    mbw, mbh = W // 16, H // 16
    inp, outp = os.path.join(tmp, "in.bin"), os.path.join(tmp, "out.bin")
    with open(inp, "wb") as fh:
        fh.write(np.array([MAGIC, W, H, stride, origin, mbw, mbh, R, me_range, c0, step, bind], np.int64).tobytes())
        fh.write(planes[1].tobytes())
        fh.write(planes[0].tobytes())
        fh.write(np.ascontiguousarray(table, np.uint16).tobytes())
        fh.write(np.ascontiguousarray(par, np.int16).tobytes())
        fh.write(np.ascontiguousarray(init, np.int32).tobytes())
        fh.write(np.ascontiguousarray(cm, np.uint16).tobytes())
    r = subprocess.run([exe, inp, outp], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = np.fromfile(outp, np.uint8)
    n = (mbw * mbh + step - 1) // step
    dec = raw[:n * 12].view(np.int32).reshape(n, 3)
    calls, hits, misses, ns = raw[n * 12:].view(np.int64)
    return dec, int(calls), int(hits), int(misses), int(ns), r.stdout


@pytest.mark.gpu
def test_me_bind_esa_1080p(hip, oracle, tmp_path):
    from x264hip import synth
    exe = build(str(tmp_path))
    W, H, R = 1920, 1088, 16
    mbw, mbh = W // 16, H // 16
    nmb = mbw * mbh
    planes, stride, origin = synth.make_sequence(2, W, H, 8, seed=11)
    dev = torch.from_numpy(planes).cuda()
    fs = planes[0].size
    table = hip.me_search_full(dev[1:], origin, stride, dev[:1], origin, stride, mbw, mbh, 1, R,
                               fenc_frame_stride=fs, ref_frame_stride=fs)
    tab = table.cpu().numpy().view(np.uint16)[0]
    # the bound table is the oracle's (checked here so the decisions below test the lookup)
    want16 = oracle.me_search_full(8, planes[1].ravel(), origin, stride, planes[0].ravel(), origin, stride, mbw,
                                   mbh, R)
    assert np.array_equal(tab[..., :2 * R + 1], want16)
    # an oracle table wide enough for every window below (R 24), as the reference's direct SADs
    R2 = 24
    w2 = oracle.me_search_full(8, planes[1].ravel(), origin, stride, planes[0].ravel(), origin, stride, mbw,
                               mbh, R2).reshape(nmb, 2 * R2 + 1, 2 * R2 + 1)
    wide = np.zeros((nmb, 2 * R2 + 1, hip.me_table_pitch(R2)), w2.dtype)     # me_esa_argmin's pitched layout
    wide[:, :, :2 * R2 + 1] = w2
    rs = np.random.default_rng(2024)
    par = np.zeros((nmb, 8), np.int16)
    par[:, 0] = rs.integers(-1, 2, nmb)
    par[:, 1] = rs.integers(-1, 2, nmb)
    par[:, 2] = rs.integers(-64, 65, nmb)
    par[:, 3] = rs.integers(-64, 65, nmb)
    mbx, mby = np.arange(nmb) % mbw, np.arange(nmb) // mbw
    par[:, 4] = -16 * mbx - 24
    par[:, 5] = -16 * mby - 24
    par[:, 6] = 16 * (mbw - 1 - mbx) + 20
    par[:, 7] = 16 * (mbh - 1 - mby) + 24
    init = rs.integers(0, 20000, nmb).astype(np.int32)
    init[::7] = 0
    cm, c0 = _cost_mv()
    # pass A: me_range 12, every MB -- every window candidate lies in the bound table
    dec, calls, hits, misses, ns, out = _run(exe, str(tmp_path), planes, stride, origin, W, H, R, 12, tab, par, init,
                                             cm, c0, 1)
    want = oracle.me_esa_argmin(8, wide, R2, 12, par, init, cm, c0)
    assert np.array_equal(dec, want), np.argwhere((dec != want).any(1))[:5]
    assert calls > 4_000_000 and hits == calls and misses == 0, out
    per_call_ns = ns / calls
    print("lookup mode: %.1f ns per COST_MV on hits (%d calls)" % (per_call_ns, calls))
    assert per_call_ns < 1000, per_call_ns
    # pass B: me_range 16 on every 97th MB -- windows reach rows / columns 17..19 beyond the
    # table, those candidates dispatch; the decisions stay exact
    step = 97
    dec, calls, hits, misses, ns, out = _run(exe, str(tmp_path), planes, stride, origin, W, H, R, 16, tab, par, init,
                                             cm, c0, step)
    want = oracle.me_esa_argmin(8, wide[::step], R2, 16, par[::step], init[::step], cm, c0)
    assert np.array_equal(dec, want), np.argwhere((dec != want).any(1))[:5]
    assert misses > 0 and hits > 0 and hits + misses == calls, out


@pytest.mark.gpu
def test_me_bind_sad_x4_and_unbound(hip, oracle):
    """sad_x3 / sad_x4 [PIXEL_16x16] answer from the table when every candidate hits; a
    fenc block that matches no MB, another plane and an unbound thread all dispatch; the
    results always equal the oracle's."""
    from x264hip import synth
    import ctypes
    W, H, R = 256, 128, 8
    mbw, mbh = W // 16, H // 16
    planes, stride, origin = synth.make_sequence(2, W, H, 8, seed=3)
    dev = torch.from_numpy(planes).cuda()
    fs = planes[0].size
    table = hip.me_search_full(dev[1:], origin, stride, dev[:1], origin, stride, mbw, mbh, 1, R,
                               fenc_frame_stride=fs, ref_frame_stride=fs)
    pixf = hip.pixel_init(8)
    f1, f0 = planes[1].ravel(), planes[0].ravel()
    fenc_buf = np.zeros(16 * 16, np.uint8)
    rs = np.random.default_rng(5)
    with hip.me_bind(8, f1, origin, f0, origin, stride, mbw, mbh, table, R) as b:
        b.stats(reset=True)
        nx4 = 0
        for mb in range(0, mbw * mbh, 3):
            mx_, my_ = mb % mbw, mb // mbw
            fo = origin + 16 * my_ * stride + 16 * mx_
            fenc_buf[:] = f1[fo + np.arange(16)[:, None] * stride + np.arange(16)].ravel()
            mvs = rs.integers(-R, R + 1, (4, 2))
            ptrs = [f0.ctypes.data + fo + int(my) * stride + int(mx) for mx, my in mvs]
            sc = (ctypes.c_int * 4)()
            pixf.sad_x4[hip.PIXEL_16x16](fenc_buf.ctypes.data, *ptrs, stride, sc)
            want = [oracle.cmp(8, "sad", 0, fenc_buf, 0, 16, f0, fo + int(my) * stride + int(mx), stride)
                    for mx, my in mvs]
            assert list(sc) == want
            nx4 += 4
            sc3 = (ctypes.c_int * 3)()
            pixf.sad_x3[hip.PIXEL_16x16](fenc_buf.ctypes.data, *ptrs[:3], stride, sc3)
            assert list(sc3) == want[:3]
            nx4 += 3
        hits, misses = b.stats()
        assert hits == nx4 and misses == 0
        # a fenc block no MB has: dispatch, exact
        odd = rs.integers(0, 256, 256).astype(np.uint8)
        p = f0.ctypes.data + origin + 3 * stride + 5
        got = pixf.sad[hip.PIXEL_16x16](odd.ctypes.data, 16, p, stride)
        assert got == oracle.cmp(8, "sad", 0, odd, 0, 16, f0, origin + 3 * stride + 5, stride)
        # a candidate in another plane: dispatch, exact
        got = pixf.sad[hip.PIXEL_16x16](fenc_buf.ctypes.data, 16, f1.ctypes.data + origin, stride)
        assert got == oracle.cmp(8, "sad", 0, fenc_buf, 0, 16, f1, origin, stride)
        assert b.stats()[1] == 2
    # unbound: every call dispatches
    _, m0 = hip.MeBinding(None).stats(reset=True)
    got = pixf.sad[hip.PIXEL_16x16](fenc_buf.ctypes.data, 16, f0.ctypes.data + origin, stride)
    assert got == oracle.cmp(8, "sad", 0, fenc_buf, 0, 16, f0, origin, stride)
    assert hip.MeBinding(None).stats() == (0, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("bd", [8, 10])
def test_me_bind_partitions_from_quadrant_tables(hip, oracle, bd):
    """With me_search_full8's quadrant tables bound (x264hip_*_me_bind_tables), sad / sad_x4 of
    PIXEL_16x8, 8x16, 8x8 -- and 16x16 with no 16x16 table -- answer from them for every
    partition of every MB (the ESA windows me.c searches per partition, analyse.c:1425-1546),
    equal to the oracle's SAD, at 8 and 10 bit (configs[4]'s high-profile lookup mode)."""
    from x264hip import synth
    import ctypes
    W, H, R = 192, 96, 8
    mbw, mbh = W // 16, H // 16
    planes, stride, origin = synth.make_sequence(2, W, H, bd, seed=21)
    dev = torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()
    fs = planes[0].size
    es = planes.itemsize
    t8 = hip.me_search_full8(dev[1:], origin, stride, dev[:1], origin, stride, mbw, mbh, 1, R,
                             fenc_frame_stride=fs, ref_frame_stride=fs)
    pixf = hip.pixel_init(bd)
    f1, f0 = planes[1].ravel(), planes[0].ravel()
    buf = np.zeros(16 * 16, planes.dtype)             # mb.pic.p_fenc: the MB at FENC_STRIDE
    rs = np.random.default_rng(9)
    parts = {hip.PIXEL_16x16: [(0, 0)], hip.PIXEL_16x8: [(0, 0), (0, 8)], hip.PIXEL_8x16: [(0, 0), (8, 0)],
             hip.PIXEL_8x8: [(0, 0), (8, 0), (0, 8), (8, 8)]}
    with hip.me_bind(bd, f1, origin, f0, origin, stride, mbw, mbh, None, R, table8=t8) as b:
        b.stats(reset=True)
        n = 0
        for mb in range(0, mbw * mbh, 2):
            mx_, my_ = mb % mbw, mb // mbw
            fo = origin + 16 * my_ * stride + 16 * mx_
            buf[:] = f1[fo + np.arange(16)[:, None] * stride + np.arange(16)].ravel()
            for ip, offs in parts.items():
                for px, py in offs:
                    mvs = rs.integers(-R, R + 1, (4, 2))
                    po = fo + py * stride + px
                    fb = buf.ctypes.data + es * (py * 16 + px)
                    ptrs = [f0.ctypes.data + es * (po + int(my) * stride + int(mx)) for mx, my in mvs]
                    want = [oracle.cmp(bd, "sad", ip, f1, po, stride, f0, po + int(my) * stride + int(mx), stride)
                            for mx, my in mvs]
                    assert pixf.sad[ip](fb, 16, ptrs[0], stride) == want[0], (ip, px, py)
                    sc = (ctypes.c_int * 4)()
                    pixf.sad_x4[ip](fb, *ptrs, stride, sc)
                    assert list(sc) == want, (ip, px, py)
                    n += 5
        hits, misses = b.stats()
        assert hits == n and misses == 0, (hits, misses, n)
