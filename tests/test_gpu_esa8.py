"""GPU parity: ESA decisions of every MB's eight sub-partitions (x264hip_*_me_search_esa8; the
plain exhaustive form of encoder/me.c:618-631 for PIXEL_16x8 / 8x16 / 8x8 at the offsets of
analyse.c:1425,1480,1546) against the oracle (oracle/oracle.c me_search_esa8), bit-exact: the
shared-template pass alone (every window centred on the MB's template), with the direct pass
for windows moved off it or clipped at the frame edges, and the direct pass alone (range 0,
10 bit)."""
import numpy as np
import pytest
import torch

import esa8_cases as ec

pytestmark = pytest.mark.gpu


def _run(hip, oracle, bd, W, H, nf, R, me_range, seed, **kw):
    from x264hip import synth
    planes, stride, origin = synth.make_sequence(nf + 1, W, H, bd, seed=seed)
    mbw, mbh = W // 16, H // 16
    nmb = mbw * mbh
    cm, c0 = ec.cost_mv()
    cen, par, ic = [], [], []
    for f in range(nf):
        c, p, i = ec.jobs(mbw, mbh, me_range, seed=seed * 10 + f, **kw)
        cen.append(c), par.append(p), ic.append(i)
    cen, par, ic = np.concatenate(cen), np.concatenate(par), np.concatenate(ic)
    dev = torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()
    fs = planes[0].size
    out = hip.me_search_esa8(dev[1:], origin, stride, dev[:-1], origin, stride, mbw, mbh, nf, R, me_range,
                             torch.from_numpy(cen).cuda(), torch.from_numpy(par).cuda(), torch.from_numpy(ic).cuda(),
                             (torch.from_numpy(cm.view(np.int16)).cuda(), c0), fenc_frame_stride=fs,
                             ref_frame_stride=fs)
    got = out.cpu().numpy()
    for f in range(nf):
        sl = slice(8 * nmb * f, 8 * nmb * (f + 1))
        want = oracle.me_search_esa8(bd, planes[f + 1].ravel(), origin, stride, planes[f].ravel(), origin, stride,
                                     mbw, mbh, me_range, par[sl], ic[sl], cm, c0)
        bad = np.argwhere((got[sl] != want).any(1)).ravel()
        assert len(bad) == 0, f"frame {f}: partitions {bad[:8]} got {got[sl][bad[:4]]} want {want[bad[:4]]}"
    return got, par, ic


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("R", [4, 8, 16, 24])
def test_esa8_template_only(hip, oracle, bd, R):
    """every partition's window centred on its MB's template centre (range = me_range): the
    shared-absdiff pass decides all of them (10 bit: column-pair lanes from the dword-aligned
    origin)"""
    got, par, ic = _run(hip, oracle, bd, 96, 64, 2, R, R, seed=R + bd, centre_amp=4)
    assert (got[:, 0] < ic).mean() > 0.3


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("R,me_range", [(16, 16), (8, 8), (16, 12), (0, 8)])
def test_esa8_moved_windows(hip, oracle, bd, R, me_range):
    """half the partitions start from a predictor up to 5 pixels off the MB's centre: their
    windows reach outside the template and the direct pass finishes them (10 bit and range 0:
    the direct pass alone)"""
    _run(hip, oracle, bd, 96, 64, 2, R, me_range, seed=3 + R + bd, spread=5, frac=0.5, centre_amp=6)


@pytest.mark.parametrize("R,me_range", [(16, 15), (16, 9), (24, 16), (8, 3)])
def test_esa8_odd_ranges(hip, oracle, R, me_range):
    """me_range below the template radius and odd (the width rounding then ends short of or at
    the template's last column), with a quarter of the windows moved"""
    _run(hip, oracle, 8, 96, 64, 2, R, me_range, seed=40 + R + me_range, spread=4, frac=0.25, centre_amp=5)


@pytest.mark.parametrize("limit", [0, 12])
def test_esa8_clipped(hip, oracle, limit):
    """mv_limit_fpel clips the windows at the frame edges (the width rounding then runs past
    max_x, me.c:626) and ties against high predictor costs"""
    _run(hip, oracle, 8, 80, 48, 2, 16, 16, seed=21 + limit, spread=2, frac=0.3, centre_amp=3, limit=limit,
         init="high")


def test_esa8_1080p_sampled(hip, oracle):
    """a 1080p frame at range 16 with x264-like partition spread: sampled MBs (corners, edges,
    random interior) against the oracle run on those MBs alone"""
    from x264hip import synth
    W, H, R = 1920, 1088, 16
    planes, stride, origin = synth.make_sequence(2, W, H, 8, seed=9)
    mbw, mbh = W // 16, H // 16
    cm, c0 = ec.cost_mv()
    cen, par, ic = ec.jobs(mbw, mbh, R, seed=9, spread=3, frac=0.25, centre_amp=5, limit=4)
    dev = torch.from_numpy(planes).cuda()
    fs = planes[0].size
    got = hip.me_search_esa8(dev[1:], origin, stride, dev[:1], origin, stride, mbw, mbh, 1, R, R,
                             torch.from_numpy(cen).cuda(), torch.from_numpy(par).cuda(), torch.from_numpy(ic).cuda(),
                             (torch.from_numpy(cm.view(np.int16)).cuda(), c0), fenc_frame_stride=fs,
                             ref_frame_stride=fs).cpu().numpy()
    rs = np.random.default_rng(2)
    mbs = {(0, 0), (0, mbw - 1), (mbh - 1, 0), (mbh - 1, mbw - 1)}
    mbs |= {(int(rs.integers(mbh)), int(rs.integers(mbw))) for _ in range(40)}
    for (y, x) in sorted(mbs):
        mb = y * mbw + x
        o = origin + 16 * (y * stride + x)
        p = par[8 * mb: 8 * mb + 8].copy()
        # the MB alone as a 1x1 frame (par holds its absolute mv limits)
        want = oracle.me_search_esa8(8, planes[1].ravel(), o, stride, planes[0].ravel(), o, stride, 1, 1, R, p,
                                     ic[8 * mb: 8 * mb + 8], cm, c0)
        assert np.array_equal(got[8 * mb: 8 * mb + 8], want), (y, x)


def test_esa8_args(hip):
    """bad range / me_range -> X264HIP_EINVAL; no MBs -> success"""
    L = hip.lib()
    fn = L.x264hip_8_me_search_esa8
    P = torch.zeros(64, dtype=torch.uint8, device="cuda")
    import ctypes
    ptr = ctypes.c_void_p(P.data_ptr())
    assert fn(ptr, 16, 0, ptr, 16, 0, 1, 1, 1, 12, 8, None, ptr, ptr, ptr, ptr, None) == -1       # range 12
    assert fn(ptr, 16, 0, ptr, 16, 0, 1, 1, 1, 16, 31, None, ptr, ptr, ptr, ptr, None) == -1      # me_range 31
    assert fn(ptr, 16, 0, ptr, 16, 0, 0, 1, 1, 16, 16, None, None, None, None, None, None) == 0
