"""GPU parity of the subpel-search inputs: half-pel planes (x264hip_*_hpel_filter,
reference x264_frame_filter + x264_frame_expand_border_filtered) and quarter-pel
SAD / SATD candidates through get_ref (x264hip_*_subpel_cmp_batch, reference
refine_subpel encoder/me.c:865-992)."""
import numpy as np
import pytest

from conftest import load_package as _x
import torch

pytestmark = pytest.mark.gpu


def _dev(a, bd):
    return torch.from_numpy(a.view(np.int16) if bd == 10 else a).cuda()


def _host(t, bd):
    a = t.cpu().numpy()
    return a.view(np.uint16) if bd == 10 else a


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("size", [(1920, 1088), (80, 48), (176, 144), (976, 32)])
@pytest.mark.parametrize("variant", ["default", "nt", "plain", "unaligned"])
def test_hpel_filter(hip, oracle, bd, size, variant):
    """Every kernel form hpel_filter can take: at 8 bit the line-aligned strips, the 62-lane strips
    (976 wide: the right border piece would start a 64-piece chunk of its own) and, for planes
    whose rows are not 16-byte
    aligned (unaligned: the origin moved 4 pixels right), the fused LDS tiles, which also serve
    10 bit; with the default store policy, nontemporal stores forced (nt) or plain stores."""
    if variant in ("nt", "plain"):
        _x().set_variant("X264HIP_STREAM_NT", 1 if variant == "nt" else 0)
    from x264hip import synth
    W, H = size
    if variant == "unaligned" and W > 1000:
        pytest.skip("the shifted origin needs stride slack")
    gen = synth.make_sequence if W > 100 else synth.random_planes
    planes, stride, origin = gen(2, W, H, bd)
    if variant == "unaligned":
        origin += 4
    dev = _dev(planes, bd)
    outs = hip.hpel_filter(dev, origin, stride, W, H)
    for f in range(2):
        want = oracle.frame_filter(bd, planes[f].ravel().copy(), origin, stride, W, H)
        for o, w, name in zip(outs, want, "hvc"):
            got = _host(o, bd)[f][:, :W + 64]
            w2 = w.reshape(planes[f].shape)[:, :W + 64]
            assert np.array_equal(got, w2), (f, name, np.argwhere(got != w2)[:4])


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("W,H", [(176, 144), (976, 32)])
def test_hpel_filter_extremes(hip, oracle, bd, W, H):
    """Pixels 0 / PIXEL_MAX only, so the 6-tap sums reach both ends of every clip
    (H and V: -10 * max .. 42 * max before the shift; centre far beyond int16)."""
    from x264hip import synth
    planes, stride, origin = synth.random_planes(2, W, H, bd, seed=5)
    planes[:] = np.where(planes & 1, (1 << bd) - 1, 0).astype(planes.dtype)
    planes[1, ::3] = 0                       # runs of equal rows / columns too
    planes[1, :, 1::4] = (1 << bd) - 1
    outs = hip.hpel_filter(_dev(planes, bd), origin, stride, W, H)
    for f in range(2):
        want = oracle.frame_filter(bd, planes[f].ravel().copy(), origin, stride, W, H)
        for o, w, name in zip(outs, want, "hvc"):
            got = _host(o, bd)[f][:, :W + 64]
            w2 = w.reshape(planes[f].shape)[:, :W + 64]
            assert np.array_equal(got, w2), (f, name, np.argwhere(got != w2)[:4])


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("op", [0, 2])
def test_subpel_cmp_random(hip, oracle, bd, op):
    """a lane per candidate: unaligned multi-dword row loads at 8 bit, dword-aligned loads +
    alignbyte at 10 bit"""
    from x264hip import synth
    W, H = 160, 96
    planes, stride, origin = synth.random_planes(2, W, H, bd, seed=11)
    dev = _dev(planes, bd)
    hv = hip.hpel_filter(dev[:1], origin, stride, W, H)
    ref_planes = [dev[0]] + [o[0] for o in hv]
    host_planes = [planes[0].ravel()] + [_host(o, bd)[0].ravel() for o in hv]
    rs = np.random.default_rng(op + bd)
    for i_pixel in range(8):
        n = 3000
        bw, bh = hip.PIXEL_SIZES[i_pixel]
        bx = rs.integers(0, W - bw + 1, n)
        by = rs.integers(0, H - bh + 1, n)
        mvx = rs.integers(-4 * 20, 4 * 20 + 1, n)                # +-20 px incl. every qpel phase
        mvy = rs.integers(-4 * 20, 4 * 20 + 1, n)
        qxy = np.stack([4 * bx + mvx, 4 * by + mvy], 1).astype(np.int32)
        fo = (planes[0].size + origin + by * stride + bx).astype(np.int64)   # fenc = frame 1
        got = hip.subpel_cmp_batch(op, i_pixel, dev.view(-1), stride, ref_planes, origin, stride,
                                   torch.from_numpy(fo).cuda(), torch.from_numpy(qxy).cuda()).cpu().numpy()
        want = oracle.subpel_list(bd, op, i_pixel, planes.ravel(), stride, host_planes, origin, stride, fo, qxy)
        assert np.array_equal(got, want), (i_pixel, np.argwhere(got != want)[:3])


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("op", [0, 2])
def test_subpel_qpel9_random(hip, oracle, bd, op):
    """the 3x3 quarter-pel neighbourhood entry equals nine get_ref + SAD / SATD candidates of
    the oracle (me.c:950-963, mc.c:221-249): half-pel centres in all four phase combinations
    (the register-window path, both diagonal pairings of x264_hpel_ref0/1), quarter-pel
    centres (the per-candidate path) mixed into the same waves, negative positions."""
    from x264hip import synth
    W, H = 160, 96
    planes, stride, origin = synth.random_planes(2, W, H, bd, seed=13)
    dev = _dev(planes, bd)
    hv = hip.hpel_filter(dev[:1], origin, stride, W, H)
    ref_planes = [dev[0]] + [o[0] for o in hv]
    host_planes = [planes[0].ravel()] + [_host(o, bd)[0].ravel() for o in hv]
    rs = np.random.default_rng(31 * op + bd)
    for i_pixel in range(4):
        n = 2000
        bw, bh = hip.PIXEL_SIZES[i_pixel]
        bx = rs.integers(0, W - bw + 1, n)
        by = rs.integers(0, H - bh + 1, n)
        mvx = 2 * rs.integers(-2 * 20, 2 * 20 + 1, n)            # half-pel centres, +-20 px
        mvy = 2 * rs.integers(-2 * 20, 2 * 20 + 1, n)
        odd = rs.random(n) < 0.15                                  # some quarter-pel centres
        mvx[odd] += rs.integers(-1, 2, odd.sum()) | 1
        cxy = np.stack([4 * bx + mvx, 4 * by + mvy], 1).astype(np.int32)
        fo = (planes[0].size + origin + by * stride + bx).astype(np.int64)
        got = hip.subpel_qpel9_batch(op, i_pixel, dev.view(-1), stride, ref_planes, origin, stride,
                                     torch.from_numpy(fo).cuda(), torch.from_numpy(cxy).cuda()).cpu().numpy()
        k = np.arange(9)
        qxy = (cxy[:, None, :] + np.stack([k % 3 - 1, k // 3 - 1], 1)[None]).reshape(-1, 2).astype(np.int32)
        want = oracle.subpel_list(bd, op, i_pixel, planes.ravel(), stride, host_planes, origin, stride,
                                  np.repeat(fo, 9), qxy).reshape(n, 9)
        assert np.array_equal(got, want), (i_pixel, np.argwhere(got != want)[:3])
    with pytest.raises(RuntimeError):
        hip.subpel_qpel9_batch(op, 4, dev.view(-1), stride, ref_planes, origin, stride,
                               torch.from_numpy(fo[:4]).cuda(), torch.from_numpy(cxy[:4]).cuda())


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("size", [(1920, 1088), (176, 144), (72, 40), (3840, 2160), (48, 32)])
@pytest.mark.parametrize("variant", ["default", "nt", "plain"])
def test_frame_init_lowres(hip, oracle, bd, size, variant):
    """x264_frame_init_lowres of 3 frames per call vs the oracle (8 bit: the two-row 16-pixel
    lanes for widths of whole MBs, else -- 72 wide, and 10 bit -- the dword kernel; nt / plain =
    nontemporal stores forced on / off, X264HIP_STREAM_NT); the source padding holds unrelated
    values (the reference duplicates column W / row H itself)."""
    if variant != "default":
        _x().set_variant("X264HIP_STREAM_NT", 1 if variant == "nt" else 0)
    W, H = size
    n = 3
    rs = np.random.default_rng(bd * 7 + W)
    stride = (W + 64 + 63) // 64 * 64
    pdt = np.uint8 if bd == 8 else np.uint16
    planes = rs.integers(0, 1 << bd, size=(n, H + 64, stride)).astype(pdt)
    planes[1, 32:40, 32:32 + W] = (1 << bd) - 1
    dev = torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()
    outs, ls = hip.frame_init_lowres(dev, 32 * stride + 32, stride, W, H)
    for f in range(n):
        want = oracle.frame_init_lowres(bd, planes[f].ravel(), 32 * stride + 32, stride, W, H, ls)
        for k in range(4):
            got = outs[k][f].cpu().numpy().view(pdt)
            assert np.array_equal(got[:, :W // 2 + 64], want[k][:, :W // 2 + 64]), (f, k)
