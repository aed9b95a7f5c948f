"""GPU parity: full-resolution refine_subpel (x264hip_*_me_refine_subpel, reference
encoder/me.c:865-992) against the oracle restatement, over partition sizes, subme levels
(1, 2, 4, 7, 9: every branch of the hpel / qpel schedule), x264_me_search_ref's and
x264_me_refine_qpel's iteration sets, fpelcmp = SAD and = SATD (TESA), 8 and 10 bit, with
mv limits shaped like analyse.c:336-349 and start mvs at full-, half- and quarter-pel."""
import numpy as np
import pytest
import torch

import refine_cases as rc

pytestmark = pytest.mark.gpu


def _run(hip, oracle, bd, W, H, nframes, i_pixel, subme, refine_qpel, fpel_satd, seed):
    from x264hip import synth
    planes, stride, origin = synth.make_sequence(nframes + 1, W, H, bd, seed=seed)
    dev = torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()
    ref = dev[:-1]
    hv = hip.hpel_filter(ref, origin, stride, W, H)
    gplanes = [ref] + list(hv)
    mbw, mbh = W // 16, H // 16
    pos, par, cost = rc.jobs(mbw, mbh, nframes, i_pixel, seed + subme, cost_scale=1 << (bd - 8))
    cm, c0 = rc.cost_mv()
    cmd = torch.from_numpy(cm.view(np.int16)).cuda()
    fs = planes[0].size
    ne = torch.full((len(pos),), -1, dtype=torch.int32, device="cuda")
    got = hip.me_refine_subpel(dev[1:], origin, stride, gplanes, origin, stride, i_pixel, subme,
                               torch.from_numpy(pos).cuda(), torch.from_numpy(par).cuda(),
                               torch.from_numpy(cost).cuda(), (cmd, c0), refine_qpel=refine_qpel,
                               fpel_satd=fpel_satd, fenc_frame_stride=fs, nevals=ne).cpu().numpy()
    ne = ne.cpu().numpy()
    hh = [h.cpu().numpy() for h in hv]
    if bd == 10:
        hh = [h.view(np.uint16) for h in hh]
    for f in range(nframes):
        sel = pos[:, 0] == f
        op = [planes[f].ravel()] + [h[f].ravel() for h in hh]
        want, wne = oracle.me_refine_subpel(bd, planes[f + 1].ravel(), origin, stride, op, origin, stride, i_pixel,
                                            subme, pos[sel, 1:], par[sel], cost[sel], cm, c0, refine_qpel, fpel_satd,
                                            counts=True)
        bad = np.argwhere((got[sel] != want).any(1))
        assert not len(bad), (f, bad[:4].ravel(), got[sel][bad[:4].ravel()], want[bad[:4].ravel()])
        assert np.array_equal(ne[sel], wne)              # the same cmp calls as the reference
    return got, par


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("i_pixel", [0, 1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("subme", [1, 2, 4, 7, 9])
@pytest.mark.parametrize("refine_qpel,fpel_satd", [(0, 0), (1, 0), (0, 1)])
def test_refine_subpel_small(hip, oracle, bd, i_pixel, subme, refine_qpel, fpel_satd):
    got, par = _run(hip, oracle, bd, 160, 96, 2, i_pixel, subme, refine_qpel, fpel_satd, seed=bd + 3 * i_pixel)
    if subme >= 4 and not refine_qpel and not fpel_satd:
        # the searches moved partitions (not a vacuous pass), to quarter-pel positions too
        assert (got[:, 1:3] != par[:, :2]).any(1).mean() > 0.02
        assert ((got[:, 1:3] & 1) != 0).any()


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("i_pixel", [0, 3, 4, 6])
def test_refine_subpel_1080p(hip, oracle, bd, i_pixel):
    """every partition of a 1920x1088 frame pair at subme 7 (x264's default preset), x264_me_search_ref's
    iterations (two hpel, two qpel)"""
    _run(hip, oracle, bd, 1920, 1088, 1, i_pixel, 7, 0, 0, seed=31 + bd)


def test_refine_subpel_args(hip):
    t = torch.zeros(64, dtype=torch.int32, device="cuda")
    p = torch.zeros((2, 160, 256), dtype=torch.uint8, device="cuda")
    pos = torch.zeros((1, 3), dtype=torch.int32, device="cuda")
    par = torch.zeros((1, 8), dtype=torch.int16, device="cuda")
    for i_pixel, subme in ((7, 7), (0, 0), (0, 12)):
        with pytest.raises(RuntimeError):
            hip.me_refine_subpel(p, 32 * 256 + 32, 256, [p, p, p, p], 32 * 256 + 32, 256, i_pixel, subme, pos, par,
                                 t[:1], (t.view(torch.int16), 0))

