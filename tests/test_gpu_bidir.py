"""GPU parity: x264_me_refine_bidir_satd at full resolution (x264hip_*_me_refine_bidir_satd,
reference encoder/me.c:994-1183 with rd = 0) against the oracle restatement (pinned by
tests/test_cpu_bidir.py's literal Python restatement): every partition 16x16 .. 8x8, SATD and SAD
mbcmp, bipred weights 32 and != 32, 8 and 10 bit, the final mvs, the last bcost and the
reference's mbcmp-call and pass counts; and a whole 1920x1088 B frame."""
import numpy as np
import pytest
import torch

import bidir_cases as bc
import refine_cases as rc
import search_cases as sc

pytestmark = pytest.mark.gpu


def _t(a, bd):
    a = np.ascontiguousarray(a)
    return torch.from_numpy(a.view(np.int16) if bd == 10 else a).cuda()


def _run(hip, oracle, bd, W, H, i_pixel, satd, seed, weights=(32, 24, 44, 32, -8)):
    mr = sc.MultiRef(bd, W, H, 1, seed=seed)
    rows = mr.fenc_y.size // mr.stride
    fenc = _t(mr.fenc_y.reshape(1, rows, -1), bd)
    l0 = [_t(p.reshape(1, rows, -1), bd) for p in mr.refs[0].luma]
    l1 = [_t(p.reshape(1, rows, -1), bd) for p in mr.refs[1].luma]
    pos, par, wt = bc.jobs(mr, i_pixel, seed=seed + 3, weights=weights)
    cm, c0 = rc.cost_mv()
    cmd = torch.from_numpy(cm.view(np.int16)).cuda()
    n = len(pos)
    cost = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    ne = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    got = hip.me_refine_bidir(fenc, mr.origin, mr.stride, l0, l1, mr.origin, mr.stride, i_pixel,
                              torch.from_numpy(pos).cuda(), torch.from_numpy(par).cuda(), torch.from_numpy(wt).cuda(),
                              (cmd, c0), satd=satd, cost=cost, nevals=ne).cpu().numpy()
    want, wcost, wne = oracle.me_refine_bidir(bd, mr.fenc_y, mr.origin, mr.stride, mr.refs[0].luma, mr.refs[1].luma,
                                              mr.origin, mr.stride, i_pixel, satd, pos[:, 1:], par, wt, cm, c0)
    bad = np.argwhere((got != want).any(1)).ravel()
    assert not len(bad), (bad[:4], got[bad[:4]], want[bad[:4]])
    assert np.array_equal(cost.cpu().numpy(), wcost)
    assert np.array_equal(ne.cpu().numpy(), wne)
    return want, wne


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("i_pixel", [0, 1, 2, 3])
@pytest.mark.parametrize("satd", [1, 0])
def test_bidir_small(hip, oracle, bd, i_pixel, satd):
    want, ne = _run(hip, oracle, bd, 96, 64, i_pixel, satd, seed=40 + bd + i_pixel)
    assert (ne >> 16).max() >= 2 and (ne == 0).any()


@pytest.mark.parametrize("bd", [8, 10])
def test_bidir_1080p(hip, oracle, bd):
    """every 16x16 partition of a 1920x1088 B frame, SATD, weights 32 / 24 / 44 / -8"""
    want, ne = _run(hip, oracle, bd, 1920, 1088, 0, 1, seed=50 + bd)
    assert ((ne >> 16) >= 3).mean() > 0.2


def test_bidir_args(hip):
    t = torch.zeros(64, dtype=torch.int32, device="cuda")
    p = torch.zeros((1, 160, 256), dtype=torch.uint8, device="cuda")
    pos = torch.zeros((1, 3), dtype=torch.int32, device="cuda")
    par = torch.zeros((1, 12), dtype=torch.int16, device="cuda")
    w = torch.full((1,), 32, dtype=torch.int32, device="cuda")
    with pytest.raises(RuntimeError):
        hip.me_refine_bidir(p, 32 * 256 + 32, 256, [p] * 4, [p] * 4, 32 * 256 + 32, 256, 4, pos, par, w,
                            (t.view(torch.int16), 0))
