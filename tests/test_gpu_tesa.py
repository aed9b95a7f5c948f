"""GPU parity: TESA integer-pel search (x264hip_*_me_tesa, reference encoder/me.c:653-748)
against the oracle restatement (itself checked against a literal per-MB Python
restatement in test_cpu_tesa.py): small frames over every me_range class, SATD and
SAD fpelcmp, clipped windows, with and without a full-search table, and whole
1080p frames at 8 and 10 bit."""
import numpy as np
import pytest

from conftest import load_package as _x
import tesa_cases as tc
import torch

pytestmark = pytest.mark.gpu


def _setup(bd, W, H, kind, seed, nframes=1):
    from x264hip import synth
    if kind == "synthetic":
        planes, stride, org = synth.make_sequence(nframes + 1, W, H, bd, seed=seed)
    else:
        planes, stride, org = synth.random_planes(nframes + 1, W, H, bd, seed=seed)
    dev = torch.from_numpy(planes.view(np.int16) if bd == 10 else planes).cuda()
    return planes, stride, org, dev


def _oracle_frames(oracle, bd, planes, stride, org, H, mbw, mbh, me_range, satd, par, init, cmv, c0):
    n1 = mbw * mbh
    out = []
    for f in range(planes.shape[0] - 1):
        f1, f0 = planes[f + 1].ravel(), planes[f].ravel()
        integ = oracle.frame_integral(bd, f0, org, stride, H, tc.PAD, False).ravel()
        out.append(oracle.me_tesa(bd, f1, org, stride, f0, org, integ, tc.PAD * stride + tc.PAD, stride, mbw, mbh,
                                  me_range, satd, par[f * n1:(f + 1) * n1], init[f * n1:(f + 1) * n1], cmv, c0))
    return np.concatenate(out)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("me_range,satd,kind", [(16, True, "synthetic"), (16, True, "random"),
                                                (8, False, "synthetic"), (24, True, "random"),
                                                (4, True, "synthetic"), (32, False, "random"),
                                                (12, True, "random"), (9, False, "synthetic")])
@pytest.mark.parametrize("mode", ["internal", "kernel", "table"])
def test_tesa_small(hip, oracle, bd, me_range, satd, kind, mode):
    """internal: no table given (me_range <= 24 builds a centred table around the predictors,
    then scans it); kernel: X264HIP_TESA_VARIANT=1 forces the SADs computed in the scan (the
    kernel of me_range > 24); table: a caller's me_search_full table over [-16, 16]"""
    use_table = mode == "table"
    if mode == "kernel":
        hip.set_variant("X264HIP_TESA_VARIANT", 1)
    W, H, nf = 160, 96, 2
    planes, stride, org, dev = _setup(bd, W, H, kind, seed=me_range + bd, nframes=nf)
    mbw, mbh = W // 16, H // 16
    fs = planes[0].size
    integ = hip.frame_integral(dev[:-1], org, stride, H)
    par, init = tc.params(mbw, mbh, me_range, seed=bd * 13 + me_range, nframes=nf)
    cmv, c0 = tc.cost_mv()
    cm_dev = torch.from_numpy(cmv.view(np.int16)).cuda()
    table = None
    rng = 0
    if use_table:                # SADs inside [-16, 16] come from the table, the rest are computed
        rng = 16
        table = hip.me_search_full(dev[1:], org, stride, dev[:-1], org, stride, mbw, mbh, nf, rng,
                                   fenc_frame_stride=fs, ref_frame_stride=fs)
    got = hip.me_tesa(dev[1:], org, stride, dev[:-1], org, stride, integ, mbw, mbh, nf, me_range,
                      torch.from_numpy(par).cuda(), torch.from_numpy(init).cuda(), (cm_dev, c0), satd=satd,
                      table=table, rng=rng).cpu().numpy()
    want = _oracle_frames(oracle, bd, planes, stride, org, H, mbw, mbh, me_range, satd, par, init, cmv, c0)
    assert np.array_equal(got, want), np.argwhere((got != want).any(1))[:5]
    assert (got[::11, 0] == 0).all() and (got[:, 0] <= init).all()


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("me_range,rng", [(16, 16), (16, 24), (12, 16), (8, 8)])
def test_tesa_centred_table(hip, oracle, bd, me_range, rng):
    """a me_search_centred table around each MB's predictor (origin-aware lookup)."""
    W, H = 160, 96
    planes, stride, org, dev = _setup(bd, W, H, "random", seed=5)
    mbw, mbh = W // 16, H // 16
    integ = hip.frame_integral(dev[:1], org, stride, H)
    par, init = tc.params(mbw, mbh, me_range, seed=bd + 3)
    cmv, c0 = tc.cost_mv()
    cm_dev = torch.from_numpy(cmv.view(np.int16)).cuda()
    cen = torch.from_numpy(np.ascontiguousarray(par[:, :2])).cuda()
    table, origin = hip.me_search_centred(dev[1:], org, stride, dev[:1], org, stride, mbw, mbh, 1, rng, cen)
    got = hip.me_tesa(dev[1:], org, stride, dev[:1], org, stride, integ, mbw, mbh, 1, me_range,
                      torch.from_numpy(par).cuda(), torch.from_numpy(init).cuda(), (cm_dev, c0),
                      table=table, rng=rng, origin=origin).cpu().numpy()
    want = _oracle_frames(oracle, bd, planes, stride, org, H, mbw, mbh, me_range, True, par, init, cmv, c0)
    assert np.array_equal(got, want), np.argwhere((got != want).any(1))[:5]


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("tv", [None, 1])
def test_tesa_1080p(hip, oracle, bd, tv):
    """every MB of a 1920x1088 frame pair at me_range 16, SATD fpelcmp, vs the oracle
    (the internal centred table, and X264HIP_TESA_VARIANT=1's in-scan SADs)."""
    if tv is not None:
        hip.set_variant("X264HIP_TESA_VARIANT", tv)
    W, H, me_range = 1920, 1088, 16
    planes, stride, org, dev = _setup(bd, W, H, "synthetic", seed=21)
    mbw, mbh = W // 16, H // 16
    integ = hip.frame_integral(dev[:1], org, stride, H)
    par, init = tc.params(mbw, mbh, me_range, seed=bd + 40, centre_spread=6)
    cmv, c0 = tc.cost_mv()
    cm_dev = torch.from_numpy(cmv.view(np.int16)).cuda()
    got = hip.me_tesa(dev[1:], org, stride, dev[:1], org, stride, integ, mbw, mbh, 1, me_range,
                      torch.from_numpy(par).cuda(), torch.from_numpy(init).cuda(), (cm_dev, c0)).cpu().numpy()
    want = _oracle_frames(oracle, bd, planes, stride, org, H, mbw, mbh, me_range, True, par, init, cmv, c0)
    assert np.array_equal(got, want), np.argwhere((got != want).any(1))[:5]
