"""GPU parity of the lookahead's lowres motion search (x264hip_*_lowres_inter_cost:
slicetype_mb_cost's P-frame inter leg, reference encoder/slicetype.c:514-713, 758-791,
with x264_me_search_ref / refine_subpel, encoder/me.c:182-420, 774-790, 865-992)
against the oracle, bit-exact, on lowres planes and intra costs produced by the GPU
(themselves pinned by test_gpu_mc / test_gpu_intra)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _host(t, bd):
    a = t.cpu().numpy()
    return a.view(np.uint16) if bd == 10 else a


def _case(hip, oracle, bd, W, H, npairs, me_method, subme, satd, random=False, aq=False, me_range=16):
    from x264hip import synth
    gen = synth.random_planes if random else synth.make_sequence
    frames, stride, origin = gen(npairs + 1, W, H, bd)
    dev = torch.from_numpy(frames.view(np.int16) if bd == 10 else frames).cuda()
    lows, ls = hip.frame_init_lowres(dev, origin, stride, W, H)
    mbw, mbh = W // 16, H // 16
    intra, _, _ = hip.lowres_intra_cost(lows[0], ls, mbw, mbh, satd, subme > 2, 1)
    cm, c0 = oracle.cost_mv_table(1, 512)
    cm_dev = torch.from_numpy(cm.view(np.int16)).cuda()
    iq = None
    if aq:
        iq_np = np.random.default_rng(W + bd).integers(100, 700, (npairs + 1, mbw * mbh)).astype(np.uint16)
        iq = torch.from_numpy(iq_np.view(np.int16)).cuda()
    fenc = lows[0][1:]
    refs = [p[:-1] for p in lows]
    got = hip.lowres_inter_cost(fenc, refs, ls, mbw, mbh, intra[1:], (cm_dev, c0), me_method=me_method,
                                subme=subme, satd=satd, me_range=me_range, inv_qscale=None if iq is None else iq[1:])
    torch.cuda.synchronize()
    got = [g.cpu().numpy() for g in got]
    hl = [_host(p, bd) for p in lows]
    ih = intra.cpu().numpy().view(np.uint16)
    lo = 32 * ls + 32
    for f in range(npairs):
        want = oracle.lowres_inter_cost(bd, hl[0][f + 1].ravel(), [p[f].ravel() for p in hl], lo, ls, mbw, mbh,
                                        ih[f + 1], me_method=me_method, subme=subme, satd=satd, me_range=me_range,
                                        inv_qscale=None if iq is None else iq_np[f + 1])
        names = ("mvs", "mv_costs", "lowres_costs", "row_satd", "est")
        for name, g, w in zip(names, got, want):
            g = g[f].reshape(w.shape).view(w.dtype) if name == "lowres_costs" else g[f].reshape(w.shape)
            assert np.array_equal(g, w), (f, name, np.argwhere(g != w)[:4])
    return got


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("me_method,subme,satd", [(1, 4, True), (0, 4, True), (0, 2, False), (1, 2, True)])
def test_lowres_inter_1080p(hip, oracle, bd, me_method, subme, satd):
    """two 1080p pairs of the synthetic sequence (half-pel lowres motion)."""
    _case(hip, oracle, bd, 1920, 1088, 2, me_method, subme, satd)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("size", [(176, 144), (64, 48), (32, 32), (96, 16)])
def test_lowres_inter_random(hip, oracle, bd, size):
    """uniform random planes (searches wander to the mv limits), small and degenerate
    frame sizes (mb_width or mb_height <= 2: every block scores), AQ on, short range."""
    W, H = size
    _case(hip, oracle, bd, W, H, 3, 1, 4, True, random=True, aq=True, me_range=8)


def test_lowres_inter_identical(hip, oracle):
    """ref == fenc: the fast skip everywhere (mv 0, cost 0)."""
    from x264hip import synth
    W, H = 256, 128
    frames, stride, origin = synth.make_sequence(1, W, H, 8)
    dev = torch.from_numpy(np.concatenate([frames, frames])).cuda()
    lows, ls = hip.frame_init_lowres(dev, origin, stride, W, H)
    mbw, mbh = W // 16, H // 16
    intra, _, _ = hip.lowres_intra_cost(lows[0], ls, mbw, mbh, True, True, 1)
    cm, c0 = oracle.cost_mv_table(1, 512)
    mvs, mvc, lc, rows, est = hip.lowres_inter_cost(lows[0][1:], [p[:-1] for p in lows], ls, mbw, mbh, intra[1:],
                                                    (torch.from_numpy(cm.view(np.int16)).cuda(), c0))
    assert not mvs.any().item() and not mvc.any().item()
    assert (lc.cpu().numpy().view(np.uint16) == (1 << 14) + 4).all()
