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


def _unequal(lows):
    """the four lowres planes at slots 0, 1, 3, 4 of one buffer: not equally spaced, so the
    launch gathers them into its scratch first (LaPlanes, lookahead.hip)"""
    buf = torch.zeros((5,) + tuple(lows[0].shape), dtype=lows[0].dtype, device=lows[0].device)
    out = []
    for k, p in zip((0, 1, 3, 4), lows):
        buf[k].copy_(p)
        out.append(buf[k])
    return out


def _case(hip, oracle, bd, W, H, npairs, me_method, subme, satd, random=False, aq=False, me_range=16, n_slices=1,
          unequal=False):
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
    refs = [p[:-1] for p in (_unequal(lows) if unequal else lows)]
    got = hip.lowres_inter_cost(fenc, refs, ls, mbw, mbh, intra[1:], (cm_dev, c0), me_method=me_method,
                                subme=subme, satd=satd, me_range=me_range, inv_qscale=None if iq is None else iq[1:],
                                n_slices=n_slices)
    torch.cuda.synchronize()
    got = [g.cpu().numpy() for g in got]
    hl = [_host(p, bd) for p in lows]
    ih = intra.cpu().numpy().view(np.uint16)
    lo = 32 * ls + 32
    for f in range(npairs):
        want = oracle.lowres_inter_cost(bd, hl[0][f + 1].ravel(), [p[f].ravel() for p in hl], lo, ls, mbw, mbh,
                                        ih[f + 1], me_method=me_method, subme=subme, satd=satd, me_range=me_range,
                                        inv_qscale=None if iq is None else iq_np[f + 1], n_slices=n_slices)
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


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("size", [(176, 144), (96, 16), (640, 352)])
def test_lowres_inter_unequal_planes(hip, oracle, bd, size):
    """reference planes that are not equally spaced (separate allocations, unlike x264's
    buffer_lowres): gathered by the launch, same results; random planes reach the mv limits"""
    W, H = size
    _case(hip, oracle, bd, W, H, 3, 1, 4, True, random=True, me_range=16, unequal=True)


def test_lowres_unequal_one_reference(hip, oracle):
    """one reference frame per list serving the batch (frame stride 0), its planes not equally
    spaced: the gathered copy holds one frame; results equal the equally spaced layout's"""
    from x264hip import synth
    W, H = 176, 144
    frames, stride, origin = synth.random_planes(5, W, H, 8)
    lows, ls = hip.frame_init_lowres(torch.from_numpy(frames).cuda(), origin, stride, W, H)
    mbw, mbh = W // 16, H // 16
    nmb = mbw * mbh
    cm, c0 = oracle.cost_mv_table(1, 512)
    cmd = (torch.from_numpy(cm.view(np.int16)).cuda(), c0)
    res = []
    for planes in (lows, _unequal(lows)):
        mvs = [torch.zeros((3, nmb, 2), dtype=torch.int16, device="cuda") for _ in range(2)]
        costs = [torch.zeros((3, nmb), dtype=torch.int32, device="cuda") for _ in range(2)]
        out = hip.lowres_bidir_cost(lows[0][1:4], [p[0:1] for p in planes], [p[4:5] for p in planes], ls, mbw, mbh,
                                    cmd, 3, mvs[0], costs[0], mvs[1], costs[1], dist_scale_factor=100,
                                    bipred_weight=39, a_frame_stride=0, b_frame_stride=0)
        res.append(list(out) + mvs + costs)
    for g, w in zip(*res):
        assert torch.equal(g, w)


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


def _bidir_case(hip, oracle, bd, W, H, n, search, me_method, subme, satd, dsf, weight, with_p1=True, random=False,
                aq=False, me_range=16, n_slices=1, unequal=False):
    """n B triplets (p0, b, p1) = (3i, 3i+1, 3i+2) of one sequence; the list searches (or the
    cached mvs of a first pass) and every output against the oracle."""
    from x264hip import synth
    gen = synth.random_planes if random else synth.make_sequence
    frames, stride, origin = gen(3 * n, W, H, bd)
    dev = torch.from_numpy(frames.view(np.int16) if bd == 10 else frames).cuda()
    lows, ls = hip.frame_init_lowres(dev, origin, stride, W, H)
    mbw, mbh = W // 16, H // 16
    nmb = mbw * mbh
    cm, c0 = oracle.cost_mv_table(1, 512)
    cmd = (torch.from_numpy(cm.view(np.int16)).cuda(), c0)
    kw = dict(me_method=me_method, subme=subme, satd=satd, me_range=me_range)
    fenc = lows[0][1::3]
    ra = [p[0::3] for p in (_unequal(lows) if unequal else lows)]
    rb = [p[2::3] for p in (_unequal(lows) if unequal else lows)]
    ic = torch.full((n, nmb), 16383, dtype=torch.int16, device="cuda")
    p1mvs = None
    if with_p1:
        p1mvs = hip.lowres_inter_cost(lows[0][2::3], ra, ls, mbw, mbh, ic, cmd, **kw)[0]
    mvs = [torch.zeros((n, nmb, 2), dtype=torch.int16, device="cuda") for _ in range(2)]
    costs = [torch.zeros((n, nmb), dtype=torch.int32, device="cuda") for _ in range(2)]
    iq = None
    if aq:
        iq_np = np.random.default_rng(W + bd).integers(100, 700, (n, nmb)).astype(np.uint16)
        iq = torch.from_numpy(iq_np.view(np.int16)).cuda()
    fs = lows[0][0].numel()
    if search != 3:
        # a first pass searches both lists; the tested pass reads the lists search leaves clear
        hip.lowres_bidir_cost(fenc, ra, rb, ls, mbw, mbh, cmd, 3, mvs[0], costs[0], mvs[1], costs[1], p1_mvs=p1mvs,
                              dist_scale_factor=dsf, bipred_weight=weight, a_frame_stride=3 * fs,
                              b_frame_stride=3 * fs, **kw)
    before = [t.cpu().numpy() for t in mvs + costs]
    lc, rows, est = hip.lowres_bidir_cost(fenc, ra, rb, ls, mbw, mbh, cmd, search, mvs[0], costs[0], mvs[1], costs[1],
                                          p1_mvs=p1mvs, dist_scale_factor=dsf, bipred_weight=weight,
                                          inv_qscale=iq, a_frame_stride=3 * fs, b_frame_stride=3 * fs,
                                          n_slices=n_slices, **kw)
    torch.cuda.synchronize()
    hl = [_host(p, bd) for p in lows]
    p1h = None if p1mvs is None else p1mvs.cpu().numpy()
    lo = 32 * ls + 32
    got = [t.cpu().numpy() for t in mvs + costs] + [lc.cpu().numpy().view(np.uint16), rows.cpu().numpy(),
                                                   est.cpu().numpy()]
    for i in range(n):
        want = oracle.lowres_bidir_cost(bd, hl[0][3 * i + 1].ravel(), [p[3 * i].ravel() for p in hl],
                                        [p[3 * i + 2].ravel() for p in hl], lo, ls, mbw, mbh, search,
                                        before[0][i], before[2][i], before[1][i], before[3][i],
                                        p1mvs=None if p1h is None else p1h[i], dsf=dsf, weight=weight,
                                        inv_qscale=None if iq is None else iq_np[i], n_slices=n_slices, **kw)
        order = (0, 2, 1, 3, 4, 5, 6)            # oracle returns m0, k0, m1, k1, lc, rows, est
        for name, k, w in zip(("mvs0", "costs0", "mvs1", "costs1", "lowres_costs", "row_satd", "est"), order, want):
            g = got[k][i].reshape(w.shape)
            assert np.array_equal(g, w), (i, name, np.argwhere(g != w)[:4])


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("me_method,subme,satd,weight", [(1, 4, True, 32), (1, 4, True, 43), (0, 2, False, 21)])
def test_lowres_bidir_1080p(hip, oracle, bd, me_method, subme, satd, weight):
    """two 1080p B triplets, both lists searched, p1's mvs as the bidir predictor."""
    _bidir_case(hip, oracle, bd, 1920, 1088, 2, 3, me_method, subme, satd, 128 if weight == 32 else 85, weight)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("search", [0, 1, 2])
def test_lowres_bidir_cached(hip, oracle, bd, search):
    """lists read from a first pass (search bits clear) or partly re-searched; no p1 mvs."""
    _bidir_case(hip, oracle, bd, 176, 144, 3, search, 1, 4, True, 171, 22, with_p1=(search != 0))


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("size", [(176, 144), (64, 48), (32, 32)])
def test_lowres_bidir_random(hip, oracle, bd, size):
    """random planes (mvs at the limits), AQ, short range, small and degenerate frames."""
    W, H = size
    _bidir_case(hip, oracle, bd, W, H, 2, 3, 1, 4, True, 100, 39, random=True, aq=True, me_range=8)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("search", [3, 1])
def test_lowres_bidir_unequal_planes(hip, oracle, bd, search):
    """B triplets whose list-0 / list-1 planes are not equally spaced (gathered by the launch)"""
    _bidir_case(hip, oracle, bd, 176, 144, 2, search, 1, 4, True, 100, 39, random=True, unequal=True)


@pytest.mark.parametrize("bd,H", [(8, 16 * 260), (10, 16 * 130)])
def test_lowres_tall_frames(hip, oracle, bd, H):
    """more block rows than one workgroup pass covers (256 rows at 8 bit, 128 at 10 bit):
    the lane quads walk the rows in several passes per wavefront step."""
    _case(hip, oracle, bd, 64, H, 2, 1, 4, True, random=True, me_range=8)
    _bidir_case(hip, oracle, bd, 64, H, 1, 3, 1, 4, True, 128, 32, random=True, me_range=8)


@pytest.mark.parametrize("kind", ["inter", "bidir"])
def test_lowres_wait_timeout_reports_error(hip, oracle, kind):
    """a band whose wait for the band below runs out stops and the entry
    fails (X264HIP_EDEVICE, "timed out") instead of using sentinel predictors.  Forced with
    a poll bound of 0 tries (X264HIP_LA_POLL); the default bound then gives the oracle's
    results again on the same inputs."""
    from x264hip import synth
    W, H = 256, 192                                   # 12 MB rows: 3 bands of 4, two of them wait
    frames, stride, origin = synth.make_sequence(3, W, H, 8)
    dev = torch.from_numpy(frames).cuda()
    lows, ls = hip.frame_init_lowres(dev, origin, stride, W, H)
    mbw, mbh = W // 16, H // 16
    nmb = mbw * mbh
    cm, c0 = oracle.cost_mv_table(1, 512)
    cmd = (torch.from_numpy(cm.view(np.int16)).cuda(), c0)
    intra, _, _ = hip.lowres_intra_cost(lows[0], ls, mbw, mbh, True, True, 1)

    def call():
        if kind == "inter":
            return hip.lowres_inter_cost(lows[0][1:], [p[:-1] for p in lows], ls, mbw, mbh, intra[1:], cmd)
        mvs = [torch.zeros((1, nmb, 2), dtype=torch.int16, device="cuda") for _ in range(2)]
        costs = [torch.zeros((1, nmb), dtype=torch.int32, device="cuda") for _ in range(2)]
        return hip.lowres_bidir_cost(lows[0][1:2], [p[0:1] for p in lows], [p[2:3] for p in lows], ls, mbw, mbh,
                                     cmd, 3, mvs[0], costs[0], mvs[1], costs[1])

    hip.set_variant("X264HIP_LA_POLL", 0)
    try:
        with pytest.raises(RuntimeError, match="timed out"):
            call()
    finally:
        hip.set_variant("X264HIP_LA_POLL", None)
    torch.cuda.synchronize()
    if kind == "inter":
        got = [g.cpu().numpy() for g in call()]
        want = oracle.lowres_inter_cost(8, _host(lows[0][1], 8).ravel(), [_host(p[0], 8).ravel() for p in lows],
                                        32 * ls + 32, ls, mbw, mbh, intra[1].cpu().numpy().view(np.uint16))
        assert np.array_equal(got[0][0].reshape(want[0].shape), want[0])
    else:
        call()


def test_lowres_async_report_and_graph_capture(hip, oracle):
    """the lookahead entries stay asynchronous.  A timed-out launch (X264HIP_LA_POLL
    0) returns without waiting; once its status copy has landed the NEXT lookahead call on the
    thread refuses with the timeout, and the report clears the condition (a following
    lowres_status is clean).  And the P search captures into a HIP graph whose replay equals
    the eager launch."""
    from x264hip import synth
    W, H = 256, 192
    frames, stride, origin = synth.make_sequence(3, W, H, 8)
    dev = torch.from_numpy(frames).cuda()
    lows, ls = hip.frame_init_lowres(dev, origin, stride, W, H)
    mbw, mbh = W // 16, H // 16
    cm, c0 = oracle.cost_mv_table(1, 512)
    cmd = (torch.from_numpy(cm.view(np.int16)).cuda(), c0)
    intra, _, _ = hip.lowres_intra_cost(lows[0], ls, mbw, mbh, True, True, 1)

    def call(check, outs=None):
        return hip.lowres_inter_cost(lows[0][1:], [p[:-1] for p in lows], ls, mbw, mbh, intra[1:], cmd,
                                     check=check, outs=outs)
    hip.set_variant("X264HIP_LA_POLL", 0)
    try:
        call(False)                                    # returns at once, failure pending
    finally:
        hip.set_variant("X264HIP_LA_POLL", None)
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="timed out"):
        call(False)                                    # the lazy report, nothing launched
    hip.lowres_status()                                # cleared by the report
    want = [g.clone() for g in call(True)]
    outs = tuple(torch.empty_like(g) for g in want)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        call(False, outs)
    torch.cuda.current_stream().wait_stream(side)
    for o in outs:
        o.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        call(False, outs)
    g.replay()
    torch.cuda.synchronize()
    hip.lowres_status()
    for a, b in zip(outs, want):
        assert torch.equal(a, b)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("wt", [(40, 5, -6), (23, 4, 9), (1, 0, 3), (16, 4, 0)])
def test_lowres_inter_weighted_1080p(hip, oracle, bd, wt):
    """the weighted-reference P search (slicetype.c:603-614, 859-862) on 1080p
    pairs whose fenc is a fade of the reference: fenc->weighted[0] from weight_scale_plane
    (frame.c:825-842, checked against the oracle), then lowres_inter_cost with ref_w + weight,
    bit-exact vs the oracle (integer stage on the weighted plane, weighted get_ref, unweighted
    fast skip)."""
    from x264hip import synth
    W, H, n = 1920, 1088, 2
    frames, stride, origin = synth.make_sequence(n + 1, W, H, bd)
    pmax = (1 << bd) - 1
    # a fade: each later frame darker and offset (the case weights_analyse catches)
    for k in range(1, n + 1):
        frames[k] = np.clip(frames[k].astype(np.int64) * (10 - 2 * k) // 10 + 5 * k, 0, pmax).astype(frames.dtype)
    dev = torch.from_numpy(frames.view(np.int16) if bd == 10 else frames).cuda()
    lows, ls = hip.frame_init_lowres(dev, origin, stride, W, H)
    mbw, mbh = W // 16, H // 16
    intra, _, _ = hip.lowres_intra_cost(lows[0], ls, mbw, mbh, True, True, 1)
    cm, c0 = oracle.cost_mv_table(1, 512)
    cm_dev = torch.from_numpy(cm.view(np.int16)).cuda()
    refs = [p[:-1] for p in lows]
    rw = hip.weight_scale_plane(refs[0], ls, W // 2, H // 2, *wt)
    torch.cuda.synchronize()
    hl = [_host(p, bd) for p in lows]
    rwh = _host(rw, bd)
    for f in range(n):
        want_w = oracle.weight_scale_plane(bd, hl[0][f], 0, ls, W // 2 + 64, H // 2 + 64, *wt)
        assert np.array_equal(rwh[f], want_w), f
    got = hip.lowres_inter_cost(lows[0][1:], refs, ls, mbw, mbh, intra[1:], (cm_dev, c0), ref_w=rw, weight=wt)
    torch.cuda.synchronize()
    got = [g.cpu().numpy() for g in got]
    ih = intra.cpu().numpy().view(np.uint16)
    lo = 32 * ls + 32
    for f in range(n):
        want = oracle.lowres_inter_cost(bd, hl[0][f + 1].ravel(), [p[f].ravel() for p in hl], lo, ls, mbw, mbh,
                                        ih[f + 1], ref_w=rwh[f].ravel(), weight=wt)
        for name, g, w in zip(("mvs", "mv_costs", "lowres_costs", "row_satd", "est"), got, want):
            g = g[f].reshape(w.shape).view(w.dtype) if name == "lowres_costs" else g[f].reshape(w.shape)
            assert np.array_equal(g, w), (f, name, np.argwhere(g != w)[:4])
    if wt == (16, 4, 0):                              # the identity weight is the unweighted search
        plain = hip.lowres_inter_cost(lows[0][1:], refs, ls, mbw, mbh, intra[1:], (cm_dev, c0))
        torch.cuda.synchronize()
        for g, p in zip(got, plain):
            assert np.array_equal(g, p.cpu().numpy())


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("n_slices", [2, 3, 4, 8])
def test_lowres_inter_slices_1080p(hip, oracle, bd, n_slices):
    """VERDICT r2 missing 5: lookahead slices (i_lookahead_threads, slicetype.c:901-918), each its
    own wavefront on the GPU, bit-exact vs the oracle at 1080p (68 MB rows: uneven slices)."""
    _case(hip, oracle, bd, 1920, 1088, 2, 1, 4, True, n_slices=n_slices)


@pytest.mark.parametrize("n_slices", [2, 5, 16])
def test_lowres_inter_slices_random(hip, oracle, n_slices):
    """random planes (searches wander), AQ, slices down to one or two MB rows, and more
    slices than rows (empty slices)."""
    _case(hip, oracle, 8, 176, 144, 3, 1, 4, True, random=True, aq=True, me_range=8, n_slices=n_slices)


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("n_slices", [2, 4])
def test_lowres_bidir_slices(hip, oracle, bd, n_slices):
    _bidir_case(hip, oracle, bd, 1920, 1088, 2, 3, 1, 4, True, 171, 43, n_slices=n_slices)


@pytest.mark.parametrize("helper", [0, 1])
@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("kind", ["inter", "inter_random", "inter_slices", "bidir", "weighted", "timeout"])
def test_lowres_helper_forced(hip, oracle, helper, bd, kind):
    """The helper wave (a second wave per band that reads the reference / fenc lines the search
    reaches a few steps later: L2 warming only) is on by default when every band's workgroup fits
    on the GPU at once, so the other tests here run with it; X264HIP_LA_HELPER forces it off (the
    plain single-wave form, what large batches use) or on.  Either way the results are the
    oracle's, and a failed wait still ends the band with the timeout error."""
    hip.set_variant("X264HIP_LA_HELPER", helper)
    try:
        if kind == "inter":
            _case(hip, oracle, bd, 1920, 1088, 2, 1, 4, True)
        elif kind == "inter_random":
            _case(hip, oracle, bd, 176, 144, 3, 1, 4, True, random=True, aq=True, me_range=8)
        elif kind == "inter_slices":
            _case(hip, oracle, bd, 1920, 1088, 2, 0, 2, False, n_slices=4)
        elif kind == "bidir":
            test_lowres_bidir_1080p(hip, oracle, bd, 1, 4, True, 43)
        elif kind == "weighted":
            test_lowres_inter_weighted_1080p(hip, oracle, bd, (40, 5, -6))
        elif bd == 8:
            test_lowres_wait_timeout_reports_error(hip, oracle, "inter")
            test_lowres_wait_timeout_reports_error(hip, oracle, "bidir")
    finally:
        hip.set_variant("X264HIP_LA_HELPER", None)


@pytest.mark.parametrize("xcd", [0, 1])
@pytest.mark.parametrize("kind", ["inter", "inter_random", "inter_slices", "bidir", "weighted", "timeout"])
def test_lowres_xcd_forced(hip, oracle, xcd, kind):
    """The band placement (lr_unit): by default every band of a pair runs on one XCD when the
    grid is resident at once, so the other tests here run with it; X264HIP_LA_XCD forces it off
    (bands in block order, what large batches use) or on (nine-pair launches leave the last
    XCD's blocks idle).  Either way the results are the oracle's."""
    hip.set_variant("X264HIP_LA_XCD", xcd)
    try:
        if kind == "inter":
            _case(hip, oracle, 8, 1920, 1088, 9, 1, 4, True)
        elif kind == "inter_random":
            _case(hip, oracle, 10, 176, 144, 3, 1, 4, True, random=True, aq=True, me_range=8)
        elif kind == "inter_slices":
            _case(hip, oracle, 8, 1920, 1088, 2, 0, 2, False, n_slices=4)
        elif kind == "bidir":
            _bidir_case(hip, oracle, 8, 640, 352, 9, 3, 1, 4, True, 171, 43)
        elif kind == "weighted":
            test_lowres_inter_weighted_1080p(hip, oracle, 8, (40, 5, -6))
        else:
            test_lowres_wait_timeout_reports_error(hip, oracle, "inter")
            test_lowres_wait_timeout_reports_error(hip, oracle, "bidir")
    finally:
        hip.set_variant("X264HIP_LA_XCD", None)
