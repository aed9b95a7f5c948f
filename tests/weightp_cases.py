"""Shared inputs of the weighted-prediction tests (test_cpu_weightp.py, test_gpu_weightp.py):
frame pairs with a brightness fade (the case x264_weights_analyse exists for,
slicetype.c:284-501) in every chroma format, with their lowres planes, intra costs,
lowres motion vectors and frame statistics computed by the oracle."""
import numpy as np

PAD = 32


def _synth():
    import conftest
    conftest.load_package()
    from x264hip import synth
    return synth


def _tex(h, w, bd, seed):
    return _synth()._texture(h, w, bd, seed)


def _fade(src, a, b, bd, rs, noise=1):
    pmax = (1 << bd) - 1
    v = np.floor(src * a + b * (1 << (bd - 8)) + 0.5).astype(np.int64)
    if noise:
        v = v + rs.integers(-noise, noise + 1, size=v.shape)
    return np.clip(v, 0, pmax)


def _bordered(core, pad_y, pad_x, stride):
    h, w = core.shape
    return np.pad(core, ((pad_y, pad_y), (pad_x, stride - w - pad_x)), mode="edge")


def _nv12_bordered(u, v, pad_y, stride):
    """interleave U/V, edge-replicate per component (x264_frame_expand_border_chroma)"""
    h, w = u.shape
    pu = np.pad(u, ((pad_y, pad_y), (16, 16)), mode="edge")
    pv = np.pad(v, ((pad_y, pad_y), (16, 16)), mode="edge")
    out = np.zeros((h + 2 * pad_y, stride), u.dtype)
    out[:, 0:2 * (w + 32):2] = pu
    out[:, 1:2 * (w + 32):2] = pv
    return out


class Frame:
    """one frame: luma plane y [H+64, ys] ((0,0) at (32, 32)); chroma per format: 'nv' (4:2:0 /
    4:2:2 interleaved, (0,0) at (32, 32) in interleaved pixels) or 'u', 'v' (4:4:4, same
    geometry as luma)"""

    def __init__(self, bd, W, H, cf, y, c):
        self.bd, self.W, self.H, self.cf = bd, W, H, cf
        dt = np.uint8 if bd == 8 else np.uint16
        self.ys = _synth().plane_stride(W)
        self.y = _bordered(y, PAD, PAD, self.ys).astype(dt)
        self.yo = PAD * self.ys + PAD
        if cf in (1, 2):
            self.cs = (2 * (W // 2) + 128 + 63) // 64 * 64
            self.nv = _nv12_bordered(c[0], c[1], PAD, self.cs).astype(dt)
            self.co = PAD * self.cs + PAD
        elif cf == 3:
            self.cs = self.ys
            self.u = _bordered(c[0], PAD, PAD, self.cs).astype(dt)
            self.v = _bordered(c[1], PAD, PAD, self.cs).astype(dt)
            self.co = self.yo
        else:
            self.cs, self.co = 0, 0

    def chroma(self):
        return {1: [getattr(self, "nv", None), None], 2: [getattr(self, "nv", None), None],
                3: [getattr(self, "u", None), getattr(self, "v", None)]}.get(self.cf, [None, None])


def make_pair(bd, W, H, cf, luma_fade=(1.0, 0.0), chroma_fade=((1.0, 0.0), (1.0, 0.0)), seed=1, shift=(3, 2),
              noise=1, flat_ref_chroma=False):
    """(ref, fenc) Frames: fenc = the reference shifted by `shift` pixels with the fades applied
    (luma (a, b) and per chroma plane), b in 8-bit units"""
    rs = np.random.default_rng(seed)
    dx, dy = shift
    hs, vs = (1, 1) if cf == 1 else (1, 0) if cf == 2 else (0, 0)
    cw, ch = W >> hs, H >> vs
    ty = _tex(H + 16, W + 16, bd, seed)
    ref_y = ty[8:8 + H, 8:8 + W]
    fen_y = _fade(ty[8 + dy:8 + dy + H, 8 + dx:8 + dx + W], *luma_fade, bd, rs, noise)
    ref_c, fen_c = [], []
    if cf:
        for p in range(2):
            tc = _tex(ch + 16, cw + 16, bd, seed + 7 + p)
            if flat_ref_chroma:
                r = np.full((ch, cw), (1 << bd) // 2, np.int64)
                r[::7, ::5] += 1                                  # ssd > 0, tiny
            else:
                r = tc[8:8 + ch, 8:8 + cw]
            cdx, cdy = dx >> hs, dy >> vs
            src = tc[8 + cdy:8 + cdy + ch, 8 + cdx:8 + cdx + cw]
            ref_c.append(r)
            fen_c.append(_fade(src, *chroma_fade[p], bd, rs, noise))
    return Frame(bd, W, H, cf, ref_y, ref_c), Frame(bd, W, H, cf, fen_y, fen_c)


class Analysis:
    """the lookahead products weights_analyse reads, from the oracle: lowres planes of both
    frames, fenc's intra costs, fenc's lowres mvs against ref, both frames' statistics"""

    def __init__(self, oracle, ref, fenc, satd=True, search_mvs=True, intra_scale=1):
        bd, W, H, cf = fenc.bd, fenc.W, fenc.H, fenc.cf
        self.mbw, self.mbh = W // 16, H // 16
        self.ls = (W // 2 + 64 + 63) // 64 * 64
        self.lo = PAD * self.ls + PAD
        self.ref_lr = [p.copy() for p in oracle.frame_init_lowres(bd, ref.y.ravel(), ref.yo, ref.ys, W, H, self.ls)]
        self.fenc_lr = [p.copy() for p in oracle.frame_init_lowres(bd, fenc.y.ravel(), fenc.yo, fenc.ys, W, H,
                                                                   self.ls)]
        flat = [p.ravel() for p in self.fenc_lr]
        self.intra = oracle.lowres_intra_cost(bd, flat[0], self.lo, self.ls, self.mbw, self.mbh, satd=satd)[0]
        if intra_scale != 1:   # (10-bit tests: the reference caps raw 10-bit SATDs by shifted intra costs)
            self.intra = np.minimum(self.intra.astype(np.int64) * intra_scale, 65535).astype(np.uint16)
        self.mvs = None
        if search_mvs:
            self.mvs = oracle.lowres_inter_cost(bd, flat[0], [p.ravel() for p in self.ref_lr], self.lo, self.ls,
                                                self.mbw, self.mbh, self.intra, satd=satd)[0]
        self.fstats = self._stats(oracle, fenc)
        self.rstats = self._stats(oracle, ref)

    def _stats(self, oracle, f):
        planes = [f.y.ravel()] + [None if c is None else c.ravel() for c in f.chroma()]
        return oracle.frame_pixel_stats(f.bd, planes, [f.yo, f.co, f.co], [f.ys, f.cs, f.cs], self.mbw, self.mbh,
                                        f.cf)


def random_mvs(mbw, mbh, seed, lim=40):
    rs = np.random.default_rng(seed)
    return rs.integers(-lim, lim + 1, size=(mbw * mbh, 2)).astype(np.int16)


def candidates(seed, n=24, max_scale=127):
    """(weighted, scale, denom, offset) lists with the extremes: unweighted, denom 0 and 7, offsets -128 / 127"""
    rs = np.random.default_rng(seed)
    c = [(0, 1, 0, 0), (1, 64, 6, 0), (1, 127, 7, 127), (1, 1, 0, -128), (1, 0, 0, 5), (1, max_scale, 0, -128)]
    while len(c) < n:
        d = int(rs.integers(0, 8))
        c.append((1, int(rs.integers(0, max_scale + 1)), d, int(rs.integers(-128, 128))))
    return c
