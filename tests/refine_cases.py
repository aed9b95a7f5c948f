"""Shared inputs of the refine_subpel tests (test_cpu_refine.py, test_gpu_refine.py): partition
lists with analyse.c-shaped mv limits and an x264-shaped mv cost table."""
import numpy as np

# partitions of an MB per i_pixel (16x16, 16x8, 8x16, 8x8): top-left offsets
PARTS = {0: [(0, 0)], 1: [(0, 0), (0, 8)], 2: [(0, 0), (8, 0)], 3: [(0, 0), (8, 0), (0, 8), (8, 8)]}
# the sub-8x8 partitions of each 8x8 (PIXEL_8x4 / 4x8 / 4x4, analyse.c:1685-1760)
_Q = [(0, 0), (8, 0), (0, 8), (8, 8)]
PARTS[4] = [(qx, qy + dy) for qx, qy in _Q for dy in (0, 4)]
PARTS[5] = [(qx + dx, qy) for qx, qy in _Q for dx in (0, 4)]
PARTS[6] = [(qx + dx, qy + dy) for qx, qy in _Q for dy in (0, 4) for dx in (0, 4)]


def cost_mv(lam=40, span=8192):
    """symmetric lambda * bits table (analyse.c:143-157 shape), mvd 0 at index span"""
    i = np.arange(-span, span + 1)
    logs = np.where(i == 0, 0.718, 2.0 * np.log2(np.abs(i) + 1) + 1.718)
    return np.minimum((lam * logs + 0.5).astype(np.int64), 65535).astype(np.uint16), span


def jobs(mbw, mbh, nframes, i_pixel, seed, motion=(12, 8), spread=24, cost_scale=1):
    """per partition: (frame, x, y), par = (mvx, mvy, mvp_x, mvp_y, mv_min_spel x, y, mv_max_spel
    x, y) and a start cost; start mvs around the sequence's true motion (qpel), inside
    [mv_min_spel + 24, mv_max_spel - 24] (the integer search's 6-pixel fpel border,
    analyse.c:333-349) so every candidate the schedule can reach lies in the padding"""
    rs = np.random.default_rng(seed)
    pos, par = [], []
    for f in range(nframes):
        for mby in range(mbh):
            for mbx in range(mbw):
                for px, py in PARTS[i_pixel]:
                    mn = (4 * (-16 * mbx - 24), 4 * (-16 * mby - 24))
                    mx_ = (4 * (16 * (mbw - mbx - 1) + 24), 4 * (16 * (mbh - mby - 1) + 24))
                    mv = [int(np.clip(motion[k] + rs.integers(-spread, spread + 1), mn[k] + 24, mx_[k] - 24))
                          for k in range(2)]
                    if rs.random() < 0.3:                                  # full-pel starts (bmv_spel)
                        mv = [int(np.clip(4 * ((v + 2) >> 2), mn[k] + 24, mx_[k] - 24)) for k, v in enumerate(mv)]
                    mvp = [int(v) for v in rs.integers(-40, 41, 2)]
                    pos.append((f, 16 * mbx + px, 16 * mby + py))
                    par.append((mv[0], mv[1], mvp[0], mvp[1], mn[0], mn[1], mx_[0], mx_[1]))
    pos = np.array(pos, np.int32)
    par = np.array(par, np.int16)
    cost = (rs.integers(200, 6000, len(pos)) * cost_scale).astype(np.int32)
    cost[::9] = 0                                                         # nothing beats the start
    return pos, par, cost


# ---------------------------------------------------------------- chroma ME / weighted references
# (x264's default preset: b_chroma_me on P slices at subme >= 5, common/macroblock.c:507-509)
LUMA2CHROMA = {1: [3, 4, 5, 6], 2: [2, 3, 7, 5], 3: [0, 1, 2, 3]}     # common/pixel.h:70-76


class ChromaCase:
    """one (ref, fenc) frame pair of weightp_cases.make_pair in chroma format cf with everything
    refine_subpel's chroma ME reads: the luma hpel planes, the NV12 / NV16 planes (4:2:0 / 4:2:2)
    or the U, V planes and their hpel planes (4:4:4).  fade: the luma / chroma fades of fenc
    (the content weighted references exist for)."""

    def __init__(self, bd, W, H, cf, seed=1, fade=False):
        import numpy_ref as nr
        import weightp_cases as wc
        lf, cfade = ((0.8, 20.0), ((0.9, 6.0), (1.1, -5.0))) if fade else ((1.0, 0.0), ((1.0, 0.0), (1.0, 0.0)))
        self.ref, self.fenc = wc.make_pair(bd, W, H, cf, luma_fade=lf, chroma_fade=cfade, seed=seed)
        self.bd, self.W, self.H, self.cf = bd, W, H, cf
        r, f = self.ref, self.fenc
        self.stride, self.origin = r.ys, r.yo
        self.luma = [r.y.ravel()] + [h.ravel() for h in nr.hpel_planes(r.y, 32, W, H, bd)]
        self.fenc_y = f.y.ravel()
        self.cs, self.co = r.cs, r.co
        if cf in (1, 2):
            self.fenc_c = [f.nv.ravel()]
            self.ref_c = [r.nv.ravel()]
        else:
            self.fenc_c = [f.u.ravel(), f.v.ravel()]
            self.ref_c = []
            for p in (r.u, r.v):
                self.ref_c += [p.ravel()] + [h.ravel() for h in nr.hpel_planes(p, 32, W, H, bd)]


# weights near the fades above (luma 0.8 * 32 / 32, +20; U 0.9, +6; V 1.1, -5), denom 0 on one
FADE_WEIGHTS = ((26, 5, 20), (29, 5, 6), (9, 3, -5))
FADE_WEIGHTS_DENOM0 = ((1, 0, 20), None, (1, 0, -5))
