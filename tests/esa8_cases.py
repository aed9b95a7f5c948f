"""Shared inputs of the sub-partition ESA tests (x264hip_*_me_search_esa8): per-MB centres and
the eight partitions' me.c inputs (par = { bmx, bmy, mvp_x, mvp_y, mv_min_x, mv_min_y,
mv_max_x, mv_max_y }, init_cost), partition order 16x8 top / bottom, 8x16 left / right, 8x8
TL / TR / BL / BR (analyse.c:1425,1480,1546)."""
import numpy as np

# (i_pixel, x, y) of partition p inside its MB
PARTS = [(1, 0, 0), (1, 0, 8), (2, 0, 0), (2, 8, 0), (3, 0, 0), (3, 8, 0), (3, 0, 8), (3, 8, 8)]
SIZE = {1: (16, 8), 2: (8, 16), 3: (8, 8)}


def cost_mv(lam=40, span=4096):
    """an x264-shaped mv cost table (analyse.c:143-157): symmetric, lambda * bits; returns
    (table, index of mvd 0)."""
    i = np.arange(-span, span + 1)
    logs = np.where(i == 0, 0.718, 2.0 * np.log2(np.abs(i) + 1) + 1.718)
    return np.minimum((lam * logs + 0.5).astype(np.int64), 65535).astype(np.uint16), span


def jobs(mbw, mbh, me_range, seed, spread=0, frac=0.0, centre_amp=0, limit=None, init="random"):
    """centres int16 [nmb, 2] and par int16 [nmb*8, 8] / init_cost int32 [nmb*8].  A partition's
    window centre bmx is the MB's centre, moved by up to `spread` pixels for a fraction `frac`
    of the partitions (x264's partitions start from their own best predictor, analyse.c:1447);
    mv limits per MB as mv_limit_fpel (analyse.c:330-349) with `limit` extra pixels of the
    24-pixel margin clipped away (None: unclipped)."""
    rs = np.random.default_rng(seed)
    nmb = mbw * mbh
    cen = rs.integers(-centre_amp, centre_amp + 1, (nmb, 2)).astype(np.int16) if centre_amp else \
        np.zeros((nmb, 2), np.int16)
    par = np.zeros((nmb * 8, 8), np.int16)
    mbx, mby = np.arange(nmb) % mbw, np.arange(nmb) // mbw
    for p in range(8):
        sl = slice(p, None, 8)
        move = rs.random(nmb) < frac
        off = rs.integers(-spread, spread + 1, (nmb, 2)) if spread else np.zeros((nmb, 2), np.int64)
        par[sl, 0] = cen[:, 0] + np.where(move, off[:, 0], 0)
        par[sl, 1] = cen[:, 1] + np.where(move, off[:, 1], 0)
        par[sl, 2] = 4 * par[sl, 0] + rs.integers(-40, 41, nmb)          # mvp (qpel)
        par[sl, 3] = 4 * par[sl, 1] + rs.integers(-40, 41, nmb)
        m = 24 - (limit if limit is not None else 0)
        # mv_limit_fpel: the block may move up to the padding edge (here 24 - limit pixels)
        par[sl, 4] = -16 * mbx - m
        par[sl, 5] = -16 * mby - m
        par[sl, 6] = 16 * (mbw - 1 - mbx) + m
        par[sl, 7] = 16 * (mbh - 1 - mby) + m
        if limit is None:
            par[sl, 4], par[sl, 5] = -10000, -10000
            par[sl, 6], par[sl, 7] = 10000, 10000
    if init == "high":
        ic = np.full(nmb * 8, 1 << 30, np.int32)
    else:
        ic = rs.integers(0, 4000, nmb * 8).astype(np.int32)
    return cen, par, ic


def esa8_py(fenc, f_origin, fs, ref, r_origin, rs_, mbw, me_range, par, init_cost, cm, c0, mbs):
    """plain-Python / numpy restatement of me.c:618-631 per partition for the MBs `mbs`
    (the second restatement the oracle is checked against)."""
    out = {}
    for mb in mbs:
        for p, (ipix, px, py) in enumerate(PARTS):
            i = 8 * mb + p
            w, h = SIZE[ipix]
            bx, by = 16 * (mb % mbw) + px, 16 * (mb // mbw) + py
            q = [int(v) for v in par[i]]
            bmx, bmy, bcost = q[0], q[1], int(init_cost[i])
            min_x, min_y = max(bmx - me_range, q[4]), max(bmy - me_range, q[5])
            max_x, max_y = min(bmx + me_range, q[6]), min(bmy + me_range, q[7])
            width = (max_x - min_x + 3) & ~3
            fb = np.array([fenc[f_origin + (by + y) * fs + bx: f_origin + (by + y) * fs + bx + w] for y in range(h)],
                          np.int64)
            for my in range(min_y, max_y + 1):
                for mx in range(min_x, min_x + width):
                    o = r_origin + (by + my) * rs_ + bx + mx
                    rb = np.array([ref[o + y * rs_: o + y * rs_ + w] for y in range(h)], np.int64)
                    cost = int(np.abs(fb - rb).sum()) + int(cm[c0 + 4 * mx - q[2]]) + int(cm[c0 + 4 * my - q[3]])
                    if cost < bcost:
                        bcost, bmx, bmy = cost, mx, my
            out[i] = (bcost, bmx, bmy)
    return out
