"""Shared inputs of the bipred refine tests (test_cpu_bidir.py, test_gpu_bidir.py) and the literal
Python restatement of x264_me_refine_bidir_satd (reference encoder/me.c:994-1183, rd = 0) over
numpy_ref's get_ref / SAD / SATD: a B frame between two references of search_cases.MultiRef (list
0 = reference 0, list 1 = reference 1), partitions starting near each list's true motion with
mvps around it, analyse.c-shaped spel limits, and bipred weights 32 (the rounding average) and
implicit weights != 32 (pixel_avg_weight_wxh, common/mc.c:77-99)."""
import numpy as np

import numpy_ref as nr
import refine_cases as rc

DIA4D = [(0, 0, 0, 0),
         (0, 0, 0, 1), (0, 0, 0, -1), (0, 0, 1, 0), (0, 0, -1, 0),
         (0, 1, 0, 0), (0, -1, 0, 0), (1, 0, 0, 0), (-1, 0, 0, 0),
         (0, 0, 1, 1), (0, 0, -1, -1), (0, 1, 1, 0), (0, -1, -1, 0),
         (1, 1, 0, 0), (-1, -1, 0, 0), (1, 0, 0, 1), (-1, 0, 0, -1),
         (0, 1, 0, 1), (0, -1, 0, -1), (1, 0, 1, 0), (-1, 0, -1, 0),
         (0, 0, -1, 1), (0, 0, 1, -1), (0, -1, 1, 0), (0, 1, -1, 0),
         (-1, 1, 0, 0), (1, -1, 0, 0), (1, 0, 0, -1), (-1, 0, 0, 1),
         (0, -1, 0, 1), (0, 1, 0, -1), (-1, 0, 1, 0), (1, 0, -1, 0)]


def jobs(mr, i_pixel, seed, weights=(32, 24, 44, 32, -8), spread=6):
    """per partition of the MultiRef's frame: pos (0, x, y), par int16 [n, 12] = (m0 mv x, y, m1 mv
    x, y, m0 mvp x, y, m1 mvp x, y, mv_min_spel x, y, mv_max_spel x, y), weight int32 [n]; a few
    partitions start on the limits' 8-qpel guard band (the early return)"""
    rs = np.random.default_rng(seed)
    mbw, mbh = mr.W // 16, mr.H // 16
    t0 = (-4 * mr.shifts[0][0], -4 * mr.shifts[0][1])
    t1 = (-4 * mr.shifts[1][0], -4 * mr.shifts[1][1])
    pos, par, wt = [], [], []
    for mby in range(mbh):
        for mbx in range(mbw):
            for px, py in rc.PARTS[i_pixel]:
                mn = (4 * (-16 * mbx - 24), 4 * (-16 * mby - 24))
                mx_ = (4 * (16 * (mbw - mbx - 1) + 24), 4 * (16 * (mbh - mby - 1) + 24))
                m0 = [int(t0[k] + rs.integers(-spread, spread + 1)) for k in range(2)]
                m1 = [int(t1[k] + rs.integers(-spread, spread + 1)) for k in range(2)]
                if len(pos) % 7 == 3:
                    m0[0] = mn[0] + 7                                    # inside the guard band
                p0 = [int(v + rs.integers(-12, 13)) for v in t0]
                p1 = [int(v + rs.integers(-12, 13)) for v in t1]
                pos.append((0, 16 * mbx + px, 16 * mby + py))
                par.append((m0[0], m0[1], m1[0], m1[1], p0[0], p0[1], p1[0], p1[1], mn[0], mn[1], mx_[0], mx_[1]))
                wt.append(int(weights[int(rs.integers(0, len(weights)))]))
    return np.array(pos, np.int32), np.array(par, np.int16), np.array(wt, np.int32)


def refine_bidir_py(fenc, planes0, planes1, origin, stride, x, y, i_pixel, satd, par, weight, cm, c0, bd):
    """me_refine_bidir with rd = 0, literally: returns ((m0x, m0y, m1x, m1y), bcost, calls | passes << 16)"""
    bw, bh = nr.SIZES[i_pixel]
    fb = nr.block(fenc, origin + y * stride + x, stride, bw, bh)
    off = origin + y * stride + x
    bm = [int(v) for v in par[0:4]]
    mvp = [int(v) for v in par[4:8]]
    mn, mx_ = (int(par[8]), int(par[9])), (int(par[10]), int(par[11]))
    cost = lambda v, p: int(cm[c0 + v - p])
    pmax = (1 << bd) - 1
    bcost, calls, passes = 1 << 28, 0, 0
    if (bm[1] < mn[1] + 8 or bm[3] < mn[1] + 8 or bm[1] > mx_[1] - 8 or bm[3] > mx_[1] - 8 or
            bm[0] < mn[0] + 8 or bm[2] < mn[0] + 8 or bm[0] > mx_[0] - 8 or bm[2] > mx_[0] - 8):
        return tuple(bm), bcost, 0
    visited = set()
    for pss in range(8):
        passes += 1
        bestj = 0
        for j in range(1 if pss else 0, 33):
            m = [bm[k] + DIA4D[j][k] for k in range(4)]
            key = (m[0] & 7, m[1] & 7, m[2] & 7, m[3] & 7)
            if pss and key in visited:
                continue
            visited.add(key)
            a = nr.get_ref(planes0, off, stride, m[0], m[1], bw, bh)
            b = nr.get_ref(planes1, off, stride, m[2], m[3], bw, bh)
            if weight == 32:
                avg = (a + b + 1) >> 1
            else:
                avg = np.clip((a * weight + b * (64 - weight) + 32) >> 6, 0, pmax)
            c = (nr.satd(fb, avg) if satd else nr.sad(fb, avg)) + cost(m[0], mvp[0]) + cost(m[1], mvp[1]) + \
                cost(m[2], mvp[2]) + cost(m[3], mvp[3])
            calls += 1
            if c < bcost:
                bcost, bestj = c, j
        if not bestj:
            break
        bm = [bm[k] + DIA4D[bestj][k] for k in range(4)]
    return tuple(bm), bcost, calls | (passes << 16)
