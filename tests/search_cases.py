"""Shared inputs and the literal Python restatement of x264_me_search_ref (reference
encoder/me.c:182-798) for tests/test_cpu_search.py and tests/test_gpu_search.py: partition lists
with analyse.c-shaped limits (analyse.c:330-349), predictor / candidate lists shaped like
x264_mb_predict_mv_ref16x16's, and the search itself over numpy_ref's SAD / get_ref."""
import numpy as np

import numpy_ref as nr
import refine_cases as rc

MVC_MAX = 14
PIXEL_SIZE_SHIFT = [0, 1, 1, 2, 3, 3, 4]
RANGE_MUL = [[3, 3, 4, 4], [3, 4, 4, 4], [4, 4, 4, 5], [4, 4, 5, 6]]
HEX2 = [(-1, -2), (-2, 0), (-1, 2), (1, 2), (2, 0), (1, -2), (-1, -2), (-2, 0)]
MOD6M1 = [5, 0, 1, 2, 3, 4, 5, 0]
SQUARE1 = [(0, 0), (0, -1), (0, 1), (-1, 0), (1, 0), (-1, -1), (-1, 1), (1, -1), (1, 1)]
HEX4 = [(0, -4), (0, 4), (-2, -3), (2, -3), (-4, -2), (4, -2), (-4, -1), (4, -1), (-4, 0), (4, 0), (-4, 1), (4, 1),
        (-4, 2), (4, 2), (-2, 3), (2, 3)]


def jobs(mbw, mbh, nframes, i_pixel, seed, motion=(12, 8), spread=40, n_mvc=(0, 9)):
    """per partition: pos (frame, x, y), par int16 [n, 12] = (mvp x, y, mv_limit_fpel min x, y,
    max x, y, mv_min_spel x, y, mv_max_spel x, y, i_mvc, 0), mvc int16 [n, 14, 2]: predictors
    around the true motion with some zero / repeated / far entries (the cases x264_predictor_clip
    drops or clips)"""
    rs = np.random.default_rng(seed)
    pos, par, mvc = [], [], []
    for f in range(nframes):
        for mby in range(mbh):
            for mbx in range(mbw):
                for px, py in rc.PARTS[i_pixel]:
                    smin = (4 * (-16 * mbx - 24), 4 * (-16 * mby - 24))
                    smax = (4 * (16 * (mbw - mbx - 1) + 24), 4 * (16 * (mbh - mby - 1) + 24))
                    fmin = ((smin[0] >> 2) + 6, (smin[1] >> 2) + 6)
                    fmax = ((smax[0] >> 2) - 6, (smax[1] >> 2) - 6)
                    mvp = [int(motion[k] + rs.integers(-spread, spread + 1)) for k in range(2)]
                    if rs.random() < 0.15:
                        mvp = [0, 0]
                    k = int(rs.integers(n_mvc[0], n_mvc[1] + 1))
                    cand = np.zeros((MVC_MAX, 2), np.int16)
                    for i in range(k):
                        r = rs.random()
                        if r < 0.1:
                            v = (0, 0)
                        elif r < 0.2:
                            v = tuple(mvp)
                        elif r < 0.3:
                            v = (int(rs.integers(-400, 400)), int(rs.integers(-300, 300)))
                        else:
                            v = tuple(int(motion[q] + rs.integers(-spread, spread + 1)) for q in range(2))
                        cand[i] = v
                    pos.append((f, 16 * mbx + px, 16 * mby + py))
                    par.append((mvp[0], mvp[1], fmin[0], fmin[1], fmax[0], fmax[1], smin[0], smin[1], smax[0],
                                smax[1], k, 0))
                    mvc.append(cand)
    return np.array(pos, np.int32), np.array(par, np.int16), np.array(mvc, np.int16)


def _s32(v):
    return (int(v) + (1 << 31)) % (1 << 32) - (1 << 31)


def _pack(a, b):
    return (a & 0xFFFF) | ((b & 0xFFFF) << 16)


def search_ref_py(fenc, planes, fw, origin, stride, x, y, i_pixel, par, mvc, cm, c0, me_method, subme, me_range,
                  weight0=None, bd=8):
    """x264_me_search_ref's integer stage and qpel conversion (me.c:182-789) for one partition:
    returns (cost, mvx, mvy, cost_mv) and (fpel calls, get_ref calls)"""
    from test_cpu_refine_chroma import _weigh
    bw, bh = nr.SIZES[i_pixel]
    fb = nr.block(fenc, origin + y * stride + x, stride, bw, bh)
    nf = [0, 0]

    def fpel(mx, my):
        nf[0] += 1
        return nr.sad(fb, nr.block(fw, origin + (y + my) * stride + x + mx, stride, bw, bh))

    def hpel(mx, my):
        nf[1] += 1
        return nr.sad(fb, _weigh(nr.get_ref(planes, origin + y * stride + x, stride, mx, my, bw, bh), weight0, bd))

    mvp = (int(par[0]), int(par[1]))
    xmin, ymin, xmax, ymax = (int(v) for v in par[2:6])
    i_mvc = int(par[10])
    cmx = lambda v: int(cm[c0 + v - mvp[0]])
    cmy = lambda v: int(cm[c0 + v - mvp[1]])
    bits = lambda mx, my: cmx(4 * mx) + cmy(4 * my)
    inr = lambda mx, my: xmin <= mx <= xmax and ymin <= my <= ymax
    clip = lambda v, lo, hi: min(max(v, lo), hi)
    st = {"bcost": 1 << 28}

    def cost_mv(mx, my):
        c = fpel(mx, my) + bits(mx, my)
        if c < st["bcost"]:
            st["bcost"], st["bmx"], st["bmy"] = c, mx, my

    bpred_cost, bpred_mv = 1 << 28, 0
    if subme >= 3:
        bpx, bpy = clip(mvp[0], 4 * xmin, 4 * xmax), clip(mvp[1], 4 * ymin, 4 * ymax)
        pmv = _pack(bpx, bpy)
        pmx, pmy = (bpx + 2) >> 2, (bpy + 2) >> 2
        bpred_cost = hpel(bpx, bpy) + cmx(bpx) + cmy(bpy)
        pmv_cost = bpred_cost
        valid = []
        for i in range(i_mvc):
            v = _pack(int(mvc[i][0]), int(mvc[i][1]))
            if not v or v == pmv:
                continue
            valid.append((clip(int(mvc[i][0]), 4 * xmin, 4 * xmax), clip(int(mvc[i][1]), 4 * ymin, 4 * ymax)))
        if valid:
            tmp = [None, (bpx, bpy)] + valid
            bpred_cost <<= 4
            for i in range(1, len(valid) + 1):
                mx, my = tmp[i + 1]
                c = hpel(mx, my) + cmx(mx) + cmy(my)
                if (c << 4) + i < bpred_cost:
                    bpred_cost = (c << 4) + i
            bpx, bpy = tmp[(bpred_cost & 15) + 1]
            bpred_cost >>= 4
        st["bmx"], st["bmy"] = (bpx + 2) >> 2, (bpy + 2) >> 2
        bpred_mv = _pack(bpx, bpy)
        if bpred_mv & 0x00030003:
            cost_mv(st["bmx"], st["bmy"])
        else:
            st["bcost"] = bpred_cost
        if pmv:
            if st["bmx"] | st["bmy"]:
                cost_mv(0, 0)
        elif pmv_cost < st["bcost"]:
            st["bcost"], st["bmx"], st["bmy"] = pmv_cost, 0, 0
    else:
        pmx = clip((mvp[0] + 2) >> 2, xmin, xmax)
        pmy = clip((mvp[1] + 2) >> 2, ymin, ymax)
        st["bmx"], st["bmy"] = pmx, pmy
        pmv = _pack(pmx, pmy)
        st["bcost"] = fpel(pmx, pmy)
        valid = []
        for i in range(i_mvc):
            mx, my = (int(mvc[i][0]) + 2) >> 2, (int(mvc[i][1]) + 2) >> 2
            v = _pack(mx, my)
            if not v or v == pmv:
                continue
            valid.append((clip(mx, xmin, xmax), clip(my, ymin, ymax)))
        if valid:
            tmp = [None, (pmx, pmy)] + valid
            b = st["bcost"] << 4
            for i in range(1, len(valid) + 1):
                mx, my = tmp[i + 1]
                c = fpel(mx, my) + bits(mx, my)
                if (c << 4) + i < b:
                    b = (c << 4) + i
            st["bmx"], st["bmy"] = tmp[(b & 15) + 1]
            st["bcost"] = b >> 4
        if pmv:
            cost_mv(0, 0)

    hexs = me_method == 1
    if me_method == 0:
        b = st["bcost"] << 4
        bmx, bmy = st["bmx"], st["bmy"]
        i = me_range
        while True:
            cs = [fpel(bmx, bmy - 1) + bits(bmx, bmy - 1), fpel(bmx, bmy + 1) + bits(bmx, bmy + 1),
                  fpel(bmx - 1, bmy) + bits(bmx - 1, bmy), fpel(bmx + 1, bmy) + bits(bmx + 1, bmy)]
            for c, code in zip(cs, (1, 3, 4, 12)):
                if (c << 4) + code < b:
                    b = (c << 4) + code
            if not b & 15:
                break
            bmx -= _s32((b << 28) & 0xFFFFFFFF) >> 30
            bmy -= _s32((b << 30) & 0xFFFFFFFF) >> 30
            b &= ~15
            i -= 1
            if not (i and inr(bmx, bmy)):
                break
        st["bcost"], st["bmx"], st["bmy"] = b >> 4, bmx, bmy
    elif me_method == 3:
        # ESA: me.c:627-631's exhaustive form (the SEA of :750-768 gives the same decision)
        bmx, bmy = st["bmx"], st["bmy"]
        min_x, min_y = max(bmx - me_range, xmin), max(bmy - me_range, ymin)
        max_x, max_y = min(bmx + me_range, xmax), min(bmy + me_range, ymax)
        width = (max_x - min_x + 3) & ~3
        for my in range(min_y, max_y + 1):
            for mx in range(min_x, min_x + width):
                cost_mv(mx, my)
    elif me_method == 2:
        thresh = lambda v: st["bcost"] < (v >> PIXEL_SIZE_SHIFT[i_pixel])

        def dia1(cx, cy):
            st["omx"], st["omy"] = cx, cy
            for dx, dy in ((0, -1), (0, 1), (-1, 0), (1, 0)):
                cost_mv(cx + dx, cy + dy)

        def cross(start, x_max, y_max):
            omx, omy = st["omx"], st["omy"]
            for i in range(start, x_max, 2):
                if omx + i <= xmax:
                    cost_mv(omx + i, omy)
                if omx - i >= xmin:
                    cost_mv(omx - i, omy)
            for i in range(start, y_max, 2):
                if omy + i <= ymax:
                    cost_mv(omx, omy + i)
                if omy - i >= ymin:
                    cost_mv(omx, omy - i)

        cross_start = 1
        ucost1 = st["bcost"]
        dia1(pmx, pmy)
        if pmx | pmy:
            dia1(0, 0)
        if i_pixel == 6:                                     # PIXEL_4x4: goto me_hex2 (me.c:438-439)
            return _umh_tail_hex(st, fpel, bits, inr, me_range, subme, bpred_cost, bpred_mv, pmv, cmx, cmy, nf)
        ucost2 = st["bcost"]
        if (st["bmx"] | st["bmy"]) and ((st["bmx"] - pmx) | (st["bmy"] - pmy)):
            dia1(st["bmx"], st["bmy"])
        if st["bcost"] == ucost2:
            cross_start = 3
        st["omx"], st["omy"] = st["bmx"], st["bmy"]
        done = False
        if st["bcost"] == ucost2 and thresh(2000):
            for dx, dy in ((0, -2), (-1, -1), (1, -1), (-2, 0), (2, 0), (-1, 1), (1, 1), (0, 2)):
                cost_mv(st["omx"] + dx, st["omy"] + dy)
            if st["bcost"] == ucost1 and thresh(500):
                done = True
            elif st["bcost"] == ucost2:
                rng = (me_range >> 1) | 1
                cross(3, rng, rng)
                for dx, dy in ((-1, -2), (1, -2), (-2, -1), (2, -1), (-2, 1), (2, 1), (-1, 2), (1, 2)):
                    cost_mv(st["omx"] + dx, st["omy"] + dy)
                if st["bcost"] == ucost2:
                    done = True
                cross_start = rng + 2
        if not done:
            if i_mvc:
                denom = 1
                if i_mvc == 1:
                    mvd = 25 if i_pixel == 0 else abs(mvp[0] - int(mvc[0][0])) + abs(mvp[1] - int(mvc[0][1]))
                else:
                    denom = i_mvc - 1
                    mvd = 0
                    if i_pixel != 0:
                        mvd = abs(mvp[0] - int(mvc[0][0])) + abs(mvp[1] - int(mvc[0][1]))
                        denom += 1
                    for i in range(i_mvc - 1):
                        mvd += abs(int(mvc[i][0]) - int(mvc[i + 1][0])) + abs(int(mvc[i][1]) - int(mvc[i + 1][1]))
                sad_ctx = 0 if thresh(1000) else 1 if thresh(2000) else 2 if thresh(4000) else 3
                mvd_ctx = 0 if mvd < 10 * denom else 1 if mvd < 20 * denom else 2 if mvd < 40 * denom else 3
                me_range = me_range * RANGE_MUL[mvd_ctx][sad_ctx] >> 2
            cross(cross_start, me_range, me_range >> 1)
            for dx, dy in ((-2, -2), (-2, 2), (2, -2), (2, 2)):
                cost_mv(st["omx"] + dx, st["omy"] + dy)
            omx, omy = st["bmx"], st["bmy"]
            i = 1
            while True:
                for dx, dy in HEX4:
                    if inr(omx + dx * i, omy + dy * i):
                        cost_mv(omx + dx * i, omy + dy * i)
                i += 1
                if i > me_range >> 2:
                    break
            hexs = inr(st["bmx"], st["bmy"])
    return _umh_tail_hex(st, fpel, bits, inr, me_range, subme, bpred_cost, bpred_mv, pmv, cmx, cmy, nf, hexs)


def _umh_tail_hex(st, fpel, bits, inr, me_range, subme, bpred_cost, bpred_mv, pmv, cmx, cmy, nf, hexs=True):
    """the hexagon + square refine (me.c:344-419) when hexs, then the qpel conversion (me.c:774-789)"""
    if hexs:
        bmx, bmy = st["bmx"], st["bmy"]

        def x3(pts):
            return [fpel(bmx + dx, bmy + dy) + bits(bmx + dx, bmy + dy) for dx, dy in pts]
        c0s = x3([(-2, 0), (-1, 2), (1, 2)]) + x3([(2, 0), (1, -2), (-1, -2)])
        b = st["bcost"] << 3
        for c, code in zip(c0s, (2, 3, 4, 5, 6, 7)):
            if (c << 3) + code < b:
                b = (c << 3) + code
        if b & 7:
            d = (b & 7) - 2
            bmx += HEX2[d + 1][0]
            bmy += HEX2[d + 1][1]
            i = (me_range >> 1) - 1
            while i > 0 and inr(bmx, bmy):
                cs = x3([HEX2[d], HEX2[d + 1], HEX2[d + 2]])
                b &= ~7
                for c, code in zip(cs, (1, 2, 3)):
                    if (c << 3) + code < b:
                        b = (c << 3) + code
                if not b & 7:
                    break
                d += (b & 7) - 2
                d = MOD6M1[d + 1]
                bmx += HEX2[d + 1][0]
                bmy += HEX2[d + 1][1]
                i -= 1
        b >>= 3
        b <<= 4
        for k in range(8):
            dx, dy = SQUARE1[k + 1]
            c = fpel(bmx + dx, bmy + dy) + bits(bmx + dx, bmy + dy)
            if (c << 4) + k + 1 < b:
                b = (c << 4) + k + 1
        bmx += SQUARE1[b & 15][0]
        bmy += SQUARE1[b & 15][1]
        st["bcost"], st["bmx"], st["bmy"] = b >> 4, bmx, bmy
    bmx, bmy, bcost = st["bmx"], st["bmy"], st["bcost"]
    if subme < 3:
        cmv = bits(bmx, bmy)
        return (bcost + (cmv if _pack(bmx, bmy) == pmv else 0), 4 * bmx, 4 * bmy, cmv), tuple(nf)
    if bpred_cost < bcost:
        mx, my = bpred_mv & 0xFFFF, bpred_mv >> 16
        mx, my = mx - 65536 if mx >= 32768 else mx, my - 65536 if my >= 32768 else my
    else:
        mx, my = 4 * bmx, 4 * bmy
    return (min(bpred_cost, bcost), mx, my, cmx(mx) + cmy(my)), tuple(nf)


class MultiRef:
    """one current frame and nref references of it (x264's default ref = 3, common/base.c:384):
    weightp_cases.make_pair with one seed gives every pair the same texture as its `ref` frame,
    so that frame is the current one and each pair's shifted, noised `fenc` frame is a reference
    -- reference k shows the current frame moved by -shifts[k] with noise noises[k] (a noisier
    reference loses to a cleaner one: the content the early exit exists for).  refs[k] carries
    ChromaCase's fields (luma F, H, V, C; ref_c), the current frame fenc_y / fenc_c."""

    def __init__(self, bd, W, H, cf, seed, shifts=((3, 2), (-2, 1), (1, -3)), noises=(1, 8, 2)):
        import numpy_ref as nr
        import weightp_cases as wc
        self.bd, self.W, self.H, self.cf, self.shifts = bd, W, H, cf, shifts
        pairs = [wc.make_pair(bd, W, H, cf, seed=seed, shift=s, noise=z) for s, z in zip(shifts, noises)]
        cur = pairs[0][0]
        self.stride, self.origin, self.cs, self.co = cur.ys, cur.yo, cur.cs, cur.co
        self.fenc_y = cur.y.ravel()
        self.fenc_c = [cur.nv.ravel()] if cf in (1, 2) else [cur.u.ravel(), cur.v.ravel()]
        self.refs = []
        for _, r in pairs:
            o = type("Ref", (), {})()
            o.luma = [r.y.ravel()] + [h.ravel() for h in nr.hpel_planes(r.y, 32, W, H, bd)]
            if cf in (1, 2):
                o.ref_c = [r.nv.ravel()]
            else:
                o.ref_c = []
                for p in (r.u, r.v):
                    o.ref_c += [p.ravel()] + [h.ravel() for h in nr.hpel_planes(p, 32, W, H, bd)]
            self.refs.append(o)

    def jobs(self, k, i_pixel, seed):
        """search_cases.jobs around reference k's true motion (-4 * shift qpel)"""
        sx, sy = self.shifts[k]
        return jobs(self.W // 16, self.H // 16, 1, i_pixel, seed=seed, motion=(-4 * sx, -4 * sy))
