"""Inputs for the TESA tests (CPU restatement check and GPU parity): frames, the
ESA integral image, per-MB search parameters shaped like x264's (analyse.c:330-349
mv limits, a predictor centre, an mvp) and an x264-shaped mv cost table."""
import numpy as np

PAD = 32


def cost_mv(lam=40, span=16384):
    """symmetric lambda * bits table (analyse.c:143-157 shape); mvd 0 at index `span`."""
    i = np.arange(-span, span + 1)
    logs = np.where(i == 0, 0.718, 2.0 * np.log2(np.abs(i) + 1) + 1.718)
    return np.minimum((lam * logs + 0.5).astype(np.int64), 65535).astype(np.uint16), span


def params(mbw, mbh, me_range, seed, nframes=1, centre_spread=12, clip_frac=0.3):
    """par int16 [n, 8] = (bmx, bmy, mvp_x, mvp_y, mv_x_min, mv_y_min, mv_x_max, mv_y_max) and
    init_cost int32 [n].  Limits follow mv_limit_fpel (-16*mb_x - 24 ..), some tightened so
    windows clip; the rounded window and its integral sums stay inside the padding."""
    rs = np.random.default_rng(seed)
    n = nframes * mbw * mbh
    mb = np.arange(n) % (mbw * mbh)
    mbx, mby = mb % mbw, mb // mbw
    par = np.zeros((n, 8), np.int16)
    lo_x, lo_y = -16 * mbx - 24, -16 * mby - 24
    hi_x, hi_y = 16 * (mbw - 1 - mbx) + 24 - 4, 16 * (mbh - 1 - mby) + 24
    par[:, 0] = np.clip(rs.integers(-centre_spread, centre_spread + 1, n), lo_x, hi_x)
    par[:, 1] = np.clip(rs.integers(-centre_spread, centre_spread + 1, n), lo_y, hi_y)
    par[:, 2] = rs.integers(-64, 65, n)
    par[:, 3] = rs.integers(-64, 65, n)
    tight = rs.integers(0, me_range + 1, (n, 4)) * (rs.random((n, 4)) < clip_frac)
    par[:, 4] = np.minimum(lo_x + tight[:, 0], par[:, 0])
    par[:, 5] = np.minimum(lo_y + tight[:, 1], par[:, 1])
    par[:, 6] = np.maximum(hi_x - tight[:, 2], par[:, 0])
    par[:, 7] = np.maximum(hi_y - tight[:, 3], par[:, 1])
    init = rs.integers(500, 30000, n).astype(np.int32)
    init[5::13] = 1 << 30                             # no predictor: any candidate wins
    init[::11] = 0                                    # predictor unbeatable
    return par, init


def tesa_python(bd, fenc, f_org, ref, r_org, integral, i_org, stride, mbx, mby, me_range, satd, p, init_cost,
                cmv, c0, sad_fn, satd_fn):
    """Literal restatement of encoder/me.c:653-748 for one MB (independent of oracle.c:
    the prune loop keeps the reference's in-place index arithmetic).  sad_fn / satd_fn(ofs)
    score the 16x16 candidate at ref offset ofs.  Returns (cost, mx, my, n_cost_mv)."""
    bmx, bmy = int(p[0]), int(p[1])
    cx = lambda v: int(cmv[c0 + v - int(p[2])])     # noqa: E731  p_cost_mvx[v]
    cy = lambda v: int(cmv[c0 + v - int(p[3])])     # noqa: E731
    min_x, min_y = max(bmx - me_range, int(p[4])), max(bmy - me_range, int(p[5]))
    max_x, max_y = min(bmx + me_range, int(p[6])), min(bmy + me_range, int(p[7]))
    width = (max_x - min_x + 3) & ~3
    mbo_f = f_org + 16 * (mby * stride + mbx)
    mbo_r = r_org + 16 * (mby * stride + mbx)
    mbo_i = i_org + 16 * (mby * stride + mbx)
    blk = fenc[mbo_f:mbo_f + 16 * stride].reshape(16, stride)[:, :16].astype(np.int64)
    enc_dc = [int(blk[:8, :8].sum()), int(blk[:8, 8:].sum()), int(blk[8:, :8].sum()), int(blk[8:, 8:].sum())]
    delta = 8 * stride
    sad_thresh = 10 if me_range <= 16 else 11 if me_range <= 24 else 12
    bsad = sad_fn(mbo_r + bmy * stride + bmx) + cx(bmx * 4) + cy(bmy * 4)
    mvsads = []
    for my in range(min_y, max_y + 1):
        ycost = cy(my * 4)
        if bsad <= ycost:
            continue
        bsad -= ycost
        thresh = bsad * 17 >> 4
        xs = []
        for i in range(width):                        # ads4, pixel.c:759-803
            s = mbo_i + min_x + i + my * stride
            ads = (abs(enc_dc[0] - int(integral[s])) + abs(enc_dc[1] - int(integral[s + 8]))
                   + abs(enc_dc[2] - int(integral[s + delta])) + abs(enc_dc[3] - int(integral[s + delta + 8]))
                   + cx((min_x + i) * 4))
            if ads < thresh:
                xs.append(i)
        for i in xs:
            mx = min_x + i
            sad = sad_fn(mbo_r + mx + my * stride) + cx(mx * 4)
            if sad < bsad * sad_thresh >> 3:
                if sad < bsad:
                    bsad = sad
                mvsads.append([sad + ycost, mx, my])
        bsad += ycost
    limit = me_range >> 1
    sad_thresh = bsad * sad_thresh >> 3
    nmvsad = len(mvsads)
    while nmvsad > limit * 2 and sad_thresh > bsad:
        sad_thresh = (sad_thresh + bsad) >> 1
        i = 0
        while i < nmvsad and mvsads[i][0] <= sad_thresh:
            i += 1
        for j in range(i, nmvsad):
            mvsads[i] = list(mvsads[j])
            sad = mvsads[j][0] & 0xFFFFFFFF
            i += ((sad - (sad_thresh + 1)) & 0xFFFFFFFF) >> 31
        nmvsad = i
    while nmvsad > limit:
        bi = 0
        for i in range(1, nmvsad):
            if mvsads[i][0] > mvsads[bi][0]:
                bi = i
        nmvsad -= 1
        mvsads[bi] = list(mvsads[nmvsad])
    bcost = int(init_cost)
    for k in range(nmvsad):
        _, mx, my = mvsads[k]
        ofs = mbo_r + my * stride + mx
        cost = (satd_fn(ofs) if satd else sad_fn(ofs)) + cx(mx * 4) + cy(my * 4)
        if cost < bcost:
            bcost, bmx, bmy = cost, mx, my
    return bcost, bmx, bmy, nmvsad
