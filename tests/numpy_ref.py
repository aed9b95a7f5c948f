"""Independent numpy restatement of the north-star kernels — TEST INFRASTRUCTURE.

Written in matrix / vectorised form, deliberately unlike oracle/oracle.c (which
follows the reference's loops and its packed two-lane SATD arithmetic), so
that the two restatements cross-check each other:

* SATD = sum over 4x4 tiles of (sum |H4 . D . H4^T|) >> 1 (reference
  common/pixel.c:265-332 computes the same value with packed 16/32-bit lanes);
* sub4x4_dct = (C4 . D . C4^T)^T with C4 the H.264 core transform, output in
  the reference's transposed order dct[x*4+y] (common/dct.c:157-189);
* DCT8_1D with its arithmetic shifts (common/dct.c:332-356), vectorised over
  blocks and with int16 wrap of the column-pass temps at 8 bit;
* QUANT_ONE in uint32 (common/quant.c:50-57);
* x264_cqm_init (common/set.c:73-206) vectorised over QP.
"""
import numpy as np

H4 = np.array([[1, 1, 1, 1], [1, 1, -1, -1], [1, -1, -1, 1], [1, -1, 1, -1]], np.int64)
C4 = np.array([[1, 1, 1, 1], [2, 1, -1, -2], [1, -1, -1, 1], [1, -2, 2, -1]], np.int64)
SIZES = [(16, 16), (16, 8), (8, 16), (8, 8), (8, 4), (4, 8), (4, 4), (4, 16)]


def block(buf, off, stride, w, h):
    idx = off + np.arange(h)[:, None] * stride + np.arange(w)[None, :]
    return buf[idx].astype(np.int64)


def sad(a, b):
    return int(np.abs(a - b).sum())


def ssd(a, b):
    return int(((a - b) ** 2).sum())


def satd(a, b):
    d = a - b
    h, w = d.shape
    t = d.reshape(h // 4, 4, w // 4, 4).transpose(0, 2, 1, 3)          # tiles [ty, tx, 4, 4]
    coef = np.einsum("ij,abjk,lk->abil", H4, t, H4)
    return int((np.abs(coef).sum(axis=(2, 3)) >> 1).sum())


def wrap(v, bd):
    """value as stored in a dctcoef (int16 at 8 bit, int32 at 10 bit)."""
    v = np.asarray(v, np.int64)
    if bd == 8:
        return ((v + 32768) & 0xFFFF) - 32768
    return ((v + (1 << 31)) & 0xFFFFFFFF) - (1 << 31)


def sub4x4_dct(d, bd):
    """d: [..., 4, 4] differences -> [..., 16] in reference order."""
    t = wrap(np.einsum("kx,...ix->...ki", C4, d), bd)        # first pass, tmp[k][i]
    o = wrap(np.einsum("kj,...ij->...ik", C4, t), bd)        # second pass, dct[i][k]
    return o.reshape(d.shape[:-2] + (16,))


def _dct8_1d(s):
    """s: [..., 8] along the last axis -> [..., 8]."""
    s07, s16, s25, s34 = s[..., 0] + s[..., 7], s[..., 1] + s[..., 6], s[..., 2] + s[..., 5], s[..., 3] + s[..., 4]
    a0, a1, a2, a3 = s07 + s34, s16 + s25, s07 - s34, s16 - s25
    d07, d16, d25, d34 = s[..., 0] - s[..., 7], s[..., 1] - s[..., 6], s[..., 2] - s[..., 5], s[..., 3] - s[..., 4]
    a4 = d16 + d25 + (d07 + (d07 >> 1))
    a5 = d07 - d34 - (d25 + (d25 >> 1))
    a6 = d07 + d34 - (d16 + (d16 >> 1))
    a7 = d16 - d25 + (d34 + (d34 >> 1))
    return np.stack([a0 + a1, a4 + (a7 >> 2), a2 + (a3 >> 1), a5 + (a6 >> 2),
                     a0 - a1, a6 - (a5 >> 2), (a2 >> 1) - a3, (a4 >> 2) - a7], axis=-1)


def sub8x8_dct8(d, bd):
    """d: [..., 8, 8] (row y, col x) -> [..., 64] with dct[x*8+i]."""
    cols = wrap(_dct8_1d(np.swapaxes(d, -1, -2)), bd)         # [..., i(col), x]  = tmp[x][i]
    tmp = np.swapaxes(cols, -1, -2)                           # tmp[y][x]
    rows = wrap(_dct8_1d(tmp), bd)                            # [..., i(row), x] -> dct[x*8+i]
    return np.swapaxes(rows, -1, -2).reshape(d.shape[:-2] + (64,))


def quadrant_blocks(d, n):
    """split a [..., 2n, 2n] block into 4 [n, n] blocks in reference order TL, TR, BL, BR."""
    return np.stack([d[..., :n, :n], d[..., :n, n:], d[..., n:, :n], d[..., n:, n:]], axis=-3)


def sub8x8_dct(d, bd):
    return sub4x4_dct(quadrant_blocks(d, 4), bd).reshape(d.shape[:-2] + (64,))


def sub16x16_dct(d, bd):
    q = quadrant_blocks(d, 8)                                  # [..., 4, 8, 8]
    return sub4x4_dct(quadrant_blocks(q, 4), bd).reshape(d.shape[:-2] + (256,))


def sub16x16_dct8(d, bd):
    return sub8x8_dct8(quadrant_blocks(d, 8), bd).reshape(d.shape[:-2] + (256,))


def sub8x8_dct_dc(d, bd):
    q = quadrant_blocks(d, 4).sum(axis=(-1, -2))               # [..., 4]
    q = wrap(q, bd)
    d0, d1, d2, d3 = q[..., 0] + q[..., 1], q[..., 2] + q[..., 3], q[..., 0] - q[..., 1], q[..., 2] - q[..., 3]
    return wrap(np.stack([d0 + d1, d0 - d1, d2 + d3, d2 - d3], -1), bd)


def sub8x16_dct_dc(d, bd):
    """d: [..., 16, 8]; 2x4 DC transform of the 8 4x4 sums (row-major 2 wide)."""
    s = d.reshape(d.shape[:-2] + (4, 4, 2, 4)).sum(axis=(-3, -1))   # [..., 4 rows, 2 cols]
    a = s.reshape(s.shape[:-2] + (8,))
    H2x4 = np.array([[1, 1, 1, 1, 1, 1, 1, 1],
                     [1, -1, 1, -1, 1, -1, 1, -1],
                     [1, 1, 1, 1, -1, -1, -1, -1],
                     [1, -1, 1, -1, -1, 1, -1, 1],
                     [1, 1, -1, -1, -1, -1, 1, 1],
                     [1, -1, -1, 1, -1, 1, 1, -1],
                     [1, 1, -1, -1, 1, 1, -1, -1],
                     [1, -1, -1, 1, 1, -1, -1, 1]], np.int64)
    return wrap(np.einsum("kj,...j->...k", H2x4, a), bd)


def dct4x4dc(d, bd):
    """in-place 4x4 DC Hadamard with (x+1)>>1 rounding (reference dct.c:47-76)."""
    d = np.asarray(d, np.int64).reshape(-1, 4, 4)
    Hd = np.array([[1, 1, 1, 1], [1, 1, -1, -1], [1, -1, -1, 1], [1, -1, 1, -1]], np.int64)
    t = wrap(np.einsum("kj,bij->bki", Hd, d), bd)              # tmp[k][i]
    o = np.einsum("kj,bij->bik", Hd, t)                        # d[i][k]
    return wrap((o + 1) >> 1, bd).reshape(-1, 16)


def quant(coef, mf, bias, bd):
    """QUANT_ONE over arrays (broadcast); returns (values as stored, nonzero flag per last axis)."""
    c = np.asarray(coef, np.int64)
    m = np.asarray(mf, np.uint64)
    f = np.asarray(bias, np.uint64)
    mag = np.where(c > 0, c, -c).astype(np.uint64)
    q = (((f + mag) & 0xFFFFFFFF) * m & 0xFFFFFFFF) >> 16
    q = q.astype(np.int64)
    v = wrap(np.where(c > 0, q, -q), bd)
    return v, (v != 0).any(axis=-1)


_QUANT4_SCALE = np.array([[13107, 8066, 5243], [11916, 7490, 4660], [10082, 6554, 4194],
                          [9362, 5825, 3647], [8192, 5243, 3355], [7282, 4559, 2893]], np.int64)
_QUANT8_SCALE = np.array([[13107, 11428, 20972, 12222, 16777, 15481], [11916, 10826, 19174, 11058, 14980, 14290],
                          [10082, 8943, 15978, 9675, 12710, 11985], [9362, 8228, 14913, 8931, 11984, 11259],
                          [8192, 7346, 13159, 7740, 10486, 9777], [7282, 6428, 11570, 6830, 9118, 8640]], np.int64)
_QUANT8_SCAN = np.array([0, 3, 4, 3, 3, 1, 5, 1, 4, 5, 2, 5, 3, 1, 5, 1])


def cqm_init(bd, lists, dz_inter=21, dz_intra=11, transform_8x8=True):
    qmax = 51 + 6 * (bd - 8)
    qs = np.arange(qmax + 1)
    dz = np.array([32 - dz_intra, 32 - dz_inter, 21, 11], np.int64)
    i16 = np.arange(16)
    i64 = np.arange(64)
    def4 = _QUANT4_SCALE[:, (i16 & 1) + ((i16 >> 2) & 1)]                  # [6, 16]
    def8 = _QUANT8_SCALE[:, _QUANT8_SCAN[((i64 >> 1) & 12) | (i64 & 3)]]   # [6, 64]
    ut = np.uint16 if bd == 8 else np.uint32

    def tables(defq, sl, nlists, shift_off, size):
        mf = np.zeros((4, qmax + 1, size), ut)
        bias = np.zeros((4, qmax + 1, size), ut)
        for l in range(nlists):
            s = np.asarray(sl[l], np.int64)[:size]
            base = (defq * 16 + (s >> 1)) // s                              # DIV, [6, size]
            b = base[qs % 6]                                                # [Q, size]
            sh = (qs // 6 + shift_off)[:, None]
            j = np.where(sh <= 0, b << np.maximum(-sh, 0), (b + (1 << np.maximum(sh - 1, 0))) >> np.maximum(sh, 0))
            mf[l] = (j & 0xFFFF).astype(ut)
            jj = np.where(j == 0, 1, j)
            bb = np.minimum(((dz[l] << 10) + (jj >> 1)) // jj, (1 << 15) // jj)
            bias[l] = np.where(j == 0, 0, bb).astype(ut)
        return mf, bias

    q4m, q4b = tables(def4, lists[:4], 4, -1, 16)
    q8m, q8b = (np.zeros((4, qmax + 1, 64), ut),) * 2
    if transform_8x8:
        q8m, q8b = tables(def8, lists[4:], 2, 0, 64)
    return q4m, q4b, q8m, q8b


def hpel_planes(plane2d, pad, width, height, bd):
    """H, V, C half-pel planes of a padded plane [h+2pad, stride] (reference
    hpel_filter mc.c:173-196 + border re-expansion frame.c:599-625), computed by
    vectorised 6-tap filtering on the interior x in [-4, W+4), y in [-8, H+8),
    then edge clamping over the padding."""
    p = plane2d.astype(np.int64)
    pm = (1 << bd) - 1
    padv = -10 * pm if bd > 9 else 0
    ys = np.arange(-8, height + 8) + pad
    xs = np.arange(-4, width + 4) + pad
    taps = np.array([1, -5, 20, 20, -5, 1])

    def vt(yy, xx):          # vertical tap at rows yy (centre rows y..y+1 as in TAPFILTER(src, stride))
        return sum(t * p[np.ix_(yy + k - 2, xx)] for k, t in enumerate(taps))

    v = vt(ys, xs)
    hsum = sum(t * p[np.ix_(ys, xs + k - 2)] for k, t in enumerate(taps))
    vwide = vt(ys, np.arange(-6, width + 7) + pad)            # intermediates for the centre filter
    b = wrap(vwide + padv, 8)                                  # int16 storage (mc.c:181)
    csum = sum(t * b[:, k:k + width + 8] for k, t in enumerate(taps))
    out = []
    for val in (np.clip((hsum + 16) >> 5, 0, pm), np.clip((v + 16) >> 5, 0, pm),
                np.clip((csum - 32 * padv + 512) >> 10, 0, pm)):
        full = np.zeros_like(p)
        yy = np.clip(np.arange(-pad, height + pad), -8, height + 7) + 8
        xx = np.clip(np.arange(-pad, width + pad), -4, width + 3) + 4
        full[pad - pad:height + 2 * pad, 0:width + 2 * pad] = val[np.ix_(yy, xx)]
        out.append(full.astype(plane2d.dtype))
    return out


HPEL_REF0 = [0, 1, 1, 1, 0, 1, 1, 1, 2, 3, 3, 3, 0, 1, 1, 1]
HPEL_REF1 = [0, 0, 1, 0, 2, 2, 3, 2, 2, 2, 3, 2, 2, 2, 3, 2]


def get_ref(planes_flat, origin, stride, qx, qy, w, h):
    """unweighted get_ref (mc.c:221-249) at absolute quarter-pel position (qx, qy)."""
    idx = ((qy & 3) << 2) + (qx & 3)
    off = origin + (qy >> 2) * stride + (qx >> 2)
    a = block(planes_flat[HPEL_REF0[idx]], off + ((qy & 3) == 3) * stride, stride, w, h)
    if idx & 5:
        b = block(planes_flat[HPEL_REF1[idx]], off + ((qx & 3) == 3), stride, w, h)
        return (a + b + 1) >> 1
    return a


# ---------------------------------------------------------------- further pixel entries
def _hadamard(n):
    h = np.array([[1]], np.int64)
    while h.shape[0] < n:
        h = np.block([[h, h], [h, -h]])
    return h


H8 = _hadamard(8)


def sa8d(a, b):
    """sa8d 8x8 / 16x16: (sum over 8x8 tiles of sum |H8 . D . H8^T| + 2) >> 2 (pixel.c:334-381)."""
    d = a - b
    h, w = d.shape
    t = d.reshape(h // 8, 8, w // 8, 8).transpose(0, 2, 1, 3)
    coef = np.einsum("ij,abjk,lk->abil", H8, t, H8)
    return int((np.abs(coef).sum() + 2) >> 2)


def hadamard_ac(p):
    """(sum8 >> 2) << 32 | (sum4 >> 1) over 8x8 tiles, where sum4 = sum |H4 coefs| of the four 4x4
    sub-blocks minus their DCs and sum8 = sum |H8 coefs| minus the DC (pixel.c:383-435)."""
    h, w = p.shape
    s4 = s8 = 0
    for y in range(0, h, 8):
        for x in range(0, w, 8):
            t = p[y:y + 8, x:x + 8]
            c8 = H8 @ t @ H8.T
            s8 += int(np.abs(c8).sum() - abs(c8[0, 0]))
            for yy in (0, 4):
                for xx in (0, 4):
                    c4 = H4 @ t[yy:yy + 4, xx:xx + 4] @ H4.T
                    s4 += int(np.abs(c4).sum() - abs(c4[0, 0]))
    return ((s8 >> 2) << 32) + (s4 >> 1)


def var(p):
    return int(p.sum()) + (int((p * p).sum()) << 32)


def var2(u, du, v, dv, h):
    """var2 over 8-wide U/V blocks (fenc - fdec differences); returns (res, ssd_u, ssd_v)."""
    shift = 7 if h == 16 else 6
    a, b = u - du, v - dv
    su, sv, qu, qv = int(a.sum()), int(b.sum()), int((a * a).sum()), int((b * b).sum())
    return qu - ((su * su) >> shift) + qv - ((sv * sv) >> shift), qu, qv


def box_sums(plane2d, k):
    """k x k box sums at every top-left position (valid region), int64."""
    c = np.pad(plane2d.astype(np.int64), ((1, 0), (1, 0))).cumsum(0).cumsum(1)
    return c[k:, k:] - c[:-k, k:] - c[k:, :-k] + c[:-k, :-k]


# ---------------------------------------------------------------- inverse path
def _idct4_1d(c0, c1, c2, c3):
    """H.264 inverse core transform butterfly on arrays (dct.c:272-297 row/column pass)."""
    s02, d02 = c0 + c2, c0 - c2
    s13, d13 = c1 + (c3 >> 1), (c1 >> 1) - c3
    return s02 + s13, d02 + d13, d02 - d13, s02 - s13


def add4x4_idct(pred, dct, bd):
    """pred (4x4 int) + idct of dct[16] (reference transposed layout); int16 temps at 8 bit."""
    d = np.asarray(dct, np.int64).reshape(4, 4)        # d[r][c] = dct[r*4+c]
    # first pass over i: uses dct[k*4+i] (column i of d^T ...) -> tmp[i][*]
    t = np.stack(_idct4_1d(d[0], d[1], d[2], d[3]), axis=1)   # t[i][k]
    t = wrap(t, bd)
    o = np.stack(_idct4_1d(t[0], t[1], t[2], t[3]), axis=0)   # o[k][i] = d_out[k*4+i]
    o = wrap((o + 32) >> 6, bd)
    return np.clip(pred + o, 0, (1 << bd) - 1)


def _idct8_1d(s):
    a0, a2 = s[0] + s[4], s[0] - s[4]
    a4, a6 = (s[2] >> 1) - s[6], (s[6] >> 1) + s[2]
    b0, b2, b4, b6 = a0 + a6, a2 + a4, a2 - a4, a0 - a6
    a1 = -s[3] + s[5] - s[7] - (s[7] >> 1)
    a3 = s[1] + s[7] - s[3] - (s[3] >> 1)
    a5 = -s[1] + s[7] + s[5] + (s[5] >> 1)
    a7 = s[3] + s[5] + s[1] + (s[1] >> 1)
    b1, b3, b5, b7 = (a7 >> 2) + a1, a3 + (a5 >> 2), (a3 >> 2) - a5, a7 - (a1 >> 2)
    return [b0 + b7, b2 + b5, b4 + b3, b6 + b1, b6 - b1, b4 - b3, b2 - b5, b0 - b7]


def add8x8_idct8(pred, dct, bd):
    d = np.asarray(dct, np.int64).reshape(8, 8).copy()     # d[x][i] = dct[x*8+i]
    d[0, 0] = wrap(d[0, 0] + 32, bd)
    d = wrap(np.stack(_idct8_1d([d[x] for x in range(8)]), 0), bd)     # column pass, stored
    o = np.stack(_idct8_1d([d[:, x] for x in range(8)]), 1)             # o[i][x] -> dst[i + x*stride]
    return np.clip(pred + (o.T >> 6), 0, (1 << bd) - 1)


def dequant(dct, dmf6, qp, shift_base):
    """dequant_4x4 (shift_base 4) / dequant_8x8 (6): dmf6 [6][n]."""
    c = np.asarray(dct, np.int64)
    mf = np.asarray(dmf6, np.int64)[qp % 6]
    q = qp // 6 - shift_base
    if q >= 0:
        return c * mf << q
    return (c * mf + (1 << (-q - 1))) >> (-q)


def decimate_score(c):
    c = list(int(v) for v in c)
    table = [3, 2, 2, 1, 1, 1] + [0] * 10 if len(c) < 64 else [3] * 4 + [2] * 8 + [1] * 12 + [0] * 40
    nzi = [i for i, v in enumerate(c) if v]
    if any(abs(c[i]) > 1 for i in nzi):
        return 9
    score = 0
    for k, i in enumerate(reversed(nzi)):
        nxt = nzi[len(nzi) - 2 - k] if k + 1 < len(nzi) else -1
        score += table[i - nxt - 1]
    return score


def zigzag_frame(n):
    """standard frame zigzag order as (row, col) of an n x n block (dct.c ZIGZAG*_FRAME)."""
    order = []
    for s in range(2 * n - 1):
        cells = [(r, s - r) for r in range(n) if 0 <= s - r < n]
        order += cells if s % 2 else cells[::-1]
    return order
