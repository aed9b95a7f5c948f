"""Synthetic luma sequences for parity tests and bench.py.

Frame 0 is seeded uniform noise (numpy PCG64) box-smoothed 5x5; frame k is
frame 0 displaced by (3k', 2k') pixels, k' = k mod 32, plus +-2 noise (seed k)
(the motion wraps every 32 frames so every frame is a window of one fixed-size
texture).  Each frame is
stored like an x264 plane: PAD (=32, reference common/frame.h:32-33) pixels of
edge replication on every side (x264_frame_expand_border semantics), rows of
``stride`` pixels.
"""
import numpy as np

PAD = 32
PERIOD = 32


def plane_stride(width, pad=PAD):
    return (width + 2 * pad + 63) // 64 * 64


def _texture(h, w, bitdepth, seed=1):
    rng = np.random.Generator(np.random.PCG64(seed))
    pmax = (1 << bitdepth) - 1
    base = rng.integers(0, pmax + 1, size=(h + 4, w + 4), dtype=np.int64)
    # 5x5 box filter via integral image
    c = np.cumsum(np.cumsum(np.pad(base, ((1, 0), (1, 0))), 0), 1)
    box = c[5:, 5:] - c[:-5, 5:] - c[5:, :-5] + c[:-5, :-5]
    return (box + 12) // 25


def make_sequence(nframes, width, height, bitdepth=8, pad=PAD, seed=1, start=0):
    """Frames start .. start+nframes-1 of the sequence.

    Returns (planes[nframes, height + 2*pad, stride] numpy, stride, origin);
    origin = element offset of pixel (0, 0) inside one frame.  Any slice of the
    sequence is identical to the same frames of a longer generation, so ranks
    can each build their own shard (x264hip.dist.frame_shard)."""
    pmax = (1 << bitdepth) - 1
    tex = _texture(height + 2 * PERIOD, width + 3 * PERIOD, bitdepth, seed)
    stride = plane_stride(width, pad)
    dt = np.uint8 if bitdepth == 8 else np.uint16
    out = np.zeros((nframes, height + 2 * pad, stride), dt)
    for i in range(nframes):
        k = start + i
        rng = np.random.Generator(np.random.PCG64(1000 + k))
        kk = k % PERIOD
        win = tex[2 * kk:2 * kk + height, 3 * kk:3 * kk + width]
        if k:
            win = win + rng.integers(-2, 3, size=win.shape)
        win = np.clip(win, 0, pmax)
        full = np.pad(win, ((pad, pad), (pad, stride - width - pad)), mode="edge")
        out[i] = full.astype(dt)
    return out, stride, pad * stride + pad


def random_planes(nframes, width, height, bitdepth=8, pad=PAD, seed=7):
    """Uniform random pixels everywhere (padding included): worst case for SAD ranges."""
    rng = np.random.Generator(np.random.PCG64(seed))
    stride = plane_stride(width, pad)
    dt = np.uint8 if bitdepth == 8 else np.uint16
    out = rng.integers(0, 1 << bitdepth, size=(nframes, height + 2 * pad, stride)).astype(dt)
    return out, stride, pad * stride + pad


def _smooth_field(rng, K, fmax):
    """K random cosine components (fx, fy in cycles/pixel, phase, amplitude ~ 1/f)"""
    f = rng.uniform(0.01, fmax, size=(K, 2)) * rng.choice([-1, 1], size=(K, 2))
    ph = rng.uniform(0, 2 * np.pi, size=K)
    amp = 1.0 / np.hypot(f[:, 0], f[:, 1])
    return f, ph, amp / amp.sum()


def _eval_field(field, xs, ys):
    """sum_i amp_i cos(2 pi (fx_i x + fy_i y) + ph_i) on the grid ys x xs: separable, so one
    rank-2K product [cos by_i, -sin by_i] . [cos ax_i, sin ax_i]^T (a 2160p field in ~0.1 s)"""
    f, ph, amp = field
    by = 2 * np.pi * np.outer(ys, f[:, 1]) + ph            # [len(ys), K]
    ax = 2 * np.pi * np.outer(xs, f[:, 0])                 # [len(xs), K]
    left = np.concatenate([np.cos(by) * amp, -np.sin(by) * amp], 1)
    right = np.concatenate([np.cos(ax), np.sin(ax)], 1)
    return left @ right.T


def make_subpel_sequence(nframes, width, height, bitdepth=8, pad=PAD, seed=3, start=0, motion=(13, 10)):
    """A 4:2:0 sequence with quarter-pel motion, for the subpel refine legs: frame k samples a
    smooth random field (24 cosine components up to 0.22 cycles/pixel) displaced by k * motion
    quarter pixels (default (3.25, 2.5) pixels per frame), plus +-1 noise (seed k); its chroma
    samples two fields of their own at half resolution with the same motion (k * motion eighth
    pixels of chroma) and is stored interleaved (NV12, x264's fenc->plane[1] layout) with 16
    rows and 16 chroma pixels (32 elements) of edge replication (x264's 4:2:0 chroma padding).
    Returns (luma[nframes, h+2pad, stride], stride, origin, nv12[nframes, h/2+32, cstride],
    cstride, corigin)."""
    pmax = (1 << bitdepth) - 1
    rng = np.random.Generator(np.random.PCG64(seed))
    fields = [_smooth_field(rng, 24, 0.22) for _ in range(3)]
    stride = plane_stride(width, pad)
    cw, ch, cpad = width // 2, height // 2, 16
    cstride = (2 * cw + 4 * cpad + 63) // 64 * 64
    dt = np.uint8 if bitdepth == 8 else np.uint16
    luma = np.zeros((nframes, height + 2 * pad, stride), dt)
    nv = np.zeros((nframes, ch + 2 * cpad, cstride), dt)
    for i in range(nframes):
        k = start + i
        nrng = np.random.Generator(np.random.PCG64(2000 + k))
        dx, dy = k * motion[0] / 4.0, k * motion[1] / 4.0
        y = _eval_field(fields[0], np.arange(width) + dx, np.arange(height) + dy)
        y = np.clip(np.floor((0.5 + 1.6 * y) * pmax + 0.5) + nrng.integers(-1, 2, size=y.shape), 0, pmax)
        luma[i] = np.pad(y, ((pad, pad), (pad, stride - width - pad)), mode="edge").astype(dt)
        planes = []
        for p in (1, 2):
            c = _eval_field(fields[p], np.arange(cw) + dx / 2, np.arange(ch) + dy / 2)
            c = np.clip(np.floor((0.5 + 1.2 * c) * pmax + 0.5) + nrng.integers(-1, 2, size=c.shape), 0, pmax)
            planes.append(np.pad(c, ((cpad, cpad), (cpad, cpad)), mode="edge"))
        nv[i, :, 0:2 * (cw + 2 * cpad):2] = planes[0]
        nv[i, :, 1:2 * (cw + 2 * cpad):2] = planes[1]
    return luma, stride, pad * stride + pad, nv, cstride, cpad * cstride + 2 * cpad
