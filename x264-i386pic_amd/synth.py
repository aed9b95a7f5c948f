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
