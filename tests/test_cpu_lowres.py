"""CPU: the oracle's x264_frame_init_lowres (mc.c:458-507 + frame.c:627-631)
against a vectorised numpy restatement.  No GPU involved."""
import numpy as np
import pytest


def _np_lowres(core, bd):
    """core: [H, W] frame; returns the 4 bordered lowres planes [(H/2+64), (W/2+64)]."""
    H, W = core.shape
    s = np.pad(core.astype(np.int64), ((0, 1), (0, 1)), mode="edge")      # duplicated last row / column
    a = lambda x, y: (x + y + 1) >> 1                                       # noqa: E731
    f = lambda p, q, r, t: (a(p, q) + a(r, t) + 1) >> 1                     # noqa: E731
    r0, r1, r2 = s[0:H:2], s[1:H + 1:2], s[2:H + 1:2]
    c0, c1, c2 = slice(0, W, 2), slice(1, W + 1, 2), slice(2, W + 1, 2)
    hl = H // 2
    r2 = np.concatenate([r2, s[H:H + 1]])[:hl] if r2.shape[0] < hl else r2
    planes = [f(r0[:, c0], r1[:, c0], r0[:, c1], r1[:, c1]), f(r0[:, c1], r1[:, c1], r0[:, c2], r1[:, c2]),
              f(r1[:, c0], r2[:, c0], r1[:, c1], r2[:, c1]), f(r1[:, c1], r2[:, c1], r1[:, c2], r2[:, c2])]
    return [np.pad(p, 32, mode="edge") for p in planes]


@pytest.mark.parametrize("bd", [8, 10])
@pytest.mark.parametrize("size", [(64, 48), (176, 144), (66, 34)])
def test_frame_init_lowres(oracle, bd, size):
    W, H = size
    rs = np.random.default_rng(bd + W)
    stride = (W + 64 + 63) // 64 * 64
    core = rs.integers(0, 1 << bd, size=(H, W))
    # padding deliberately NOT replicated: the reference overwrites column W / row H itself
    full = rs.integers(0, 1 << bd, size=(H + 64, stride))
    full[32:32 + H, 32:32 + W] = core
    full = full.astype(oracle.pixel_dtype(bd)).ravel()
    ls = (W // 2 + 64 + 63) // 64 * 64
    got = oracle.frame_init_lowres(bd, full, 32 * stride + 32, stride, W, H, ls)
    want = _np_lowres(core, bd)
    for g, w in zip(got, want):
        assert np.array_equal(g[:, :W // 2 + 64], w)
