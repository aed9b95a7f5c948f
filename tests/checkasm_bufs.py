"""The input buffers of the reference's tools/checkasm.c, reproduced exactly.

checkasm seeds glibc's srand(seed) and fills buf1 / pbuf1 with rand() in main
(tools/checkasm.c:3036-3060); check_pixel overwrites pbuf3 / pbuf4 with the
"maximize sum" overflow patterns (checkasm.c:368-382) and check_dct builds five
crafted 16x16 overflow blocks in pbuf3 / pbuf4 (checkasm.c:909-928).  The same
glibc rand() is called here through ctypes, so for a given seed these are
byte-for-byte the buffers checkasm8 / checkasm10 would test with.
"""
import ctypes

import numpy as np

_libc = ctypes.CDLL("libc.so.6")
_libc.rand.restype = ctypes.c_int
_libc.srand.argtypes = [ctypes.c_uint]

SEED = 12345     # the seed of the survey's checkasm run


def srand(seed):
    _libc.srand(seed)


def rand():
    return _libc.rand()


def rand30():
    """checkasm.c:72"""
    return ((rand() & 0x7FFF) << 15) + (rand() & 0x7FFF)


class Bufs:
    """buf1..4 / pbuf1..4 of checkasm for one bit depth.  pbufN are numpy views
    (pixel dtype) with the same element offsets the C code uses."""

    def __init__(self, bd, seed=SEED):
        self.bd = bd
        self.pixel_max = (1 << bd) - 1
        sp = 1 if bd == 8 else 2
        pdt = np.uint8 if bd == 8 else np.uint16
        srand(seed)
        self.buf1 = np.zeros(0x1E00 + 0x2000 * sp, np.uint8)
        self.pbuf1 = np.zeros(0x1E00, pdt)
        for i in range(0x1E00):
            self.buf1[i] = rand() & 0xFF
            self.pbuf1[i] = rand() & self.pixel_max
        # buf3 = buf1 + 0x1e00, buf4 = buf3 + 0x1000*SIZEOF_PIXEL (checkasm.c:3047-3054)
        self.pbuf2_off = 0xF00
        self.buf3 = np.zeros(0x1000 * sp, np.uint8)
        self.buf4 = np.zeros(0x1000 * sp, np.uint8)
        self.pbuf3 = self.buf3.view(pdt)
        self.pbuf4 = self.buf4.view(pdt)

    # --------------------------------------------------------- pixel tests
    def fill_pixel_overflow(self):
        """checkasm.c:368-382"""
        pm = self.pixel_max
        for i in range(256):
            z = i | (i >> 4)
            z ^= z >> 2
            z ^= z >> 1
            self.pbuf4[i] = (-(z & 1)) & pm
            self.pbuf3[i] = (~int(self.pbuf4[i])) & pm
        for i in range(256, 0x1000):
            self.pbuf4[i] = (-(int(self.pbuf1[i & ~0x88]) & 1)) & pm
            self.pbuf3[i] = (~int(self.pbuf4[i])) & pm

    # ----------------------------------------------------------- dct tests
    def fill_dct_overflow(self):
        """checkasm.c:909-928: five 16x16 blocks of PIXEL_MAX/0 stripes, fenc
        stride 16 in pbuf3, fdec stride 32 in pbuf4."""
        pm = self.pixel_max
        for i in range(5):
            e0 = 16 * i * 16
            d0 = 16 * i * 32
            for j in range(16):
                cond_a = 1 if i < 2 else int((j & 3) == 0 or (j & 3) == (i - 1))
                cond_b = 1 if i == 0 else int(not cond_a)
                a = pm if cond_a else 0
                b = pm if cond_b else 0
                row = e0 + j * 16
                for k in (0, 1, 4, 5, 8, 9, 12, 13):
                    self.pbuf3[row + k] = a
                for k in (2, 3, 6, 7, 10, 11, 14, 15):
                    self.pbuf3[row + k] = b
                drow = d0 + j * 32
                for k in range(4):
                    self.pbuf4[drow + k] = pm - int(self.pbuf3[row + k])


def init_quant8(j, bd):
    """INIT_QUANT8 (checkasm.c:2149-2157): 64 coefficients, block on/off by j."""
    pm = (1 << bd) - 1
    scale1d = [32, 31, 24, 31, 32, 31, 24, 31]
    out = np.zeros(64, np.int64)
    for i in range(64):
        scale = (pm * scale1d[(i >> 3) & 7] * scale1d[i & 7]) // 16
        out[i] = (rand30() % (2 * scale + 1)) - scale if (j >> (i >> 6)) & 1 else 0
    return out


def init_quant4(j, n, bd):
    """INIT_QUANT4 (checkasm.c:2159-2167): n coefficients (16 or 64)."""
    pm = (1 << bd) - 1
    scale1d = [4, 6, 4, 6]
    out = np.zeros(n, np.int64)
    for i in range(n):
        scale = pm * scale1d[(i >> 2) & 3] * scale1d[i & 3]
        out[i] = (rand30() % (2 * scale + 1)) - scale if (j >> (i >> 4)) & 1 else 0
    return out


# CQM configurations of check_quant (checkasm.c:2098-2140)
CQM_TEST4 = [6, 4, 6, 4, 4, 3, 4, 3, 6, 4, 6, 4, 4, 3, 4, 3]
CQM_TEST8 = [3, 3, 4, 3, 3, 3, 4, 3, 3, 3, 4, 3, 3, 3, 4, 3, 4, 4, 5, 4, 4, 4, 5, 4, 3, 3, 4, 3, 3, 3, 4, 3,
             3, 3, 4, 3, 3, 3, 4, 3, 3, 3, 4, 3, 3, 3, 4, 3, 4, 4, 5, 4, 4, 4, 5, 4, 3, 3, 4, 3, 3, 3, 4, 3]
FLAT16 = [16] * 64
# H.264 default matrices (spec Tables 7-3/7-4; reference common/tables.c:191-237)
JVT4I = [6, 13, 20, 28, 13, 20, 28, 32, 20, 28, 32, 37, 28, 32, 37, 42]
JVT4P = [10, 14, 20, 24, 14, 20, 24, 27, 20, 24, 27, 30, 24, 27, 30, 34]
JVT8I = [6, 10, 13, 16, 18, 23, 25, 27, 10, 11, 16, 18, 23, 25, 27, 29, 13, 16, 18, 23, 25, 27, 29, 31,
         16, 18, 23, 25, 27, 29, 31, 33, 18, 23, 25, 27, 29, 31, 33, 36, 23, 25, 27, 29, 31, 33, 36, 38,
         25, 27, 29, 31, 33, 36, 38, 40, 27, 29, 31, 33, 36, 38, 40, 42]
JVT8P = [9, 13, 15, 17, 19, 21, 22, 24, 13, 13, 17, 19, 21, 22, 24, 25, 15, 17, 19, 21, 22, 24, 25, 27,
         17, 19, 21, 22, 24, 25, 27, 28, 19, 21, 22, 24, 25, 27, 28, 30, 21, 22, 24, 25, 27, 28, 30, 32,
         22, 24, 25, 27, 28, 30, 32, 33, 24, 25, 27, 28, 30, 32, 33, 35]


def cqm_lists(i_cqm, bd):
    """scaling_list[8] of configuration i_cqm (0..5); configuration 4 draws rand()."""
    if i_cqm == 0:
        return [FLAT16] * 8
    if i_cqm == 1:
        return [JVT4I, JVT4P, JVT4I, JVT4P, JVT8I, JVT8P, JVT8I, JVT8P]
    if i_cqm == 2:
        return [CQM_TEST4] * 4 + [FLAT16] * 4
    if i_cqm == 3:
        return [FLAT16] * 4 + [CQM_TEST8] * 4
    if i_cqm == 4:
        max_scale = 255 if bd < 10 else 228
        buf = [10 + rand() % (max_scale - 9) for _ in range(64)]
        return [buf] * 8
    return [[1] * 64] * 8
