"""ctypes front-end of the CPU oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE.

Every function takes numpy arrays and returns numpy arrays / ints; pointers
into arrays are passed as (array, element offset).  Only tests/, the smoke
check and bench.py's cpu_baseline leg use this module.
"""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# X264HIP_ORACLE_LIB selects another build of the same sources (the sanitizer build,
# tests/test_cpu_sanitize.py)
_L = C.CDLL(os.environ.get("X264HIP_ORACLE_LIB") or os.path.join(ROOT, "oracle", "liboracle.so"))
_P, _IP = C.c_void_p, C.c_ssize_t


def pixel_dtype(bd):
    return np.uint8 if bd == 8 else np.uint16


def coef_dtype(bd):
    return np.int16 if bd == 8 else np.int32


def ucoef_dtype(bd):
    return np.uint16 if bd == 8 else np.uint32


def sad_dtype(bd):
    return np.uint16 if bd == 8 else np.uint32


def _addr(a, off=0):
    return C.c_void_p(a.ctypes.data + int(off) * a.itemsize)


def _f(bd, name, argtypes, restype=None):
    fn = getattr(_L, f"oracle{bd}_{name}")
    fn.argtypes = argtypes
    fn.restype = restype
    return fn


for _bd in (8, 10):
    for _n in ("sad", "ssd", "satd"):
        _f(_bd, _n, [C.c_int, _P, _IP, _P, _IP], C.c_int)
    for _n in ("sad_x3", "satd_x3"):
        _f(_bd, _n, [C.c_int, _P, _P, _P, _P, _IP, _P])
    for _n in ("sad_x4", "satd_x4"):
        _f(_bd, _n, [C.c_int, _P, _P, _P, _P, _P, _IP, _P])
    _f(_bd, "cmp_list", [C.c_int, C.c_int, _P, _IP, _P, _IP, _P, _P, C.c_int, _P])
    for _n in ("sub4x4_dct", "sub8x8_dct", "sub16x16_dct", "sub8x8_dct_dc", "sub8x16_dct_dc",
               "sub8x8_dct8", "sub16x16_dct8"):
        _f(_bd, _n, [_P, _P, _P])
    _f(_bd, "sub_dct_list", [C.c_int, _P, _IP, _P, _IP, _P, _P, C.c_int, _P])
    _f(_bd, "dct4x4dc", [_P])
    _f(_bd, "dct2x4dc", [_P, _P])
    for _n in ("quant_8x8", "quant_4x4", "quant_4x4x4"):
        _f(_bd, _n, [_P, _P, _P], C.c_int)
    for _n in ("quant_4x4_dc", "quant_2x2_dc"):
        _f(_bd, _n, [_P, C.c_int, C.c_int], C.c_int)
    _f(_bd, "cqm_init", [_P, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P], C.c_int)
    _f(_bd, "me_search_full", [_P, _IP, _P, _IP, C.c_int, C.c_int, C.c_int, _P])
    _f(_bd, "me_search_full8", [_P, _IP, _P, _IP, C.c_int, C.c_int, C.c_int, _P])
    _f(_bd, "mb_dct_quant", [C.c_int, _P, _IP, _P, _IP, C.c_int, C.c_int, _P, _P, _P, _P])
    _f(_bd, "hpel_filter", [_P, _P, _P, _P, _IP, C.c_int, C.c_int, _P])
    _f(_bd, "get_ref", [_P, _P, _P, _IP, C.c_int, C.c_int, C.c_int, C.c_int], _P)
    _f(_bd, "me_esa_argmin", [_P, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P, _P])
    _f(_bd, "me_search_esa8", [_P, _IP, _P, _IP, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P])
    _f(_bd, "ssd_wxh", [_P, _IP, _P, _IP, C.c_int, C.c_int], C.c_uint64)
    _f(_bd, "ssd_nv12", [_P, _IP, _P, _IP, C.c_int, C.c_int, _P, _P])
    _f(_bd, "me_tesa", [_P, _IP, _P, _P, _IP, C.c_int, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P])
    _f(_bd, "me_search_centred", [_P, _IP, _P, _IP, C.c_int, C.c_int, C.c_int, _P, _P, _P])
    _f(_bd, "me_refine_subpel", [_P, _IP, _P, _IP, C.c_int, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P, C.c_int, _P,
                                 _P])
    _f(_bd, "me_search_ref", [_P, _IP, _P, _P, _IP, C.c_int, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P, C.c_int, _P,
                              _P, _P, _P, _IP, _P, _IP])
    _f(_bd, "me_refine_subpel_ex", [_P, _IP, _P, _IP, C.c_int, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P, C.c_int,
                                    _P, _P, _P, _P, _IP, _P, _IP])
    _f(_bd, "me_search_ref_thresh", [_P, _IP, _P, _P, _IP, C.c_int, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P,
                                     C.c_int, _P, _P, _P, _P, _IP, _P, _IP, _P, _P])
    _f(_bd, "me_refine_bidir", [_P, _IP, _P, _P, _IP, C.c_int, C.c_int, _P, _P, _P, _P, C.c_int, _P, _P, _P])
    _f(_bd, "me_refine_qpel_refdupe", [_P, _IP, _P, _IP, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P, C.c_int, _P, _P,
                                       _P, _P, _IP, _P, _IP, _P, _P])
    _f(_bd, "frame_filter", [_P, _P, _P, _P, _IP, C.c_int, C.c_int])
    _f(_bd, "subpel_list", [C.c_int, C.c_int, _P, _IP, _P, _P, _P, _P, _IP, _P, _P, C.c_int, _P])
    _f(_bd, "sa8d", [C.c_int, _P, _IP, _P, _IP], C.c_int)
    _f(_bd, "sa8d_satd", [_P, _IP, _P, _IP], C.c_uint64)
    _f(_bd, "hadamard_ac", [C.c_int, _P, _IP], C.c_uint64)
    _f(_bd, "var", [C.c_int, _P, _IP], C.c_uint64)
    _f(_bd, "var2", [C.c_int, _P, _P, _P], C.c_int)
    _f(_bd, "var2_s", [C.c_int, _P, _IP, _IP, _P, _IP, _IP, _P], C.c_int)
    _f(_bd, "vsad", [_P, _IP, C.c_int], C.c_int)
    _f(_bd, "asd8", [_P, _IP, _P, _IP, C.c_int], C.c_int)
    _f(_bd, "ads", [C.c_int, _P, _P, C.c_int, _P, _P, C.c_int, C.c_int], C.c_int)
    _f(_bd, "frame_integral", [_P, _IP, C.c_int, C.c_int, C.c_int, _P])
    _f(_bd, "idct4x4dc", [_P])
    for _n in ("add4x4_idct", "add8x8_idct", "add16x16_idct", "add8x8_idct_dc", "add16x16_idct_dc",
               "add8x8_idct8", "add16x16_idct8"):
        _f(_bd, _n, [_P, _P])
    _f(_bd, "add_idct_list", [C.c_int, _P, _IP, _P, _P, C.c_int])
    for _n in ("dequant_4x4", "dequant_8x8", "dequant_4x4_dc"):
        _f(_bd, _n, [_P, _P, C.c_int])
    _f(_bd, "idct_dequant_2x4_dc", [_P, _P, _P, C.c_int])
    _f(_bd, "idct_dequant_2x4_dconly", [_P, _P, C.c_int])
    _f(_bd, "optimize_chroma_2x2_dc", [_P, C.c_int], C.c_int)
    _f(_bd, "optimize_chroma_2x4_dc", [_P, C.c_int], C.c_int)
    _f(_bd, "denoise_dct", [_P, _P, _P, C.c_int])
    for _n in ("decimate_score15", "decimate_score16", "decimate_score64"):
        _f(_bd, _n, [_P], C.c_int)
    _f(_bd, "coeff_last", [_P, C.c_int], C.c_int)
    _f(_bd, "coeff_level_run", [_P, C.c_int, _P, _P, _P], C.c_int)
    _f(_bd, "zigzag_scan_8x8", [C.c_int, _P, _P])
    _f(_bd, "zigzag_scan_4x4", [C.c_int, _P, _P])
    _f(_bd, "zigzag_sub_s", [C.c_int, C.c_int, _P, _P, _IP, _P, _IP, _P], C.c_int)
    _f(_bd, "zigzag_interleave_8x8_cavlc", [_P, _P, _P])
    _f(_bd, "cqm_dequant", [_P, C.c_int, _P, _P])
    _f(_bd, "frame_init_lowres", [_P, _IP, C.c_int, C.c_int, _P, _IP])
    _f(_bd, "mb_dequant_idct_add", [C.c_int, _P, C.c_int, C.c_int, _P, _P, _P, _IP, _P, _IP])
    _f(_bd, "predict_8x8_filter", [_P, _P, C.c_int, C.c_int])
    _f(_bd, "predict_8x8", [C.c_int, _P, _P])
    _f(_bd, "predict", [C.c_int, C.c_int, _P])
    _f(_bd, "intra_x3", [C.c_int, C.c_int, _P, _P, _P])
    _f(_bd, "lowres_intra_cost", [_P, _IP, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P])
    _f(_bd, "lowres_inter_cost", [_P, _P, _P, _P, _P, _IP, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                  C.c_int, C.c_int, _P, _P, _P, _P, _P, _P, _P, _P])
    _f(_bd, "lowres_inter_cost_ex", [_P, _P, _P, _P, _P, _P, _P, C.c_int, _IP, C.c_int, C.c_int, C.c_int, C.c_int,
                                     C.c_int, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P, _P, _P, _P, _P])
    _f(_bd, "weight_scale_plane", [_P, _IP, _P, _IP, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int])
    _f(_bd, "mc_weight", [_P, _IP, _P, _IP, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int])
    _f(_bd, "lowres_bidir_cost", [_P, _P, _P, _IP, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                  C.c_int, _P, _P, _P, _P, _P, _P, _P, C.c_int, C.c_int, _P, _P, _P, _P])
    _f(_bd, "lowres_bidir_cost_ex", [_P, _P, _P, _IP, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                     C.c_int, _P, _P, _P, _P, _P, _P, _P, C.c_int, C.c_int, _P, _P, _P, _P,
                                     C.c_int])
_L.oracle8_me_search_full_mt.argtypes = [_P, _IP, _P, _IP, C.c_int, C.c_int, C.c_int, _P, C.c_int]
_L.oracle8_me_search_full_mt.restype = C.c_int
_L.oracle8_mb_dct_quant_mt.argtypes = [C.c_int, _P, _IP, _P, _IP, C.c_int, C.c_int, _P, _P, _P, _P, C.c_int]
_L.oracle8_mb_dct_quant_mt.restype = C.c_int
_L.oracle8_subpel_list_mt.argtypes = [C.c_int, C.c_int, _P, _IP, _P, _P, _P, _P, _IP, _P, _P, C.c_int, _P, C.c_int]
_L.oracle8_subpel_list_mt.restype = C.c_int
_L.oracle8_ssim_bands_mt.argtypes = [_P, _IP, _P, _IP, C.c_int, _P, C.c_int, _P, _P, C.c_int]
_L.oracle8_ssim_bands_mt.restype = C.c_int

_OPS = {"sad": 0, "ssd": 1, "satd": 2}


def cmp(bd, op, i_pixel, a, a_off, sa, b, b_off, sb):
    """reference sad/ssd/satd of size i_pixel at a[a_off] (stride sa) vs b[b_off] (stride sb)."""
    return getattr(_L, f"oracle{bd}_{op}")(i_pixel, _addr(a, a_off), sa, _addr(b, b_off), sb)


def cmp_x(bd, op, n, i_pixel, fenc, f_off, ref, offs, stride):
    """sad_x3/x4, satd_x3/x4 (fenc stride 16)."""
    out = np.zeros(4, np.int32)
    args = [_addr(ref, o) for o in offs]
    getattr(_L, f"oracle{bd}_{op}_x{n}")(i_pixel, _addr(fenc, f_off), *args, stride, _addr(out))
    return out[:n].copy()


def cmp_list(bd, op, i_pixel, fenc, fs, ref, rs, fenc_off, ref_off):
    fo = np.ascontiguousarray(fenc_off, np.int64)
    ro = np.ascontiguousarray(ref_off, np.int64)
    out = np.zeros(len(fo), np.int32)
    getattr(_L, f"oracle{bd}_cmp_list")(_OPS.get(op, op), i_pixel, _addr(fenc), fs, _addr(ref), rs,
                                       _addr(fo), _addr(ro), len(fo), _addr(out))
    return out


DCT_OUT = {"sub4x4_dct": 16, "sub8x8_dct": 64, "sub16x16_dct": 256, "sub8x8_dct_dc": 4,
           "sub8x16_dct_dc": 8, "sub8x8_dct8": 64, "sub16x16_dct8": 256}
DCT_KINDS = ["sub4x4_dct", "sub8x8_dct", "sub16x16_dct", "sub8x8_dct_dc", "sub8x16_dct_dc",
             "sub8x8_dct8", "sub16x16_dct8"]


def sub_dct(bd, name, a, a_off, b, b_off):
    """reference entry with implicit strides FENC_STRIDE=16 / FDEC_STRIDE=32."""
    out = np.zeros(DCT_OUT[name], coef_dtype(bd))
    getattr(_L, f"oracle{bd}_{name}")(_addr(out), _addr(a, a_off), _addr(b, b_off))
    return out


def sub_dct_list(bd, kind, fenc, fs, fdec, ds, fenc_off, fdec_off):
    fo = np.ascontiguousarray(fenc_off, np.int64)
    do = np.ascontiguousarray(fdec_off, np.int64)
    out = np.zeros(len(fo) * DCT_OUT[DCT_KINDS[kind]], coef_dtype(bd))
    getattr(_L, f"oracle{bd}_sub_dct_list")(kind, _addr(fenc), fs, _addr(fdec), ds, _addr(fo), _addr(do),
                                           len(fo), _addr(out))
    return out


def dct4x4dc(bd, d):
    d = np.array(d, coef_dtype(bd))
    getattr(_L, f"oracle{bd}_dct4x4dc")(_addr(d))
    return d


def dct2x4dc(bd, dct4x4):
    src = np.array(dct4x4, coef_dtype(bd)).reshape(8, 16).copy()
    out = np.zeros(8, coef_dtype(bd))
    getattr(_L, f"oracle{bd}_dct2x4dc")(_addr(out), _addr(src))
    return out, src


def quant(bd, name, dct, mf=None, bias=None):
    """returns (quantised copy, nz)."""
    d = np.array(dct, coef_dtype(bd))
    fn = getattr(_L, f"oracle{bd}_{name}")
    if name in ("quant_4x4_dc", "quant_2x2_dc"):
        nz = fn(_addr(d), int(mf), int(bias))
    else:
        m = np.ascontiguousarray(mf, ucoef_dtype(bd))
        b = np.ascontiguousarray(bias, ucoef_dtype(bd))
        nz = fn(_addr(d), _addr(m), _addr(b))
    return d, nz


def cqm_init(bd, scaling_lists, dz_inter=21, dz_intra=11, transform_8x8=True):
    qp1 = 52 + 6 * (bd - 8)
    ut = ucoef_dtype(bd)
    q4m, q4b = np.zeros((4, qp1, 16), ut), np.zeros((4, qp1, 16), ut)
    q8m, q8b = np.zeros((4, qp1, 64), ut), np.zeros((4, qp1, 64), ut)
    lists = [np.ascontiguousarray(np.asarray(s, np.uint8)) for s in scaling_lists]
    ptrs = (_P * 8)(*[x.ctypes.data for x in lists])
    getattr(_L, f"oracle{bd}_cqm_init")(ptrs, dz_inter, dz_intra, int(transform_8x8), _addr(q4m), _addr(q4b),
                                       _addr(q8m), _addr(q8b))
    return q4m, q4b, q8m, q8b


def me_search_full(bd, fenc, f_origin, fs, ref, r_origin, rs, mbw, mbh, rng):
    """one frame: table [mbh, mbw, 2r+1, 2r+1]."""
    w = 2 * rng + 1
    out = np.zeros((mbh, mbw, w, w), sad_dtype(bd))
    getattr(_L, f"oracle{bd}_me_search_full")(_addr(fenc, f_origin), fs, _addr(ref, r_origin), rs, mbw, mbh,
                                             rng, _addr(out))
    return out


def me_search_full8(bd, fenc, f_origin, fs, ref, r_origin, rs, mbw, mbh, rng):
    """one frame's 8x8 quadrant tables: [mbh, mbw, 4, 2r+1, 2r+1] uint16."""
    w = 2 * rng + 1
    out = np.zeros((mbh, mbw, 4, w, w), np.uint16)
    getattr(_L, f"oracle{bd}_me_search_full8")(_addr(fenc, f_origin), fs, _addr(ref, r_origin), rs, mbw, mbh,
                                              rng, _addr(out))
    return out


def me_search_full_mt(fenc, f_origin, fs, ref, r_origin, rs, mbw, mbh, rng, nthreads):
    w = 2 * rng + 1
    out = np.zeros((mbh, mbw, w, w), np.uint16)
    used = _L.oracle8_me_search_full_mt(_addr(fenc, f_origin), fs, _addr(ref, r_origin), rs, mbw, mbh, rng,
                                        _addr(out), nthreads)
    return out, used


def mb_dct_quant(bd, transform, fenc, f_origin, fs, pred, p_origin, ps, mbw, mbh, mf, bias):
    dct = np.zeros((mbh * mbw, 256), coef_dtype(bd))
    nz = np.zeros(mbh * mbw, np.int32)
    m = np.ascontiguousarray(mf, ucoef_dtype(bd))
    b = np.ascontiguousarray(bias, ucoef_dtype(bd))
    getattr(_L, f"oracle{bd}_mb_dct_quant")(transform, _addr(fenc, f_origin), fs, _addr(pred, p_origin), ps,
                                           mbw, mbh, _addr(m), _addr(b), _addr(dct), _addr(nz))
    return dct, nz


def mb_dct_quant_mt(transform, fenc, f_origin, fs, pred, p_origin, ps, mbw, mbh, mf, bias, nthreads):
    dct = np.zeros((mbh * mbw, 256), np.int16)
    nz = np.zeros(mbh * mbw, np.int32)
    m = np.ascontiguousarray(mf, np.uint16)
    b = np.ascontiguousarray(bias, np.uint16)
    used = _L.oracle8_mb_dct_quant_mt(transform, _addr(fenc, f_origin), fs, _addr(pred, p_origin), ps, mbw, mbh,
                                      _addr(m), _addr(b), _addr(dct), _addr(nz), nthreads)
    return dct, nz, used


def frame_filter(bd, plane, origin, stride, width, height):
    """half-pel planes (H, V, C) of one padded plane (flat numpy), same layout."""
    outs = [np.zeros_like(plane) for _ in range(3)]
    getattr(_L, f"oracle{bd}_frame_filter")(_addr(plane, origin), _addr(outs[0], origin), _addr(outs[1], origin),
                                           _addr(outs[2], origin), stride, width, height)
    return outs


def subpel_list(bd, op, i_pixel, fenc, fs, planes, p_origin, rs, fenc_off, qxy):
    fo = np.ascontiguousarray(fenc_off, np.int64)
    q = np.ascontiguousarray(qxy, np.int32)
    out = np.zeros(len(fo), np.int32)
    getattr(_L, f"oracle{bd}_subpel_list")(_OPS.get(op, op), i_pixel, _addr(fenc), fs,
                                          *[_addr(p, p_origin) for p in planes], rs, _addr(fo), _addr(q),
                                          len(fo), _addr(out))
    return out


def subpel_list_mt(op, i_pixel, fenc, fs, planes, p_origin, rs, fenc_off, qxy, nthreads):
    """8-bit subpel_list split over nthreads (cpubench.c); returns (scores, threads used)."""
    fo = np.ascontiguousarray(fenc_off, np.int64)
    q = np.ascontiguousarray(qxy, np.int32)
    out = np.zeros(len(fo), np.int32)
    used = _L.oracle8_subpel_list_mt(_OPS.get(op, op), i_pixel, _addr(fenc), fs, *[_addr(p, p_origin) for p in planes],
                                     rs, _addr(fo), _addr(q), len(fo), _addr(out), nthreads)
    return out, used


def me_esa_argmin(bd, table, rng, me_range, par, init_cost, cost_mv, c0, origin=None):
    """table: numpy [nmb, 2r+1, pitch]; cost_mv numpy uint16 with mvd 0 at index c0;
    origin: int16 [nmb, 2] table origins (None = centred on mv 0)."""
    t = np.ascontiguousarray(table)
    p = np.ascontiguousarray(par, np.int16)
    ic = np.ascontiguousarray(init_cost, np.int32)
    out = np.zeros((len(p), 3), np.int32)
    o = None if origin is None else _addr(np.ascontiguousarray(origin, np.int16))
    getattr(_L, f"oracle{bd}_me_esa_argmin")(_addr(t), rng, len(p), me_range, o, _addr(p), _addr(ic),
                                            _addr(cost_mv, c0), _addr(out))
    return out


def me_search_esa8(bd, fenc, f_origin, fs, ref, r_origin, rs, mbw, mbh, me_range, par, init_cost, cost_mv, c0):
    """one frame: ESA decisions of every MB's eight sub-partitions (16x8 x2, 8x16 x2, 8x8 x4);
    par int16 [nmb*8, 8], init_cost int32 [nmb*8] -> out int32 [nmb*8, 3]."""
    p = np.ascontiguousarray(par, np.int16)
    ic = np.ascontiguousarray(init_cost, np.int32)
    out = np.zeros((len(p), 3), np.int32)
    getattr(_L, f"oracle{bd}_me_search_esa8")(_addr(fenc, f_origin), fs, _addr(ref, r_origin), rs, mbw, mbh,
                                             me_range, _addr(p), _addr(ic), _addr(cost_mv, c0), _addr(out))
    return out


def ssd_wxh(bd, a, a_off, sa, b, b_off, sb, w, h):
    """x264_pixel_ssd_wxh over a w x h rectangle (pixel.c:112-151)."""
    return int(getattr(_L, f"oracle{bd}_ssd_wxh")(_addr(a, a_off), sa, _addr(b, b_off), sb, w, h))


def ssd_nv12(bd, a, a_off, sa, b, b_off, sb, w, h):
    """x264_pixel_ssd_nv12 (pixel.c:153-178): (ssd_u, ssd_v)."""
    u = np.zeros(1, np.uint64)
    v = np.zeros(1, np.uint64)
    getattr(_L, f"oracle{bd}_ssd_nv12")(_addr(a, a_off), sa, _addr(b, b_off), sb, w, h, _addr(u), _addr(v))
    return int(u[0]), int(v[0])


def me_tesa(bd, fenc, f_origin, fs, ref, r_origin, integral, i_origin, rs, mbw, mbh, me_range, satd, par,
            init_cost, cost_mv, c0):
    """TESA decision of one frame (oracle me_tesa, me.c:653-748): int32 [nmb, 4] =
    (cost, mx, my, COST_MV evaluations).  integral: uint16 array with (0,0) at i_origin, stride rs."""
    p = np.ascontiguousarray(par, np.int16)
    ic = np.ascontiguousarray(init_cost, np.int32)
    out = np.zeros((len(p), 4), np.int32)
    getattr(_L, f"oracle{bd}_me_tesa")(_addr(fenc, f_origin), fs, _addr(ref, r_origin), _addr(integral, i_origin), rs,
                                      mbw, mbh, me_range, int(bool(satd)), _addr(p), _addr(ic), _addr(cost_mv, c0),
                                      _addr(out))
    return out


def me_search_centred(bd, fenc, f_origin, fs, ref, r_origin, rs, mbw, mbh, rng, centre):
    """one frame: (table [mbh, mbw, 2r+1, me_centred_pitch], origin int16 [mbh*mbw, 2])."""
    w = 2 * rng + 1
    pw = (2 * rng + (6 if bd == 8 else 4) + 3) // 4 * 4
    out = np.zeros((mbh, mbw, w, pw), sad_dtype(bd))
    org = np.zeros((mbh * mbw, 2), np.int16)
    c = np.ascontiguousarray(centre, np.int16)
    getattr(_L, f"oracle{bd}_me_search_centred")(_addr(fenc, f_origin), fs, _addr(ref, r_origin), rs, mbw, mbh,
                                                rng, _addr(c), _addr(out), _addr(org))
    return out, org


def refine_ext(b_chroma_me=0, chroma_format=1, mvy_offset=0, weights=(None, None, None)):
    """the ext[15] array of me_refine_subpel_ex: b_chroma_me, chroma_format, mvy_offset, then
    m->weight[0..2] as (weighted, scale, denom, offset); weights[p] = (scale, denom, offset) or None"""
    e = [int(b_chroma_me), int(chroma_format), int(mvy_offset)]
    for w in weights:
        e += [0, 0, 0, 0] if w is None else [1] + [int(v) for v in w]
    return np.array(e, np.int32)


def me_refine_subpel(bd, fenc, f_origin, fs, planes, r_origin, rs, i_pixel, subme, pos_xy, par, cost, cost_mv, c0,
                     refine_qpel=False, fpel_satd=False, counts=False, ext=None, fenc_c=None, fc_origin=0, fcs=0,
                     ref_c=None, rc_origin=0, rcs=0):
    """one frame: refine_subpel (me.c:865-992) of the partitions at pos_xy int32 [n, 2]; planes =
    the four reference planes (numpy, same layout); returns int32 [n, 4] (and the per-partition
    cmp-call counts, luma sad | luma satd << 16 | chroma mbcmp << 24, with counts=True).  ext
    (refine_ext) turns on chroma ME / weighted references: fenc_c = [NV12 plane] or [U, V],
    ref_c = [NV12 plane] or the F, H, V, C planes of U then V (4:4:4), with their origins /
    strides."""
    n = len(pos_xy)
    pos = np.ascontiguousarray(pos_xy, np.int32)
    p = np.ascontiguousarray(par, np.int16)
    c = np.ascontiguousarray(cost, np.int32)
    out = np.zeros((n, 4), np.int32)
    ne = np.zeros(n, np.int32)
    arr = (C.c_void_p * 4)(*[_addr(q, r_origin).value for q in planes])
    fca = (C.c_void_p * 2)(*([_addr(q, fc_origin).value for q in (fenc_c or [])] + [None] * 2)[:2])
    rca = (C.c_void_p * 8)(*([_addr(q, rc_origin).value for q in (ref_c or [])] + [None] * 8)[:8])
    e = None if ext is None else np.ascontiguousarray(ext, np.int32)
    getattr(_L, f"oracle{bd}_me_refine_subpel_ex")(_addr(fenc, f_origin), fs, arr, rs, i_pixel, subme,
                                                  int(bool(refine_qpel)), int(bool(fpel_satd)), _addr(pos), _addr(p),
                                                  _addr(c), _addr(cost_mv, c0), n, _addr(out), _addr(ne),
                                                  None if e is None else _addr(e), fca, fcs, rca, rcs)
    return (out, ne) if counts else out


def me_search_ref(bd, fenc, f_origin, fs, planes, fw, r_origin, rs, i_pixel, me_method, subme, me_range, pos_xy,
                  par, mvc, cost_mv, c0, ext=None, fenc_c=None, fc_origin=0, fcs=0, ref_c=None, rc_origin=0, rcs=0,
                  thresh=None, ref_cost=None, out_fill=0):
    """one frame: x264_me_search_ref (me.c:182-798) of the partitions at pos_xy int32 [n, 2] with
    me_method 0 DIA / 1 HEX / 2 UMH; par int16 [n, 12], mvc int16 [n, 14, 2] (search_cases.jobs);
    planes = F, H, V, C, fw = the weighted F plane (or F).  Returns int32 [n, 4] = (cost, mvx, mvy,
    cost_mv) and the call counts int32 [n, 2] (integer stage fpel | get_ref << 16, the refine's).
    thresh: int32 [n] p_halfpel_thresh per partition, updated in place (me_search_ref_thresh),
    ref_cost int32 [n] (or None); out starts filled with out_fill (the early exit leaves
    cost_mv as it was)."""
    n = len(pos_xy)
    pos = np.ascontiguousarray(pos_xy, np.int32)
    p = np.ascontiguousarray(par, np.int16)
    m = np.ascontiguousarray(mvc, np.int16)
    out = np.full((n, 4), out_fill, np.int32)
    ne = np.zeros((n, 2), np.int32)
    arr = (C.c_void_p * 4)(*[_addr(q, r_origin).value for q in planes])
    fca = (C.c_void_p * 2)(*([_addr(q, fc_origin).value for q in (fenc_c or [])] + [None] * 2)[:2])
    rca = (C.c_void_p * 8)(*([_addr(q, rc_origin).value for q in (ref_c or [])] + [None] * 8)[:8])
    e = None if ext is None else np.ascontiguousarray(ext, np.int32)
    args = [_addr(fenc, f_origin), fs, arr, _addr(fw, r_origin), rs, i_pixel, me_method, subme, me_range, _addr(pos),
            _addr(p), _addr(m), _addr(cost_mv, c0), n, _addr(out), _addr(ne), None if e is None else _addr(e), fca, fcs,
            rca, rcs]
    if thresh is None:
        getattr(_L, f"oracle{bd}_me_search_ref")(*args)
    else:
        assert thresh.dtype == np.int32 and thresh.flags.c_contiguous and len(thresh) == n
        rcst = None if ref_cost is None else np.ascontiguousarray(ref_cost, np.int32)
        getattr(_L, f"oracle{bd}_me_search_ref_thresh")(*args, _addr(thresh), None if rcst is None else _addr(rcst))
    return out, ne


def me_refine_bidir(bd, fenc, f_origin, fs, planes0, planes1, r_origin, rs, i_pixel, satd, pos_xy, par, weight,
                    cost_mv, c0):
    """one frame: x264_me_refine_bidir_satd (me.c:994-1183) of the partitions at pos_xy int32 [n, 2];
    planes0 / planes1 = F, H, V, C of the list 0 / 1 references; par int16 [n, 12] = (m0 mv x, y,
    m1 mv x, y, m0 mvp x, y, m1 mvp x, y, mv_min_spel x, y, mv_max_spel x, y); weight int32 [n].
    Returns (out int32 [n, 4] = m0 mv, m1 mv; cost int32 [n]; counts int32 [n] = calls | passes << 16)."""
    n = len(pos_xy)
    pos = np.ascontiguousarray(pos_xy, np.int32)
    p = np.ascontiguousarray(par, np.int16)
    w = np.ascontiguousarray(weight, np.int32)
    out = np.zeros((n, 4), np.int32)
    cost = np.zeros(n, np.int32)
    ne = np.zeros(n, np.int32)
    a0 = (C.c_void_p * 4)(*[_addr(q, r_origin).value for q in planes0])
    a1 = (C.c_void_p * 4)(*[_addr(q, r_origin).value for q in planes1])
    getattr(_L, f"oracle{bd}_me_refine_bidir")(_addr(fenc, f_origin), fs, a0, a1, rs, i_pixel, int(bool(satd)),
                                              _addr(pos), _addr(p), _addr(w), _addr(cost_mv, c0), n, _addr(out),
                                              _addr(cost), _addr(ne))
    return out, cost, ne


def me_refine_qpel_refdupe(bd, fenc, f_origin, fs, planes, r_origin, rs, i_pixel, subme, pos_xy, par, cost, cost_mv,
                           c0, thresh=None, ref_cost=None, out_fill=0, fpel_satd=False, ext=None, fenc_c=None,
                           fc_origin=0, fcs=0, ref_c=None, rc_origin=0, rcs=0):
    """one frame: x264_me_refine_qpel_refdupe (me.c:812-815) of the partitions at pos_xy; par /
    cost as me_refine_subpel, thresh / ref_cost / out_fill as me_search_ref.  Returns (out, counts)."""
    n = len(pos_xy)
    pos = np.ascontiguousarray(pos_xy, np.int32)
    p = np.ascontiguousarray(par, np.int16)
    c = np.ascontiguousarray(cost, np.int32)
    out = np.full((n, 4), out_fill, np.int32)
    ne = np.zeros(n, np.int32)
    arr = (C.c_void_p * 4)(*[_addr(q, r_origin).value for q in planes])
    fca = (C.c_void_p * 2)(*([_addr(q, fc_origin).value for q in (fenc_c or [])] + [None] * 2)[:2])
    rca = (C.c_void_p * 8)(*([_addr(q, rc_origin).value for q in (ref_c or [])] + [None] * 8)[:8])
    e = None if ext is None else np.ascontiguousarray(ext, np.int32)
    if thresh is not None:
        assert thresh.dtype == np.int32 and thresh.flags.c_contiguous and len(thresh) == n
    rcst = None if ref_cost is None else np.ascontiguousarray(ref_cost, np.int32)
    getattr(_L, f"oracle{bd}_me_refine_qpel_refdupe")(
        _addr(fenc, f_origin), fs, arr, rs, i_pixel, subme, int(bool(fpel_satd)), _addr(pos), _addr(p), _addr(c),
        _addr(cost_mv, c0), n, _addr(out), _addr(ne), None if e is None else _addr(e), fca, fcs, rca, rcs,
        None if thresh is None else _addr(thresh), None if rcst is None else _addr(rcst))
    return out, ne


# ---------------------------------------------------------------- further pixel entries
def sa8d(bd, i_pixel, a, a_off, sa, b, b_off, sb):
    return getattr(_L, f"oracle{bd}_sa8d")(i_pixel, _addr(a, a_off), sa, _addr(b, b_off), sb)


def sa8d_satd(bd, a, a_off, sa, b, b_off, sb):
    return getattr(_L, f"oracle{bd}_sa8d_satd")(_addr(a, a_off), sa, _addr(b, b_off), sb)


def hadamard_ac(bd, i_pixel, a, a_off, sa):
    return getattr(_L, f"oracle{bd}_hadamard_ac")(i_pixel, _addr(a, a_off), sa)


def var(bd, i_pixel, a, a_off, sa):
    return getattr(_L, f"oracle{bd}_var")(i_pixel, _addr(a, a_off), sa)


def var2(bd, i_pixel, fenc, f_off, fdec, d_off):
    """table form: fenc stride 16 (V at +8), fdec stride 32 (V at +16); returns (res, ssd_u, ssd_v)."""
    ssd = np.zeros(2, np.int32)
    r = getattr(_L, f"oracle{bd}_var2")(i_pixel, _addr(fenc, f_off), _addr(fdec, d_off), _addr(ssd))
    return r, int(ssd[0]), int(ssd[1])


def var2_s(bd, h, fenc, f_off, fs, fvd, fdec, d_off, ds, dvd):
    ssd = np.zeros(2, np.int32)
    r = getattr(_L, f"oracle{bd}_var2_s")(h, _addr(fenc, f_off), fs, fvd, _addr(fdec, d_off), ds, dvd, _addr(ssd))
    return r, int(ssd[0]), int(ssd[1])


def vsad(bd, a, a_off, stride, height):
    return getattr(_L, f"oracle{bd}_vsad")(_addr(a, a_off), stride, height)


def asd8(bd, a, a_off, sa, b, b_off, sb, height):
    return getattr(_L, f"oracle{bd}_asd8")(_addr(a, a_off), sa, _addr(b, b_off), sb, height)


def ads(bd, nsums, enc_dc, sums, s_off, delta, cost_mvx, c_off, width, thresh):
    """x264_pixel_ads{4,2,1}; returns the candidate index list (int16)."""
    dc = np.ascontiguousarray(enc_dc, np.int32)
    mvs = np.zeros(max(width, 1), np.int16)
    n = getattr(_L, f"oracle{bd}_ads")(nsums, _addr(dc), _addr(sums, s_off), delta, _addr(cost_mvx, c_off),
                                       _addr(mvs), width, thresh)
    return mvs[:n].copy()


def frame_integral(bd, plane, origin, stride, lines, padh, sub8x8):
    """integral part of x264_frame_filter; returns the uint16 buffer [(2 if sub8x8 else 1)*(lines+64), stride]
    whose element (32*stride + padh) is the integral's (0, 0)."""
    rows = (lines + 64) * (2 if sub8x8 else 1)
    buf = np.zeros(rows * stride, np.uint16)
    getattr(_L, f"oracle{bd}_frame_integral")(_addr(plane, origin), stride, lines, padh, sub8x8,
                                             _addr(buf, 32 * stride + padh))
    return buf.reshape(rows, stride)


# ---------------------------------------------------------------- inverse path
IDCT_KINDS = ["add4x4_idct", "add8x8_idct", "add16x16_idct", "add8x8_idct_dc", "add16x16_idct_dc",
              "add8x8_idct8", "add16x16_idct8"]
IDCT_IN = [16, 64, 256, 4, 16, 64, 256]
IDCT_W = [4, 8, 16, 8, 16, 8, 16]


def fn(bd, name):
    return getattr(_L, f"oracle{bd}_{name}")


def add_idct(bd, name, dst, d_off, dct):
    """table form (dst stride 32) on copies; returns (dst', dct') since the C path mutates dct."""
    dst = dst.copy()
    d = np.ascontiguousarray(dct, coef_dtype(bd)).copy()
    fn(bd, name)(_addr(dst, d_off), _addr(d))
    return dst, d


def add_idct_list(bd, kind, dst, ds, dst_off, dct):
    dst = dst.copy()
    do = np.ascontiguousarray(dst_off, np.int64)
    d = np.ascontiguousarray(dct, coef_dtype(bd))
    fn(bd, "add_idct_list")(kind, _addr(dst), ds, _addr(do), _addr(d), len(do))
    return dst


def cqm_dequant(scaling_lists, transform_8x8=True):
    lists = [np.ascontiguousarray(np.asarray(x, np.uint8)) for x in scaling_lists]
    ptrs = (C.c_void_p * 8)(*[x.ctypes.data for x in lists])
    dq4 = np.zeros((4, 6, 16), np.int32)
    dq8 = np.zeros((2, 6, 64), np.int32)
    _L.oracle8_cqm_dequant(ptrs, int(bool(transform_8x8)), _addr(dq4), _addr(dq8))
    return dq4, dq8


def inplace(bd, name, dct, *args):
    d = np.ascontiguousarray(dct, coef_dtype(bd)).copy()
    r = fn(bd, name)(_addr(d), *args)
    return d, r


def coeff_level_run(bd, dct, num):
    d = np.ascontiguousarray(dct, coef_dtype(bd))
    last, mask = C.c_int32(), C.c_int32()
    level = np.zeros(18, coef_dtype(bd))
    n = fn(bd, "coeff_level_run")(_addr(d), num, C.byref(last), C.byref(mask), _addr(level))
    return n, last.value, mask.value, level[:n].copy()


def zigzag_scan(bd, n, field, dct):
    d = np.ascontiguousarray(dct, coef_dtype(bd))
    level = np.zeros(n, coef_dtype(bd))
    fn(bd, f"zigzag_scan_{'8x8' if n == 64 else '4x4'}")(int(field), _addr(level), _addr(d))
    return level


def zigzag_sub(bd, kind, field, src, s_off, ss, dst, d_off, ds):
    """returns (nz, level, dc, dst')"""
    dst = dst.copy()
    level = np.zeros(64 if kind == 2 else 16, coef_dtype(bd))
    dc = np.zeros(1, coef_dtype(bd))
    nz = fn(bd, "zigzag_sub_s")(kind, int(field), _addr(level), _addr(src, s_off), ss, _addr(dst, d_off), ds,
                               _addr(dc))
    return nz, level, int(dc[0]), dst


def mb_dequant_idct_add(bd, transform, dct, mbw, mbh, dmf, qp, pred, p_origin, ps, recon, r_origin, rs):
    """one frame; recon is modified in place and returned."""
    d = np.ascontiguousarray(dct, coef_dtype(bd))
    m = np.ascontiguousarray(dmf, np.int32)
    q = np.ascontiguousarray(qp, np.int32)
    fn(bd, "mb_dequant_idct_add")(transform, _addr(d), mbw, mbh, _addr(m), _addr(q), _addr(pred, p_origin), ps,
                                  _addr(recon, r_origin), rs)
    return recon


def frame_init_lowres(bd, plane, origin, stride, width, height, dst_stride):
    """returns 4 lowres planes [(height/2 + 64), dst_stride] with (0,0) at (32, 32)."""
    hl = height // 2
    outs = [np.zeros((hl + 64) * dst_stride, pixel_dtype(bd)) for _ in range(4)]
    ptrs = (C.c_void_p * 4)(*[o.ctypes.data + (32 * dst_stride + 32) * o.itemsize for o in outs])
    fn(bd, "frame_init_lowres")(_addr(plane, origin), stride, width, height, ptrs, dst_stride)
    return [o.reshape(hl + 64, dst_stride) for o in outs]


FDEC_STRIDE, FENC_STRIDE = 32, 16
INTRA_SIZES = {0: (4, 4), 1: (8, 8), 2: (8, 16), 3: (16, 16), 4: (8, 8)}   # X264HIP_INTRA_* -> (w, h)


def predict_8x8(bd, mode, edge):
    """predict_8x8[mode] from a 36-entry edge; returns the 8x8 block"""
    e = np.ascontiguousarray(edge, pixel_dtype(bd))
    buf = np.zeros(9 * FDEC_STRIDE, pixel_dtype(bd))
    fn(bd, "predict_8x8")(mode, _addr(buf, FDEC_STRIDE + 8), _addr(e))
    return buf[FDEC_STRIDE:].reshape(8, FDEC_STRIDE)[:, 8:16].copy()


def predict_8x8_filter(bd, fdec, off, i_neighbor=15, i_filters=15, edge=None):
    """predict_8x8_filter on an FDEC-layout buffer at element offset off; returns edge[36]"""
    e = np.zeros(36, pixel_dtype(bd)) if edge is None else np.ascontiguousarray(edge, pixel_dtype(bd)).copy()
    fn(bd, "predict_8x8_filter")(_addr(fdec, off), _addr(e), i_neighbor, i_filters)
    return e


def intra_x3(bd, kind, op, fenc, f_off, fdec, d_off):
    """intra_*_x3 of kind X264HIP_INTRA_* (fenc stride 16, fdec stride 32 or edge[36] for kind 4)"""
    out = np.zeros(3, np.int32)
    fn(bd, "intra_x3")(kind, op, _addr(fenc, f_off), _addr(fdec, d_off), _addr(out))
    return out


def lowres_intra_cost(bd, plane, origin, stride, mbw, mbh, satd=True, all_modes=True, lam=4, inv_qscale=None):
    """slicetype_mb_cost's intra leg over one lowres plane: (intra_cost u16 [mbh*mbw], row_satd, est[2])"""
    cost = np.zeros(mbw * mbh, np.uint16)
    rows = np.zeros(mbh, np.int32)
    est = np.zeros(2, np.int32)
    iq = None if inv_qscale is None else np.ascontiguousarray(inv_qscale, np.uint16)
    fn(bd, "lowres_intra_cost")(_addr(plane, origin), stride, mbw, mbh, int(satd), int(all_modes), lam,
                                None if iq is None else _addr(iq), _addr(cost), _addr(rows), _addr(est))
    return cost, rows, est


def cost_mv_table(lam=1, mv_range=512):
    """h->cost_mv[qp] of analyse.c:143-157 for lambda `lam` (X264_LOOKAHEAD_QP = 12 -> 1):
    uint16 over mvd in [-8*mv_range, 8*mv_range]; returns (table, index of mvd 0).  logs
    are evaluated in float32 like the reference's log2f."""
    span = 2 * 4 * mv_range
    i = np.arange(span + 1, dtype=np.float32)
    logs = np.where(i == 0, np.float32(0.718), np.log2(i + np.float32(1)).astype(np.float32) * np.float32(2)
                    + np.float32(1.718)).astype(np.float32)
    half = np.minimum((np.float32(lam) * logs + np.float32(0.5)).astype(np.int64), 65535).astype(np.uint16)
    return np.concatenate([half[:0:-1], half]).astype(np.uint16), span


def weight_scale_plane(bd, src, src_off, stride, width, height, scale, denom, offset, dst=None):
    """x264_weight_scale_plane (frame.c:825-842) of the width x height region at src[src_off]
    (stride), into a copy of src (or dst) at the same offset; returns the destination array."""
    out = np.array(src, copy=True) if dst is None else dst
    fn(bd, "weight_scale_plane")(_addr(out, src_off), stride, _addr(src, src_off), stride, width, height, scale,
                                 denom, offset)
    return out


def lowres_inter_cost(bd, fenc, ref_planes, origin, stride, mbw, mbh, intra_cost, me_method=1, subme=4, satd=True,
                      me_range=16, mv_range=512, lam=1, cost_mv=None, inv_qscale=None, ref_w=None, weight=None,
                      n_slices=1):
    """slicetype_mb_cost's P-frame inter leg over one lowres pair (numpy planes, (0,0) at origin):
    (mvs int16 [mbs, 2], mv_costs int32 [mbs], lowres_costs uint16 [mbs], row_satd int32 [mbh], est int32 [3]).
    ref_w / weight (scale, denom, offset): the weighted-reference form (fenc->weighted[0])."""
    if cost_mv is None:
        cost_mv = cost_mv_table(lam, mv_range)
    cm, c0 = cost_mv
    n = mbw * mbh
    mvs = np.zeros((n, 2), np.int16)
    mvc = np.zeros(n, np.int32)
    lc = np.zeros(n, np.uint16)
    rows = np.zeros(mbh, np.int32)
    est = np.zeros(3, np.int32)
    ic = np.ascontiguousarray(intra_cost, np.uint16)
    iq = None if inv_qscale is None else np.ascontiguousarray(inv_qscale, np.uint16)
    wt = None if weight is None else np.ascontiguousarray(weight, np.int32)
    fn(bd, "lowres_inter_cost_ex")(_addr(fenc, origin), *[_addr(p, origin) for p in ref_planes],
                                  None if ref_w is None else _addr(ref_w, origin), None if wt is None else _addr(wt),
                                  n_slices, stride, mbw, mbh, me_method, subme, int(satd), me_range, mv_range, lam, _addr(cm, c0),
                                  _addr(ic), None if iq is None else _addr(iq), _addr(mvs), _addr(mvc), _addr(lc),
                                  _addr(rows), _addr(est))
    return mvs, mvc, lc, rows, est


def lowres_bidir_cost(bd, fenc, ref_a, ref_b, origin, stride, mbw, mbh, search, mvs0, costs0, mvs1, costs1,
                      p1mvs=None, dsf=128, weight=32, me_method=1, subme=4, satd=True, me_range=16, mv_range=512,
                      lam=1, cost_mv=None, inv_qscale=None, n_slices=1):
    """slicetype_mb_cost's B-frame leg over one lowres triplet.  mvs_l int16 [mbs, 2] / costs_l
    int32 [mbs] are read (search bit clear) or written (set); copies are returned:
    (mvs0, costs0, mvs1, costs1, lowres_costs uint16 [mbs], row_satd int32 [mbh], est int32 [2])"""
    if cost_mv is None:
        cost_mv = cost_mv_table(lam, mv_range)
    cm, c0 = cost_mv
    n = mbw * mbh
    m0, k0 = np.array(mvs0, np.int16).reshape(n, 2).copy(), np.array(costs0, np.int32).reshape(n).copy()
    m1, k1 = np.array(mvs1, np.int16).reshape(n, 2).copy(), np.array(costs1, np.int32).reshape(n).copy()
    lc = np.zeros(n, np.uint16)
    rows = np.zeros(mbh, np.int32)
    est = np.zeros(2, np.int32)
    srch = (C.c_int * 2)(search & 1, (search >> 1) & 1)
    pa = (C.c_void_p * 4)(*[p.ctypes.data + origin * p.itemsize for p in ref_a])
    pb = (C.c_void_p * 4)(*[p.ctypes.data + origin * p.itemsize for p in ref_b])
    p1 = None if p1mvs is None else np.ascontiguousarray(p1mvs, np.int16)
    iq = None if inv_qscale is None else np.ascontiguousarray(inv_qscale, np.uint16)
    fn(bd, "lowres_bidir_cost_ex")(_addr(fenc, origin), pa, pb, stride, mbw, mbh, me_method, subme, int(satd),
                                   me_range, mv_range, lam, _addr(cm, c0), srch, _addr(m0), _addr(k0), _addr(m1),
                                   _addr(k1), None if p1 is None else _addr(p1), dsf, weight,
                                   None if iq is None else _addr(iq), _addr(lc), _addr(rows), _addr(est), n_slices)
    return m0, k0, m1, k1, lc, rows, est


# ---- weighted-prediction analysis (slicetype.c:63-501, ratecontrol.c:225-257,406-414) ----
for _bd in (8, 10):
    _f(_bd, "mc_chroma", [_P, _P, _IP, _P, _IP, C.c_int, C.c_int, C.c_int, C.c_int])
    _f(_bd, "frame_pixel_stats", [_P, _P, C.c_int, C.c_int, C.c_int, _P, _P])
    _f(_bd, "weight_cost_list", [C.c_int, _P, _P, _IP, C.c_int, C.c_int, _P, _P, C.c_int, C.c_int, C.c_int,
                                 C.c_int, _P, C.c_int, _P])
    _f(_bd, "weights_analyse", [_P, _P, _IP, C.c_int, C.c_int, _P, _P, C.c_int, _P, _P, _P, _P, _P, _P, _P,
                                C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _P, _P, _P])


def _ptrs(arrs_offs):
    return (C.c_void_p * len(arrs_offs))(*[None if a is None else a.ctypes.data + int(o) * a.itemsize
                                           for a, o in arrs_offs])


def mc_chroma(bd, src, s_off, ss, mvx, mvy, w, h):
    """mc_chroma (mc.c:252-283) of an interleaved plane: (u, v) uint arrays [h, w]"""
    u = np.zeros((h, w), pixel_dtype(bd))
    v = np.zeros((h, w), pixel_dtype(bd))
    fn(bd, "mc_chroma")(_addr(u), _addr(v), w, _addr(src, s_off), ss, mvx, mvy, w, h)
    return u, v


def frame_pixel_stats(bd, planes, origins, strides, mbw, mbh, chroma_format):
    """(sum uint32 [3], ssd uint64 [3]) as x264_adaptive_quant_frame leaves i_pixel_sum / i_pixel_ssd;
    planes = [luma, NV12 plane or U, V (4:4:4) or None]"""
    s = np.zeros(3, np.uint32)
    d = np.zeros(3, np.uint64)
    pp = _ptrs([(p, o) if p is not None else (None, 0) for p, o in zip(planes, origins)])
    st = (C.c_ssize_t * 3)(*[int(x) for x in strides])
    fn(bd, "frame_pixel_stats")(pp, st, mbw, mbh, chroma_format, _addr(s), _addr(d))
    return s, d


def weight_cost_list(bd, kind, fenc, refs, origin, stride, mbw, mbh, cands, intra=None, mvs=None, satd=True,
                     plane=0, lam=1, n_slices=1):
    """weight_cost_luma / _chroma / _chroma444 of each (weighted, scale, denom, offset) in cands: uint32 [n]"""
    c = np.ascontiguousarray(np.array(cands, np.int32).reshape(-1, 4))
    out = np.zeros(len(c), np.uint32)
    rp = _ptrs([(r, origin) for r in refs] + [(None, 0)] * (4 - len(refs)))
    ic = None if intra is None else np.ascontiguousarray(intra, np.uint16)
    mv = None if mvs is None else np.ascontiguousarray(mvs, np.int16)
    fn(bd, "weight_cost_list")(kind, _addr(fenc, origin), rp, stride, mbw, mbh, None if ic is None else _addr(ic),
                               None if mv is None else _addr(mv), int(satd), plane, lam, n_slices, _addr(c), len(c),
                               _addr(out))
    return out


def weights_analyse(bd, fenc_lr, ref_lr, lr_origin, lrs, mbw, mbh, intra, fstats, rstats, mvs=None,
                    chroma_format=0, fenc_c=(None, None), ref_c=(None, None), c_origin=0, cs=0, b_lookahead=True,
                    subme=7, satd=True, lam=1, n_slices=1, weightp_fake=False, weighted=None):
    """x264_weights_analyse: (weights int32 [3, 4] = (weighted, scale, denom, offset), cost_delta or None).
    fstats / rstats = (sum [3], ssd [3]); weighted (lowres plane array like ref_lr[0]) receives the
    weighted lowres reference in the lookahead."""
    w = np.zeros((3, 4), np.int32)
    cd = np.full(1, -1.0, np.float32)
    ic = np.ascontiguousarray(intra, np.uint16)
    mv = None if mvs is None else np.ascontiguousarray(mvs, np.int16)
    rl = _ptrs([(r, lr_origin) for r in ref_lr])
    fp = _ptrs([(fenc_lr, lr_origin), (fenc_c[0], c_origin), (fenc_c[1], c_origin)])
    rp = _ptrs([(ref_lr[0], lr_origin), (ref_c[0], c_origin), (ref_c[1], c_origin)])
    ps = (C.c_ssize_t * 3)(lrs, cs, cs)
    if chroma_format in (1, 2):   # the oracle reads NV12 as plane[1]
        fp[2], rp[2] = fp[1], rp[1]
    fs_ = np.array(fstats[0], np.uint32), np.array(fstats[1], np.uint64)
    rs_ = np.array(rstats[0], np.uint32), np.array(rstats[1], np.uint64)
    fn(bd, "weights_analyse")(_addr(fenc_lr, lr_origin), rl, lrs, mbw, mbh, _addr(ic),
                              None if mv is None else _addr(mv), chroma_format, fp, rp, ps, _addr(fs_[0]),
                              _addr(fs_[1]), _addr(rs_[0]), _addr(rs_[1]), int(b_lookahead), subme, int(satd), lam,
                              n_slices, int(weightp_fake), w.ctypes.data, _addr(cd),
                              None if weighted is None else _addr(weighted, lr_origin))
    return w, (None if cd[0] == -1.0 else float(cd[0]))


# ---- SSIM (pixel.c:627-714) ----
for _bd in (8, 10):
    _f(_bd, "ssim_4x4x2_core", [_P, _IP, _P, _IP, _P])
    _f(_bd, "ssim_end4", [_P, _P, C.c_int], C.c_float)
    _f(_bd, "ssim_wxh", [_P, _IP, _P, _IP, C.c_int, C.c_int, _P], C.c_float)


def ssim_4x4x2_core(bd, a, a_off, sa, b, b_off, sb):
    s = np.zeros((2, 4), np.int32)
    fn(bd, "ssim_4x4x2_core")(_addr(a, a_off), sa, _addr(b, b_off), sb, _addr(s))
    return s


def ssim_end4(bd, sum0, sum1, width):
    s0 = np.ascontiguousarray(sum0, np.int32).reshape(5, 4)
    s1 = np.ascontiguousarray(sum1, np.int32).reshape(5, 4)
    return np.float32(fn(bd, "ssim_end4")(_addr(s0), _addr(s1), width))


def ssim_bands_mt(a, a_off, sa, b, b_off, sb, width, bands, nthreads):
    """8-bit x264_pixel_ssim_wxh over the { y, h } bands of a frame pair on nthreads pthreads
    (cpubench.c): (ssim float32 [nbands], cnt int32 [nbands])"""
    bd_ = np.ascontiguousarray(bands, np.int32)
    out = np.zeros(len(bd_), np.float32)
    cnt = np.zeros(len(bd_), np.int32)
    used = _L.oracle8_ssim_bands_mt(_addr(a, a_off), sa, _addr(b, b_off), sb, width, _addr(bd_), len(bd_),
                                    _addr(out), _addr(cnt), nthreads)
    assert used > 0
    return out, cnt


def ssim_wxh(bd, a, a_off, sa, b, b_off, sb, width, height):
    """x264_pixel_ssim_wxh: (ssim float32, cnt)"""
    cnt = C.c_int(0)
    v = fn(bd, "ssim_wxh")(_addr(a, a_off), sa, _addr(b, b_off), sb, width, height, C.byref(cnt))
    return np.float32(v), cnt.value
