"""x264hip — host-side mirror of x264's pixel / dct / quant function tables,
backed by the gfx950 HIP kernels in ``libx264hip.so`` (C ABI: include/x264hip.h).

Two layers, mirroring the C ABI:

* ``pixel_init(bitdepth)``, ``dct_init(bitdepth)``, ``quant_init(bitdepth)``
  return ctypes structs laid out exactly like the reference's
  ``x264_pixel_function_t`` / ``x264_dct_function_t`` / ``x264_quant_function_t``
  (reference common/pixel.h:78-144, common/dct.h:29-59, common/quant.h:30-70),
  filled by ``x264hip_{8,10}_*_init(X264HIP_CPU_HIP, ...)``.  Entries are called
  like the reference's (``pixf.sad[PIXEL_16x16](pix1, 16, pix2, 64)``) and each
  call runs one GPU dispatch.
* Batched wrappers (``me_search_full``, ``pixel_cmp_batch``, ``sub_dct_batch``,
  ``dc_batch``, ``quant_batch``, ``quant_dc_batch``, ``mb_dct_quant``) take
  device-resident torch tensors and enqueue on the current torch stream.

There is no CPU fallback: if the shared library is missing or no gfx950 device
is usable, every entry point raises ``BackendUnavailable``.
"""
import ctypes
import os

import numpy as np

__all__ = [
    "LIB_PATH", "BackendUnavailable", "lib", "init", "pixel_init", "dct_init", "quant_init",
    "cqm_init", "pixel_cmp_batch", "me_search_full", "sub_dct_batch", "dc_batch", "quant_batch",
    "quant_dc_batch", "mb_dct_quant", "hpel_filter", "subpel_cmp_batch", "subpel_qpel9_batch", "me_table_pitch", "me_centred_pitch", "me_refine_subpel", "me_search_ref", "ssim_bands", "ssim_encoder_bands", "refine_ext", "RefineExt", "lowres_status", "trim", "me_esa_argmin", "me_tesa", "me_search_esa", "me_search_esa8", "me_analyse_p16x16", "ssd_plane_batch", "ssd_nv12_batch", "alloc_planes", "PIXEL_16x16", "PIXEL_16x8", "PIXEL_8x16",
    "PIXEL_8x8", "PIXEL_8x4", "PIXEL_4x8", "PIXEL_4x4", "PIXEL_4x16", "PIXEL_SIZES",
    "CMP_SAD", "CMP_SSD", "CMP_SATD", "CPU_HIP", "set_variant", "set_thread_device", "thread_device",
    "backend_banner", "forward_ref", "upload", "me_bind", "MeBinding", "weight_scale_plane", "stream_pair", "stream_pair_destroy", "me_search_full8",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
# X264HIP_LIBRARY: an alternative in-tree build of the same library (A/B timing of two
# builds of one kernel, tools/lib_ab.py); the default is the package's own build
LIB_PATH = os.environ.get("X264HIP_LIBRARY") or os.path.join(_HERE, "libx264hip.so")

# reference common/pixel.h:37-59
PIXEL_16x16, PIXEL_16x8, PIXEL_8x16, PIXEL_8x8, PIXEL_8x4, PIXEL_4x8, PIXEL_4x4, PIXEL_4x16 = range(8)
PIXEL_SIZES = [(16, 16), (16, 8), (8, 16), (8, 8), (8, 4), (4, 8), (4, 4), (4, 16)]
CMP_SAD, CMP_SSD, CMP_SATD, CMP_SA8D = 0, 1, 2, 3
STAT_VAR, STAT_HADAMARD_AC, STAT_SA8D_SATD, STAT_VSAD, STAT_ASD8 = 0, 1, 2, 3, 4
IDCT_ADD4x4, IDCT_ADD8x8, IDCT_ADD16x16, IDCT_ADD8x8_DC, IDCT_ADD16x16_DC, IDCT_ADD8x8_8, IDCT_ADD16x16_8 = range(7)
IDCT_IN_SIZE = [16, 64, 256, 4, 16, 64, 256]
DEQUANT_4x4, DEQUANT_8x8, DEQUANT_4x4_DC = 0, 1, 2
COEF_DECIMATE15, COEF_DECIMATE16, COEF_DECIMATE64, COEF_LAST4, COEF_LAST8, COEF_LAST15, COEF_LAST16, COEF_LAST64 = range(8)
ZIGZAG_SUB_4x4, ZIGZAG_SUB_4x4AC, ZIGZAG_SUB_8x8 = 0, 1, 2
INTRA_4x4, INTRA_8x8C, INTRA_8x16C, INTRA_16x16, INTRA_8x8 = range(5)
INTRA_SIZES = [(4, 4), (8, 8), (8, 16), (16, 16), (8, 8)]
DC_I4x4 = 2
DCT_SUB4x4, DCT_SUB8x8, DCT_SUB16x16, DCT_SUB8x8_DC, DCT_SUB8x16_DC, DCT_SUB8x8_8, DCT_SUB16x16_8 = range(7)
DCT_OUT_SIZE = [16, 64, 256, 4, 8, 64, 256]
DC_4x4, DC_2x4 = 0, 1
QUANT_8x8, QUANT_4x4, QUANT_4x4x4, QUANT_4x4_DC, QUANT_2x2_DC = range(5)
CPU_HIP = 1 << 26
FENC_STRIDE, FDEC_STRIDE = 16, 32
PAD = 32  # x264 PADH / PADV, reference common/frame.h:32-33


class BackendUnavailable(RuntimeError):
    """The gfx950 backend (libx264hip.so or a gfx950 device) is not usable."""


_lib = None


def lib():
    """Load libx264hip.so (no fallback: raises if it is missing)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise BackendUnavailable(
                f"{LIB_PATH} not built; run `make -C x264-i386pic_amd/csrc` (or __graft_entry__.build())")
        # Bind the library to torch's HIP runtime: torch bundles libamdhip64.so with the
        # same SONAME (libamdhip64.so.7), so loading torch first makes the dynamic loader
        # reuse that copy instead of mapping a second HIP/HSA runtime from /opt/rocm
        # (two runtimes in one process cannot share the GPU).
        import torch  # noqa: F401
        _lib = ctypes.CDLL(LIB_PATH)
        _declare(_lib)
    return _lib


def init(device=0):
    """x264hip_init(device); raises BackendUnavailable if no gfx950 device."""
    rc = lib().x264hip_init(device)
    if rc != 0:
        raise BackendUnavailable(f"x264hip_init({device}) = {rc}: {lib().x264hip_last_error().decode()}")


def set_variant(name, value=None):
    """Select an A/B kernel variant by its environment name (``X264HIP_ME_VARIANT`` ...);
    ``None`` / -1 restores the default.  Every variant is bit-exact."""
    v = -1 if value is None or value == "default" else int(value)
    if lib().x264hip_set_variant(name.encode(), v) != 0:
        raise ValueError(f"unknown kernel variant switch {name!r}")


def set_thread_device(device):
    """Bind the calling thread's table entries to ``device`` (-1: the process device)."""
    rc = lib().x264hip_set_thread_device(device)
    if rc != 0:
        raise BackendUnavailable(f"x264hip_set_thread_device({device}) = {rc}: {lib().x264hip_last_error().decode()}")


def thread_device():
    return lib().x264hip_thread_device()


def backend_banner():
    return lib().x264hip_backend_banner().decode()


def forward_ref(dst, dst_device, src, src_device):
    """Peer-copy a reconstructed reference (torch tensors of equal size) to the next GPU."""
    import torch
    nbytes = src.numel() * src.element_size()
    if dst.numel() * dst.element_size() != nbytes:
        raise ValueError("forward_ref: size mismatch")
    with torch.cuda.device(src.device):
        _rc(lib().x264hip_forward_ref(_c.c_void_p(dst.data_ptr()), dst_device, _c.c_void_p(src.data_ptr()),
                                      src_device, nbytes, _stream()), "forward_ref")
    return dst


def upload(dst, src):
    """Copy a pinned host tensor into a device tensor of the same size with the
    library's PCIe-read kernel (x264hip_upload) on the current stream."""
    nbytes = src.numel() * src.element_size()
    if dst.numel() * dst.element_size() != nbytes or not src.is_pinned() or not dst.is_cuda:
        raise ValueError("upload: needs a pinned host source and a device destination of equal size")
    _rc(lib().x264hip_upload(_c.c_void_p(dst.data_ptr()), _c.c_void_p(src.data_ptr()), nbytes, _stream()), "upload")
    return dst


class PlaneUpload(ctypes.Structure):
    """x264hip_plane_upload_t"""
    _fields_ = [("dst", ctypes.c_void_p), ("dst_stride", ctypes.c_ssize_t), ("host_src", ctypes.c_void_p),
                ("src_stride", ctypes.c_ssize_t), ("width_bytes", ctypes.c_int32), ("height", ctypes.c_int32),
                ("unit", ctypes.c_int32), ("pad_x", ctypes.c_int32), ("pad_y", ctypes.c_int32)]


def plane_upload(dst, dst_origin, dst_stride, src, unit=1, pad_x=32, pad_y=32):
    """one x264hip_plane_upload_t: the pinned host picture plane `src` [height, width] (rows may be
    longer) into the padded device plane `dst` whose pixel (0,0) is element dst_origin (dst_stride
    elements per row), borders expanded by pad_x bytes / pad_y rows, unit = the edge element's
    bytes"""
    if not src.is_pinned() or not dst.is_cuda:
        raise ValueError("plane_upload: needs a pinned host source and a device destination")
    es = dst.element_size()
    return PlaneUpload(dst.data_ptr() + dst_origin * es, dst_stride * es, src.data_ptr(),
                       src.stride(0) * src.element_size(), src.shape[1] * src.element_size(), src.shape[0], unit,
                       pad_x, pad_y)


def upload_planes(uploads):
    """x264hip_upload_planes: the plane_upload() records of one picture (1..3) in one launch on
    the current stream"""
    arr = (PlaneUpload * len(uploads))(*uploads)
    _rc(lib().x264hip_upload_planes(len(uploads), arr, _stream()), "upload_planes")


def upload_plane(dst, dst_origin, dst_stride, src, unit=1, pad_x=32, pad_y=32):
    """x264hip_upload_plane: one picture plane (see plane_upload)"""
    u = plane_upload(dst, dst_origin, dst_stride, src, unit, pad_x, pad_y)
    _rc(lib().x264hip_upload_plane(_c.c_void_p(u.dst), _c.c_ssize_t(u.dst_stride), _c.c_void_p(u.host_src),
                                   _c.c_ssize_t(u.src_stride), u.width_bytes, u.height, unit, pad_x, pad_y,
                                   _stream()), "upload_plane")
    return dst


def stream_pair(reserve_cus=16):
    """(compute, copy) torch external streams on complementary CU sets of the current device
    (x264hip_stream_pair_create): the copy stream owns the first `reserve_cus` CUs."""
    import torch
    a, b = _c.c_void_p(), _c.c_void_p()
    _rc(lib().x264hip_stream_pair_create(reserve_cus, _c.byref(a), _c.byref(b)), "stream_pair_create")
    return torch.cuda.ExternalStream(a.value), torch.cuda.ExternalStream(b.value)


def stream_pair_destroy(pair):
    """Release the streams of stream_pair() (after a device synchronise; the torch wrappers must
    not be used afterwards)."""
    import torch
    torch.cuda.synchronize()
    for st in pair:
        _rc(lib().x264hip_stream_destroy(_c.c_void_p(st.cuda_stream)), "stream_destroy")


# ----------------------------------------------------------------- tables
_c = ctypes
_P = _c.c_void_p
_IP = _c.c_ssize_t   # intptr_t

CMP_T = _c.CFUNCTYPE(_c.c_int, _P, _IP, _P, _IP)
CMP_X3_T = _c.CFUNCTYPE(None, _P, _P, _P, _P, _IP, _P)
CMP_X4_T = _c.CFUNCTYPE(None, _P, _P, _P, _P, _P, _IP, _P)
DCT_T = _c.CFUNCTYPE(None, _P, _P, _P)            # sub*_dct*(dct, pix1, pix2)
DC_T = _c.CFUNCTYPE(None, _P)                     # dct4x4dc(d)
DC2_T = _c.CFUNCTYPE(None, _P, _P)                # dct2x4dc(dct, dct4x4)
QUANT_T = _c.CFUNCTYPE(_c.c_int, _P, _P, _P)      # quant_*(dct, mf, bias)
QUANT_DC_T = _c.CFUNCTYPE(_c.c_int, _P, _c.c_int, _c.c_int)
VSAD_T = _c.CFUNCTYPE(_c.c_int, _P, _IP, _c.c_int)                 # vsad(pix, stride, height)
ASD8_T = _c.CFUNCTYPE(_c.c_int, _P, _IP, _P, _IP, _c.c_int)        # asd8(p1, s1, p2, s2, height)
CMP64_T = _c.CFUNCTYPE(_c.c_uint64, _P, _IP, _P, _IP)              # sa8d_satd
VAR_T = _c.CFUNCTYPE(_c.c_uint64, _P, _IP)                         # var / hadamard_ac
VAR2_T = _c.CFUNCTYPE(_c.c_int, _P, _P, _P)                        # var2(fenc, fdec, ssd[2])
ADS_T = _c.CFUNCTYPE(_c.c_int, _P, _P, _c.c_int, _P, _P, _c.c_int, _c.c_int)
IDCT_T = _c.CFUNCTYPE(None, _P, _P)                                # add*_idct*(p_dst, dct)
DEQ_T = _c.CFUNCTYPE(None, _P, _P, _c.c_int)                       # dequant_*(dct, dmf, qp)
IDQ24_T = _c.CFUNCTYPE(None, _P, _P, _P, _c.c_int)                 # idct_dequant_2x4_dc
IDQ24O_T = _c.CFUNCTYPE(None, _P, _P, _c.c_int)                    # idct_dequant_2x4_dconly
OPTC_T = _c.CFUNCTYPE(_c.c_int, _P, _c.c_int)                      # optimize_chroma_*_dc
DENOISE_T = _c.CFUNCTYPE(None, _P, _P, _P, _c.c_int)
COEF_T = _c.CFUNCTYPE(_c.c_int, _P)                                # decimate / coeff_last
RUNLEVEL_T = _c.CFUNCTYPE(_c.c_int, _P, _P)
ZSCAN_T = _c.CFUNCTYPE(None, _P, _P)
ZSUB_T = _c.CFUNCTYPE(_c.c_int, _P, _P, _P)
ZSUBAC_T = _c.CFUNCTYPE(_c.c_int, _P, _P, _P, _P)
ZINTER_T = _c.CFUNCTYPE(None, _P, _P, _P)
INTRA_X3_T = _c.CFUNCTYPE(None, _P, _P, _P)                        # intra_*_x3(fenc, fdec|edge, res[3])
SSD_NV12_T = _c.CFUNCTYPE(None, _P, _IP, _P, _IP, _c.c_int, _c.c_int, _P, _P)   # ssd_nv12_core
SSIM_CORE_T = _c.CFUNCTYPE(None, _P, _IP, _P, _IP, _P)             # ssim_4x4x2_core(p1, s1, p2, s2, sums)
SSIM_END4_T = _c.CFUNCTYPE(_c.c_float, _P, _P, _c.c_int)           # ssim_end4(sum0, sum1, width)


class PixelFunctions(_c.Structure):
    """Layout of x264_pixel_function_t, reference common/pixel.h:78-144."""
    _fields_ = [
        ("sad", CMP_T * 8), ("ssd", CMP_T * 8), ("satd", CMP_T * 8), ("ssim", CMP_T * 7),
        ("sa8d", CMP_T * 4), ("mbcmp", CMP_T * 8), ("mbcmp_unaligned", CMP_T * 8),
        ("fpelcmp", CMP_T * 8), ("fpelcmp_x3", CMP_X3_T * 7), ("fpelcmp_x4", CMP_X4_T * 7),
        ("sad_aligned", CMP_T * 8), ("vsad", VSAD_T), ("asd8", ASD8_T), ("sa8d_satd", CMP64_T * 1),
        ("var", VAR_T * 4), ("var2", VAR2_T * 4), ("hadamard_ac", VAR_T * 4),
        ("ssd_nv12_core", SSD_NV12_T), ("ssim_4x4x2_core", SSIM_CORE_T), ("ssim_end4", SSIM_END4_T),
        ("sad_x3", CMP_X3_T * 7), ("sad_x4", CMP_X4_T * 7),
        ("satd_x3", CMP_X3_T * 7), ("satd_x4", CMP_X4_T * 7), ("ads", ADS_T * 7),
    ] + [(n, INTRA_X3_T) for n in (
        "intra_mbcmp_x3_16x16", "intra_satd_x3_16x16", "intra_sad_x3_16x16",
        "intra_mbcmp_x3_4x4", "intra_satd_x3_4x4", "intra_sad_x3_4x4",
        "intra_mbcmp_x3_chroma", "intra_satd_x3_chroma", "intra_sad_x3_chroma",
        "intra_mbcmp_x3_8x16c", "intra_satd_x3_8x16c", "intra_sad_x3_8x16c",
        "intra_mbcmp_x3_8x8c", "intra_satd_x3_8x8c", "intra_sad_x3_8x8c",
        "intra_mbcmp_x3_8x8", "intra_sa8d_x3_8x8", "intra_sad_x3_8x8")] + [(n, _P) for n in (
        "intra_mbcmp_x9_4x4", "intra_satd_x9_4x4", "intra_sad_x9_4x4",
        "intra_mbcmp_x9_8x8", "intra_sa8d_x9_8x8", "intra_sad_x9_8x8")]


class DctFunctions(_c.Structure):
    """Layout of x264_dct_function_t, reference common/dct.h:29-59."""
    _fields_ = [
        ("sub4x4_dct", DCT_T), ("add4x4_idct", IDCT_T), ("sub8x8_dct", DCT_T), ("sub8x8_dct_dc", DCT_T),
        ("add8x8_idct", IDCT_T), ("add8x8_idct_dc", IDCT_T), ("sub8x16_dct_dc", DCT_T), ("sub16x16_dct", DCT_T),
        ("add16x16_idct", IDCT_T), ("add16x16_idct_dc", IDCT_T), ("sub8x8_dct8", DCT_T), ("add8x8_idct8", IDCT_T),
        ("sub16x16_dct8", DCT_T), ("add16x16_idct8", IDCT_T), ("dct4x4dc", DC_T), ("idct4x4dc", DC_T),
        ("dct2x4dc", DC2_T),
    ]


class QuantFunctions(_c.Structure):
    """Layout of x264_quant_function_t, reference common/quant.h:30-70."""
    _fields_ = [
        ("quant_8x8", QUANT_T), ("quant_4x4", QUANT_T), ("quant_4x4x4", QUANT_T),
        ("quant_4x4_dc", QUANT_DC_T), ("quant_2x2_dc", QUANT_DC_T),
        ("dequant_8x8", DEQ_T), ("dequant_4x4", DEQ_T), ("dequant_4x4_dc", DEQ_T),
        ("idct_dequant_2x4_dc", IDQ24_T), ("idct_dequant_2x4_dconly", IDQ24O_T),
        ("optimize_chroma_2x2_dc", OPTC_T), ("optimize_chroma_2x4_dc", OPTC_T), ("denoise_dct", DENOISE_T),
        ("decimate_score15", COEF_T), ("decimate_score16", COEF_T), ("decimate_score64", COEF_T),
        ("coeff_last", COEF_T * 14), ("coeff_last4", COEF_T), ("coeff_last8", COEF_T),
        ("coeff_level_run", RUNLEVEL_T * 13), ("coeff_level_run4", RUNLEVEL_T), ("coeff_level_run8", RUNLEVEL_T),
        ("trellis_cabac_4x4", _P), ("trellis_cabac_8x8", _P), ("trellis_cabac_4x4_psy", _P),
        ("trellis_cabac_8x8_psy", _P), ("trellis_cabac_dc", _P), ("trellis_cabac_chroma_422_dc", _P),
    ]


class ZigzagFunctions(_c.Structure):
    """Layout of x264_zigzag_function_t, reference common/dct.h:61-70."""
    _fields_ = [("scan_8x8", ZSCAN_T), ("scan_4x4", ZSCAN_T), ("sub_8x8", ZSUB_T), ("sub_4x4", ZSUB_T),
                ("sub_4x4ac", ZSUBAC_T), ("interleave_8x8_cavlc", ZINTER_T)]


def _check_bd(bitdepth):
    if bitdepth not in (8, 10):
        raise ValueError("bitdepth must be 8 or 10")


def _table(kind, struct, bitdepth, cpu):
    _check_bd(bitdepth)
    init()  # loud failure without a gfx950 device
    tab = struct()
    fn = getattr(lib(), f"x264hip_{bitdepth}_{kind}_init")
    if kind == "quant":
        fn(None, cpu, _c.byref(tab))
    else:
        fn(cpu, _c.byref(tab))
    return tab


def pixel_init(bitdepth=8, cpu=CPU_HIP):
    """x264_pixel_init equivalent (reference common/pixel.c:809)."""
    return _table("pixel", PixelFunctions, bitdepth, cpu)


def dct_init(bitdepth=8, cpu=CPU_HIP):
    """x264_dct_init equivalent (reference common/dct.c:477)."""
    return _table("dct", DctFunctions, bitdepth, cpu)


def quant_init(bitdepth=8, cpu=CPU_HIP):
    """x264_quant_init equivalent (reference common/quant.c:414)."""
    return _table("quant", QuantFunctions, bitdepth, cpu)


def zigzag_init(bitdepth=8, cpu=CPU_HIP):
    """x264_zigzag_init equivalent (reference common/dct.c:938): (progressive, interlaced)."""
    _check_bd(bitdepth)
    init()
    p, i = ZigzagFunctions(), ZigzagFunctions()
    getattr(lib(), f"x264hip_{bitdepth}_zigzag_init")(cpu, _c.byref(p), _c.byref(i))
    return p, i


def cqm_dequant(scaling_lists, transform_8x8=True):
    """dequant4_mf [4][6][16], dequant8_mf [2][6][64] (int32) of x264_cqm_init (reference common/set.c:124-159)."""
    import numpy as np
    lists = [np.ascontiguousarray(np.asarray(x, np.uint8)) for x in scaling_lists]
    ptrs = (_P * 8)(*[x.ctypes.data for x in lists])
    dq4 = np.zeros((4, 6, 16), np.int32)
    dq8 = np.zeros((2, 6, 64), np.int32)
    lib().x264hip_cqm_dequant(ptrs, int(bool(transform_8x8)), dq4.ctypes.data, dq8.ctypes.data)
    return dq4, dq8


# ----------------------------------------------------------------- declarations
def _declare(L):
    L.x264hip_init.argtypes = [_c.c_int]
    L.x264hip_init.restype = _c.c_int
    L.x264hip_last_error.restype = _c.c_char_p
    L.x264hip_available.restype = _c.c_int
    L.x264hip_set_thread_device.argtypes = [_c.c_int]
    L.x264hip_set_thread_device.restype = _c.c_int
    L.x264hip_thread_device.restype = _c.c_int
    L.x264hip_forward_ref.argtypes = [_P, _c.c_int, _P, _c.c_int, _c.c_size_t, _P]
    L.x264hip_forward_ref.restype = _c.c_int
    L.x264hip_upload.argtypes = [_P, _P, _c.c_size_t, _P]
    L.x264hip_upload.restype = _c.c_int
    L.x264hip_upload_plane.argtypes = [_P, _IP, _P, _IP, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _P]
    L.x264hip_upload_plane.restype = _c.c_int
    L.x264hip_upload_planes.argtypes = [_c.c_int, _P, _P]
    L.x264hip_upload_planes.restype = _c.c_int
    L.x264hip_stream_pair_create.argtypes = [_c.c_int, _P, _P]
    L.x264hip_stream_pair_create.restype = _c.c_int
    L.x264hip_stream_destroy.argtypes = [_P]
    L.x264hip_stream_destroy.restype = _c.c_int
    L.x264hip_backend_banner.restype = _c.c_char_p
    L.x264hip_set_variant.argtypes = [_c.c_char_p, _c.c_int]
    L.x264hip_set_variant.restype = _c.c_int
    L.x264hip_cqm_dequant.argtypes = [_P, _c.c_int, _P, _P]
    L.x264hip_me_unbind.restype = None
    L.x264hip_me_bind_stats.argtypes = [_P, _P, _c.c_int]
    L.x264hip_me_bind_stats.restype = None
    for bd in (8, 10):
        f = lambda n: getattr(L, f"x264hip_{bd}_{n}")  # noqa: E731
        f("me_bind").argtypes = [_P, _P, _IP, _c.c_int, _c.c_int, _P, _c.c_int]
        f("me_bind").restype = _c.c_int
        f("me_bind_tables").argtypes = [_P, _P, _IP, _c.c_int, _c.c_int, _P, _P, _c.c_int]
        f("me_bind_tables").restype = _c.c_int
        f("pixel_init").argtypes = [_c.c_uint32, _P]
        f("dct_init").argtypes = [_c.c_uint32, _P]
        f("quant_init").argtypes = [_P, _c.c_uint32, _P]
        f("pixel_init_hip").argtypes = [_P]
        f("dct_init_hip").argtypes = [_P]
        f("quant_init_hip").argtypes = [_P]
        f("cqm_init").argtypes = [_P, _c.c_int, _c.c_int, _c.c_int, _P, _P, _P, _P]
        f("cqm_init").restype = _c.c_int
        f("pixel_cmp_batch").argtypes = [_c.c_int, _c.c_int, _P, _IP, _P, _IP, _P, _P, _c.c_int, _P, _P]
        f("me_search_full").argtypes = [_P, _IP, _IP, _P, _IP, _IP, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _P, _P]
        f("me_search_full8").argtypes = [_P, _IP, _IP, _P, _IP, _IP, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _P, _P]
        f("me_search_full8").restype = _c.c_int
        f("sub_dct_batch").argtypes = [_c.c_int, _P, _IP, _P, _IP, _P, _P, _c.c_int, _P, _P]
        f("dc_batch").argtypes = [_c.c_int, _P, _P, _c.c_int, _P]
        f("quant_batch").argtypes = [_c.c_int, _P, _P, _P, _c.c_int, _P, _P]
        f("quant_dc_batch").argtypes = [_c.c_int, _P, _c.c_int, _c.c_int, _c.c_int, _P, _P]
        f("me_esa_argmin").argtypes = [_P, _c.c_int, _c.c_int, _c.c_int, _P, _P, _P, _P, _P]
        f("me_esa_argmin_at").argtypes = [_P, _c.c_int, _c.c_int, _c.c_int, _P, _P, _P, _P, _P, _P]
        f("me_search_centred").argtypes = [_P, _IP, _IP, _P, _IP, _IP, _c.c_int, _c.c_int, _c.c_int, _c.c_int,
                                           _P, _P, _P, _P]
        f("me_esa_argmin_at").restype = _c.c_int
        f("me_tesa").argtypes = [_P, _IP, _IP, _P, _IP, _IP, _P, _IP, _c.c_int, _c.c_int, _c.c_int, _c.c_int,
                                 _c.c_int, _P, _c.c_int, _P, _P, _P, _P, _P, _P]
        f("me_tesa").restype = _c.c_int
        for n in ("ssd_plane_batch", "ssd_nv12_batch"):
            f(n).argtypes = [_P, _IP, _IP, _P, _IP, _IP, _c.c_int, _c.c_int, _c.c_int, _P, _P]
            f(n).restype = _c.c_int
        f("me_search_centred").restype = _c.c_int
        f("hpel_filter").argtypes = [_P, _P, _P, _P, _IP, _IP, _c.c_int, _c.c_int, _c.c_int, _P]
        f("subpel_cmp_batch").argtypes = [_c.c_int, _c.c_int, _P, _IP, _P, _P, _P, _P, _IP, _P, _P, _c.c_int, _P, _P]
        f("subpel_qpel9_batch").argtypes = [_c.c_int, _c.c_int, _P, _IP, _P, _P, _P, _P, _IP, _P, _P, _c.c_int, _P,
                                            _P]
        f("subpel_qpel9_batch").restype = _c.c_int
        f("mb_dct_quant").argtypes = [_c.c_int, _P, _IP, _IP, _P, _IP, _IP, _c.c_int, _c.c_int, _c.c_int,
                                      _P, _P, _P, _P, _P]
        f("pixel_stat_batch").argtypes = [_c.c_int, _c.c_int, _P, _IP, _P, _IP, _P, _P, _c.c_int, _c.c_int, _P, _P]
        f("var2_batch").argtypes = [_c.c_int, _P, _IP, _IP, _P, _IP, _IP, _P, _P, _c.c_int, _P, _P]
        f("ads_batch").argtypes = [_c.c_int, _P, _P, _c.c_int, _P, _P, _P, _P, _P, _c.c_int, _P, _c.c_int, _P, _P]
        f("frame_integral").argtypes = [_P, _IP, _IP, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _P, _IP, _P]
        f("zigzag_init").argtypes = [_c.c_uint32, _P, _P]
        f("zigzag_init_hip").argtypes = [_P, _P]
        f("add_idct_batch").argtypes = [_c.c_int, _P, _IP, _P, _P, _c.c_int, _P]
        f("dequant_batch").argtypes = [_c.c_int, _P, _P, _P, _c.c_int, _P]
        f("idct_dequant_2x4_batch").argtypes = [_c.c_int, _P, _P, _P, _P, _c.c_int, _P]
        f("optimize_chroma_dc_batch").argtypes = [_c.c_int, _P, _P, _c.c_int, _P, _P]
        f("denoise_dct_batch").argtypes = [_P, _c.c_int, _c.c_int, _P, _P, _P]
        f("coef_stat_batch").argtypes = [_c.c_int, _P, _c.c_int64, _c.c_int, _P, _P]
        f("coeff_level_run_batch").argtypes = [_c.c_int, _P, _c.c_int64, _c.c_int, _P, _P, _P, _P, _P]
        f("zigzag_scan_batch").argtypes = [_c.c_int, _c.c_int, _P, _P, _c.c_int, _P]
        f("zigzag_sub_batch").argtypes = [_c.c_int, _c.c_int, _P, _P, _P, _IP, _P, _IP, _P, _P, _c.c_int, _P, _P]
        f("zigzag_interleave_batch").argtypes = [_P, _P, _P, _c.c_int, _P]
        f("frame_init_lowres").argtypes = [_P, _IP, _IP, _c.c_int, _c.c_int, _c.c_int, _P, _IP, _IP, _P]
        f("frame_init_lowres").restype = _c.c_int
        f("intra_cmp_x3_batch").argtypes = [_c.c_int, _c.c_int, _P, _IP, _P, _IP, _P, _P, _c.c_int, _P, _P]
        f("intra_cmp_x3_batch").restype = _c.c_int
        f("lowres_intra_cost").argtypes = [_P, _IP, _IP, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_int,
                                           _c.c_int, _P, _P, _P, _P, _P]
        f("lowres_intra_cost").restype = _c.c_int
        f("lowres_inter_cost").argtypes = [_P, _IP, _P, _P, _P, _P, _IP, _IP, _c.c_int, _c.c_int, _c.c_int, _c.c_int,
                                           _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _P, _P, _P, _P, _P, _P,
                                           _P, _P, _P]
        f("lowres_inter_cost").restype = _c.c_int
        f("lowres_inter_cost_ex").argtypes = f("lowres_inter_cost").argtypes[:-1] + [_P, _c.c_int, _c.c_int,
                                                                                    _c.c_int, _c.c_int, _P]
        f("lowres_inter_cost_ex").restype = _c.c_int
        f("weight_scale_plane").argtypes = [_P, _IP, _IP, _P, _IP, _IP, _c.c_int, _c.c_int, _c.c_int, _c.c_int,
                                            _c.c_int, _c.c_int, _P]
        f("weight_scale_plane").restype = _c.c_int
        f("lowres_bidir_cost").argtypes = [_P, _IP, _P, _P, _P, _P, _IP, _P, _P, _P, _P, _IP, _IP, _c.c_int,
                                           _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_int,
                                           _c.c_int, _P, _c.c_int, _P, _P, _P, _P, _P, _c.c_int, _c.c_int, _P, _P,
                                           _P, _P, _P]
        f("lowres_bidir_cost_ex").argtypes = f("lowres_bidir_cost").argtypes[:-1] + [_c.c_int, _P]
        f("lowres_bidir_cost_ex").restype = _c.c_int
        f("lowres_bidir_cost").restype = _c.c_int
        f("mb_dequant_idct_add").argtypes = [_c.c_int, _P, _c.c_int, _c.c_int, _c.c_int, _P, _P, _P, _IP, _IP,
                                             _P, _IP, _IP, _P]
        for n in ("add_idct_batch", "dequant_batch", "idct_dequant_2x4_batch", "optimize_chroma_dc_batch",
                  "denoise_dct_batch", "coef_stat_batch", "coeff_level_run_batch", "zigzag_scan_batch",
                  "zigzag_sub_batch", "zigzag_interleave_batch", "mb_dequant_idct_add"):
            f(n).restype = _c.c_int
        for n in ("pixel_stat_batch", "var2_batch", "ads_batch", "frame_integral", "pixel_cmp_batch", "me_search_full", "me_esa_argmin", "hpel_filter", "subpel_cmp_batch", "sub_dct_batch", "dc_batch", "quant_batch",
                  "quant_dc_batch", "mb_dct_quant"):
            f(n).restype = _c.c_int


# ----------------------------------------------------------------- CQM
def cqm_init(bitdepth, scaling_lists, deadzone_inter=21, deadzone_intra=11, transform_8x8=True):
    """Quant mf/bias tables (restated x264_cqm_init, reference common/set.c:73-206).

    scaling_lists: 8 sequences (4 of 16, 4 of 64 entries) like sps->scaling_list.
    Returns numpy arrays (quant4_mf, quant4_bias [4][QP+1][16], quant8_mf, quant8_bias [4][QP+1][64]).
    """
    import numpy as np
    _check_bd(bitdepth)
    qp1 = 52 + 6 * (bitdepth - 8)
    ut = np.uint16 if bitdepth == 8 else np.uint32
    q4m = np.zeros((4, qp1, 16), ut)
    q4b = np.zeros((4, qp1, 16), ut)
    q8m = np.zeros((4, qp1, 64), ut)
    q8b = np.zeros((4, qp1, 64), ut)
    lists = [np.ascontiguousarray(np.asarray(s, np.uint8)) for s in scaling_lists]
    ptrs = (_P * 8)(*[x.ctypes.data for x in lists])
    getattr(lib(), f"x264hip_{bitdepth}_cqm_init")(
        ptrs, deadzone_inter, deadzone_intra, int(bool(transform_8x8)),
        q4m.ctypes.data, q4b.ctypes.data, q8m.ctypes.data, q8b.ctypes.data)
    return q4m, q4b, q8m, q8b


# ----------------------------------------------------------------- batched (torch)
def _stream():
    import torch
    return _c.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t, offset_elems=0):
    return _c.c_void_p(t.data_ptr() + offset_elems * t.element_size())


def _rc(rc, name):
    if rc != 0:
        raise RuntimeError(f"x264hip {name} failed ({rc}): {lib().x264hip_last_error().decode()}")


def _pix_bd(t):
    import torch
    if t.dtype == torch.uint8:
        return 8
    if t.dtype in (torch.int16, torch.uint16):
        return 10
    raise TypeError("pixel tensors are uint8 (8-bit) or int16/uint16 (10-bit)")


def alloc_planes(nframes, width, height, bitdepth=8, device="cuda", pad=PAD):
    """Padded plane stack like x264's frames (PADH/PADV = pad, reference common/frame.c:59-87).

    Returns (tensor[nframes, height + 2*pad, stride], stride, origin) where origin is
    the element offset of pixel (0,0) of frame 0 and stride is a multiple of 64 pixels.
    """
    import torch
    stride = (width + 2 * pad + 63) // 64 * 64
    dt = torch.uint8 if bitdepth == 8 else torch.int16
    t = torch.zeros((nframes, height + 2 * pad, stride), dtype=dt, device=device)
    return t, stride, pad * stride + pad


def pixel_cmp_batch(op, i_pixel, fenc, fenc_stride, ref, ref_stride, fenc_off, ref_off, scores=None):
    """scores[i] = op(fenc + fenc_off[i], ref + ref_off[i]) (device int64 offsets, pixels)."""
    import torch
    bd = _pix_bd(fenc)
    n = fenc_off.numel()
    if scores is None:
        scores = torch.empty(n, dtype=torch.int32, device=fenc.device)
    _rc(getattr(lib(), f"x264hip_{bd}_pixel_cmp_batch")(
        op, i_pixel, _ptr(fenc), fenc_stride, _ptr(ref), ref_stride, _ptr(fenc_off), _ptr(ref_off), n,
        _ptr(scores), _stream()), "pixel_cmp_batch")
    return scores


def pixel_stat_batch(op, i_pixel, pix1, stride1, off1, pix2=None, stride2=0, off2=None, height=0, out=None):
    """out[i] (uint64 as int64 tensor) = STAT_* entry at pix1 + off1[i] (and pix2 + off2[i])."""
    import torch
    bd = _pix_bd(pix1)
    n = off1.numel()
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=pix1.device)
    p2 = pix2 if pix2 is not None else pix1
    o2 = off2 if off2 is not None else off1
    _rc(getattr(lib(), f"x264hip_{bd}_pixel_stat_batch")(
        op, i_pixel, _ptr(pix1), stride1, _ptr(p2), stride2 or stride1, _ptr(off1), _ptr(o2), height, n,
        _ptr(out), _stream()), "pixel_stat_batch")
    return out


def var2_batch(i_pixel, fenc, fenc_stride, fenc_vdelta, fdec, fdec_stride, fdec_vdelta, fenc_off, fdec_off,
               out=None):
    """int32 [n, 3] = (var2 result, ssd_u, ssd_v) per U/V block pair."""
    import torch
    bd = _pix_bd(fenc)
    n = fenc_off.numel()
    if out is None:
        out = torch.empty((n, 3), dtype=torch.int32, device=fenc.device)
    _rc(getattr(lib(), f"x264hip_{bd}_var2_batch")(
        i_pixel, _ptr(fenc), fenc_stride, fenc_vdelta, _ptr(fdec), fdec_stride, fdec_vdelta, _ptr(fenc_off),
        _ptr(fdec_off), n, _ptr(out), _stream()), "var2_batch")
    return out


def ads_batch(bitdepth, i_pixel, enc_dc, sums, delta, sums_off, cost_mvx, cost_off, width, thresh, mvs_pitch=None):
    """n calls of ads[i_pixel]; returns (mvs int16 [n, pitch], nmv int32 [n])."""
    import torch
    _check_bd(bitdepth)
    n = sums_off.numel()
    pitch = mvs_pitch if mvs_pitch is not None else max(1, int(width.max().item()) if n else 1)
    mvs = torch.full((n, pitch), -1, dtype=torch.int16, device=sums.device)
    nmv = torch.empty(n, dtype=torch.int32, device=sums.device)
    _rc(getattr(lib(), f"x264hip_{bitdepth}_ads_batch")(
        i_pixel, _ptr(enc_dc), _ptr(sums), delta, _ptr(sums_off), _ptr(cost_mvx), _ptr(cost_off), _ptr(width),
        _ptr(thresh), n, _ptr(mvs), pitch, _ptr(nmv), _stream()), "ads_batch")
    return mvs, nmv


def frame_integral(planes, origin, stride, lines, padh=PAD, sub8x8=False, out=None):
    """ESA integral image per frame: uint16 (as int16) [n, (2 if sub8x8 else 1) * (lines + 2*PAD), stride];
    element [f, PAD + y, padh + x] is (x, y).  planes: [n, rows, stride] padded planes."""
    import torch
    bd = _pix_bd(planes)
    n = planes.shape[0]
    rows = (lines + 2 * PAD) * (2 if sub8x8 else 1)
    if out is None:
        out = torch.zeros((n, rows, stride), dtype=torch.int16, device=planes.device)
    _rc(getattr(lib(), f"x264hip_{bd}_frame_integral")(
        _ptr(planes, origin), stride, planes[0].numel(), lines, padh, int(bool(sub8x8)), n,
        _ptr(out, PAD * stride + padh), out[0].numel(), _stream()), "frame_integral")
    return out


def add_idct_batch(kind, dst, dst_stride, dst_off, dct):
    """in-place add*_idct* (IDCT_*) on dst + dst_off[i]; dct [n, size] (not modified)."""
    bd = _pix_bd(dst)
    _rc(getattr(lib(), f"x264hip_{bd}_add_idct_batch")(kind, _ptr(dst), dst_stride, _ptr(dst_off), _ptr(dct),
                                                        dst_off.numel(), _stream()), "add_idct_batch")
    return dst


def dequant_batch(kind, dct, dequant_mf, qp):
    """in-place dequant (DEQUANT_*) of dct [n, 16|64] with one list's int32 [6][16|64] and qp[n]."""
    bd = _coef_bd(dct)
    _rc(getattr(lib(), f"x264hip_{bd}_dequant_batch")(kind, _ptr(dct), _ptr(dequant_mf), _ptr(qp), qp.numel(),
                                                       _stream()), "dequant_batch")
    return dct


def idct_dequant_2x4_batch(dconly, dct, dequant_mf, qp, dct4x4=None):
    bd = _coef_bd(dct)
    _rc(getattr(lib(), f"x264hip_{bd}_idct_dequant_2x4_batch")(
        int(dconly), _ptr(dct), _ptr(dct4x4) if dct4x4 is not None else None, _ptr(dequant_mf), _ptr(qp),
        qp.numel(), _stream()), "idct_dequant_2x4_batch")
    return dct4x4 if dct4x4 is not None else dct


def optimize_chroma_dc_batch(c422, dct, dequant_mf):
    import torch
    bd = _coef_bd(dct)
    n = dequant_mf.numel()
    nz = torch.empty(n, dtype=torch.int32, device=dct.device)
    _rc(getattr(lib(), f"x264hip_{bd}_optimize_chroma_dc_batch")(int(c422), _ptr(dct), _ptr(dequant_mf), n,
                                                                  _ptr(nz), _stream()), "optimize_chroma_dc_batch")
    return nz


def denoise_dct_batch(dct, size, sums, offset):
    bd = _coef_bd(dct)
    _rc(getattr(lib(), f"x264hip_{bd}_denoise_dct_batch")(_ptr(dct), size, dct.numel() // size, _ptr(sums),
                                                           _ptr(offset), _stream()), "denoise_dct_batch")
    return dct


def coef_stat_batch(kind, dct, pitch, n):
    import torch
    bd = _coef_bd(dct)
    out = torch.empty(n, dtype=torch.int32, device=dct.device)
    _rc(getattr(lib(), f"x264hip_{bd}_coef_stat_batch")(kind, _ptr(dct), pitch, n, _ptr(out), _stream()),
        "coef_stat_batch")
    return out


def coeff_level_run_batch(num, dct, pitch, n):
    """returns (last, mask, count, level [n, 18])"""
    import torch
    bd = _coef_bd(dct)
    last, mask, count = (torch.empty(n, dtype=torch.int32, device=dct.device) for _ in range(3))
    level = torch.zeros((n, 18), dtype=dct.dtype, device=dct.device)
    _rc(getattr(lib(), f"x264hip_{bd}_coeff_level_run_batch")(num, _ptr(dct), pitch, n, _ptr(last), _ptr(mask),
                                                               _ptr(count), _ptr(level), _stream()),
        "coeff_level_run_batch")
    return last, mask, count, level


def zigzag_scan_batch(size, field, dct):
    import torch
    bd = _coef_bd(dct)
    n = dct.numel() // (size * size)
    level = torch.empty_like(dct)
    _rc(getattr(lib(), f"x264hip_{bd}_zigzag_scan_batch")(size, int(field), _ptr(level), _ptr(dct), n, _stream()),
        "zigzag_scan_batch")
    return level


def zigzag_sub_batch(kind, field, src, src_stride, dst, dst_stride, src_off, dst_off):
    """returns (level [n, 16|64], dc [n], nz [n]); dst blocks become the src blocks."""
    import torch
    bd = _pix_bd(src)
    n = src_off.numel()
    w = 8 if kind == 2 else 4
    ct = torch.int16 if bd == 8 else torch.int32
    level = torch.empty((n, w * w), dtype=ct, device=src.device)
    dc = torch.zeros(n, dtype=ct, device=src.device)
    nz = torch.empty(n, dtype=torch.int32, device=src.device)
    _rc(getattr(lib(), f"x264hip_{bd}_zigzag_sub_batch")(kind, int(field), _ptr(level), _ptr(dc), _ptr(src),
                                                          src_stride, _ptr(dst), dst_stride, _ptr(src_off),
                                                          _ptr(dst_off), n, _ptr(nz), _stream()), "zigzag_sub_batch")
    return level, dc, nz


def zigzag_interleave_batch(src):
    import torch
    bd = _coef_bd(src)
    n = src.numel() // 64
    dst = torch.empty_like(src)
    nnz = torch.zeros((n, 16), dtype=torch.uint8, device=src.device)
    _rc(getattr(lib(), f"x264hip_{bd}_zigzag_interleave_batch")(_ptr(dst), _ptr(src), _ptr(nnz), n, _stream()),
        "zigzag_interleave_batch")
    return dst, nnz


def mb_dequant_idct_add(transform, dct, mb_width, mb_height, nframes, dequant_mf, qp, pred, pred_origin,
                        pred_stride, recon, recon_origin, recon_stride, pred_frame_stride=None,
                        recon_frame_stride=None):
    """recon = clip(pred + idct(dequant(dct))) per MB (x264hip_*_mb_dequant_idct_add)."""
    bd = _pix_bd(pred)
    pfs = pred_frame_stride if pred_frame_stride is not None else (pred[0].numel() if pred.dim() == 3 else 0)
    rfs = recon_frame_stride if recon_frame_stride is not None else (recon[0].numel() if recon.dim() == 3 else 0)
    _rc(getattr(lib(), f"x264hip_{bd}_mb_dequant_idct_add")(
        transform, _ptr(dct), mb_width, mb_height, nframes, _ptr(dequant_mf), _ptr(qp), _ptr(pred, pred_origin),
        pred_stride, pfs, _ptr(recon, recon_origin), recon_stride, rfs, _stream()), "mb_dequant_idct_add")
    return recon


def frame_init_lowres(planes, origin, stride, width, height, outs=None):
    """x264_frame_init_lowres of every frame of `planes` [n, rows, stride]: four half-resolution
    planes [n, height/2 + 2*PAD, lowres_stride] with (0,0) at (PAD, PAD); returns (outs, lowres_stride)."""
    import torch
    bd = _pix_bd(planes)
    n = planes.shape[0]
    wl, hl = width // 2, height // 2
    ls = plane_stride(wl)
    if outs is None:
        # one buffer, the four planes equally spaced as x264's buffer_lowres (frame.c), which the
        # lookahead kernels address by plane index
        buf = torch.zeros((4, n, hl + 2 * PAD, ls), dtype=planes.dtype, device=planes.device)
        outs = [buf[k] for k in range(4)]
    ptrs = (_P * 4)(*[o.data_ptr() + (PAD * ls + PAD) * o.element_size() for o in outs])
    _rc(getattr(lib(), f"x264hip_{bd}_frame_init_lowres")(
        _ptr(planes, origin), stride, planes[0].numel(), width, height, n, ptrs, ls, outs[0][0].numel(), _stream()),
        "frame_init_lowres")
    return outs, ls


def intra_cmp_x3_batch(kind, op, fenc, fenc_stride, fdec, fdec_stride, fenc_off, fdec_off, out=None):
    """int32 [n, 3] = intra_*_x3 of kind INTRA_* per block (fdec_off: the block's (0,0) in fdec, or the
    start of its 36-entry edge for INTRA_8x8)."""
    import torch
    bd = _pix_bd(fenc)
    n = fenc_off.numel()
    if out is None:
        out = torch.empty((n, 3), dtype=torch.int32, device=fenc.device)
    _rc(getattr(lib(), f"x264hip_{bd}_intra_cmp_x3_batch")(
        kind, op, _ptr(fenc), fenc_stride, _ptr(fdec), fdec_stride, _ptr(fenc_off), _ptr(fdec_off), n,
        _ptr(out), _stream()), "intra_cmp_x3_batch")
    return out


def lowres_intra_cost(lowres, lowres_stride, mb_width, mb_height, satd=True, all_modes=True, lam=4,
                      inv_qscale=None, with_rows=True, outs=None):
    """The lookahead's intra estimate of every lowres plane in `lowres` [n, rows, stride] (lowres[0] of
    frame_init_lowres, (0,0) at (PAD, PAD)): (intra_cost uint16-as-int16 [n, mbh*mbw],
    row_satd int32 [n, mbh], cost_est int32 [n, 2])."""
    import torch
    bd = _pix_bd(lowres)
    n = lowres.shape[0]
    dev = lowres.device
    if outs is not None:
        cost, rows, est = outs
    else:
        cost = torch.empty((n, mb_width * mb_height), dtype=torch.int16, device=dev)
        rows = torch.empty((n, mb_height), dtype=torch.int32, device=dev) if with_rows else None
        est = torch.empty((n, 2), dtype=torch.int32, device=dev) if with_rows else None
    _rc(getattr(lib(), f"x264hip_{bd}_lowres_intra_cost")(
        _ptr(lowres, PAD * lowres_stride + PAD), lowres_stride, lowres[0].numel(), mb_width, mb_height, n,
        int(bool(satd)), int(bool(all_modes)), lam, _ptr(inv_qscale) if inv_qscale is not None else None,
        _ptr(cost), _ptr(rows) if rows is not None else None, _ptr(est) if est is not None else None,
        _stream()), "lowres_intra_cost")
    return cost, rows, est


def _frame_stride(*planes):
    """element distance between consecutive frames of [n, rows, stride] plane tensors (views such
    as lowres[0][1::3] included); every plane of one reference must share it."""
    fs = {p.stride(0) if p.shape[0] > 1 else p[0].numel() for p in planes}
    if len(fs) != 1:
        raise ValueError(f"planes disagree on the frame stride: {sorted(fs)}")
    for p in planes:
        if p.stride(1) != p.shape[2] or p.stride(2) != 1:
            raise ValueError("each frame's plane must be row-contiguous")
    return fs.pop()


def weight_scale_plane(src, lowres_stride, width, height, scale, denom, offset, out=None):
    """x264_weight_scale_plane over whole padded lowres planes [n, rows, stride] (the
    reference's call of slicetype.c:490-499: from pixel (-PAD, -PAD), width + 2*PAD columns,
    height + 2*PAD rows): fenc->weighted[0] of each plane.  Returns `out` (same shape)."""
    import torch
    bd = _pix_bd(src)
    w = width + 2 * PAD
    cov = 0
    while cov < w - 8:
        cov += 16
    cov = cov + 8 if cov < w else cov
    if cov > lowres_stride:                            # the last row's strip would leave the plane
        raise ValueError("weight_scale_plane: the reference's 8/16-wide strips overrun the stride")
    if out is None:
        out = torch.empty_like(src)
    n = src.shape[0]
    _rc(getattr(lib(), f"x264hip_{bd}_weight_scale_plane")(
        _ptr(out), lowres_stride, _frame_stride(out), _ptr(src), lowres_stride, _frame_stride(src),
        width + 2 * PAD, height + 2 * PAD, n, scale, denom, offset, _stream()), "weight_scale_plane")
    return out


def lowres_inter_cost(fenc, refs, lowres_stride, mb_width, mb_height, intra_cost, cost_mv_center, me_method=1,
                      subme=4, satd=True, me_range=16, mv_range=512, lam=1, inv_qscale=None, outs=None,
                      ref_w=None, weight=None, n_slices=1, check=True):
    """The lookahead's P-frame lowres motion search (x264hip_*_lowres_inter_cost) for the pairs
    (fenc[i], refs[*][i]): fenc = lowres[0] planes [n, rows, stride], refs = the four lowres planes
    (F, H, V, C) of the references, same shape; (0,0) at (PAD, PAD).  intra_cost [n, mbs] from
    lowres_intra_cost; cost_mv_center = (uint16-as-int16 tensor, element offset of mvd 0).  Returns
    (mvs int16 [n, mbs, 2], mv_costs int32 [n, mbs], lowres_costs uint16-as-int16 [n, mbs],
    row_satd int32 [n, mbh], est int32 [n, 3]).  ref_w (weighted F planes, weight_scale_plane) and
    weight = (scale, denom, offset): the weighted-reference search (x264hip_*_lowres_inter_cost_w).
    The launch is asynchronous; check=True then waits for it and raises if its wavefront timed
    out (lowres_status), check=False leaves that to a later lowres_status() / lookahead call."""
    import torch
    bd = _pix_bd(fenc)
    n = fenc.shape[0]
    nmb = mb_width * mb_height
    dev = fenc.device
    if outs is None:
        outs = (torch.empty((n, nmb, 2), dtype=torch.int16, device=dev),
                torch.empty((n, nmb), dtype=torch.int32, device=dev),
                torch.empty((n, nmb), dtype=torch.int16, device=dev),
                torch.empty((n, mb_height), dtype=torch.int32, device=dev),
                torch.empty((n, 3), dtype=torch.int32, device=dev))
    mvs, mvc, lc, rows, est = outs
    cm, c0 = cost_mv_center
    o = PAD * lowres_stride + PAD
    if (ref_w is None) != (weight is None):
        raise ValueError("lowres_inter_cost: ref_w and weight go together")
    rfs = _frame_stride(*refs) if ref_w is None else _frame_stride(*refs, ref_w)
    w = (0, 0, 0) if weight is None else tuple(int(v) for v in weight)
    _rc(getattr(lib(), f"x264hip_{bd}_lowres_inter_cost_ex")(
        _ptr(fenc, o), _frame_stride(fenc), *[_ptr(r, o) for r in refs], lowres_stride, rfs,
        mb_width, mb_height, n, me_method, subme, int(bool(satd)), me_range, mv_range, lam, _ptr(cm, c0),
        _ptr(intra_cost), _ptr(inv_qscale) if inv_qscale is not None else None, _ptr(mvs), _ptr(mvc), _ptr(lc),
        _ptr(rows), _ptr(est), None if ref_w is None else _ptr(ref_w, o), *w, n_slices, _stream()),
        "lowres_inter_cost")
    if check:
        lowres_status()
    return mvs, mvc, lc, rows, est


def lowres_bidir_cost(fenc, refs_a, refs_b, lowres_stride, mb_width, mb_height, cost_mv_center, search,
                      mvs0, costs0, mvs1, costs1, p1_mvs=None, dist_scale_factor=128, bipred_weight=32,
                      me_method=1, subme=4, satd=True, me_range=16, mv_range=512, lam=1, inv_qscale=None,
                      outs=None, a_frame_stride=None, b_frame_stride=None, n_slices=1, check=True):
    """The lookahead's B-frame costs (x264hip_*_lowres_bidir_cost_ex; n_slices lookahead slices) for
    the triplets (fenc[i],
    refs_a[*][i], refs_b[*][i]); a reference tensor with one frame and a frame stride of 0 serves
    the whole batch.  mvs_l int16 [n, mbs, 2] / costs_l int32 [n, mbs] are searched into (search
    bit l set) or read.  Returns (lowres_costs uint16-as-int16 [n, mbs], row_satd int32 [n, mbh],
    est int32 [n, 2]).  check as lowres_inter_cost."""
    import torch
    bd = _pix_bd(fenc)
    n = fenc.shape[0]
    nmb = mb_width * mb_height
    dev = fenc.device
    if outs is None:
        outs = (torch.empty((n, nmb), dtype=torch.int16, device=dev),
                torch.empty((n, mb_height), dtype=torch.int32, device=dev),
                torch.empty((n, 2), dtype=torch.int32, device=dev))
    lc, rows, est = outs
    cm, c0 = cost_mv_center
    o = PAD * lowres_stride + PAD
    afs = _frame_stride(*refs_a) if a_frame_stride is None else a_frame_stride
    bfs = _frame_stride(*refs_b) if b_frame_stride is None else b_frame_stride
    _rc(getattr(lib(), f"x264hip_{bd}_lowres_bidir_cost_ex")(
        _ptr(fenc, o), _frame_stride(fenc), *[_ptr(r, o) for r in refs_a], afs, *[_ptr(r, o) for r in refs_b], bfs,
        lowres_stride, mb_width, mb_height, n, me_method, subme, int(bool(satd)), me_range, mv_range, lam,
        _ptr(cm, c0), search, _ptr(mvs0), _ptr(costs0), _ptr(mvs1), _ptr(costs1),
        _ptr(p1_mvs) if p1_mvs is not None else None, dist_scale_factor, bipred_weight,
        _ptr(inv_qscale) if inv_qscale is not None else None, _ptr(lc), _ptr(rows), _ptr(est), n_slices,
        _stream()), "lowres_bidir_cost")
    if check:
        lowres_status()
    return lc, rows, est


class Weight(_c.Structure):
    """x264hip_weight_t: x264_weight_t as x264_weights_analyse leaves it (weighted = weightfn set)"""
    _fields_ = [("weighted", _c.c_int32), ("scale", _c.c_int32), ("denom", _c.c_int32), ("offset", _c.c_int32)]

    def tuple(self):
        return (self.weighted, self.scale, self.denom, self.offset)


WCOST_LUMA, WCOST_CHROMA420, WCOST_CHROMA422, WCOST_CHROMA444 = 0, 1, 2, 3


def _plane_ptr(t, origin):
    return None if t is None else _ptr(t, origin)


def ssim_wxh(pix1, origin1, stride1, pix2, origin2, stride2, width, height):
    """x264_pixel_ssim_wxh (x264hip_*_ssim_wxh): (ssim float, cnt); planes with the region's
    top-left at element origin1 / origin2"""
    import torch
    bd = _pix_bd(pix1)
    out = torch.empty(1, dtype=torch.float32, device=pix1.device)
    cnt = _c.c_int(0)
    f = getattr(lib(), f"x264hip_{bd}_ssim_wxh")
    f.argtypes = [_P, _IP, _P, _IP, _c.c_int, _c.c_int, _P, _P, _P]
    _rc(f(_ptr(pix1, origin1), stride1, _ptr(pix2, origin2), stride2, width, height, _ptr(out), _c.byref(cnt),
          _stream()), "ssim_wxh")
    return float(out.item()), cnt.value


def ssim_encoder_bands(mb_height, height, slices=None):
    """the (first row, height) of every band the encoder measures SSIM on (encoder.c:2412-2420,
    2490, 2516-2528: fdec_filter_row per MB row of each thread slice [start, end), relative to
    plane + 2), int32 [n, 2]; slices defaults to one slice [0, mb_height)"""
    import numpy as np
    out = []
    for start, end in (slices or [(0, mb_height)]):
        for mb_y in range(start + 1, end + 1):
            min_y = mb_y - 1
            b_start, b_end = min_y == start, mb_y == end
            minpix = min_y * 16 - 4 * (not b_start)
            maxpix = min(mb_y * 16 - 4 * (not b_end), height)
            minpix += 2 if b_start else -6
            out.append((minpix, maxpix - minpix))
    return np.array(out, np.int32).reshape(-1, 2)


def ssim_bands(pix1, origin1, stride1, pix2, origin2, stride2, width, bands, out=None):
    """x264hip_*_ssim_bands: every band's x264_pixel_ssim_wxh float of every frame pair, float32
    tensor [n_frames, n_bands]; pix* [n, rows, stride] tensors, origin* = element offset of the
    bands' left column at row 0 (plane (2, 0) as the encoder passes it), bands = int32 tensor
    [n_bands, 2] on the device (ssim_encoder_bands)"""
    import torch
    bd = _pix_bd(pix1)
    nf = pix1.shape[0] if pix1.dim() == 3 else 1
    nb = bands.shape[0]
    if out is None:
        out = torch.empty((nf, nb), dtype=torch.float32, device=pix1.device)
    f = getattr(lib(), f"x264hip_{bd}_ssim_bands")
    f.argtypes = [_P, _IP, _IP, _P, _IP, _IP, _c.c_int, _P, _c.c_int, _c.c_int, _P, _P]
    f1 = pix1.stride(0) if pix1.dim() == 3 else 0
    f2 = pix2.stride(0) if pix2.dim() == 3 else 0
    _rc(f(_ptr(pix1, origin1), stride1, f1, _ptr(pix2, origin2), stride2, f2, width, _ptr(bands), nb, nf, _ptr(out),
          _stream()), "ssim_bands")
    return out


def frame_pixel_stats(luma, luma_origin, luma_stride, mb_width, mb_height, chroma_format=0, chroma_u=None,
                      chroma_v=None, chroma_origin=0, chroma_stride=0, out=None):
    """fenc->i_pixel_sum / i_pixel_ssd of one frame (x264hip_*_frame_pixel_stats): int64 tensor [6] =
    sum[0..2], ssd[0..2] (uint64 bit patterns).  chroma_u = the NV12 / NV16 plane for 4:2:0 / 4:2:2."""
    import torch
    bd = _pix_bd(luma)
    if out is None:
        out = torch.empty(6, dtype=torch.int64, device=luma.device)
    f = getattr(lib(), f"x264hip_{bd}_frame_pixel_stats")
    f.argtypes = [_P, _IP, _P, _P, _IP, _c.c_int, _c.c_int, _c.c_int, _P, _P]
    _rc(f(_ptr(luma, luma_origin), luma_stride, _plane_ptr(chroma_u, chroma_origin),
          _plane_ptr(chroma_v, chroma_origin), chroma_stride, mb_width, mb_height, chroma_format, _ptr(out),
          _stream()), "frame_pixel_stats")
    return out


def _weights(cands):
    arr = (Weight * max(1, len(cands)))()
    for i, c in enumerate(cands):
        arr[i] = Weight(*[int(v) for v in c])
    return arr


def weight_cost_batch(kind, fenc, refs, origin, stride, mb_width, mb_height, cands, intra_cost=None, mvs=None,
                      satd=True, plane=0, lam=1, n_slices=1, out=None):
    """weight_cost_luma / _chroma / _chroma444 (slicetype.c:191-282) of every (weighted, scale, denom,
    offset) in cands (x264hip_*_weight_cost_batch): uint32-as-int32 tensor [n].  fenc / refs = planes
    with pixel (0,0) at element `origin` (refs: the four lowres planes for WCOST_LUMA with mvs, else one)."""
    import torch
    bd = _pix_bd(fenc)
    n = len(cands)
    if out is None:
        out = torch.empty(max(1, n), dtype=torch.int32, device=fenc.device)
    rp = (_P * 4)(*([r.data_ptr() + origin * r.element_size() for r in refs] + [None] * (4 - len(refs))))
    f = getattr(lib(), f"x264hip_{bd}_weight_cost_batch")
    f.argtypes = [_c.c_int, _P, _P, _IP, _c.c_int, _c.c_int, _P, _P, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _P,
                  _c.c_int, _P, _P]
    _rc(f(kind, _ptr(fenc, origin), rp, stride, mb_width, mb_height,
          None if intra_cost is None else _ptr(intra_cost), None if mvs is None else _ptr(mvs), int(bool(satd)),
          plane, lam, n_slices, _weights(cands), n, _ptr(out), _stream()), "weight_cost_batch")
    return out[:n]


def weights_analyse(fenc_lowres, ref_lowres, lowres_stride, mb_width, mb_height, intra_cost, fenc_stats,
                    ref_stats, mvs=None, chroma_format=0, fenc_chroma=(None, None), ref_chroma=(None, None),
                    chroma_origin=0, chroma_stride=0, b_lookahead=True, subme=7, satd=True, lam=1, n_slices=1,
                    weightp_fake=False, weighted_lowres=None):
    """x264_weights_analyse (x264hip_*_weights_analyse; synchronous).  Lowres planes are single frames
    [rows, stride] with (0,0) at (PAD, PAD); ref_lowres = the four planes (F, H, V, C); chroma planes
    have (0,0) at chroma_origin.  fenc_stats / ref_stats = (sum [3], ssd [3]) host ints.  Returns
    (weights [(weighted, scale, denom, offset)] * 3, cost_delta or None); weighted_lowres (a plane
    like ref_lowres[0]) receives fenc->weighted[0] in the lookahead when a luma weight is found."""
    bd = _pix_bd(fenc_lowres)
    o = PAD * lowres_stride + PAD
    rl = (_P * 4)(*[r.data_ptr() + o * r.element_size() for r in ref_lowres])
    fc = (_P * 2)(*[None if t is None else t.data_ptr() + chroma_origin * t.element_size() for t in fenc_chroma])
    rc = (_P * 2)(*[None if t is None else t.data_ptr() + chroma_origin * t.element_size() for t in ref_chroma])
    fsum = (_c.c_uint32 * 3)(*[int(v) & 0xFFFFFFFF for v in fenc_stats[0]])
    fssd = (_c.c_uint64 * 3)(*[int(v) & 0xFFFFFFFFFFFFFFFF for v in fenc_stats[1]])
    rsum = (_c.c_uint32 * 3)(*[int(v) & 0xFFFFFFFF for v in ref_stats[0]])
    rssd = (_c.c_uint64 * 3)(*[int(v) & 0xFFFFFFFFFFFFFFFF for v in ref_stats[1]])
    w = (Weight * 3)()
    cd = _c.c_float(-1.0)
    f = getattr(lib(), f"x264hip_{bd}_weights_analyse")
    f.argtypes = [_P, _P, _IP, _c.c_int, _c.c_int, _P, _P, _c.c_int, _P, _P, _IP, _P, _P, _P, _P, _c.c_int,
                  _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _P, _P, _P, _P]
    _rc(f(_ptr(fenc_lowres, o), rl, lowres_stride, mb_width, mb_height, _ptr(intra_cost),
          None if mvs is None else _ptr(mvs), chroma_format, fc, rc, chroma_stride, fsum, fssd, rsum, rssd,
          int(bool(b_lookahead)), subme, int(bool(satd)), lam, n_slices, int(bool(weightp_fake)),
          None if weighted_lowres is None else _ptr(weighted_lowres, o), w, _c.byref(cd), _stream()),
        "weights_analyse")
    return [w[i].tuple() for i in range(3)], (None if cd.value == -1.0 else cd.value)


def lowres_status():
    """Wait for the current stream; raise if a lookahead launch of this thread on its device
    timed out in the band wavefront (x264hip_lowres_status; reporting clears it)."""
    f = lib().x264hip_lowres_status
    f.argtypes, f.restype = [_P], _c.c_int
    _rc(f(_stream()), "lowres_status")


def plane_stride(width, pad=PAD):
    """x264-style stride of a padded plane: width + 2*pad rounded up to 64 pixels."""
    return (width + 2 * pad + 63) // 64 * 64


class MeBinding:
    """A thread's lookup-mode binding (x264hip_{8,10}_me_bind): keeps the host planes and
    table alive; ``close()`` (or leaving the ``with`` block) unbinds."""

    def __init__(self, arrays):
        self._arrays = arrays

    def stats(self, reset=False):
        h, m = _c.c_uint64(), _c.c_uint64()
        lib().x264hip_me_bind_stats(_c.byref(h), _c.byref(m), int(reset))
        return h.value, m.value

    def close(self):
        lib().x264hip_me_unbind()
        self._arrays = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def me_bind(bitdepth, fenc, fenc_origin, ref, ref_origin, stride, mb_width, mb_height, table, rng, table8=None):
    """Bind one frame pair's full-search tables for the calling thread's SAD table entries
    (lookup mode, include/x264hip.h x264hip_me_bind_tables).  fenc / ref: host numpy planes
    (uint8 / uint16) with pixel (0,0) at element offset *_origin; table: the me_search_full
    table of that pair, table8: its me_search_full8 quadrant tables (either may be None;
    numpy or torch, copied to host if on the device)."""
    def host(t, dt, n, name):
        if t is None:
            return None
        if hasattr(t, "cpu"):
            t = t.cpu().numpy()
        t = np.ascontiguousarray(t).view(dt)
        if t.size < n:
            raise ValueError("me_bind: %s smaller than its [mbh, mbw, ...] shape" % name)
        return t
    fenc = np.ascontiguousarray(fenc)
    ref = np.ascontiguousarray(ref)
    pt = np.uint8 if bitdepth == 8 else np.uint16
    st = np.uint16 if bitdepth == 8 else np.uint32
    fenc, ref = fenc.view(pt), ref.view(pt)
    n1 = mb_width * mb_height * (2 * rng + 1) * me_table_pitch(rng)
    table = host(table, st, n1, "table")
    table8 = host(table8, np.uint16, 4 * n1, "table8")
    es = fenc.itemsize
    rc = getattr(lib(), f"x264hip_{bitdepth}_me_bind_tables")(
        _c.c_void_p(fenc.ctypes.data + fenc_origin * es), _c.c_void_p(ref.ctypes.data + ref_origin * es), stride,
        mb_width, mb_height, None if table is None else _c.c_void_p(table.ctypes.data),
        None if table8 is None else _c.c_void_p(table8.ctypes.data), rng)
    _rc(rc, "me_bind")
    return MeBinding((fenc, ref, table, table8))


def trim(device=-1):
    """Release the idle blocks of the library's scratch pools (x264hip_trim)."""
    _rc(lib().x264hip_trim(device), "trim")


def me_table_pitch(rng):
    """row pitch of a full-search table: 2*range+1 rounded up to a multiple of 4"""
    return (2 * rng + 1 + 3) // 4 * 4


def me_centred_pitch(bitdepth, rng):
    """row pitch (= columns) of a me_search_centred table: me.c's ESA window around the centre,
    2*range+6 (8 bit) / 2*range+4 (10 bit) columns rounded up to a multiple of 4"""
    return (2 * rng + (6 if bitdepth == 8 else 4) + 3) // 4 * 4


def me_search_full(fenc, fenc_origin, fenc_stride, ref, ref_origin, ref_stride, mb_width, mb_height,
                   nframes, rng=16, table=None, fenc_frame_stride=None, ref_frame_stride=None):
    """Exhaustive 16x16 SAD table [nframes, mb_height, mb_width, 2r+1, pitch] (x264hip_*_me_search_full);
    pitch = align4(2r+1), entries [..., 2r+1:] are padding."""
    import torch
    bd = _pix_bd(fenc)
    w = 2 * rng + 1
    if table is None:
        table = torch.empty((nframes, mb_height, mb_width, w, me_table_pitch(rng)),
                            dtype=torch.int16 if bd == 8 else torch.int32, device=fenc.device)
    if table.numel() * table.element_size() < nframes * mb_height * mb_width * w * me_table_pitch(rng) * (
            2 if bd == 8 else 4):
        raise ValueError("me_search_full: table smaller than [nframes, mbh, mbw, 2r+1, pitch]")
    ffs = fenc_frame_stride if fenc_frame_stride is not None else (fenc[0].numel() if fenc.dim() == 3 else 0)
    rfs = ref_frame_stride if ref_frame_stride is not None else (ref[0].numel() if ref.dim() == 3 else 0)
    _rc(getattr(lib(), f"x264hip_{bd}_me_search_full")(
        _ptr(fenc, fenc_origin), fenc_stride, ffs, _ptr(ref, ref_origin), ref_stride, rfs,
        mb_width, mb_height, nframes, rng, _ptr(table), _stream()), "me_search_full")
    return table


def me_search_full8(fenc, fenc_origin, fenc_stride, ref, ref_origin, ref_stride, mb_width, mb_height,
                    nframes, rng=16, table8=None, fenc_frame_stride=None, ref_frame_stride=None):
    """8x8 quadrant SAD tables [nframes, mb_height, mb_width, 4, 2r+1, pitch] uint16-as-int16
    (x264hip_*_me_search_full8; q = 0 top-left, 1 top-right, 2 bottom-left, 3 bottom-right),
    8 and 10 bit."""
    import torch
    bd = _pix_bd(fenc)
    w = 2 * rng + 1
    shape = (nframes, mb_height, mb_width, 4, w, me_table_pitch(rng))
    if table8 is None:
        table8 = torch.empty(shape, dtype=torch.int16, device=fenc.device)
    if table8.numel() < int(np.prod(shape)) or table8.element_size() != 2 or not table8.is_contiguous():
        raise ValueError("me_search_full8: table8 must be a contiguous 16-bit tensor of %s" % (shape,))
    ffs = fenc_frame_stride if fenc_frame_stride is not None else (fenc[0].numel() if fenc.dim() == 3 else 0)
    rfs = ref_frame_stride if ref_frame_stride is not None else (ref[0].numel() if ref.dim() == 3 else 0)
    _rc(getattr(lib(), f"x264hip_{bd}_me_search_full8")(
        _ptr(fenc, fenc_origin), fenc_stride, ffs, _ptr(ref, ref_origin), ref_stride, rfs,
        mb_width, mb_height, nframes, rng, _ptr(table8), _stream()), "me_search_full8")
    return table8


def sub_dct_batch(kind, fenc, fenc_stride, fdec, fdec_stride, fenc_off, fdec_off, out=None):
    import torch
    bd = _pix_bd(fenc)
    n = fenc_off.numel()
    if out is None:
        out = torch.empty(n * DCT_OUT_SIZE[kind], dtype=torch.int16 if bd == 8 else torch.int32,
                          device=fenc.device)
    _rc(getattr(lib(), f"x264hip_{bd}_sub_dct_batch")(
        kind, _ptr(fenc), fenc_stride, _ptr(fdec), fdec_stride, _ptr(fenc_off), _ptr(fdec_off), n,
        _ptr(out), _stream()), "sub_dct_batch")
    return out


def _coef_bd(t):
    import torch
    if t.dtype == torch.int16:
        return 8
    if t.dtype == torch.int32:
        return 10
    raise TypeError("dctcoef tensors are int16 (8-bit) or int32 (10-bit)")


def dc_batch(kind, dct, dct4x4=None, n=None):
    bd = _coef_bd(dct)
    if n is None:
        n = dct.numel() // (16 if kind in (DC_4x4, DC_I4x4) else 8)
    _rc(getattr(lib(), f"x264hip_{bd}_dc_batch")(
        kind, _ptr(dct), _ptr(dct4x4) if dct4x4 is not None else None, n, _stream()), "dc_batch")
    return dct


def quant_batch(kind, dct, mf, bias, nz=None):
    import torch
    bd = _coef_bd(dct)
    n = dct.numel() // (64 if kind in (QUANT_8x8, QUANT_4x4x4) else 16)
    if nz is None:
        nz = torch.empty(n, dtype=torch.int32, device=dct.device)
    _rc(getattr(lib(), f"x264hip_{bd}_quant_batch")(
        kind, _ptr(dct), _ptr(mf), _ptr(bias), n, _ptr(nz), _stream()), "quant_batch")
    return nz


def quant_dc_batch(kind, dct, mf, bias, nz=None):
    import torch
    bd = _coef_bd(dct)
    n = dct.numel() // (16 if kind == QUANT_4x4_DC else 4)
    if nz is None:
        nz = torch.empty(n, dtype=torch.int32, device=dct.device)
    _rc(getattr(lib(), f"x264hip_{bd}_quant_dc_batch")(
        kind, _ptr(dct), int(mf), int(bias), n, _ptr(nz), _stream()), "quant_dc_batch")
    return nz


def mb_dct_quant(transform, fenc, fenc_origin, fenc_stride, pred, pred_origin, pred_stride,
                 mb_width, mb_height, nframes, mf, bias, dct=None, nz=None,
                 fenc_frame_stride=None, pred_frame_stride=None):
    """Fused residual transform + quant per MB (x264hip_*_mb_dct_quant)."""
    import torch
    bd = _pix_bd(fenc)
    nmb = nframes * mb_height * mb_width
    if dct is None:
        dct = torch.empty((nmb, 256), dtype=torch.int16 if bd == 8 else torch.int32, device=fenc.device)
    if nz is None:
        nz = torch.empty(nmb, dtype=torch.int32, device=fenc.device)
    ffs = fenc_frame_stride if fenc_frame_stride is not None else (fenc[0].numel() if fenc.dim() == 3 else 0)
    pfs = pred_frame_stride if pred_frame_stride is not None else (pred[0].numel() if pred.dim() == 3 else 0)
    _rc(getattr(lib(), f"x264hip_{bd}_mb_dct_quant")(
        transform, _ptr(fenc, fenc_origin), fenc_stride, ffs, _ptr(pred, pred_origin), pred_stride, pfs,
        mb_width, mb_height, nframes, _ptr(mf), _ptr(bias), _ptr(dct), _ptr(nz), _stream()), "mb_dct_quant")
    return dct, nz


def hpel_filter(planes, origin, stride, width, height, outs=None):
    """Half-pel planes (H, V, centre) of a stack of padded planes [n, height+64, stride]
    (x264hip_*_hpel_filter); returns three tensors of the same shape."""
    import torch
    bd = _pix_bd(planes)
    n = planes.shape[0] if planes.dim() == 3 else 1
    if outs is None:
        outs = [torch.zeros_like(planes) for _ in range(3)]
    fs = planes[0].numel() if planes.dim() == 3 else 0
    _rc(getattr(lib(), f"x264hip_{bd}_hpel_filter")(
        _ptr(planes, origin), _ptr(outs[0], origin), _ptr(outs[1], origin), _ptr(outs[2], origin), stride, fs,
        width, height, n, _stream()), "hpel_filter")
    return outs


def subpel_cmp_batch(op, i_pixel, fenc, fenc_stride, planes, ref_origin, ref_stride, fenc_off, qpel_xy, scores=None):
    """Quarter-pel candidate costs (x264hip_*_subpel_cmp_batch): planes = [fpel, H, V, C]
    tensors (same layout), qpel_xy int32 [n, 2] absolute quarter-pel positions."""
    import torch
    bd = _pix_bd(fenc)
    n = fenc_off.numel()
    if scores is None:
        scores = torch.empty(n, dtype=torch.int32, device=fenc.device)
    _rc(getattr(lib(), f"x264hip_{bd}_subpel_cmp_batch")(
        op, i_pixel, _ptr(fenc), fenc_stride, *[_ptr(p, ref_origin) for p in planes], ref_stride,
        _ptr(fenc_off), _ptr(qpel_xy), n, _ptr(scores), _stream()), "subpel_cmp_batch")
    return scores


def subpel_qpel9_batch(op, i_pixel, fenc, fenc_stride, planes, ref_origin, ref_stride, fenc_off, centre_xy,
                       scores=None):
    """The 3x3 quarter-pel neighbourhood of each block's centre (x264hip_*_subpel_qpel9_batch):
    centre_xy int32 [n, 2] quarter-pel positions; returns int32 [n, 9], index 3*(dy+1)+(dx+1)."""
    import torch
    bd = _pix_bd(fenc)
    n = fenc_off.numel()
    if scores is None:
        scores = torch.empty((n, 9), dtype=torch.int32, device=fenc.device)
    _rc(getattr(lib(), f"x264hip_{bd}_subpel_qpel9_batch")(
        op, i_pixel, _ptr(fenc), fenc_stride, *[_ptr(p, ref_origin) for p in planes], ref_stride,
        _ptr(fenc_off), _ptr(centre_xy), n, _ptr(scores), _stream()), "subpel_qpel9_batch")
    return scores


class RefineExt(_c.Structure):
    """x264hip_refine_ext_t: chroma ME and weighted references of me_refine_subpel_ex"""
    _fields_ = [("b_chroma_me", _c.c_int32), ("chroma_format", _c.c_int32), ("mvy_offset", _c.c_int32),
                ("weight", Weight * 3), ("fenc_chroma", _c.c_void_p * 2), ("fenc_chroma_stride", _c.c_ssize_t),
                ("fenc_chroma_frame_stride", _c.c_ssize_t), ("ref_chroma", _c.c_void_p * 8),
                ("ref_chroma_stride", _c.c_ssize_t), ("ref_chroma_frame_stride", _c.c_ssize_t)]


def refine_ext(b_chroma_me=0, chroma_format=1, mvy_offset=0, weights=(None, None, None), fenc_chroma=(),
               fenc_chroma_origin=0, fenc_chroma_stride=0, ref_chroma=(), ref_chroma_origin=0, ref_chroma_stride=0):
    """the x264hip_refine_ext_t of me_refine_subpel(ext=...): weights[p] = (scale, denom, offset)
    or None (m->weight[0..2]); fenc_chroma = [NV12 / NV16 tensor] or [U, V] (4:4:4), ref_chroma =
    [NV12 / NV16 tensor] or the F, H, V, C tensors of U then V ([n, rows, stride] each, the
    chroma (0,0) at *_origin).  Frame strides are the tensors' own."""
    e = RefineExt()
    e.b_chroma_me, e.chroma_format, e.mvy_offset = int(b_chroma_me), int(chroma_format), int(mvy_offset)
    for k, w in enumerate(weights):
        if w is not None:
            e.weight[k] = Weight(1, *[int(v) for v in w])
    for k, t in enumerate(fenc_chroma):
        e.fenc_chroma[k] = _ptr(t, fenc_chroma_origin).value
    for k, t in enumerate(ref_chroma):
        e.ref_chroma[k] = _ptr(t, ref_chroma_origin).value
    e.fenc_chroma_stride, e.ref_chroma_stride = fenc_chroma_stride, ref_chroma_stride
    if fenc_chroma:
        e.fenc_chroma_frame_stride = _frame_stride(*fenc_chroma)
    if ref_chroma:
        e.ref_chroma_frame_stride = _frame_stride(*ref_chroma)
    e._keep = (tuple(fenc_chroma), tuple(ref_chroma))    # the tensors outlive the call
    return e


def me_refine_subpel(fenc, fenc_origin, fenc_stride, planes, ref_origin, ref_stride, i_pixel, subme, pos, par,
                     init_cost, cost_mv_center, refine_qpel=False, fpel_satd=False, out=None, fenc_frame_stride=None,
                     ref_frame_stride=None, nevals=None, ext=None):
    """refine_subpel (encoder/me.c:865-992) of n partitions (x264hip_*_me_refine_subpel, or _ex
    with ext = refine_ext(...): chroma ME / weighted references): planes = [F, H, V, C] tensors
    of the references (hpel_filter's), pos int32 [n, 3] = (frame, x, y), par int16 [n, 8] = (mvx,
    mvy, mvp_x, mvp_y, mv_min_spel x, y, mv_max_spel x, y), init_cost int32 [n]; returns int32
    [n, 4] = (cost, mvx, mvy, cost_mv).  nevals: optional int32 [n] receiving the reference's cmp
    calls per partition (luma SADs | luma SATDs << 16 | chroma calls << 24)."""
    import torch
    bd = _pix_bd(fenc)
    n = pos.shape[0]
    if out is None:
        out = torch.empty((n, 4), dtype=torch.int32, device=fenc.device)
    ffs = fenc_frame_stride if fenc_frame_stride is not None else (fenc[0].numel() if fenc.dim() == 3 else 0)
    rfs = ref_frame_stride if ref_frame_stride is not None else _frame_stride(*planes)
    cm, c0 = cost_mv_center
    args = [_ptr(fenc, fenc_origin), fenc_stride, ffs, *[_ptr(p, ref_origin) for p in planes], ref_stride, rfs,
            i_pixel, subme, int(bool(refine_qpel)), int(bool(fpel_satd)), _ptr(pos), _ptr(par), _ptr(init_cost),
            _ptr(cm, c0), n, _ptr(out), _ptr(nevals) if nevals is not None else None]
    types = [_P, _IP, _IP, _P, _P, _P, _P, _IP, _IP, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _P, _P, _P, _P,
             _c.c_int, _P, _P]
    name = f"x264hip_{bd}_me_refine_subpel" + ("_ex" if ext is not None else "")
    if ext is not None:
        args.append(_c.byref(ext))
        types.append(_P)
    fn = getattr(lib(), name)
    fn.argtypes = types + [_P]
    fn.restype = _c.c_int
    _rc(fn(*args, _stream()), name)
    return out


def me_search_ref(fenc, fenc_origin, fenc_stride, fpel_w, planes, ref_origin, ref_stride, i_pixel, me_method, subme,
                  me_range, pos, par, mvc, cost_mv_center, out=None, fenc_frame_stride=None, ref_frame_stride=None,
                  nevals=None, ext=None, halfpel_thresh=None, ref_cost=None):
    """x264_me_search_ref (encoder/me.c:182-798) of n partitions (x264hip_*_me_search_ref): me_method
    0 DIA / 1 HEX / 2 UMH; fpel_w = the weighted F plane the integer search reads (m->p_fref_w, or
    planes[0]); planes = [F, H, V, C]; pos int32 [n, 3] = (frame, x, y); par int16 [n, 12] = (mvp
    x, y, mv_limit_fpel min x, y, max x, y, mv_min_spel x, y, mv_max_spel x, y, i_mvc, 0); mvc
    int16 [n, 14, 2]; ext = refine_ext(...) for chroma ME / weights.  Returns int32 [n, 4] =
    (m->cost, m->mv x, y, m->cost_mv); nevals: optional int32 [n, 2] (integer stage fpel | get_ref
    << 16, refine counts).  halfpel_thresh: int32 [n] p_halfpel_thresh per partition, read and
    written (x264hip_*_me_search_ref_thresh, me.c:931-944), with ref_cost int32 [n] or None (the
    i_ref_cost analyse.c:1271 / 1310 hold it less during the search); on the early exit
    out[i, 3] keeps what `out` held."""
    import torch
    bd = _pix_bd(fenc)
    n = pos.shape[0]
    if out is None:
        out = torch.empty((n, 4), dtype=torch.int32, device=fenc.device)
    ffs = fenc_frame_stride if fenc_frame_stride is not None else (fenc[0].numel() if fenc.dim() == 3 else 0)
    rfs = ref_frame_stride if ref_frame_stride is not None else _frame_stride(fpel_w, *planes)
    cm, c0 = cost_mv_center
    thr = halfpel_thresh is not None
    name = f"x264hip_{bd}_me_search_ref" + ("_thresh" if thr else "")
    fn = getattr(lib(), name)
    fn.argtypes = [_P, _IP, _IP, _P, _P, _P, _P, _P, _IP, _IP, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _P, _P, _P,
                   _P, _c.c_int, _P, _P] + ([_P, _P] if thr else []) + [_P, _P]
    fn.restype = _c.c_int
    extra = [_ptr(halfpel_thresh), _ptr(ref_cost) if ref_cost is not None else None] if thr else []
    _rc(fn(_ptr(fenc, fenc_origin), fenc_stride, ffs, _ptr(fpel_w, ref_origin), *[_ptr(p, ref_origin) for p in planes],
           ref_stride, rfs, i_pixel, me_method, subme, me_range, _ptr(pos), _ptr(par), _ptr(mvc), _ptr(cm, c0), n,
           _ptr(out), _ptr(nevals) if nevals is not None else None, *extra,
           _c.byref(ext) if ext is not None else None, _stream()), name)
    return out


def me_analyse_p16x16(fenc, fenc_origin, fenc_stride, fpel_w, planes, ref_origin, ref_stride, mb_width, mb_height,
                      nframes, me_method, subme, me_range, cost_mv_center, mv_range=512, lowres_mv=None, ref_mv=None,
                      ref_mv_scale=0, out=None, nevals=None, ext=None, fenc_frame_stride=None, ref_frame_stride=None):
    """x264's P16x16 reference-0 analysis of whole frames with mvpred.c's predictors
    (x264hip_*_me_analyse_p16x16): every MB searched in raster order's dependency (a wavefront of
    MB anti-diagonals) with mvp = x264_mb_predict_mv_16x16 and mvc = x264_mb_predict_mv_ref16x16.
    lowres_mv / ref_mv: int16 [nframes, mbs, 2] or None.  Returns int32 [nframes, mbs, 4] =
    (m->cost, mvx, mvy, cost_mv) in raster order."""
    import torch
    bd = _pix_bd(fenc)
    nmb = mb_width * mb_height
    if out is None:
        out = torch.empty((nframes, nmb, 4), dtype=torch.int32, device=fenc.device)
    ffs = fenc_frame_stride if fenc_frame_stride is not None else (fenc[0].numel() if fenc.dim() == 3 else 0)
    rfs = ref_frame_stride if ref_frame_stride is not None else _frame_stride(fpel_w, *planes)
    cm, c0 = cost_mv_center
    fn = getattr(lib(), f"x264hip_{bd}_me_analyse_p16x16")
    fn.argtypes = [_P, _IP, _IP, _P, _P, _P, _P, _P, _IP, _IP] + [_c.c_int] * 7 + [_P, _P, _c.c_int, _P, _P, _P, _P,
                                                                                   _P]
    fn.restype = _c.c_int
    _rc(fn(_ptr(fenc, fenc_origin), fenc_stride, ffs, _ptr(fpel_w, ref_origin), *[_ptr(p, ref_origin) for p in planes],
           ref_stride, rfs, mb_width, mb_height, nframes, me_method, subme, me_range, mv_range,
           _ptr(lowres_mv) if lowres_mv is not None else None, _ptr(ref_mv) if ref_mv is not None else None,
           ref_mv_scale, _ptr(cm, c0), _ptr(out), _ptr(nevals) if nevals is not None else None,
           _c.byref(ext) if ext is not None else None, _stream()), "me_analyse_p16x16")
    return out


def me_refine_bidir(fenc, fenc_origin, fenc_stride, planes0, planes1, ref_origin, ref_stride, i_pixel, pos, par,
                    weight, cost_mv_center, satd=True, out=None, cost=None, nevals=None, fenc_frame_stride=None,
                    ref_frame_stride=None):
    """x264_me_refine_bidir_satd (encoder/me.c:994-1183) of n bipred partitions
    (x264hip_*_me_refine_bidir_satd): planes0 / planes1 = [F, H, V, C] of the list 0 / 1
    references, pos int32 [n, 3] = (frame, x, y), par int16 [n, 12] = (m0 mv x, y, m1 mv x, y,
    m0 mvp x, y, m1 mvp x, y, mv_min_spel x, y, mv_max_spel x, y), weight int32 [n].  Returns
    int32 [n, 4] = (m0 mv x, y, m1 mv x, y); cost / nevals: optional int32 [n] outputs."""
    import torch
    bd = _pix_bd(fenc)
    n = pos.shape[0]
    if out is None:
        out = torch.empty((n, 4), dtype=torch.int32, device=fenc.device)
    ffs = fenc_frame_stride if fenc_frame_stride is not None else (fenc[0].numel() if fenc.dim() == 3 else 0)
    rfs = ref_frame_stride if ref_frame_stride is not None else _frame_stride(*planes0, *planes1)
    cm, c0 = cost_mv_center
    name = f"x264hip_{bd}_me_refine_bidir_satd"
    fn = getattr(lib(), name)
    fn.argtypes = [_P, _IP, _IP] + [_P] * 8 + [_IP, _IP, _c.c_int, _c.c_int, _P, _P, _P, _P, _c.c_int, _P, _P, _P, _P]
    fn.restype = _c.c_int
    _rc(fn(_ptr(fenc, fenc_origin), fenc_stride, ffs, *[_ptr(p, ref_origin) for p in planes0],
           *[_ptr(p, ref_origin) for p in planes1], ref_stride, rfs, i_pixel, int(bool(satd)), _ptr(pos), _ptr(par),
           _ptr(weight), _ptr(cm, c0), n, _ptr(out), _ptr(cost) if cost is not None else None,
           _ptr(nevals) if nevals is not None else None, _stream()), name)
    return out


def me_refine_qpel_refdupe(fenc, fenc_origin, fenc_stride, planes, ref_origin, ref_stride, i_pixel, subme, pos, par,
                           init_cost, cost_mv_center, halfpel_thresh=None, ref_cost=None, fpel_satd=False, out=None,
                           fenc_frame_stride=None, ref_frame_stride=None, nevals=None, ext=None):
    """x264_me_refine_qpel_refdupe (encoder/me.c:812-815) of n partitions
    (x264hip_*_me_refine_qpel_refdupe): arguments as me_refine_subpel (par's mv = reference 0's
    result, init_cost = m->cost as the caller holds it), halfpel_thresh / ref_cost as
    me_search_ref."""
    import torch
    bd = _pix_bd(fenc)
    n = pos.shape[0]
    if out is None:
        out = torch.empty((n, 4), dtype=torch.int32, device=fenc.device)
    ffs = fenc_frame_stride if fenc_frame_stride is not None else (fenc[0].numel() if fenc.dim() == 3 else 0)
    rfs = ref_frame_stride if ref_frame_stride is not None else _frame_stride(*planes)
    cm, c0 = cost_mv_center
    name = f"x264hip_{bd}_me_refine_qpel_refdupe"
    fn = getattr(lib(), name)
    fn.argtypes = [_P, _IP, _IP, _P, _P, _P, _P, _IP, _IP, _c.c_int, _c.c_int, _c.c_int, _P, _P, _P, _P, _c.c_int,
                   _P, _P, _P, _P, _P, _P]
    fn.restype = _c.c_int
    _rc(fn(_ptr(fenc, fenc_origin), fenc_stride, ffs, *[_ptr(p, ref_origin) for p in planes], ref_stride, rfs, i_pixel,
           subme, int(bool(fpel_satd)), _ptr(pos), _ptr(par), _ptr(init_cost), _ptr(cm, c0), n, _ptr(out),
           _ptr(nevals) if nevals is not None else None,
           _ptr(halfpel_thresh) if halfpel_thresh is not None else None,
           _ptr(ref_cost) if ref_cost is not None else None, _c.byref(ext) if ext is not None else None, _stream()),
        name)
    return out


def me_esa_argmin(table, rng, me_range, par, init_cost, cost_mv_center, out=None, origin=None):
    """ESA decision per MB over a full-search table (x264hip_*_me_esa_argmin, or
    x264hip_*_me_esa_argmin_at when `origin` [n, 2] int16 from me_search_centred is given).
    par int16 [n, 8], init_cost int32 [n], cost_mv_center: (uint16-as-int16 tensor, element
    offset of mvd 0).  Returns int32 [n, 3] = (cost, mx, my)."""
    import torch
    bd = 8 if table.dtype == torch.int16 else 10
    n = par.shape[0]
    if out is None:
        out = torch.empty((n, 3), dtype=torch.int32, device=table.device)
    cm, c0 = cost_mv_center
    if origin is None:
        _rc(getattr(lib(), f"x264hip_{bd}_me_esa_argmin")(
            _ptr(table), rng, n, me_range, _ptr(par), _ptr(init_cost), _ptr(cm, c0), _ptr(out), _stream()),
            "me_esa_argmin")
    else:
        _rc(getattr(lib(), f"x264hip_{bd}_me_esa_argmin_at")(
            _ptr(table), rng, n, me_range, _ptr(origin), _ptr(par), _ptr(init_cost), _ptr(cm, c0), _ptr(out),
            _stream()), "me_esa_argmin_at")
    return out


def me_search_centred(fenc, fenc_origin, fenc_stride, ref, ref_origin, ref_stride, mb_width, mb_height, nframes,
                      rng, centre, table=None, origin=None, fenc_frame_stride=None, ref_frame_stride=None):
    """Full search of me.c's ESA window around per-MB centres (x264hip_*_me_search_centred):
    centre int16 [n_mbs, 2]; returns (table [nframes, mbh, mbw, 2r+1, me_centred_pitch(bd, r)],
    origin int16 [n_mbs, 2])."""
    import torch
    bd = _pix_bd(fenc)
    w = 2 * rng + 1
    if table is None:
        table = torch.empty((nframes, mb_height, mb_width, w, me_centred_pitch(bd, rng)),
                            dtype=torch.int16 if bd == 8 else torch.int32, device=fenc.device)
    if origin is None:
        origin = torch.empty((nframes * mb_height * mb_width, 2), dtype=torch.int16, device=fenc.device)
    ffs = fenc_frame_stride if fenc_frame_stride is not None else (fenc[0].numel() if fenc.dim() == 3 else 0)
    rfs = ref_frame_stride if ref_frame_stride is not None else (ref[0].numel() if ref.dim() == 3 else 0)
    _rc(getattr(lib(), f"x264hip_{bd}_me_search_centred")(
        _ptr(fenc, fenc_origin), fenc_stride, ffs, _ptr(ref, ref_origin), ref_stride, rfs, mb_width, mb_height,
        nframes, rng, _ptr(centre), _ptr(table), _ptr(origin), _stream()), "me_search_centred")
    return table, origin


def me_tesa(fenc, fenc_origin, fenc_stride, ref, ref_origin, ref_stride, integral, mb_width, mb_height, nframes,
            me_range, par, init_cost, cost_mv_center, satd=True, table=None, rng=0, origin=None, out=None,
            fenc_frame_stride=None, ref_frame_stride=None, integral_origin=None):
    """TESA integer-pel decision per 16x16 MB (x264hip_*_me_tesa, reference encoder/me.c:653-748).

    integral: frame_integral() output [n, rows, ref_stride] (its (0,0) at integral_origin, default
    PAD*stride+PAD); par int16 [n_mbs, 8], init_cost int32 [n_mbs], cost_mv_center as me_esa_argmin;
    table / rng / origin: an optional me_search_full / me_search_centred table of the same pairs.
    Returns int32 [n_mbs, 4] = (cost, mx, my, number of COST_MV candidates)."""
    import torch
    bd = _pix_bd(fenc)
    n = par.shape[0]
    if out is None:
        out = torch.empty((n, 4), dtype=torch.int32, device=fenc.device)
    ffs = fenc_frame_stride if fenc_frame_stride is not None else (fenc[0].numel() if fenc.dim() == 3 else 0)
    rfs = ref_frame_stride if ref_frame_stride is not None else (ref[0].numel() if ref.dim() == 3 else 0)
    io = integral_origin if integral_origin is not None else PAD * ref_stride + PAD
    cm, c0 = cost_mv_center
    _rc(getattr(lib(), f"x264hip_{bd}_me_tesa")(
        _ptr(fenc, fenc_origin), fenc_stride, ffs, _ptr(ref, ref_origin), ref_stride, rfs, _ptr(integral, io),
        integral[0].numel() if integral.dim() == 3 else 0, mb_width, mb_height, nframes, me_range, int(bool(satd)),
        _ptr(table) if table is not None else None, rng, _ptr(origin) if origin is not None else None, _ptr(par),
        _ptr(init_cost), _ptr(cm, c0), _ptr(out), _stream()), "me_tesa")
    return out


def _plane_ssd(name, nv12, pix1, origin1, stride1, pix2, origin2, stride2, width, height, nframes, out,
               frame_stride1, frame_stride2):
    import torch
    bd = _pix_bd(pix1)
    if out is None:
        out = torch.empty((nframes, 2) if nv12 else (nframes,), dtype=torch.int64, device=pix1.device)
    f1 = frame_stride1 if frame_stride1 is not None else (pix1[0].numel() if pix1.dim() == 3 else 0)
    f2 = frame_stride2 if frame_stride2 is not None else (pix2[0].numel() if pix2.dim() == 3 else 0)
    _rc(getattr(lib(), f"x264hip_{bd}_{name}")(
        _ptr(pix1, origin1), stride1, f1, _ptr(pix2, origin2), stride2, f2, width, height, nframes, _ptr(out),
        _stream()), name)
    return out


def ssd_plane_batch(pix1, origin1, stride1, pix2, origin2, stride2, width, height, nframes, out=None,
                    frame_stride1=None, frame_stride2=None):
    """x264_pixel_ssd_wxh per frame pair (x264hip_*_ssd_plane_batch, pixel.c:112-151): int64 [n]
    (uint64 values)."""
    return _plane_ssd("ssd_plane_batch", False, pix1, origin1, stride1, pix2, origin2, stride2, width, height,
                      nframes, out, frame_stride1, frame_stride2)


def ssd_nv12_batch(pix1, origin1, stride1, pix2, origin2, stride2, width, height, nframes, out=None,
                   frame_stride1=None, frame_stride2=None):
    """x264_pixel_ssd_nv12 per frame pair (x264hip_*_ssd_nv12_batch, pixel.c:153-178): int64 [n, 2] =
    (ssd_u, ssd_v); width = chroma samples per row."""
    return _plane_ssd("ssd_nv12_batch", True, pix1, origin1, stride1, pix2, origin2, stride2, width, height,
                      nframes, out, frame_stride1, frame_stride2)


def me_search_esa8(fenc, fenc_origin, fenc_stride, ref, ref_origin, ref_stride, mb_width, mb_height, nframes, rng,
                   me_range, centre, par, init_cost, cost_mv_center, out=None, fenc_frame_stride=None,
                   ref_frame_stride=None):
    """ESA decisions of every MB's eight sub-partitions (x264hip_*_me_search_esa8; 16x8 top /
    bottom, 8x16 left / right, 8x8 TL / TR / BL / BR at index 8*mb + p): par int16 [8*n_mbs, 8],
    init_cost int32 [8*n_mbs], centre int16 [n_mbs, 2] (the shared template's centre, None =
    mv 0), rng the template radius (0 = direct SADs only).  Returns int32 [8*n_mbs, 3]."""
    import torch
    bd = _pix_bd(fenc)
    n = par.shape[0]
    if out is None:
        out = torch.empty((n, 3), dtype=torch.int32, device=fenc.device)
    ffs = fenc_frame_stride if fenc_frame_stride is not None else (fenc[0].numel() if fenc.dim() == 3 else 0)
    rfs = ref_frame_stride if ref_frame_stride is not None else (ref[0].numel() if ref.dim() == 3 else 0)
    cm, c0 = cost_mv_center
    fn = getattr(lib(), f"x264hip_{bd}_me_search_esa8")
    fn.argtypes = [_P, _IP, _IP, _P, _IP, _IP, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _P, _P, _P, _P,
                   _P, _P]
    fn.restype = _c.c_int
    _rc(fn(_ptr(fenc, fenc_origin), fenc_stride, ffs, _ptr(ref, ref_origin), ref_stride, rfs, mb_width, mb_height,
           nframes, rng, me_range, None if centre is None else _ptr(centre), _ptr(par), _ptr(init_cost),
           _ptr(cm, c0), _ptr(out), _stream()), "me_search_esa8")
    return out


def me_search_esa(fenc, fenc_origin, fenc_stride, ref, ref_origin, ref_stride, mb_width, mb_height, nframes, rng,
                  me_range, par, init_cost, cost_mv_center, out=None, fenc_frame_stride=None, ref_frame_stride=None):
    """Fused full search around each MB's predictor + ESA decision (x264hip_*_me_search_esa):
    the result of me_search_centred(centre = par[:, :2]) followed by me_esa_argmin(origin=...),
    without the table.  Returns int32 [n, 3] = (cost, mx, my)."""
    import torch
    bd = _pix_bd(fenc)
    n = par.shape[0]
    if out is None:
        out = torch.empty((n, 3), dtype=torch.int32, device=fenc.device)
    ffs = fenc_frame_stride if fenc_frame_stride is not None else (fenc[0].numel() if fenc.dim() == 3 else 0)
    rfs = ref_frame_stride if ref_frame_stride is not None else (ref[0].numel() if ref.dim() == 3 else 0)
    cm, c0 = cost_mv_center
    fn = getattr(lib(), f"x264hip_{bd}_me_search_esa")
    fn.argtypes = [_P, _IP, _IP, _P, _IP, _IP, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _P, _P, _P, _P, _P]
    fn.restype = _c.c_int
    _rc(fn(_ptr(fenc, fenc_origin), fenc_stride, ffs, _ptr(ref, ref_origin), ref_stride, rfs, mb_width, mb_height,
           nframes, rng, me_range, _ptr(par), _ptr(init_cost), _ptr(cm, c0), _ptr(out), _stream()), "me_search_esa")
    return out
