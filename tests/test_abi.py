"""CPU: the C ABI boundary.

* libx264hip.so loads and exports every function include/x264hip.h declares;
* the re-declared tables have the reference's field order and layout (checked
  by compiling the header with gcc and comparing with the ctypes mirror);
* the host-side CQM restatement in the product equals the oracle's.
No kernel is launched (no GPU in this container)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT, ensure_built, load_package

HEADER = os.path.join(ROOT, "include", "x264hip.h")


def declared_functions():
    src = open(HEADER).read()
    names = set()
    # per-bit-depth entries inside X264HIP_DECLARE_ENTRIES
    m = re.search(r"#define X264HIP_DECLARE_ENTRIES(.*?)\n\n", src, re.S)
    for n in re.findall(r"\bx264hip_##BD##_(\w+)\s*\(", m.group(1)):
        for bd in (8, 10):
            names.add(f"x264hip_{bd}_{n}")
    # plain prototypes outside the macros
    body = re.sub(r"#define X264HIP_DECLARE_\w+.*?\n\n", "", src, flags=re.S)
    for n in re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(x264hip_\w+)\s*\(", body, re.M):
        names.add(n)
    return sorted(names)


def test_header_declares_entries():
    names = declared_functions()
    assert "x264hip_init" in names and "x264hip_8_me_search_full" in names
    assert "x264hip_10_pixel_init" in names and "x264hip_8_quant_init_hip" in names
    assert len(names) >= 30


def test_library_exports_every_declared_symbol():
    so = ensure_built("hip")
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing


def test_library_loads_and_resolves():
    x = load_package()
    L = x.lib()
    for n in declared_functions():
        assert getattr(L, n) is not None


def test_library_is_gfx950_code():
    so = ensure_built("hip")
    out = subprocess.run(["strings", so], capture_output=True, text=True).stdout
    assert "gfx950" in out


_PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include "x264hip.h"
#define P(T, F) printf(#T " " #F " %zu\n", offsetof(T, F));
int main(void) {
    printf("pixel8 %zu\npixel10 %zu\ndct8 %zu\ndct10 %zu\nquant8 %zu\nquant10 %zu\n",
           sizeof(x264hip_8_pixel_function_t), sizeof(x264hip_10_pixel_function_t),
           sizeof(x264hip_8_dct_function_t), sizeof(x264hip_10_dct_function_t),
           sizeof(x264hip_8_quant_function_t), sizeof(x264hip_10_quant_function_t));
    P(x264hip_8_pixel_function_t, sad_x3) P(x264hip_8_pixel_function_t, satd_x4)
    P(x264hip_8_pixel_function_t, ads) P(x264hip_8_pixel_function_t, intra_sad_x9_8x8)
    P(x264hip_8_dct_function_t, sub16x16_dct8) P(x264hip_8_dct_function_t, dct2x4dc)
    P(x264hip_8_quant_function_t, quant_2x2_dc) P(x264hip_8_quant_function_t, coeff_level_run)
    P(x264hip_8_quant_function_t, trellis_cabac_chroma_422_dc)
    printf("zigzag8 %zu\nzigzag10 %zu\nrunlevel8 %zu\nrunlevel10 %zu\n",
           sizeof(x264hip_8_zigzag_function_t), sizeof(x264hip_10_zigzag_function_t),
           sizeof(x264hip_8_run_level_t), sizeof(x264hip_10_run_level_t));
    P(x264hip_8_zigzag_function_t, sub_4x4ac) P(x264hip_8_run_level_t, level) P(x264hip_10_run_level_t, level)
    return 0;
}
"""


def test_table_layout_matches_ctypes(tmp_path):
    c = tmp_path / "probe.c"
    c.write_text(_PROBE)
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe)], check=True)
    lines = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    vals = {}
    for ln in lines:
        if ln:
            *k, v = ln.split()
            vals[" ".join(k)] = int(v)
    x = load_package()
    assert vals["pixel8"] == vals["pixel10"] == ctypes.sizeof(x.PixelFunctions)
    assert vals["dct8"] == vals["dct10"] == ctypes.sizeof(x.DctFunctions)
    assert vals["quant8"] == vals["quant10"] == ctypes.sizeof(x.QuantFunctions)
    assert vals["x264hip_8_pixel_function_t sad_x3"] == x.PixelFunctions.sad_x3.offset
    assert vals["x264hip_8_pixel_function_t satd_x4"] == x.PixelFunctions.satd_x4.offset
    assert vals["x264hip_8_pixel_function_t ads"] == x.PixelFunctions.ads.offset
    assert vals["x264hip_8_pixel_function_t intra_sad_x9_8x8"] == x.PixelFunctions.intra_sad_x9_8x8.offset
    assert vals["x264hip_8_dct_function_t sub16x16_dct8"] == x.DctFunctions.sub16x16_dct8.offset
    assert vals["x264hip_8_dct_function_t dct2x4dc"] == x.DctFunctions.dct2x4dc.offset
    assert vals["x264hip_8_quant_function_t quant_2x2_dc"] == x.QuantFunctions.quant_2x2_dc.offset
    assert vals["x264hip_8_quant_function_t coeff_level_run"] == x.QuantFunctions.coeff_level_run.offset
    assert vals["zigzag8"] == vals["zigzag10"] == ctypes.sizeof(x.ZigzagFunctions) == 6 * 8
    assert vals["x264hip_8_zigzag_function_t sub_4x4ac"] == x.ZigzagFunctions.sub_4x4ac.offset
    # x264_run_level_t (bitstream.h:50-55): level 16-byte aligned after last / mask
    assert vals["x264hip_8_run_level_t level"] == vals["x264hip_10_run_level_t level"] == 16
    assert vals["runlevel8"] == 64 and vals["runlevel10"] == 96
    # reference field counts: pixel.h:78-144 has 8*8+7+4+2*7+... pointers
    n_ptr = vals["pixel8"] // 8
    assert n_ptr == 8 * 7 + 7 + 4 + 7 * 2 + 1 + 1 + 1 + 4 + 4 + 4 + 3 + 7 * 4 + 7 + 15 + 3 + 6


def _prefilled(struct):
    """A table whose every pointer slot holds a recognisable non-NULL value, as if the
    caller's C init (x264_*_init) had filled it."""
    tab = struct()
    raw = (ctypes.c_uint64 * (ctypes.sizeof(struct) // 8)).from_buffer(tab)
    for i in range(len(raw)):
        raw[i] = 0x5EED0000 + i
    return tab, bytes(raw)


@pytest.mark.parametrize("kind", ["pixel", "dct", "quant", "zigzag"])
@pytest.mark.parametrize("bd", [8, 10])
def test_init_leaves_caller_table_untouched_without_device(kind, bd):
    """No gfx950 device here: neither the flag form (with and without X264HIP_CPU_HIP) nor
    the _init_hip form may change a table the caller's C init filled (the OpenCL
    fallback convention, reference common/opencl.c:400-409; every used entry stays
    non-NULL, encoder/encoder.c:1419-1422)."""
    x = load_package()
    L = x.lib()
    if L.x264hip_available():
        pytest.skip("a gfx950 device is visible")
    struct = {"pixel": x.PixelFunctions, "dct": x.DctFunctions, "quant": x.QuantFunctions,
              "zigzag": x.ZigzagFunctions}[kind]
    tab, before = _prefilled(struct)
    tab2, before2 = _prefilled(struct)
    init = getattr(L, f"x264hip_{bd}_{kind}_init")
    init_hip = getattr(L, f"x264hip_{bd}_{kind}_init_hip")
    for cpu in (0, x.CPU_HIP):
        if kind == "quant":
            init(None, cpu, ctypes.byref(tab))
        elif kind == "zigzag":
            init(cpu, ctypes.byref(tab), ctypes.byref(tab2))
        else:
            init(cpu, ctypes.byref(tab))
    if kind == "zigzag":
        init_hip(ctypes.byref(tab), ctypes.byref(tab2))
    else:
        init_hip(ctypes.byref(tab))
    assert bytes((ctypes.c_uint64 * (ctypes.sizeof(struct) // 8)).from_buffer(tab)) == before
    assert bytes((ctypes.c_uint64 * (ctypes.sizeof(struct) // 8)).from_buffer(tab2)) == before2


def test_runtime_entries_without_device():
    """Runtime calls fail with a status, never abort, when no device exists."""
    x = load_package()
    L = x.lib()
    if L.x264hip_available():
        pytest.skip("a gfx950 device is visible")
    assert L.x264hip_init(0) == -3                        # X264HIP_ENODEV
    assert L.x264hip_set_thread_device(0) == -3
    assert L.x264hip_thread_device() == -1
    assert L.x264hip_set_thread_device(-1) == 0
    assert L.x264hip_set_variant(b"X264HIP_ME_XCD", 0) == 0
    assert L.x264hip_set_variant(b"X264HIP_ME_XCD", -1) == 0
    assert L.x264hip_set_variant(b"NOT_A_SWITCH", 1) == -1
    assert L.x264hip_set_variant(b"X264HIP_ME_VARIANT", 3) == -1          # removed: one kernel per input
    assert L.x264hip_forward_ref(None, 0, None, 0, 16, None) == -1
    assert L.x264hip_forward_ref(None, 0, None, 0, 0, None) == 0
    L.x264hip_upload.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    assert L.x264hip_upload(None, None, 16, None) == -1            # EINVAL before any HIP call
    assert L.x264hip_upload(None, None, 0, None) == 0              # nothing to copy
    assert "no device" in L.x264hip_backend_banner().decode()


@pytest.mark.parametrize("bd", [8, 10])
def test_centred_esa_range_bound(bd):
    """The centred ESA entries take a template range >= me_range: the centred table holds
    me.c's whole width-rounded window (me.c:621-626) around an aligned-down origin, so
    range = me_range is exact; range < me_range is X264HIP_EINVAL, checked before any HIP
    call, and so is a template range other than 4 / 8 / 16 / 24 for the fused search."""
    x = load_package()
    L = x.lib()
    esa = getattr(L, f"x264hip_{bd}_me_search_esa")
    at = getattr(L, f"x264hip_{bd}_me_esa_argmin_at")
    V = ctypes.c_void_p
    for rng, me_range in ((16, 17), (24, 25), (8, 9), (4, 5), (12, 12)):
        assert esa(V(), 0, 0, V(), 0, 0, 0, 0, 0, rng, me_range, V(), V(), V(), V(), V()) == -1, (rng, me_range)
        if rng != 12:
            assert at(V(), rng, 0, me_range, V(8), V(), V(), V(), V(), V()) == -1, (rng, me_range)
    # in bounds: an empty launch is accepted (no frames, nothing to do)
    for rng, me_range in ((24, 24), (16, 16), (8, 8), (4, 4), (24, 16)):
        assert esa(V(), 0, 0, V(), 0, 0, 0, 0, 0, rng, me_range, V(), V(), V(), V(), V()) in (0, -2, -3), \
            (rng, me_range)


def test_table_pitch_entry():
    """x264hip_me_table_pitch: full tables align4(2R+1), centred tables me.c's ESA window
    (align4(2R+6) at 8 bit, align4(2R+4) at 10 bit), as the Python mirror computes them."""
    x = load_package()
    L = x.lib()
    for bd in (8, 10):
        for r in (4, 8, 16, 24, 29):
            assert L.x264hip_me_table_pitch(bd, r, 0) == x.me_table_pitch(r)
            assert L.x264hip_me_table_pitch(bd, r, 1) == x.me_centred_pitch(bd, r)
    assert L.x264hip_me_table_pitch(8, 16, 1) == 40 and L.x264hip_me_table_pitch(10, 16, 1) == 36
    assert L.x264hip_me_table_pitch(9, 16, 0) == 0 and L.x264hip_me_table_pitch(8, 30, 0) == 0


# ---------------------------------------------------------------- reference layout
REF = "/root/reference/common"


def _struct_fields(body):
    """Ordered (name, extent) of a C struct body: function pointers `(*name[n])(...)`,
    plain members `type name[n]`; comments and macro continuations stripped."""
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    body = re.sub(r"//[^\n]*", "", body)
    body = re.sub(r"#define(?:[^\n]*\\\n)*[^\n]*", "", body)   # TRELLIS_PARAMS (quant.h:57-60)
    body = body.replace("\\\n", "\n")                            # our header's macro continuations
    body = body.replace("TRELLIS_PARAMS,", "")
    out = []
    for decl in body.split(";"):
        d = " ".join(decl.split())
        if not d:
            continue
        m = re.match(r"^[\w\s\*]*?\(\s*\*\s*(\w+)\s*(?:\[(\w+)\])?\s*\)", d)
        if not m:
            m = re.match(r"^.*?(\w+)\s*(?:\[(\w+)\])?\s*$", d.split("(")[0] if "(" not in d else d)
        assert m, d
        name = m.group(1)
        name = re.sub(r"^x264hip_##BD##_", "", name)
        out.append((name, m.group(2) or "1"))
    return out


def _ref_struct(path, tname):
    src = open(path).read()
    m = re.search(r"typedef struct\s*\{([^{}]*)\}\s*" + tname + r"\s*;", src, re.S)
    assert m, tname
    return _struct_fields(m.group(1))


def _our_struct(tname):
    src = open(HEADER).read()
    m = re.search(r"typedef struct\s*\\\s*\{([^{}]*)\}\s*x264hip_##BD##_" + tname + r"\s*;", src, re.S)
    assert m, tname
    return _struct_fields(m.group(1))


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present (GPU box)")
@pytest.mark.parametrize("ref_file,tname", [("pixel.h", "pixel_function_t"), ("dct.h", "dct_function_t"),
                                             ("dct.h", "zigzag_function_t"), ("quant.h", "quant_function_t")])
def test_tables_match_reference_headers(ref_file, tname):
    """include/x264hip.h's re-declared tables have the reference's field names, order and
    array extents (reference common/pixel.h:78-144, dct.h:29-70, quant.h:30-70), parsed
    from the reference headers as text."""
    want = _ref_struct(os.path.join(REF, ref_file), "x264_" + tname)
    got = _our_struct(tname)
    assert got == want
    assert len(want) >= 6


@pytest.mark.parametrize("bd", [8, 10])
def test_product_cqm_equals_oracle(oracle, bd):
    import checkasm_bufs as cb
    x = load_package()
    cb.srand(cb.SEED)
    for i_cqm in range(6):
        lists = cb.cqm_lists(i_cqm, bd)
        for dz in ((21, 11), (0, 0), (5, 30)):
            got = x.cqm_init(bd, lists, dz[0], dz[1])
            want = oracle.cqm_init(bd, lists, dz[0], dz[1])
            for g, w in zip(got, want):
                assert np.array_equal(g, w), (i_cqm, dz)
