"""CPU: the constant tables the oracle and the product restate, pinned to the reference's
own text.  Parity of the arithmetic stays unpinned (the reference
cannot be built here), but every table both sides copied from it is
checked value for value against the reference source, read as text:

* common/set.c:31-71        dequant4/8_scale, quant4/8_scale, quant8_scan
* common/tables.c:183-184   x264_hpel_ref0 / x264_hpel_ref1
* encoder/me.c:53-56        mod6m1, hex2, square1
* common/dct.c:768-816      the 8x8 / 4x4 frame and field zigzag scans (ZIG(i,y,x) lists)

Skipped where /root/reference is absent (the GPU box)."""
import os
import re

import numpy as np
import pytest

from conftest import ROOT

REF = "/root/reference"
pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present (GPU box)")

ORACLE = os.path.join(ROOT, "oracle", "oracle.c")
CSRC = os.path.join(ROOT, "x264-i386pic_amd", "csrc")


def _text(path):
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    return re.sub(r"//[^\n]*", " ", src)


def c_array(path, name, nth=0):
    """Integers of the brace initialiser of array `name` in a C/C++/HIP file (comments
    stripped), in order; `nth` picks among several definitions of the name."""
    src = _text(path)
    hits = [m for m in re.finditer(r"\b" + re.escape(name) + r"\s*(?:\[[^\]]*\]\s*)+=\s*\{", src)]
    assert len(hits) > nth, (path, name)
    i = hits[nth].end() - 1
    depth, j = 0, i
    while True:
        if src[j] == "{":
            depth += 1
        elif src[j] == "}":
            depth -= 1
            if depth == 0:
                break
        j += 1
    return [int(v) for v in re.findall(r"-?\d+", src[i:j + 1])]


def zig_macro(name):
    """(y, x) pairs of dct.c's ZIGZAG macro `name` in scan order (ZIG / ZIGDC(i,y,x))."""
    src = open(os.path.join(REF, "common", "dct.c")).read()
    m = re.search(r"#define " + name + r"\\\n((?:[^\n]*\\\n)*[^\n]*)", src)
    assert m, name
    items = re.findall(r"ZIG(?:DC)?\(\s*(\d+)\s*,\s*(\d+)\s*,\s*(\d+)\s*\)", m.group(1))
    items = sorted((int(i), int(y), int(x)) for i, y, x in items)
    assert [i for i, _, _ in items] == list(range(len(items)))
    return [v for _, y, x in items for v in (y, x)]


SET_C = os.path.join(REF, "common", "set.c")


@pytest.mark.parametrize("ref_name,ours", [
    ("dequant4_scale", [(ORACLE, "dequant4_scale"), (os.path.join(CSRC, "capi.cpp"), "k_dequant4_scale")]),
    ("dequant8_scale", [(ORACLE, "dequant8_scale"), (os.path.join(CSRC, "capi.cpp"), "k_dequant8_scale")]),
    ("quant4_scale", [(ORACLE, "quant4_scale"), (os.path.join(CSRC, "capi.cpp"), "k_quant4_scale")]),
    ("quant8_scale", [(ORACLE, "quant8_scale"), (os.path.join(CSRC, "capi.cpp"), "k_quant8_scale")]),
    ("quant8_scan", [(ORACLE, "quant8_scan"), (os.path.join(CSRC, "capi.cpp"), "k_quant8_scan"),
                     (os.path.join(CSRC, "capi.cpp"), "k_quant8_scan16")]),
])
def test_cqm_scale_tables(ref_name, ours):
    want = c_array(SET_C, ref_name)
    assert len(want) in (16, 18, 36)
    for path, name in ours:
        assert c_array(path, name) == want, (path, name)


def test_hpel_ref_tables():
    tables = os.path.join(REF, "common", "tables.c")
    for k in (0, 1):
        want = c_array(tables, "x264_hpel_ref%d" % k)
        assert len(want) == 16
        assert c_array(ORACLE, "hpel_ref%d" % k) == want
        assert c_array(os.path.join(CSRC, "lookahead.hip"), "c_lr_ref%d" % k) == want


def test_me_pattern_tables():
    me = os.path.join(REF, "encoder", "me.c")
    la = os.path.join(CSRC, "lookahead.hip")
    for ref_name, orc_name, hip_name, n in (("mod6m1", "lr_mod6m1", "c_mod6m1", 8),
                                           ("hex2", "lr_hex2", "c_hex2", 16),
                                           ("square1", "lr_square1", "c_square1", 18)):
        want = c_array(me, ref_name)
        assert len(want) == n
        assert c_array(ORACLE, orc_name) == want, orc_name
        assert c_array(la, hip_name) == want, hip_name


def test_zigzag_scans():
    f8, d8 = zig_macro("ZIGZAG8_FRAME"), zig_macro("ZIGZAG8_FIELD")
    f4, d4 = zig_macro("ZIGZAG4_FRAME"), zig_macro("ZIGZAG4_FIELD")
    assert len(f8) == len(d8) == 128 and len(f4) == len(d4) == 32
    assert c_array(ORACLE, "zz8_frame") == f8
    assert c_array(ORACLE, "zz8_field") == d8
    assert c_array(ORACLE, "zz4_frame") == f4
    assert c_array(ORACLE, "zz4_field") == d4
    idct = os.path.join(CSRC, "idct.hip")
    assert c_array(idct, "c_zz8") == f8 + d8
    assert c_array(idct, "c_zz4") == f4 + d4
    assert c_array(idct, "yx", 0) == f8 + d8           # ZZ<8, FIELD>'s compile-time copy
    assert c_array(idct, "yx", 1) == f4 + d4           # ZZ<4, FIELD>
    # every scan is a permutation of the block
    for t, w in ((f8, 8), (d8, 8), (f4, 4), (d4, 4)):
        pos = np.array(t).reshape(-1, 2)
        assert len({(y, x) for y, x in pos}) == w * w


def test_zigzag_4x4_field_copy_regions():
    """zigzag_scan_4x4_field (dct.c:835-841) copies level[0..1] and [6..15] straight from
    dct and permutes 2..5: the ZIGZAG4_FIELD list agrees, i.e. dct[x*4+y] == index i there."""
    d4 = np.array(zig_macro("ZIGZAG4_FIELD")).reshape(-1, 2)
    for i in list(range(2)) + list(range(6, 16)):
        y, x = d4[i]
        assert x * 4 + y == i


def test_jvt_cqm_lists():
    """The JVT default scaling lists the checkasm CQM cases use (tests/checkasm_bufs.py,
    checkasm.c:2098-2113) equal common/tables.c:191-226."""
    import checkasm_bufs as cb
    tables = os.path.join(REF, "common", "tables.c")
    for ours, name in ((cb.JVT4I, "x264_cqm_jvt4i"), (cb.JVT4P, "x264_cqm_jvt4p"), (cb.JVT8I, "x264_cqm_jvt8i"),
                       (cb.JVT8P, "x264_cqm_jvt8p")):
        assert list(ours) == c_array(tables, name), name
