"""CPU: code-generation guards on the built library's gfx950 code objects.

Round 4 found three faults by reading the ISA, each one more memory dependency on a latency-bound
search's serial chain ("Lookahead in round 4"): flat loads (an integer round trip
of a pointer made the lookahead's window loads `flat_load`, which also count against the LDS
wait counter), per-lane `__constant__` table loads, and arrays indexed per lane that the
compiler put in scratch memory (refine_subpel).  These tests disassemble every code object in
`libx264hip.so` (clang-offload-bundler + llvm-objdump, no GPU needed) and keep them out."""
import os
import re
import shutil
import subprocess

import pytest

from conftest import ROOT

LLVM = "/opt/rocm/lib/llvm/bin"
SO = os.path.join(ROOT, "x264-i386pic_amd", "libx264hip.so")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _tool(name):
    p = os.path.join(LLVM, name)
    return p if os.path.exists(p) else shutil.which(name)


@pytest.fixture(scope="module")
def kernels(tmp_path_factory):
    """{kernel symbol: [instruction lines]} over every gfx950 code object in the library"""
    objcopy, bundler, objdump = _tool("llvm-objcopy"), _tool("clang-offload-bundler"), _tool("llvm-objdump")
    if not (objcopy and bundler and objdump and os.path.exists(SO)):
        pytest.skip("LLVM tools or the built library missing")
    d = tmp_path_factory.mktemp("codegen")
    fat = d / "fat.bin"
    subprocess.run([objcopy, "--dump-section", f".hip_fatbin={fat}", SO, str(d / "so.tmp")], check=True,
                   capture_output=True)
    data = fat.read_bytes()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    assert starts, "no offload bundle in .hip_fatbin"
    out = {}
    for i, s in enumerate(starts):
        e = starts[i + 1] if i + 1 < len(starts) else len(data)
        chunk, co = d / f"b{i}.bin", d / f"b{i}.co"
        chunk.write_bytes(data[s:e])
        r = subprocess.run([bundler, "--unbundle", "--type=o", f"--input={chunk}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
        if r.returncode or not co.exists() or co.stat().st_size == 0:
            continue
        dis = subprocess.run([objdump, "-d", str(co)], capture_output=True, text=True, check=True).stdout
        name = None
        for line in dis.splitlines():
            m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
            if m:
                name = m.group(1)
                out.setdefault(name, [])
            elif name and line.startswith("\t"):
                out[name].append(line.strip())
    assert len(out) > 100, len(out)
    return out


def _ops(lines, pat):
    return [l for l in lines if re.match(pat, l)]


def test_no_flat_memory_ops(kernels):
    """every kernel addresses global memory as global_* and LDS as ds_* (no flat_*)"""
    bad = {k: _ops(v, r"flat_(load|store|atomic)")[:2] for k, v in kernels.items()}
    bad = {k: v for k, v in bad.items() if v}
    assert not bad, bad


def test_no_scratch_in_search_kernels(kernels):
    """the lookahead searches and refine_subpel keep all their state in registers / LDS"""
    hot = [k for k in kernels if "lowres_inter_kernel" in k or "lowres_bidir_kernel" in k or "refine" in k]
    assert hot
    bad = {k: _ops(kernels[k], r"scratch_")[:2] for k in hot}
    bad = {k: v for k, v in bad.items() if v}
    assert not bad, bad


def test_no_byte_table_loads_in_lookahead(kernels):
    """the reference's small tables (hpel_ref, hex2, mod6m1, square1) are immediates, not byte
    loads, in the lookahead searches (their only byte-sized global reads would be table reads:
    the planes are read as dwords)"""
    hot = [k for k in kernels if "lowres_inter_kernel" in k or "lowres_bidir_kernel" in k]
    assert hot
    bad = {k: _ops(kernels[k], r"global_load_(ubyte|sbyte)")[:2] for k in hot}
    bad = {k: v for k, v in bad.items() if v}
    assert not bad, bad
