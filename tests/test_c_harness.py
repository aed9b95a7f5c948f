"""The C boundary from a plain C99 program (tests/c/checkasm_hip.c): it includes
only include/x264hip.h (+ the HIP runtime API for one device-memory call), fills
the tables with x264hip_8_*_init(X264HIP_CPU_HIP) and checks every entry it calls
against the oracle, the way x264's own tools/checkasm.c would after the
INTEGRATION.md hook.  CPU: it compiles and links with gcc -std=c99 -Wall -Werror;
GPU: it runs clean."""
import os
import subprocess

import pytest

from conftest import ROOT, ensure_built

SRC = os.path.join(ROOT, "tests", "c", "checkasm_hip.c")


def build(tmp):
    ensure_built("hip")
    ensure_built("oracle")
    exe = os.path.join(tmp, "checkasm_hip")
    lib, orc = os.path.join(ROOT, "x264-i386pic_amd"), os.path.join(ROOT, "oracle")
    cmd = ["gcc", "-std=c99", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include",
           "-D__HIP_PLATFORM_AMD__", SRC, "-L", lib, "-lx264hip", "-L", orc, "-loracle", "-L", "/opt/rocm/lib",
           "-lamdhip64", f"-Wl,-rpath,{lib}:{orc}:/opt/rocm/lib", "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def test_c_harness_builds(tmp_path):
    exe = build(str(tmp_path))
    assert os.path.exists(exe)


@pytest.mark.gpu
def test_c_harness_runs(tmp_path):
    exe = build(str(tmp_path))
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "checkasm_hip: all ok" in r.stdout
