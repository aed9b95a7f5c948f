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


def build(tmp, sanitize=False):
    """sanitize: the harness itself and the oracle build from oracle/Makefile's `asan` target
    under ASan + UBSan (host code only; the GPU side has no sanitizer on this pool)."""
    ensure_built("hip")
    ensure_built("oracle")
    exe = os.path.join(tmp, "checkasm_hip_asan" if sanitize else "checkasm_hip")
    lib, orc = os.path.join(ROOT, "x264-i386pic_amd"), os.path.join(ROOT, "oracle")
    san = ["-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"]
    if sanitize:
        subprocess.run(["make", "-s", "-C", orc, "asan"], check=True, capture_output=True)
    olib = orc + "/liboracle_asan.so" if sanitize else "-loracle"
    cmd = ["gcc", "-std=c99", "-O2", "-Wall", "-Werror", *(san if sanitize else []), "-I", os.path.join(ROOT, "include"),
           "-I", "/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", SRC, "-L", lib, "-lx264hip", "-L", orc, olib,
           "-L", "/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{lib}:{orc}:/opt/rocm/lib", "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def test_c_harness_builds(tmp_path):
    exe = build(str(tmp_path))
    assert os.path.exists(exe)


def test_c_harness_builds_sanitized(tmp_path):
    assert os.path.exists(build(str(tmp_path), sanitize=True))


@pytest.mark.gpu
def test_c_harness_runs_sanitized(tmp_path):
    """The same run with the harness and the oracle under ASan + UBSan: the host buffers the
    harness allocates carry redzones for every oracle and boundary call on them."""
    exe = build(str(tmp_path), sanitize=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:protect_shadow_gap=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "checkasm_hip: all ok" in r.stdout


@pytest.mark.gpu
def test_c_harness_runs(tmp_path):
    exe = build(str(tmp_path))
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "checkasm_hip: all ok" in r.stdout
