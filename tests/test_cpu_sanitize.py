"""The CPU restatement under AddressSanitizer + UndefinedBehaviorSanitizer.

oracle/Makefile's `asan` target compiles the same oracle.c / cpubench.c with
-fsanitize=address,undefined (-fwrapv kept, so only the wraps the reference relies
on are defined); this test re-runs the oracle-only CPU suites against that build in
a child interpreter with libasan preloaded, so every numpy buffer the tests hand
over carries redzones and any read or write past it, use after free or undefined
arithmetic aborts the child.  SURVEY.md §5 lists this (ASan on the CPU restatement)
as the sanitizer leg of the reference's own test strategy; GPU-side sanitizers are
not available on this pool."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

SUITES = ["test_cpu_oracle.py", "test_cpu_tesa.py", "test_cpu_ssd_plane.py", "test_cpu_lowres.py",
          "test_cpu_lookahead.py", "test_cpu_intra.py", "test_cpu_inverse.py", "test_cpu_pixel_ext.py",
          "test_golden.py"]


def _runtime(name):
    p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


def test_oracle_suites_clean_under_asan_ubsan():
    asan, ubsan = _runtime("libasan.so"), _runtime("libubsan.so")
    if not asan or not ubsan:
        pytest.skip("gcc sanitizer runtimes not installed")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True, capture_output=True)
    env = dict(os.environ)
    env.update(LD_PRELOAD=f"{asan}:{ubsan}", ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               X264HIP_ORACLE_LIB=os.path.join(ROOT, "oracle", "liboracle_asan.so"))
    tests = [os.path.join(ROOT, "tests", s) for s in SUITES]
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "not gpu",
                        *tests], env=env, capture_output=True, text=True, timeout=900, cwd=ROOT)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert " passed" in out
