"""Shared test plumbing.

* registers the ``gpu`` marker (GPU tests run on the MI355X box only);
* builds the CPU oracle (oracle/liboracle.so, test infrastructure) if missing;
* imports the product package ``x264-i386pic_amd`` under the name ``x264hip``.
"""
import importlib.util
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.join(ROOT, "tests")
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


def load_package():
    if "x264hip" in sys.modules:
        return sys.modules["x264hip"]
    pkg = os.path.join(ROOT, "x264-i386pic_amd")
    spec = importlib.util.spec_from_file_location("x264hip", os.path.join(pkg, "__init__.py"),
                                                  submodule_search_locations=[pkg])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["x264hip"] = mod
    spec.loader.exec_module(mod)
    return mod


def ensure_built(target):
    """Build oracle or HIP library in-tree if the .so is missing."""
    if target == "oracle":
        so = os.path.join(ROOT, "oracle", "liboracle.so")
        if not os.path.exists(so):
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True,
                           stdout=subprocess.DEVNULL)
        return so
    so = os.path.join(ROOT, "x264-i386pic_amd", "libx264hip.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-j8", "-C", os.path.join(ROOT, "x264-i386pic_amd", "csrc")], check=True,
                       stdout=subprocess.DEVNULL)
    return so


@pytest.fixture(scope="session")
def oracle():
    ensure_built("oracle")
    import oracle_lib
    return oracle_lib


@pytest.fixture(scope="session")
def hip():
    """The product package with a live gfx950 device (GPU tests only)."""
    ensure_built("hip")
    x = load_package()
    x.init(0)
    return x


_VARIANT_SWITCHES = ("X264HIP_TESA_VARIANT", "X264HIP_INTEGRAL_VARIANT", "X264HIP_LA_POLL", "X264HIP_UPLOAD_WGS",
                     "X264HIP_ME_XCD", "X264HIP_STREAM_XCD", "X264HIP_STREAM_NT", "X264HIP_LA_HELPER",
                     "X264HIP_LA_XCD")


@pytest.fixture(autouse=True)
def _reset_kernel_variants():
    """A/B kernel switches (x264hip_set_variant) never leak from one test into the next."""
    yield
    x = sys.modules.get("x264hip")
    if x is not None and getattr(x, "_lib", None) is not None:
        for name in _VARIANT_SWITCHES:
            x.set_variant(name, None)
