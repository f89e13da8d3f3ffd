"""The C-ABI library loads and exports every symbol include/bppo.h declares
(no compute calls: this runs without a GPU)."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def so():
    p = os.path.join(ROOT, "burn-ppo_amd", "bppo", "libbppo.so")
    if not os.path.exists(p):
        subprocess.run(["make", "-j8", "-C", os.path.join(ROOT, "burn-ppo_amd")], check=True)
    return p


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "bppo.h")).read()
    return sorted(set(re.findall(r"\b(bppo_[a-z_0-9]+)\s*\(", txt)))


def test_header_declares_expected_surface():
    syms = header_symbols()
    import bppo._lib as L
    assert sorted(L.EXPORTS) == syms


def test_library_exports_every_header_symbol(so):
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (bppo_[a-z_0-9]+)$", out, re.M))
    missing = [s for s in header_symbols() if s not in exported]
    assert not missing, missing


def test_library_loads_and_reports_version(so):
    import bppo._lib as L
    lib = L.lib()
    assert lib.bppo_version().decode().startswith("bppo-mi355x")


def test_offload_arch_is_gfx950(so):
    # the embedded clang offload bundle names its targets (no extraction to disk)
    data = open(so, "rb").read()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in data


def test_host_libm_path_without_gpu():
    import numpy as np
    import bppo._lib as L
    x = np.linspace(1e-6, 1.0, 1000, dtype=np.float32)
    y = np.zeros_like(x)
    assert L.lib().bppo_debug_libm(0, 0, x.ctypes.data, y.ctypes.data, x.size) == 0
    assert np.allclose(y, np.log(x), rtol=1e-6, atol=1e-7)
