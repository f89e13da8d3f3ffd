"""The product's glibc logf/sinf/cosf/expf restatement (burn-ppo_amd/csrc/bppo_math.h)
against the platform glibc the reference's Rust code calls (utils.rs:25,
cartpole.rs:51-52).  A one-off exhaustive run over every finite float found zero
mismatches; this test re-checks every Gumbel input plus dense and
random samples so the CPU suite stays fast."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.fixture(scope="module")
def chk(tmp_path_factory):
    out = tmp_path_factory.mktemp("libm") / "libm_check.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
                    "-march=x86-64-v3", "-I", os.path.join(ROOT, "burn-ppo_amd", "csrc"),
                    os.path.join(HERE, "native", "libm_check.cpp"), "-o", str(out), "-lm"], check=True)
    L = C.CDLL(str(out))
    f32 = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
    L.mismatch_logf.restype = C.c_size_t
    L.mismatch_logf.argtypes = [f32, C.c_size_t, f32, f32]
    L.mismatch_expf.restype = C.c_size_t
    L.mismatch_expf.argtypes = [f32, C.c_size_t, f32, f32]
    L.mismatch_sincos.restype = C.c_size_t
    L.mismatch_sincos.argtypes = [f32, C.c_size_t, f32, f32, f32, f32]
    L.mismatch_tanhf.restype = C.c_size_t
    L.mismatch_tanhf.argtypes = [f32, C.c_size_t, f32, f32]
    L.mismatch_gumbel_all.restype = C.c_size_t
    return L


def _run_logf(L, x):
    x = np.ascontiguousarray(x, np.float32)
    r = np.empty_like(x); g = np.empty_like(x)
    return L.mismatch_logf(x, x.size, r, g)


def _run_sincos(L, x):
    x = np.ascontiguousarray(x, np.float32)
    a = [np.empty_like(x) for _ in range(4)]
    return L.mismatch_sincos(x, x.size, *a)


def test_every_gumbel_input(chk):
    assert chk.mismatch_gumbel_all() == 0


def test_logf_samples(chk):
    rng = np.random.default_rng(0)
    bits = rng.integers(0, 0x7F800000, size=4_000_000, dtype=np.uint32)
    assert _run_logf(chk, bits.view(np.float32)) == 0
    # subnormals, specials
    special = np.array([0.0, -0.0, 1.0, np.inf, -1.0, np.nan, 1e-45, 1e-40, 3.4e38], np.float32)
    assert _run_logf(chk, special) == 0


def test_sincos_cartpole_range_dense(chk):
    # every 3rd float in |theta| < 0.5 (CartPole's angle stays within ~0.25 rad)
    lo = np.arange(0, np.float32(0.5).view(np.uint32), 3, dtype=np.uint32)
    x = lo.view(np.float32)
    assert _run_sincos(chk, x) == 0
    assert _run_sincos(chk, -x) == 0


def test_sincos_wide_samples(chk):
    rng = np.random.default_rng(1)
    bits = rng.integers(0, 0x7F800000, size=2_000_000, dtype=np.uint32)
    x = bits.view(np.float32)
    assert _run_sincos(chk, x) == 0
    assert _run_sincos(chk, -x) == 0


def test_expf_samples(chk):
    rng = np.random.default_rng(2)
    bits = rng.integers(0, 2**32, size=4_000_000, dtype=np.uint64).astype(np.uint32)
    x = bits.view(np.float32)
    x = x[~np.isnan(x)]
    xs = np.ascontiguousarray(x)
    r = np.empty_like(xs); g = np.empty_like(xs)
    assert chk.mismatch_expf(xs, xs.size, r, g) == 0
    # the two inputs where glibc's contracted reduction is not correctly rounded
    hard = np.array([float.fromhex("0x1.04845ep+5"), float.fromhex("-0x1.f8cbb2p+5")], np.float32)
    r = np.empty_like(hard); g = np.empty_like(hard)
    assert chk.mismatch_expf(hard, 2, r, g) == 0
    # log-softmax range
    dense = np.linspace(-30, 0, 1_000_001, dtype=np.float32)
    r = np.empty_like(dense); g = np.empty_like(dense)
    assert chk.mismatch_expf(dense, dense.size, r, g) == 0


def test_tanhf_samples(chk):
    """tanh activation (mlp.rs:187-191): every 7th float with |x| < 22 (both
    signs, every expm1f branch), random bit patterns, and the specials."""
    lo = np.arange(0, np.float32(22.0).view(np.uint32), 7, dtype=np.uint32).view(np.float32)
    for x in (lo, -lo):
        xs = np.ascontiguousarray(x); r = np.empty_like(xs); g = np.empty_like(xs)
        assert chk.mismatch_tanhf(xs, xs.size, r, g) == 0
    rng = np.random.default_rng(3)
    x = rng.integers(0, 2**32, size=2_000_000, dtype=np.uint64).astype(np.uint32).view(np.float32)
    x = np.ascontiguousarray(x[~np.isnan(x)])
    r = np.empty_like(x); g = np.empty_like(x)
    assert chk.mismatch_tanhf(x, x.size, r, g) == 0
    sp = np.array([0.0, -0.0, np.inf, -np.inf, 1e-45, -1e-40, 2.0**-56, 22.0, -22.0, 1.0, -1.0], np.float32)
    r = np.empty_like(sp); g = np.empty_like(sp)
    assert chk.mismatch_tanhf(sp, sp.size, r, g) == 0
