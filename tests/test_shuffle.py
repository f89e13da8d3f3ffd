"""ppo_update's per-epoch shuffle (ppo.rs:1816, rand 0.8.5 SliceRandom::shuffle
on StdRng): the product's host draw chain (shuffle_host.cpp, AVX-512 or scalar
walker, ChaCha12 words made by its own SIMD generator) against the oracle's
gen_range(0..i+1) loop, and the device Fisher-Yates (k_shuffle.hip) against the
sequential swap pass.  Bit-exact: swap targets, word positions, permutations."""
import ctypes as C

import numpy as np
import pytest

import bppo._lib as L
import oracle_ffi as O


def _oracle_targets(seed, stream, pos, n):
    r = O.Rng()
    O.lib().or_rng_seed_u64(C.byref(r), seed)
    r.stream = stream
    r.word_pos = pos
    J = np.zeros(n, np.uint32)
    O.lib().or_shuffle_targets(C.byref(r), J, n)
    return J, r.word_pos


@pytest.mark.parametrize("seed,stream,pos,n", [
    (42, 0, 0, 1), (42, 0, 0, 2), (42, 0, 7, 3), (7, 0, 123, 1000),
    (42, 0, 262_141, 70_001),            # crosses the 2^18-word chunk boundary mid-walk
    (42, 3, 5, 1 << 17),                 # rank stream 3, n a power of two (first draw never rejects)
    (9, 0, 1_000_003, (1 << 16) + 1),    # n just above a power of two (rejection ~1/2)
])
def test_host_chain_matches_oracle(seed, stream, pos, n):
    J = np.zeros(n, np.uint32)
    end = C.c_uint64()
    assert L.lib().bppo_debug_shuffle_chain(seed, stream, pos, n, J.ctypes.data, C.byref(end)) == 0
    Jo, endo = _oracle_targets(seed, stream, pos, n)
    assert np.array_equal(J, Jo)
    assert end.value == endo


def test_host_chain_full_cfgb_epoch():
    """one CfgB epoch (B = 2^23 draws, ~11.6 M words): targets and end position"""
    n = 1 << 23
    J = np.zeros(n, np.uint32)
    end = C.c_uint64()
    assert L.lib().bppo_debug_shuffle_chain(42, 0, 16_777_216, n, J.ctypes.data, C.byref(end)) == 0
    Jo, endo = _oracle_targets(42, 0, 16_777_216, n)
    assert end.value == endo
    assert np.array_equal(J, Jo)
    assert np.all(J <= np.arange(n, dtype=np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 3, 17, 1000, 8193, 100_003, (1 << 20) - 1, 1 << 20, 3_000_017, 1 << 23])
def test_device_fisher_yates_matches_sequential(n):
    rng = np.random.default_rng(n)
    i = np.arange(n, dtype=np.uint64)
    J = np.minimum((rng.random(n) * (i + 1)).astype(np.uint64), i).astype(np.uint32)
    J[0] = 0
    if n > 10:
        J[n // 2] = n // 2            # self-swaps
        J[n - 1] = 0                  # a long bucket at 0
    perm = np.zeros(n, np.uint32)
    assert L.lib().bppo_debug_fisher_yates(0, J.ctypes.data, n, perm.ctypes.data) == 0
    ref = np.arange(n, dtype=np.uint32)
    O.lib().or_apply_swaps(J, ref, n)
    assert np.array_equal(perm, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["identity", "half", "front"])
def test_device_fisher_yates_skewed_targets(kind):
    """Inputs far from J[i] ~ U[0, i]: target ranges overflow their LDS capacity
    (front: every step targets the first 4096 positions) and the gated direct
    bucketing must produce the permutation; identity / half stay in the ranged
    path.  n = 2^20 (the ranged path's minimum).  (The direct path orders each
    target's steps by insertion sort: quadratic in the largest bucket, which is
    ~ln n for RNG-drawn J; a J with 10^5+ steps on one target is not a case.)"""
    n = 1 << 20
    i = np.arange(n, dtype=np.uint64)
    if kind == "identity":
        J = i.astype(np.uint32)
    elif kind == "half":
        J = (i // 2).astype(np.uint32)
    else:                                   # every step targets one of the first 4096 positions
        rng = np.random.default_rng(5)
        J = np.minimum(rng.integers(0, 4096, n, dtype=np.uint64), i).astype(np.uint32)
    J[0] = 0
    perm = np.zeros(n, np.uint32)
    assert L.lib().bppo_debug_fisher_yates(0, J.ctypes.data, n, perm.ctypes.data) == 0
    ref = np.arange(n, dtype=np.uint32)
    O.lib().or_apply_swaps(J, ref, n)
    assert np.array_equal(perm, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,start,n,epochs,gap,jobs", [
    (42, 1_000_003, 1 << 23, 4, 16_777_216, 3),   # CfgB: 3 updates (the 2nd and 3rd meet speculative walks)
    (7, 5, 100_003, 6, 700_000, 3),                # small n, many epochs
    (3, 0, 2, 3, 5, 2),                            # degenerate
    (11, 12_345, (1 << 20) + 1, 2, 0, 2),
])
def test_shuffle_engine_equals_sequential_walks(seed, start, n, epochs, gap, jobs):
    """The engine (GPU-made words, speculative walks for the next update spliced
    at a meeting checkpoint, J rebuilt on the GPU from checkpoint states) returns
    exactly the chained single-thread walks."""
    J = np.zeros(n * epochs * jobs, np.uint32)
    ends = np.zeros(epochs * jobs, np.uint64)
    met = np.zeros(epochs * jobs, np.int32)
    assert L.lib().bppo_debug_shuffle_engine(seed, 0, start, n, epochs, gap, jobs, 0, J.ctypes.data,
                                             ends.ctypes.data, met.ctypes.data) == 0
    pos = start
    for j in range(jobs):
        for e in range(epochs):
            k = j * epochs + e
            Je = np.zeros(n, np.uint32)
            end = C.c_uint64()
            assert L.lib().bppo_debug_shuffle_chain(seed, 0, pos, n, Je.ctypes.data, C.byref(end)) == 0
            assert ends[k] == end.value, (j, e, met)
            assert np.array_equal(J[k * n:(k + 1) * n], Je), (j, e, met)
            pos = end.value
        pos += gap
    if n == 1 << 23:
        assert (met[epochs:] >= 0).any(), met      # at CfgB size the speculation does meet


@pytest.mark.gpu
@pytest.mark.parametrize("policy", ["0", "2", "k6"])
@pytest.mark.parametrize("seed,start,n,epochs,gap,jobs", [
    (5, 77, 1 << 23, 4, 16_777_216, 3),
    (9, 3, 100_003, 6, 700_000, 3),
])
def test_shuffle_engine_policies_equal_sequential(monkeypatch, policy, seed, start, n, epochs, gap, jobs):
    """The job-start speculation policy (BPPO_SHUFFLE_FRONTIER=0), frontier depth 2 and six
    guessed walks per boundary (BPPO_SHUFFLE_SPEC=6) give the same J and word positions as
    the sequential walk (the default is covered above)."""
    if policy == "k6":
        monkeypatch.setenv("BPPO_SHUFFLE_SPEC", "6")
    else:
        monkeypatch.setenv("BPPO_SHUFFLE_FRONTIER", policy)
    J = np.zeros(n * epochs * jobs, np.uint32)
    ends = np.zeros(epochs * jobs, np.uint64)
    met = np.zeros(epochs * jobs, np.int32)
    assert L.lib().bppo_debug_shuffle_engine(seed, 0, start, n, epochs, gap, jobs, 0, J.ctypes.data,
                                             ends.ctypes.data, met.ctypes.data) == 0
    pos = start
    for j in range(jobs):
        for e in range(epochs):
            k = j * epochs + e
            Je = np.zeros(n, np.uint32)
            end = C.c_uint64()
            assert L.lib().bppo_debug_shuffle_chain(seed, 0, pos, n, Je.ctypes.data, C.byref(end)) == 0
            assert ends[k] == end.value, (j, e, met)
            assert np.array_equal(J[k * n:(k + 1) * n], Je), (j, e, met)
            pos = end.value
        pos += gap


def _window(n):
    return 2 * n + (1 << 20)      # shuffle_window (bppo_internal.h)


@pytest.mark.gpu
@pytest.mark.parametrize("gpu_words", ["0", "1"])
@pytest.mark.parametrize("threads", ["16", "2"])
@pytest.mark.parametrize("seed,start,n,epochs,gap,jobs", [
    (5, 77, 1 << 23, 4, 16_777_216, 3),
    (9, 3, 100_003, 6, 700_000, 3),
])
def test_shuffle_engine_windows_equal_sequential(monkeypatch, gpu_words, threads, seed, start, n, epochs, gap, jobs):
    """shuffle_windows: epoch e of an update starts at S + e * (2 n + 2^20), the next
    update gap words after S + epochs * (2 n + 2^20).  The engine walks the epochs at
    once, exactly (no speculation), with 16 or 2 host CPUs; J and the end positions must
    equal the single-thread walks from those starts."""
    monkeypatch.setenv("BPPO_HOST_THREADS", threads)
    monkeypatch.setenv("BPPO_SHUFFLE_GPU_WORDS", gpu_words)     # 1: the walks read the GPU's words (SDMA copies)
    J = np.zeros(n * epochs * jobs, np.uint32)
    ends = np.zeros(epochs * jobs, np.uint64)
    assert L.lib().bppo_debug_shuffle_engine(seed, 0, start, n, epochs, gap, jobs, 1, J.ctypes.data,
                                             ends.ctypes.data, None) == 0
    S = start
    for j in range(jobs):
        for e in range(epochs):
            k = j * epochs + e
            Je = np.zeros(n, np.uint32)
            end = C.c_uint64()
            assert L.lib().bppo_debug_shuffle_chain(seed, 0, S + e * _window(n), n, Je.ctypes.data, C.byref(end)) == 0
            assert ends[k] == end.value, (j, e)
            assert end.value - (S + e * _window(n)) < _window(n)      # the walk stays inside its window
            assert np.array_equal(J[k * n:(k + 1) * n], Je), (j, e)
        S = S + epochs * _window(n) + gap


@pytest.mark.parametrize("seed,pa,pb,n,piece", [
    (1, 0, 5, 1000, 1024), (7, 123, 99_999, 100_003, 1024), (42, 16_777_216, 1 << 30, 1 << 20, 1024),
    (3, 1, 2, 70_000, 37), (9, 0, 0, 5000, 1), (11, 1 << 33, 77, 3, 1024)])
def test_two_chain_walker_equals_sequential(seed, pa, pb, n, piece):
    """the interleaved two-chain walker (shuffle_windows pairs, shuffle_host.cpp
    chain_walk2_nj) over words handed over in pieces, incl. 1-word and odd-length pieces
    and band edges: both chains end exactly where the sequential walks end (host only)"""
    ea, eb = C.c_uint64(), C.c_uint64()
    assert L.lib().bppo_debug_chain_walk2(seed, 0, pa, pb, n, piece, C.byref(ea), C.byref(eb)) == 0
    for p, got in ((pa, ea.value), (pb, eb.value)):
        J = np.zeros(n, np.uint32)
        end = C.c_uint64()
        assert L.lib().bppo_debug_shuffle_chain(seed, 0, p, n, J.ctypes.data, C.byref(end)) == 0
        assert got == end.value
