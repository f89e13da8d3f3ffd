"""Policy helpers (utils.rs tests :146-278) against the oracle."""
import ctypes as C
import math

import numpy as np

import oracle_ffi as O


def test_log_prob_uniform():                       # utils.rs:171-184
    lp = O.lib().or_log_prob(np.zeros(4, np.float32), 4, 0)
    assert abs(lp - math.log(0.25)) < 1e-4


def test_entropy_uniform():                        # utils.rs:187-198
    assert abs(O.lib().or_entropy(np.zeros(4, np.float32), 4) - math.log(4)) < 1e-4


def test_normalize_advantages():                   # utils.rs:201-215
    out = np.zeros(4, np.float32)
    m, s, lo, hi = (C.c_float() for _ in range(4))
    O.lib().or_normalize_advantages(np.array([1, 2, 3, 4], np.float32), 4, out, C.byref(m),
                                    C.byref(s), C.byref(lo), C.byref(hi))
    assert abs(out.mean()) < 1e-5
    assert abs(out.std(ddof=1) - 1.0) < 1e-4
    assert (lo.value, hi.value) == (1.0, 4.0)


def test_sample_dominant_logit():                  # utils.rs:158-168
    r = O.new_rng(42)
    a = np.zeros(1, np.int32)
    O.lib().or_sample_categorical(C.byref(r), np.array([0, 0, 100, 0], np.float32), 1, 4, a)
    assert a[0] == 2
    assert r.word_pos == 4                        # one u32 word per (env, action)


def test_masked_action_never_sampled():            # utils.rs:257-278
    r = O.new_rng(42)
    logits = np.zeros((10, 4), np.float32)
    logits[:, 0] = -np.inf
    a = np.zeros(10, np.int32)
    O.lib().or_sample_categorical(C.byref(r), logits.reshape(-1), 10, 4, a)
    assert np.all(a != 0)


def test_gumbel_argmax_matches_formula():
    r = O.new_rng(1234)
    rng = np.random.default_rng(0)
    logits = rng.normal(size=(64, 7)).astype(np.float32)
    a = np.zeros(64, np.int32)
    O.lib().or_sample_categorical(C.byref(r), logits.reshape(-1), 64, 7, a)
    w = O.stdrng_words(1234, 64 * 7)
    u = ((w >> 9) | 0x3F800000).view(np.float32) - np.float32(1)
    u = (u * np.float32(1.0) + np.float32(1e-10)).astype(np.float32)
    g = -np.log(-np.log(u.astype(np.float64))).astype(np.float32)
    ref = np.argmax(logits + g.reshape(64, 7), axis=1)
    assert np.mean(ref == a) > 0.98            # numpy log is not glibc logf: near-ties may differ
