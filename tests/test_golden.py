"""The committed golden fixtures (tests/golden/make_fixtures.py, SURVEY 8(c)
plan item 5) against the oracle: the oracle still produces them bit for bit
(every other parity check compares against the live oracle, so this is what
catches an oracle regression)."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_fixtures as MF  # noqa: E402

FIX = {"cartpole_traj_16x32": MF.cartpole_traj,
       "c4_scripted": lambda: MF.scripted(1, 6, 60, 86, 7, 2, 0, 0.0),
       "ld_scripted": lambda: MF.scripted(2, 4, 80, 270, 49, 4, 120, 0.05),
       "minibatch_cfgB": MF.minibatch,
       "w_cfgA": MF.cfgA}


@pytest.mark.parametrize("name", sorted(FIX))
def test_oracle_reproduces_fixture(name):
    ref = np.load(os.path.join(HERE, "golden", name + ".npz"))
    got = FIX[name]()
    assert sorted(ref.files) == sorted(got)
    for k in ref.files:
        a, b = np.atleast_1d(np.asarray(got[k])), np.atleast_1d(ref[k])
        assert a.shape == b.shape and a.dtype.kind == b.dtype.kind, k
        if a.dtype.kind == "f":
            a = a.astype(b.dtype)   # Python floats (f64) of 0-d entries
            assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), k
        else:
            assert np.array_equal(a, b), k


def test_fixture_content_is_nontrivial():
    t = np.load(os.path.join(HERE, "golden", "cartpole_traj_16x32.npz"))
    assert t["dones"].sum() >= 10 and int(t["rng_pos"]) == 16 * 32 * 2
    m = np.load(os.path.join(HERE, "golden", "minibatch_cfgB.npz"))
    assert 0.2 < float(m["clip_fraction"]) < 0.8          # the clipped branch of ppo.rs:1455-1461 runs
    assert not np.array_equal(m["params"], m["params_after"])
    ld = np.load(os.path.join(HERE, "golden", "ld_scripted.npz"))
    assert ld["dones"].sum() >= 4 and (ld["rewards"] != 0).any()
