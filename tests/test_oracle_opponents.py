"""Oracle restatement of the opponent-pool seat shuffle (opponent_pool.rs:107-123)
and of collect_rollouts_with_opponents' learner-row bookkeeping (ppo.rs:537-1063).
Parity unpinned against the reference (no Rust toolchain, HashMap batch order
unspecified there); these check the restatement's invariants and RNG use."""
import ctypes as C

import numpy as np
import pytest

import oracle_ffi as O


def _rng(seed, pos=0):
    r = O.Rng()
    O.lib().or_rng_seed_u64(C.byref(r), seed)
    r.word_pos = pos
    return r


@pytest.mark.parametrize("P", [2, 3, 4])
def test_shuffle_positions_invariants_and_words(P):
    assigned = np.arange(10, 10 + P - 1, dtype=np.int32)
    seen = set()
    for s in range(300):
        r = _rng(s)
        lp = C.c_int32(); po = np.zeros(P, np.int32)
        O.lib().or_shuffle_positions(C.byref(r), P, assigned, C.byref(lp), po)
        assert 0 <= lp.value < P and po[lp.value] == -1
        assert sorted(po[po >= 0].tolist()) == assigned.tolist()
        seen.add((lp.value, tuple(po)))
        # usize gen_range(0..P): two-word u64 draws, then P-2 u32 shuffle draws
        r2 = _rng(s)
        first = O.lib().or_gen_range_u64(C.byref(r2), 0, P)
        assert first == lp.value and r2.word_pos % 2 == 0
        assert r.word_pos >= r2.word_pos + (P - 2)
    import math
    assert len(seen) == P * math.factorial(P - 1)    # every seating occurs


def test_gen_range_u64_power_of_two_rejection():
    # rand 0.8.5's zone (range << lz) - 1 rejects half of the draws for ranges 2^k
    r = _rng(11)
    n = 4000
    v = [O.lib().or_gen_range_u64(C.byref(r), 0, 4) for _ in range(n)]
    assert set(v) == {0, 1, 2, 3}
    assert 3.6 < r.word_pos / n < 4.4          # ~2 tries x 2 words


def test_opponent_rollout_learner_rows():
    """An oracle opponent rollout + update: self-play envs are all learner rows,
    opponent envs about 1/P of them; the update trains on exactly those rows."""
    from bppo import host
    N, T, n_opp, P, K = 24, 20, 16, 2, 2
    cfg = host.make_config("connect_four", num_envs=N, num_steps=T, hidden_size=32, num_hidden=1,
                           num_minibatches=2, num_epochs=1)
    params = host.orthogonal_init(cfg, seed=1)
    ocfg = O.train_cfg(env_kind=O.ENV_CONNECT_FOUR, num_envs=N, num_steps=T, hidden=32, num_hidden=1,
                       normalize_obs=False, normalize_returns=False, num_minibatches=2, num_epochs=1)
    ot = O.Trainer(ocfg, params)
    opp = np.stack([host.orthogonal_init(cfg, seed=7 + k) for k in range(K)])
    rng = np.random.default_rng(0)
    lp = rng.integers(0, P, n_opp).astype(np.int32)
    po = np.where(np.arange(P)[None, :] == lp[:, None], -1, rng.integers(0, K, (n_opp, P))).astype(np.int32)
    ot.set_opponents(opp, None, n_opp, lp, po.reshape(-1), np.array([1], np.int32))
    pos0 = ot.rng_pos()
    ot.collect()
    v = ot.buffer("valid").reshape(T, N)
    assert v[:, n_opp:].min() == 1.0
    assert 0.3 < v[:, :n_opp].mean() < 0.7
    # the rollout drew N*A Gumbel words per step plus the seat reshuffles
    assert ot.rng_pos() >= pos0 + T * N * 7
    lp2, po2 = ot.opponent_envs(n_opp, P)
    assert np.all((po2.reshape(n_opp, P) == -1) == (np.arange(P)[None, :] == lp2[:, None]))
    ot.gae()
    m = ot.update()
    assert m["num_updates"] == 2 and np.isfinite(m["policy_loss"])
    ot.close()
