"""The oracle's W-rank update (or_trainers_update, oracle/ppo.c), which pins libbppo's
W > 1 semantics in tests/test_gpu_multirank.py, checked on CPU:
  * W = 2 ranks holding IDENTICAL shards take exactly the W = 1 step (the summed
    gradient g + g scaled by 1/2 is g bit for bit), so their parameters equal the
    single-rank run's bit for bit;
  * with distinct shards (env seeds seed + r*N + i, main-RNG stream r) the ranks'
    rollouts differ, their parameters stay identical, and the step is the mean of
    the two single-rank gradients: it equals the update of one rank whose
    minibatch gradient is replaced by that mean (checked through the first Adam step,
    where Adam's update depends on the gradient alone)."""
import numpy as np

import bppo
import oracle_ffi as O
from parity_util import oracle_train_cfg


def _cfg(**kw):
    return bppo.make_config("cartpole", num_envs=32, num_steps=16, **kw)


def test_identical_shards_equal_single_rank():
    cfg = _cfg()
    params = bppo.orthogonal_init(cfg, seed=3)
    solo = O.Trainer(oracle_train_cfg(cfg), params)
    pair = [O.Trainer(oracle_train_cfg(cfg), params) for _ in range(2)]
    for _ in range(2):
        solo.collect(); solo.gae()
        for t in pair:
            t.collect(); t.gae()
        m = solo.update()
        ms = O.Trainer.update_ranks(pair)
        for t in pair:
            assert np.array_equal(t.params().view(np.uint32), solo.params().view(np.uint32))
            assert t.rng_pos() == solo.rng_pos()
        for k in ("policy_loss", "value_loss", "approx_kl", "value_error_max", "adv_mean_raw"):
            assert abs(ms[0][k] - m[k]) <= 1e-6 * max(1.0, abs(m[k])), k
    for t in [solo] + pair:
        t.close()


def test_distinct_shards_share_one_step():
    cfg = _cfg(num_epochs=1, num_minibatches=1)
    params = bppo.orthogonal_init(cfg, seed=4)
    ranks = [O.Trainer(oracle_train_cfg(cfg, rank=r, world=2), params) for r in range(2)]
    solos = [O.Trainer(oracle_train_cfg(cfg, rank=r, world=2), params) for r in range(2)]
    for t in ranks + solos:
        t.collect(); t.gae()
    a0, a1 = ranks[0].buffer("actions", np.int32), ranks[1].buffer("actions", np.int32)
    assert not np.array_equal(a0, a1)                       # distinct env seeds / streams
    # rank 1's stream differs from the reference's stream 0
    ref = O.Trainer(oracle_train_cfg(cfg), params)
    ref.collect()
    assert not np.array_equal(ref.buffer("actions", np.int32), a1)
    ms = O.Trainer.update_ranks(ranks)
    assert np.array_equal(ranks[0].params().view(np.uint32), ranks[1].params().view(np.uint32))
    assert ms[0]["policy_loss"] == ms[1]["policy_loss"]
    # one epoch x one minibatch: each solo rank's first Adam step moves a parameter by
    # -lr * m1c / (sqrt(m2c) + eps) with m1c = g, m2c = g^2 after bias correction, i.e.
    # -lr * sign(g) (|g| >> eps); the W = 2 step moves by -lr * sign(g0 + g1): where the
    # two ranks' steps agree in sign, the shared step agrees with both
    for t in solos:
        t.update()
    d0 = solos[0].params() - params
    d1 = solos[1].params() - params
    dw = ranks[0].params() - params
    agree = (np.sign(d0) == np.sign(d1)) & (np.abs(d0) > 1e-6) & (np.abs(d1) > 1e-6)
    assert agree.sum() > 100
    assert np.array_equal(np.sign(dw[agree]), np.sign(d0[agree]))
    for t in ranks + solos + [ref]:
        t.close()


def test_shuffle_windows_positions():
    """shuffle_windows: epoch e shuffles from S + e * (2B + 2^20) and the update ends at
    S + epochs * (2B + 2^20); epoch 0 is the reference's shuffle, so with one epoch the
    parameters equal the sequential run's, only the RNG position after the update moves"""
    cfg = _cfg(num_epochs=1)
    params = bppo.orthogonal_init(cfg, seed=5)
    seq = O.Trainer(oracle_train_cfg(cfg), params)
    win = O.Trainer(oracle_train_cfg(dict(cfg, shuffle_windows=True)), params)
    B = cfg["num_envs"] * cfg["num_steps"]
    for t in (seq, win):
        t.collect(); t.gae()
    S = win.rng_pos()
    assert seq.rng_pos() == S
    seq.update(); win.update()
    assert np.array_equal(seq.params().view(np.uint32), win.params().view(np.uint32))
    assert win.rng_pos() == S + (2 * B + (1 << 20))
    assert seq.rng_pos() < win.rng_pos()
    # four epochs: epochs 1..3 shuffle from their windows, so the run departs from the
    # sequential one
    cfg4 = _cfg(num_epochs=4)
    a = O.Trainer(oracle_train_cfg(cfg4), params)
    b = O.Trainer(oracle_train_cfg(dict(cfg4, shuffle_windows=True)), params)
    for t in (a, b):
        t.collect(); t.gae(); t.update()
    assert b.rng_pos() == S + 4 * (2 * B + (1 << 20))
    assert not np.array_equal(a.params().view(np.uint32), b.params().view(np.uint32))
    for t in (seq, win, a, b):
        t.close()


def test_popart_two_ranks_absorb_both_ranks_returns():
    """PopArt at W = 2 (normalize_values): each rank's running statistics absorb rank 0's
    returns, then rank 1's (a sequential Welford over both), so both ranks rescale the
    value head the same way and keep identical parameters"""
    cfg = _cfg(num_epochs=1, num_minibatches=2, normalize_values=True)
    params = bppo.orthogonal_init(cfg, seed=6)
    ranks = [O.Trainer(oracle_train_cfg(cfg, rank=r, world=2), params) for r in range(2)]
    for t in ranks:
        t.collect(); t.gae()
    rets = [t.buffer("returns").astype(np.float64) for t in ranks]
    O.Trainer.update_ranks(ranks)
    st = [t.popart() for t in ranks]
    assert np.array_equal(st[0], st[1])
    n, mean, m2 = 0.0, 0.0, 0.0
    for x in np.concatenate(rets):               # the sequential Welford, rank 0's rows first
        n += 1.0
        d = x - mean
        mean += d / n
        m2 += d * (x - mean)
    assert st[0][2] == n and st[0][0] == mean and st[0][1] == m2
    assert np.array_equal(ranks[0].params().view(np.uint32), ranks[1].params().view(np.uint32))
    for t in ranks:
        t.close()


def test_opponent_pool_two_ranks_lockstep():
    """opponent pools at W = 2: the ranks' learner-row counts differ (their own seats), each
    cuts its rows into num_minibatches of its own sizes and the slots run in lockstep; both
    ranks end with identical parameters, and W = 2 ranks with IDENTICAL shards and seats
    equal the single-rank opponent-pool update bit for bit"""
    cfg = bppo.make_config("connect_four", num_envs=24, num_steps=8, hidden_size=32, num_epochs=2,
                           num_minibatches=3)
    params = bppo.orthogonal_init(cfg, seed=8)
    K, n_opp, P = 2, 20, 2
    pool = np.stack([bppo.orthogonal_init(cfg, seed=40 + k) for k in range(K)])

    def seats(seed, n):
        rng = np.random.default_rng(seed)
        lp = rng.integers(0, P, n).astype(np.int32)
        po = np.full((n, P), -1, np.int32)
        for e in range(n):
            po[e, 1 - lp[e]] = rng.integers(0, K)
        return n, lp, po.reshape(-1), rng.integers(0, K, P - 1).astype(np.int32)

    ranks = [O.Trainer(oracle_train_cfg(cfg, rank=r, world=2), params) for r in range(2)]
    for r, t in enumerate(ranks):
        t.set_opponents(pool, [None] * K, *seats(r, n_opp - 8 * r))
        t.collect(); t.gae()
    rows = [int((t.buffer("valid") > 0.5).sum()) for t in ranks]
    assert rows[0] != rows[1]
    O.Trainer.update_ranks(ranks)
    assert np.array_equal(ranks[0].params().view(np.uint32), ranks[1].params().view(np.uint32))
    # identical shards and seats at W = 2 = the single-rank update
    solo = O.Trainer(oracle_train_cfg(cfg), params)
    pair = [O.Trainer(oracle_train_cfg(cfg), params) for _ in range(2)]
    for t in [solo] + pair:
        t.set_opponents(pool, [None] * K, *seats(5, n_opp))
        t.collect(); t.gae()
    solo.update()
    O.Trainer.update_ranks(pair)
    for t in pair:
        assert np.array_equal(t.params().view(np.uint32), solo.params().view(np.uint32))
    for t in ranks + pair + [solo]:
        t.close()
