"""GAE known-answer tests, ported from the reference's own tests
(ppo.rs:2146-2734), run against the oracle's restatement (oracle/ppo.c)."""
import numpy as np
import pytest

import oracle_ffi as O

G, L = 0.99, 0.95


def f32(x):
    return np.array(x, np.float32)


def mp(dones, players, all_rewards, values, lvpp, gamma=G, lam=L):
    d = f32(dones)
    T, N = d.shape
    adv, ret = O.compute_gae_mp(f32(all_rewards), np.array(players, np.int32), d, f32(values),
                                f32(lvpp), gamma, lam)
    return adv.reshape(-1), ret


def test_gae_single_player_nonzero():            # ppo.rs:2146-2177
    adv, ret = O.compute_gae(np.ones((4, 2), np.float32), np.zeros((4, 2), np.float32),
                             np.full((4, 2), 0.5, np.float32), f32([0.5, 0.5]), G, L)
    assert np.any(np.abs(adv) > 0.01)
    assert np.allclose(ret, adv + 0.5)


def test_gae_single_player_exact_recurrence():
    rng = np.random.default_rng(0)
    T, N = 16, 5
    r = rng.normal(size=(T, N)).astype(np.float32)
    d = (rng.random((T, N)) < 0.2).astype(np.float32)
    v = rng.normal(size=(T, N)).astype(np.float32)
    lv = rng.normal(size=N).astype(np.float32)
    adv, ret = O.compute_gae(r, d, v, lv, G, L)
    last = np.zeros(N, np.float64)
    for t in reversed(range(T)):
        nv = lv if t == T - 1 else v[t + 1]
        delta = G * nv * (1 - d[t]) + r[t] - v[t]
        last = delta + G * L * (1 - d[t]) * last
        np.testing.assert_allclose(adv[t], last, rtol=1e-5, atol=1e-6)


def test_same_player_consecutive():               # ppo.rs:2227-2283
    adv, _ = mp([[0.0], [1.0]], [[0], [0]], [[[0.0, 0.0]], [[1.0, 0.0]]], [[0.5], [0.8]], [[0.8, 0.0]])
    s1 = 1.0 - 0.8
    assert abs(adv[1] - s1) < 1e-5
    assert abs(adv[0] - ((G * 0.8 - 0.5) + G * L * s1)) < 1e-5


def test_different_player_terminal_no_bleed():    # ppo.rs:2286-2342
    adv, _ = mp([[0.0], [1.0], [1.0]], [[0], [1], [0]],
                [[[0.0, 0.0]], [[-1.0, 1.0]], [[1.0, -1.0]]], [[0.0], [0.0], [0.9]], [[0.9, 0.0]])
    assert adv[0] < -0.9


def test_reward_attribution_boundary():            # ppo.rs:2345-2396
    adv, _ = mp([[0.0], [1.0], [0.0], [1.0]], [[0], [1], [0], [1]],
                [[[0.0, 0.0]], [[-1.0, 1.0]], [[0.0, 0.0]], [[10.0, -10.0]]], np.zeros((4, 1)),
                [[0.0, 0.0]])
    assert adv[0] < 0.0 and adv[1] > 0.0 and adv[2] > 5.0


def test_three_players():                          # ppo.rs:2399-2443
    adv, _ = mp([[0.0], [0.0], [1.0]], [[0], [1], [2]],
                [[[0.0, 0.0, 0.0]], [[0.0, 0.0, 0.0]], [[-1.0, -1.0, 2.0]]], np.zeros((3, 1)),
                [[0.0, 0.0, 0.0]])
    assert adv[0] < 0 and adv[1] < 0 and adv[2] > 0


def test_long_alternating_episode():               # ppo.rs:2446-2534
    adv, _ = mp([[0.0]] * 5 + [[1.0]], [[0], [1], [0], [1], [0], [1]],
                [[[0.0, 0.0]]] * 5 + [[[1.0, -1.0]]], [[0.3], [0.6], [0.5], [0.4], [0.7], [0.2]],
                [[0.7, 0.2]])
    assert adv[0] > 0 and adv[2] > 0 and adv[4] > 0
    assert adv[1] < 0 and adv[3] < 0 and adv[5] < 0
    assert abs(adv[0]) > abs(adv[2])


def test_different_player_terminal_exact():        # ppo.rs:2537-2576
    adv, _ = mp([[0.0], [1.0]], [[0], [1]], [[[0.0, 0.0]], [[-1.0, 1.0]]], np.zeros((2, 1)),
                [[0.0, 0.0]])
    assert abs(adv[1] - 1.0) < 1e-5
    assert abs(adv[0] + 1.0) < 1e-5


def test_same_player_across_boundary():            # ppo.rs:2579-2635
    adv, _ = mp([[0.0], [1.0], [1.0]], [[0], [0], [0]],
                [[[0.0, 0.0]], [[-1.0, 0.0]], [[10.0, 0.0]]], [[0.0], [0.0], [5.0]], [[5.0, 0.0]])
    assert abs(adv[2] - 5.0) < 1e-5
    assert abs(adv[1] + 1.0) < 1e-5
    assert abs(adv[0] + 0.99 * 0.95) < 1e-5


def test_multiple_envs_isolated():                 # ppo.rs:2638-2691
    adv, _ = mp([[0.0, 0.0], [1.0, 0.0]], [[0, 0], [1, 1]],
                [[[0.0, 0.0], [0.0, 0.0]], [[-1.0, 1.0], [0.0, 0.0]]], [[0.5, 0.3], [0.4, 0.4]],
                [[0.5, 0.4], [0.3, 0.5]])
    assert abs(adv[2] - 0.6) < 1e-5
    assert abs(adv[3] - (0.99 * 0.5 - 0.4)) < 1e-4


def test_no_done_flags():                          # ppo.rs:2694-2734
    adv, _ = mp(np.zeros((3, 1)), [[0], [1], [0]], [[[0.1, 0.0]], [[0.0, 0.2]], [[0.3, 0.0]]],
                [[0.5], [0.5], [0.5]], [[0.5, 0.6]])
    assert np.all(np.isfinite(adv))
    assert abs(adv[2] - (0.3 + 0.99 * 0.5 - 0.5)) < 1e-4


def test_explained_variance_cases():               # ppo.rs:2776-2830
    ev = lambda v, r: O.lib().or_explained_variance(f32(v), f32(r), len(v))
    assert abs(ev([1, 2, 3, 4], [1, 2, 3, 4]) - 1.0) < 1e-5
    assert ev([0, 0, 0, 0], [1, 2, 3, 4]) < 1.0
    assert abs(ev([1, 2, 3, 4], [2.5] * 4)) < 1e-5
    assert abs(ev([1.0], [1.0])) < 1e-5
    assert abs(O.lib().or_explained_variance(f32([0]), f32([0]), 0)) < 1e-5
    e = ev([1, 2.5, 3, 4.5], [1, 2, 3, 4])
    assert 0 < e < 1


@pytest.mark.parametrize("B,M,expected", [(100, 4, [25] * 4), (893, 4, [224, 223, 223, 223]),
                                          (14, 4, [4, 4, 3, 3]), (3, 4, [1, 1, 1]), (1, 4, [1]),
                                          (0, 4, [])])
def test_minibatch_split(B, M, expected):           # ppo.rs:2946-3038
    import bppo.host as H
    assert H.minibatch_sizes(B, M) == expected


def test_explained_variance_f32_sequential_restatement():
    """The oracle's f32 sums (ppo.rs:1268-1294) equal a second restatement bit
    for bit, at a size where f32 sequential drift is visible (vs f64)."""
    from parity_util import ev_f32_sequential, ev_f64
    rng = np.random.default_rng(3)
    n = 300_000
    r = rng.normal(20.0, 5.0, n).astype(np.float32)
    v = (r + rng.normal(0.0, 4.0, n)).astype(np.float32)
    o = O.lib().or_explained_variance(v, r, n)
    assert np.float32(o) == ev_f32_sequential(v, r)
    assert abs(o - ev_f64(v, r)) < 0.05
