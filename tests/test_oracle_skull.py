"""Oracle Skull (oracle/skull.c) pinned by the reference's own Skull tests
(envs/skull.rs:1608-3285), ported one for one where they assert behaviour of
the hot path (transitions, masks, observation layout, rewards, placements,
privileged obs).  The skipped ones exercise the CLI (parse/describe/render) or
need a trained checkpoint.  Direct field writes below mirror the reference
tests' `env.field = ...` setups through the ctypes view of the state."""
import ctypes as C

import numpy as np
import pytest

import oracle_ffi as O

PLACE_SKULL, PLACE_ROSE, BID_BASE, PASS, REVEAL0 = 0, 1, 2, 26, 27
MAXP, OBS, ACT, PRIV, PRIV_EXACT = 6, 135, 33, 200, 103
PLACING, BIDDING, REVEALING = 0, 1, 2
L = O.lib


def new(n=4, seed=42):
    e = O.Skull()
    L().or_skull_new(C.byref(e), n, seed)
    L().or_skull_reset(C.byref(e), None)
    return e


def step(e, a, shaping=0.0):
    r = np.zeros(MAXP, np.float32)
    d, bad = C.c_int(), C.c_int()
    L().or_skull_step(C.byref(e), a, shaping, None, r, C.byref(d), C.byref(bad))
    return r, bool(d.value), bool(bad.value)


def mask(e):
    m = np.zeros(ACT, np.uint8)
    L().or_skull_mask(C.byref(e), m)
    return m.astype(bool)


def obs(e):
    o = np.zeros(OBS, np.float32)
    L().or_skull_get_obs(C.byref(e), o)
    return o


def priv(e):
    g = np.zeros(PRIV, np.float32)
    L().or_skull_priv(C.byref(e), g)
    return g


def placements(e):
    p = np.zeros(MAXP, np.int32)
    L().or_skull_placements(C.byref(e), p)
    return p[:e.n]


def final_rewards(e):
    r = np.zeros(MAXP, np.float32)
    L().or_skull_final_rewards(C.byref(e), r)
    return r[:e.n]


def alive(e, p):
    return p < e.n and (e.has_trap[p] or e.rose_count[p] > 0)


def coasters(e, p):
    return 0 if p >= e.n else e.has_trap[p] + e.rose_count[p]


def push(e, p, skull):
    e.stack[p][e.stack_len[p]] = 1 if skull else 0
    e.stack_len[p] += 1


def valid_actions(e):
    return [a for a, v in enumerate(mask(e)) if v]


def test_invalid_action_panics():                                          # skull.rs:1612-1620
    e = new()
    assert step(e, ACT + 1)[2]
    assert step(e, ACT + 10)[2]                                             # :2165-2173


def test_new_game_initial_state():                                         # :1647-1671
    e = new(4)
    for p in range(4):
        assert alive(e, p) and coasters(e, p) == 4 and e.has_trap[p] and e.rose_count[p] == 3
        assert e.stack_len[p] == 0
    for p in range(4, MAXP):
        assert not alive(e, p) and coasters(e, p) == 0
    assert e.phase == PLACING and not e.game_over and e.current_bid == 0 and e.current_bidder == -1


def test_relative_observation_symmetry():                                  # :1673-1713
    e = new(4)
    for p in range(4):
        push(e, p, False)
        e.wins[p] = p
    for cur in range(4):
        e.current = cur
        o = obs(e)
        assert o[8] == e.stack_len[cur] / 4
        assert o[32 + cur] == 1.0


def test_placing_masks():                                                  # :1715-1800
    e = new(4)
    m = mask(e)
    assert m[PLACE_SKULL] and m[PLACE_ROSE] and not m[PASS] and not m[BID_BASE:BID_BASE + 24].any()
    step(e, PLACE_SKULL)
    for _ in range(3):
        step(e, PLACE_ROSE)
    m = mask(e)
    assert not m[PLACE_SKULL] and m[PLACE_ROSE]
    # all three roses placed -> only the skull left
    e = new(4)
    player = e.current
    for _ in range(3):
        while e.current != player:
            step(e, PLACE_ROSE)
        step(e, PLACE_ROSE)
    while e.current != player:
        step(e, PLACE_ROSE)
    m = mask(e)
    assert m[PLACE_SKULL] and not m[PLACE_ROSE]
    # a card in the stack allows bids 1..total
    e = new(4)
    for _ in range(4):
        step(e, PLACE_ROSE)
    m = mask(e)
    assert m[BID_BASE] and m[BID_BASE + 3] and not m[BID_BASE + 4]


def test_placing_advances_to_next_player():                                # :1802-1814
    e = new(4)
    first = e.current
    step(e, PLACE_ROSE)
    assert e.current != first


def test_bidding():                                                        # :1816-1920
    e = new(4)
    for _ in range(4):
        step(e, PLACE_ROSE)
    first = e.current
    step(e, BID_BASE)
    assert e.phase == BIDDING and e.current_bid == 1 and e.current_bidder == first
    m = mask(e)
    assert m[BID_BASE + 1] and m[BID_BASE + 3] and not m[BID_BASE] and not m[BID_BASE + 4] and m[PASS]
    step(e, BID_BASE + 1)
    assert e.current_bid == 2 and e.current_bidder != first
    passing = e.current
    step(e, PASS)
    assert e.passed[passing]
    # max bid -> reveal
    e = new(4)
    for _ in range(4):
        step(e, PLACE_ROSE)
    step(e, BID_BASE + 3)
    assert e.phase == REVEALING
    # all others pass -> the bidder reveals
    e = new(4)
    for _ in range(4):
        step(e, PLACE_ROSE)
    bidder = e.current
    step(e, BID_BASE)
    for _ in range(3):
        step(e, PASS)
    assert e.phase == REVEALING and e.current_bidder == bidder


def test_revealing():                                                      # :1922-2030
    e = new(4)
    for _ in range(4):
        step(e, PLACE_ROSE)
    bidder = e.current
    step(e, BID_BASE + 3)
    m = mask(e)
    assert m[REVEAL0 + bidder] and all(not m[REVEAL0 + p] for p in range(4) if p != bidder)
    step(e, REVEAL0 + bidder)
    m = mask(e)
    assert all(m[REVEAL0 + p] for p in range(4) if p != bidder)
    for p in range(4):
        if p != bidder:
            step(e, REVEAL0 + p)
    assert e.wins[bidder] == 1 and e.phase == PLACING
    # the bidder's own skull ends the round and costs a coaster
    e = new(4)
    p0 = e.current
    step(e, PLACE_SKULL)
    for _ in range(3):
        step(e, PLACE_ROSE)
    step(e, BID_BASE + 3)
    step(e, REVEAL0 + p0)
    assert e.phase == PLACING and coasters(e, p0) < 4


def test_two_wins_ends_game():                                             # :2032-2055
    e = new(4)
    e.current = 0
    e.wins[0] = 1
    for p in range(4):
        push(e, p, False)
    e.phase, e.current_bid, e.current_bidder, e.must_reveal_own = REVEALING, 4, 0, 1
    for p in range(4):
        step(e, REVEAL0 + p)
    assert e.game_over and e.winner == 0


def test_last_player_standing_wins():                                      # :2057-2081
    e = new(4)
    for p in range(1, 4):
        e.has_trap[p] = 0
        e.rose_count[p] = 0
        e.elim_order[e.num_elim] = p
        e.num_elim += 1
    push(e, 0, False)
    e.phase, e.current, e.current_bid, e.current_bidder, e.must_reveal_own = REVEALING, 0, 1, 0, 1
    step(e, REVEAL0)
    assert e.game_over and e.winner == 0


def test_elimination_when_no_coasters():                                   # :2083-2107
    e = new(4)
    e.has_trap[0] = 1
    e.rose_count[0] = 0
    push(e, 0, True)
    e.phase, e.current, e.current_bid, e.current_bidder, e.must_reveal_own = REVEALING, 0, 1, 0, 1
    step(e, REVEAL0)
    assert not alive(e, 0) and 0 in list(e.elim_order[:e.num_elim])


def test_two_and_six_player_games():                                       # :2109-2140
    e = new(2)
    assert e.n == 2 and alive(e, 0) and alive(e, 1) and not alive(e, 2) and not alive(e, 3)
    for _ in range(2):
        step(e, PLACE_ROSE)
    step(e, BID_BASE + 1)
    m = mask(e)
    assert not m[REVEAL0 + 2] and not m[REVEAL0 + 3]
    e = new(6)
    assert all(alive(e, p) and coasters(e, p) == 4 for p in range(6))


def test_deterministic_seeding():                                          # :2142-2163
    a, b = new(4, 12345), new(4, 12345)
    assert a.current == b.current
    for _ in range(4):
        step(a, PLACE_ROSE)
        step(b, PLACE_ROSE)
    assert a.current == b.current and a.phase == b.phase


def test_action_after_game_over():                                         # :2175-2184
    e = new(4)
    e.game_over = 1
    r, d, _ = step(e, PLACE_ROSE)
    assert d and not r.any()


def test_reward_shaping_coefficient():                                     # :2186-2213
    e = new(4)
    push(e, 0, True)
    for p in range(1, 4):
        push(e, p, False)
    e.phase, e.current, e.current_bid, e.current_bidder, e.must_reveal_own = REVEALING, 0, 4, 0, 1
    r, _, _ = step(e, REVEAL0, shaping=0.1)
    assert (r != 0).sum() > 0
    # skull.rs:446-462 exactly: the failed bidder pays 1/4 of the coefficient
    assert r[0] == np.float32(0.0) - np.float32(0.25) * np.float32(0.1) and not r[1:].any()


def _play(e, pick, limit=10000):
    total = np.zeros(MAXP, np.float32)
    steps, done = 0, False
    while not done and steps < limit:
        va = valid_actions(e)
        if not va:
            break
        r, done, bad = step(e, pick(va, steps))
        assert not bad
        total += r
        steps += 1
    return total, done


def test_zero_sum_rewards():                                               # :2215-2255
    e = new(4)
    total, done = _play(e, lambda va, s: va[s % len(va)])
    if done:
        assert abs(total[:e.n].sum()) < 0.01


def test_observation_layout():                                             # :2257-2319
    e = new(3)
    o = obs(e)
    assert list(o[26:32]) == [1, 1, 1, 0, 0, 0]
    e = new(4)
    o = obs(e)
    assert o[38] == 1.0 and o[39] == 0.0 and o[40] == 0.0
    for _ in range(4):
        step(e, PLACE_ROSE)
    step(e, BID_BASE)
    step(e, BID_BASE + 1)
    assert e.hist_len == 2
    o = obs(e)
    assert o[OBS - 64: OBS - 64 + MAXP].sum() == 1.0


def test_random_games_complete_with_valid_placements():                    # :2321-2427, 3000-3035
    rng = np.random.default_rng(42)
    for seed in range(100):
        e = new(4, seed)
        total, done = _play(e, lambda va, s: va[rng.integers(len(va))])
        assert done and e.game_over
        pl = placements(e)
        if e.winner >= 0:
            assert pl[e.winner] == 1
        assert ((pl >= 1) & (pl <= e.n)).all()
        assert abs(final_rewards(e).sum()) < 0.001


def _setup(n, wins, coast, elim, winner):                                  # :2631-2654
    e = new(n)
    for p, w in enumerate(wins[:n]):
        e.wins[p] = w
    for p, (t, r) in enumerate(coast[:n]):
        e.has_trap[p] = int(t)
        e.rose_count[p] = r
    for k, p in enumerate(elim):
        e.elim_order[k] = p
    e.num_elim = len(elim)
    e.winner = -1 if winner is None else winner
    e.game_over = 1
    return e


@pytest.mark.parametrize("args,want", [                                    # :2656-2738, 3037-3081
    ((4, [2, 1, 0, 0], [(1, 2), (1, 3), (1, 3), (1, 2)], [], 0), [1, 2, 3, 4]),
    ((4, [2, 0, 0, 0], [(1, 3), (1, 3), (1, 2), (1, 1)], [], 0), [1, 2, 3, 4]),
    ((4, [2, 0, 0, 0], [(1, 3), (0, 0), (0, 0), (0, 0)], [2, 1], 0), [1, 3, 4, 2]),
    ((4, [2, 0, 0, 0], [(1, 3), (1, 3), (1, 3), (1, 2)], [], 0), [1, 2, 2, 4]),
    ((4, [2, 0, 0, 0], [(1, 3), (1, 3), (1, 3), (1, 3)], [], 0), [1, 2, 2, 2]),
    ((4, [2, 1, 0, 0], [(1, 3), (1, 1), (1, 3), (0, 0)], [3], 0), [1, 2, 3, 4]),
])
def test_placements(args, want):
    assert list(placements(_setup(*args))) == want


def test_tie_rewards():                                                    # :2740-2814
    r = final_rewards(_setup(4, [2, 0, 0, 0], [(1, 3), (1, 3), (1, 3), (1, 2)], [], 0))
    assert abs(r[0] - 1.0) < 1e-3 and abs(r[1] - r[2]) < 1e-3 and abs(r[1]) < 1e-3
    assert abs(r[3] + 1.0) < 1e-3 and abs(r.sum()) < 1e-3
    r = final_rewards(_setup(4, [2, 0, 0, 0], [(1, 3)] * 4, [], 0))
    want = (1.0 / 3.0 - 1.0 / 3.0 - 1.0) / 3.0
    assert abs(r[0] - 1.0) < 1e-3 and all(abs(x - want) < 1e-3 for x in r[1:]) and abs(r.sum()) < 1e-3
    # skull.rs:421-440 in f32: 1 - 2 (p - 1) / (n - 1), summed over the group, / size
    f = np.float32
    t = (f(1) - f(2) * (f(2) - f(1)) / (f(4) - f(1))) + (f(1) - f(2) * (f(3) - f(1)) / (f(4) - f(1)))
    assert r.dtype == np.float32
    r2 = final_rewards(_setup(4, [2, 0, 0, 0], [(1, 3), (1, 3), (1, 3), (1, 2)], [], 0))
    assert r2[1] == t / f(2)


def test_privileged_obs():                                                 # :3083-3129
    for n in (4, 6):
        e = new(n)
        g = priv(e)
        assert g.shape == (PRIV,) and not g[PRIV_EXACT:].any()
    e = new(4)
    g = priv(e)
    assert list(g[:3]) == [1, 0, 0] and g[5] == 0.0 and g[6] == -1.0
    assert g[37] == 0.0 and list(g[38:43]) == [0, 0, 1, 0, 0]
    assert list(g[43:53]) == [1, 0, 1, 1, 1, 0, 0, 0, 0, 0]                 # seat 0 at reset
    assert not g[43 + 10 * 4: 103].any()                                    # seats 4, 5 do not exist


def test_bidding_end_transitions():                                        # :3131-3238
    e = new(2)
    step(e, PLACE_ROSE)
    step(e, PLACE_ROSE)
    step(e, BID_BASE)
    assert e.phase == BIDDING and e.current == 1
    step(e, PASS)
    assert e.phase == REVEALING and e.current_bidder == 0 and mask(e).any()
    e = new(3)
    for _ in range(3):
        step(e, PLACE_ROSE)
    step(e, BID_BASE)
    assert e.phase == BIDDING and e.current == 1
    step(e, PASS)
    assert e.phase == BIDDING and e.current == 2
    step(e, PASS)
    assert e.phase == REVEALING
    e = new(3)
    for _ in range(6):
        step(e, PLACE_ROSE)
    step(e, BID_BASE)
    step(e, PASS)
    step(e, PASS)
    assert e.phase == REVEALING and mask(e)[REVEAL0]


def test_eliminated_bidder_starts_valid_player():                          # :3240-3285
    e = new(4)
    e.has_trap[0] = 1
    e.rose_count[0] = 0
    push(e, 0, True)
    for p in (1, 2, 3):
        push(e, p, False)
    e.phase, e.current, e.current_bidder, e.current_bid, e.must_reveal_own = REVEALING, 0, 0, 4, 1
    _, done, _ = step(e, REVEAL0)
    assert not done and not alive(e, 0) and alive(e, e.current) and e.current != 0 and mask(e).any()


def test_vecenv_pads_rewards_to_six_players():                             # env.rs:474-478
    v = L().or_vecenv_new_np(O.ENV_SKULL, 4, 7, 3)
    try:
        N = 4
        rng = np.random.default_rng(0)
        for _ in range(300):
            m = np.zeros(N * ACT, np.uint8)
            L().or_vecenv_get_masks(v, m)
            a = np.array([rng.choice(np.flatnonzero(m[i * ACT:(i + 1) * ACT])) for i in range(N)], np.int32)
            r = np.zeros(N * MAXP, np.float32)
            d = np.zeros(N, np.uint8)
            L().or_vecenv_step(v, a, np.zeros(N * OBS, np.float32), r, d, None, 0)
            assert not r.reshape(N, MAXP)[:, 3:].any()
        assert L().or_vecenv_invalid(v) == 0
    finally:
        L().or_vecenv_free(v)
