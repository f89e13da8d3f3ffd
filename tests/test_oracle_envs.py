"""Environment rules against the reference's own env tests
(cartpole.rs:325-443, connect_four.rs:332-637, liars_dice.rs:746-1595,
env.rs:520-789, envs/mod.rs:160-165)."""
import ctypes as C

import numpy as np

import oracle_ffi as O

L = O.lib


def cp(seed=42):
    e = O.CartPole()
    L().or_cartpole_new(C.byref(e), seed)
    return e


def cp_step(e, a):
    obs = np.zeros(5, np.float32)
    r = C.c_float(); d = C.c_int()
    L().or_cartpole_step(C.byref(e), a, obs, C.byref(r), C.byref(d))
    return obs, r.value, bool(d.value)


def test_cartpole_reset_and_step():
    e = cp()
    obs = np.zeros(5, np.float32)
    L().or_cartpole_reset(C.byref(e), obs)
    assert np.all(np.abs(obs[:4]) < 0.1) and obs[4] == 0.0
    o, r, d = cp_step(e, 1)
    assert r == 1.0 and not d and abs(o[4] - 0.002) < 0.001


def test_cartpole_reset_draws_four_gen_range_words():
    e = cp(42)
    # new() resets once: 4 words consumed, values = gen_range(-0.05..0.05) of words 0-3
    w = O.stdrng_words(42, 4)
    v = ((w >> 9) | 0x3F800000).view(np.float32) - np.float32(1)
    exp = (v * np.float32(0.1) + np.float32(-0.05)).astype(np.float32)
    assert np.array_equal(np.array([e.x, e.x_dot, e.theta, e.theta_dot], np.float32), exp)
    assert e.rng.word_pos == 4


def test_cartpole_terminations():
    e = cp(); e.theta = 12 * np.pi / 180 + 0.1
    assert cp_step(e, 0)[2]
    e = cp(); e.x = 2.5
    o, r, d = cp_step(e, 0)
    assert d and r == 0.0
    e = cp(); e.steps = 499
    o, r, d = cp_step(e, 0)
    assert d and r == 1.0                       # truncation at 500 keeps reward 1


def test_cartpole_push_direction_and_reproducible():
    a = cp(); a.x = 0; a.x_dot = 0
    b = cp(); b.x = 0; b.x_dot = 0
    cp_step(a, 1); cp_step(b, 0)
    assert a.x > b.x
    x, y = cp(7), cp(7)
    for k in range(50):
        ox, rx, dx = cp_step(x, k % 2)
        oy, ry, dy = cp_step(y, k % 2)
        assert np.array_equal(ox, oy) and rx == ry and dx == dy
    assert (x.x, x.theta) == (y.x, y.theta)


def c4():
    e = O.ConnectFour()
    L().or_c4_new(C.byref(e))
    return e


def c4_step(e, a):
    obs = np.zeros(86, np.float32); r = np.zeros(2, np.float32); d = C.c_int()
    L().or_c4_step(C.byref(e), a, obs, r, C.byref(d))
    return obs, r, bool(d.value)


def test_c4_vertical_win_and_rewards():
    e = c4()
    for a in (0, 1, 0, 1, 0, 1):
        o, r, d = c4_step(e, a)
        assert not d
    o, r, d = c4_step(e, 0)
    assert d and r[0] == 1.0 and r[1] == -1.0


def test_c4_horizontal_win_player2():
    e = c4()
    for a in (0, 1, 0, 2, 0, 3, 5):
        o, r, d = c4_step(e, a)
        assert not d
    o, r, d = c4_step(e, 4)
    assert d and r[1] == 1.0 and r[0] == -1.0


def test_c4_mask_obs_and_invalid():
    e = c4()
    for _ in range(6):
        c4_step(e, 3)
    m = np.zeros(7, np.uint8)
    L().or_c4_mask(C.byref(e), m)
    assert m.tolist() == [1, 1, 1, 0, 1, 1, 1]
    obs = np.zeros(86, np.float32)
    L().or_c4_get_obs(C.byref(e), obs)
    assert obs[:84].sum() == 6 and obs[84] == 1.0 and obs[85] == 0.0
    # column 3 bottom (row 5) holds player 1 -> P1 plane index 5*7+3
    assert obs[5 * 7 + 3] == 1.0 and obs[42 + 4 * 7 + 3] == 1.0
    o, r, d = c4_step(e, 3)
    assert d and np.all(r == 0)


def test_c4_draw_zero_rewards():
    e = c4()
    # fill the board column-pair-wise without four in a row
    seq = [0, 1, 0, 1, 0, 1, 1, 0, 1, 0, 1, 0, 2, 3, 2, 3, 2, 3, 3, 2, 3, 2, 3, 2,
           4, 5, 4, 5, 4, 5, 5, 4, 5, 4, 5, 4, 6, 6, 6, 6, 6, 6]
    for i, a in enumerate(seq):
        o, r, d = c4_step(e, a)
        if d:
            break
    assert d and i == 41 and np.all(r == 0.0)


def ld(seed=1):
    e = O.LiarsDice()
    L().or_ld_new(C.byref(e), seed)
    return e


def ld_step(e, a, shaping=0.0):
    obs = np.zeros(270, np.float32); r = np.zeros(4, np.float32); d = C.c_int()
    L().or_ld_step(C.byref(e), a, shaping, obs, r, C.byref(d))
    return obs, r, bool(d.value)


def test_ld_initial_mask_and_dims():
    e = ld()
    m = np.zeros(49, np.uint8)
    L().or_ld_mask(C.byref(e), m)
    assert m[48] == 0 and m[:48].sum() == 48     # any bid, no call
    g = np.zeros(120, np.float32)
    L().or_ld_priv(C.byref(e), g)
    assert np.all(g[110:] == 0)


def test_ld_bid_then_mask_and_call_resolution():
    e = ld(3)
    ld_step(e, (2 - 1) * 6 + (3 - 1))            # bid two 3s
    m = np.zeros(49, np.uint8)
    L().or_ld_mask(C.byref(e), m)
    assert m[48] == 1 and m[(2 - 1) * 6 + (3 - 1)] == 0 and m[(2 - 1) * 6 + (4 - 1)] == 1
    dice = np.array([[e.dice[p][d] for d in range(2)] for p in range(4)])
    count = int(np.sum((dice == 3) | (dice == 1)))
    caller = e.current
    o, r, d = ld_step(e, 48, shaping=0.05)
    loser = 0 if count < 2 else caller          # caller correct -> bidder (player 0) loses
    assert e.num_dice[loser] == 1
    assert not d and all(abs(x - 0.05) < 1e-7 for x in r)


def test_ld_wild_ones():
    e = ld(5)
    e.dice[0][0], e.dice[0][1] = 1, 1
    e.dice[1][0], e.dice[1][1] = 5, 5
    e.dice[2][0], e.dice[2][1] = 2, 3
    e.dice[3][0], e.dice[3][1] = 4, 6
    ld_step(e, (4 - 1) * 6 + (5 - 1))            # bid four 5s: 2 fives + 2 wild ones = 4
    o, r, d = ld_step(e, 48)                     # caller (player 1) wrong -> caller loses
    assert e.num_dice[1] == 1


def test_ld_game_end_placement_rewards():
    e = ld(9)
    # leave players 0 and 1 with one die each, eliminate 2 and 3
    e.num_dice[2] = 0; e.num_dice[3] = 0
    e.elim_order[0] = 2; e.elim_order[1] = 3; e.num_elim = 2
    e.num_dice[1] = 1; e.num_dice[0] = 1
    e.dice[0][0] = 6; e.dice[1][0] = 6
    ld_step(e, (2 - 1) * 6 + (6 - 1))            # P0 bids two 6s (true)
    o, r, d = ld_step(e, 48)                     # P1 calls, wrong -> P1 eliminated
    assert d
    assert r.tolist() == [np.float32(1.0), np.float32(0.33), np.float32(-1.0), np.float32(-0.33)]


def test_vecenv_auto_reset_and_double_reset():
    N = 4
    v = L().or_vecenv_new(O.ENV_CARTPOLE, N, 100)
    # env i = CartPole::new(100+i) (reset #1, words 0-3) then VecEnv reset #2 (words 4-7)
    obs = np.zeros(N * 5, np.float32)
    L().or_vecenv_get_obs(v, obs)
    for i in range(N):
        w = O.stdrng_words(100 + i, 8)[4:8]
        x = ((w >> 9) | 0x3F800000).view(np.float32) - np.float32(1)
        exp = (x * np.float32(0.1) + np.float32(-0.05)).astype(np.float32)
        assert np.array_equal(obs[i * 5:i * 5 + 4], exp)
    acts = np.zeros(N, np.int32)
    rw = np.zeros(N, np.float32); dn = np.zeros(N, np.uint8)
    eps = (O.Episode * 64)()
    total = 0
    for s in range(200):
        total += L().or_vecenv_step(v, acts, obs, rw, dn, eps, 64)
        if dn.any():
            i = int(np.argmax(dn))
            assert obs[i * 5 + 4] == 0.0         # reset obs replaces terminal obs
            break
    L().or_vecenv_free(v)
    assert total >= 1


def test_obs_dims():                               # envs/mod.rs:160-165
    for kind, dim in ((O.ENV_CARTPOLE, 5), (O.ENV_CONNECT_FOUR, 86), (O.ENV_LIARS_DICE, 270)):
        v = L().or_vecenv_new(kind, 1, 0)
        lib = L()
        lib.or_vecenv_obs_dim.restype = C.c_int
        lib.or_vecenv_obs_dim.argtypes = [C.c_void_p]
        assert lib.or_vecenv_obs_dim(v) == dim
        L().or_vecenv_free(v)
