"""Parity at the sizes the bench runs (every benched kernel
oracle-checked at the size it runs), through libbppo.so against the oracle.

  * CfgA (configs/test.toml, --num-envs 8 --num-steps 128: 1x16 relu, 1 epoch x
    1 minibatch): the per-lane VALU rollout and k_minibatch<16,1,relu>, two
    updates;
  * the other VALU relu shapes (16x2, 32x1, 32x2, 64x1);
  * CfgB at full size (N=65536, T=128): rollout + return normalizer + obs
    normalizer + bootstrap + GAE, every buffer;
  * one CfgB ppo_update at N=8192 (B=1,048,576, minibatches of 262,144 rows):
    the MFMA minibatch kernel over all 256 blocks x 8 waves, the gradient slab
    reduction, the epoch advantage chunking and k_pack_rows;
  * Connect Four / Liar's Dice (MLP + CTDE) at N=1024: full GEMM tiles and
    split-K weight gradients reduced across blocks;
  * the opponent pool at N=49152 with 45056 opponent envs (thousands of games
    finishing in one step: the seat reshuffle's LDS word window refills, more
    than SEAT_CHUNK opponent envs, several envs per k_opp_group thread);
  * the error statuses the reference panics on (utils.rs:115-123, ppo.rs:363-366).
Tolerances: tests/parity_util.py."""
import ctypes as C

import numpy as np
import pytest

import bppo
import bppo._lib as L
import oracle_ffi as O
from parity_util import assert_metrics_close, assert_params_close, bits, cartpole_pair, cmp_cartpole_rollout

pytestmark = pytest.mark.gpu


def _update_pair(cfg, tr, ot, inject=True):
    """one ppo_update on both sides from identical GAE outputs"""
    if inject:
        tr.ctx.set_buffer("advantages", ot.buffer("advantages"))
        tr.ctx.set_buffer("returns", ot.buffer("returns"))
    start = tr.ctx.rng_pos()
    m = bppo.ppo_update(tr.ctx, bppo.schedule_get(cfg["learning_rate"], 0), bppo.schedule_get(cfg["entropy_coef"], 0))
    om = ot.update()
    assert tr.ctx.rng_pos() == ot.rng_pos()
    return m, om, start


def _last_perm(seed, start, B, epochs):
    r = O.new_rng(seed)
    r.word_pos = start
    for _ in range(epochs):
        p = np.arange(B, dtype=np.uint32)
        O.lib().or_shuffle_u32(C.byref(r), p, B)
    return p, r.word_pos


# ------------------------------------------------------------------ CfgA ---
def test_cfgA_test_preset_two_updates():
    """configs/test.toml at CfgA's --num-envs 8 --num-steps 128."""
    cfg, tr, ot = cartpole_pair(8, 128, preset="test")
    assert cfg["hidden_size"] == 16 and cfg["num_hidden"] == 1 and cfg["num_epochs"] == 1
    for rnd in range(2):
        if rnd:   # layered: the oracle's parameters and normalizer state
            tr.model.set_params(ot.params())
            tr.ctx.set_ret_norm(ot.ret_norm_state(), tr.ctx.ret_norm()[1])
        bppo.collect_rollouts(tr.ctx); ot.collect()
        cmp_cartpole_rollout(tr, ot)
        bppo.compute_gae(tr.ctx); ot.gae()
        m, om, _ = _update_pair(cfg, tr, ot)
        assert_metrics_close(m, om, values=ot.buffer("values"), returns=ot.buffer("returns"), advantages=ot.buffer("advantages"))
        assert_params_close(tr.model.get_params(), ot.params())
    tr.close(); ot.close()


@pytest.mark.parametrize("H,NL", [(16, 2), (32, 1), (32, 2), (64, 1)])
def test_relu_valu_shapes(H, NL):
    cfg, tr, ot = cartpole_pair(64, 32, hidden_size=H, num_hidden=NL, num_epochs=2)
    bppo.collect_rollouts(tr.ctx); ot.collect()
    cmp_cartpole_rollout(tr, ot)
    bppo.compute_gae(tr.ctx); ot.gae()
    m, om, _ = _update_pair(cfg, tr, ot)
    assert_metrics_close(m, om, values=ot.buffer("values"), returns=ot.buffer("returns"), advantages=ot.buffer("advantages"))
    assert_params_close(tr.model.get_params(), ot.params())
    tr.close(); ot.close()


# ------------------------------------------------------------- CfgB full ---
def test_cfgB_full_size_rollout_and_gae():
    """N=65536, T=128: the benched rollout, normalizers, bootstrap and GAE."""
    N, T = 65536, 128
    cfg, tr, ot = cartpole_pair(N, T)
    info = bppo.collect_rollouts(tr.ctx)
    n_eps = ot.collect()
    cmp_cartpole_rollout(tr, ot)
    assert info.episodes == n_eps
    m, v, c = tr.ctx.obs_norm()
    mo, vo, co = ot.obs_norm_state(5)
    assert c == co == N * T
    np.testing.assert_allclose(m, mo, rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(v, vo, rtol=1e-10)
    mvc, rets = tr.ctx.ret_norm()
    omvc, orets = ot.ret_norm_state(returns=True)
    assert np.array_equal(rets, orets)
    np.testing.assert_allclose(mvc, omvc, rtol=1e-12)
    # GAE on identical inputs is bit-exact (the bootstrap uses the updated obs stats)
    tr.ctx.set_buffer("rewards", ot.buffer("rewards"))
    bppo.compute_gae(tr.ctx); ot.gae()
    assert np.array_equal(bits(tr.buffer.advantages.reshape(-1)), bits(ot.buffer("advantages")))
    assert np.array_equal(bits(tr.buffer.returns.reshape(-1)), bits(ot.buffer("returns")))
    tr.close(); ot.close()


def test_cfgB_update_at_262k_row_minibatches():
    """CfgB's update (4 epochs x 4 minibatches, 2x64 relu MFMA kernel) at N=8192:
    every minibatch spans all 256 blocks x 8 waves."""
    N, T = 8192, 128
    cfg, tr, ot = cartpole_pair(N, T)
    bppo.collect_rollouts(tr.ctx); ot.collect()
    cmp_cartpole_rollout(tr, ot)
    bppo.compute_gae(tr.ctx); ot.gae()
    m, om, start = _update_pair(cfg, tr, ot)
    perm, end = _last_perm(cfg["seed"], start, N * T, cfg["num_epochs"])
    assert end == tr.ctx.rng_pos()
    assert np.array_equal(tr.ctx.buffer("perm", np.uint32), perm)
    assert_metrics_close(m, om, values=ot.buffer("values"), returns=ot.buffer("returns"), advantages=ot.buffer("advantages"))
    assert_params_close(tr.model.get_params(), ot.params())
    tr.close(); ot.close()


# ------------------------------------------------------ multi-player wide ---
WIDE = {"connect_four": (O.ENV_CONNECT_FOUR, 86, 7, 2, 0), "liars_dice": (O.ENV_LIARS_DICE, 270, 49, 4, 120)}


def wide_pair(env, N, T, seed=42, ctde=None, init_seed=5, **kw):
    kind, D, A, P, G = WIDE[env]
    if env == "connect_four":
        cfg = bppo.make_config("connect_four", num_envs=N, num_steps=T, seed=seed, **kw)
    else:
        cfg = bppo.make_config("liars_dice_ctde", num_envs=N, num_steps=T, seed=seed, **kw)
        if ctde is False:
            cfg.update(network_type="mlp", hidden_size=128)
    params = bppo.orthogonal_init(cfg, seed=init_seed)
    tr = bppo.Trainer(cfg, params=params)
    ocfg = O.train_cfg(env_kind=kind, num_envs=N, num_steps=T, seed=seed, hidden=cfg["hidden_size"],
                       num_hidden=cfg["num_hidden"], ctde=cfg["network_type"] == "ctde",
                       relu=cfg["activation"] == "relu", critic_hidden=cfg["critic_hidden_size"] or 0,
                       critic_num_hidden=cfg["critic_num_hidden"] or 0, normalize_obs=bool(cfg["normalize_obs"]),
                       normalize_returns=bool(cfg["normalize_returns"]), gamma=cfg["gamma"],
                       gae_lambda=cfg["gae_lambda"], lr=bppo.schedule_get(cfg["learning_rate"], 0),
                       ent_coef=bppo.schedule_get(cfg["entropy_coef"], 0),
                       reward_shaping=cfg["reward_shaping_coef"], num_epochs=cfg["num_epochs"],
                       num_minibatches=cfg["num_minibatches"], clip=cfg["clip_epsilon"],
                       value_coef=cfg["value_coef"], target_kl=cfg["target_kl"])
    ot = O.Trainer(ocfg, params)
    return cfg, tr, ot


def cmp_wide_rollout(env, tr, ot):
    kind, D, A, P, G = WIDE[env]
    b = tr.buffer
    assert np.array_equal(b.acting_players.reshape(-1), ot.buffer("players", np.int32))
    assert np.array_equal(bits(b.observations.reshape(-1)), bits(ot.buffer("obs")))
    assert np.array_equal(b.action_masks.reshape(-1), ot.buffer("masks"))
    if G and tr.model.is_ctde():
        assert np.array_equal(bits(b.privileged_obs.reshape(-1)), bits(ot.buffer("priv")))
    assert np.array_equal(b.actions.reshape(-1), ot.buffer("actions", np.int32))
    assert np.array_equal(bits(b.values.reshape(-1)), bits(ot.buffer("values")))
    assert np.array_equal(bits(b.log_probs.reshape(-1)), bits(ot.buffer("log_probs")))
    assert np.array_equal(b.dones.reshape(-1), ot.buffer("dones"))
    assert np.array_equal(bits(b.rewards.reshape(-1)), bits(ot.buffer("rewards")))
    assert np.array_equal(bits(b.all_rewards.reshape(-1)), bits(ot.buffer("all_rewards")))
    assert tr.ctx.rng_pos() == ot.rng_pos()


@pytest.mark.parametrize("env,N,T,ctde", [("connect_four", 1024, 8, None), ("liars_dice", 1024, 8, None),
                                          ("liars_dice", 1024, 8, False)])
def test_wide_at_full_gemm_tiles(env, N, T, ctde):
    """the configs' own epochs x minibatches (C4 6x4, LD 4x8) and target_kl"""
    cfg, tr, ot = wide_pair(env, N, T, ctde=ctde)
    bppo.collect_rollouts(tr.ctx); ot.collect()
    cmp_wide_rollout(env, tr, ot)
    bppo.compute_gae(tr.ctx); ot.gae()
    assert np.array_equal(bits(tr.buffer.advantages.reshape(-1)), bits(ot.buffer("advantages")))
    m, om, _ = _update_pair(cfg, tr, ot, inject=False)
    assert_metrics_close(m, om, values=ot.buffer("values"), returns=ot.buffer("returns"), advantages=ot.buffer("advantages"))
    assert_params_close(tr.model.get_params(), ot.params())
    tr.model.set_params(ot.params())
    bppo.collect_rollouts(tr.ctx); ot.collect()
    cmp_wide_rollout(env, tr, ot)
    tr.close(); ot.close()


# ------------------------------------------------------- opponent pool ---
def test_opponent_pool_at_scale():
    """49152 Connect Four envs, 45056 of them against a 3-model pool;
    compare valid flags, seats and the RNG position bit-exactly after a rollout
    in which thousands of opponent games finish per step, then one update over
    the learner rows."""
    env, N, T, n_opp, K = "connect_four", 49152, 24, 45056, 3
    cfg, tr, ot = wide_pair(env, N, T, hidden_size=64, num_epochs=1)
    kind, D, A, P, G = WIDE[env]
    rng = np.random.default_rng(11)
    params = np.stack([bppo.orthogonal_init(cfg, seed=200 + k) for k in range(K)])
    norms = [None, None, (rng.normal(size=D) * 0.1, (rng.random(D) + 0.5) * 500.0, 500.0)]
    lp = rng.integers(0, P, n_opp).astype(np.int32)
    po = np.full((n_opp, P), -1, np.int32)
    for p in range(P):
        sel = lp != p
        po[sel, p] = rng.integers(0, K, int(sel.sum()))
    co = rng.integers(0, K, P - 1).astype(np.int32)
    tr.ctx.set_opponents(params, norms, n_opp, lp, po, co)
    ot.set_opponents(params, norms, n_opp, lp, po.reshape(-1), co)
    bppo.collect_rollouts(tr.ctx); ot.collect()
    cmp_wide_rollout(env, tr, ot)
    assert np.array_equal(tr.ctx.buffer("valid"), ot.buffer("valid"))
    dlp, dpo = tr.ctx.opponent_envs()
    olp, opo = ot.opponent_envs(n_opp, P)
    assert np.array_equal(dlp, olp) and np.array_equal(dpo.reshape(-1), opo)
    # the large-N paths really ran: > 2048 opponent games (~2 seat words each, a
    # 4096-word LDS window) finished in one step
    d = ot.buffer("dones").reshape(T, N)[:, :n_opp]
    assert d.sum(axis=1).max() > 2100, d.sum(axis=1)
    bppo.compute_gae(tr.ctx); ot.gae()
    assert np.array_equal(bits(tr.buffer.advantages.reshape(-1)), bits(ot.buffer("advantages")))
    m, om, _ = _update_pair(cfg, tr, ot, inject=False)
    v = ot.buffer("valid") > 0.5
    assert_metrics_close(m, om, values=ot.buffer("values")[v], returns=ot.buffer("returns")[v], advantages=ot.buffer("advantages")[v])
    assert_params_close(tr.model.get_params(), ot.params())
    tr.close(); ot.close()


# --------------------------------------------------------- error statuses ---
def _sample(A, logits, masks, seed=7, pos=0):
    B = logits.shape[0]
    act = np.zeros(B, np.int32)
    lp = np.zeros(B, np.float32)
    st = L.lib().bppo_debug_sample(A, B, np.ascontiguousarray(logits, np.float32).ctypes.data,
                                   None if masks is None else np.ascontiguousarray(masks, np.uint8).ctypes.data,
                                   seed, 0, pos, act.ctypes.data, lp.ctypes.data)
    return st, act, lp


@pytest.mark.parametrize("A", [2, 7, 49])
def test_device_sampler_matches_oracle_and_reference_tests(A):
    rng = np.random.default_rng(A)
    B = 4096
    logits = rng.normal(0, 2, (B, A)).astype(np.float32)
    masks = (rng.random((B, A)) < 0.6).astype(np.uint8) if A > 2 else None
    if masks is not None:
        masks[np.arange(B), rng.integers(0, A, B)] = 1
    st, act, lp = _sample(A, logits, masks, seed=7, pos=1000)
    assert st == 0
    x = logits.copy()
    if masks is not None:
        x = np.where(masks > 0, x, np.float32(-np.inf)).astype(np.float32)
    r = O.new_rng(7)
    r.word_pos = 1000
    oa = np.zeros(B, np.int32)
    O.lib().or_sample_categorical(C.byref(r), np.ascontiguousarray(x), B, A, oa)
    assert np.array_equal(act, oa)
    olp = np.array([O.lib().or_log_prob(np.ascontiguousarray(x[i]), A, int(oa[i])) for i in range(B)], np.float32)
    assert np.array_equal(bits(lp), bits(olp))
    if masks is not None:   # utils.rs:257-278: a masked action is never sampled
        assert masks[np.arange(B), act].all()
    # utils.rs:158-168: a dominant logit (100) is always the argmax
    dom = np.zeros((64, A), np.float32)
    dom[:, min(2, A - 1)] = 100.0
    st, act, lp = _sample(A, dom, None)
    assert st == 0 and (act == min(2, A - 1)).all()
    # utils.rs:171-184: log-prob of a uniform row is ln(1/A)
    st, act, lp = _sample(A, np.zeros((8, A), np.float32), None)
    assert np.allclose(lp, np.log(1.0 / A), atol=1e-6)


def test_empty_mask_and_nonfinite_statuses():
    # utils.rs:246-254: a row without any valid action panics -> BPPO_ERR_EMPTY_MASK
    for A in (7, 49):
        m = np.ones((16, A), np.uint8)
        m[5] = 0
        st, _, _ = _sample(A, np.zeros((16, A), np.float32), m)
        assert st == L.ERR_EMPTY_MASK
    # ppo.rs:363-366: non-finite log-probs -> BPPO_ERR_NONFINITE
    lg = np.zeros((16, 7), np.float32)
    lg[3, :] = np.nan
    st, _, _ = _sample(7, lg, None)
    assert st == L.ERR_NONFINITE
    # the same statuses out of collect_rollouts with NaN parameters
    for preset, N in (("cartpole", 256), ("cartpole", 64), ("connect_four", 64)):
        kw = dict(hidden_size=32) if N == 64 and preset == "cartpole" else {}
        cfg = bppo.make_config(preset, num_envs=N, num_steps=4, **kw)
        tr = bppo.Trainer(cfg)
        p = tr.model.get_params()
        p[:] = np.nan
        tr.model.set_params(p)
        with pytest.raises(L.BppoError) as ei:
            bppo.collect_rollouts(tr.ctx)
        assert ei.value.status == L.ERR_NONFINITE, (preset, N, ei.value)
        tr.close()


@pytest.mark.parametrize("preset,N,T", [("cartpole", 4096, 64), ("connect_four", 256, 16)])
def test_train_step_equals_three_calls(preset, N, T):
    """bppo_train_step (rollout, bootstrap/GAE and update enqueued with one host wait)
    gives bit-for-bit the parameters, metrics, rollout info and RNG position of
    collect_rollouts + compute_gae + ppo_update; a NaN rollout still returns
    BPPO_ERR_NONFINITE."""
    cfg = bppo.make_config(preset, num_envs=N, num_steps=T, seed=11)
    a, b = bppo.Trainer(cfg, init_seed=3), bppo.Trainer(cfg, init_seed=3)
    try:
        for _ in range(3):
            ia = bppo.collect_rollouts(a.ctx)
            bppo.compute_gae(a.ctx)
            ma = bppo.ppo_update(a.ctx, 3e-4, 0.01)
            ib, mb = bppo.train_step(b.ctx, 3e-4, 0.01)
            assert (ia.episodes, ia.mean_return, ia.mean_length, ia.rng_word_pos) == \
                   (ib.episodes, ib.mean_return, ib.mean_length, ib.rng_word_pos)
            assert bits(a.model.get_params()).tolist() == bits(b.model.get_params()).tolist()
            for k, v in ma.items():
                assert bits(np.float32(v)) == bits(np.float32(mb[k])) or (np.isnan(v) and np.isnan(mb[k])), k
        p = b.model.get_params()
        p[:] = np.nan
        b.model.set_params(p)
        with pytest.raises(L.BppoError) as ei:
            bppo.train_step(b.ctx, 3e-4, 0.01)
        assert ei.value.status == L.ERR_NONFINITE
    finally:
        a.close()
        b.close()


@pytest.mark.parametrize("preset,N,T", [("cartpole", 4096, 64), ("connect_four", 256, 16)])
def test_train_steps_pipelined_equals_sequential(preset, N, T):
    """bppo_train_steps (each rollout enqueued behind the previous update) returns, for
    every iteration, the metrics and rollout info of sequential bppo_train_step calls,
    and leaves the same parameters and RNG position."""
    cfg = bppo.make_config(preset, num_envs=N, num_steps=T, seed=13)
    a, b = bppo.Trainer(cfg, init_seed=4), bppo.Trainer(cfg, init_seed=4)
    try:
        seq = [a.train_update() for _ in range(4)]
        pip, sums = b.train_updates(4, ("rollout", "update"))
        assert sums["rollout"] > 0 and sums["update"] > 0
        for ma, mb in zip(seq, pip):
            for k, v in ma.items():
                assert bits(np.float32(v)) == bits(np.float32(mb[k])) or (np.isnan(v) and np.isnan(mb[k])), k
        assert bits(a.model.get_params()).tolist() == bits(b.model.get_params()).tolist()
        pa, pb = C.c_uint64(), C.c_uint64()
        assert L.lib().bppo_rng_get(a.ctx.h, C.byref(pa)) == 0 and L.lib().bppo_rng_get(b.ctx.h, C.byref(pb)) == 0
        assert pa.value == pb.value
        # and the pipelined context carries on like the sequential one
        assert bits(np.float32(a.train_update()["policy_loss"])) == bits(np.float32(b.train_update()["policy_loss"]))
    finally:
        a.close()
        b.close()


def test_fused_row_packing_equals_pack_pass(monkeypatch):
    """The update rows written by the MFMA rollout and the segmented GAE give bit-for-bit
    the parameters and metrics of the k_pack_rows pass (BPPO_NO_FUSED_PACK=1)."""
    cfg = bppo.make_config("cartpole", num_envs=8192, num_steps=128, seed=21)
    a = bppo.Trainer(cfg, init_seed=6)
    monkeypatch.setenv("BPPO_NO_FUSED_PACK", "1")
    b = bppo.Trainer(cfg, init_seed=6)
    try:
        for _ in range(2):
            monkeypatch.delenv("BPPO_NO_FUSED_PACK", raising=False)
            ma = a.train_update()
            monkeypatch.setenv("BPPO_NO_FUSED_PACK", "1")
            mb = b.train_update()
            for k, v in ma.items():
                assert bits(np.float32(v)) == bits(np.float32(mb[k])) or (np.isnan(v) and np.isnan(mb[k])), k
        assert bits(a.model.get_params()).tolist() == bits(b.model.get_params()).tolist()
    finally:
        a.close()
        b.close()
