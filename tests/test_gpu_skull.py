"""Skull (envs/skull.rs) on the device vs the oracle restatement (oracle/skull.c,
pinned by the reference's own Skull tests in tests/test_oracle_skull.py).

Bit-exact: VecEnv transitions for 2/4/6 players (observations, privileged obs,
masks, acting players, rewards incl. shaping and tie-averaged placement
rewards, dones, episode records, the env RNG's lose_coaster draws), rollouts
(masked Gumbel-max actions, log-probs, values), multi-player GAE over the 6-seat
player axis.  The update: every UpdateMetrics field within 1e-5 relative and
parameters within rtol 1e-4 / atol 2e-5 (tests/parity_util.py), as for the
other multi-player envs.  An action outside the mask (a panic in the reference)
is BPPO_ERR_ARG."""
import numpy as np
import pytest

import bppo
import oracle_ffi as O
from parity_util import assert_metrics_close, assert_params_close

pytestmark = pytest.mark.gpu
D, A, P, G = 135, 33, 6, 200


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("players,ctde,shaping", [(4, True, 0.1), (2, False, 0.0), (6, True, 0.0), (3, False, 0.05)])
def test_vecenv_matches_oracle(players, ctde, shaping):
    N = 256
    cfg = bppo.make_config("skull_ctde" if ctde else "skull", num_envs=N, num_steps=4, player_count=players,
                           reward_shaping_coef=shaping)
    ctx = bppo.Context(cfg)
    ve = bppo.VecEnv.new(ctx)
    ov = O.lib().or_vecenv_new_np(O.ENV_SKULL, N, cfg["seed"], players)
    O.lib().or_vecenv_set_shaping(ov, shaping)
    obs_o = np.zeros(N * D, np.float32); m_o = np.zeros(N * A, np.uint8); pl_o = np.zeros(N, np.int32)
    g_o = np.zeros(N * G, np.float32); rw = np.zeros(N * P, np.float32); dn = np.zeros(N, np.uint8)
    eps = (O.Episode * N)()
    rng = np.random.default_rng(3)
    n_done = 0
    for t in range(500):
        O.lib().or_vecenv_get_obs(ov, obs_o)
        O.lib().or_vecenv_get_masks(ov, m_o)
        O.lib().or_vecenv_get_players(ov, pl_o)
        assert np.array_equal(ve.get_observations(), obs_o), t
        assert np.array_equal(ve.get_action_masks(), m_o.astype(bool)), t
        assert np.array_equal(ve.get_current_players(), pl_o), t
        if ctde:
            O.lib().or_vecenv_get_priv(ov, g_o)
            assert np.array_equal(ve.get_privileged_obs(), g_o), t
        m = m_o.reshape(N, A).astype(bool)
        a = np.array([rng.choice(np.flatnonzero(row)) for row in m], np.int32)
        o, r, d, ep = ve.step(a)
        ne = O.lib().or_vecenv_step(ov, a, obs_o, rw, dn, eps, N)
        assert np.array_equal(_bits(o), _bits(obs_o)), t
        assert np.array_equal(_bits(r.reshape(-1)), _bits(rw)), t
        assert np.array_equal(d, dn.astype(bool)), t
        assert len(ep) == ne
        for i, e in enumerate(ep):
            assert e["env_index"] == eps[i].env_index and e["length"] == eps[i].length
            assert np.array_equal(_bits(e["total_rewards"]), _bits(eps[i].total_rewards[:P]))
        n_done += int(d.sum())
    assert n_done > 20 and O.lib().or_vecenv_invalid(ov) == 0
    # an action outside the mask: the reference panics (skull.rs:1113-1128)
    m = ve.get_action_masks().reshape(N, A)
    a = np.array([np.flatnonzero(row)[0] for row in m], np.int32)
    a[0] = int(np.flatnonzero(~m[0])[0])
    with pytest.raises(bppo.BppoError):
        ve.step(a)
    O.lib().or_vecenv_free(ov)
    ctx.close()


def test_player_count_validation():
    for bad in (1, 7):
        with pytest.raises(bppo.BppoError):
            bppo.Context(bppo.make_config("skull", num_envs=8, num_steps=4, player_count=bad))


def _pair(N, T, ctde, players, seed=42, **kw):
    cfg = bppo.make_config("skull_ctde" if ctde else "skull", num_envs=N, num_steps=T, seed=seed,
                           player_count=players, hidden_size=64, num_hidden=2, critic_hidden_size=64,
                           critic_num_hidden=2, **kw)
    params = bppo.orthogonal_init(cfg, seed=5)
    tr = bppo.Trainer(cfg, params=params)
    ocfg = O.train_cfg(env_kind=O.ENV_SKULL, num_envs=N, num_steps=T, seed=seed, hidden=cfg["hidden_size"],
                       num_hidden=cfg["num_hidden"], ctde=ctde, relu=True,
                       critic_hidden=cfg["critic_hidden_size"] if ctde else 0,
                       critic_num_hidden=cfg["critic_num_hidden"] if ctde else 0,
                       normalize_obs=bool(cfg["normalize_obs"]), normalize_returns=False,
                       gamma=cfg["gamma"], gae_lambda=cfg["gae_lambda"],
                       lr=bppo.schedule_get(cfg["learning_rate"], 0), ent_coef=bppo.schedule_get(cfg["entropy_coef"], 0),
                       reward_shaping=cfg["reward_shaping_coef"], num_epochs=cfg["num_epochs"],
                       num_minibatches=cfg["num_minibatches"], clip=cfg["clip_epsilon"], value_coef=cfg["value_coef"],
                       target_kl=cfg["target_kl"], player_count=players)
    return cfg, tr, O.Trainer(ocfg, params)


def _cmp_rollout(tr, ot, ctde):
    b = tr.buffer
    assert np.array_equal(b.acting_players.reshape(-1), ot.buffer("players", np.int32))
    assert np.array_equal(_bits(b.observations.reshape(-1)), _bits(ot.buffer("obs")))
    assert np.array_equal(b.action_masks.reshape(-1), ot.buffer("masks"))
    if ctde:
        assert np.array_equal(_bits(b.privileged_obs.reshape(-1)), _bits(ot.buffer("priv")))
    assert np.array_equal(b.actions.reshape(-1), ot.buffer("actions", np.int32))
    assert np.array_equal(_bits(b.values.reshape(-1)), _bits(ot.buffer("values")))
    assert np.array_equal(_bits(b.log_probs.reshape(-1)), _bits(ot.buffer("log_probs")))
    assert np.array_equal(b.dones.reshape(-1), ot.buffer("dones"))
    assert np.array_equal(_bits(b.rewards.reshape(-1)), _bits(ot.buffer("rewards")))
    assert np.array_equal(_bits(b.all_rewards.reshape(-1)), _bits(ot.buffer("all_rewards")))
    assert tr.ctx.rng_pos() == ot.rng_pos()


@pytest.mark.parametrize("N,T,ctde,players", [(64, 32, True, 4), (48, 24, False, 6), (1024, 16, True, 3)])
def test_rollout_gae_update_second_rollout(N, T, ctde, players):
    cfg, tr, ot = _pair(N, T, ctde, players)
    info = bppo.collect_rollouts(tr.ctx)
    n_eps = ot.collect()
    _cmp_rollout(tr, ot, ctde)
    assert info.episodes == n_eps
    bppo.compute_gae(tr.ctx); ot.gae()
    assert np.array_equal(_bits(tr.ctx.buffer("last_v_pp")), _bits(ot.buffer("last_v_pp")))
    assert np.array_equal(_bits(tr.buffer.advantages.reshape(-1)), _bits(ot.buffer("advantages")))
    assert np.array_equal(_bits(tr.buffer.returns.reshape(-1)), _bits(ot.buffer("returns")))
    m = bppo.ppo_update(tr.ctx, bppo.schedule_get(cfg["learning_rate"], 0), bppo.schedule_get(cfg["entropy_coef"], 0))
    om = ot.update()
    assert tr.ctx.rng_pos() == ot.rng_pos()
    assert_metrics_close(m, om, values=ot.buffer("values"), returns=ot.buffer("returns"), advantages=ot.buffer("advantages"))
    assert_params_close(tr.model.get_params(), ot.params())
    tr.model.set_params(ot.params())
    bppo.collect_rollouts(tr.ctx); ot.collect()
    _cmp_rollout(tr, ot, ctde)
    tr.close(); ot.close()


@pytest.mark.parametrize("players,ctde", [(4, True), (5, False)])
def test_opponent_pool_rollout_update(players, ctde):
    """collect_rollouts_with_opponents over the seated players (EnvState with
    main.rs:552's actual_player_count): seat draws, opponent batches, learner-only
    update -- bit-exact rollouts, update within the usual tolerances."""
    N, T, n_opp, K = 48, 12, 32, 2
    cfg, tr, ot = _pair(N, T, ctde, players)
    rng = np.random.default_rng(7)
    params = np.stack([bppo.orthogonal_init(cfg, seed=100 + k) for k in range(K)])
    lp = rng.integers(0, players, n_opp).astype(np.int32)
    po = np.full((n_opp, players), -1, np.int32)
    for e in range(n_opp):
        for p in range(players):
            if p != lp[e]:
                po[e, p] = rng.integers(0, K)
    co = rng.integers(0, K, players - 1).astype(np.int32)
    tr.ctx.set_opponents(params, [None] * K, n_opp, lp, po, co)
    ot.set_opponents(params, [None] * K, n_opp, lp, po.reshape(-1), co)
    for _ in range(2):
        bppo.collect_rollouts(tr.ctx); ot.collect()
        _cmp_rollout(tr, ot, ctde)
        assert np.array_equal(tr.ctx.buffer("valid"), ot.buffer("valid"))
        l1, p1 = tr.ctx.opponent_envs()
        l2, p2 = ot.opponent_envs(n_opp, players)
        assert np.array_equal(l1, l2) and np.array_equal(p1.reshape(-1), p2)
        bppo.compute_gae(tr.ctx); ot.gae()
        assert np.array_equal(_bits(tr.buffer.advantages.reshape(-1)), _bits(ot.buffer("advantages")))
        m = bppo.ppo_update(tr.ctx, bppo.schedule_get(cfg["learning_rate"], 0),
                            bppo.schedule_get(cfg["entropy_coef"], 0))
        om = ot.update()
        assert tr.ctx.rng_pos() == ot.rng_pos()
        vm = ot.buffer("valid") > 0.5
        assert_metrics_close(m, om, values=ot.buffer("values")[vm], returns=ot.buffer("returns")[vm], advantages=ot.buffer("advantages")[vm])
        assert_params_close(tr.model.get_params(), ot.params())
        tr.model.set_params(ot.params())
    tr.close(); ot.close()
