"""PopArt value normalization (normalize_values; normalization.rs:262-366,
ppo.rs:1599-1653, 1780-1808, 1859-1897, main.rs:898-907) on the device against
the oracle, SURVEY 8(f)-4:
  * first update: statistics initialise from the returns and the value head is
    rescaled (old mean 0, std 1); minibatch returns / old values normalized;
  * second rollout: stored and bootstrap values denormalized, bit-exact given
    the oracle's parameters and PopArt state;
  * state, rescale magnitude and value_norm_target_mean/std match."""
import numpy as np
import pytest

import bppo
import oracle_ffi as O
from parity_util import assert_metrics_close, assert_params_close, bits, cartpole_pair, cmp_cartpole_rollout

pytestmark = pytest.mark.gpu


def _cartpole(N, T, **kw):
    cfg = bppo.make_config("cartpole", num_envs=N, num_steps=T, normalize_values=True, **kw)
    params = bppo.orthogonal_init(cfg, seed=1)
    tr = bppo.Trainer(cfg, params=params)
    ocfg = O.train_cfg(num_envs=N, num_steps=T, lr=1e-3, hidden=cfg["hidden_size"], num_hidden=cfg["num_hidden"],
                       num_epochs=cfg["num_epochs"], num_minibatches=cfg["num_minibatches"], normalize_values=True)
    return cfg, tr, O.Trainer(ocfg, params)


def _wide(env, N, T, ctde=None, **kw):
    kind = O.ENV_CONNECT_FOUR if env == "connect_four" else O.ENV_LIARS_DICE
    preset = "connect_four" if env == "connect_four" else "liars_dice_ctde"
    cfg = bppo.make_config(preset, num_envs=N, num_steps=T, normalize_values=True, **kw)
    if ctde is False:
        cfg.update(network_type="mlp", hidden_size=128)
    params = bppo.orthogonal_init(cfg, seed=5)
    tr = bppo.Trainer(cfg, params=params)
    ocfg = O.train_cfg(env_kind=kind, num_envs=N, num_steps=T, seed=cfg["seed"], hidden=cfg["hidden_size"],
                       num_hidden=cfg["num_hidden"], ctde=cfg["network_type"] == "ctde", relu=True,
                       critic_hidden=cfg["critic_hidden_size"] or 0, critic_num_hidden=cfg["critic_num_hidden"] or 0,
                       normalize_obs=False, normalize_returns=False, gamma=cfg["gamma"], gae_lambda=cfg["gae_lambda"],
                       lr=bppo.schedule_get(cfg["learning_rate"], 0), ent_coef=bppo.schedule_get(cfg["entropy_coef"], 0),
                       reward_shaping=cfg["reward_shaping_coef"], num_epochs=cfg["num_epochs"],
                       num_minibatches=cfg["num_minibatches"], clip=cfg["clip_epsilon"], value_coef=cfg["value_coef"],
                       target_kl=cfg["target_kl"], normalize_values=True)
    return cfg, tr, O.Trainer(ocfg, params)


def _rounds(cfg, tr, ot, cmp, rounds=3):
    lr = bppo.schedule_get(cfg["learning_rate"], 0)
    ent = bppo.schedule_get(cfg["entropy_coef"], 0)
    for rnd in range(rounds):
        if rnd:        # layered: the oracle's parameters, PopArt and normalizer state
            tr.model.set_params(ot.params())
            tr.ctx.set_popart(ot.popart())
            if cfg["env"] == "cartpole":
                tr.ctx.set_obs_norm(*ot.obs_norm_state(5))
                tr.ctx.set_ret_norm(*ot.ret_norm_state(returns=True))
        bppo.collect_rollouts(tr.ctx); ot.collect()
        cmp(tr, ot)
        bppo.compute_gae(tr.ctx); ot.gae()
        if cfg["env"] == "cartpole":
            # bootstrap denormalized (main.rs:898-907); rewards differ in rare last ulps
            np.testing.assert_allclose(tr.buffer.advantages.reshape(-1), ot.buffer("advantages"), rtol=1e-5, atol=1e-6)
            tr.ctx.set_buffer("advantages", ot.buffer("advantages"))
            tr.ctx.set_buffer("returns", ot.buffer("returns"))
        else:
            assert np.array_equal(bits(tr.buffer.advantages.reshape(-1)), bits(ot.buffer("advantages")))
        m = bppo.ppo_update(tr.ctx, lr, ent)
        om = ot.update()
        assert tr.ctx.rng_pos() == ot.rng_pos()
        dp, op = tr.ctx.popart(), ot.popart()
        assert dp[2] == op[2] and dp[3] == op[3]
        np.testing.assert_allclose(dp[:2], op[:2], rtol=1e-12)
        assert not np.isnan(m["value_norm_rescale_mag"])
        assert_metrics_close(m, om, values=ot.buffer("values"), returns=ot.buffer("returns"), advantages=ot.buffer("advantages"))
        assert_params_close(tr.model.get_params(), ot.params())


def test_popart_cartpole():
    cfg, tr, ot = _cartpole(64, 32)
    _rounds(cfg, tr, ot, cmp_cartpole_rollout)
    tr.close(); ot.close()


def _cmp_wide(tr, ot):
    b = tr.buffer
    assert np.array_equal(b.actions.reshape(-1), ot.buffer("actions", np.int32))
    assert np.array_equal(bits(b.values.reshape(-1)), bits(ot.buffer("values")))
    assert np.array_equal(bits(b.log_probs.reshape(-1)), bits(ot.buffer("log_probs")))
    assert np.array_equal(bits(tr.ctx.buffer("last_v_pp")), bits(ot.buffer("last_v_pp")))
    assert tr.ctx.rng_pos() == ot.rng_pos()


@pytest.mark.parametrize("env,N,T,ctde", [("connect_four", 64, 16, None), ("liars_dice", 48, 12, None),
                                          ("liars_dice", 40, 10, False)])
def test_popart_multiplayer(env, N, T, ctde):
    cfg, tr, ot = _wide(env, N, T, ctde=ctde)
    _rounds(cfg, tr, ot, _cmp_wide)
    tr.close(); ot.close()


def test_popart_world2_rank_slot_checked():
    """PopArt at W > 1 gathers every rank's batch statistics into the slot bppo_set_rank
    names (popart.hip popart_gather).  A context that never set its rank fails
    the update with BPPO_ERR_ARG instead of writing a default slot 0 (every rank in one slot:
    the SUM scales that slot by W on all ranks alike and no cross-rank check sees it); two
    contexts in one slot are caught from the gathered statistics.  One process, the
    host-staged callback standing in for the other rank: a no-op (the other rank's slot and
    gradient all zero), then a doubling (a second context with the same data and rank)."""
    import ctypes as C
    import bppo._lib as L
    hip = C.CDLL("libamdhip64.so")
    N, T = 256, 16
    cfg = bppo.make_config("cartpole", num_envs=N, num_steps=T, normalize_values=True)
    params = bppo.orthogonal_init(cfg, seed=1)
    lr, ent = bppo.schedule_get(cfg["learning_rate"], 0), bppo.schedule_get(cfg["entropy_coef"], 0)

    def run(setup):
        tr = bppo.Trainer(cfg, params=params)
        try:
            keep = setup(tr)
            bppo.collect_rollouts(tr.ctx)
            bppo.compute_gae(tr.ctx)
            with pytest.raises(L.BppoError) as e:
                bppo.ppo_update(tr.ctx, lr, ent)
            del keep
            return e.value
        finally:
            tr.close()

    def no_rank(tr):
        cb = L.ALLREDUCE_FN(lambda p, n, user: 0)
        assert L.lib().bppo_set_allreduce(tr.ctx.h, cb, None, 2) == L.OK
        return cb

    def doubled(p, n):
        buf = np.zeros(n, np.float32)
        assert hip.hipMemcpy(buf.ctypes.data_as(C.c_void_p), C.c_void_p(p), C.c_size_t(4 * n), 2) == 0   # D2H
        buf *= 2.0
        assert hip.hipMemcpy(C.c_void_p(p), buf.ctypes.data_as(C.c_void_p), C.c_size_t(4 * n), 1) == 0   # H2D

    def same_rank(tr):
        tr.ctx.rank = 0
        tr.ctx.set_allreduce(doubled, 2)
        return None

    e = run(no_rank)
    assert e.status == L.ERR_ARG and "bppo_set_rank" in str(e), e
    e = run(same_rank)
    assert e.status == L.ERR_ARG and "another rank wrote" in str(e), e
