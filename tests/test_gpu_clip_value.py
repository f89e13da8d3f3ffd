"""The clipped value loss (config.clip_value, ppo.rs:1467-1474) on the device, against
the oracle:

    v_clipped = v_old + clamp(v - v_old, -eps, eps)
    value_loss = max((v - R)^2, (v_clipped - R)^2)

through the CartPole MFMA minibatch kernel (k_minibatch_mfma, CfgB's 2x64 relu net) and
the multi-player masked loss (k_wide_loss: Connect Four MLP, Liar's Dice CTDE).

In the first minibatch of the first epoch the parameters are the rollout's, so the
network's value of every row equals the stored old value bit for bit: there
v - v_old = 0 and the two squared errors TIE (max_pair's gradient routing at q1 == q2).
The test also rewrites the old values of chosen rows so that v - v_old is EXACTLY +eps
or -eps (the clamp's boundary, where Burn's clamp passes the gradient), beyond +-eps
(clamped: the gradient goes to the unclipped branch only when it is the larger) and
inside it.  Later minibatches run with updated parameters, the ordinary clipped case.
Bar: every UpdateMetrics field 1e-5 relative, parameters at PARAM_RTOL / PARAM_ATOL
(tests/parity_util.py)."""
import numpy as np
import pytest

import bppo
import oracle_ffi as O
from parity_util import assert_metrics_close, assert_params_close, bits, oracle_train_cfg

pytestmark = pytest.mark.gpu


def _exact_old_value(v, d):
    """an f32 v_old with f32(v - v_old) == d exactly, or None"""
    v, d = np.float32(v), np.float32(d)
    vo = np.float32(v - d)
    for _ in range(8):
        diff = np.float32(v - vo)
        if diff == d:
            return vo
        vo = np.nextafter(vo, np.float32(np.inf) if diff > d else np.float32(-np.inf), dtype=np.float32)
    return None


def craft_old_values(values, eps, seed=0):
    """old values: rows at exactly -eps / +eps from the current value, beyond the clip
    range on both sides, inside it, and the rest untouched (v == v_old: ties)"""
    rng = np.random.default_rng(seed)
    vo = np.array(values, np.float32)
    kind = rng.integers(0, 8, vo.size)
    n_exact = 0
    for i in np.flatnonzero(kind <= 1):                      # boundary rows
        x = _exact_old_value(vo[i], eps if kind[i] == 0 else -eps)
        if x is not None:
            vo[i] = x
            n_exact += 1
    far = kind == 2
    vo[far] = vo[far] + np.float32(3.0 * eps)                # clamped below
    far = kind == 3
    vo[far] = vo[far] - np.float32(3.0 * eps)                # clamped above
    ins = kind == 4
    vo[ins] = vo[ins] + np.float32(0.25 * eps)               # inside
    return vo.astype(np.float32), n_exact


def _check(cfg, tr, ot, inject_rewards):
    bppo.collect_rollouts(tr.ctx); ot.collect()
    if inject_rewards:   # CartPole's normalized rewards carry rtol 2e-7 (merge order)
        tr.ctx.set_buffer("rewards", ot.buffer("rewards"))
    bppo.compute_gae(tr.ctx); ot.gae()
    assert np.array_equal(bits(tr.buffer.advantages.reshape(-1)), bits(ot.buffer("advantages")))
    v = ot.buffer("values")
    assert np.array_equal(bits(tr.buffer.values.reshape(-1)), bits(v))
    vo, n_exact = craft_old_values(v, np.float32(cfg["clip_epsilon"]))
    assert n_exact > vo.size // 32       # hundreds of rows sit exactly on the clamp boundary
    tr.ctx.set_buffer("values", vo)
    ot.set_buffer("values", vo)
    lr, ent = bppo.schedule_get(cfg["learning_rate"], 0), bppo.schedule_get(cfg["entropy_coef"], 0)
    m = bppo.ppo_update(tr.ctx, lr, ent)
    om = ot.update()
    assert tr.ctx.rng_pos() == ot.rng_pos()
    assert_metrics_close(m, om, values=vo, returns=ot.buffer("returns"), advantages=ot.buffer("advantages"))
    assert_params_close(tr.model.get_params(), ot.params())
    return m, om


def test_clip_value_cartpole_mfma():
    cfg = bppo.make_config("cartpole", num_envs=2048, num_steps=32, clip_value=True)
    params = bppo.orthogonal_init(cfg, seed=2)
    tr = bppo.Trainer(cfg, params=params)
    ot = O.Trainer(oracle_train_cfg(cfg), params)
    try:
        m, om = _check(cfg, tr, ot, inject_rewards=True)
        # the clip changed the loss: the same update without clip_value differs
        cfg2 = dict(cfg, clip_value=False)
        ot2 = O.Trainer(oracle_train_cfg(cfg2), params)
        ot2.collect(); ot2.gae()
        ot2.set_buffer("values", craft_old_values(ot2.buffer("values"), np.float32(cfg["clip_epsilon"]))[0])
        om2 = ot2.update()
        assert om2["value_loss"] != om["value_loss"]
        ot2.close()
    finally:
        tr.close(); ot.close()


@pytest.mark.parametrize("preset,over", [
    ("connect_four", dict(hidden_size=64)),
    ("liars_dice_ctde", dict(hidden_size=64, critic_hidden_size=64, critic_num_hidden=2))])
def test_clip_value_wide_loss(preset, over):
    cfg = bppo.make_config(preset, num_envs=256, num_steps=16, clip_value=True, **over)
    params = bppo.orthogonal_init(cfg, seed=2)
    tr = bppo.Trainer(cfg, params=params)
    ot = O.Trainer(oracle_train_cfg(cfg), params)
    try:
        _check(cfg, tr, ot, inject_rewards=False)
    finally:
        tr.close(); ot.close()
