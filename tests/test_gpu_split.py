"""CartPole nets the fused CartPole kernels do not cover, and split_networks, on the
GEMM-engine path.

  * CartPole MLPs of any width / depth (mlp.rs:76-132 accepts them): the rollout,
    bootstrap and update run on the f32 MFMA GEMM engine like Connect Four's, with
    CartPole's env step on the device (k_wide.hip EnvT<CARTPOLE>) -- widths past
    matrixmultiply's KC = 256 block included;
  * split_networks (config.rs:860; mlp.rs:40-130, 139-206): separate actor and
    critic trunks on the observation, parameters in Burn record order (layers,
    critic_layers, policy_head, value_head), for CartPole, Connect Four and Liar's
    Dice MLPs.

Each case: first rollout bit-exact against the oracle (oracle/net.c restates the
split forward/backward; tests/test_oracle_backward.py pins it against torch
autograd), GAE bit-exact on identical rewards, one update from the oracle's
advantages within the tests/parity_util.py tolerances, then the second rollout
bit-exact after injecting the oracle's parameters and normalizer state."""
import numpy as np
import pytest

import bppo
import oracle_ffi as O
from parity_util import (assert_metrics_close, assert_params_close, bits, cmp_cartpole_rollout,
                         oracle_train_cfg)
from test_gpu_scale import cmp_wide_rollout

pytestmark = pytest.mark.gpu


def _pair(preset, init_seed=7, **kw):
    cfg = bppo.make_config(preset, **kw)
    params = bppo.orthogonal_init(cfg, seed=init_seed)
    tr = bppo.Trainer(cfg, params=params)
    ot = O.Trainer(oracle_train_cfg(cfg), params)
    return cfg, tr, ot


def _update(cfg, tr, ot, inject):
    if inject:
        tr.ctx.set_buffer("advantages", ot.buffer("advantages"))
        tr.ctx.set_buffer("returns", ot.buffer("returns"))
    m = bppo.ppo_update(tr.ctx, bppo.schedule_get(cfg["learning_rate"], 0), bppo.schedule_get(cfg["entropy_coef"], 0))
    om = ot.update()
    assert tr.ctx.rng_pos() == ot.rng_pos()
    assert_metrics_close(m, om, values=ot.buffer("values"), returns=ot.buffer("returns"), advantages=ot.buffer("advantages"))
    assert_params_close(tr.model.get_params(), ot.params())


@pytest.mark.parametrize("H,NL,act,split", [(128, 2, "relu", False), (48, 3, "tanh", False), (300, 1, "relu", False),
                                            (64, 2, "relu", True), (16, 1, "tanh", True)])
def test_cartpole_gemm_path(H, NL, act, split):
    N, T = 256, 32
    cfg, tr, ot = _pair("cartpole", num_envs=N, num_steps=T, hidden_size=H, num_hidden=NL, activation=act,
                        split_networks=split)
    try:
        assert tr.ctx.n_params == ot.n_params == bppo.orthogonal_init(cfg).size
        bppo.collect_rollouts(tr.ctx); ot.collect()
        cmp_cartpole_rollout(tr, ot)
        # GAE on identical (return-normalized) rewards is bit-exact (compute_gae, ppo.rs:1069-1124)
        tr.ctx.set_buffer("rewards", ot.buffer("rewards"))
        bppo.compute_gae(tr.ctx); ot.gae()
        assert np.array_equal(bits(tr.buffer.advantages.reshape(-1)), bits(ot.buffer("advantages")))
        _update(cfg, tr, ot, inject=True)
        tr.model.set_params(ot.params())
        tr.ctx.set_obs_norm(*ot.obs_norm_state(5))
        tr.ctx.set_ret_norm(ot.ret_norm_state(), tr.ctx.ret_norm()[1])
        bppo.collect_rollouts(tr.ctx); ot.collect()
        cmp_cartpole_rollout(tr, ot)
    finally:
        tr.close(); ot.close()


@pytest.mark.parametrize("env,preset,kw", [
    ("connect_four", "connect_four", dict(hidden_size=64, num_envs=256, num_steps=16)),
    ("liars_dice", "liars_dice_ctde", dict(network_type="mlp", hidden_size=64, num_hidden=3, num_envs=96, num_steps=12)),
])
def test_split_networks_multiplayer(env, preset, kw):
    cfg, tr, ot = _pair(preset, split_networks=True, **kw)
    try:
        bppo.collect_rollouts(tr.ctx); ot.collect()
        cmp_wide_rollout(env, tr, ot)
        bppo.compute_gae(tr.ctx); ot.gae()
        assert np.array_equal(bits(tr.buffer.advantages.reshape(-1)), bits(ot.buffer("advantages")))
        _update(cfg, tr, ot, inject=False)
        tr.model.set_params(ot.params())
        bppo.collect_rollouts(tr.ctx); ot.collect()
        cmp_wide_rollout(env, tr, ot)
    finally:
        tr.close(); ot.close()


def test_split_networks_record_order_and_forward():
    """bppo_forward of a split net equals the oracle's, and the flat parameters are the
    Burn record (layers, critic_layers, policy_head, value_head): permuting the critic
    trunk's weights changes only the values, the actor's only the logits."""
    cfg = bppo.make_config("connect_four", num_envs=64, num_steps=4, hidden_size=32, split_networks=True)
    p = bppo.orthogonal_init(cfg, seed=2)
    tr = bppo.Trainer(cfg, params=p)
    try:
        obs = np.random.default_rng(0).random((300, 86)).astype(np.float32)
        lg, v = tr.model.forward(obs)
        desc = O.mlp_desc(86, 7, 32, 2, split=True)
        olg, ov = O.net_forward(desc, p, obs)
        assert np.array_equal(bits(lg), bits(olg)) and np.array_equal(bits(v[:, 0]), bits(ov))
        shapes, _ = bppo.host.layer_shapes(cfg)
        crit0 = sum(i * o + o for i, o in shapes[:2])           # first critic layer's W
        q = p.copy()
        q[crit0:crit0 + 86 * 32] *= 1.5
        tr.model.set_params(q)
        lg2, v2 = tr.model.forward(obs)
        assert np.array_equal(bits(lg2), bits(lg)) and not np.array_equal(bits(v2), bits(v))
    finally:
        tr.close()
