"""The device (libbppo.so) against the committed golden fixtures
(tests/golden/make_fixtures.py; pinned to the oracle by tests/test_golden.py):
a CartPole rollout + GAE, scripted Connect Four / Liar's Dice games through
the VecEnv surface, and one minibatch's loss, gradient and Adam step."""
import os

import numpy as np
import pytest

import bppo
from parity_util import PARAM_ATOL, PARAM_RTOL, RTOL, bits

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(GOLD, name + ".npz"))


def test_cartpole_trajectory_fixture():
    f = _load("cartpole_traj_16x32")
    N, T = int(f["num_envs"]), int(f["num_steps"])
    tr = bppo.Trainer(bppo.make_config("cartpole", num_envs=N, num_steps=T), params=f["params"])
    info = bppo.collect_rollouts(tr.ctx)
    assert info.episodes == int(f["episodes"]) and tr.ctx.rng_pos() == int(f["rng_pos"])
    b = tr.buffer
    assert np.array_equal(b.actions.reshape(-1), f["actions"])
    assert np.array_equal(b.dones.reshape(-1), f["dones"])
    for k, got in (("obs", b.observations), ("values", b.values), ("log_probs", b.log_probs)):
        assert np.array_equal(bits(got.reshape(-1)), bits(f[k])), k
    np.testing.assert_allclose(b.rewards.reshape(-1), f["rewards"], rtol=2e-7, atol=0)
    m, v, c = tr.ctx.obs_norm()
    assert c == float(f["obs_norm_count"])
    np.testing.assert_allclose(m, f["obs_norm_mean"], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(v, f["obs_norm_m2"], rtol=1e-10)
    tr.ctx.set_buffer("rewards", f["rewards"])
    bppo.compute_gae(tr.ctx)
    assert np.array_equal(bits(b.advantages.reshape(-1)), bits(f["advantages"]))
    assert np.array_equal(bits(b.returns.reshape(-1)), bits(f["returns"]))
    tr.close()


@pytest.mark.parametrize("name,preset", [("c4_scripted", "connect_four"), ("ld_scripted", "liars_dice_ctde")])
def test_scripted_games_fixture(name, preset):
    f = _load(name)
    N = int(f["num_envs"])
    cfg = bppo.make_config(preset, num_envs=N, num_steps=4, seed=int(f["seed"]),
                           reward_shaping_coef=float(f["shaping"]))
    ctx = bppo.Context(cfg)
    ve = bppo.VecEnv.new(ctx)
    for t in range(f["actions"].shape[0]):
        assert np.array_equal(bits(ve.get_observations()), bits(f["obs"][t])), t
        assert np.array_equal(ve.get_action_masks(), f["masks"][t].astype(bool)), t
        assert np.array_equal(ve.get_current_players(), f["players"][t]), t
        if ctx.priv_dim:
            assert np.array_equal(bits(ve.get_privileged_obs()), bits(f["priv"][t])), t
        o, r, d, _ = ve.step(f["actions"][t])
        assert np.array_equal(bits(o), bits(f["next_obs"][t])), t
        assert np.array_equal(bits(r.reshape(-1)), bits(f["rewards"][t])), t
        assert np.array_equal(d, f["dones"][t].astype(bool)), t
    ctx.close()


def test_minibatch_loss_grad_adam_fixture():
    f = _load("minibatch_cfgB")
    N, T = 16, 32
    cfg = bppo.make_config("cartpole", num_envs=N, num_steps=T, num_epochs=1, num_minibatches=1)
    tr = bppo.Trainer(cfg, params=f["params"])
    for k in ("obs", "actions", "log_probs", "values", "advantages", "returns"):
        tr.ctx.set_buffer(k, f[k])
    m = bppo.ppo_update(tr.ctx, float(f["lr"]), float(f["ent_coef"]))
    for k, floor in (("policy_loss", 1.0), ("value_loss", 0.0), ("entropy", 0.0), ("approx_kl", 0.0),
                     ("clip_fraction", 0.0), ("total_loss", 1.0)):
        ref = float(f["loss"]) if k == "total_loss" else float(f[k])
        assert abs(m[k] - ref) <= RTOL * max(abs(ref), floor), (k, m[k], ref)
    assert abs(m["adv_mean_raw"] - float(f["adv_mean"])) <= RTOL * abs(float(f["adv_std"]))
    assert abs(m["adv_std_raw"] - float(f["adv_std"])) <= RTOL * abs(float(f["adv_std"]))
    g = tr.ctx.buffer("grad")
    # per tensor, within 1e-5 of the tensor's largest entry (f32 sums in another order)
    np.testing.assert_allclose(g, f["grads"], rtol=0, atol=RTOL * float(np.abs(f["grads"]).max()))
    np.testing.assert_allclose(tr.model.get_params(), f["params_after"], rtol=PARAM_RTOL, atol=PARAM_ATOL)
    tr.close()
