"""Parity of the HIP path (through the C-ABI, libbppo.so) against the CPU
oracle on identical seeds.  Bit-exact for integer/index work (actions, dones,
episode boundaries, RNG positions, shuffled indices) and for every value the
reference computes element-wise in f32 (env transitions, observations, Gumbel
sampling, log-probs, values, GAE); reductions (normalizer stats, advantage
stats, gradients) within the stated tolerances."""
import ctypes as C

import numpy as np
import pytest

import bppo
import bppo._lib as L
import oracle_ffi as O
from parity_util import assert_metrics_close, assert_params_close

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch


# ----------------------------------------------------------------- libm ---
@pytest.mark.parametrize("which", [0, 1, 2, 3, 4, 5])
def test_device_libm_matches_host(which):
    rng = np.random.default_rng(which)
    if which == 3:   # every Gumbel input u
        k = np.arange(1 << 23, dtype=np.uint32)
        v = (k | 0x3F800000).view(np.float32) - np.float32(1)
        x = (v * np.float32(1.0) + np.float32(1e-10)).astype(np.float32)
    elif which in (1, 2):
        x = np.concatenate([rng.uniform(-0.5, 0.5, 2_000_000), rng.uniform(-200, 200, 500_000)]).astype(np.float32)
    elif which == 4:
        x = rng.uniform(-100, 20, 2_000_000).astype(np.float32)
    elif which == 5:   # every 16th float with |x| < 22, both signs
        lo = np.arange(0, np.float32(22.0).view(np.uint32), 16, dtype=np.uint32).view(np.float32)
        x = np.concatenate([lo, -lo])
    else:
        x = rng.integers(0, 0x7F800000, 2_000_000, dtype=np.uint32).view(np.float32)
    yh = np.zeros_like(x)
    yd = np.zeros_like(x)
    assert L.lib().bppo_debug_libm(which, 0, x.ctypes.data, yh.ctypes.data, x.size) == 0
    assert L.lib().bppo_debug_libm(which, 1, x.ctypes.data, yd.ctypes.data, x.size) == 0
    assert np.array_equal(yh.view(np.uint32), yd.view(np.uint32))


# ------------------------------------------------------------------ GAE ---
@pytest.mark.parametrize("T,N", [(1, 1), (7, 3), (128, 4096), (64, 1000), (100, 4096), (5, 256), (129, 64),
                                 (128, 65536)])
def test_gae_device_bit_exact(T, N):
    torch = _torch()
    rng = np.random.default_rng(T * 1000 + N)
    r = (rng.random((T, N)) < 0.98).astype(np.float32)
    d = (rng.random((T, N)) < 0.01).astype(np.float32)
    v = rng.normal(50, 20, (T, N)).astype(np.float32)
    lv = rng.normal(50, 20, N).astype(np.float32)
    adv_o, ret_o = O.compute_gae(r, d, v, lv, 0.99, 0.95)
    dev = [torch.from_numpy(a).cuda() for a in (r, d, v, lv)]
    adv = torch.empty((T, N), device="cuda")
    ret = torch.empty((T, N), device="cuda")
    st = L.lib().bppo_gae_device(*[t.data_ptr() for t in dev], T, N, 0.99, 0.95, adv.data_ptr(),
                                 ret.data_ptr(), None)
    assert st == 0
    torch.cuda.synchronize()
    assert np.array_equal(adv.cpu().numpy().view(np.uint32), adv_o.view(np.uint32))
    assert np.array_equal(ret.cpu().numpy().view(np.uint32), ret_o.view(np.uint32))


@pytest.mark.parametrize("T,N", [(128, 4096), (37, 1000), (16, 1002)])
def test_gae_rows_device_bit_exact(T, N):
    """bppo_gae_rows_device (the bench path's GAE: the [advantage, return] pair of every
    minibatch row too) = the oracle"""
    torch = _torch()
    rng = np.random.default_rng(T + N)
    r = (rng.random((T, N)) < 0.98).astype(np.float32)
    d = (rng.random((T, N)) < 0.01).astype(np.float32)
    v = rng.normal(50, 20, (T, N)).astype(np.float32)
    lv = rng.normal(50, 20, N).astype(np.float32)
    adv_o, ret_o = O.compute_gae(r, d, v, lv, 0.99, 0.95)
    dev = [torch.from_numpy(a).cuda() for a in (r, d, v, lv)]
    adv = torch.empty((T, N), device="cuda")
    ret = torch.empty((T, N), device="cuda")
    pairs = torch.full((T * N, 2), 7.0, device="cuda")
    st = L.lib().bppo_gae_rows_device(*[t.data_ptr() for t in dev], T, N, 0.99, 0.95, adv.data_ptr(),
                                      ret.data_ptr(), pairs.data_ptr(), None)
    if N % 4:
        assert st == L.ERR_UNSUPPORTED
        return
    assert st == 0
    torch.cuda.synchronize()
    pw = pairs.cpu().numpy()
    assert np.array_equal(adv.cpu().numpy().view(np.uint32), adv_o.view(np.uint32))
    assert np.array_equal(pw[:, 0].view(np.uint32), adv_o.reshape(-1).view(np.uint32))
    assert np.array_equal(pw[:, 1].view(np.uint32), ret_o.reshape(-1).view(np.uint32))


@pytest.mark.parametrize("P,T,N", [(2, 64, 2048), (3, 64, 2048), (4, 64, 2048), (4, 128, 32768), (6, 37, 1000),
                                   (2, 129, 300), (1, 16, 64)])
def test_gae_multiplayer_device_bit_exact(P, T, N):
    """k_gae_mp_seg (T <= 128: T split over the waves of a block) and k_gae_mp (longer T)"""
    torch = _torch()
    rng = np.random.default_rng(P)
    pl = rng.integers(0, P, (T, N)).astype(np.int32)
    d = (rng.random((T, N)) < 0.05).astype(np.float32)
    ar = np.where(rng.random((T, N, P)) < 0.1, rng.choice([-1.0, 1.0, 0.33, -0.33], (T, N, P)), 0.0).astype(np.float32)
    v = rng.normal(0, 0.5, (T, N)).astype(np.float32)
    lvpp = rng.normal(0, 0.5, (N, P)).astype(np.float32)
    adv_o, ret_o = O.compute_gae_mp(ar, pl, d, v, lvpp, 0.97, 0.90)
    dev = [torch.from_numpy(a).cuda() for a in (ar, pl, d, v, lvpp)]
    adv = torch.empty((T, N), device="cuda")
    ret = torch.empty((T, N), device="cuda")
    st = L.lib().bppo_gae_mp_device(*[t.data_ptr() for t in dev], T, N, P, 0.97, 0.90, adv.data_ptr(),
                                    ret.data_ptr(), None)
    assert st == 0
    torch.cuda.synchronize()
    assert np.array_equal(adv.cpu().numpy().view(np.uint32), adv_o.view(np.uint32))


def test_gae_mp_known_answers_on_device():
    """ppo.rs:2579-2635 same_player_across_boundary through the device kernel."""
    torch = _torch()
    d = np.array([[0.0], [1.0], [1.0]], np.float32)
    pl = np.zeros((3, 1), np.int32)
    ar = np.array([[[0.0, 0.0]], [[-1.0, 0.0]], [[10.0, 0.0]]], np.float32)
    v = np.array([[0.0], [0.0], [5.0]], np.float32)
    lv = np.array([[5.0, 0.0]], np.float32)
    dev = [torch.from_numpy(a).cuda() for a in (ar, pl, d, v, lv)]
    adv = torch.empty((3, 1), device="cuda"); ret = torch.empty((3, 1), device="cuda")
    assert L.lib().bppo_gae_mp_device(*[t.data_ptr() for t in dev], 3, 1, 2, 0.99, 0.95, adv.data_ptr(),
                                      ret.data_ptr(), None) == 0
    a = adv.cpu().numpy().reshape(-1)
    assert abs(a[2] - 5.0) < 1e-5 and abs(a[1] + 1.0) < 1e-5 and abs(a[0] + 0.99 * 0.95) < 1e-5


# --------------------------------------------------------------- VecEnv ---
def test_vecenv_reset_and_steps_match_oracle():
    N = 256
    cfg = bppo.make_config("cartpole", num_envs=N, num_steps=8)
    ctx = bppo.Context(cfg)
    ve = bppo.VecEnv.new(ctx)
    ov = O.lib().or_vecenv_new(O.ENV_CARTPOLE, N, cfg["seed"])
    obs_o = np.zeros(N * 5, np.float32)
    O.lib().or_vecenv_get_obs(ov, obs_o)
    assert np.array_equal(ve.get_observations(), obs_o)
    rng = np.random.default_rng(0)
    rw = np.zeros(N, np.float32); dn = np.zeros(N, np.uint8)
    eps = (O.Episode * N)()
    n_done = 0
    for t in range(600):
        a = rng.integers(0, 2, N).astype(np.int32)
        o, r, d, ep = ve.step(a)
        O.lib().or_vecenv_step(ov, a, obs_o, rw, dn, eps, N)
        assert np.array_equal(o, obs_o), t
        assert np.array_equal(r.reshape(-1), rw), t
        assert np.array_equal(d, dn.astype(bool)), t
        n_done += int(d.sum())
    assert n_done > 100
    O.lib().or_vecenv_free(ov)
    ctx.close()


# -------------------------------------------------------------- rollout ---
def _pair(N, T, seed=42, **kw):
    cfg = bppo.make_config("cartpole", num_envs=N, num_steps=T, seed=seed, **kw)
    params = bppo.orthogonal_init(cfg, seed=1)
    tr = bppo.Trainer(cfg, params=params)
    ocfg = O.train_cfg(num_envs=N, num_steps=T, seed=seed, lr=1e-3,
                       hidden=cfg["hidden_size"], num_hidden=cfg["num_hidden"],
                       relu=cfg["activation"] == "relu",
                       num_epochs=cfg["num_epochs"], num_minibatches=cfg["num_minibatches"])
    ot = O.Trainer(ocfg, params)
    return cfg, tr, ot


def _cmp_rollout(tr, ot, exact_rewards=False):
    b = tr.buffer
    assert np.array_equal(b.actions.reshape(-1), ot.buffer("actions", np.int32))
    assert np.array_equal(b.dones.reshape(-1), ot.buffer("dones"))
    assert np.array_equal(b.observations.reshape(-1).view(np.uint32), ot.buffer("obs").view(np.uint32))
    assert np.array_equal(b.values.reshape(-1).view(np.uint32), ot.buffer("values").view(np.uint32))
    assert np.array_equal(b.log_probs.reshape(-1).view(np.uint32), ot.buffer("log_probs").view(np.uint32))
    rg, ro = b.rewards.reshape(-1), ot.buffer("rewards")
    if exact_rewards:
        assert np.array_equal(rg, ro)
    # return normaliser: f64 Chan-merge scan vs sequential Welford -> f32 results
    # identical except for rare last-ulp ties
    np.testing.assert_allclose(rg, ro, rtol=2e-7, atol=0)
    assert tr.ctx.rng_pos() == ot.rng_pos()


@pytest.mark.parametrize("N,T", [(8, 128), (256, 64)])
def test_first_rollout_bit_exact(N, T):
    cfg, tr, ot = _pair(N, T)
    bppo.collect_rollouts(tr.ctx)
    ot.collect()
    _cmp_rollout(tr, ot)
    m, v, c = tr.ctx.obs_norm()
    mo, vo, co = ot.obs_norm_state(5)
    assert c == co
    np.testing.assert_allclose(m, mo, rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(v, vo, rtol=1e-10)
    bppo.compute_gae(tr.ctx)
    ot.gae()
    np.testing.assert_allclose(tr.buffer.advantages.reshape(-1), ot.buffer("advantages"), rtol=1e-5, atol=1e-6)
    tr.close(); ot.close()


def test_update_matches_oracle_and_rng_chain_exact():
    N, T = 64, 32
    cfg, tr, ot = _pair(N, T, num_minibatches=4, num_epochs=2)
    bppo.collect_rollouts(tr.ctx); ot.collect()
    bppo.compute_gae(tr.ctx); ot.gae()
    # identical GAE inputs for the update comparison
    tr.ctx.set_buffer("advantages", ot.buffer("advantages"))
    tr.ctx.set_buffer("returns", ot.buffer("returns"))
    m = bppo.ppo_update(tr.ctx, 1e-3, 0.01)
    om = ot.update()
    assert tr.ctx.rng_pos() == ot.rng_pos()           # shuffle chain consumed the same words
    # last epoch's permutation == oracle Fisher-Yates from the same stream position
    perm = tr.ctx.buffer("perm", np.uint32)
    p_words = ot.rng_pos()
    assert sorted(perm.tolist()) == list(range(N * T))
    assert_metrics_close(m, om, values=ot.buffer("values"), returns=ot.buffer("returns"), advantages=ot.buffer("advantages"))
    assert_params_close(tr.model.get_params(), ot.params())
    tr.close(); ot.close()


def test_shuffle_permutation_bit_exact():
    N, T = 50, 20
    cfg, tr, ot = _pair(N, T, num_minibatches=3, num_epochs=1)
    bppo.collect_rollouts(tr.ctx); ot.collect()
    bppo.compute_gae(tr.ctx); ot.gae()
    start = tr.ctx.rng_pos()
    bppo.ppo_update(tr.ctx, 1e-3, 0.01)
    perm = tr.ctx.buffer("perm", np.uint32)
    r = O.Rng()
    O.lib().or_rng_seed_u64(C.byref(r), cfg["seed"])
    r.word_pos = start
    ref = np.arange(N * T, dtype=np.uint32)
    O.lib().or_shuffle_u32(C.byref(r), ref, ref.size)
    assert np.array_equal(perm, ref)
    assert tr.ctx.rng_pos() == r.word_pos
    tr.close(); ot.close()


def test_second_rollout_bit_exact_given_oracle_state():
    """Layered parity: after one update, inject the oracle's params and
    normaliser state; the next rollout is again bit-identical."""
    N, T = 128, 64
    cfg, tr, ot = _pair(N, T)
    bppo.collect_rollouts(tr.ctx); ot.collect()
    bppo.compute_gae(tr.ctx); ot.gae()
    bppo.ppo_update(tr.ctx, 1e-3, 0.01); ot.update()
    assert tr.ctx.rng_pos() == ot.rng_pos()
    tr.model.set_params(ot.params())
    m, v, c = ot.obs_norm_state(5)
    tr.ctx.set_obs_norm(m, v, c)
    mvc = ot.ret_norm_state()
    tr.ctx.set_ret_norm(mvc, tr.ctx.ret_norm()[1])
    bppo.collect_rollouts(tr.ctx); ot.collect()
    _cmp_rollout(tr, ot)
    tr.close(); ot.close()


def test_training_improves_cartpole_return():
    cfg = bppo.make_config("cartpole", num_envs=1024, num_steps=128)
    tr = bppo.Trainer(cfg, init_seed=3)
    rets = []
    for _ in range(12):
        m = tr.train_update()
        rets.append(m["mean_return"])
    tr.close()
    assert rets[-1] > 3 * max(rets[0], 10.0), rets


# ------------------------------------------------------ tanh activation ---
# config.rs:990-992 default activation (every shipped config says relu):
# mlp.rs:187-191 tanh through glibc tanhf, restated bit-exactly on the device
TANH_NETS = [(64, 2), (32, 1), (16, 2)]


@pytest.mark.parametrize("H,NL", TANH_NETS)
def test_tanh_first_rollout_bit_exact(H, NL):
    cfg, tr, ot = _pair(64, 32, activation="tanh", hidden_size=H, num_hidden=NL)
    bppo.collect_rollouts(tr.ctx); ot.collect()
    _cmp_rollout(tr, ot)
    tr.close(); ot.close()


@pytest.mark.parametrize("H,NL", TANH_NETS)
def test_tanh_update_matches_oracle(H, NL):
    cfg, tr, ot = _pair(64, 32, activation="tanh", hidden_size=H, num_hidden=NL,
                        num_minibatches=4, num_epochs=2)
    bppo.collect_rollouts(tr.ctx); ot.collect()
    bppo.compute_gae(tr.ctx); ot.gae()
    tr.ctx.set_buffer("advantages", ot.buffer("advantages"))
    tr.ctx.set_buffer("returns", ot.buffer("returns"))
    m = bppo.ppo_update(tr.ctx, 1e-3, 0.01)
    om = ot.update()
    assert tr.ctx.rng_pos() == ot.rng_pos()
    assert_metrics_close(m, om, values=ot.buffer("values"), returns=ot.buffer("returns"), advantages=ot.buffer("advantages"))
    assert_params_close(tr.model.get_params(), ot.params())
    tr.close(); ot.close()


def test_tanh_second_rollout_and_forward_rows_bit_exact():
    N, T = 128, 32
    cfg, tr, ot = _pair(N, T, activation="tanh")
    bppo.collect_rollouts(tr.ctx); ot.collect()
    bppo.compute_gae(tr.ctx); ot.gae()
    bppo.ppo_update(tr.ctx, 1e-3, 0.01); ot.update()
    tr.model.set_params(ot.params())
    m, v, c = ot.obs_norm_state(5)
    tr.ctx.set_obs_norm(m, v, c)
    tr.ctx.set_ret_norm(ot.ret_norm_state(), tr.ctx.ret_norm()[1])
    bppo.collect_rollouts(tr.ctx); ot.collect()
    _cmp_rollout(tr, ot)
    # the batched forward entry on the rollout's own observations reproduces
    # the values the rollout stored
    obs = tr.buffer.observations.reshape(-1, 5)
    lg, vals = tr.model.forward(obs)
    assert np.array_equal(vals.reshape(-1).view(np.uint32), ot.buffer("values").view(np.uint32))
    tr.close(); ot.close()


@pytest.mark.parametrize("lanes64", ["1", "0"])
@pytest.mark.parametrize("N", [1000, 2048])
def test_rollout_lanes64_bit_exact(monkeypatch, N, lanes64):
    """both CfgB rollout kernels — the 64-lane k_cartpole_rollout_mfma64 (default:
    transposed layers, permlane32 input swaps, W1 and H2 through LDS) and r03's half-wave
    k_cartpole_rollout_mfma (BPPO_ROLLOUT_LANES64=0) — bit-exact against the oracle over
    two consecutive rollouts (env state, episode and RNG carry), a partial last wave at
    N = 1000, with obs + return normalizers"""
    import oracle_ffi as O
    from parity_util import cmp_cartpole_rollout, oracle_train_cfg
    monkeypatch.setenv("BPPO_ROLLOUT_LANES64", lanes64)
    cfg = bppo.make_config("cartpole", num_envs=N, num_steps=32)
    params = bppo.orthogonal_init(cfg, seed=11)
    tr = bppo.Trainer(cfg, params=params)
    ot = O.Trainer(oracle_train_cfg(cfg), params)
    try:
        for _ in range(2):
            bppo.collect_rollouts(tr.ctx); ot.collect()
            cmp_cartpole_rollout(tr, ot)
            tr.ctx.set_buffer("rewards", ot.buffer("rewards"))
            bppo.compute_gae(tr.ctx); ot.gae()
            bppo.ppo_update(tr.ctx, bppo.schedule_get(cfg["learning_rate"], 0), bppo.schedule_get(cfg["entropy_coef"], 0))
            ot.update()
            tr.model.set_params(ot.params())
            mvc, rets = ot.ret_norm_state(returns=True)
            tr.ctx.set_ret_norm(mvc, rets)
            tr.ctx.set_obs_norm(*ot.obs_norm_state(5))
    finally:
        tr.close(); ot.close()


@pytest.mark.parametrize("pool_k", ["16", "2", "0"])
def test_rollout_lanes64_episodes_and_reset_pool(monkeypatch, pool_k):
    """the 64-lane rollout's episode records (deferred slot reservation) and resets from
    k_reset_pool's states drawn ahead (16: the default pool; 2: most envs run past the pool
    and fall back to drawing in the kernel; 0: no pool) -- records, env state and RNG
    positions bit-exact against the oracle over two rollouts of T = 128"""
    import oracle_ffi as O
    from parity_util import cmp_cartpole_rollout, oracle_train_cfg
    monkeypatch.setenv("BPPO_RESET_POOL_K", pool_k)
    N, T = 2048, 128
    cfg = bppo.make_config("cartpole", num_envs=N, num_steps=T)
    params = bppo.orthogonal_init(cfg, seed=5)
    tr = bppo.Trainer(cfg, params=params)
    ot = O.Trainer(oracle_train_cfg(cfg), params)
    try:
        for _ in range(2):
            info = bppo.collect_rollouts(tr.ctx)
            n_eps = ot.collect()
            cmp_cartpole_rollout(tr, ot)
            assert info.episodes == n_eps > N
            dev = [(np.float32(e["total_rewards"][0]).view(np.uint32).item(), e["length"], e["env_index"])
                   for e in bppo.rollout_episodes(tr.ctx)]
            oe = ot.episodes()            # the oracle stores the first 4 N + 1024 (oracle/ppo.c eps_cap)
            assert len(dev) == n_eps and len(oe) >= min(n_eps, 4 * N)
            assert dev[:len(oe)] == oe
            tr.ctx.set_buffer("rewards", ot.buffer("rewards"))
            bppo.compute_gae(tr.ctx); ot.gae()
            bppo.ppo_update(tr.ctx, bppo.schedule_get(cfg["learning_rate"], 0), bppo.schedule_get(cfg["entropy_coef"], 0))
            ot.update()
            tr.model.set_params(ot.params())
            mvc, rets = ot.ret_norm_state(returns=True)
            tr.ctx.set_ret_norm(mvc, rets)
            tr.ctx.set_obs_norm(*ot.obs_norm_state(5))
    finally:
        tr.close(); ot.close()


@pytest.mark.parametrize("threads", ["16", "2"])
def test_shuffle_windows_single_rank_matches_oracle(monkeypatch, threads):
    """shuffle_windows at W = 1 through the pipelined bppo_train_steps (the engine walks the
    epochs at once: alone with 16 CPUs, in interleaved pairs with 2): permutations, RNG
    positions, metrics and parameters against the oracle's windowed update, two updates"""
    import oracle_ffi as O
    from parity_util import oracle_train_cfg
    monkeypatch.setenv("BPPO_HOST_THREADS", threads)
    cfg = bppo.make_config("cartpole", num_envs=2048, num_steps=32, shuffle_windows=True)
    params = bppo.orthogonal_init(cfg, seed=12)
    tr = bppo.Trainer(cfg, params=params)
    ot = O.Trainer(oracle_train_cfg(cfg), params)
    try:
        bppo.collect_rollouts(tr.ctx); ot.collect()
        tr.ctx.set_buffer("rewards", ot.buffer("rewards"))
        bppo.compute_gae(tr.ctx); ot.gae()
        m = bppo.ppo_update(tr.ctx, bppo.schedule_get(cfg["learning_rate"], 0), bppo.schedule_get(cfg["entropy_coef"], 0))
        om = ot.update()
        assert tr.ctx.rng_pos() == ot.rng_pos()
        assert_metrics_close(m, om, values=ot.buffer("values"), returns=ot.buffer("returns"), advantages=ot.buffer("advantages"))
        assert_params_close(tr.model.get_params(), ot.params())
        # second update through the pipelined path, from the oracle's state
        tr.model.set_params(ot.params())
        mvc, rets = ot.ret_norm_state(returns=True)
        tr.ctx.set_ret_norm(mvc, rets)
        tr.ctx.set_obs_norm(*ot.obs_norm_state(5))
        ms2, _ = tr.train_updates(1)
        ot.collect(); ot.gae()
        assert np.array_equal(tr.buffer.actions.reshape(-1), ot.buffer("actions", np.int32))
        om2 = ot.update()
        assert tr.ctx.rng_pos() == ot.rng_pos()
        assert_metrics_close(ms2[0], om2, values=ot.buffer("values"), returns=ot.buffer("returns"), advantages=ot.buffer("advantages"))
        assert_params_close(tr.model.get_params(), ot.params())
    finally:
        tr.close(); ot.close()
