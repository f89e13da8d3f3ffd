"""The split-bf16 contraction of the GEMM engine (k_gemm.hip k_gemm_split): the wide nets'
update GEMMs (forward, input gradient, weight gradient) of every minibatch after the
update's first.

Each f32 operand is split exactly into three round-to-nearest bf16 pieces x = x0 + x1 + x2
and the six products of order <= 2 are accumulated in f32 on v_mfma_f32_32x32x16_bf16;
the dropped products are within (2^-23 + 2^-32) |x y| (tests/test_split_bf16.py), so each
output is within that of the f64 dot product plus the f32 accumulation error: the same
1e-5-of-|products| bar as the engine's other non-chained forms (test_gpu_gemm.py).

  * through bppo_debug_gemm (modes 5 / 6 / 7) on the wide nets' shapes and ragged edges,
    unaligned operands included (K = 86 rows: the scalar-load path);
  * the whole minibatch gradient from IDENTICAL parameters and buffers against the oracle's
    or_minibatch_loss_grad (ppo.rs:1923-1959 loss -> backward), for the Connect Four MLP and
    the Liar's Dice CTDE nets, with the split contraction on (bppo_set_minibatch_kernel 2)
    and with the exact chains (1): the losses within 1e-5 relative and every gradient entry
    within 1e-5 of its tensor's largest |entry|."""
import ctypes as C

import numpy as np
import pytest

import bppo
import bppo._lib as L
import oracle_ffi as O
from bppo.host import layer_shapes
from parity_util import summand_magnitude
from test_gpu_gemm import FWD_SHAPES, _gemm
from test_gpu_wide import _pair

pytestmark = pytest.mark.gpu

TOL = 1e-5


@pytest.mark.parametrize("M,N,K", FWD_SHAPES + [(4096, 512, 512)])
def test_split_forward(M, N, K):
    rng = np.random.default_rng(M * 5 + N + K)
    X = rng.standard_normal((M, K)).astype(np.float32)
    if K == 86:
        X = (rng.random((M, K)) < 0.3).astype(np.float32)
    W = (rng.standard_normal((K, N)) / np.sqrt(K)).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32) * 0.1
    z = X.astype(np.float64) @ W.astype(np.float64) + b
    mag = np.abs(X.astype(np.float64)) @ np.abs(W.astype(np.float64)) + np.abs(b)
    y, _ = _gemm(5, M, N, K, X, W, b, relu=1)
    assert np.all(np.abs(y - np.maximum(z, 0.0)) <= TOL * mag + 1e-30)
    y, _ = _gemm(5, M, N, K, X, W, b, relu=0)
    err = np.abs(y - z)
    assert np.all(err <= TOL * mag + 1e-30)
    # the split arithmetic, not a bf16 one: far inside the bound on average
    assert err.mean() <= 1e-6 * mag.mean()


@pytest.mark.parametrize("M,N,K", [(300, 512, 512), (257, 86, 512), (100, 256, 49), (70, 512, 1),
                                   (129, 512, 8), (4096, 512, 512)])
def test_split_dx(M, N, K):
    rng = np.random.default_rng(M + 3 * N + K)
    dZ = rng.standard_normal((M, K)).astype(np.float32)
    W = rng.standard_normal((N, K)).astype(np.float32)
    H = rng.standard_normal((M, N)).astype(np.float32)
    g = dZ.astype(np.float64) @ W.astype(np.float64).T
    mag = np.abs(dZ.astype(np.float64)) @ np.abs(W.astype(np.float64)).T
    out, _ = _gemm(6, M, N, K, dZ, W, H)
    assert np.all(np.abs(out - g * (H > 0)) <= TOL * mag + 1e-30)
    out, _ = _gemm(6, M, N, K, dZ, W, None)
    assert np.all(np.abs(out - g) <= TOL * mag + 1e-30)


@pytest.mark.parametrize("Kin,N,rows", [(512, 512, 5000), (86, 512, 4099), (256, 49, 3000), (512, 1, 2500),
                                        (390, 512, 70000), (64, 8, 31), (512, 8, 16384)])
def test_split_weight_grad(Kin, N, rows):
    rng = np.random.default_rng(Kin + 7 * N + rows)
    X = rng.standard_normal((rows, Kin)).astype(np.float32)
    dZ = rng.standard_normal((rows, N)).astype(np.float32)
    out, db = _gemm(7, Kin, N, rows, X, dZ, None)
    ref = X.astype(np.float64).T @ dZ.astype(np.float64)
    mag = np.abs(X.astype(np.float64)).T @ np.abs(dZ.astype(np.float64))
    assert np.all(np.abs(out - ref) <= TOL * mag + 1e-30)
    dbr = dZ.astype(np.float64).sum(0)
    assert np.all(np.abs(db - dbr) <= TOL * np.abs(dZ).astype(np.float64).sum(0) + 1e-30)


NETS = [("connect_four", None), ("liars_dice", True)]


@pytest.mark.parametrize("env,ctde", NETS)
@pytest.mark.parametrize("mode", [2, 1, 0])
def test_wide_gradient_from_identical_parameters(env, ctde, mode):
    N, T = 512, 16
    cfg, tr, ot = _pair(env, N, T, ctde=ctde, num_epochs=1, num_minibatches=1)
    try:
        tr.ctx.set_minibatch_kernel(mode)
        bppo.collect_rollouts(tr.ctx); ot.collect()
        bppo.compute_gae(tr.ctx); ot.gae()
        B = N * T
        rng = np.random.default_rng(17)
        logp = (ot.buffer("log_probs") + rng.normal(0, 0.3, B)).astype(np.float32)
        val = (ot.buffer("values") + rng.normal(0, 0.2, B)).astype(np.float32)
        for k, v in (("log_probs", logp), ("values", val), ("advantages", ot.buffer("advantages")),
                     ("returns", ot.buffer("returns"))):
            tr.ctx.set_buffer(k, v)
        ot.set_buffer("log_probs", logp); ot.set_buffer("values", val)
        p0 = tr.model.get_params()
        lr, ent = bppo.schedule_get(cfg["learning_rate"], 0), bppo.schedule_get(cfg["entropy_coef"], 0)
        m = bppo.ppo_update(tr.ctx, lr, ent)
        g = tr.ctx.buffer("grad")
        is_ctde = cfg["network_type"] == "ctde"
        _, D, A, P, G = {"connect_four": (0, 86, 7, 2, 0), "liars_dice": (0, 270, 49, 4, 120)}[env]
        if is_ctde:
            desc = O.ctde_desc(D, G, A, cfg["hidden_size"], cfg["num_hidden"], cfg["critic_hidden_size"],
                               cfg["critic_num_hidden"], cfg["activation"] == "relu")
        else:
            desc = O.mlp_desc(D, A, cfg["hidden_size"], cfg["num_hidden"], cfg["activation"] == "relu")
        adv = ot.buffer("advantages")
        advn = np.zeros(B, np.float32)
        st = [C.c_float() for _ in range(4)]
        O.lib().or_normalize_advantages(adv, B, advn, *[C.byref(x) for x in st])
        go = np.zeros(desc.n_params, np.float32)
        ms = O.MbStats()
        pc = O.ppo_cfg(num_epochs=1, num_minibatches=1, clip=cfg["clip_epsilon"], value_coef=cfg["value_coef"])
        priv = ot.buffer("priv") if is_ctde else None
        masks = ot.buffer("masks")
        O.lib().or_minibatch_loss_grad(C.byref(desc), p0, B, ot.buffer("obs"), None if priv is None else priv.ctypes.data,
                                       ot.buffer("actions", np.int32), logp, advn, ot.buffer("returns"), val,
                                       masks.ctypes.data, C.byref(pc), ent, go, C.byref(ms))
        assert 0.05 < ms.clip_fraction < 0.95
        floors = {"policy_loss": summand_magnitude(adv), "value_loss": 0.0, "entropy": 0.0,
                  "approx_kl": 0.0, "clip_fraction": 1.0 / B}
        for k, fl in floors.items():
            o = getattr(ms, k)
            assert abs(m[k] - o) <= TOL * max(abs(o), fl), (k, m[k], o)
        shapes, _ = layer_shapes(cfg)
        off, worst = 0, []
        for i, o in shapes:
            for n in (i * o, o):
                a, b = g[off:off + n], go[off:off + n]
                tol = TOL * max(np.abs(b).max(), 1e-30)
                worst.append((off, n, float(np.abs(a - b).max() / tol), int((np.abs(a - b) > tol).sum())))
                off += n
        assert off == desc.n_params
        if mode == 1:   # the exact chains and row-ordered f64 weight gradients
            assert all(w[2] <= 1.0 for w in worst), (mode, worst)
        else:
            # the split forward (mode 2) and the f32 split-K weight gradients (mode 0) differ from
            # the oracle's in the last bits: a ReLU pre-activation within that distance of zero
            # switches its unit for one row, which moves that row's contribution in a few
            # entries.  Every entry within 1e-4 of its tensor's largest |entry| (10x the exact
            # bar) and at most 0.5 % of all entries past 1e-5 of it
            assert all(w[2] <= 10.0 for w in worst), (mode, worst)
            assert sum(w[3] for w in worst) <= 0.005 * desc.n_params, (mode, worst)
    finally:
        tr.close(); ot.close()
