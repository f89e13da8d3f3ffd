"""The split-bf16 minibatch kernel (k_update.hip k_minibatch_split, CfgB's 2x64 relu MLP)
pinned directly against the oracle.

By default the split kernel runs every minibatch of an update but the first, i.e. only
after an Adam step, where the parameters already differ from the oracle's in the last
bits.  bppo_set_minibatch_kernel(ctx, 2) runs it on the first minibatch too, so its
loss and gradient can be compared with the oracle's from IDENTICAL parameters and
identical buffers (ppo.rs:1923-1959: loss -> backward):

  * test_split_kernel_gradient_from_identical_parameters: one epoch x one minibatch over
    the whole buffer (N = 8,192 envs x T = 32), old log-probs and values perturbed so the
    ratio moves off 1 and both clip branches are taken; the losses within 1e-5 relative
    and every gradient entry within 1e-5 of its tensor's largest |entry|, for the split
    kernel (mode 2) and the exact kernel (mode 1) alike;
  * test_split_kernel_minibatch_by_minibatch: the CfgB update schedule (4 epochs x 4
    minibatches) at N = 8,192, T = 32, each of the 16 minibatches' statistics
    (bppo_minibatch_rows) against the oracle's (or_trainer_mb_log) at 1e-5, with the
    default kernel choice and with the split kernel on every minibatch.

The split arithmetic: every f32 operand x = x0 + x1 + x2 exactly (three RNE bf16 pieces),
the six products of order <= 2 accumulated in f32 by v_mfma_f32_32x32x16_bf16; each dropped
product (x1 y2, x2 y1, x2 y2) is at most 2^-24 |x y| (together <= 2^-23 + 2^-32), so a
product is within 2^-22 of x y after the f32 additions (tests/test_split_bf16.py emulates
it on the host).  These tests check the hardware's accumulation as it runs."""
import ctypes as C

import numpy as np
import pytest

import bppo
import oracle_ffi as O
from parity_util import bits, cartpole_pair, cmp_cartpole_rollout, summand_magnitude

pytestmark = pytest.mark.gpu

N, T = 8192, 32
TOL = 1e-5


def _rollout_gae(tr, ot):
    bppo.collect_rollouts(tr.ctx); ot.collect()
    cmp_cartpole_rollout(tr, ot)
    tr.ctx.set_buffer("rewards", ot.buffer("rewards"))   # return normalizer: rtol 2e-7 (merge order)
    bppo.compute_gae(tr.ctx); ot.gae()
    assert np.array_equal(bits(tr.buffer.advantages.reshape(-1)), bits(ot.buffer("advantages")))


@pytest.mark.parametrize("mode", [2, 1])
def test_split_kernel_gradient_from_identical_parameters(mode):
    cfg, tr, ot = cartpole_pair(N, T, num_epochs=1, num_minibatches=1, init_seed=3)
    try:
        tr.ctx.set_minibatch_kernel(mode)
        _rollout_gae(tr, ot)
        B = N * T
        rng = np.random.default_rng(11)
        logp = (ot.buffer("log_probs") + rng.normal(0, 0.3, B)).astype(np.float32)
        val = (ot.buffer("values") + rng.normal(0, 0.2, B)).astype(np.float32)
        tr.ctx.set_buffer("log_probs", logp); ot.set_buffer("log_probs", logp)
        tr.ctx.set_buffer("values", val); ot.set_buffer("values", val)
        p0 = tr.model.get_params()
        lr, ent = bppo.schedule_get(cfg["learning_rate"], 0), bppo.schedule_get(cfg["entropy_coef"], 0)
        m = bppo.ppo_update(tr.ctx, lr, ent)
        g = tr.ctx.buffer("grad")
        desc = O.mlp_desc(5, 2, 64, 2, True)
        adv = ot.buffer("advantages")
        advn = np.zeros(B, np.float32)
        st = [C.c_float() for _ in range(4)]
        O.lib().or_normalize_advantages(adv, B, advn, *[C.byref(x) for x in st])
        go = np.zeros(desc.n_params, np.float32)
        ms = O.MbStats()
        pc = O.ppo_cfg(num_epochs=1, num_minibatches=1, clip=cfg["clip_epsilon"], value_coef=cfg["value_coef"])
        O.lib().or_minibatch_loss_grad(C.byref(desc), p0, B, ot.buffer("obs"), None, ot.buffer("actions", np.int32),
                                       logp, advn, ot.buffer("returns"), val, None, C.byref(pc), ent, go,
                                       C.byref(ms))
        assert 0.05 < ms.clip_fraction < 0.95        # both clip branches are taken
        floors = {"policy_loss": summand_magnitude(adv), "value_loss": 0.0, "entropy": 0.0,
                  "approx_kl": 0.0, "clip_fraction": 1.0 / B}
        for k, fl in floors.items():
            o = getattr(ms, k)
            assert abs(m[k] - o) <= TOL * max(abs(o), fl), (k, m[k], o)
        shapes = [(5, 64), (64, 64), (64, 2), (64, 1)]     # record order: hidden, hidden, policy, value
        off = 0
        for i, o in shapes:
            for n in (i * o, o):
                a, b = g[off:off + n], go[off:off + n]
                np.testing.assert_allclose(a, b, rtol=0, atol=TOL * max(np.abs(b).max(), 1e-30),
                                           err_msg=f"tensor at {off} ({n} entries), kernel mode {mode}")
                off += n
        assert off == desc.n_params == g.size
    finally:
        tr.close(); ot.close()


@pytest.mark.parametrize("mode", [0, 2])
def test_split_kernel_minibatch_by_minibatch(mode):
    cfg, tr, ot = cartpole_pair(N, T, init_seed=5)
    try:
        assert (cfg["num_epochs"], cfg["num_minibatches"]) == (4, 4)     # configs/cartpole.toml
        tr.ctx.set_minibatch_kernel(mode)
        _rollout_gae(tr, ot)
        lr, ent = bppo.schedule_get(cfg["learning_rate"], 0), bppo.schedule_get(cfg["entropy_coef"], 0)
        bppo.ppo_update(tr.ctx, lr, ent)
        ot.update()
        rows, log = tr.ctx.minibatch_rows(), ot.minibatch_log()
        assert len(rows) == len(log) == 16
        mb = N * T // 4
        # relative to max(|oracle|, floor); policy_loss is a mean of signed summands -A_n ratio
        # that cancel (floor: their magnitude, tests/parity_util.py).  approx_kl: an ABSOLUTE
        # bound 2^-24 / sqrt(mb) besides: each row's (ratio - 1) - log(ratio) is evaluated in f32
        # from a ratio near 1 (resolution 2^-24), and on the first minibatch the split kernel's
        # ratio is 1 only to the last bits where the oracle's is exactly 1
        floors = {"policy_loss": summand_magnitude(ot.buffer("advantages")), "value_loss": 0.0, "entropy": 0.0,
                  "approx_kl": 0.0, "clip_fraction": 1.0 / mb, "value_mean": 0.0,
                  "returns_mean": 0.0, "value_error_mean": 0.0, "value_error_max": 0.0}
        absf = {"approx_kl": 2.0 ** -24 / np.sqrt(mb)}
        worst = []
        for k, (r, o) in enumerate(zip(rows, log)):
            n = r[10]
            assert n == mb
            dev = {"policy_loss": r[0] / n, "value_loss": 0.5 * r[1] / n, "entropy": r[2] / n,
                   "approx_kl": r[3] / n, "clip_fraction": r[4] / n, "value_mean": r[5] / n, "returns_mean": r[6] / n,
                   "value_error_mean": r[7] / n, "value_error_max": r[9]}
            # each field's error as a fraction of its tolerance
            rel = {f: abs(dev[f] - o[f]) / max(TOL * max(abs(o[f]), floors[f]), absf.get(f, 0.0), 1e-37) for f in dev}
            f = max(rel, key=rel.get)
            worst.append((k, f, rel[f]))
        bad = [w for w in worst if w[2] > 1.0]
        assert not bad, (mode, bad)
    finally:
        tr.close(); ot.close()



def test_first_minibatch_forward_is_exact():
    """The update's first minibatch runs with the rollout's parameters, so the reference's
    ratio is exactly 1 there.  Since r06 it runs k_minibatch_split<true> (the exact f32 forward
    of k_minibatch_mfma, the split-bf16 backward): every row's new log-prob must equal the
    stored one bit for bit, i.e. the minibatch's approx_kl sum and clip count are exactly 0
    (one differing row adds (ratio - 1) - log ratio != 0); the second minibatch, after an Adam
    step, is not at ratio 1.  CfgB's 4 x 4 schedule at N = 8,192, T = 32."""
    cfg, tr, ot = cartpole_pair(N, T, init_seed=5)
    try:
        _rollout_gae(tr, ot)
        lr, ent = bppo.schedule_get(cfg["learning_rate"], 0), bppo.schedule_get(cfg["entropy_coef"], 0)
        bppo.ppo_update(tr.ctx, lr, ent)
        rows = tr.ctx.minibatch_rows()
        assert rows[0][10] == N * T // 4
        assert rows[0][3] == 0.0 and rows[0][4] == 0.0, (rows[0][3], rows[0][4])
        assert rows[1][3] != 0.0
    finally:
        tr.close(); ot.close()
