"""Explained variance as the reference computes it (ppo.rs:1268-1294):
bppo_set_explained_variance_mode(ctx, 1) makes UpdateMetrics.explained_variance the
reference's four sequential f32 sums over the buffer, bit for bit equal to the oracle's
restatement (or_explained_variance) and to a second, numpy restatement
(parity_util.ev_f32_sequential), at a size where that f32 value drifts ~1e-3 from the
exact one.  Mode 0 stays the f64 value.  The pipelined bppo_train_steps (the next
rollout enqueued behind the update, which rewrites the copied buffers) gives the same
bits as one call per update."""
import numpy as np
import pytest

import bppo
from parity_util import bits, cartpole_pair, ev_f32_sequential, ev_f64

pytestmark = pytest.mark.gpu


def test_reference_f32_explained_variance_cfgB_update():
    N, T = 8192, 128
    cfg, tr, ot = cartpole_pair(N, T)
    try:
        tr.ctx.set_explained_variance_mode(1)
        bppo.collect_rollouts(tr.ctx); ot.collect()
        tr.ctx.set_buffer("rewards", ot.buffer("rewards"))
        bppo.compute_gae(tr.ctx); ot.gae()
        v, r = ot.buffer("values"), ot.buffer("returns")
        assert np.array_equal(bits(tr.buffer.returns.reshape(-1)), bits(r))
        m = bppo.ppo_update(tr.ctx, 1e-3, 0.01)
        om = ot.update()
        ref = ev_f32_sequential(v, r)
        assert bits(np.float32(m["explained_variance"])) == bits(np.float32(om["explained_variance"])) == bits(ref)
        # the f32 value really differs from the exact one here (what mode 0 reports)
        assert abs(float(ref) - ev_f64(v, r)) > 1e-6
        tr.ctx.set_explained_variance_mode(0)
        bppo.collect_rollouts(tr.ctx); bppo.compute_gae(tr.ctx)
        v2, r2 = tr.buffer.values.reshape(-1), tr.buffer.returns.reshape(-1)
        m2 = bppo.ppo_update(tr.ctx, 1e-3, 0.01)
        assert abs(m2["explained_variance"] - ev_f64(v2, r2)) <= 1e-6
    finally:
        tr.close(); ot.close()


@pytest.mark.parametrize("preset,N,T", [("cartpole", 4096, 64), ("connect_four", 256, 16)])
def test_reference_ev_pipelined_equals_sequential(preset, N, T):
    cfg = bppo.make_config(preset, num_envs=N, num_steps=T, seed=5)
    a, b = bppo.Trainer(cfg, init_seed=2), bppo.Trainer(cfg, init_seed=2)
    try:
        for t in (a, b):
            t.ctx.set_explained_variance_mode(1)
        seq = []
        for _ in range(3):
            m = a.train_update(track_returns=True)        # collect, GAE, update: three calls
            v, r = a.buffer.values.reshape(-1), a.buffer.returns.reshape(-1)   # the update leaves them
            assert bits(np.float32(m["explained_variance"])) == bits(ev_f32_sequential(v, r))
            seq.append(m["explained_variance"])
        pip, _ = b.train_updates(3)
        assert [bits(np.float32(x["explained_variance"])) for x in pip] == [bits(np.float32(x)) for x in seq]
    finally:
        a.close(); b.close()
