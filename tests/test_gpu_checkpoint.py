"""Checkpoint interop through a device context (checkpoint.rs, main.rs:1276-1310
save; main.rs:294-414 resume):
  * save_rng_state draws 32 bytes = 8 words of the main RNG, the bytes the
    oracle's fill_bytes gives at the same position, and the device position
    moves by 8 (so checkpoint_freq shifts the sampling stream as in the reference);
  * a fresh context resumed from the files holds the same params, Adam state,
    normalizers and the RNG StdRng::from_seed(rng_state.bin);
  * the resumed context trains on like an oracle trainer resumed from the same
    files: rollout bit-exact, update within tests/parity_util.py's tolerances."""
import ctypes as C
import os

import numpy as np
import pytest

import bppo
import bppo._lib as L
import oracle_ffi as O
from bppo import checkpoint as K
from parity_util import assert_metrics_close, assert_params_close, cartpole_pair, cmp_cartpole_rollout

pytestmark = pytest.mark.gpu


def _opt(ctx):
    n = ctx.n_params
    m1, m2 = np.zeros(n, np.float32), np.zeros(n, np.float32)
    st = np.zeros(L.lib().bppo_num_param_tensors(ctx.h), np.int32)
    ctx._chk(L.lib().bppo_optimizer_get(ctx.h, m1.ctypes.data, m2.ctypes.data, st.ctypes.data, n))
    return m1, m2, st


def test_save_resume_continues_like_the_oracle(tmp_path):
    N, T = 256, 32
    cfg, tr, ot = cartpole_pair(N, T)
    for _ in range(2):
        tr.train_update()
    pos = tr.ctx.rng_pos()
    key = np.zeros(8, np.uint32)
    tr.ctx._chk(L.lib().bppo_rng_key_get(tr.ctx.h, key.ctypes.data))
    mgr = K.CheckpointManager(str(tmp_path))
    meta = K.CheckpointMetadata.for_config(cfg, tr.global_step, 100.0, recent_returns=[99.0, 101.0])
    path = K.save_training_checkpoint(mgr, tr.ctx, tr.model.get_params(), meta)
    # rng_state.bin = fill_bytes(32) of the main RNG at `pos` (rand_core BlockRng, LE words)
    r = O.Rng()
    O.lib().or_rng_seed_u64(C.byref(r), cfg["seed"])
    r.word_pos = pos
    ob = np.zeros(32, np.uint8)
    O.lib().or_rng_fill_bytes(C.byref(r), ob, 32)
    assert open(os.path.join(path, "rng_state.bin"), "rb").read() == ob.tobytes()
    assert tr.ctx.rng_pos() == pos + 8 == r.word_pos
    assert sorted(os.listdir(path)) == ["metadata.json", "model.mpk", "normalizer.json", "optimizer.mpk",
                                        "return_normalizer.json", "rng_state.bin"]
    saved = (tr.model.get_params(), _opt(tr.ctx), tr.ctx.obs_norm(), tr.ctx.ret_norm())
    tr.close(); ot.close()

    # resume into a fresh device context and a fresh oracle trainer
    cfg2, tr2, ot2 = cartpole_pair(N, T)
    m = K.resume_training_checkpoint(tr2.ctx, os.path.join(str(tmp_path), "checkpoints", "latest"))
    assert m.step == meta.step and m.recent_returns == [99.0, 101.0]
    assert np.array_equal(tr2.model.get_params(), saved[0])
    for a, b in zip(_opt(tr2.ctx), saved[1]):
        assert np.array_equal(a, b)
    for a, b in zip(tr2.ctx.obs_norm(), saved[2]):
        assert np.array_equal(np.asarray(a), np.asarray(b))
    for a, b in zip(tr2.ctx.ret_norm(), saved[3]):
        assert np.array_equal(a, b)
    assert tr2.ctx.rng_pos() == 0
    k2 = np.zeros(8, np.uint32)
    tr2.ctx._chk(L.lib().bppo_rng_key_get(tr2.ctx.h, k2.ctypes.data))
    assert np.array_equal(k2, ob.view("<u4"))                     # StdRng::from_seed(bytes)
    # the oracle resumed from the same files
    O.lib().or_trainer_set_params(ot2.h, np.ascontiguousarray(K.load_model(os.path.join(path, "model.mpk"))))
    m1, m2, st = saved[1]
    O.lib().or_trainer_set_adam(ot2.h, m1, m2, st, st.size)
    mean, m2n, cnt = saved[2]
    mvc, rets = saved[3]
    O.lib().or_trainer_set_norms(ot2.h, np.ascontiguousarray(mean).ctypes.data, np.ascontiguousarray(m2n).ctypes.data,
                                 float(cnt), np.ascontiguousarray(mvc).ctypes.data, np.ascontiguousarray(rets).ctypes.data)
    O.lib().or_trainer_set_rng(ot2.h, ob.view("<u4").copy(), 0)
    bppo.collect_rollouts(tr2.ctx); ot2.collect()
    cmp_cartpole_rollout(tr2, ot2)
    bppo.compute_gae(tr2.ctx); ot2.gae()
    tr2.ctx.set_buffer("advantages", ot2.buffer("advantages"))
    tr2.ctx.set_buffer("returns", ot2.buffer("returns"))
    md = bppo.ppo_update(tr2.ctx, 1e-3, 0.01)
    mo = ot2.update()
    assert tr2.ctx.rng_pos() == ot2.rng_pos()
    assert_metrics_close(md, mo, values=ot2.buffer("values"), returns=ot2.buffer("returns"), advantages=ot2.buffer("advantages"))
    assert_params_close(tr2.model.get_params(), ot2.params())
    tr2.close(); ot2.close()


def test_rng_state_wrong_length_is_an_error(tmp_path):
    cfg = bppo.make_config("cartpole", num_envs=16, num_steps=8)
    ctx = bppo.Context(cfg)
    (tmp_path / "rng_state.bin").write_bytes(b"\0" * 31)
    with pytest.raises(ValueError):
        K.load_rng_state(ctx, str(tmp_path))
    ctx.close()
