"""W > 1 pinned against the oracle.

Two ranks share cuda:0, each with its OWN shard: envs seeded seed + r*N + i and the
main RNG on ChaCha stream r (bppo.dist.shard).  Rank r must reproduce, bit for bit,
rank r of the oracle's W-rank restatement (`or_trainers_update`, oracle/ppo.c): its
rollout (Gumbel words from stream r), its normalizers, its GAE, the Fisher-Yates
permutation of its rows from stream r and the RNG positions after rollout and update.
The update itself sums the two ranks' gradients (f32) and scales by 1/2 before clip
+ Adam, so both ranks' parameters must be IDENTICAL to each other and within the
parameter bar of the oracle's; the metrics are those of both ranks' rows together
(value_error_max, adv_*_raw and explained_variance per rank), 1e-5 relative.

The all-reduce runs two ways: host-staged gloo (bppo_set_allreduce: the stream is
drained before the callback) and the stream-ordered form bench.py uses
(bppo_set_allreduce_async, mode device_async: the reduction is enqueued on the
context's stream, here a gloo all-reduce of a CUDA tensor since RCCL cannot put
two ranks on one GPU).  A second round injects the oracle's parameters and checks
the second rollout and update the same way, through the pipelined bppo_train_steps."""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CASES = {
    # CfgB's net (2x64 relu: the MFMA rollout and minibatch kernels), obs + return normalizers
    "cartpole": dict(preset="cartpole", N=1024, T=32, over={}),
    # the GEMM-engine path with action masks and the configs' target_kl (6 epochs x 4)
    "connect_four": dict(preset="connect_four", N=256, T=16, over=dict(hidden_size=64)),
    # CTDE (actor on obs, critic on cat[priv, obs]), 4 epochs x 8 minibatches
    "liars_dice_ctde": dict(preset="liars_dice_ctde", N=256, T=8,
                            over=dict(hidden_size=64, critic_hidden_size=64, critic_num_hidden=2)),
    # shuffle_windows (bench.py's W > 1 mode): epoch e shuffles from S + e * (2B + 2^20)
    "cartpole_windows": dict(preset="cartpole", N=1024, T=32, over=dict(shuffle_windows=True)),
    "connect_four_windows": dict(preset="connect_four", N=256, T=16,
                                 over=dict(hidden_size=64, shuffle_windows=True)),
    # PopArt (normalize_values): each rank's statistics absorb both ranks' returns in rank
    # order (an all-gather of the batch statistics through the callback), so the value-head
    # rescale and the normalized targets agree and the ranks stay in lockstep
    "cartpole_popart": dict(preset="cartpole", N=1024, T=32, over=dict(normalize_values=True)),
    "connect_four_popart": dict(preset="connect_four", N=256, T=16, over=dict(hidden_size=64, normalize_values=True)),
    # opponent pools: each rank plays its own seat assignment against the same pool, so its
    # learner-row count differs from the other rank's; the minibatch slots run in lockstep
    # (per-rank sizes, one all-reduce each).  Three-call path only (round 1)
    "connect_four_opp": dict(preset="connect_four", N=128, T=16, over=dict(hidden_size=64), opp=(96, 2)),
    "liars_dice_opp": dict(preset="liars_dice_ctde", N=96, T=12,
                           over=dict(hidden_size=64, critic_hidden_size=64, critic_num_hidden=2), opp=(64, 3)),
}


def _opp_arrays(cfg, D, P, n_opp, K, rank):
    """the pool (the same models on every rank, one with its own obs normalizer) and this
    rank's seats (learner position, the model on every other seat, current opponents)"""
    import bppo
    rng = np.random.default_rng(100 + rank)
    params = np.stack([bppo.orthogonal_init(cfg, seed=300 + k) for k in range(K)])
    nrng = np.random.default_rng(7)
    norms = [None] * K
    norms[K - 1] = (nrng.normal(size=D) * 0.1, (nrng.random(D) + 0.5) * 500.0, 500.0)
    lp = rng.integers(0, P, n_opp).astype(np.int32)
    po = np.full((n_opp, P), -1, np.int32)
    for e in range(n_opp):
        for p in range(P):
            if p != lp[e]:
                po[e, p] = rng.integers(0, K)
    co = rng.integers(0, K, P - 1).astype(np.int32)
    return params, norms, lp, po, co


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_ranks(cfg, params, world):
    import oracle_ffi as O
    from parity_util import oracle_train_cfg
    return [O.Trainer(oracle_train_cfg(cfg, rank=r, world=world), params) for r in range(world)]


def _last_perm(seed, stream, start, B, epochs, windows=False, num_epochs=0):
    import oracle_ffi as O
    r = O.new_rng(seed)
    r.stream = stream
    r.word_pos = start
    win = 2 * B + (1 << 20)
    for e in range(epochs):
        if windows:
            r.word_pos = start + e * win
        p = np.arange(B, dtype=np.uint32)
        O.lib().or_shuffle_u32(C.byref(r), p, B)
    return p, (start + num_epochs * win if windows else r.word_pos)


def _worker(rank, world, port, q, case, mode):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {"rank": rank}
    try:
        import bppo
        import oracle_ffi as O
        from bppo.dist import make_allreduce
        from parity_util import assert_metrics_close, assert_params_close, bits
        from test_gpu_scale import cmp_cartpole_rollout, cmp_wide_rollout
        c = CASES[case]
        cfg = bppo.make_config(c["preset"], num_envs=c["N"], num_steps=c["T"], **c["over"])
        params = bppo.orthogonal_init(cfg, seed=7)
        tr = bppo.Trainer(cfg, params=params, rank=rank, world=world)
        if mode == "host_staged":
            tr.ctx.set_allreduce(make_allreduce(dist, mode="host_staged"), world)
        else:
            tr.ctx.set_allreduce(make_allreduce(dist, mode="device_async", stream=tr.ctx.stream), world,
                                 stream_ordered=True)
        ots = _oracle_ranks(cfg, params, world)      # both ranks' oracle (deterministic in every process)
        ot = ots[rank]
        env = cfg["env"]
        opp = c.get("opp")
        if opp:
            n_opp, K = opp
            D, P = {"connect_four": (86, 2), "liars_dice": (270, 4)}[env]
            for r, o in enumerate(ots):        # rank r: its own seats on n_opp - 16 r envs
                n_r = n_opp - 16 * r
                pr, nr, lp, po, co = _opp_arrays(cfg, D, P, n_r, K, r)
                o.set_opponents(pr, nr, n_r, lp, po.reshape(-1), co)
                if r == rank:
                    tr.ctx.set_opponents(pr, nr, n_r, lp, po, co)
        lr, ent = bppo.schedule_get(cfg["learning_rate"], 0), bppo.schedule_get(cfg["entropy_coef"], 0)
        # ---- round 1: the three calls, every stage compared --------------------------
        bppo.collect_rollouts(tr.ctx)
        for o in ots:
            o.collect()
        if env == "cartpole":
            cmp_cartpole_rollout(tr, ot)
        else:
            wide = {"connect_four": "connect_four", "liars_dice": "liars_dice"}[env]
            cmp_wide_rollout(wide, tr, ot)
        out["actions"] = tr.buffer.actions.reshape(-1).copy()
        if env == "cartpole":
            # the normalized rewards carry rtol 2e-7 (return-normalizer merge order): GAE
            # itself is compared on the oracle's rewards
            tr.ctx.set_buffer("rewards", ot.buffer("rewards"))
        bppo.compute_gae(tr.ctx)
        for o in ots:
            o.gae()
        assert np.array_equal(bits(tr.buffer.advantages.reshape(-1)), bits(ot.buffer("advantages")))
        assert np.array_equal(bits(tr.buffer.returns.reshape(-1)), bits(ot.buffer("returns")))
        start = tr.ctx.rng_pos()
        m = bppo.ppo_update(tr.ctx, lr, ent)
        oms = O.Trainer.update_ranks(ots)
        assert tr.ctx.rng_pos() == ot.rng_pos()
        B = c["N"] * c["T"]
        if not opp:     # (opponent pools shuffle the learner rows: the RNG position covers it)
            perm, end = _last_perm(cfg["seed"], rank, start, B, m["epochs_run"],
                                   bool(cfg.get("shuffle_windows")), cfg["num_epochs"])
            assert end == tr.ctx.rng_pos()
            assert np.array_equal(tr.ctx.buffer("perm", np.uint32)[:B], perm)
        if opp:
            vm = ot.buffer("valid") > 0.5
            assert np.array_equal(tr.ctx.buffer("valid"), ot.buffer("valid"))
            out["rows"] = int(vm.sum())
            assert_metrics_close(m, oms[rank], values=ot.buffer("values")[vm], returns=ot.buffer("returns")[vm],
                                 advantages=ot.buffer("advantages")[vm])
        else:
            assert_metrics_close(m, oms[rank], values=ot.buffer("values"), returns=ot.buffer("returns"), advantages=ot.buffer("advantages"))
        p1 = tr.model.get_params()
        assert_params_close(p1, ot.params())
        assert np.array_equal(bits(ots[0].params()), bits(ots[1].params()))   # the oracle's ranks agree
        out["p1"] = p1
        out["m1"] = m
        if cfg.get("normalize_values"):
            pd, po = tr.ctx.popart(), ot.popart()
            np.testing.assert_allclose(pd[:3], po[:3], rtol=1e-12)       # Chan merges vs the sequential Welford
            out["pa"] = pd
        if opp:                         # three-call path only
            out["p2"] = p1
            tr.close()
            for o in ots:
                o.close()
            out["ok"] = True
            return
        # ---- round 2: the oracle's state injected, the pipelined bench path -----------
        tr.model.set_params(ot.params())
        if cfg.get("normalize_values"):
            tr.ctx.set_popart(ot.popart())
        if env == "cartpole":
            mvc, rets = ot.ret_norm_state(returns=True)
            tr.ctx.set_ret_norm(mvc, rets)
            tr.ctx.set_obs_norm(*ot.obs_norm_state(5))
        ms2, _ = tr.train_updates(1)
        for o in ots:
            o.collect(); o.gae()
        assert np.array_equal(tr.buffer.actions.reshape(-1), ot.buffer("actions", np.int32))
        assert np.array_equal(bits(tr.buffer.log_probs.reshape(-1)), bits(ot.buffer("log_probs")))
        if env != "cartpole":   # the multi-player rollout is exact; CartPole's rewards carry rtol 2e-7
            assert np.array_equal(bits(tr.buffer.advantages.reshape(-1)), bits(ot.buffer("advantages")))
        oms2 = O.Trainer.update_ranks(ots)
        assert tr.ctx.rng_pos() == ot.rng_pos()
        assert_metrics_close(ms2[0], oms2[rank], values=ot.buffer("values"), returns=ot.buffer("returns"), advantages=ot.buffer("advantages"))
        p2 = tr.model.get_params()
        assert_params_close(p2, ot.params())
        out["p2"] = p2
        tr.close()
        for o in ots:
            o.close()
        out["ok"] = True
    except BaseException as e:   # report, so the parent fails with the reason instead of a timeout
        import traceback
        out["ok"] = False
        out["err"] = traceback.format_exc()[-4000:]
    finally:
        q.put(out)
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["host_staged", "device_async"])
@pytest.mark.parametrize("case", list(CASES))
def test_two_ranks_distinct_shards_match_oracle(case, mode):
    world, port = 2, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, case, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in range(world)), key=lambda d: d["rank"])
    for p in procs:
        p.join(60)
    for r in res:
        assert r["ok"], f"rank {r['rank']}:\n{r.get('err')}"
    for p in procs:
        assert p.exitcode == 0
    # the shards really differ (distinct env seeds and sampling streams) ...
    assert not np.array_equal(res[0]["actions"], res[1]["actions"])
    # ... and the ranks still take the same step
    for k in ("p1", "p2"):
        assert np.array_equal(res[0][k].view(np.uint32), res[1][k].view(np.uint32)), k
    if "pa" in res[0]:                  # PopArt: the same running statistics on both ranks
        assert np.array_equal(res[0]["pa"], res[1]["pa"])
    if "rows" in res[0]:                # opponent pools: the ranks trained on different row counts
        assert res[0]["rows"] != res[1]["rows"]
    for f in ("policy_loss", "value_loss", "approx_kl", "entropy", "clip_fraction", "value_error_std"):
        assert np.float32(res[0]["m1"][f]) == np.float32(res[1]["m1"][f]), f
