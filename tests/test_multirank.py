"""N>1 data-parallel path: world_size-2 ranks.

CPU (gloo): the all-reduce callback libbppo calls once per minibatch leaves the
SUM over ranks in place, and the per-rank sharding (env seeds, RNG streams).
GPU (gloo, host-staged, both ranks on cuda:0): two ranks fed IDENTICAL shards
must apply the same step as one rank alone — x+x then x0.5 is exact in f32 — so
their parameters equal the single-rank run bit for bit, and the two ranks stay
in sync.  This pins the callback placement, the 1/world scaling before clip +
Adam, and the metric-partial reduction."""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import bppo
from bppo.dist import make_allreduce, shard
from bppo.host import to_struct


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _cpu_worker(rank, world, port, q):
    dist = _init(rank, world, port)
    try:
        fn = make_allreduce(dist, mode="host")
        n = 4739 + 11
        buf = (np.arange(n, dtype=np.float32) * (rank + 1)).astype(np.float32)
        fn(buf.ctypes.data, n)
        cfg = bppo.make_config("cartpole", num_envs=64)
        s = to_struct(cfg, rank, world, 64)
        q.put((rank, buf.copy(), s.env_seed_base, s.rng_stream))
    finally:
        dist.destroy_process_group()


def test_allreduce_callback_and_sharding_gloo():
    world, port = 2, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_cpu_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    n = res[0][1].size
    want = np.arange(n, dtype=np.float32) * 3
    for rank, buf, seed_base, stream in res:
        assert np.array_equal(buf, want)
        assert seed_base == 42 + rank * 64
        assert stream == rank
    assert shard(bppo.make_config("cartpole"), 0, 1, 64) == (42, 0)


def _gpu_worker(rank, world, port, q, updates, pipelined=False):
    dist = _init(rank, world, port)
    try:
        cfg = bppo.make_config("cartpole", num_envs=256, num_steps=32)
        # identical shards on purpose: rank=0 seeding for both processes
        tr = bppo.Trainer(cfg, device=0, init_seed=3)
        tr.ctx.set_allreduce(make_allreduce(dist, mode="host_staged"), world)
        ms = tr.train_updates(updates)[0] if pipelined else [tr.train_update() for _ in range(updates)]
        q.put((rank, tr.model.get_params(), ms[-1]["policy_loss"]))
        tr.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("pipelined", [False, True])
def test_two_ranks_identical_shards_match_single_rank(pipelined):
    updates = 3
    cfg = bppo.make_config("cartpole", num_envs=256, num_steps=32)
    solo = bppo.Trainer(cfg, device=0, init_seed=3)
    ms = [solo.train_update() for _ in range(updates)]
    p_solo = solo.model.get_params()
    solo.close()
    world, port = 2, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gpu_worker, args=(r, world, port, q, updates, pipelined)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert np.array_equal(res[0][1], res[1][1]), "ranks diverged"
    assert np.array_equal(res[0][1], p_solo)
    assert abs(res[0][2] - ms[-1]["policy_loss"]) <= 1e-6 + 1e-5 * abs(ms[-1]["policy_loss"])


@pytest.mark.gpu
@pytest.mark.parametrize("pipelined", [False, True])
def test_stream_ordered_allreduce_matches_single_rank(pipelined):
    """bppo_set_allreduce_async: the callback only ENQUEUES its reduction on the
    context's stream (staging copies + a torch op on an ExternalStream), with no
    host wait per minibatch.  An emulated 2-rank SUM of identical shards (x2,
    then libbppo's /2) must reproduce the single-rank parameters bit for bit,
    which fails if any of the enqueued steps ran out of order."""
    import torch
    from bppo.dist import make_allreduce
    updates = 3
    cfg = bppo.make_config("cartpole", num_envs=256, num_steps=32)
    solo = bppo.Trainer(cfg, device=0, init_seed=3)
    for _ in range(updates):
        solo.train_update()
    p_solo = solo.model.get_params()
    solo.close()
    tr = bppo.Trainer(cfg, device=0, init_seed=3)
    fn = make_allreduce(None, mode="device_async", stream=tr.ctx.stream, reduce=lambda t: t.mul_(2.0))
    tr.ctx.set_allreduce(fn, 2, stream_ordered=True)
    if pipelined:        # bench.py's form: bppo_train_steps, rollouts enqueued behind updates
        tr.train_updates(updates)
    else:
        for _ in range(updates):
            tr.train_update()
    p = tr.model.get_params()
    tr.close()
    assert np.array_equal(p, p_solo)


def test_bench_launcher_starts_world_size_ranks_gloo():
    """`bench.py --gpus N` must start N ranks itself (a
    torch.distributed.run child) and report n_gpus = N; --selftest runs the
    launcher, rank plumbing, barrier and max-over-ranks timing with gloo."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--selftest", "--steps", "3", "--warmup", "1"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["selftest"] and d["config"]["parallelism"] == "dp2"


def _rccl_worker(port, q, updates):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        cfg = bppo.make_config("cartpole", num_envs=256, num_steps=32)
        tr = bppo.Trainer(cfg, device=0, init_seed=3)
        # bench.py's N > 1 wiring: the RCCL all-reduce enqueued on the context's
        # stream through an ExternalStream (bppo_set_allreduce_async); a one-rank
        # group stands in for two ranks with identical shards (RCCL SUM, then x2,
        # then libbppo's 1/world), since the box has one GPU
        def reduce(t):
            dist.all_reduce(t)
            t.mul_(2.0)
        fn = make_allreduce(dist, mode="device_async", max_elems=tr.ctx.n_params + 64, stream=tr.ctx.stream,
                            reduce=reduce)
        calls = [0]

        def counted(ptr, n):
            calls[0] += 1
            fn(ptr, n)
        tr.ctx.set_allreduce(counted, 2, stream_ordered=True)
        tr.train_updates(updates)
        q.put((tr.model.get_params(), calls[0], dist.get_backend()))
        tr.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_rccl_collective_on_the_context_stream_world1():
    """The RCCL leg of SURVEY 8(e) executed on hardware: a one-rank "nccl" (= RCCL)
    process group, the all-reduce wired as bench.py wires it for N > 1 (device_async
    on the context's stream, stream_ordered), through the pipelined
    bppo_train_steps.  The RCCL SUM over one rank then x2 emulates two ranks with
    identical shards (x+x then /2 is exact in f32), so the parameters must equal the
    run without a collective bit for bit, and the callback must have run once per
    minibatch (ppo.rs:1661-2112: epochs x minibatches per update)."""
    updates = 3
    cfg = bppo.make_config("cartpole", num_envs=256, num_steps=32)
    solo = bppo.Trainer(cfg, device=0, init_seed=3)
    solo.train_updates(updates)
    p_solo = solo.model.get_params()
    solo.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_port(), q, updates))
    p.start()
    params, calls, backend = q.get(timeout=300)
    p.join(60)
    assert p.exitcode == 0
    assert backend == "nccl"
    assert calls == updates * cfg["num_epochs"] * cfg["num_minibatches"]
    assert np.array_equal(params, p_solo)
