"""bench.py — env-steps/sec of burn-ppo's hot path (rollout + GAE + PPO update)
on MI355X.

One "step" = one full PPO update of CfgB: CartPole, num_envs=65536
per GPU, num_steps=128, 2x64 relu MLP, 4 epochs x 4 minibatches (configs/cartpole.toml),
i.e. 8,388,608 env-steps per GPU per step, synthetic fixed-seed data (seed 42).

N>1 runs as one process per GPU (torch.distributed.run): each rank owns its own
65536 envs (global env index rank*65536 + i) and the gradient is all-reduced
(RCCL over xGMI) once per minibatch, enqueued on the context's stream (the host
never waits per minibatch); weak scaling.

Prints ONE JSON line (rank 0).  `roofline` is the dominant kernel's (the fused
minibatch forward/backward) algorithmic FLOP rate against the FP32 dense peak;
`gae_roofline` the GAE scan's algorithmic HBM rate; `cpu_baseline` the CPU
oracle (a restatement of the reference's ndarray path) timed on a bounded sample
of the same workload on this host.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "burn-ppo_amd"))

METRIC = "env-steps/sec (rollout+GAE+PPO update) at 1/2/4/8 MI355X; steps-to-475-return CartPole"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3       # MI355X_MICROARCH.md: FP32 vector / matrix dense peak
FLOP_PER_ROW_FWD_BWD = 27_008  # CfgB forward + backward per env-step (per minibatch row)
GAE_BYTES_PER_ELEM = 20        # r, d, v in; adv, ret out (f32)
# rocprofv3 PMC, CfgB, per launch (profiles/r01k_pmc_traffic.txt). FETCH_SIZE/WRITE_SIZE are KiB;
# k_gae_1p's 16-B/lane streaming reads take the gfx950 x2 FETCH_SIZE correction, the minibatch
# kernel's 64-B row gathers do not (raw FETCH = 1.03 x the 2097152 x 64 B packed rows).
MB_TRAFFIC_BYTES = int((134902.7 + 4756.0) * 1024)
GAE_TRAFFIC_BYTES = int((2 * 49302.0 + 65536.0) * 1024)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--num-envs", type=int, default=65536, help="envs per GPU")
    p.add_argument("--num-steps", type=int, default=128)
    p.add_argument("--cpu-envs", type=int, default=1024, help="CPU baseline sample size (envs)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    return p.parse_args()


def cpu_baseline(args):
    """The oracle (CPU restatement of the reference ndarray path) on a bounded
    sample: same config, num_envs = --cpu-envs, one full update."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import oracle_ffi as O
    import bppo
    n = args.cpu_envs
    cfg = bppo.make_config("cartpole", num_envs=n, num_steps=args.num_steps)
    params = bppo.orthogonal_init(cfg, seed=0)
    ot = O.Trainer(O.train_cfg(num_envs=n, num_steps=args.num_steps, lr=1e-3), params)
    t0 = time.perf_counter()
    ot.collect(); ot.gae(); ot.update()
    dt = time.perf_counter() - t0
    ot.close()
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return {"value": n * args.num_steps / dt, "unit": "env-steps/sec", "cores": threads,
            "kind": "port",
            "sample": f"1 full update (rollout+GAE+4x4 PPO) of CfgB at num_envs={n}, T={args.num_steps}; "
                      f"env stepping OpenMP x{threads}, MLP/GAE/shuffle single-threaded; {dt:.1f}s"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch
    import bppo
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    else:
        torch.cuda.set_device(0)
    N, T = args.num_envs, args.num_steps
    cfg = bppo.make_config("cartpole", num_envs=N * world, num_steps=T)
    tr = bppo.Trainer(cfg, device=local, init_seed=0, rank=rank, world=world, envs_per_rank=N)
    if world > 1:
        # RCCL all-reduce of the gradient enqueued on the context's stream: no
        # host wait per minibatch (bppo_set_allreduce_async)
        from bppo.dist import make_allreduce
        fn = make_allreduce(dist, mode="device_async", max_elems=tr.ctx.n_params + 64, stream=tr.ctx.stream)
        tr.ctx.set_allreduce(fn, world, stream_ordered=True)

    for _ in range(args.warmup):
        tr.train_update()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    phase = {"rollout": 0.0, "return_norm": 0.0, "gae": 0.0, "minibatch": 0.0, "shuffle": 0.0, "update": 0.0,
             "shuffle_walk": 0.0, "shuffle_wait": 0.0, "shuffle_met": 0.0}
    last = None
    for _ in range(args.steps):
        last = tr.train_update()
        for k in phase:
            phase[k] += tr.ctx.kernel_ms(k)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    if rank != 0:
        dist.destroy_process_group()
        return
    env_steps = N * T * world * args.steps
    value = env_steps / dt
    ms_step = dt / args.steps * 1000.0
    # dominant kernel: the fused minibatch forward/loss/backward (16 launches per update)
    mb_rows = N * T // cfg["num_minibatches"]
    mb_ms = phase["minibatch"] / args.steps          # last minibatch launch of each update
    flops = mb_rows * FLOP_PER_ROW_FWD_BWD
    achieved = flops / (mb_ms * 1e-3) / 1e12
    # HBM bytes per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes on CfgB
    # (scripts/pmc_traffic.sh, profiles/r01k_pmc_traffic.txt); PMC cannot be read live here,
    # so it is reported only for the configuration it was measured on.
    pmc_cfg = (N == 65536 and T == 128 and cfg["num_minibatches"] == 4)
    roof = {"bound": "mfma", "achieved": round(achieved, 3), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / FP32_PEAK_TFLOPS, 4),
            "traffic": MB_TRAFFIC_BYTES if pmc_cfg else None, "traffic_unit": "B/launch",
            "kernel": "k_minibatch_mfma", "launch_ms": round(mb_ms, 4),
            "algorithmic": f"{mb_rows} rows x {FLOP_PER_ROW_FWD_BWD} FLOP"}
    gae_ms = phase["gae"] / args.steps
    gae_bytes = N * T * GAE_BYTES_PER_ELEM
    gae_gbs = gae_bytes / (gae_ms * 1e-3) / 1e9
    gae_roof = {"bound": "hbm", "achieved": round(gae_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(gae_gbs / HBM_PEAK_GBS, 4), "traffic": GAE_TRAFFIC_BYTES if pmc_cfg else None,
                "traffic_unit": "B/launch", "kernel": "k_gae_1p",
                "launch_ms": round(gae_ms, 4), "algorithmic": f"{N * T} x {GAE_BYTES_PER_ELEM} B"}
    out = {"metric": METRIC, "value": round(value, 1), "unit": "env-steps/sec", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
           "data": "synthetic (fixed-seed CartPole envs, orthogonal-init weights)",
           "config": {"workload": "CfgB: CartPole num_envs=65536/GPU num_steps=128, 2x64 relu MLP, "
                                  "4 epochs x 4 minibatches (configs/cartpole.toml)",
                      "num_envs_per_gpu": N, "num_steps": T, "env_steps_per_update": N * T * world,
                      "parallelism": f"dp{world}"},
           "roofline": roof, "gae_roofline": gae_roof,
           "phase_ms_per_update": {k: round(v / args.steps, 3) for k, v in phase.items()},
           "last_update": {k: (round(v, 5) if isinstance(v, float) else v) for k, v in last.items()
                           if k in ("policy_loss", "value_loss", "entropy", "approx_kl", "mean_return",
                                    "episodes", "explained_variance")}}
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args)
    else:
        out["cpu_baseline"] = None
    print(json.dumps(out), flush=True)
    tr.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
