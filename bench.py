"""bench.py — env-steps/sec of burn-ppo's hot path (rollout + GAE + PPO update)
on MI355X, plus the CartPole steps-to-475 learning metric.

One "step" = one full PPO update of CfgB: CartPole, num_envs=65536
per GPU, num_steps=128, 2x64 relu MLP, 4 epochs x 4 minibatches (configs/cartpole.toml),
i.e. 8,388,608 env-steps per GPU per step, synthetic fixed-seed data (seed 42).

N>1 runs as one process per GPU.  `python bench.py --gpus N` starts the N ranks
itself (a torch.distributed.run child process) when it is not already running
under a launcher; each rank owns its own 65536 envs (global env index
rank*65536 + i) and the gradient is all-reduced (RCCL over xGMI, the
torch.distributed "nccl" backend) once per minibatch, enqueued on the context's
stream (the host never waits per minibatch); weak scaling.

Prints ONE JSON line (rank 0):
  roofline      the dominant kernel (fused minibatch forward/loss/backward):
                algorithmic FLOP rate against the FP32 dense peak, timed with HIP
                events on the context's stream; `traffic` = HBM bytes per launch
                from the rocprofv3 PMC passes in pmc_traffic.json, reported only
                when that profile was taken of the current kernel source;
  gae_roofline  the GAE scan's algorithmic HBM rate (north star: >= 40 %);
  steps_to_475  global_step at which the 100-episode rolling mean return
                (main.rs:842-853) first reaches 475 (CartPole-v1 solved, max 500),
                for CfgB and for configs/cartpole.toml (N=32, T=128), trained
                outside the timed region (rank 0, N=1 only);
  cpu_baseline  the CPU oracle (C restatement of the reference's ndarray path)
                timed on a bounded sample of the same workload on this host.
`--selftest` runs the launcher, rank plumbing, barrier and max-over-ranks
timing with gloo and no GPU work (the CPU test of the N>1 harness).
"""
import argparse
import hashlib
import json
import resource
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "burn-ppo_amd"))

METRIC = "env-steps/sec (rollout+GAE+PPO update) at 1/2/4/8 MI355X; steps-to-475-return CartPole"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3       # MI355X_MICROARCH.md: FP32 vector / matrix dense peak
FLOP_PER_ROW_FWD_BWD = 27_008  # CfgB forward + backward per env-step (per minibatch row)
GAE_BYTES_PER_ELEM = 28        # r, d, v in; adv, ret out (f32) = 20 B, plus the
                               # [advantage, return] pair of the minibatch rows the bench path writes (8 B)
TRAFFIC_JSON = os.path.join(ROOT, "pmc_traffic.json")   # copy of a scripts/pmc_traffic.sh summary
CSRC = os.path.join(ROOT, "burn-ppo_amd", "csrc")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--num-envs", type=int, default=65536, help="envs per GPU")
    p.add_argument("--num-steps", type=int, default=128)
    p.add_argument("--cpu-envs", type=int, default=8192, help="CPU baseline sample size (envs)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-learning", action="store_true", help="skip the steps-to-475 runs")
    p.add_argument("--no-gae-isolated", action="store_true",
                   help="skip the isolated GAE launches (kernel traces of the in-loop launches only)")
    p.add_argument("--selftest", action="store_true", help="N>1 harness check with gloo and no GPU work")
    p.add_argument("--host-cpus", type=int, default=0,
                   help="pin each rank to K host CPUs (its share of an 8-rank node) and size the shuffle "
                        "engine's threads for K (BPPO_HOST_THREADS); default: affinity/quota / ranks per node")
    p.add_argument("--shuffle-windows", choices=("auto", "on", "off"), default="auto",
                   help="the shuffle_windows mode (epoch e of an update shuffles from a fixed window of the "
                        "rank's RNG stream, so the host walks all epochs at once: bppo.h): auto = on for N>1 "
                        "(per-rank streams already depart from the reference's), off at N=1 (reference-exact)")
    return p.parse_args()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """--gpus N without a launcher: run N ranks under torch.distributed.run as a
    CHILD process (nothing here has touched the GPU) and exit with its code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def cgroup_cpu_quota():
    """CPUs the cgroup (v2 cpu.max) lets this process use, or None if unlimited/unknown."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def thread_cpu_ms():
    """CPU time (ms) of this process's threads summed by thread name (/proc task stat)."""
    out = {}
    tick = os.sysconf("SC_CLK_TCK")
    for t in os.listdir("/proc/self/task"):
        try:
            st = open(f"/proc/self/task/{t}/stat").read()
        except OSError:
            continue
        name = st[st.index("(") + 1:st.rindex(")")]
        f = st[st.rindex(")") + 2:].split()
        out[name] = out.get(name, 0.0) + (int(f[11]) + int(f[12])) * 1000.0 / tick
    return out


def idle_cpus_sample(cpus, secs):
    """busy fraction of each CPU over `secs` (/proc/stat deltas)"""
    def snap():
        out = {}
        for line in open("/proc/stat"):
            if line.startswith("cpu") and line[3].isdigit():
                f = line.split()
                v = [int(x) for x in f[1:]]
                out[int(f[0][3:])] = (sum(v), v[3] + v[4])     # total, idle + iowait
        return out
    a = snap()
    time.sleep(secs)
    b = snap()
    busy = {}
    for c in cpus:
        if c in a and c in b and b[c][0] > a[c][0]:
            busy[c] = 1.0 - (b[c][1] - a[c][1]) / (b[c][0] - a[c][0])
    return busy


def host_cpu_budget(local_world):
    """CPUs this rank may use for the shuffle engine's host threads: the CPUs
    the process may run on (affinity, cgroup quota) / ranks on this node."""
    n = len(os.sched_getaffinity(0))
    q = cgroup_cpu_quota()
    if q is not None:
        n = min(n, max(1, int(q)))
    return max(1, n // max(1, local_world))


def traffic_for(kernel, source):
    """HBM bytes per launch from the committed PMC summary, only if it profiled
    the current source of the kernel."""
    try:
        prof = json.load(open(TRAFFIC_JSON))
        e = prof["kernels"][kernel]
    except (OSError, KeyError, ValueError):
        return None, "no PMC profile"
    sha = hashlib.sha256(open(os.path.join(CSRC, source), "rb").read()).hexdigest()[:16]
    if e.get("source_sha") != sha or "traffic_bytes" not in e:
        return None, f"PMC profile {prof.get('tag')} is of other {source} source"
    return e["traffic_bytes"], f"rocprofv3 FETCH_SIZE x{e['fetch_correction']:g} + WRITE_SIZE ({prof.get('tag')})"


def cpu_baseline(args):
    """The oracle (C restatement of the reference ndarray path) on a bounded
    sample: CfgB's config at num_envs = --cpu-envs, 1 warm-up update then 2
    timed full updates.  Env stepping OpenMP over all host threads (rayon in the
    reference); MLP, GAE, normalizers, sampling and shuffle single-threaded (the
    reference's matrixmultiply sgemm and serial loops).  Every phase is linear in
    T*N, so env-steps/s at this N stands for CfgB's."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    import bppo
    n = args.cpu_envs
    cfg = bppo.make_config("cartpole", num_envs=n, num_steps=args.num_steps)
    params = bppo.orthogonal_init(cfg, seed=0)
    O.lib().or_set_mlp_parallel(0)
    ot = O.Trainer(O.train_cfg(num_envs=n, num_steps=args.num_steps, lr=1e-3), params)
    ot.collect(); ot.gae(); ot.update()          # warm-up
    t0 = time.perf_counter()
    for _ in range(2):
        ot.collect(); ot.gae(); ot.update()
    dt = time.perf_counter() - t0
    ot.close()
    O.lib().or_set_mlp_parallel(1)
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": 2 * n * args.num_steps / dt, "unit": "env-steps/sec", "cores": threads, "kind": "port",
            "cpu": model, "cfgA": cpu_baseline_cfgA(),
            "sample": f"CfgB config (cartpole.toml, 2x64 relu, 4x4 PPO) at num_envs={n}, T={args.num_steps}: "
                      f"1 warm-up + 2 timed full updates (rollout+GAE+update) = {2 * n * args.num_steps} env-steps "
                      f"in {dt:.1f}s; env stepping OpenMP x{threads}, MLP/GAE/normalizers/sampling/shuffle "
                      f"single-threaded as in the reference; per-env-step cost is independent of N"}


def cpu_baseline_cfgA(seconds=5.0):
    """BASELINE.json configs[0]: configs/test.toml at --num-envs 8 --num-steps 128 (1x16 relu,
    1 epoch x 1 minibatch) on the oracle, from the committed weights tests/golden/w_cfgA.npz
    (SURVEY 8(d)), single-threaded as the reference's ndarray path; full updates until
    `seconds` have passed."""
    import numpy as np
    import oracle_ffi as O
    import bppo
    from parity_util import oracle_train_cfg
    w = np.load(os.path.join(ROOT, "tests", "golden", "w_cfgA.npz"))
    cfg = bppo.make_config("test", num_envs=int(w["num_envs"]), num_steps=int(w["num_steps"]))
    O.lib().or_set_mlp_parallel(0)
    ot = O.Trainer(oracle_train_cfg(cfg, threads=1), np.ascontiguousarray(w["params"]))
    ot.collect(); ot.gae(); ot.update()                 # warm-up
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        ot.collect(); ot.gae(); ot.update()
        n += 1
    dt = time.perf_counter() - t0
    ot.close()
    O.lib().or_set_mlp_parallel(1)
    steps = n * cfg["num_envs"] * cfg["num_steps"]
    return {"value": steps / dt, "unit": "env-steps/sec", "cores": 1, "kind": "port",
            "sample": f"CfgA (configs/test.toml, --num-envs 8 --num-steps 128, weights tests/golden/w_cfgA.npz): "
                      f"{n} full updates = {steps} env-steps in {dt:.1f}s, one thread"}


def gae_isolated_ms(N, T, gamma=0.99, lam=0.95, reps=20):
    """k_gae_1p_seg at the workload's [T, N] shape on its own stream, nothing else on
    the GPU, in the variant the update loop runs: it also stores the advantage /
    return pair of every packed 64-byte update row (bppo_gae_rows_device).  In the
    loop it co-runs with the side-stream Fisher-Yates passes, so its in-loop
    duration measures the sharing, not the kernel."""
    import torch
    from bppo import _lib as L
    g = torch.Generator(device="cuda").manual_seed(0)
    r = torch.rand(T, N, device="cuda", generator=g)
    d = (torch.rand(T, N, device="cuda", generator=g) < 0.01).float()
    v = torch.rand(T, N, device="cuda", generator=g)
    lv = torch.rand(N, device="cuda", generator=g)
    adv, ret = torch.empty_like(r), torch.empty_like(r)
    rows = torch.zeros(T * N * 2, device="cuda")
    st = torch.cuda.Stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()

    def once():
        rc = L.lib().bppo_gae_rows_device(r.data_ptr(), d.data_ptr(), v.data_ptr(), lv.data_ptr(), T, N, gamma,
                                          lam, adv.data_ptr(), ret.data_ptr(), rows.data_ptr(), st.cuda_stream)
        if rc != 0:
            raise RuntimeError(f"bppo_gae_rows_device status {rc}")
    with torch.cuda.stream(st):
        for _ in range(3):
            once()
        e0.record(st)
        for _ in range(reps):
            once()
        e1.record(st)
    st.synchronize()
    return e0.elapsed_time(e1) / reps


def steps_to_475(bppo, preset_over, max_steps, init_seed=0):
    """Train until the 100-episode rolling mean return (main.rs:842-853) reaches
    475; -> global_step after that rollout, or None within max_steps."""
    cfg = bppo.make_config("cartpole", **preset_over)
    tr = bppo.Trainer(cfg, init_seed=init_seed)
    T, N = cfg["num_steps"], cfg["num_envs"]
    step, best, reached, t0 = 0, 0.0, None, time.perf_counter()
    try:
        while step < max_steps:
            tr.train_update(track_returns=True)
            step += T * N
            mr = tr.mean_recent_return()
            best = max(best, mr)
            if len(tr.recent_returns) == 100 and mr >= 475.0:
                reached = step
                break
    finally:
        tr.close()
    return {"steps": reached, "best_mean_return": round(best, 2), "updates": step // (T * N),
            "num_envs": N, "num_steps": T, "seconds": round(time.perf_counter() - t0, 2)}


def selftest_main(args, world, rank):
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    x = torch.ones(4)
    for _ in range(args.warmup):
        dist.all_reduce(x)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dist.all_reduce(x)
    dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        assert world == args.gpus, (world, args.gpus)
        print(json.dumps({"metric": METRIC, "value": None, "unit": "env-steps/sec", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "ms_per_step": float(t.item()) / args.steps * 1e3,
                          "higher_is_better": True, "scaling": "weak", "selftest": True,
                          "data": "selftest: launcher + gloo ranks, no GPU work",
                          "config": {"parallelism": f"dp{world}", "backend": "gloo"}}), flush=True)
    dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    if args.selftest:
        return selftest_main(args, world, rank)
    if args.host_cpus > 0:
        # before any GPU call: the runtime's and the engine's threads inherit the mask.
        # The K CPUs are the idlest ones over a 0.5 s sample (the box's other tenants
        # run on some of its CPUs: pinning to busy ones measures their load, not a
        # K-CPU budget -- r03b's first-K pinning ran 31.8 ms/step at K = 16)
        k = args.host_cpus
        cpus = sorted(os.sched_getaffinity(0))
        busy = idle_cpus_sample(cpus, 0.5)
        ranked = sorted(cpus, key=lambda c: busy.get(c, 1.0))
        mine = ranked[local * k:(local + 1) * k] if len(ranked) >= (local + 1) * k else ranked[:k]
        os.sched_setaffinity(0, mine)
        os.environ["BPPO_HOST_THREADS"] = str(len(mine))
        os.environ["BPPO_BENCH_PINNED_BUSY"] = f"{sum(busy.get(c, 1.0) for c in mine) / len(mine):.3f}"
    os.environ.setdefault("BPPO_HOST_THREADS", str(host_cpu_budget(local_world)))

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
    windows = args.shuffle_windows == "on" or (args.shuffle_windows == "auto" and world > 1)
    cfg = bppo.make_config("cartpole", num_envs=N * world, num_steps=T, shuffle_windows=windows)
    tr = bppo.Trainer(cfg, device=local, init_seed=0, rank=rank, world=world, envs_per_rank=N)
    if world > 1:
        # RCCL all-reduce of the gradient enqueued on the context's stream: no
        # host wait per minibatch (bppo_set_allreduce_async)
        from bppo.dist import make_allreduce
        fn = make_allreduce(dist, mode="device_async", max_elems=tr.ctx.n_params + 64, stream=tr.ctx.stream)
        tr.ctx.set_allreduce(fn, world, stream_ordered=True)

    try:   # name the driving thread (after the runtime's threads exist: they inherit the name
        # at creation) so host_cpu_ms_per_step_by_thread tells it from them
        import ctypes
        ctypes.CDLL(None).prctl(15, b"bench-main", 0, 0, 0)       # PR_SET_NAME
    except (OSError, AttributeError):
        pass
    # BPPO_BENCH_EXTRA_STREAMS=k (diagnostic): k more torch streams with one small kernel each
    # before the timed region, as a multi-rank run's collective streams would add (an idle extra
    # low-priority stream of the library cost ~2.5 ms per update)
    extra = [torch.cuda.Stream() for _ in range(int(os.environ.get("BPPO_BENCH_EXTRA_STREAMS", "0")))]
    for st_x in extra:
        with torch.cuda.stream(st_x):
            torch.zeros(1024, device="cuda").add_(1.0)
    tr.train_updates(args.warmup)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    th0 = thread_cpu_ms()
    phase = {"rollout": 0.0, "return_norm": 0.0, "gae": 0.0, "minibatch": 0.0, "shuffle": 0.0, "update": 0.0,
             "shuffle_walk": 0.0, "shuffle_wait": 0.0, "shuffle_met": 0.0,
             "shuffle_spec_mwords": 0.0, "shuffle_true_mwords": 0.0,
             "shuffle_walk_tsc_ms": 0.0, "shuffle_words_tsc_ms": 0.0, "host_enqueue": 0.0, "host_sync_wait": 0.0,
             "minibatch_kernel": 0.0, "minibatch_kernel_min": 0.0, "minibatch_kernel_max": 0.0,
             "minibatch_kernel_split": 0.0, "minibatch_kernel_exact": 0.0}
    # the K updates in one pipelined call (bppo_train_steps: each rollout enqueued behind
    # the previous update, per-update phase times summed on the host side of the library)
    if os.environ.get("BPPO_BENCH_SEQUENTIAL") == "1":     # A/B: one train_update call per step
        last = None
        for _ in range(args.steps):
            last = tr.train_update()
            for k in phase:
                phase[k] += tr.ctx.kernel_ms(k)
    else:
        mets, sums = tr.train_updates(args.steps, tuple(phase))
        phase.update(sums)
        last = mets[-1]
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    th1 = thread_cpu_ms()
    host_cpu_threads = {k: round((v - th0.get(k, 0.0)) / args.steps, 1) for k, v in th1.items()
                        if v - th0.get(k, 0.0) > 0.5 * args.steps}
    if os.environ.get("BPPO_BENCH_THREADS") == "1":      # diagnostic: every thread's CPU and wait channel
        tick = os.sysconf("SC_CLK_TCK")
        for t in sorted(os.listdir("/proc/self/task"), key=int):
            try:
                st = open(f"/proc/self/task/{t}/stat").read()
                wch = open(f"/proc/self/task/{t}/wchan").read()
            except OSError:
                continue
            f = st[st.rindex(")") + 2:].split()
            ms = (int(f[11]) + int(f[12])) * 1000.0 / tick
            if ms > 0:
                print(f"thread {t} {st[st.index('(') + 1:st.rindex(')')]:16s} cpu {ms:9.1f} ms wchan {wch}",
                      file=sys.stderr)
    host_cpu_ms = ((ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)) * 1e3 / args.steps
    if dist:
        t = torch.tensor([dt], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    tr.close()
    if rank != 0:
        dist.destroy_process_group()
        return
    env_steps = N * T * world * args.steps
    value = env_steps / dt
    ms_step = dt / args.steps * 1000.0
    # dominant kernel: the fused minibatch forward/loss/backward (16 launches per update):
    # k_minibatch_split for 15 of them; the update's first (ratio exactly 1) runs its exact-forward
    # variant k_minibatch_split<true> (r06; k_minibatch_mfma with BPPO_MB_FIRST_MFMA=1)
    mb_rows = N * T // cfg["num_minibatches"]
    # the kernel alone (HIP events around EVERY launch, on its stream): the mean of the
    # split kernel's launches; the side-stream shuffle passes share the GPU with some of
    # them (min / max over all 16 launches reported beside it)
    mb_all = phase["minibatch_kernel"] / args.steps
    mb_ms = phase["minibatch_kernel_split"] / args.steps or mb_all
    mb_ex = phase["minibatch_kernel_exact"] / args.steps
    mb_min, mb_max = phase["minibatch_kernel_min"] / args.steps, phase["minibatch_kernel_max"] / args.steps
    flop = mb_rows * FLOP_PER_ROW_FWD_BWD
    # (no timed launches, BPPO_MB_EVENTS=0 diagnostic runs: no roofline figure)
    achieved = flop / (mb_ms * 1e-3) / 1e12 if mb_ms > 0 else 0.0
    cfgB = (N == 65536 and T == 128)
    kname = "k_minibatch_split" if phase["minibatch_kernel_split"] > 0 else "k_minibatch_mfma"
    mb_tr, mb_src = traffic_for(kname, "k_update.hip") if cfgB else (None, "not the profiled shape")
    roof = {"bound": "mfma", "achieved": round(achieved, 3), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / FP32_PEAK_TFLOPS, 4), "traffic": mb_tr, "traffic_unit": "B/launch",
            "traffic_source": mb_src, "kernel": kname, "launch_ms": round(mb_ms, 4),
            "launch_ms_min_max": [round(mb_min, 4), round(mb_max, 4)],
            "measured": "mean over the split kernel's minibatch launches of the timed updates (15 of 16 per "
                        "update; HIP events around each launch)",
            "algorithmic": f"{mb_rows} rows x {FLOP_PER_ROW_FWD_BWD} FLOP",
            # the 64x64 contractions run as six bf16 products per f32 product (exact 3-piece splits): their
            # matrix-pipe ceiling is 16/6 of the f32 one; layer 1 and the dZ2 step stay on the f32 MFMA
            "split_note": "f32-accurate: layer 2, dZ1 and dW1 on v_mfma_f32_32x32x16_bf16 with operands split "
                          "exactly into 3 bf16 pieces (6 products); peak quoted is the FP32 MFMA peak",
            "exact_first_minibatch": {"kernel": "k_minibatch_mfma" if os.environ.get("BPPO_MB_FIRST_MFMA") == "1"
                                      else "k_minibatch_split<true> (exact f32 forward, split-bf16 backward)",
                                      "launch_ms": round(mb_ex, 4),
                                      "frac": round(flop / (mb_ex * 1e-3) / 1e12 / FP32_PEAK_TFLOPS, 4)
                                      if mb_ex > 0 else None},
            "mean_all_launches_ms": round(mb_all, 4)}
    gae_loop_ms = phase["gae"] / args.steps
    gae_ms = gae_loop_ms if args.no_gae_isolated else gae_isolated_ms(N, T)
    gae_gbs = N * T * GAE_BYTES_PER_ELEM / (gae_ms * 1e-3) / 1e9
    g_tr, g_src = traffic_for("k_gae_1p_seg", "k_gae.hip") if cfgB else (None, "not the profiled shape")
    gae_roof = {"bound": "hbm", "achieved": round(gae_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(gae_gbs / HBM_PEAK_GBS, 4), "traffic": g_tr, "traffic_unit": "B/launch",
                "traffic_source": g_src, "kernel": "k_gae_1p_seg", "launch_ms": round(gae_ms, 4),
                "measured": "achieved: isolated launches of the in-loop variant ([advantage, return] "
                            "pair of each minibatch row stored too) at the workload shape after the timed region "
                            "(HIP events on the launch stream); launch_ms_in_loop: the same kernel inside the "
                            "update loop, where every launch overlaps the side-stream Fisher-Yates passes "
                            "(k_fyb_link / k_fy_final, random-access HBM) of the update's first epoch: "
                            "scripts/kt_overlap.py on the kernel trace, profiles/r03_gae_overlap.txt",
                "launch_ms_in_loop": round(gae_loop_ms, 4),
                "algorithmic": f"{N * T} x {GAE_BYTES_PER_ELEM} B"}
    out = {"metric": METRIC, "value": round(value, 1), "unit": "env-steps/sec", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
           "data": "synthetic (fixed-seed CartPole envs, orthogonal-init weights)",
           "config": {"workload": "CfgB: CartPole num_envs=65536/GPU num_steps=128, 2x64 relu MLP, "
                                  "4 epochs x 4 minibatches (configs/cartpole.toml)",
                      "num_envs_per_gpu": N, "num_steps": T, "env_steps_per_update": N * T * world,
                      "parallelism": f"dp{world}",
                      "collective": ("RCCL all-reduce (torch.distributed nccl) of the gradient, 1 per minibatch, "
                                     "stream-ordered" if world > 1 else None),
                      "w_gt_1_semantics": ("rank r: envs seed+r*N+i, ChaCha stream r, per-rank obs/return "
                                           "normalizers and minibatch advantage stats, gradients summed then /W "
                                           "(oracle-pinned: tests/test_gpu_multirank.py); shuffle_windows "
                                           "epoch placement (config.shuffle)" if world > 1 else None),
                      "shuffle": ("shuffle_windows: epoch e shuffles from S + e*(2B + 2^20), all epochs "
                                  "walked at once" if windows else "sequential (the reference's word positions)"),
                      "host_cpus_per_rank": int(os.environ["BPPO_HOST_THREADS"]),
                      "host_cpu_affinity": len(os.sched_getaffinity(0)),
                      "host_cpu_quota": cgroup_cpu_quota(),
                      "host_cpus_pinned_busy_before": (float(os.environ["BPPO_BENCH_PINNED_BUSY"])
                                                       if "BPPO_BENCH_PINNED_BUSY" in os.environ else None)},
           # this process's CPU time per update over the timed region (all threads:
           # shuffle engine walkers and word producers, the driver thread, HIP runtime)
           "host_cpu_ms_per_step": round(host_cpu_ms, 2),
           "host_cpu_ms_per_step_by_thread": host_cpu_threads,
           "roofline": roof, "gae_roofline": gae_roof,
           "phase_ms_per_update": {k: round(v / args.steps, 3) for k, v in phase.items()},
           # the reference's perf/* scalars (main.rs:1092-1132) over the timed interval: the
           # job's env steps per second and the phases' summed device seconds (rollout = the
           # rollout kernels + return normalizer; gae = GAE; update = the PPO update)
           "perf": {k: round(v, 6) for k, v in bppo.perf_scalars(
               env_steps, dt, phase["rollout"] + phase["return_norm"], phase["gae"], phase["update"]).items()},
           "last_update": {k: (round(v, 5) if isinstance(v, float) else v) for k, v in last.items()
                           if k in ("policy_loss", "value_loss", "entropy", "approx_kl", "mean_return",
                                    "episodes", "explained_variance")},
           "explained_variance_note": "from f64 sums (the reference sums sequentially in f32, ~1e-3 off "
                                      "at 1e6 rows; INTEGRATION.md section 7)"}
    if world == 1 and not args.no_learning:
        out["steps_to_475"] = {
            "window": "100 episodes (main.rs:842-853), checked after each rollout",
            "cfgB": steps_to_475(bppo, dict(num_envs=N, num_steps=T), max_steps=40 * N * T),
            "cartpole_toml": steps_to_475(bppo, dict(num_envs=32, num_steps=128), max_steps=1_000_000)}
    else:
        out["steps_to_475"] = None
    out["cpu_baseline"] = None if args.no_cpu_baseline else cpu_baseline(args)
    print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
