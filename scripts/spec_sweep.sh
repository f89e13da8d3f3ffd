# shuffle-engine CPU vs wait trade-off on one box, unpinned: bench.py (20 steps) with the
# engine sized by BPPO_SHUFFLE_SPEC (walks per boundary) / BPPO_HOST_THREADS (CPU budget).
# usage: scripts/spec_sweep.sh TAG
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1
run() {   # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-learning --no-cpu-baseline \
    > gpurun_out/${TAG}_${name}.log 2>&1 || exit 3
  python3 - gpurun_out/${TAG}_${name}.log $name <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ph = d["phase_ms_per_update"]
print(f"{sys.argv[2]:10s} {d['ms_per_step']:7.3f} ms/step  wait {ph['shuffle_wait']:6.2f}  walk {ph['shuffle_walk']:6.2f}  "
      f"spec {ph['shuffle_spec_mwords']:6.1f} Mw  true {ph['shuffle_true_mwords']:5.1f} Mw  cpu {d['host_cpu_ms_per_step']:6.1f} "
      f"{d['host_cpu_ms_per_step_by_thread']}")
PY
}
run default
run spec3 BPPO_SHUFFLE_SPEC=3
run spec2 BPPO_SHUFFLE_SPEC=2
run spec1 BPPO_SHUFFLE_SPEC=1
run hc8 BPPO_HOST_THREADS=8
run hc4 BPPO_HOST_THREADS=4
run hc2 BPPO_HOST_THREADS=2
