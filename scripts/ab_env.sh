# interleaved A/B of two environment settings on one box: bench.py under env A / env B,
# ROUNDS times each, alternating.  usage: scripts/ab_env.sh TAG ROUNDS "VAR=x ..." "VAR=y ..."
# ("-" for an empty setting)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1; ROUNDS=$2; EA=$3; EB=$4
[ "$EA" = "-" ] && EA=""
[ "$EB" = "-" ] && EB=""
for i in $(seq 1 $ROUNDS); do
  for v in A B; do
    e=$EA; [ $v = B ] && e=$EB
    env $e timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-learning --no-cpu-baseline > gpurun_out/${TAG}_${v}_$i.log 2>&1 || exit 3
    python3 - gpurun_out/${TAG}_${v}_$i.log $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ph = d["phase_ms_per_update"]; r = d["roofline"]
print(f"{sys.argv[2]} {d['ms_per_step']:7.3f} ms/step  mb {r['launch_ms']:.4f}  rollout {ph['rollout']:.3f} "
      f"wait {ph['shuffle_wait']:.2f} walk {ph['shuffle_walk']:.2f} cpu {d['host_cpu_ms_per_step']} {d['host_cpu_ms_per_step_by_thread']}")
PY
  done
done
