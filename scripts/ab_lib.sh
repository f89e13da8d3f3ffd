# interleaved A/B of two builds of libbppo on one box: bench.py under BPPO_LIB_PATH=A / B,
# ROUNDS times each, alternating.  usage: scripts/ab_lib.sh TAG ROUNDS LIB_A LIB_B
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1; ROUNDS=$2; A=$3; B=$4
for i in $(seq 1 $ROUNDS); do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    BPPO_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-learning --no-cpu-baseline > gpurun_out/${TAG}_${v}_$i.log 2>&1 || exit 3
    python3 - gpurun_out/${TAG}_${v}_$i.log $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ph = d["phase_ms_per_update"]; r = d["roofline"]
print(f"{sys.argv[2]} {d['ms_per_step']:7.3f} ms/step  mb {r['launch_ms']:.4f} {r['launch_ms_min_max']}  rollout {ph['rollout']:.3f} "
      f"gae {ph['gae']:.3f} rn {ph.get('return_norm', 0):.3f} wait {ph['shuffle_wait']:.2f} cpu {d['host_cpu_ms_per_step']}")
PY
  done
done
