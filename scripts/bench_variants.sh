# one bench.py line per variant (A/B on one box): each argument is
#   "NAME|VAR=x VAR2=y|bench flags"
# e.g. bash scripts/bench_variants.sh TAG "t2on|BPPO_HOST_THREADS=2|--shuffle-windows on"
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=$1; shift
for v in "$@"; do
  IFS='|' read -r name envs flags <<< "$v"
  log=gpurun_out/${TAG}_${name}.log
  timeout -k 10 300 env $envs python bench.py --no-learning --no-cpu-baseline $flags > $log 2>&1
  rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 - $log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ph, rf = d["phase_ms_per_update"], d["roofline"]
print(f"  {d['ms_per_step']} ms/step {d['value']/1e6:.1f} M/s cpu {d['host_cpu_ms_per_step']} {d['host_cpu_ms_per_step_by_thread']} "
      f"walk {ph['shuffle_walk']} wait {ph['shuffle_wait']} walk_tsc {ph['shuffle_walk_tsc_ms']} words_tsc {ph['shuffle_words_tsc_ms']} "
      f"rollout {ph['rollout']} update {ph['update']} mb {rf['launch_ms']}")
PY
  grep "^thread" $log | sort -k6 -n -r | head -8 || true
done
