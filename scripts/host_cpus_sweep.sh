# 1-GPU CfgB bench at K host CPUs per rank (bench.py --host-cpus K: the process is
# pinned to the K idlest CPUs of the box, the shuffle engine sized for K) -- the share
# each rank of an 8-GPU node gets when the node's CPU budget is split 8 ways.
#   usage: scripts/host_cpus_sweep.sh TAG [K ...]
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r03}; shift || true
KS=${@:-16 8 4 2}
for k in $KS; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --host-cpus $k --no-learning --no-cpu-baseline > gpurun_out/hostcpus_${TAG}_k$k.log 2>&1
  rc=$?; echo "K=$k rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 - gpurun_out/hostcpus_${TAG}_k$k.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ph = d["phase_ms_per_update"]
print(f"  {d['ms_per_step']} ms/step  {d['value']/1e6:.1f} M/s  cpu {d['host_cpu_ms_per_step']} ms/step "
      f"{d['host_cpu_ms_per_step_by_thread']}  walk {ph['shuffle_walk']} wait {ph['shuffle_wait']} "
      f"spec {ph['shuffle_spec_mwords']}M true {ph['shuffle_true_mwords']}M met {ph['shuffle_met']} "
      f"pinned-busy-before {d['config'].get('host_cpus_pinned_busy_before')}")
PY
done
