# shuffle engine probe: per-epoch walk logs and step time for a few engine settings.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-probe}
shift || true
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python3 -c "import os; print(len(os.sched_getaffinity(0)))"; } > gpurun_out/${TAG}_cpu.txt
i=0
for v in "$@"; do
  env $v BPPO_SHUFFLE_DEBUG=1 timeout -k 10 180 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-learning \
      > gpurun_out/${TAG}_$i.log 2> gpurun_out/${TAG}_$i.err
  rc=$?; echo "[$v] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['phase_ms_per_update'])" gpurun_out/${TAG}_$i.log
  i=$((i+1))
done
