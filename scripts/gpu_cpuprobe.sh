# frontier depth A/B with per-thread CPU time
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
STEPS=20 bash scripts/bench_ab.sh ab_cpu 2 BPPO_SHUFFLE_FRONTIER=1 BPPO_SHUFFLE_FRONTIER=2 "BPPO_SHUFFLE_FRONTIER=2 BPPO_SHUFFLE_SPEC=4"
