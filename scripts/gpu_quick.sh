# GPU suite then the default bench twice (per-thread CPU, walk/wait split)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_quick.log; [ $rc -eq 0 ] || exit $rc
STEPS=20 bash scripts/bench_ab.sh ab_quick 2 BPPO_SHUFFLE_FRONTIER=1
