set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_shuffle.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_frontier.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_frontier.log; [ $rc -eq 0 ] || exit $rc
STEPS=20 bash scripts/bench_ab.sh ab_cpu 3 BPPO_FY_LATE_INLINE=0 BPPO_FY_LATE_INLINE=1
