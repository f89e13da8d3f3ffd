# Fisher-Yates ahead on a side stream: GPU suite, then A/B against in-update permutations
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread > gpurun_out/pytest_fyahead.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_fyahead.log; [ $rc -eq 0 ] || exit $rc
STEPS=20 bash scripts/bench_ab.sh ab_fy 2 BPPO_FY_AHEAD=1 BPPO_FY_AHEAD=0 "BPPO_FY_AHEAD=1 BPPO_ADV_STREAM=0"
