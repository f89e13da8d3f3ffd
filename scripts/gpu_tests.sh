# GPU parity tests (one pytest process, per-test timeout), then a short bench.
# usage: scripts/gpu_tests.sh TAG [pytest selection...]
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-r02}; shift || true
SEL=${@:-tests}
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -v --timeout 240 --timeout-method thread -rf > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|PASSED|FAILED|ERROR" gpurun_out/pytest_$TAG.log | tail -60
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_$TAG.log 2>&1
rc2=$?; echo "bench rc=$rc2"; tail -3 gpurun_out/bench_$TAG.log
exit $rc2
