# round-3 GPU run: smoke, the GPU suite (PYTEST_K: optional -k expression,
# PYTEST_SEL: optional test paths), then a default bench line.  Every GPU step has
# its own time limit; stop at the first failure of a GPU step (a failing test
# still lets the bench run).
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r03}
SEL=${PYTEST_SEL:-tests}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke_$TAG.log; [ $rc -eq 0 ] || exit $rc
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 1000 python -u -m pytest $SEL -m gpu -v -s --timeout 300 --timeout-method thread -rf -k "$PYTEST_K" > gpurun_out/pytest_$TAG.log 2>&1
else
  timeout -k 10 1000 python -u -m pytest $SEL -m gpu -v -s --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_$TAG.log 2>&1
fi
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR|agreement|first differing|worst metric" gpurun_out/pytest_$TAG.log | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ "${NO_BENCH:-0}" = "1" ]; then exit $rc; fi
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.log 2>&1
rc2=$?; echo "bench rc=$rc2"; tail -2 gpurun_out/bench_$TAG.log
exit $rc2
