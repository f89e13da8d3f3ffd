# round-2 evidence run: smoke, GPU tests, default bench, rocprof kernel trace,
# PMC passes.  Each GPU step has its own time limit; stop at the first failure.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r02}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -rf > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_$TAG.log | tail -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$TAG -o kt -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-learning > gpurun_out/kt_$TAG.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py $(find gpurun_out/kt_$TAG -name "*.db" | head -1) > gpurun_out/kt_$TAG.txt
python3 scripts/kt_timeline.py $(find gpurun_out/kt_$TAG -name "*.db" | head -1) > gpurun_out/kt_${TAG}_timeline.txt
bash scripts/pmc_traffic.sh $TAG
