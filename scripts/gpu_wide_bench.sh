# multi-player workloads: throughput lines + a kernel-trace profile of one CfgC and one CfgD update
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:-r01}
timeout -k 10 300 python scripts/bench_wide.py --workload cfgC --steps 3 --warmup 1 > gpurun_out/wide_cfgC_$TAG.log 2>&1
rc=$?; echo "cfgC rc=$rc"; tail -3 gpurun_out/wide_cfgC_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_wide.py --workload cfgD --steps 3 --warmup 1 > gpurun_out/wide_cfgD_$TAG.log 2>&1
rc=$?; echo "cfgD rc=$rc"; tail -3 gpurun_out/wide_cfgD_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfgC_$TAG -o kt -- python3 scripts/bench_wide.py --workload cfgC --steps 1 --warmup 0 > gpurun_out/prof_cfgC_$TAG.log 2>&1
rc=$?; echo "profC rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfgD_$TAG -o kt -- python3 scripts/bench_wide.py --workload cfgD --steps 1 --warmup 0 > gpurun_out/prof_cfgD_$TAG.log 2>&1
rc=$?; echo "profD rc=$rc"
exit $rc
