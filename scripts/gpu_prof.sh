# rocprofv3 kernel trace + stats of the default bench, then separate PMC passes
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o kt -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "kt rc=$rc"; tail -5 gpurun_out/prof_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch_$TAG -o pf -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch_$TAG.log 2>&1
rc=$?; echo "fetch rc=$rc"; tail -3 gpurun_out/pmc_fetch_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write_$TAG -o pw -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write_$TAG.log 2>&1
rc=$?; echo "write rc=$rc"; tail -3 gpurun_out/pmc_write_$TAG.log
find gpurun_out -name "*.csv" | head -30
exit $rc
