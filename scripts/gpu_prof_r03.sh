# kernel trace of a short CfgB bench (rocprofv3 --kernel-trace --stats) -> per-kernel
# summary and the compute-stream timeline of one update, under gpurun_out/kt_TAG*
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r03}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$TAG -o kt -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-learning > gpurun_out/kt_$TAG.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py $(find gpurun_out/kt_$TAG -name "*.db" | head -1) > gpurun_out/kt_$TAG.txt
python3 scripts/kt_timeline.py $(find gpurun_out/kt_$TAG -name "*.db" | head -1) > gpurun_out/kt_${TAG}_timeline.txt
head -25 gpurun_out/kt_$TAG.txt; head -8 gpurun_out/kt_${TAG}_timeline.txt
