# CNN (network_type = "cnn", Connect Four): GPU parity tests (incl. split_networks),
# throughput of CfgC with the CNN at the config defaults and a 64-channel variant,
# and a kernel trace of one update of each.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:-cnn}
timeout -k 10 600 python -u -m pytest tests/test_gpu_cnn.py tests/test_gpu_split.py tests/test_gpu_checkpoint.py -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_pytest.log; [ $rc -le 1 ] || exit $rc
for w in cfgC_cnn cfgC_cnn64; do
  timeout -k 10 300 python scripts/bench_wide.py --workload $w --steps 2 --warmup 1 > gpurun_out/${TAG}_$w.log 2>&1
  rc=$?; echo "$w rc=$rc"; tail -1 gpurun_out/${TAG}_$w.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_${TAG}_$w -o kt -- python3 scripts/bench_wide.py --workload $w --steps 1 --warmup 0 > gpurun_out/kt_${TAG}_$w.log 2>&1
  rc=$?; echo "kt $w rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 scripts/rocpd_summary.py $(find gpurun_out/kt_${TAG}_$w -name "*.db" | head -1) > gpurun_out/kt_${TAG}_$w.txt
  head -16 gpurun_out/kt_${TAG}_$w.txt
done
