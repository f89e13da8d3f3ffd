# A/B of the 16-row minibatch kernel (BPPO_MB16=1) against the 32-row one:
# MFMA 16x16x4 probe, GPU parity suite under MB16, kernel trace of both, benches.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-mb16}
timeout -k 10 60 ./scripts/probes/mfma16_probe.bin > gpurun_out/${TAG}_probe.txt 2>&1; echo "probe rc=$?"; cat gpurun_out/${TAG}_probe.txt
BPPO_MB16=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_scale.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/${TAG}_pytest.log; [ $rc -le 1 ] || exit $rc
for v in 0 1 0 1; do
  BPPO_MB16=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-learning > gpurun_out/${TAG}_bench_$v.log 2>&1 || exit 3
  python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/${TAG}_bench_$v.log') if l.startswith('{')][-1])
print('MB16=$v', d['ms_per_step'], 'mb launch', d['roofline']['launch_ms'], 'frac', d['roofline']['frac'], 'wait', d['phase_ms_per_update']['shuffle_wait'])"
done
BPPO_MB16=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$TAG -o kt -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-learning > gpurun_out/kt_$TAG.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py $(find gpurun_out/kt_$TAG -name "*.db" | head -1) > gpurun_out/kt_$TAG.txt
head -12 gpurun_out/kt_$TAG.txt
