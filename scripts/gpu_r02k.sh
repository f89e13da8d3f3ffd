# r02k: parity after the heads split; isolated k_expand_J timing; bench kernel trace
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r02k}
timeout -k 10 600 python -u -m pytest tests/test_shuffle.py tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_golden.py tests/test_gpu_wide.py -m gpu -q -x --timeout 240 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ktx_$TAG -o kt -- python3 -m pytest tests/test_shuffle.py -m gpu -q -k "engine_equals" > gpurun_out/ktx_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/ktx_$TAG.log; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py $(find gpurun_out/ktx_$TAG -name "*.db" | head -1) > gpurun_out/ktx_$TAG.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kt_$TAG -o kt -- python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline --no-learning > gpurun_out/kt_$TAG.log 2>&1
rc=$?; tail -1 gpurun_out/kt_$TAG.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
python3 scripts/rocpd_summary.py $(find gpurun_out/kt_$TAG -name "*.db" | head -1) > gpurun_out/kt_$TAG.txt
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-learning > gpurun_out/bench_$TAG.log 2>&1
rc=$?; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['frac'], d['phase_ms_per_update'])" gpurun_out/bench_$TAG.log
exit $rc
