# round-4 GPU evidence: smoke + the whole GPU suite (part "tests"), or two CfgB bench
# lines + PMC passes + a kernel trace (part "prof").  Every GPU step under its own time
# limit; stop at the first failure.
#   bash scripts/gpu_round4.sh tests TAG | bash scripts/gpu_round4.sh prof TAG
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
PART=${1:-tests}
TAG=${2:-r04}
if [ "$PART" = tests ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|agreement" gpurun_out/${TAG}_pytest_gpu.log | tail -12
  exit $rc
fi
for i in 1 2; do
  timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench_$i.log 2>&1
  rc=$?; echo "bench $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 - gpurun_out/${TAG}_bench_$i.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ph, rf = d["phase_ms_per_update"], d["roofline"]
print(f"  {d['ms_per_step']} ms/step {d['value']/1e6:.1f} M/s cpu {d['host_cpu_ms_per_step']} "
      f"walk {ph['shuffle_walk']} wait {ph['shuffle_wait']} mb {rf['launch_ms']} frac {rf['frac']} exact {rf['exact_first_minibatch']}")
PY
done
bash scripts/pmc_traffic.sh ${TAG}
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_${TAG} -o kt -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-learning > gpurun_out/kt_${TAG}.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
DB=$(find gpurun_out/kt_${TAG} -name "*.db" | head -1)
python3 scripts/rocpd_summary.py $DB > gpurun_out/${TAG}_kernels.txt
python3 scripts/kt_timeline.py $DB > gpurun_out/${TAG}_timeline.txt
python3 scripts/kt_overlap.py $DB k_minibatch_split > gpurun_out/${TAG}_mb_overlap.txt
head -12 gpurun_out/${TAG}_kernels.txt; head -5 gpurun_out/${TAG}_timeline.txt; cat gpurun_out/${TAG}_mb_overlap.txt
