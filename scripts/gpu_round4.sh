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
if [ "$PART" = win ]; then
  # shuffle_windows parity + the 2-CPU bench (an 8-rank node's per-rank share) with and
  # without the windows, then the default bench and one PMC pass (LDS bank conflicts)
  timeout -k 10 900 python -u -m pytest ${WIN_TESTS:-tests/test_shuffle.py tests/test_gpu_multirank.py} -m gpu -q -k "${WIN_K:-windows}" --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest_win.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/${TAG}_pytest_win.log | tail -12; [ $rc -eq 0 ] || exit $rc
  for v in "2 on" "2 off" "0 auto"; do
    set -- $v
    if [ $1 = 0 ]; then unset BPPO_HOST_THREADS; else export BPPO_HOST_THREADS=$1; fi
    timeout -k 10 400 python bench.py --no-learning --no-cpu-baseline --shuffle-windows $2 > gpurun_out/${TAG}_bench_t$1_$2.log 2>&1
    rc=$?; echo "bench threads=$1 windows=$2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python3 - gpurun_out/${TAG}_bench_t$1_$2.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ph, rf = d["phase_ms_per_update"], d["roofline"]
print(f"  {d['ms_per_step']} ms/step {d['value']/1e6:.1f} M/s cpu {d['host_cpu_ms_per_step']} "
      f"walk {ph['shuffle_walk']} wait {ph['shuffle_wait']} mb {rf['launch_ms']} frac {rf['frac']} threads {d['config']['host_cpus_per_rank']}")
PY
  done
  unset BPPO_HOST_THREADS
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "k_minibatch_split" --output-format csv -d gpurun_out/pmc_${TAG}_lds -o p -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-learning > gpurun_out/pmc_${TAG}_lds.log 2>&1
  rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 scripts/pmc_json.py ${TAG}_lds gpurun_out/pmc_${TAG}_lds > gpurun_out/${TAG}_lds_pmc.txt; cat gpurun_out/${TAG}_lds_pmc.txt | head -40
  exit 0
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
