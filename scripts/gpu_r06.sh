# round-6 GPU steps; every GPU step under its own time limit, stop at the first failure.
#   bash scripts/gpu_r06.sh tests TAG     pytest -m gpu of $TESTS (default: the whole GPU suite) + smoke
#   bash scripts/gpu_r06.sh wide TAG      CfgC / CfgD bench_wide lines (WIDE_VARIANTS="name|args|envs;...")
#   bash scripts/gpu_r06.sh widekt TAG    rocprofv3 kernel traces of CfgC / CfgD (WIDE_KT)
#   bash scripts/gpu_r06.sh bench TAG     default CfgB bench line(s) (BENCH_REPS, BENCH_FLAGS, BENCH_ENV)
#   bash scripts/gpu_r06.sh kt TAG        rocprofv3 kernel trace of the CfgB bench line
#   bash scripts/gpu_r06.sh pmc TAG       PMC passes on the CfgB bench (scripts/pmc_traffic.sh)
#   bash scripts/gpu_r06.sh ab TAG        interleaved bench lines under env variants (AB_VARIANTS, AB_REPS)
#   bash scripts/gpu_r06.sh mbstamp TAG   split minibatch kernel segment stamps (libbppo_stamps.so)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
PART=${1:-tests}
TAG=${2:-r06}
summ() {
  python3 - "$1" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ph, rf = d["phase_ms_per_update"], d["roofline"]
print(f"  {d['ms_per_step']} ms/step {d['value']/1e6:.1f} M/s cpu {d['host_cpu_ms_per_step']} "
      f"walk {ph['shuffle_walk']} wait {ph['shuffle_wait']} mb {rf['launch_ms']} frac {rf['frac']} "
      f"exact {rf.get('exact_first_minibatch', {}).get('launch_ms')} threads {d['config']['host_cpus_per_rank']}")
PY
}
case "$PART" in
tests)
  if [ -z "${TESTS:-}" ]; then
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
    rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
  fi
  timeout -k 10 ${TEST_TIMEOUT:-1000} python -u -m pytest ${TESTS:-tests} -m gpu -v -s --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|worst|differing" gpurun_out/${TAG}_pytest_gpu.log | tail -30
  exit $rc ;;
wide)
  IFS=';' read -ra VS <<< "${WIDE_VARIANTS:-cfgC|--workload cfgC;cfgD|--workload cfgD}"
  for v in "${VS[@]}"; do
    IFS='|' read -r name args envs <<< "$v"
    timeout -k 10 400 env ${envs:-BPPO_NOP=0} python scripts/bench_wide.py $args > gpurun_out/${TAG}_wide_${name}.log 2>&1
    rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/${TAG}_wide_${name}.log; exit $rc; }
    tail -1 gpurun_out/${TAG}_wide_${name}.log | cut -c1-500
  done ;;
widekt)
  for w in ${WIDE_KT:-cfgC cfgD}; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_${TAG}_$w -o kt -- python3 scripts/bench_wide.py --workload $w --steps 2 --warmup 1 > gpurun_out/kt_${TAG}_$w.log 2>&1
    rc=$?; echo "kt $w rc=$rc"; [ $rc -eq 0 ] || exit $rc
    DB=$(find gpurun_out/kt_${TAG}_$w -name "*.db" | head -1)
    python3 scripts/rocpd_summary.py $DB > gpurun_out/${TAG}_${w}_kernels.txt
    head -22 gpurun_out/${TAG}_${w}_kernels.txt | cut -c1-140
  done ;;
bench)
  for rep in $(seq 1 ${BENCH_REPS:-1}); do
    timeout -k 10 300 env ${BENCH_ENV:-BPPO_NOP=0} python bench.py ${BENCH_FLAGS:-} > gpurun_out/${TAG}_bench_$rep.log 2>&1
    rc=$?; echo "bench/$rep rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/${TAG}_bench_$rep.log; exit $rc; }
    summ gpurun_out/${TAG}_bench_$rep.log
  done ;;
ab)
  # interleaved A/B of bench lines: AB_VARIANTS="name|ENV=1 ENV2=x;name2|...", AB_REPS rounds
  IFS=';' read -ra VS <<< "${AB_VARIANTS:-base|BPPO_NOP=0}"
  for rep in $(seq 1 ${AB_REPS:-2}); do
    for v in "${VS[@]}"; do
      IFS='|' read -r name envs <<< "$v"
      timeout -k 10 300 env ${envs:-BPPO_NOP=0} python bench.py ${BENCH_FLAGS:---no-cpu-baseline --no-learning} > gpurun_out/${TAG}_ab_${name}_$rep.log 2>&1
      rc=$?; echo "$name/$rep rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/${TAG}_ab_${name}_$rep.log; exit $rc; }
      summ gpurun_out/${TAG}_ab_${name}_$rep.log
    done
  done ;;
kt)
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_${TAG}_cfgB -o kt -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-learning > gpurun_out/kt_${TAG}_cfgB.log 2>&1
  rc=$?; echo "kt cfgB rc=$rc"; [ $rc -eq 0 ] || exit $rc
  DB=$(find gpurun_out/kt_${TAG}_cfgB -name "*.db" | head -1)
  python3 scripts/rocpd_summary.py $DB > gpurun_out/${TAG}_cfgB_kernels.txt
  head -24 gpurun_out/${TAG}_cfgB_kernels.txt | cut -c1-140 ;;
pmc)
  bash scripts/pmc_traffic.sh $TAG ;;
mbstamp)
  # split minibatch kernel segment stamps (diagnostic build burn-ppo_amd/bppo/libbppo_stamps.so)
  timeout -k 10 300 env BPPO_LIB_PATH=$GRAFT_REPO_ROOT/burn-ppo_amd/bppo/libbppo_stamps.so python bench.py --steps 6 --warmup 1 --no-learning --no-cpu-baseline --no-gae-isolated > gpurun_out/${TAG}_mbstamps.log 2>&1
  rc=$?; echo "mbstamp rc=$rc"; grep mbstamp gpurun_out/${TAG}_mbstamps.log | tail -2; exit $rc ;;
*) echo "unknown part $PART"; exit 2 ;;
esac
