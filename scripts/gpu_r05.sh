# round-5 GPU steps; every GPU step under its own time limit, stop at the first failure.
#   bash scripts/gpu_r05.sh probe TAG   HIP last-error probe + the split-kernel parity tests
#   bash scripts/gpu_r05.sh tests TAG   smoke + the whole GPU suite
#   bash scripts/gpu_r05.sh t2 TAG      2-CPU shuffle_windows bench variants (the r04u failure)
#   bash scripts/gpu_r05.sh wide TAG    CfgC / CfgD (and CNN) bench_wide lines (WIDE_VARIANTS="name|args|envs;...")
#   bash scripts/gpu_r05.sh ab TAG      interleaved CfgB bench A/B (AB_VARIANTS="name|envs;...", AB_REPS)
#   bash scripts/gpu_r05.sh kt TAG      rocprofv3 kernel trace of the CfgB bench line; widekt: of CfgC / CfgD
#   bash scripts/gpu_r05.sh mbstamp TAG split minibatch kernel segment stamps (libbppo_stamps.so);
#                                       rostamp: the 64-lane rollout's (RO_LIBS); cnn, cnnprobe: CNN parity;
#                                       mfmaprobe, fpprobe: the MFMA / f32 rounding probes
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
PART=${1:-tests}
TAG=${2:-r05}
summ() {
  python3 - "$1" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ph, rf = d["phase_ms_per_update"], d["roofline"]
print(f"  {d['ms_per_step']} ms/step {d['value']/1e6:.1f} M/s cpu {d['host_cpu_ms_per_step']} "
      f"walk {ph['shuffle_walk']} wait {ph['shuffle_wait']} mb {rf['launch_ms']} frac {rf['frac']} threads {d['config']['host_cpus_per_rank']}")
PY
}
if [ "$PART" = probe ]; then
  timeout -k 10 60 ./scripts/probes/last_error_probe > gpurun_out/${TAG}_last_error_probe.txt 2>&1
  rc=$?; echo "probe rc=$rc"; cat gpurun_out/${TAG}_last_error_probe.txt; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 600 python -u -m pytest ${PROBE_TESTS:-tests/test_gpu_split_kernel.py} -m gpu -v --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest_split.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error|assert" gpurun_out/${TAG}_pytest_split.log | tail -20
  exit $rc
fi
if [ "$PART" = tests ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|agreement" gpurun_out/${TAG}_pytest_gpu.log | tail -12
  exit $rc
fi
if [ "$PART" = t2 ]; then
  # name|env|flags
  # variants separated by ';' (fields inside a variant by '|')
  IFS=';' read -ra VS <<< "${T2_VARIANTS:-t2|BPPO_HOST_THREADS=2|--shuffle-windows on;t2gw|BPPO_HOST_THREADS=2 BPPO_SHUFFLE_GPU_WORDS=1|--shuffle-windows on;t2np|BPPO_HOST_THREADS=2 BPPO_SHUFFLE_PAIR=0|--shuffle-windows on;t2wp|BPPO_HOST_THREADS=2 BPPO_SHUFFLE_WIN_PRODUCERS=1|--shuffle-windows on}"
  for v in "${VS[@]}"; do
    IFS='|' read -r name envs flags <<< "$v"
    timeout -k 10 300 env $envs python bench.py --no-learning --no-cpu-baseline $flags > gpurun_out/${TAG}_${name}.log 2>&1
    rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/${TAG}_${name}.log; exit $rc; }
    summ gpurun_out/${TAG}_${name}.log
  done
  exit 0
fi
if [ "$PART" = wide ]; then
  # multi-player workloads on the current tree (name|bench_wide args)
  IFS=';' read -ra VS <<< "${WIDE_VARIANTS:-cfgC|--workload cfgC;cfgD|--workload cfgD;cnn64|--workload cfgC_cnn64;cnn64f32|--workload cfgC_cnn64 --minibatch-kernel 2}"
  for v in "${VS[@]}"; do
    IFS='|' read -r name args envs <<< "$v"
    timeout -k 10 400 env ${envs:-BPPO_NOP=0} python scripts/bench_wide.py $args > gpurun_out/${TAG}_wide_${name}.log 2>&1
    rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/${TAG}_wide_${name}.log; exit $rc; }
    tail -1 gpurun_out/${TAG}_wide_${name}.log | cut -c1-400
  done
  exit 0
fi
if [ "$PART" = cnn ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_cnn.py ${CNN_TESTS:-} -m gpu -v --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest_cnn.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error|assert" gpurun_out/${TAG}_pytest_cnn.log | tail -20
  exit $rc
fi
if [ "$PART" = cnnprobe ]; then
  timeout -k 10 600 python -u scripts/probes/${CNN_PROBE:-cnn_exact_probe}.py > gpurun_out/${TAG}_cnn_exact_probe.log 2>&1
  rc=$?; echo "cnn probe rc=$rc"; cat gpurun_out/${TAG}_cnn_exact_probe.log | grep -v amdgpu.ids | cut -c1-600
  exit $rc
fi
if [ "$PART" = ab ]; then
  # interleaved A/B of env variants on the default bench line: AB_VARIANTS="name|VAR=x ..." (repeated AB_REPS times)
  for rep in $(seq 1 ${AB_REPS:-2}); do
    IFS=';' read -ra VS <<< "${AB_VARIANTS:-def|BPPO_MB_EVENTS=1;ev0|BPPO_MB_EVENTS=0}"
    for v in "${VS[@]}"; do
      IFS='|' read -r name envs <<< "$v"
      timeout -k 10 300 env $envs python bench.py --no-learning --no-cpu-baseline ${AB_FLAGS:-} > gpurun_out/${TAG}_ab_${name}_${rep}.log 2>&1
      rc=$?; echo "$name/$rep rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/${TAG}_ab_${name}_${rep}.log; exit $rc; }
      summ gpurun_out/${TAG}_ab_${name}_${rep}.log
    done
  done
  exit 0
fi
if [ "$PART" = widekt ]; then
  # kernel trace of the multi-player workloads (rocprofv3 --kernel-trace --stats)
  for w in ${WIDE_KT:-cfgC cfgD}; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_${TAG}_$w -o kt -- python3 scripts/bench_wide.py --workload $w --steps 2 --warmup 1 > gpurun_out/kt_${TAG}_$w.log 2>&1
    rc=$?; echo "kt $w rc=$rc"; [ $rc -eq 0 ] || exit $rc
    DB=$(find gpurun_out/kt_${TAG}_$w -name "*.db" | head -1)
    python3 scripts/rocpd_summary.py $DB > gpurun_out/${TAG}_${w}_kernels.txt
    head -22 gpurun_out/${TAG}_${w}_kernels.txt | cut -c1-140
  done
  exit 0
fi
if [ "$PART" = kt ]; then
  # kernel trace of the default CfgB bench line (rocprofv3 --kernel-trace --stats)
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_${TAG}_cfgB -o kt -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-learning > gpurun_out/kt_${TAG}_cfgB.log 2>&1
  rc=$?; echo "kt cfgB rc=$rc"; [ $rc -eq 0 ] || exit $rc
  DB=$(find gpurun_out/kt_${TAG}_cfgB -name "*.db" | head -1)
  python3 scripts/rocpd_summary.py $DB > gpurun_out/${TAG}_cfgB_kernels.txt
  head -24 gpurun_out/${TAG}_cfgB_kernels.txt | cut -c1-140
  exit 0
fi
if [ "$PART" = mfmaprobe ]; then
  timeout -k 10 60 ./scripts/probes/mfma_round_probe > gpurun_out/${TAG}_mfma_round_probe.txt 2>&1
  rc=$?; echo "mfma probe rc=$rc"; cat gpurun_out/${TAG}_mfma_round_probe.txt
  exit $rc
fi
if [ "$PART" = fpprobe ]; then
  timeout -k 10 120 ./scripts/probes/fp_rounding_probe > gpurun_out/${TAG}_fp_rounding_probe.txt 2>&1
  rc=$?; echo "fp probe rc=$rc"; cat gpurun_out/${TAG}_fp_rounding_probe.txt
  exit $rc
fi
if [ "$PART" = rostamp ]; then
  # CfgB rollout segment stamps (diagnostic build burn-ppo_amd/bppo/libbppo_rostamps.so)
  for L in ${RO_LIBS:-rostamps}; do
    timeout -k 10 300 env BPPO_LIB_PATH=$GRAFT_REPO_ROOT/burn-ppo_amd/bppo/libbppo_$L.so python bench.py --steps 8 --warmup 0 --no-learning --no-cpu-baseline --no-gae-isolated > gpurun_out/${TAG}_$L.log 2>&1
    rc=$?; echo "$L rc=$rc"; grep rostamp gpurun_out/${TAG}_$L.log | tail -1; [ $rc -eq 0 ] || exit $rc
  done
  exit 0
fi
if [ "$PART" = mbstamp ]; then
  # split minibatch kernel segment stamps (diagnostic build burn-ppo_amd/bppo/libbppo_stamps.so)
  timeout -k 10 300 env BPPO_LIB_PATH=$GRAFT_REPO_ROOT/burn-ppo_amd/bppo/libbppo_stamps.so python bench.py --steps 6 --warmup 1 --no-learning --no-cpu-baseline --no-gae-isolated > gpurun_out/${TAG}_mbstamps.log 2>&1
  rc=$?; echo "mbstamp rc=$rc"; grep mbstamp gpurun_out/${TAG}_mbstamps.log | tail -2; exit $rc
fi
echo "unknown part $PART"; exit 2
