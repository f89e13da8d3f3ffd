# round-5 GPU steps; every GPU step under its own time limit, stop at the first failure.
#   bash scripts/gpu_r05.sh probe TAG   HIP last-error probe + the split-kernel parity tests
#   bash scripts/gpu_r05.sh tests TAG   smoke + the whole GPU suite
#   bash scripts/gpu_r05.sh t2 TAG      2-CPU shuffle_windows bench variants (the r04u failure)
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
  for v in ${T2_VARIANTS:-"t2|BPPO_HOST_THREADS=2|--shuffle-windows on" "t2gw|BPPO_HOST_THREADS=2 BPPO_SHUFFLE_GPU_WORDS=1|--shuffle-windows on" "t2np|BPPO_HOST_THREADS=2 BPPO_SHUFFLE_PAIR=0|--shuffle-windows on" "t2wp|BPPO_HOST_THREADS=2 BPPO_SHUFFLE_WIN_PRODUCERS=1|--shuffle-windows on"}; do
    IFS='|' read -r name envs flags <<< "$v"
    timeout -k 10 300 env $envs python bench.py --no-learning --no-cpu-baseline $flags > gpurun_out/${TAG}_${name}.log 2>&1
    rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/${TAG}_${name}.log; exit $rc; }
    summ gpurun_out/${TAG}_${name}.log
  done
  exit 0
fi
echo "unknown part $PART"; exit 2
