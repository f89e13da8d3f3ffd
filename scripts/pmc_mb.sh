# Kernel trace + SQ counters of the minibatch kernels: one rocprofv3 pass per
# counter set (<= 8 SQ counters each), a one-update bench per pass.
#   bash scripts/pmc_mb.sh TAG [extra env assignments for the bench]
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-mb}
shift || true
for kv in "$@"; do export "$kv"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_${TAG} -o kt -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/kt_${TAG}.log 2>&1
rc=$?; echo "kt rc=$rc"
[ $rc -eq 0 ] || exit $rc
SETS=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
      "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_COEXEC_CYCLES")
i=0
for s in "${SETS[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc $s --kernel-include-regex "k_minibatch" -d gpurun_out/pmc_${TAG}_$i -o p -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_${TAG}_$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
