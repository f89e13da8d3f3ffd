# SQ counter passes of the minibatch kernels under BPPO_MB16=0/1 (one rocprofv3 pass per set)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-mb16p}
SETS=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
      "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_COEXEC_CYCLES")
for v in 1 0; do
i=0
for s in "${SETS[@]}"; do
  BPPO_MB16=$v timeout -s KILL 120 rocprofv3 --pmc $s --kernel-include-regex "k_minibatch" -d gpurun_out/pmc_${TAG}_${v}_$i -o p -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-learning > gpurun_out/pmc_${TAG}_${v}_$i.log 2>&1
  rc=$?; echo "mb16=$v pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
done
python3 - <<'PY'
import glob, csv, collections, os
for f in sorted(glob.glob('gpurun_out/pmc_*/**/*counter_collection.csv', recursive=True)):
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(f)):
        acc[(row['Kernel_Name'][:40], row['Counter_Name'])].append(float(row['Counter_Value']))
    for (k, c), v in sorted(acc.items()):
        print(f.split('/')[1], k, c, f"{sum(v)/len(v):.4g}", len(v))
PY
