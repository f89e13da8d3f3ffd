# Kernel-trace A/B: per env variant, total device time per update of kernel groups
#   bash scripts/kt_sum.sh TAG VAR=VAL [VAR=VAL ...]
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
i=0
for v in "$@"; do
  d=gpurun_out/ks_${TAG}_$i
  export $v
  timeout -k 10 240 rocprofv3 --kernel-trace -d $d -o kt -- python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline --no-learning > $d.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "[$v] rc=$rc"; exit $rc; }
  python3 scripts/ks_summary.py $d
  unset ${v%%=*}
  i=$((i+1))
done
