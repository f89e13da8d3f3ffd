# Kernel-trace A/B of whole updates under env variants (scripts/kt_updates.py per run):
#   bash scripts/kt_ab.sh TAG VAR=VAL [VAR=VAL ...]     (each variant once, in order)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
i=0
for v in "$@"; do
  d=gpurun_out/ka_${TAG}_$i
  export $v
  timeout -k 10 240 rocprofv3 --kernel-trace -d $d -o kt -- python3 bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-learning --no-gae-isolated > $d.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "[$v] rc=$rc"; exit $rc; }
  python3 scripts/kt_updates.py $(find $d -name "*.db" | head -1) "[$v]"
  unset ${v%%=*}
  i=$((i+1))
done
