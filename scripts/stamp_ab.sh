# A/B of the split minibatch kernel's per-wave cycles (s_memtime segment stamps) across
# diagnostic builds: bash scripts/stamp_ab.sh TAG lib1.so lib2.so ... (each run once, in order)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1; i=0
shift; for L in "$@"; do
  timeout -k 10 300 env BPPO_LIB_PATH=$GRAFT_REPO_ROOT/$L python bench.py --steps 6 --warmup 1 --no-learning --no-cpu-baseline --no-gae-isolated > gpurun_out/${TAG}_st_$i.log 2>&1
  rc=$?; echo "$L rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep mbstamp gpurun_out/${TAG}_st_$i.log | tail -1
  i=$((i+1))
done
