# HBM traffic of the roofline kernels (k_minibatch_mfma, k_gae_1p): one rocprofv3 --pmc pass
# per TCC counter (FETCH_SIZE and WRITE_SIZE do not fit one pass), one-update bench each.
#   bash scripts/pmc_traffic.sh TAG
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-traffic}
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "k_minibatch_mfma|k_gae_1p" --output-format csv -d gpurun_out/pmc_${TAG}_$c -o p -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_${TAG}_$c.log 2>&1
  rc=$?; echo "pass $c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
