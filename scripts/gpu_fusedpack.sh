# packed update rows written by the rollout + GAE: GPU suite, then A/B against k_pack_rows
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread > gpurun_out/pytest_fusedpack.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_fusedpack.log; [ $rc -eq 0 ] || exit $rc
STEPS=20 bash scripts/bench_ab.sh ab_fp 3 BPPO_NO_FUSED_PACK= BPPO_NO_FUSED_PACK=1
