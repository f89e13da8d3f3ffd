# PMC passes over one CfgB update (bench.py --steps 1 --warmup 1): HBM bytes of
# the roofline kernels (FETCH_SIZE and WRITE_SIZE need a pass each on gfx950)
# and the MFMA / issue counters of the minibatch kernel, then the JSON summary
# (gpurun_out/pmc_<tag>.json; bench.py reads the copy at pmc_traffic.json).
#   bash scripts/pmc_traffic.sh TAG
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-traffic}
RE="k_minibatch_mfma|k_minibatch_split|k_gae_1p|k_cartpole_rollout_mfma|k_pack_rows"
timeout -s KILL 60 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
have() { grep -qw "$1" gpurun_out/rocprof_counters.txt; }
pick() { local out=""; for c in "$@"; do if have $c; then out="$out $c"; fi; done; echo $out; }
PASSES=("FETCH_SIZE" "WRITE_SIZE"
        "$(pick SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE)"
        "$(pick SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE)")
DIRS=""
i=0
for c in "${PASSES[@]}"; do
  [ -n "$c" ] || { i=$((i+1)); continue; }
  d=gpurun_out/pmc_${TAG}_$i
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "$RE" --output-format csv -d $d -o p -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-learning > $d.log 2>&1
  rc=$?; echo "pass $i ($c) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  DIRS="$DIRS $d"
  i=$((i+1))
done
python3 scripts/pmc_json.py $TAG $DIRS > gpurun_out/${TAG}_pmc.txt
cat gpurun_out/${TAG}_pmc.txt
