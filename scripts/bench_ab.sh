# interleaved A/B of env settings on one box: ms/step and shuffle phases per run
#   bash scripts/bench_ab.sh TAG ROUNDS VAR=VAL VAR=VAL ...
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1; R=$2; shift 2
for i in $(seq 1 $R); do
  for v in "$@"; do
    env $v timeout -k 10 300 python3 bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-learning > gpurun_out/${TAG}.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; exit $rc; }
    python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; p=d['phase_ms_per_update']; print(sys.argv[2], d['ms_per_step'], 'walk', p['shuffle_walk'], 'wait', p['shuffle_wait'], 'update', p['update'], 'cpu', d.get('host_cpu_ms_per_step'), 'spec', p.get('shuffle_spec_mwords'), 'true', p.get('shuffle_true_mwords'), 'tsc walk/words', p.get('shuffle_walk_tsc_ms'), p.get('shuffle_words_tsc_ms'), 'met', p['shuffle_met'], 'host enq/sync', p.get('host_enqueue'), p.get('host_sync_wait'), d.get('host_cpu_ms_per_step_by_thread'))" gpurun_out/${TAG}.log "$v"
  done
done
