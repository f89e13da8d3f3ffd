# default bench.py run repeated on one box (the driver's command shape): the spread of
# the headline number.  usage: scripts/bench_repeats.sh TAG N
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1; N=${2:-4}
for i in $(seq 1 $N); do
  timeout -k 10 300 python bench.py > gpurun_out/${TAG}_$i.log 2>&1 || exit 3
  python3 - gpurun_out/${TAG}_$i.log $i <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ph = d["phase_ms_per_update"]; r = d["roofline"]
print(sys.argv[2], f"{d['value']/1e6:.1f} M env-steps/s  {d['ms_per_step']} ms/update  minibatch {r['launch_ms']} ms ({r['frac']})  "
      f"wait {ph['shuffle_wait']} walk {ph['shuffle_walk']} cpu {d['host_cpu_ms_per_step']} ms/update  steps {d['steps']}")
PY
done
