# repeated short benches (no profiler): ms/step and phases per run
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-rep}; N=${2:-3}
for i in $(seq 1 $N); do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-learning > gpurun_out/${TAG}_$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; exit $rc; }
  python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(d['ms_per_step'], d['roofline']['frac'], d['phase_ms_per_update'])" gpurun_out/${TAG}_$i.log
done
