set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
(cat /sys/fs/cgroup/cpu.max; nproc; python3 -c "import os; print(len(os.sched_getaffinity(0)))"; lscpu | grep -E "Thread|Core|Socket|Model name|MHz") > gpurun_out/cpuinfo_box.txt 2>&1
for i in 1 2; do
timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-learning > gpurun_out/bench_cpu_$i.log 2>&1 || exit $?
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['host_cpu_ms_per_step'], d['config']['host_cpu_quota'], d['phase_ms_per_update'])" gpurun_out/bench_cpu_$i.log
done
