# A/B of one kernel's duration under env variants: rocprofv3 kernel trace per
# variant, median / min / mean of the matching kernel's launches.
#   bash scripts/kt_variants.sh TAG KERNEL_REGEX VAR=VAL [VAR=VAL ...]
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; RE=$2; shift 2
i=0
for v in "$@"; do
  d=gpurun_out/kv_${TAG}_$i
  export $v
  timeout -k 10 240 rocprofv3 --kernel-trace -d $d -o kt -- python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline --no-learning --no-gae-isolated > $d.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "[$v] rc=$rc"; exit $rc; }
  python3 - "$v" "$RE" $d <<'PY'
import glob, re, sqlite3, statistics, sys
v, rx, d = sys.argv[1:4]
db = sqlite3.connect(glob.glob(d + "/**/*.db", recursive=True)[0])
ds = [r[1] / 1000.0 for r in db.execute("select name, duration from kernels") if re.search(rx, r[0])]
print(f"[{v}] n={len(ds)} median={statistics.median(ds):.2f}us min={min(ds):.2f} mean={statistics.mean(ds):.2f}")
PY
  unset ${v%%=*}
  i=$((i+1))
done
