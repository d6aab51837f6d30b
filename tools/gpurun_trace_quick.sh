# GPU: rocprofv3 kernel trace of a short bench; prints per-kernel average (steady iterations).
set -u
mkdir -p gpurun_out/tq
export TMPDIR=/tmp
REPO=$(pwd)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/gpurun_out/tq -o tq -- \
  python3 $REPO/bench.py --no-cpu-baseline --steps 6 --warmup 2 "$@" > $REPO/gpurun_out/tq/bench.json 2> $REPO/gpurun_out/tq/err.log || exit $?
cd $REPO
python3 - <<'PY'
import csv, glob, collections
rows = []
for f in glob.glob("gpurun_out/tq/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = collections.defaultdict(list)
for r in rows:
    d[r["Kernel_Name"][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    v2 = sorted(v)
    print(f"{len(v):4d} x  median {v2[len(v2)//2]:9.1f} us  total {sum(v):10.1f}  {k}")
PY
