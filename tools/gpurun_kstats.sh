# GPU: per-kernel average durations (rocprofv3 kernel trace) of the default bench for env configs.
# usage: bash tools/gpurun_kstats.sh "CFG1" "CFG2" ...   (CFG = ':'-joined VAR=VALUE list)
set -u
REPO=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
n=0
for c in "$@"; do
  n=$((n + 1))
  OUT=$REPO/gpurun_out/kst_$n
  (cd /tmp && env $(echo $c | tr ':' ' ') timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o k -- \
    python3 $REPO/bench.py --no-cpu-baseline --steps 10 --warmup 3 > "$OUT.json" 2> "$OUT.err") || { tail -20 "$OUT.err"; exit 1; }
  echo "[$c]"
  python3 - "$OUT" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if int(r["Calls"]) >= 10:
            print(f'{float(r["AverageNs"])/1e3:10.1f} us x{r["Calls"]:>4}  {r["Name"][:80]}')
PY
done
