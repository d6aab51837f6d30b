#!/bin/bash
# Per-iterate trace of the bench workload (tools/iter_trace.py) plus per-dispatch PMC passes of
# the same iterates. Run through gpurun from the repo root:
#   bash tools/iter_trace.sh TAG [ITERS] [N]
# Output: gpurun_out/itr_TAG/{times,corr,dbg}.jsonl and pmc_*/ (rocprofv3 counter_collection.csv)
set -u
TAG=${1:-itr}
ITERS=${2:-50}
N=${3:-10000000}
REPO=$(pwd)
OUT=$REPO/gpurun_out/itr_$TAG
mkdir -p "$OUT"
timeout -k 10 300 python3 -u tools/iter_trace.py $N $ITERS --no-corr > "$OUT/times.jsonl" 2> "$OUT/times.err" || { tail -20 "$OUT/times.err"; exit 1; }
timeout -k 10 300 python3 -u tools/iter_trace.py $N $ITERS --dbg > "$OUT/corr_dbg.jsonl" 2> "$OUT/corr_dbg.err" || { tail -20 "$OUT/corr_dbg.err"; exit 1; }
export TMPDIR=/tmp
cd /tmp
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/pmc_$name" -o pmc -- \
    python3 $REPO/tools/iter_trace.py $N $ITERS --no-corr > "$OUT/pmc_$name.jsonl" 2> "$OUT/pmc_$name.err" || { tail -20 "$OUT/pmc_$name.err"; exit 1; }
}
pass l2 TCC_HIT_sum TCC_MISS_sum || exit 1
pass fetch FETCH_SIZE || exit 1
pass write WRITE_SIZE || exit 1
pass sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD || exit 1
cd "$REPO"
python3 tools/iter_trace_summary.py "$OUT" > "$OUT/summary.txt" 2>&1
cat "$OUT/summary.txt"
