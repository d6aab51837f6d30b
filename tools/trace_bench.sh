#!/bin/bash
# rocprofv3 kernel trace + stats of one bench run (GPU box, repo root), summary printed.
# usage: bash tools/trace_bench.sh TAG [bench args...]
set -u
TAG=$1; shift
R=$(pwd)
OUT=$R/gpurun_out/trace_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o "$TAG" -- \
  python3 "$R/bench.py" "$@" > "$OUT/bench.json" 2> "$OUT/trace.err" || exit $?
cd "$R"
python3 tools/kstats.py "$OUT"/*kernel_stats.csv
