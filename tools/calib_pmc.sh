#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration for the search kernel's access widths (tools/fetch_calib.hip).
# Build here first:  hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
# usage (gpurun, repo root): bash tools/calib_pmc.sh TAG
set -u
TAG=${1:-calib}
REPO=$(pwd)
OUT=$REPO/gpurun_out/calib_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BIN=$REPO/tools/fetch_calib
cd /tmp
timeout -k 10 120 "$BIN" 3 > "$OUT/plain.jsonl" 2> "$OUT/plain.err" || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o calib -- "$BIN" 3 \
  > /dev/null 2> "$OUT/trace.err" || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o calib -- "$BIN" 3 \
  > /dev/null 2> "$OUT/pmc_fetch.err" || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o calib -- "$BIN" 3 \
  > /dev/null 2> "$OUT/pmc_write.err" || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d "$OUT/pmc_rdreq" -o calib -- "$BIN" 3 \
  > /dev/null 2> "$OUT/pmc_rdreq.err" || true
cd "$REPO"
python3 tools/calib_summary.py "$OUT" > "$OUT/calibration.json"
cat "$OUT/calibration.json"
