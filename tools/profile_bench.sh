#!/bin/bash
# Profile the bench command with rocprofv3 (kernel trace + stats; then separate PMC passes).
# usage (on the GPU box, from the repo root): bash tools/profile_bench.sh TAG [N]
# STEPS / WARMUP (default 20 / 5: the driver's own arguments) set the timed window of every pass.
set -u
TAG=${1:-r01}
N=${2:-10000000}
STEPS=${STEPS:-20}
WARMUP=${WARMUP:-5}
REPO=$(pwd)
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
# BENCH_EXTRA: workload arguments of bench.py (e.g. --scene); WORKLOAD: its bench.py workload_key
BENCH="$REPO/bench.py --points $N --no-cpu-baseline --no-parity --no-registration ${BENCH_EXTRA:-}"
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o "$TAG" -- \
  python3 $BENCH --steps $STEPS --warmup $WARMUP > "$OUT/bench_traced.json" 2> "$OUT/trace.err" || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o "$TAG" -- \
  python3 $BENCH --steps $STEPS --warmup $WARMUP > /dev/null 2> "$OUT/pmc_fetch.err" || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o "$TAG" -- \
  python3 $BENCH --steps $STEPS --warmup $WARMUP > /dev/null 2> "$OUT/pmc_write.err" || exit $?
timeout -k 10 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/pmc_l2" -o "$TAG" -- \
  python3 $BENCH --steps $STEPS --warmup $WARMUP > /dev/null 2> "$OUT/pmc_l2.err" || exit $?
# the VALU / SALU issue of the search kernel (the bound that binds it: SQ_INSTS_VALU x 4 cycles per
# wave64 instruction over 1024 SIMDs x the kernel's cycles)
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_sq" -o "$TAG" -- \
  python3 $BENCH --steps $STEPS --warmup $WARMUP > /dev/null 2> "$OUT/pmc_sq.err" || exit $?
cd "$REPO"
python3 tools/pmc_traffic.py "$OUT" "$N" 1 "${WORKLOAD:-blob|q=0.0|dup=1}" > "$OUT/traffic.json"
cat "$OUT/traffic.json"
