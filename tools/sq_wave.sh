#!/bin/bash
# SQ counter passes on the search kernel k_nn_wave<true> (steady-state launches), 10M, 3 timed
# steps + 2 warmup. One rocprofv3 run per counter set (gpurun's rule: <= 8 SQ counters a pass).
# usage (gpurun, repo root): bash tools/sq_wave.sh TAG [bench.py args, e.g. --config KEY=VALUE]
set -u
TAG=${1:-sq}
shift || true
EXTRA="$*"
REPO=$(pwd); OUT=$REPO/gpurun_out/sq_$TAG; rm -rf $OUT; mkdir -p $OUT; export TMPDIR=/tmp
cd /tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_FMA_F64" \
           "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o p -- \
    python3 $REPO/bench.py --points 10000000 --steps 3 --warmup 2 --no-cpu-baseline --no-parity $EXTRA > /dev/null 2> $OUT/p$i.err || { echo "pass $i rc=$?"; exit 1; }
done
cd $REPO
python3 tools/sq_summary.py $OUT "k_nn_wave<true" | tee $OUT/summary.txt
