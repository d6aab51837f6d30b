#!/bin/bash
# SQ/TA counter passes on the search kernel for the given variants (1 step timed, 1 warmup).
set -u
REPO=$(pwd); OUT=$REPO/gpurun_out/sq; mkdir -p $OUT; export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
cd /tmp
for v in ${1:-"4"}; do
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_THREAD_CYCLES_VALU" \
             "TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
             "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_CVT"; do
    i=$((i+1))
    ICP_NN_VARIANT=$v timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/v${v}_p$i -o p -- \
      python3 $REPO/bench.py --points 10000000 --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/v${v}_p$i.err || echo "pass $i v$v rc=$?"
  done
done
cd $REPO
python3 - <<'PY'
import csv, glob, collections
for v in (1, 2, 3, 4):
    agg = collections.defaultdict(float); cnt = collections.defaultdict(set)
    for f in glob.glob(f"gpurun_out/sq/v{v}_p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_nn4<true" in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]].add(r["Dispatch_Id"])
    print(f"variant {v}:")
    for k in sorted(agg): print(f"  {k:32s} {agg[k]/max(1,len(cnt[k])):.4g}")
PY
