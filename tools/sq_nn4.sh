#!/bin/bash
# SQ counter passes on k_nn4 (current build), 1 timed step + 1 warmup at 10M.
set -u
REPO=$(pwd); OUT=$REPO/gpurun_out/sq2; rm -rf $OUT; mkdir -p $OUT; export TMPDIR=/tmp
cd /tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_FMA_F64 GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o p -- \
    python3 $REPO/bench.py --points 10000000 --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/p$i.err || { echo "pass $i rc=$?"; exit 1; }
done
cd $REPO
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(float); cnt = collections.defaultdict(set)
for f in glob.glob("gpurun_out/sq2/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_nn4<true" in r["Kernel_Name"]:
            k = r["Counter_Name"]
            key = (f, k)
            agg[key] += float(r["Counter_Value"]); cnt[key].add(r["Dispatch_Id"])
tot = collections.defaultdict(list)
for (f, k), v in agg.items():
    tot[k].append(v / max(1, len(cnt[(f, k)])))
for k in sorted(tot):
    print(f"  {k:28s} {sum(tot[k])/len(tot[k]):.5g}")
PY
