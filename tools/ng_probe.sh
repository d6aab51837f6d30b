set -u
mkdir -p gpurun_out/ng
for NG in 1 2 4; do
  timeout -k 10 300 python3 -u tools/iter_trace.py 10000000 8 --dbg-only --config scan_groups=$NG > gpurun_out/ng/dbg_$NG.jsonl 2> gpurun_out/ng/dbg_$NG.err || exit 1
done
export TMPDIR=/tmp
REPO=$(pwd)
cd /tmp
for NG in 1 2 4; do
  [ "$NG" = 1 ] && continue; timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d $REPO/gpurun_out/ng/pmc_$NG -o pmc -- python3 $REPO/tools/iter_trace.py 10000000 8 --no-corr --config scan_groups=$NG > $REPO/gpurun_out/ng/pmc_$NG.jsonl 2> $REPO/gpurun_out/ng/pmc_$NG.err || exit 1
done
