# Diagnostics of the search (ICP_NN_DEBUG counters) on the 10M bench workload.
set -u
mkdir -p gpurun_out
ICP_NN_DEBUG=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 --warmup 2 "$@" > gpurun_out/bench_dbg.json 2> gpurun_out/bench_dbg.err
rc=$?; echo rc=$rc; grep "icp dbg" gpurun_out/bench_dbg.err | head -30
exit $rc
