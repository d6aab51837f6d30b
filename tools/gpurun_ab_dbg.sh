set -u
mkdir -p gpurun_out
PYTEST_VARIANT=4 bash tools/ab_bench.sh "3 4" || exit $?
ICP_NN_VARIANT=4 ICP_NN_DEBUG=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 2 > gpurun_out/bench_dbg.json 2> gpurun_out/bench_dbg.err
grep "icp dbg" gpurun_out/bench_dbg.err | head -4
