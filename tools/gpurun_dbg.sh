set -u
mkdir -p gpurun_out
ICP_NN_VARIANT=4 ICP_NN_DEBUG=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 --warmup 2 > gpurun_out/bench_dbg.json 2> gpurun_out/bench_dbg.err
echo rc=$?; grep "icp dbg" gpurun_out/bench_dbg.err | head -20
bash tools/sq_profile.sh "4"
