set -u
mkdir -p gpurun_out
ICP_NN_DEBUG=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > /dev/null 2> gpurun_out/dbg_phase.err || exit $?
grep 'icp dbg' gpurun_out/dbg_phase.err | grep 'iter=2'
