set -u
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_octree_build.py -x -v --timeout 120 --timeout-method thread -s > gpurun_out/pytest_f2.log 2>&1 || { tail -60 gpurun_out/pytest_f2.log; exit 1; }
grep -E "passed|failed|device build of" gpurun_out/pytest_f2.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_all.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_all.log
timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/bench_f2.json 2> gpurun_out/bench_f2.err || { tail -20 gpurun_out/bench_f2.err; exit 1; }
cat gpurun_out/bench_f2.json
