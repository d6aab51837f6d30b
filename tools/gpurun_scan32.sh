set -u
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "scan32 or variants or kat or octree or edge or 100k" > gpurun_out/pytest_s32.log 2>&1 || { tail -60 gpurun_out/pytest_s32.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_s32.log | tail -3
bash tools/ab_env.sh "ICP_CELLS=1 ICP_CELLS=0"; bash tools/gpurun_dbg.sh
