# GPU: config 5 (50M <-> 50M) parity test and a bench line at that size.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_config5.py -x -v -s --timeout 600 --timeout-method thread > gpurun_out/pytest_cfg5.log 2>&1 || { tail -40 gpurun_out/pytest_cfg5.log; exit 1; }
grep -E "passed|failed|50M|synth|source|iterations|oracle" gpurun_out/pytest_cfg5.log
timeout -k 10 600 python3 -u bench.py --points 50000000 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_50m.json 2> gpurun_out/bench_50m.err || { tail -20 gpurun_out/bench_50m.err; exit 1; }
cat gpurun_out/bench_50m.json
