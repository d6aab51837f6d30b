# GPU: full -m gpu suite, then one bench line (no CPU baseline) with the iteration breakdown.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for k in 1 2; do
timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench.json'));r=d['roofline'];print(d['value'],'Mcorr/s',d['ms_per_step'],'ms/step knn',r['kernel_ms_avg'],'iter',r['iterate_device_ms_avg'],'fb',r['exact_fallback_queries'],'ball',r['ball_search_queries'],'lane',r['lane_search_queries'], 'setup', d['setup_s'])"
done
