# Quick GPU check: -m gpu suite, debug counters, one bench line.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpurun_dbg.sh || exit $?
timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench.json'));r=d['roofline'];print(d['value'],'Mcorr/s',d['ms_per_step'],'ms/step knn',r['kernel_ms_avg'],'iter',r['iterate_device_ms_avg'],'fb',r['exact_fallback_queries'],'ball',r['ball_search_queries'],'lane',r['lane_search_queries'])"
