# GPU: full -m gpu suite, then interleaved bench lines for two env configs (A/B).
# usage: bash tools/gpurun_ab2.sh "ICP_XCD=1" "ICP_XCD=0"
set -u
mkdir -p gpurun_out
A=${1:-ICP_XCD=1}; B=${2:-ICP_XCD=0}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for rep in 1 2; do
for c in "$A" "$B"; do
  env $(echo $c | tr ':' ' ') timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { tail -20 gpurun_out/bench_ab.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_ab.json'));r=d['roofline'];print('[$c]',d['value'],'Mcorr/s',d['ms_per_step'],'ms/step knn',r['kernel_ms_avg'],'iter',r['iterate_device_ms_avg'],'fb',r['exact_fallback_queries'],'ball',r['ball_search_queries'],'lane',r['lane_search_queries'])"
done
done
