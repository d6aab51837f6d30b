# GPU: interleaved bench lines for two env configs (A/B), no test suite.
# usage: bash tools/gpurun_abn.sh "ICP_XCD=1" "ICP_XCD=0" [reps]
set -u
mkdir -p gpurun_out
A=${1:-ICP_XCD=1}; B=${2:-ICP_XCD=0}; R=${3:-2}
for rep in $(seq $R); do
for c in "$A" "$B"; do
  env $(echo $c | tr ':' ' ') timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { tail -20 gpurun_out/bench_ab.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_ab.json'));r=d['roofline'];print('[$c]',d['value'],'Mcorr/s',d['ms_per_step'],'ms/step knn',r['kernel_ms_avg'],'iter',r['iterate_device_ms_avg'],'fb',r['exact_fallback_queries'],'ball',r['ball_search_queries'],'lane',r['lane_search_queries'])"
done
done
