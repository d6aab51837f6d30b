# GPU: interleaved bench lines for several env configs (A/B/C...), no test suite.
# usage: bash tools/gpurun_abk.sh REPS "CFG1" "CFG2" ...   (CFG = ':'-joined VAR=VALUE list)
set -u
mkdir -p gpurun_out
R=$1; shift
for rep in $(seq $R); do
for c in "$@"; do
  env $(echo $c | tr ':' ' ') timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { tail -20 gpurun_out/bench_ab.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_ab.json'));r=d['roofline'];print('[$c]',d['value'],'Mcorr/s',d['ms_per_step'],'ms/step knn',r['kernel_ms_avg'],'iter',r['iterate_device_ms_avg'],'ball',r['ball_search_queries'])"
done
done
