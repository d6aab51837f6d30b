# A/B of environment settings in one GPU session. Each config is a ':'-joined list of VAR=VALUE.
# Parity tests (parity + fullsize) per config, then interleaved bench lines (2 rounds).
# usage: bash tools/ab_env.sh "ICP_SCAN_GROUP=64 ICP_SCAN_GROUP=16:ICP_WAVE_POINTS=768"
set -u
mkdir -p gpurun_out
CONFIGS=${1:-"ICP_SCAN_GROUP=64"}
k=0
for c in $CONFIGS; do
  k=$((k+1))
  env $(echo $c | tr ':' ' ') timeout -k 10 600 python3 -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q -p no:cacheprovider > gpurun_out/pytest_c$k.log 2>&1
  rc=$?; echo "[$c] pytest rc=$rc: $(tail -1 gpurun_out/pytest_c$k.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/pytest_c$k.log; exit $rc; }
  env $(echo $c | tr ':' ' ') ICP_NN_DEBUG=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > /dev/null 2> gpurun_out/dbg_c$k.err || exit $?
  grep 'icp dbg' gpurun_out/dbg_c$k.err | grep 'iter=2' | grep -v lane_list | sed "s/^/[$c] /"
done
for rep in 1 2; do
k=0
for c in $CONFIGS; do
  k=$((k+1))
  env $(echo $c | tr ':' ' ') timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/bench_c$k.json 2> gpurun_out/bench_c$k.err || { tail -5 gpurun_out/bench_c$k.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_c$k.json'));r=d['roofline'];print('[$c]', d['value'],'Mcorr/s',d['ms_per_step'],'ms/step knn',r['kernel_ms_avg'],'iter',r['iterate_device_ms_avg'],'ball',r['ball_search_queries'])"
done
done
