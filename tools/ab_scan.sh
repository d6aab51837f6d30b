# A/B of the scan lane-group size (ICP_SCAN_GROUP) in one GPU session: parity tests per setting,
# then one bench line (and debug counters) per setting. usage: bash tools/ab_scan.sh "64 16 8"
set -u
mkdir -p gpurun_out
for g in ${1:-"64 16 8"}; do
  ICP_SCAN_GROUP=$g timeout -k 10 600 python3 -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q -p no:cacheprovider > gpurun_out/pytest_g$g.log 2>&1
  rc=$?; echo "group $g pytest rc=$rc: $(tail -1 gpurun_out/pytest_g$g.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/pytest_g$g.log; exit $rc; }
done
for g in ${1:-"64 16 8"}; do
  ICP_SCAN_GROUP=$g ICP_NN_DEBUG=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > /dev/null 2> gpurun_out/dbg_g$g.err || exit $?
  echo "group $g: $(grep 'icp dbg' gpurun_out/dbg_g$g.err | grep 'iter=2 waves' | head -1)"
done
for rep in 1 2; do
for g in ${1:-"64 16 8"}; do
  ICP_SCAN_GROUP=$g timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/bench_g$g.json 2> gpurun_out/bench_g$g.err || { tail -5 gpurun_out/bench_g$g.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_g$g.json'));r=d['roofline'];print('group $g', d['value'],'Mcorr/s',d['ms_per_step'],'ms/step knn',r['kernel_ms_avg'],'iter',r['iterate_device_ms_avg'],'ball',r['ball_search_queries'])"
done
done
