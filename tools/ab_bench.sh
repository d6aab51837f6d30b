#!/bin/bash
# A/B the search-kernel variants in one GPU session: GPU parity tests (default variant) and
# one bench line per variant. usage: bash tools/ab_bench.sh "1 2" [extra bench args]
set -u
mkdir -p gpurun_out
VARIANTS=${1:-"1 2"}
shift || true
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log
if [ $rc -ge 124 ]; then exit $rc; fi
if [ -n "${PYTEST_VARIANT:-}" ]; then
  ICP_NN_VARIANT=$PYTEST_VARIANT timeout -k 10 900 python -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q -p no:cacheprovider > gpurun_out/pytest_gpu_v$PYTEST_VARIANT.log 2>&1
  rc=$?; echo "pytest variant $PYTEST_VARIANT rc=$rc"; tail -15 gpurun_out/pytest_gpu_v$PYTEST_VARIANT.log
  if [ $rc -ge 124 ]; then exit $rc; fi
fi
for v in $VARIANTS; do
  ICP_NN_VARIANT=$v timeout -k 10 600 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench_v$v.json 2> gpurun_out/bench_v$v.err
  rc=$?; echo "variant $v rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench_v$v.err; exit $rc; fi
  python -c "import json;d=json.load(open('gpurun_out/bench_v$v.json'));r=d['roofline'];print('v$v', d['value'],'Mcorr/s', d['ms_per_step'],'ms/step', 'knn', r['kernel_ms_avg'],'ms', 'iter', r['iterate_device_ms_avg'], 'fb', r.get('exact_fallback_queries'), 'lane', r.get('lane_search_queries'))"
done
