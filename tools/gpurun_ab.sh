#!/bin/bash
# Same-box A/B of library builds and configurations: optional -m gpu tests (pytest -k expression,
# "" = none, "all" = the whole suite) on the working build, then REPS interleaved bench lines per arm.
# usage (gpurun): bash tools/gpurun_ab.sh TAG KEXPR REPS ARM1 [ARM2 ...]
#   ARM = LIB[:KEY=VAL[,KEY=VAL...]]   LIB = a .so path or "cur"; KEY=VAL = icp_hip_config fields
set -u
TAG=$1; K=$2; REPS=$3; shift 3
mkdir -p gpurun_out
if [ "$K" = "all" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_$TAG.pytest.log 2>&1 || { tail -40 gpurun_out/ab_$TAG.pytest.log; exit 1; }
  tail -2 gpurun_out/ab_$TAG.pytest.log
elif [ -n "$K" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/ab_$TAG.pytest.log 2>&1 || { tail -40 gpurun_out/ab_$TAG.pytest.log; exit 1; }
  tail -2 gpurun_out/ab_$TAG.pytest.log
fi
for r in $(seq 1 $REPS); do
  a=0
  for ARM in "$@"; do
    a=$((a+1))
    L=${ARM%%:*}; CF=""
    if [ "$ARM" != "$L" ]; then for kv in $(echo "${ARM#*:}" | tr ',' ' '); do CF="$CF --config $kv"; done; fi
    if [ "$L" = "cur" ]; then unset ICP_HIP_LIB; else export ICP_HIP_LIB=$PWD/$L; fi
    OUTF=gpurun_out/ab_$TAG.$r.$a.json
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity --no-registration $CF > $OUTF 2> gpurun_out/ab_$TAG.err || { tail -20 gpurun_out/ab_$TAG.err; exit 1; }
    python3 -c "
import json,sys; j=json.load(open(sys.argv[1])); r=j['roofline'] or {}
print(f\"{sys.argv[2]:48s} value {j['value']:9.1f} median {j['median']['value']:9.1f} k_nn_wave {r.get('kernel_ms_avg')} ms iter_dev {r.get('iterate_device_ms_avg')} ball {j['search_paths']['ball']} lane {j['search_paths']['lane']} exact {j['search_paths']['exact_fallback']}\")" $OUTF "$ARM"
  done
done
