#!/bin/bash
# Copy one gpurun_round.sh run's summaries from gpurun_out/ (scratch) into profiles/TAG (tracked).
# usage: bash tools/collect_profile.sh TAG
set -eu
TAG=$1
D=profiles/$TAG
mkdir -p $D
cp gpurun_out/bench_$TAG.json $D/bench_1gpu.json
cp gpurun_out/prof_$TAG/bench_traced.json $D/bench_under_rocprof.json
cp gpurun_out/prof_$TAG/trace/*kernel_stats.csv $D/kernel_stats_bench.csv
cp gpurun_out/pytest_gpu_$TAG.log $D/pytest_gpu.log
python3 tools/pmc_traffic.py gpurun_out/prof_$TAG 10000000 1 > $D/traffic.json
cp $D/traffic.json profiles/traffic_latest.json
ls -la $D
