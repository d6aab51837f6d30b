#!/bin/bash
# One runner for the GPU-box measurement steps (run through gpurun from the repo root). Every
# GPU step runs under its own `timeout`; a failing step ends the call (no retries).
#
#   bash tools/gpu.sh round TAG              -m gpu suite, a default bench line, rocprof trace + PMC
#   bash tools/gpu.sh ab TAG KEXPR REPS ARM...   optional tests (pytest -k KEXPR, "" none, "all"),
#                                            then REPS interleaved bench lines per ARM
#                                            (ARM = LIB[:key=val,...], LIB = a .so path or "cur";
#                                            AB_BENCH_ARGS: extra bench.py arguments, e.g. --points)
#   bash tools/gpu.sh configs                bench lines of BASELINE configs 2, 3 (1 mm grid), 5
#   bash tools/gpu.sh cfg5                   the 50M parity tests and a 50M bench line with parity
#   bash tools/gpu.sh multi [PTS]            N > 1 rehearsals on one GPU: torchrun ranks over the host
#                                            exchange (W = 2, 4) and the in-process group (--gpus 4)
#   bash tools/gpu.sh probe [ITERS] [LIB]    the wave search's debug counters per iteration
#   bash tools/gpu.sh phases                 phase clocks (libicp_hip_clk.so) and SQ counter passes
#   bash tools/gpu.sh shard [WORLDS] [LIB_B] per-rank iteration cost at 1/W of 10M (LIB_B: A/B)
#   bash tools/gpu.sh timeline [bench args]  kernel trace of a short bench, per-kernel medians
set -u
mkdir -p gpurun_out
CMD=${1:-}
shift || true

bench_line() {  # file arm-label: one summary line of a bench JSON
  python3 -c "
import json,sys; j=json.load(open(sys.argv[1])); r=j['roofline'] or {}; p=j.get('parity') or {}
t=j.get('timed_state_parity') or {}; g=j.get('registration') or {}
print(f\"{sys.argv[2]:44s} value {j['value']:9.1f} median {j['median']['value']:9.1f} k_nn_wave {r.get('kernel_ms_avg')} ms \"
      f\"iter_dev {r.get('iterate_device_ms_avg')} frac {r.get('frac')} ball {j['search_paths']['ball']} \"
      f\"exact {j['search_paths']['exact_fallback']} T_rmse {p.get('final_transform_rmse_vs_cpu')} \"
      f\"timed_mismatch {t.get('idx_mismatch')}/{t.get('dist_mismatch')} reg {g.get('iterations')} it {g.get('mean_value')}\")" "$1" "$2"
}

case "$CMD" in
round)
  TAG=${1:-r03}
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu_$TAG.log
  timeout -k 10 600 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
  cat gpurun_out/bench_$TAG.json
  bash tools/profile_bench.sh $TAG 10000000 || exit 1
  python3 - "$TAG" <<'PY'
import csv, glob, sys
tag = sys.argv[1]
for f in glob.glob(f"gpurun_out/prof_{tag}/trace/*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        print(f'{float(r["AverageNs"])/1e3:10.1f} us x{r["Calls"]:>4} {float(r["Percentage"]):6.2f}%  {r["Name"][:90]}')
PY
  ;;
ab)
  TAG=$1; K=$2; REPS=$3; shift 3
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
      timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity --no-registration $CF ${AB_BENCH_ARGS:-} > $OUTF 2> gpurun_out/ab_$TAG.err || { tail -20 gpurun_out/ab_$TAG.err; exit 1; }
      bench_line $OUTF "$ARM"
    done
  done
  ;;
configs)
  mkdir -p gpurun_out/configs
  timeout -k 10 300 python3 bench.py --points 100000 --steps 200 --cpu-sample 100000 > gpurun_out/configs/config2.json 2> gpurun_out/configs/config2.err || exit 1
  timeout -k 10 300 python3 bench.py --points 1000000 --steps 200 --quantize 0.001 --cpu-sample 200000 > gpurun_out/configs/config3_grid.json 2> gpurun_out/configs/config3_grid.err || exit 1
  timeout -k 10 600 python3 bench.py --points 50000000 --steps 50 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/configs/config5.json 2> gpurun_out/configs/config5.err || exit 1
  for f in gpurun_out/configs/*.json; do bench_line $f $(basename $f .json); done
  ;;
cfg5)
  timeout -k 10 900 python3 -u -m pytest tests/test_gpu_config5.py -x -v -s --timeout 900 --timeout-method thread > gpurun_out/pytest_cfg5.log 2>&1 || { tail -40 gpurun_out/pytest_cfg5.log; exit 1; }
  grep -E "passed|failed|50M|synth|source|iterations|oracle|RMSE" gpurun_out/pytest_cfg5.log
  timeout -k 10 900 python3 -u bench.py --points 50000000 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/bench_50m.json 2> gpurun_out/bench_50m.err || { tail -20 gpurun_out/bench_50m.err; exit 1; }
  cat gpurun_out/bench_50m.json
  ;;
multi)
  PTS=${1:-10000000}
  for W in 2 4; do
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port 2951$W \
       bench.py --gpus $W --points $PTS --steps 10 --warmup 3 --no-cpu-baseline --exchange host \
       > gpurun_out/bench_${W}rank_host.json 2> gpurun_out/bench_${W}rank_host.err || { echo "W=$W failed"; grep -v "^$" gpurun_out/bench_${W}rank_host.err | tail -25; exit 1; }
    bench_line gpurun_out/bench_${W}rank_host.json "torchrun W=$W host exchange"
  done
  timeout -k 10 300 python3 bench.py --gpus 4 --points $PTS --steps 10 --warmup 3 --no-cpu-baseline --no-parity \
    > gpurun_out/bench_group4.json 2> gpurun_out/bench_group4.err || { tail -25 gpurun_out/bench_group4.err; exit 1; }
  bench_line gpurun_out/bench_group4.json "in-process group of 4 on one GPU"
  ;;
probe)
  ITERS=${1:-12}
  LIB=${2:-}
  if [ -n "$LIB" ]; then export ICP_HIP_LIB=$PWD/$LIB; fi
  timeout -k 10 300 python3 tools/counter_probe.py 10000000 $ITERS > gpurun_out/counters.jsonl 2>gpurun_out/counters.err || { tail -20 gpurun_out/counters.err; exit 1; }
  tail -3 gpurun_out/counters.jsonl
  ;;
phases)
  ICP_HIP_LIB=$PWD/iterativeclosestpoint_amd/libicp_hip_clk.so timeout -k 10 300 python3 tools/phase_probe.py > gpurun_out/phase.txt 2>&1 || { tail -20 gpurun_out/phase.txt; exit 1; }
  cat gpurun_out/phase.txt
  bash tools/sq_wave.sh cur "$@"
  ;;
shard)
  W=${1:-1,2,4,8}
  LIB_B=${2:-}
  timeout -k 10 300 python3 tools/shard_probe.py $W || exit 1
  RCCL=1 timeout -k 10 300 python3 tools/shard_probe.py 1,8 || exit 1
  if [ -n "$LIB_B" ]; then ICP_HIP_LIB=$PWD/$LIB_B timeout -k 10 300 python3 tools/shard_probe.py $W || exit 1; fi
  ;;
timeline)
  mkdir -p gpurun_out/tl
  rm -rf gpurun_out/tl/*
  export TMPDIR=/tmp
  REPO=$(pwd)
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/gpurun_out/tl -o tl -- \
    python3 $REPO/bench.py --no-cpu-baseline --no-parity --no-registration --steps 6 --warmup 2 "$@" > $REPO/gpurun_out/tl/bench.json 2> $REPO/gpurun_out/tl/err.log || exit $?
  cd $REPO
  python3 tools/timeline.py gpurun_out/tl
  ;;
*)
  sed -n '2,17p' "$0"
  exit 2
  ;;
esac
