# One GPU call: the -m gpu suite, a default bench line, then the rocprof trace + PMC passes.
# usage (gpurun): bash tools/gpurun_round.sh TAG
set -u
TAG=${1:-r03}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
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
