set -u
mkdir -p gpurun_out
bash tools/profile_bench.sh r03 10000000
python3 - <<'PY'
import csv,glob
for f in glob.glob("gpurun_out/prof_r03/trace/*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        print(f'{float(r["AverageNs"])/1e3:10.1f} us x{r["Calls"]:>4} {float(r["Percentage"]):6.2f}%  {r["Name"][:90]}')
PY
