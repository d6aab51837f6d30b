"""Per-kernel medians and the last search iteration's timeline from a rocprofv3 kernel trace."""
import collections
import csv
import glob
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tl"
rows = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
per = collections.defaultdict(list)
for r in rows:
    per[r["Kernel_Name"][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
    v2 = sorted(v)
    print(f"{len(v):4d} x  median {v2[len(v2) // 2]:9.1f} us  total {sum(v):10.1f}  {k}")
starts = [i for i, r in enumerate(rows) if "k_nn_wave" in r["Kernel_Name"]]
if len(starts) >= 3:
    a, b = starts[-3], starts[-2]  # one full iteration (the last one is the untimed probe)
    t0 = int(rows[a]["Start_Timestamp"])
    prev_end = t0
    print("timeline of one timed iteration (us): start  dur  gap-before  kernel")
    for r in rows[a:b + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"  {(s - t0) / 1e3:8.1f} {(e - s) / 1e3:8.1f} {(s - prev_end) / 1e3:7.1f}  {r['Kernel_Name'][:70]}")
        prev_end = e
# the first iterate of each session (k_nn_wave<false, ...>: no previous residuals)
firsts = [i for i, r in enumerate(rows) if "k_nn_wave<false" in r["Kernel_Name"]]
for a in firsts:
    nxt = [i for i in starts if i > a]
    b = nxt[0] if nxt else len(rows) - 1
    t0 = int(rows[a]["Start_Timestamp"])
    prev_end = t0
    print("timeline of a first iterate (us): start  dur  gap-before  kernel")
    for r in rows[a:b + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"  {(s - t0) / 1e3:8.1f} {(e - s) / 1e3:8.1f} {(s - prev_end) / 1e3:7.1f}  {r['Kernel_Name'][:70]}")
        prev_end = e
