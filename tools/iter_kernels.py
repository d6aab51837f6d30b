#!/usr/bin/env python3
"""Per-iterate kernel durations from a rocprofv3 kernel trace of a bench run (the search-path
kernels and the tail), one row per iterate: an iterate starts at each k_nn_wave dispatch.

usage: python3 tools/iter_kernels.py TRACE_DIR [FIRST_N]
"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
first_n = int(sys.argv[2]) if len(sys.argv) > 2 else 0
rows = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
short = {"k_nn_wave": "wave", "k_nn_wide": "wide", "k_nn_half": "half", "k_nn_ball": "ball",
         "k_moments": "mom", "k_merge_moments_last": "momL", "k_cull_waves": "cull"}
iters = []
for r in rows:
    name = r["Kernel_Name"]
    key = next((v for k, v in short.items() if k in name), None)
    if key is None:
        continue
    if key == "wave":
        iters.append({"t0": int(r["Start_Timestamp"]), "k": collections.defaultdict(float), "end": 0})
    if not iters:
        continue
    it = iters[-1]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    it["k"][key] += (e - s) / 1e3
    it["end"] = max(it["end"], e)
cols = ["wave", "half", "wide", "ball", "mom", "momL", "cull"]
print("iter " + " ".join(f"{c:>9s}" for c in cols) + "   span_us  (us; ball summed over its launches)")
for n, it in enumerate(iters):
    if first_n and n >= first_n:
        break
    print(f"{n:4d} " + " ".join(f"{it['k'].get(c, 0.0):9.1f}" for c in cols) + f" {(it['end'] - it['t0']) / 1e3:9.1f}")
