#!/usr/bin/env python3
"""Join tools/iter_trace.sh's outputs into one table per iterate: search time, displacement,
match changes, the wave search's debug counters and the per-dispatch PMC counters of the
iterate's k_nn_wave launch (FETCH_SIZE x the calibrated read factor, WRITE_SIZE, L2 hit rate).

usage: iter_trace_summary.py OUT_DIR  -> text table on stdout, OUT_DIR/joined.jsonl
"""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_traffic import READ_FACTOR, WRITE_FACTOR  # noqa: E402

out = Path(sys.argv[1])


def jl(p):
    f = out / p
    if not f.exists():
        return []
    return [json.loads(x) for x in f.read_text().splitlines() if x.startswith("{")]


def pmc(sub):
    """counter -> list of per-dispatch values of the search launches, dispatch order"""
    vals = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(str(out / sub / "**" / "*counter_collection.csv"), recursive=True):
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                if "k_nn_wave" not in r.get("Kernel_Name", ""):
                    continue
                vals[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return {c: [v[d] for d in sorted(v)] for c, v in vals.items()}


times = jl("times.jsonl")
cd = jl("corr_dbg.jsonl")
n_it = len(times)
corr = cd[:n_it]
dbg = cd[n_it:]
pm = {}
for sub in ("pmc_l2", "pmc_fetch", "pmc_write", "pmc_sq"):
    pm.update(pmc(sub))

rows = []
for k in range(n_it):
    r = dict(times[k])
    if k < len(corr) and "match_changed" in corr[k]:
        r["match_changed"] = corr[k]["match_changed"]
    if k < len(dbg):
        for key in ("cache_hits", "cache_stores", "overflow_waves", "walk_batches", "staged_points", "scan_pairs",
                    "reused_entries", "candidates", "fp64_scan_waves", "not_joined", "halves", "walk_moved",
                    "walk_loose"):
            if key in dbg[k]:
                r[key] = dbg[k][key]
    for c, v in pm.items():
        if k < len(v):
            r[c] = v[k]
    if "FETCH_SIZE" in r:
        r["read_gb"] = r["FETCH_SIZE"] * 1024 * READ_FACTOR / 1e9
    if "WRITE_SIZE" in r:
        r["write_gb"] = r["WRITE_SIZE"] * 1024 * WRITE_FACTOR / 1e9
    if "TCC_HIT_sum" in r and "TCC_MISS_sum" in r:
        r["l2_hit"] = r["TCC_HIT_sum"] / max(1.0, r["TCC_HIT_sum"] + r["TCC_MISS_sum"])
    rows.append(r)

with open(out / "joined.jsonl", "w") as fh:
    for r in rows:
        fh.write(json.dumps(r) + "\n")

cols = [("iterate", "{:>3}"), ("search_ms", "{:7.3f}"), ("disp_mean_mm", "{:7.2f}"), ("disp_max_mm", "{:7.2f}"),
        ("match_changed", "{:6.3f}"), ("cache_hits", "{:7d}"), ("cache_stores", "{:6d}"), ("walk_batches", "{:6d}"),
        ("reused_entries", "{:9d}"), ("staged_points", "{:9d}"), ("read_gb", "{:6.3f}"), ("write_gb", "{:6.3f}"),
        ("l2_hit", "{:6.3f}"), ("SQ_WAIT_ANY", "{:10.3g}"), ("SQ_BUSY_CYCLES", "{:10.3g}")]
print(" ".join(c for c, _ in cols))
for r in rows:
    cells = []
    for c, f in cols:
        v = r.get(c)
        cells.append(f.format(v) if v is not None else "-")
    print(" ".join(cells))
# correlation of the search time with each column over iterates 2..
import numpy as np  # noqa: E402

st = np.array([r["search_ms"] for r in rows[2:]])
print("\ncorrelation with search_ms over iterates 2..:")
for c, _ in cols[2:]:
    v = [r.get(c) for r in rows[2:]]
    if all(x is not None for x in v) and len(v) > 3 and np.std(v) > 0:
        print(f"  {c:16s} {np.corrcoef(st, np.array(v, float))[0, 1]:+.3f}")
