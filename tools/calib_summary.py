#!/usr/bin/env python3
"""Summarise tools/calib_pmc.sh: per access pattern, the counter bytes per dispatch and the factor
true_bytes / counter_bytes (true bytes = the 2 GiB each calibration dispatch touches once).

usage: calib_summary.py CALIB_DIR -> JSON on stdout
"""
import csv
import glob
import json
import sys
from collections import defaultdict

PATTERNS = ("k_stream16", "k_stream8", "k_gather32", "k_gather64", "k_store8", "k_store4")
TRUE_BYTES = 2 << 30


def counters(d, sub):
    vals = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for f in glob.glob(f"{d}/{sub}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f, newline="")):
            name = next((p for p in PATTERNS if p in r.get("Kernel_Name", "")), None)
            if name:
                vals[name][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {p: {c: sum(v.values()) / len(v) for c, v in cs.items()} for p, cs in vals.items()}


def main():
    d = sys.argv[1]
    fetch, write, rdreq = counters(d, "pmc_fetch"), counters(d, "pmc_write"), counters(d, "pmc_rdreq")
    ms = defaultdict(list)
    for f in glob.glob(f"{d}/trace/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f, newline="")):
            name = next((p for p in PATTERNS if p in r["Name"]), None)
            if name:
                ms[name].append(float(r["AverageNs"]) / 1e6)
    out = {"true_bytes_per_dispatch": TRUE_BYTES, "patterns": {}}
    for p in PATTERNS:
        e = {}
        if p in fetch and "FETCH_SIZE" in fetch[p]:
            kib = fetch[p]["FETCH_SIZE"]
            e["fetch_size_kib"] = kib
            e["read_factor"] = TRUE_BYTES / (kib * 1024) if kib else None
        if p in write and "WRITE_SIZE" in write[p]:
            kib = write[p]["WRITE_SIZE"]
            e["write_size_kib"] = kib
            e["write_factor"] = TRUE_BYTES / (kib * 1024) if kib else None
        if p in rdreq:
            e.update({k: v for k, v in rdreq[p].items()})
        if ms.get(p):
            e["trace_ms"] = ms[p][0]
            e["gbs"] = TRUE_BYTES / (ms[p][0] * 1e-3) / 1e9
        out["patterns"][p] = e
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
