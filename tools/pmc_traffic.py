#!/usr/bin/env python3
"""Summarise rocprofv3 output of the bench into profiles/ (HBM traffic per search launch).

Reads the kernel-trace stats and the counter-collection CSVs written by tools/profile_bench.sh
and applies the read/write factors calibrated for the search kernel's own access widths by
tools/calib_pmc.sh (profiles/calibration.json: 8-B/lane streams and 24-of-32-B / 56-of-64-B record
gathers all read as 1/2 of the true bytes in FETCH_SIZE; stores read exactly in WRITE_SIZE).
FETCH_SIZE/WRITE_SIZE are KiB and count L2 <-> fabric traffic (Infinity-Cache hits included).

usage: pmc_traffic.py PROF_DIR N WORLD  -> JSON on stdout
"""
import csv
import glob
import json
import sys
from collections import defaultdict

KERNEL = "k_nn_wave<true"


def _factors():
    import json as _j
    from pathlib import Path as _P
    c = _j.loads((_P(__file__).resolve().parents[1] / "profiles" / "calibration.json").read_text())["patterns"]
    reads = [c[k]["read_factor"] for k in ("k_stream8", "k_gather32", "k_gather64")]
    writes = [c[k]["write_factor"] for k in ("k_store8", "k_store4")]
    return sum(reads) / len(reads), sum(writes) / len(writes)


READ_FACTOR, WRITE_FACTOR = _factors()


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f, newline="") as fh:
            out.extend(csv.DictReader(fh))
    return out


def per_dispatch(prof, sub):
    """Per-dispatch averages of the search kernel's counters over the dispatches of the profiled
    workload: the largest grid (the context's process warm-up runs the same kernel on a 4096-point
    pair first, icp_ctx.hip warm_kernels; those dispatches are left out)."""
    rs = [r for r in rows(f"{prof}/{sub}/**/*counter_collection.csv") if KERNEL in r.get("Kernel_Name", "")]
    if not rs:
        return {}
    gmax = max(int(r["Grid_Size"]) for r in rs)
    vals = defaultdict(lambda: defaultdict(float))
    for r in rs:
        if int(r["Grid_Size"]) == gmax:
            vals[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: (sum(v.values()) / len(v), len(v)) for k, v in vals.items() if v}


def main():
    prof, n, world = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    # the profiled workload (bench.py workload_key): a profile counts only for the same data
    workload = sys.argv[4] if len(sys.argv) > 4 else "blob|q=0.0|dup=1"
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    from bench import search_source_sha1
    out = {"kernel": KERNEL, "n": n, "world": world, "workload": workload, "search_src_sha1": search_source_sha1()}
    # the kernel's durations over the profiled workload's dispatches (largest grid; see per_dispatch)
    tr = [r for r in rows(f"{prof}/trace/**/*kernel_trace.csv") if KERNEL in r.get("Kernel_Name", "")]
    if tr:
        gmax = max(int(r["Grid_Size_X"]) for r in tr)
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in tr if int(r["Grid_Size_X"]) == gmax]
        out["trace_calls"] = len(d)
        out["trace_avg_ms"] = sum(d) / len(d)
        out["trace_min_ms"] = min(d)
        out["trace_max_ms"] = max(d)
    fetch = per_dispatch(prof, "pmc_fetch").get("FETCH_SIZE")
    write = per_dispatch(prof, "pmc_write").get("WRITE_SIZE")
    hits = per_dispatch(prof, "pmc_l2")
    if fetch:
        out["fetch_size_kib_raw"] = fetch[0]
        out["read_factor"] = READ_FACTOR
        out["fetch_bytes_corrected"] = fetch[0] * 1024 * READ_FACTOR
        out["pmc_dispatches"] = fetch[1]
    if write:
        out["write_size_kib_raw"] = write[0]
        out["write_factor"] = WRITE_FACTOR
        out["write_bytes"] = write[0] * 1024 * WRITE_FACTOR
    if fetch and write:
        out["bytes_per_launch"] = out["fetch_bytes_corrected"] + out["write_bytes"]
    if "TCC_HIT_sum" in hits and "TCC_MISS_sum" in hits:
        h, m = hits["TCC_HIT_sum"][0], hits["TCC_MISS_sum"][0]
        out["l2_hit_rate"] = h / (h + m) if h + m else None
    sq = per_dispatch(prof, "pmc_sq")
    if "SQ_WAVES" in sq and "SQ_INSTS_VALU" in sq and "GRBM_GUI_ACTIVE" in sq:
        waves = sq["SQ_WAVES"][0]
        cyc = sq["GRBM_GUI_ACTIVE"][0] / 8  # GRBM_GUI_ACTIVE sums the 8 XCDs
        out["sq"] = {k: v[0] for k, v in sorted(sq.items())}
        out["valu_per_wave"] = sq["SQ_INSTS_VALU"][0] / waves
        out["salu_per_wave"] = sq["SQ_INSTS_SALU"][0] / waves if "SQ_INSTS_SALU" in sq else None
        out["kernel_cycles"] = cyc
        # a wave64 VALU instruction occupies its SIMD (16 lanes wide) 4 cycles; 256 CUs x 4 SIMDs
        out["valu_issue_frac"] = sq["SQ_INSTS_VALU"][0] * 4 / (1024 * cyc)
        if "SQ_ACTIVE_INST_VALU" in sq:
            out["valu_active_frac"] = sq["SQ_ACTIVE_INST_VALU"][0] * 4 / (1024 * cyc)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
