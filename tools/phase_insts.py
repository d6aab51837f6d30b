#!/usr/bin/env python3
"""Instructions per wave of each phase of the wave search (k_nn_wave), from SQ counters.

A diagnostic build (`-DICP_PHASE_STOP=1`, tools/build_variant.sh pstop) lets one launch of the
search return after a chosen phase (icp_hip_debug_phase_stop; nn_kernels.hip PSTOP): the counters
of launches stopped after phases 1..6 and of a full one (0) give each phase's instructions per
wave as differences. The stopped launch is the LAST search launch of its process; its results are
not the search's (the session's later records are not used).

  run:        ICP_HIP_LIB=.../libicp_hip_pstop.so python3 tools/phase_insts.py run MODE STOP [N]
              MODE: first (a source's first iterate), second (the iterate after it: every wave
              walks), steady (the 11th iterate of a session: the driver window's state)
  summarize:  python3 tools/phase_insts.py summarize DIR  (DIR/<mode>_<stop>/**/counter_collection.csv)
"""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

PHASES = {1: "first round trip (query, previous match, cache record)", 2: "guess", 3: "search box",
          4: "walk (cells + batches, walking waves only)", 5: "scan + winner's fp64 distance",
          6: "certify, write, queue", 0: "wave record (covariance sums)"}
ORDER = [1, 2, 3, 4, 5, 6, 0]
STEPS = {"first": 0, "second": 1, "steady": 10}
KERNEL = "k_nn_wave<"


def run(mode, stop, n):
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import ctypes as C

    import iterativeclosestpoint_amd as icp
    setter = icp.lib().icp_hip_debug_phase_stop  # only the ICP_PHASE_STOP build exports it
    setter.argtypes, setter.restype = [C.c_int], C.c_int
    tgt, src, _ = icp.synth_pair(n)
    with icp.Context(0, icp.config()) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        ctx.set_source(src)
        sess = ctx.session(icp.params_default(max_iterations=64, tolerance=1e-6, flags=icp.FLAG_NO_EARLY_STOP))
        for _ in range(STEPS[mode]):
            sess.step()
        assert setter(stop) == 0
        sess.step()  # the counted launch (the last search launch of this process)
        assert setter(0) == 0
    print(json.dumps({"mode": mode, "stop": stop, "n": n}))


def last_dispatch(d):
    rs = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        with open(f, newline="") as fh:
            rs.extend(r for r in csv.DictReader(fh) if KERNEL in r.get("Kernel_Name", ""))
    if not rs:
        return None, None
    gmax = max(int(r["Grid_Size"]) for r in rs)
    last = max(int(r["Dispatch_Id"]) for r in rs if int(r["Grid_Size"]) == gmax)
    vals = defaultdict(float)
    name = None
    for r in rs:
        if int(r["Dispatch_Id"]) == last:
            vals[r["Counter_Name"]] += float(r["Counter_Value"])
            name = r["Kernel_Name"]
    return vals, name


def summarize(root):
    out = {}
    for mode in STEPS:
        cum = {}
        kname = None
        for stop in range(7):
            v, name = last_dispatch(f"{root}/{mode}_{stop}")
            if v is None:
                continue
            w = max(1.0, v.get("SQ_WAVES", 0.0))
            cum[stop] = {k: v[k] / w for k in v if k != "SQ_WAVES"}
            cum[stop]["waves"] = w
            if stop == 0:
                kname = name
        if len(cum) < 7:
            continue
        rows, prev = [], {k: 0.0 for k in cum[0]}
        for stop in ORDER:
            c = cum[stop]
            rows.append({"phase": PHASES[stop],
                         **{k.replace("SQ_INSTS_", "").lower(): round(c[k] - prev.get(k, 0.0), 1)
                            for k in c if k.startswith("SQ_INSTS_")}})
            prev = c
        out[mode] = {"kernel": kname, "waves": cum[0]["waves"],
                     "total_per_wave": {k.replace("SQ_INSTS_", "").lower(): round(cum[0][k], 1)
                                        for k in cum[0] if k.startswith("SQ_INSTS_")},
                     "phases": rows}
    print(json.dumps(out, indent=1))
    for mode, m in out.items():
        cols = [k for k in m["total_per_wave"]]
        print(f"\n{mode}: {m['kernel'][:60]}  waves {m['waves']:.0f}")
        print(f"  {'phase':54s}" + "".join(f"{c:>10s}" for c in cols))
        for r in m["phases"]:
            print(f"  {r['phase']:54s}" + "".join(f"{r.get(c, 0.0):10.1f}" for c in cols))
        print(f"  {'total':54s}" + "".join(f"{m['total_per_wave'][c]:10.1f}" for c in cols))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]) if len(sys.argv) > 4 else 10_000_000)
    else:
        summarize(sys.argv[2])
