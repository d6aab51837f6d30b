#!/usr/bin/env python3
"""How the 3-sigma threshold moves from iterate to iterate, and how many residuals lie near it.

For the bench workload's trajectory (host loop, engine rules, increments from the statistics),
per iterate k: mean, sd, threshold, the ratio thr_k / thr_{k-1}, the share of residuals in the
band (thr_{k-1} (1 - delta), thr_{k-1} (1 + delta)] for several delta, and the queries the wave
search left to the other searches (ball / exact / per-lane lists). The fused statistics of the
wave search sum the residuals below the band in the search kernel and settle the band
afterwards: this is the data that sizes the band.

usage: python3 tools/band_probe.py [N] [ITERS]
"""
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import iterativeclosestpoint_amd as icp  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 50
deltas = (0.01, 0.02, 0.05, 0.1, 0.2, 0.5)
tgt, src, _ = icp.synth_pair(n)
with icp.Context(0) as ctx:
    ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
    ctx.set_source(src)
    T = None
    prev_thr = None
    for k in range(iters):
        st = ctx.iterate(T, k, icp.RULES_ENGINE, 3.0)
        _, d = ctx.get_correspondences()
        rec = {"iterate": k, "mean": st.mean, "sd": st.std, "thr": st.threshold, "valid": int(st.valid),
               "ball": int(st.n_ball_search), "exact": int(st.n_fallback), "lane": int(st.n_lane_search)}
        if prev_thr is not None:
            rec["ratio"] = st.threshold / prev_thr
            for dl in deltas:
                lo, hi = prev_thr * (1 - dl), prev_thr * (1 + dl)
                rec[f"band_{dl}"] = float(np.count_nonzero((d > lo) & (d <= hi))) / n
                rec[f"in_{dl}"] = bool(lo <= st.threshold <= hi)
        rec["above_thr"] = float(np.count_nonzero(d > st.threshold)) / n
        print(json.dumps(rec), flush=True)
        prev_thr = st.threshold
        T = icp.best_fit_from_stats(st)
