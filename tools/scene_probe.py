#!/usr/bin/env python3
"""Per-iterate search-path counts and kernel times on the LiDAR-like scene (icp_synth_scene),
with scene overrides from the command line (KEY=VALUE), to find what makes a follow-up path slow.

usage: python3 tools/scene_probe.py N ITERS [KEY=VALUE ...]
"""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import iterativeclosestpoint_amd as icp  # noqa: E402

n = int(sys.argv[1])
iters = int(sys.argv[2])
kw = {}
cfg = {}
for a in sys.argv[3:]:
    k, v = a.split("=", 1)
    if k.startswith("cfg."):
        cfg[k[4:]] = float(v) if "." in v else int(v)
    else:
        kw[k] = float(v) if "." in v or "e" in v else int(v)
tgt, src, _ = icp.synth_scene(n, **kw)
base = {"debug_counters": 1, "timing_stride": 1}
base.update(cfg)  # e.g. cfg.debug_counters=0: the product instances' times (no counter atomics)
with icp.Context(0, icp.config(**base)) as ctx:
    ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
    ctx.set_source(src)
    # the engine's own loop (icp_session_step: the reference's increments and stops)
    sess = ctx.session(icp.params_default(max_iterations=iters, tolerance=0.0, flags=icp.FLAG_NO_EARLY_STOP))
    for it in range(iters):
        t0 = time.perf_counter()
        rec = sess.step()
        wall = (time.perf_counter() - t0) * 1e3
        c = ctx.debug_counters()
        nn_ms, it_ms = ctx.last_timing()
        out = {"it": it, "wall_ms": round(wall, 3), "search_ms": round(nn_ms, 4), "iter_ms": round(it_ms, 4),
               "rmse": None if rec is None else rec.rmse}
        for k in ("waves", "overflow_waves", "not_joined", "not_covered", "ball_overflow", "ball_points",
                  "fp64_scan_waves", "cache_hits", "scan_pairs", "staged_points", "bb_queries", "bb_steps",
                  "lane_handed", "bb_overflow", "wide_waves", "wide_segments", "wide_stack", "wide_undecided",
                  "wide_points", "lane_exact", "cache_stores", "walk_moved", "walk_loose", "reused_entries",
                  "candidates", "group_points"):
            out[k] = c.get(k)
        print(json.dumps(out), flush=True)
    sess.finish()
    sess.close()
