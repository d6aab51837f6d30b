#!/usr/bin/env python3
"""The wave search's debug counters on the bench workload, per iteration (library chosen by
ICP_HIP_LIB; debug counters on). Prints one JSON line per iteration.

usage: python3 tools/counter_probe.py [N] [ITERS]
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import iterativeclosestpoint_amd as icp  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 8
tgt, src, _ = icp.synth_pair(n)
with icp.Context(0, icp.config(debug_counters=1, timing_stride=1)) as ctx:
    ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
    ctx.set_source(src)
    sess = ctx.session(icp.params_default(max_iterations=iters, tolerance=1e-12, flags=icp.FLAG_NO_EARLY_STOP))
    for it in range(iters):
        sess.step()
        c = ctx.debug_counters()
        c["iteration"] = it
        c["search_ms"] = round(ctx.last_timing()[0], 4)
        print(json.dumps(c), flush=True)
