#!/usr/bin/env python3
"""Per-iterate search-kernel and iterate device times of a long session at the bench workload
(timing events on every iterate), then a second session on the same context and source: shows how
the per-iterate cost evolves from the first iterates to the steady state.

usage: python3 tools/iter_probe.py [N] [ITERS]
"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import iterativeclosestpoint_amd as icp  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 80
tgt, src, _ = icp.synth_pair(n)
with icp.Context(0, icp.config(timing_stride=1)) as ctx:
    ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
    for run in range(2):
        ctx.set_source(src)
        t0 = time.perf_counter()
        sess = ctx.session(icp.params_default(max_iterations=iters, tolerance=1e-12, flags=icp.FLAG_NO_EARLY_STOP))
        step_ms = sess.step_n_timed(iters)
        wall = time.perf_counter() - t0
        nn_ms, it_ms = ctx.timings(min(iters, 256))
        sess.close()
        print(json.dumps({"run": run, "wall_s": round(wall, 4),
                          "nn_ms": [round(float(x), 4) for x in nn_ms],
                          "it_ms": [round(float(x), 4) for x in it_ms],
                          "step_ms": [round(float(x), 4) for x in step_ms]}), flush=True)
