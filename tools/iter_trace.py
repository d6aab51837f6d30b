#!/usr/bin/env python3
"""Per-iterate trace of one bench-workload session: what changes from iterate to iterate.

For every iterate k of a session (engine rules, no early stop) it records
  * the search kernel's and the iterate's device time (timing events on every iterate),
  * the displacement of the queries by the increment T_k applied at that iterate (max, mean,
    95th percentile of |T_k x - x| over a fixed 1M-query sample),
  * the fraction of queries whose match changed from the previous iterate,
  * with --dbg, the wave search's debug counters (a second session on a debug context: the same
    trajectory, the counters' atomics make its times meaningless).
One JSON line per iterate. Run it under rocprofv3 --pmc for per-dispatch counters of the same
iterates (the search launch is the k-th k_nn_wave dispatch).

usage: python3 tools/iter_trace.py [N] [ITERS] [--dbg] [--dbg-only] [--no-corr] [--config KEY=VALUE ...]
"""
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import iterativeclosestpoint_amd as icp  # noqa: E402

argv = sys.argv[1:]
overrides = {}
while "--config" in argv:
    k = argv.index("--config")
    key, val = argv[k + 1].split("=", 1)
    overrides[key] = float(val) if "." in val else int(val)
    del argv[k:k + 2]
args = [a for a in argv if not a.startswith("--")]
n = int(args[0]) if args else 10_000_000
iters = int(args[1]) if len(args) > 1 else 50
dbg_only = "--dbg-only" in argv
dbg = "--dbg" in argv or dbg_only
corr = "--no-corr" not in argv

tgt, src, _ = icp.synth_pair(n)
rng = np.random.default_rng(7)
samp = rng.choice(n, size=min(n, 1_000_000), replace=False)
xs = np.ascontiguousarray(src[samp])
params = icp.params_default(max_iterations=iters, tolerance=1e-12, flags=icp.FLAG_NO_EARLY_STOP)


def session_trace(cfg, with_counters):
    xq = xs.copy()
    pending = np.eye(4)  # the increment the next iterate's search applies (T_k = T_cum_k T_cum_{k-1}^-1)
    prev_cum = np.eye(4)
    idx_prev = None
    with icp.Context(0, cfg) as ctx:
        ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
        ctx.set_source(src)
        sess = ctx.session(params)
        for k in range(iters):
            sess.step()
            rec = {"iterate": k}
            if not with_counters:
                nn_ms, it_ms = ctx.last_timing()
                rec["search_ms"] = round(float(nn_ms), 4)
                rec["iterate_ms"] = round(float(it_ms), 4)
                moved = xq @ pending[:3, :3].T + pending[:3, 3]
                dsp = np.sqrt(((moved - xq) ** 2).sum(1))
                xq = moved
                rec["disp_max_mm"] = round(float(dsp.max()) * 1e3, 4)
                rec["disp_mean_mm"] = round(float(dsp.mean()) * 1e3, 4)
                rec["disp_p95_mm"] = round(float(np.percentile(dsp, 95)) * 1e3, 4)
                if corr:
                    idx, _d = ctx.get_correspondences()
                    if idx_prev is not None:
                        rec["match_changed"] = round(float(np.mean(idx != idx_prev)), 5)
                    idx_prev = idx
            else:
                rec.update(ctx.debug_counters())
            T_cum = sess.transform()
            pending = T_cum @ np.linalg.inv(prev_cum)
            prev_cum = T_cum
            print(json.dumps(rec), flush=True)
        sess.close()


if not dbg_only:
    session_trace(icp.config(timing_stride=1, **overrides), False)
if dbg:
    session_trace(icp.config(timing_stride=1, debug_counters=1, **overrides), True)
