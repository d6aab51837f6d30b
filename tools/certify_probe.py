#!/usr/bin/env python3
"""The previous-match certificate (icp_hip_config.certify_prev) on two 10M workloads: config 4's
sliding pair (bench.py's) and a registration near convergence (anisotropic cloud moved by a few
mm, 0.5 mm noise). Per mode: median search-kernel and iterate ms over iterations 4..ITERS, and
the share of queries the certificate settled (debug counters, a separate run). One JSON line per
(workload, mode).

usage: python3 tools/certify_probe.py [N] [ITERS]
"""
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import iterativeclosestpoint_amd as icp  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 16
workloads = {
    "config4": {},
    "near_converged": dict(sigma=[8.0, 4.0, 1.5], yaw_deg=0.02, pitch_deg=0.0, roll_deg=0.0,
                           t=[0.002, -0.001, 0.0005], noise_sigma=0.0005),
}
for name, spec in workloads.items():
    tgt, src, _ = icp.synth_pair(n, **spec)
    for mode in (0, 1, 2, 3):
        out = {"workload": name, "n": n, "certify_prev": mode}
        for counters in (0, 1):
            with icp.Context(0, icp.config(certify_prev=mode, debug_counters=counters, timing_stride=1)) as ctx:
                ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
                ctx.set_source(src)
                sess = ctx.session(icp.params_default(max_iterations=iters, tolerance=0.0,
                                                      flags=icp.FLAG_NO_EARLY_STOP))
                settled = []
                for _ in range(iters):
                    sess.step()
                    if counters:
                        c = ctx.debug_counters()
                        settled.append(c["prev_cert_lanes"] / n)
                if not counters:
                    nn_ms, it_ms = ctx.timings(iters)
                    out["search_ms"] = round(float(np.median(nn_ms[3:])), 4)
                    out["iterate_ms"] = round(float(np.median(it_ms[3:])), 4)
                else:
                    out["settled_share"] = round(float(np.median(settled[3:])), 4)
                sess.close()
        print(json.dumps(out), flush=True)
