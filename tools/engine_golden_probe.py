#!/usr/bin/env python3
"""Engine-rule golden cases (tests/golden/engine_rules.npz, the real core engine's histories) run
on contexts with different search configurations: per case and configuration, the first
iteration whose cumulative transform leaves 1e-10 of the reference's, the largest difference,
and whether the valid counts match. Localises a parity difference to a search option.

usage: python3 tools/engine_golden_probe.py [CASE ...]   (configs: KEY=VAL,KEY=VAL via --cfg)
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import iterativeclosestpoint_amd as icp  # noqa: E402

golden = np.load(ROOT / "tests" / "golden" / "engine_rules.npz")
meta = json.loads((ROOT / "tests" / "golden" / "golden.json").read_text())["engine_rules"]
args = [a for a in sys.argv[1:] if not a.startswith("--cfg=")]
cfgs = [dict(kv.split("=") for kv in a[len("--cfg="):].split(",")) for a in sys.argv[1:] if a.startswith("--cfg=")]
cfgs = [{k: int(v) for k, v in c.items()} for c in cfgs] or [{}]
cases = args or ["e1k", "e10k", "far", "relaxed", "params", "diverge"]
for name in cases:
    m = meta[name]
    g = {k[len(name) + 1:]: golden[k] for k in golden.files if k.startswith(name + "_")}
    hist = g["history"].reshape(-1, 22)
    p = m["params"]
    params = icp.params_default(max_iterations=p["max_iterations"], tolerance=p["tolerance"],
                                sigma_multiplier=p["sigma"], octree_max_points=p["max_points"],
                                octree_max_depth=p["max_depth"])
    for cfg in cfgs:
        with icp.Context(0, cfg or None) as ctx:
            ctx.set_target(g["target"], p["max_points"], p["max_depth"], icp.RULES_ENGINE)
            ctx.set_source(g["source"])
            rc, res, rh = ctx.run(params)
        first, worst, valid_ok = None, 0.0, True
        for k, (r, h) in enumerate(zip(rh, hist)):
            dT = float(np.abs(np.array(r.transform).reshape(4, 4) - h[4:20].reshape(4, 4)).max())
            valid_ok = valid_ok and r.valid_points == int(h[2])
            worst = max(worst, dT)
            if first is None and dT > 1e-10:
                first = k
        print(json.dumps({"case": name, "cfg": cfg, "n_records": [len(rh), len(hist)], "first_iter_over_1e-10": first,
                          "max_dT": worst, "valid_counts_equal": valid_ok}), flush=True)
