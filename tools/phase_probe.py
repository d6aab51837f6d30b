#!/usr/bin/env python3
"""Per-phase clocks and counters of the wave search on the bench workload (diagnostic build of
the library with -DICP_PHASE_CLOCKS=1 loaded through ICP_HIP_LIB; debug counters enabled).

usage: ICP_HIP_LIB=iterativeclosestpoint_amd/libicp_hip_clk.so python3 tools/phase_probe.py [N] [first]
  first: the phases of a source's first iterate (descent guesses, every wave walks) instead of a
  steady one
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402

import iterativeclosestpoint_amd as icp  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
tgt, src, _ = icp.synth_pair(n)
with icp.Context(0, icp.config(debug_counters=1, timing_stride=1)) as ctx:
    ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
    ctx.set_source(src)
    if len(sys.argv) > 2 and sys.argv[2] == "first":
        st = ctx.iterate(None, 0, icp.RULES_ENGINE, 3.0)
    else:
        sess = ctx.session(icp.params_default(max_iterations=20, tolerance=1e-6, flags=icp.FLAG_NO_EARLY_STOP))
        for _ in range(6):
            sess.step()
        st = ctx.iterate(None, 1, icp.RULES_ENGINE, 3.0)
    import ctypes as C
    out = np.zeros(icp._lib.DBG_SLOTS, np.uint64)
    icp._lib._check(icp.lib().icp_hip_debug_counters(ctx.handle, icp._lib._ptr(out)))
    nn_ms, _ = ctx.last_timing()
    w = max(1, int(out[0]))
    names = {16: "guess", 17: "box", 18: "walk (cells + batches)", 19: "scan", 20: "certify+write"}
    tot = sum(int(out[k]) for k in names)
    w = max(w, (n + 63) // 64)
    print(f"waves {w}  k_nn_wave {nn_ms:.4f} ms  candidates/wave {out[7] / w:.1f}  walk batches/wave {out[5] / w:.2f}"
          f"  start nodes/wave {out[21] / w:.1f}  overflow waves {out[1]}  rescan pts {out[4]}")
    for k, nm in names.items():
        print(f"  {nm:24s} {out[k] / w:9.0f} clk/wave  {100.0 * out[k] / max(1, tot):5.1f} %")
