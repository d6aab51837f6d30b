"""Per-rank cost of one ICP iteration at world size W, probed on one GPU (no collectives): the
full 10M target, rank 0's source shard (spatial: a kd-order range; SPATIAL=0: a plain range of the
shuffled cloud). Estimates the strong-scaling floor of bench.py --gpus W. RCCL=1 runs the
iterations over a 1-rank RCCL communicator: the multi-rank path (two ncclAllGather + rank-order
device merges per iteration) without the network. DEVICE_LOOP=1 runs the device-resident loop
(icp_hip_config.device_loop; default 0: the host steps every iteration). STRIDE: timing events
on every STRIDE-th iterate (default 1; an event on a dispatch costs ~3-5 us, so the wall time per
step of STRIDE=1 includes them: use 8 or more for the W table)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import iterativeclosestpoint_amd as icp
from bench import shard_range

n = int(os.environ.get("N", "10000000"))
worlds = [int(w) for w in (sys.argv[1] if len(sys.argv) > 1 else "1,2,4,8").split(",")]
tgt, src, _ = icp.synth_pair(n)
device_loop = int(os.environ.get("DEVICE_LOOP", "0"))
ctx = icp.Context(0, icp.config(device_loop=device_loop, timing_stride=int(os.environ.get("STRIDE", "1"))))
ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
if os.environ.get("RCCL", "0") == "1":
    ctx.comm_init(1, 0, icp.Context.unique_id())
order = icp.source_shard_order(src) if os.environ.get("SPATIAL", "1") == "1" else np.arange(n)
k_steps = int(os.environ.get("STEPS", "10"))
for w in worlds:
    lo, hi = shard_range(n, 0, w)
    ctx.set_source(src[order[lo:hi]])
    sess = ctx.session(icp.params_default(max_iterations=k_steps + 10, tolerance=1e-6, flags=icp.FLAG_NO_EARLY_STOP))
    for _ in range(3):
        sess.step()
    ctx.synchronize()
    k = int(os.environ.get("STEPS", "10"))
    t0 = time.perf_counter()
    sess.step_n(k)
    ctx.synchronize()
    dt = (time.perf_counter() - t0) / k
    nn, it = ctx.timings(min(k, 256))
    nn, it = nn[np.isfinite(nn)], it[np.isfinite(it)]
    print(json.dumps({"world": w, "device_loop": device_loop, "rccl": os.environ.get("RCCL", "0") == "1", "shard": hi - lo, "stride": int(os.environ.get("STRIDE", "1")), "ms_per_step": round(dt * 1e3, 4),
                      "knn_ms": round(float(np.mean(nn)), 4), "iter_device_ms": round(float(np.mean(it)), 4),
                      "est_mcorr_s": round(n / dt / 1e6, 1)}), flush=True)
    sess.finish()
ctx.close()
