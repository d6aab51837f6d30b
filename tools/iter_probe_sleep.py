"""Per-iterate search time of a 60-iterate session, a 0.5 s idle pause, then 40 more iterates of the
same session: separates a time-dependent (clock) from a state-dependent ramp."""
import json, sys, time
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import iterativeclosestpoint_amd as icp
n = 10_000_000
tgt, src, _ = icp.synth_pair(n)
with icp.Context(0, icp.config(timing_stride=1)) as ctx:
    ctx.set_target(tgt, 10, 20, icp.RULES_ENGINE)
    ctx.set_source(src)
    sess = ctx.session(icp.params_default(max_iterations=200, tolerance=1e-12, flags=icp.FLAG_NO_EARLY_STOP))
    a = sess.step_n_timed(60)
    nn_a, _ = ctx.timings(60)
    time.sleep(0.5)
    b = sess.step_n_timed(40)
    nn_b, _ = ctx.timings(40)
    print(json.dumps({"a": [round(float(x), 3) for x in nn_a], "b_after_sleep": [round(float(x), 3) for x in nn_b]}), flush=True)
