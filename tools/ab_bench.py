#!/usr/bin/env python3
"""Interleaved same-box A/B of two library builds on bench.py (one child process per run; this
parent never touches the GPU).

usage: python3 tools/ab_bench.py REPS LIB_A LIB_B -- BENCH_ARGS...
  LIB_* = a path to a libicp_hip*.so, or "cur" (the in-tree libicp_hip.so)
One summary line per run: value, median, search kernel ms (HIP events), iterate device ms,
registration wall ms (when the leg ran).
"""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
argv = sys.argv[1:]
sep = argv.index("--") if "--" in argv else len(argv)
reps, libs, bench_args = int(argv[0]), argv[1:sep], argv[sep + 1:]
for r in range(reps):
    for lib in libs:
        env = dict(os.environ)
        env.pop("ICP_HIP_LIB", None)
        if lib != "cur":
            env["ICP_HIP_LIB"] = str(ROOT / lib) if not os.path.isabs(lib) else lib
        p = subprocess.run([sys.executable, str(ROOT / "bench.py"), *bench_args], env=env, capture_output=True,
                           text=True, timeout=900)
        if p.returncode != 0:
            print(f"{lib}: rc {p.returncode}\n{p.stderr[-2000:]}", flush=True)
            sys.exit(p.returncode)
        d = json.loads(p.stdout.strip().splitlines()[-1])
        rf = d.get("roofline", {})
        reg = d.get("registration") or {}
        print(f"{lib:44s} value {d['value']:9.1f} median {d['median']['value']:9.1f} "
              f"search {rf.get('kernel_ms_avg')} ms iter_dev {rf.get('iterate_device_ms_avg')} ms "
              f"reg {reg.get('wall_ms')} ms tsp {(d.get('timed_state_parity') or {}).get('idx_mismatch')}", flush=True)
