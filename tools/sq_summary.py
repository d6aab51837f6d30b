#!/usr/bin/env python3
"""Average SQ counters per dispatch of one kernel over the rocprofv3 passes of tools/sq_wave.sh,
plus derived rates (VALU instructions per wave, VALU issue utilisation at the measured clock).

usage: sq_summary.py DIR KERNEL_SUBSTRING
"""
import csv
import glob
import sys
from collections import defaultdict

d, kern = sys.argv[1], sys.argv[2]
vals = defaultdict(lambda: defaultdict(float))
for f in glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f, newline="")):
        if kern in r["Kernel_Name"]:
            vals[(f, r["Counter_Name"])][r["Dispatch_Id"]] += float(r["Counter_Value"])
c = defaultdict(list)
for (f, k), v in vals.items():
    c[k].append(sum(v.values()) / len(v))
c = {k: sum(v) / len(v) for k, v in c.items()}
for k in sorted(c):
    print(f"  {k:28s} {c[k]:.5g}")
if c.get("SQ_WAVES"):
    w = c["SQ_WAVES"]
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD"):
        if k in c:
            print(f"  {k + ' / wave':28s} {c[k] / w:.1f}")
if c.get("GRBM_GUI_ACTIVE") and c.get("SQ_INSTS_VALU"):
    # GRBM_GUI_ACTIVE sums the 8 XCDs; a wave64 VALU instruction occupies its SIMD32 2 cycles;
    # 256 CUs x 4 SIMDs
    cyc = c["GRBM_GUI_ACTIVE"] / 8
    print(f"  {'kernel cycles (GRBM/8)':28s} {cyc:.5g}")
    print(f"  {'VALU issue utilisation':28s} {c['SQ_INSTS_VALU'] * 2 / (1024 * cyc):.3f}")
