#!/usr/bin/env python3
"""Readable summary of a rocprofv3 kernel_stats.csv: short kernel names, calls, avg/min/max us."""
import csv
import re
import sys

for path in sys.argv[1:]:
    for r in list(csv.DictReader(open(path)))[:24]:
        m = re.search(r"(k_[a-z_0-9]+(<[^>]*>)?)", r["Name"])
        n = m.group(1) if m else r["Name"][:44]
        print(f"{n:46s} {r['Calls']:>5s} avg {float(r['AverageNs']) / 1000:9.2f} us  "
              f"min {float(r['MinNs']) / 1000:8.2f}  max {float(r['MaxNs']) / 1000:8.2f}  {r['Percentage']}%")
