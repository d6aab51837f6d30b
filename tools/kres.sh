#!/bin/bash
# Per-kernel resource usage (VGPRs, scratch, spills, occupancy) of one HIP source, compiled as the
# Makefile does: bash tools/kres.sh [SOURCE] [FILTER-REGEX]  (run from the repo root, build container)
SRC=${1:-iterativeclosestpoint_amd/csrc/nn_kernels.hip}
FILT=${2:-.}
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude --offload-arch=gfx950 ${EXTRA:-} -c "$SRC" -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re, sys, subprocess
rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m: continue
    t = m.group(1)
    if t.startswith("Function Name: "):
        cur = {"name": t.split(": ", 1)[1]}; rows.append(cur)
    elif cur is not None and ": " in t:
        k, v = t.split(": ", 1); cur[k.strip()] = v.strip()
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
filt = re.compile(sys.argv[1])
for r, n in zip(rows, names):
    n = n.replace("icp::(anonymous namespace)::", "").replace("(icp::NNLaunch)", "")
    if not filt.search(n): continue
    g = lambda k: r.get(k, "?")
    print("%-60s vgpr %4s scratch %4s vspill %3s sspill %4s occ %s" % (n[:60], g("VGPRs"), g("ScratchSize [bytes/lane]"), g("VGPRs Spill"), g("SGPRs Spill"), g("Occupancy [waves/SIMD]")))
' "$FILT"
