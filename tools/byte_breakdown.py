#!/usr/bin/env python3
"""Per-stream byte breakdown of one k_nn_wave launch, reconciled with the PMC count of the same
iterate (tools/iter_trace.sh output: debug counters of a debug-instance run of the same trajectory,
FETCH_SIZE / WRITE_SIZE of the product instance, calibrated).

Streams (bytes per launch):
  queries      x, y, z read (24 B per query)                      compulsory
  prev_pos     previous match position read (4 B)                 compulsory (the guess)
  records      wave cache records (64 B per wave)
  entries      cache entries streamed by reusing waves (16 B each; ICP_DBG_REUSED_ENTRIES)
  walk_nodes   walk batches x up to 128 node records (64 B)       (upper bound: full batches)
  walk_cands   candidates gathered by walking waves (32-B records)
  rescans      fp64 re-scan gathers (32-B records)
  gathers      the rest of the measured reads: previous-match and winner gathers (32 B records,
               64-B fabric requests, shared between neighbouring queries through L2)
  writes       moved query 24 + pos 4 + residual 8 per query; cache stores (entries 16 B + record)

usage: byte_breakdown.py JOINED.jsonl ITERATE [N]
"""
import json
import sys

path, it = sys.argv[1], int(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 10_000_000
row = None
for line in open(path):
    r = json.loads(line)
    if r["iterate"] == it:
        row = r
if row is None:
    sys.exit(f"iterate {it} not in {path}")
waves = (n + 63) // 64
MB = 1e6
rd = {
    "queries": 24 * n,
    "prev_pos": 4 * n,
    "records": 64 * waves,
    "entries": 16 * row.get("reused_entries", 0),
    "walk_nodes": 64 * 128 * row.get("walk_batches", 0),
    # ICP_DBG_CANDIDATES counts every wave's list (reusing waves' too): the walkers' share
    "walk_cands": 32 * max(0, row.get("candidates", 0) - row.get("reused_entries", 0)),
    "rescans": 32 * row.get("fp64_scan_waves", 0) * 200,
}
measured_rd = row["read_gb"] * 1e9
rd["gathers (rest)"] = measured_rd - sum(rd.values())
stores = row.get("cache_stores", 0)
entries_per_store = row.get("reused_entries", 0) / max(1, row.get("cache_hits", 1))
wr = {"queries+pos+dist": 36 * n, "cache stores": stores * (16 * entries_per_store + 64)}
measured_wr = row["write_gb"] * 1e9
wr["rest"] = measured_wr - sum(wr.values())
compulsory = 64 * n + 28 * n + 56 * 3567687  # the roofline's compulsory bytes
print(f"iterate {it}: search {row['search_ms']} ms, PMC reads {measured_rd / MB:.0f} MB, writes {measured_wr / MB:.0f} MB, "
      f"L2 hit {row.get('l2_hit', float('nan')):.3f}; compulsory model {compulsory / MB:.0f} MB")
print("reads (MB):")
for k, v in rd.items():
    print(f"  {k:16s} {v / MB:8.1f}  ({v / measured_rd * 100:5.1f} %)")
print("writes (MB):")
for k, v in wr.items():
    print(f"  {k:16s} {v / MB:8.1f}  ({v / measured_wr * 100:5.1f} %)")
g = rd["gathers (rest)"]
print(f"gathers: {g / (2 * n):.1f} B per gather over 2 gathers per query (32-B records; 64-B requests x miss rate)")
