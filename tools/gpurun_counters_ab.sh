# GPU: the wave search's debug counters per iteration for two library builds (same box).
# usage (gpurun): bash tools/gpurun_counters_ab.sh LIB_A LIB_B [ITERS]
set -u
for L in "$1" "$2"; do
  echo "== $L"
  ICP_HIP_LIB=$PWD/$L timeout -k 10 300 python3 tools/counter_probe.py 10000000 ${3:-12} 2>/dev/null | python3 -c "
import json, sys
for line in sys.stdin:
    c = json.loads(line); w = c['waves']
    print(c['iteration'], 'cand/w %.1f' % (c['candidates'] / w), 'staged/w %.1f' % (c['staged_points'] / w),
          'pairs/w %.1f' % (c['scan_pairs'] / w), 'rounds/w %.2f' % (c['scan_rounds'] / w), 'hits', c['cache_hits'],
          'stores', c['cache_stores'], 'ovf', c['overflow_waves'], 'ms', c['search_ms'])" || exit 1
done
