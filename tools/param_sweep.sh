#!/bin/bash
# One bench line per configuration override (the same box, one after the other; the first and
# last lines are the defaults, to bound the drift). usage: bash tools/param_sweep.sh STEPS KEY=VAL...
set -u
STEPS=$1; shift
run() {
  timeout -k 10 200 python3 bench.py --steps $STEPS --warmup 5 --no-cpu-baseline --no-parity --no-registration "$@" > /tmp/sweep.json 2> /tmp/sweep.err || { tail -5 /tmp/sweep.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('/tmp/sweep.json').read().strip().splitlines()[-1]); r=d['roofline']
print(f\"{' '.join(sys.argv[1:]) or 'default':28s} value {d['value']:9.1f} median {d['median']['value']:9.1f} search {r['kernel_ms_avg']} iter_dev {r['iterate_device_ms_avg']} ball {d['search_paths']['ball']}\")" "$@"
}
run
for kv in "$@"; do run --config "$kv"; done
run
