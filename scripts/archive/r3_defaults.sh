#!/bin/bash
# the default bench lines (per-config layouts), the GPU suite and smoke
set -o pipefail
OUT=gpurun_out/r3/defaults
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests \
  > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for c in cfg2 cfg3 cfg5; do
  A=""; [ "$c" != "cfg2" ] && A="--no-cpu-baseline"
  timeout -k 10 400 python3 bench.py --config $c $A > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -20 $OUT/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d.get('e2e',{}).get('value'), (d.get('cpu_baseline') or {}).get('value'))"
done
