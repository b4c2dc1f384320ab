#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3/host
mkdir -p $OUT
for A in "" "--sets 18" "--chain behind --hw-queues 6" "--sampler-lanes 4 --hw-queues 8 --sets 12" "--time-every 1000"; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --e2e-steps 0 $A > $OUT/b.json 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
  python3 -c "
import json; a=json.load(open('$OUT/b.json'))
print('[$A]', round(a['value']), round(a['ms_per_step'],4), round(a['roofline']['avg_launch_ms'],3), {k: round(v,4) for k,v in (a.get('host') or {}).items()})"
done
