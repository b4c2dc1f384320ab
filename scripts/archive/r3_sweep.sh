#!/bin/bash
# layout sweep: sampler lanes / side layout / hw queues / buffer sets, steady (500 steps) and
# at the driver's 20 steps
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3/${TAG:-sweep}
mkdir -p $OUT
C=${CONFIG:-cfg2}
for L in ${LAYS:-3:a:5:9 3:b:6:9 4:a:6:12 4:b:7:12 4:a:6:8 5:a:7:10}; do
  IFS=: read l s q n <<< "$L"
  A="--config $C --sampler-lanes $l --side-layout $s --hw-queues $q --sets $n --no-cpu-baseline --e2e-steps 0"
  timeout -k 10 200 python3 bench.py $A > $OUT/b_${C}_$l$s$q$n.json 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
  timeout -k 10 200 python3 bench.py $A --steps 20 --warmup 5 > $OUT/d_${C}_$l$s$q$n.json 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
  python3 -c "
import json; a=json.load(open('$OUT/b_${C}_$l$s$q$n.json')); b=json.load(open('$OUT/d_${C}_$l$s$q$n.json'))
print('$C $L', round(a['value']), round(a['roofline']['avg_launch_ms'],3), '| 20 steps', round(b['value']))"
done
