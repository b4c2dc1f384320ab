#!/bin/bash
# Round 5: the driver's 20-step window against the number of hardware queues (7 = one per
# pipeline stream; the process also owns its default stream), 6 interleaved runs each.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/hwq
mkdir -p $OUT
for rep in 1 2 3 4 5 6; do
  for q in 7 8 12; do
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --e2e-steps 0 --no-cpu-baseline --hw-queues $q > $OUT/q${q}_$rep.json 2> $OUT/q${q}_$rep.err || { tail -20 $OUT/q${q}_$rep.err; exit 1; }
    echo "q$q $rep $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],4), d.get('verified'))" $OUT/q${q}_$rep.json)"
  done
done
