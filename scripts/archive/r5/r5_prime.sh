#!/bin/bash
# Round 5: the driver's 20-step window against the warm-up length (5 = the driver's; 20 = every
# buffer set used before the timed steps), 4 runs each, interleaved.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/prime
mkdir -p $OUT
for rep in 1 2 3 4 5; do
  for w in 5; do
    timeout -k 10 300 python3 bench.py --steps 20 --warmup $w --e2e-steps 0 --no-cpu-baseline > $OUT/w${w}_$rep.json 2> $OUT/w${w}_$rep.err || { tail -20 $OUT/w${w}_$rep.err; exit 1; }
    echo "w$w $rep $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],4), d.get('verified'), d.get('host'))" $OUT/w${w}_$rep.json)"
  done
done
