#!/bin/bash
# Round 5: the driver's 20-step window traced (bench.py --timeline), 8 runs: what differs
# between the ~71k and the ~79k runs.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/tl
mkdir -p $OUT
for n in 1 2 3 4 5 6 7 8; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --e2e-steps 0 --no-cpu-baseline --timeline $OUT/tl_$n.json > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  echo "run $n $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],4), d.get('host'))" $OUT/b_$n.json)"
  python3 tools/timeline_report.py $OUT/tl_$n.json --skip 0 --show 20 > $OUT/tl_$n.txt 2>&1 || true
done
