#!/bin/bash
# Round 5: every task's standalone cost (tools/bench_side.py) per config, and the halves of the
# cfg2 pipeline alone (bench.py --diag-only) at 500 steps.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/side
mkdir -p $OUT
for c in cfg2 cfg3 cfg5; do
timeout -k 10 300 python3 tools/bench_side.py --config $c --json $OUT/side_$c.json > $OUT/side_$c.log 2>&1 || { tail -20 $OUT/side_$c.log; exit 1; }
cat $OUT/side_$c.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['config'], d['side_sum_us'], {k: v['us'] for k, v in d.items() if isinstance(v, dict)})"
done
for d in side samplers; do
timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --steps 500 --diag-only $d --no-verify > $OUT/b_$d.json 2> $OUT/b_$d.err || { tail -20 $OUT/b_$d.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/b_$d.json')); print('$d', round(d['value']), round(d['ms_per_step'],4))"
done
echo done
