#!/bin/bash
# Round 5: where the whole-model step's time goes (bench.py --model, cfg2 and cfg3): the e2e
# number itself, then a rocprofv3 kernel trace + stats and the per-queue occupancy report.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/model
mkdir -p $OUT
for c in cfg2 cfg3; do
  timeout -k 10 300 python3 bench.py --model --config $c --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 > $OUT/b_$c.json 2> $OUT/b_$c.err || { tail -20 $OUT/b_$c.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']), round(d['ms_per_step'],4), d.get('verified'), d['config'].get('streams'))" $OUT/b_$c.json $c
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$c -o run -- python3 bench.py --model --config $c --steps 100 --warmup 10 --no-cpu-baseline --e2e-steps 0 --latency-reps 0 --no-verify > $OUT/trace_$c.json 2> $OUT/trace_$c.err || { tail -20 $OUT/trace_$c.err; exit 1; }
  S=$(find $OUT/trace_$c -name "*kernel_stats.csv" | head -1)
  cp "$S" $OUT/kernel_stats_model_$c.csv
  T=$(find $OUT/trace_$c -name "*kernel_trace.csv" | head -1)
  python3 tools/lane_report.py "$T" > $OUT/lanes_model_$c.txt && head -40 $OUT/lanes_model_$c.txt
  find $OUT/trace_$c -name "*.csv" -size +20M -delete
done
