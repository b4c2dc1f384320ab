#!/bin/bash
# Refresh the round's bench lines (cfg2 default run, cfg3, cfg5) and the geometric kernel-trace
# summaries of the same commands; each GPU step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/refresh
mkdir -p $OUT
export TMPDIR=/tmp
for c in cfg2 cfg3 cfg5; do
  timeout -k 10 300 python bench.py --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -5 $OUT/bench_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$c.json'));print('$c', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d.get('e2e',{}).get('value'))"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$c -o run -- python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 > $OUT/prof_$c.log 2>&1 || { tail -5 $OUT/prof_$c.log; exit 1; }
done
echo done
