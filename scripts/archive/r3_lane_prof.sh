#!/bin/bash
# kernel traces of the multi-sampler-lane pipeline (cfg2 / cfg3 / cfg5, 2 sampler lanes) and
# the per-queue occupancy report of each (tools/lane_report.py)
set -o pipefail
OUT=gpurun_out/r3/lanes
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in ${CONFIGS:-cfg2 cfg3 cfg5}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$c -o run -- \
    python3 bench.py --config $c --steps 60 --warmup 10 --no-cpu-baseline --e2e-steps 0 \
    --sampler-lanes ${LANES:-2} ${BENCH_ARGS:-} > $OUT/bench_$c.json 2> $OUT/bench_$c.err \
    || { tail -20 $OUT/bench_$c.err; exit 1; }
  f=$(ls $OUT/prof_$c/*/run_kernel_trace.csv 2>/dev/null | head -1)
  [ -z "$f" ] && f=$(find $OUT/prof_$c -name '*kernel_trace.csv' | head -1)
  python3 tools/lane_report.py $f 40 > $OUT/lanes_$c.txt && cat $OUT/lanes_$c.txt
  python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', round(d['value']), round(d['ms_per_step'],4))"
done
for c in ${CONFIGS:-cfg2 cfg3 cfg5}; do
  timeout -k 10 200 python3 tools/host_overhead.py --config $c --steps 100 --geometry-only --sampler-lanes ${LANES:-2} | tee $OUT/host_$c.json
done
