#!/bin/bash
# Round 6: rocprofv3 kernel stats of the pipelined step per config (CONFIGS), the lane report
# of each; optional copy-peak sweep (COPY=1, tools/ubench/copy_peak).
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6/prof}
mkdir -p $OUT
if [ -n "${COPY:-}" ]; then
  timeout -k 10 120 tools/ubench/copy_peak > $OUT/copy_peak_sweep.jsonl || exit 1
  sort -t: -k5 -n $OUT/copy_peak_sweep.jsonl | tail -3
fi
for c in ${CONFIGS:-cfg2 cfg3 cfg5}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$c -o run -- python3 bench.py --config $c --steps 200 --warmup 20 --no-cpu-baseline --e2e-steps 0 --latency-reps 0 --no-verify ${BENCH_ARGS:-} > $OUT/prof_$c.json 2> $OUT/prof_$c.err
  rc=$?; echo "rocprofv3 $c exit $rc"; [ $rc -eq 0 ] || { tail -20 $OUT/prof_$c.err; exit 1; }
  S=$(find $OUT/prof_$c -name "*kernel_stats.csv" | head -1); cp "$S" $OUT/kernel_stats_$c.csv
  T=$(find $OUT/prof_$c -name "*kernel_trace.csv" | head -1)
  python3 tools/lane_report.py "$T" > $OUT/lanes_$c.txt || exit 1
  head -24 $OUT/lanes_$c.txt
  find $OUT/prof_$c -name "*kernel_trace.csv" -delete
done
