#!/bin/bash
# End-of-round evidence (round 6), part 2: rocprofv3 kernel stats per config (and the profiled
# run's exit status), the cfg2 lane report and critical path, the sampler start attribution
# (kernel + HIP runtime trace), PMC HBM traffic (one counter per pass), sampler stamps.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6/final}
mkdir -p $OUT
for c in cfg2 cfg3 cfg5; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$c -o run -- python3 bench.py --config $c --steps 200 --warmup 20 --no-cpu-baseline --e2e-steps 0 --latency-reps 0 --no-verify > $OUT/prof_$c.json 2> $OUT/prof_$c.err
  rc=$?; echo "rocprofv3 $c exit $rc"; [ $rc -eq 0 ] || { tail -20 $OUT/prof_$c.err; exit 1; }
  S=$(find $OUT/prof_$c -name "*kernel_stats.csv" | head -1); cp "$S" $OUT/kernel_stats_$c.csv
done
T=$(find $OUT/prof_cfg2 -name "*kernel_trace.csv" | head -1)
python3 tools/critical_path.py "$T" > $OUT/critical_path_cfg2.txt || exit 1
python3 tools/lane_report.py "$T" > $OUT/lanes_cfg2.txt || exit 1
head -30 $OUT/lanes_cfg2.txt
find $OUT -name "*kernel_trace.csv" -delete
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --e2e-steps 0 --latency-reps 0 --no-verify > $OUT/trace.json 2> $OUT/trace.err || { tail -20 $OUT/trace.err; exit 1; }
python3 tools/sampler_start.py $OUT/trace > $OUT/sampler_start_attribution.txt || exit 1
head -8 $OUT/sampler_start_attribution.txt
rm -rf $OUT/trace
for cb in cfg2:16 cfg3:16 cfg5:8; do
  c=${cb%%:*}; b=${cb##*:}
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_${C}_$c -o run -- python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --e2e-steps 0 --latency-reps 0 --no-verify > $OUT/pmc_${C}_$c.log 2>&1 || { tail -5 $OUT/pmc_${C}_$c.log; exit 1; }
  done
  python3 tools/pmc_summary.py $OUT/pmc_FETCH_SIZE_$c $OUT/pmc_WRITE_SIZE_$c > $OUT/pmc_traffic_${c}_B$b.json || exit 1
  rm -rf $OUT/pmc_FETCH_SIZE_$c $OUT/pmc_WRITE_SIZE_$c
done
timeout -k 10 200 python3 tools/stamp_fps_cull.py --json $OUT/sa1_cull_stamps.json > $OUT/stamps.log 2>&1 || { tail -20 $OUT/stamps.log; exit 1; }
timeout -k 10 200 python3 tools/stamp_fps_cull.py --msg --json $OUT/msg_cull_stamps.json > $OUT/stamps_msg.log 2>&1 || { tail -20 $OUT/stamps_msg.log; exit 1; }
du -sh $OUT
echo done
