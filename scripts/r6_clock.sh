#!/bin/bash
# Round 6: the SA1 sampler's clock in the pipelined step against alone (GRBM_GUI_ACTIVE per
# kernel / its duration), one counter per pass.
set -o pipefail
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r6/clk}
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pipe -o run -- python3 bench.py --steps 60 --warmup 10 --no-cpu-baseline --e2e-steps 0 --latency-reps 0 --no-verify > $O/pipe.log 2>&1 || { tail -5 $O/pipe.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/alone -o run -- python3 tools/bench_sampler.py --reps 5 --inner 4 > $O/alone.log 2>&1 || { tail -5 $O/alone.log; exit 1; }
for d in pipe alone; do
  python3 tools/clock_report.py $O/$d > $O/clock_$d.txt || exit 1
  cat $O/clock_$d.txt
done
find $O -name "*.csv" -size +1M -delete
