#!/bin/bash
# Round 5 start: the driver's command twice on this box, then the SA1 sampler start attribution
# (rocprofv3 kernel trace + HIP runtime trace, tools/sampler_start.py) of the cfg2 pipeline.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/start
mkdir -p $OUT
for n in 1 2; do
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 > $OUT/b_drv_$n.json 2> $OUT/b_drv_$n.err || { tail -20 $OUT/b_drv_$n.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/b_drv_$n.json')); print('drv', round(d['value']), d['ms_per_step'], d['verified'], d['host'])"
done
timeout -k 10 300 python3 bench.py --steps 500 --no-cpu-baseline --e2e-steps 0 > $OUT/b_500.json 2> $OUT/b_500.err || { tail -20 $OUT/b_500.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/b_500.json')); print('500', round(d['value']), d['ms_per_step'], d['verified'], d['host'])"
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --e2e-steps 0 --latency-reps 0 --no-verify > $OUT/trace.json 2> $OUT/trace.err || { tail -20 $OUT/trace.err; exit 1; }
python3 tools/sampler_start.py $OUT/trace | tee $OUT/sampler_start_attribution.txt
T=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 tools/lane_report.py "$T" > $OUT/lanes_cfg2.txt && head -30 $OUT/lanes_cfg2.txt
find $OUT/trace -name "*.csv" -size +20M -delete
echo done
