#!/bin/bash
# Round 4: per-step timelines (bench.py --timeline, no profiler) of the pipelined cfg2 run at
# 200 and at the driver's 20 steps.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/tl
mkdir -p $OUT
for n in 1 2; do
timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --steps 20 --warmup 5 --timeline $OUT/timeline_20_$n.json > $OUT/b_tl20_$n.json 2> $OUT/b_tl20_$n.err || { tail -20 $OUT/b_tl20_$n.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/b_tl20_$n.json')); print(round(d['value']), d['ms_per_step'])"
python3 tools/timeline_report.py $OUT/timeline_20_$n.json --skip 0 --show 20 | tee $OUT/timeline_20_$n.txt
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --steps 200 --timeline $OUT/timeline_200.json > $OUT/b_tl200.json 2> $OUT/b_tl200.err || { tail -20 $OUT/b_tl200.err; exit 1; }
python3 tools/timeline_report.py $OUT/timeline_200.json | tee $OUT/timeline_200.txt
timeout -k 10 120 python3 tools/cu_mask_probe.py > $OUT/cu_mask_probe.json 2>&1 || { tail -20 $OUT/cu_mask_probe.json; exit 1; }
cat $OUT/cu_mask_probe.json
