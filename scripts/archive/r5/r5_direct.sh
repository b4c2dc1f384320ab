#!/bin/bash
# Round 5: side segments' kernels launched directly by the plan (pn2_plan_graph_direct) vs as
# graph launches: pipeline parity tests, then the driver's command and 500 steps, A/B.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/direct
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_a_fullsize.py -k pipeline > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
run() { n=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['verified'], {k: round(v,4) for k,v in d['host'].items()})"; }
for i in 1 2; do
run drv_direct_$i --steps 20 --warmup 5
run drv_graph_$i --steps 20 --warmup 5 --graph-launch
done
run 500_direct --steps 500
run 500_graph --steps 500 --graph-launch
run cfg3_direct --config cfg3
run cfg5_direct --config cfg5
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --e2e-steps 0 --latency-reps 0 --no-verify > $OUT/trace.json 2> $OUT/trace.err || { tail -20 $OUT/trace.err; exit 1; }
python3 tools/sampler_start.py $OUT/trace | tee $OUT/sampler_start_attribution.txt
T=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 tools/lane_report.py "$T" > $OUT/lanes_cfg2.txt && head -30 $OUT/lanes_cfg2.txt
find $OUT/trace -name "*.csv" -size +20M -delete
echo done
