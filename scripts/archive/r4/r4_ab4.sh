#!/bin/bash
# Round 4 A/B 4: launch segments split at new cross-lane waits (SA1's grouping no longer waits
# for the later samplers' chain) vs the round-3 merge (PN2_SEG_MERGE=1); cfg5 with one grid
# of edge 0.2; a kernel trace of the new default with its critical path.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/ab4
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_a_fullsize.py -k "pipeline or stack or cfg4" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
run() {  # name, bench args
  n=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['verified'], round(d['latency_ms_per_batch'],3), d['host'])"
}
run split
PN2_SEG_MERGE=1 run merge
run drv_split --steps 20 --warmup 5
PN2_SEG_MERGE=1 run drv_merge --steps 20 --warmup 5
run drv_split2 --steps 20 --warmup 5
PN2_SEG_MERGE=1 run drv_merge2 --steps 20 --warmup 5
run cfg5 --config cfg5
run cfg3 --config cfg3
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_cfg2 -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --e2e-steps 0 --no-verify --latency-reps 5 > $OUT/trace_cfg2.log 2>&1 || { tail -20 $OUT/trace_cfg2.log; exit 1; }
T=$(find $OUT/trace_cfg2 -name "*kernel_trace.csv" | head -1)
python3 tools/critical_path.py $T --out $OUT/critical_path_cfg2.txt | head -12
timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --steps 200 --timeline $OUT/timeline_200.json > $OUT/b_tl200.json 2> $OUT/b_tl200.err || { tail -20 $OUT/b_tl200.err; exit 1; }
python3 tools/timeline_report.py $OUT/timeline_200.json | tee $OUT/timeline_200.txt
timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --steps 20 --warmup 5 --timeline $OUT/timeline_20.json > $OUT/b_tl20.json 2> $OUT/b_tl20.err || { tail -20 $OUT/b_tl20.err; exit 1; }
python3 tools/timeline_report.py $OUT/timeline_20.json --skip 0 --show 20 | tee $OUT/timeline_20.txt
