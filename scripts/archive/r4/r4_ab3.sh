#!/bin/bash
# Round 4 A/B 3: the lean-LDS culled sampler (exactness, standalone time, in the pipeline) and
# a kernel trace of the CU-partitioned pipeline (why a single step's latency doubles there).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/ab3
mkdir -p $OUT
B=pointcloud-segmentation-attention_amd/csrc/build
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_a_fullsize.py -k "sched" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python3 tools/fps_hot_check.py --algos 0,7 --reps 20 > $OUT/fps_lean.jsonl 2>&1 || { tail -20 $OUT/fps_lean.jsonl; exit 1; }
tail -1 $OUT/fps_lean.jsonl
run() {  # name, bench args
  n=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['verified'], round(d['latency_ms_per_batch'],3), d['host'])"
}
run default
PN2HIP_LIB=$B/libpn2hip_v_lean.so run lean
run drv_default --steps 20 --warmup 5
PN2HIP_LIB=$B/libpn2hip_v_lean.so run drv_lean --steps 20 --warmup 5
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_cup64 -o run -- python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline --e2e-steps 0 --no-verify --latency-reps 5 --cu-partition 64 > $OUT/trace_cup64.log 2>&1 || { tail -20 $OUT/trace_cup64.log; exit 1; }
T=$(find $OUT/trace_cup64 -name "*kernel_trace.csv" | head -1)
python3 tools/lane_report.py $T > $OUT/lanes_cup64.txt; head -24 $OUT/lanes_cup64.txt
python3 tools/timeline.py $T -1 > $OUT/timeline_cup64_last.txt; tail -30 $OUT/timeline_cup64_last.txt
