#!/bin/bash
# Round 4: side lanes alternated over two streams by buffer-set parity (--alt-lanes), FP4's
# lane (2) first: it was the saturated lane of the timeline (its end 1.26 ms after the
# sampler's, the others 0.38-0.49 ms).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/alt
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_a_fullsize.py -k "pipeline" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
run() {  # name, bench args
  n=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['verified'], round(d['latency_ms_per_batch'],3), d['host'])"
}
run default
run alt2 --alt-lanes 2 --hw-queues 8
run alt12 --alt-lanes 1,2 --hw-queues 9
run alt123 --alt-lanes 1,2,3 --hw-queues 10
run alt2own2 --alt-lanes 2 --chain own2 --hw-queues 9
run alt2l4 --alt-lanes 2 --sampler-lanes 4 --hw-queues 9 --sets 12
run drv_default --steps 20 --warmup 5
run drv_alt2 --steps 20 --warmup 5 --alt-lanes 2 --hw-queues 8
run drv_alt12 --steps 20 --warmup 5 --alt-lanes 1,2 --hw-queues 9
timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --steps 200 --alt-lanes 2 --hw-queues 8 --timeline $OUT/timeline_alt2.json > $OUT/b_tl_alt2.json 2> $OUT/b_tl_alt2.err || { tail -20 $OUT/b_tl_alt2.err; exit 1; }
python3 tools/timeline_report.py $OUT/timeline_alt2.json --show 4
run cfg3 --config cfg3
run cfg3_alt2 --config cfg3 --alt-lanes 2 --hw-queues 7
run cfg5 --config cfg5
run cfg5_alt2 --config cfg5 --alt-lanes 2 --hw-queues 9
