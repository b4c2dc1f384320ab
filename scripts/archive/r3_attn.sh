#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3/${TAG:-attn}
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_fused_layers.py tests/test_gpu_a_fullsize.py tests/test_gpu_parity.py -k "attention or fused or full or pipeline or stack or attn" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python3 tools/bench_attn.py > $OUT/bench_attn.log 2>&1 || { tail -5 $OUT/bench_attn.log; exit 1; }
tail -8 $OUT/bench_attn.log
for c in cfg3 cfg2; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --e2e-steps 0 > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -20 $OUT/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --e2e-steps 0 --diag-only side > $OUT/side_$c.json 2> $OUT/side_$c.err || { tail -20 $OUT/side_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/side_$c.json')); print('$c side-only', round(d['value']), round(d['ms_per_step'],4))"
done
