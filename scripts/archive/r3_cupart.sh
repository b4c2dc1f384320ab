#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3/cupart
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_a_fullsize.py -k "pipeline and 64" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for L in "cfg2:0:7" "cfg2:64:8" "cfg2:96:8" "cfg2:128:8" "cfg3:0:6" "cfg3:64:7" "cfg3:96:7" "cfg5:0:8" "cfg5:96:9" "cfg5:128:9"; do
  IFS=: read c p q <<< "$L"
  A="--config $c --cu-partition $p --hw-queues $q --no-cpu-baseline --e2e-steps 0"
  timeout -k 10 200 python3 bench.py $A > $OUT/b.json 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
  timeout -k 10 200 python3 bench.py $A --steps 20 --warmup 5 > $OUT/d.json 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
  python3 -c "
import json; a=json.load(open('$OUT/b.json')); b=json.load(open('$OUT/d.json'))
print('$L', round(a['value']), round(a['roofline']['avg_launch_ms'],3), '| 20 steps', round(b['value']))"
done
