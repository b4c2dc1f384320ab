#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3/chainown
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_a_fullsize.py -k "pipeline" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for L in "cfg2:3:b:6:9:" "cfg2:3:b:7:9:--chain own" "cfg2:4:b:8:12:--chain own" "cfg2:3:a:6:9:--chain own" "cfg3:2:a:5:6:" "cfg3:2:a:6:6:--chain own" "cfg3:3:a:7:9:--chain own" "cfg5:5:a:8:10:" "cfg5:4:a:8:10:--chain own"; do
  IFS=: read c l s q n x <<< "$L"
  A="--config $c --sampler-lanes $l --side-layout $s --hw-queues $q --sets $n --no-cpu-baseline --e2e-steps 0 $x"
  timeout -k 10 200 python3 bench.py $A > $OUT/b.json 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
  timeout -k 10 200 python3 bench.py $A --steps 20 --warmup 5 > $OUT/d.json 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
  python3 -c "
import json; a=json.load(open('$OUT/b.json')); b=json.load(open('$OUT/d.json'))
print('$L', round(a['value']), round(a['roofline']['avg_launch_ms'],3), '| 20 steps', round(b['value']))"
done
