#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3/${TAG:-layers}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_fused_layers.py > $OUT/pytest_fused.log 2>&1 || { tail -30 $OUT/pytest_fused.log; exit 1; }
tail -1 $OUT/pytest_fused.log
timeout -k 10 200 python3 tools/bench_layers.py --json $OUT/layers_cfg2.json || exit 1
timeout -k 10 200 python3 tools/bench_layers.py --config cfg3 --json $OUT/layers_cfg3.json || exit 1
