#!/bin/bash
# FP fused-interpolation checks and micro-benchmark across the unroll variants (tools/bench_fp.py).
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/bench_fp.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "interp or fp or three" > gpurun_out/pytest_fp.log 2>&1 || { tail -30 gpurun_out/pytest_fp.log; exit 1; }
tail -1 gpurun_out/pytest_fp.log
for U in ${UNROLLS:-0 1 2 4}; do
  PN2_FP_UNROLL=$U timeout -k 10 120 python -u tools/bench_fp.py >> gpurun_out/bench_fp.log 2>&1 || { tail -20 gpurun_out/bench_fp.log; exit 1; }
done
cat gpurun_out/bench_fp.log
