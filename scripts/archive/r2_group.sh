#!/bin/bash
# Grouping checks and micro-benchmark (tools/bench_group.py).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "group or sa or stack or smoke" > gpurun_out/pytest_group.log 2>&1 || { tail -30 gpurun_out/pytest_group.log; exit 1; }
tail -1 gpurun_out/pytest_group.log
timeout -k 10 120 python -u tools/bench_group.py > gpurun_out/bench_group.log 2>&1 || { tail -20 gpurun_out/bench_group.log; exit 1; }
cat gpurun_out/bench_group.log
