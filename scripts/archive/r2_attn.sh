#!/bin/bash
# Attention reduction checks and micro-benchmark (tools/bench_attn.py).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "attn or attention or stack" > gpurun_out/pytest_attn.log 2>&1 || { tail -30 gpurun_out/pytest_attn.log; exit 1; }
tail -1 gpurun_out/pytest_attn.log
timeout -k 10 120 python -u tools/bench_attn.py > gpurun_out/bench_attn.log 2>&1 || { tail -20 gpurun_out/bench_attn.log; exit 1; }
cat gpurun_out/bench_attn.log
