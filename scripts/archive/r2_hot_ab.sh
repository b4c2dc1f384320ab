#!/bin/bash
# Round 2: GPU suite, then the SA1 sampler A/B (v9 vs hot-set variants) with exactness checks.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 240 python -u tools/fps_hot_check.py --reps 20 --algos 1,2,3,4,5 > gpurun_out/hot_ab.log 2>&1 || { tail -30 gpurun_out/hot_ab.log; exit 1; }
cat gpurun_out/hot_ab.log
