#!/bin/bash
# Round 2: phase stamps of the hot-set samplers (lab build) and the hot-loop micro-benchmark.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/stamp_fps_hot.py > gpurun_out/stamp_hot.log 2>&1 || { tail -30 gpurun_out/stamp_hot.log; exit 1; }
timeout -k 10 120 python -u tools/stamp_fps_hota.py > gpurun_out/stamp_hota.log 2>&1 || { tail -30 gpurun_out/stamp_hota.log; exit 1; }
timeout -k 10 120 python -u tools/hot_loop_bench.py > gpurun_out/hot_loop.log 2>&1 || { tail -30 gpurun_out/hot_loop.log; exit 1; }
cat gpurun_out/stamp_hot.log gpurun_out/stamp_hota.log gpurun_out/hot_loop.log
