#!/bin/bash
# Round 2: culled hot-set sampler (algo 6) -- exactness + A/B timing vs v9, then phase stamps.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/fps_hot_check.py --reps 20 --algo 0 --algos 1,0,6 > gpurun_out/cull_ab.log 2>&1 || { tail -30 gpurun_out/cull_ab.log; exit 1; }
cat gpurun_out/cull_ab.log
timeout -k 10 300 make -s -C tools/fps_lab > gpurun_out/lab_build.log 2>&1 && timeout -k 10 120 python -u tools/stamp_fps_cull.py > gpurun_out/stamp_cull.log 2>&1 || { tail -30 gpurun_out/stamp_cull.log; exit 1; }
cat gpurun_out/stamp_cull.log
