#!/bin/bash
# Sampler diagnostics: phase stamps of the culled SA1 sampler and the latency floors
# (tools/ubench/pick_floor.hip); JSON in gpurun_out/r3/.
set -o pipefail
OUT=gpurun_out/r3
mkdir -p $OUT
timeout -k 10 300 python -u tools/stamp_fps_cull.py --json $OUT/sa1_cull_stamps.json > $OUT/stamp_fps_cull.log 2>&1 || { tail -30 $OUT/stamp_fps_cull.log; exit 1; }
grep -v amdgpu.ids $OUT/stamp_fps_cull.log | tail -6
timeout -k 10 120 python -u tools/ubench/run_floor.py --out $OUT/sampler_floor.json > $OUT/floor.log 2>&1 || { tail -30 $OUT/floor.log; exit 1; }
tail -1 $OUT/floor.log
