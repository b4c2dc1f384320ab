#!/bin/bash
# Round 4: the SA1 sampler's round structure (stamped lab build, tools/fps_stamp): phase
# cycles and per-round cold-wave lag behind the hot wave's end.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/stamps
mkdir -p $OUT
timeout -k 10 200 python3 tools/stamp_fps_cull.py --json $OUT/sa1_cull_stamps.json > $OUT/stamps.log 2>&1 || { tail -20 $OUT/stamps.log; exit 1; }
tail -5 $OUT/stamps.log
timeout -k 10 200 python3 tools/fps_stamp/lag_events.py > $OUT/lag.log 2>&1 || { tail -20 $OUT/lag.log; exit 1; }
tail -3 $OUT/lag.log
