#!/bin/bash
# MSG sampler stamps; cfg2 kernel trace with the lanes touched in order (queue mapping)
set -o pipefail
OUT=gpurun_out/r3
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/stamp_fps_cull.py --msg --json $OUT/msg_cull_stamps.json > $OUT/stamp_fps_cull_msg.log 2>&1 || { tail -30 $OUT/stamp_fps_cull_msg.log; exit 1; }
cat $OUT/stamp_fps_cull_msg.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_touch_cfg2 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 > $OUT/prof_touch_cfg2.log 2>&1 || { tail -20 $OUT/prof_touch_cfg2.log; exit 1; }
tail -1 $OUT/prof_touch_cfg2.log | cut -c1-200
echo ok
