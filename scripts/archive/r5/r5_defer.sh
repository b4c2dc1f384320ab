#!/bin/bash
# Round 5: the SA1 sampler with the deferred cold tail (build flag PN2_CULL_DEFER) against the
# product build: index-exact on every SSG sampler case, then kernel times at the cfg2 shape.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/defer
mkdir -p $OUT
timeout -k 10 300 python3 tools/fps_hot_check.py --algos 0 --reps 20 \
  --lib defer=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_v_defer.so > $OUT/hot_check.log 2>&1 || { tail -30 $OUT/hot_check.log; exit 1; }
tail -12 $OUT/hot_check.log
# round-phase stamps of both (tools/fps_stamp; the _defer library built with -DPN2_CULL_DEFER=1)
timeout -k 10 200 python3 tools/stamp_fps_cull.py --json $OUT/stamps_main.json > $OUT/stamps_main.log 2>&1 || { tail -20 $OUT/stamps_main.log; exit 1; }
PN2_STAMP_LIB=tools/fps_stamp/libpn2fpsstamp_defer.so timeout -k 10 200 python3 tools/stamp_fps_cull.py --json $OUT/stamps_defer.json > $OUT/stamps_defer.log 2>&1 || { tail -20 $OUT/stamps_defer.log; exit 1; }
python3 -c "
import json
for n in ('main','defer'):
    d=json.load(open('$OUT/stamps_'+n+'.json')); print(n, {k: d[k] for k in ('kernel_cycles','rounds','round_cycles','hot_cycles_per_pick','stalls')}, d.get('median_round_events'))"
