#!/bin/bash
# Round 5: the SA1 sampler with the hot wave's SIMD free of cold waves (ISO, -DPN2_CULL_ISO=1):
# wave-to-SIMD placement check, index checks + times vs the product, round stamps.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/iso
mkdir -p $OUT
: timeout -k 10 60 tools/ubench/simd_id > $OUT/simd_id.txt 2>&1 || { cat $OUT/simd_id.txt; exit 1; }
: head
timeout -k 10 300 python3 tools/fps_hot_check.py --algos 0 --reps 20 \
  --lib iso=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_v_iso.so > $OUT/hot_check.log 2>&1 || { tail -30 $OUT/hot_check.log; exit 1; }
tail -2 $OUT/hot_check.log
PN2_STAMP_LIB=tools/fps_stamp/libpn2fpsstamp_iso.so timeout -k 10 200 python3 tools/stamp_fps_cull.py --json $OUT/stamps_iso.json > $OUT/stamps_iso.log 2>&1 || { tail -20 $OUT/stamps_iso.log; exit 1; }
python3 -c "
import json
d=json.load(open('$OUT/stamps_iso.json')); print('iso', {k: d[k] for k in ('kernel_cycles','rounds','round_cycles','hot_cycles_per_pick','stalls')}, d.get('median_round_events'))"
