#!/bin/bash
# Round 5: split grid build, workgroups per cloud capped by kBuildMinBlocks (1 = no split).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/gb4
mkdir -p $OUT
for v in main ts main ts; do
  if [ "$v" = main ]; then L=""; else L=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_v_$v.so; fi
  PN2HIP_LIB=$L timeout -k 10 120 python3 tools/bench_gridbuild.py > $OUT/$v.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  cat $OUT/$v.json
done
