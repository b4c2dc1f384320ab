#!/bin/bash
# Round 5: FP4 kernel phase stamps (stamped build).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/fpgst
mkdir -p $OUT
PN2HIP_LIB=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_v_fpgst.so timeout -k 10 120 python3 tools/stamp_fp4.py > $OUT/stamps.json 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/stamps.json
