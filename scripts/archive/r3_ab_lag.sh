#!/bin/bash
# A/B of a sampler variant library (csrc/build/libpn2hip_$1.so) against the product: index
# parity on the SA1 and MSG cases, then interleaved HIP-event timings; logs in gpurun_out/r3/.
set -o pipefail
OUT=gpurun_out/r3
V=${1:-lag}
mkdir -p $OUT
timeout -k 10 300 python -u tools/fps_hot_check.py --reps 20 --algos 0 --lib $V=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_$V.so > $OUT/ab_${V}_sa1.log 2>&1 || { tail -30 $OUT/ab_${V}_sa1.log; exit 1; }
tail -2 $OUT/ab_${V}_sa1.log
timeout -k 10 300 python -u tools/fps_hot_check.py --msg --shape 8,16384,512 --reps 20 --algos 0 --lib $V=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_$V.so > $OUT/ab_${V}_msg.log 2>&1 || { tail -30 $OUT/ab_${V}_msg.log; exit 1; }
tail -2 $OUT/ab_${V}_msg.log
