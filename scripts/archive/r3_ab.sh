#!/bin/bash
# A/B: the product library (schedule 0) against csrc/build/libpn2hip_<name>.so builds given as
# arguments (index parity on the SA1 and MSG cases, interleaved HIP-event timings), then the
# first-collected GPU parity file; logs in gpurun_out/r3/.
set -o pipefail
OUT=gpurun_out/r3
mkdir -p $OUT
LIBS=""
for V in "$@"; do LIBS="$LIBS --lib $V=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_$V.so"; done
TAG=${TAG:-ab}
timeout -k 10 300 python -u tools/fps_hot_check.py --reps 30 --algos 0 $LIBS > $OUT/${TAG}_sa1.log 2>&1 || { tail -30 $OUT/${TAG}_sa1.log; exit 1; }
tail -1 $OUT/${TAG}_sa1.log
timeout -k 10 300 python -u tools/fps_hot_check.py --msg --shape 8,16384,512 --reps 30 --algos 0 $LIBS > $OUT/${TAG}_msg.log 2>&1 || { tail -30 $OUT/${TAG}_msg.log; exit 1; }
tail -1 $OUT/${TAG}_msg.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_a_fullsize.py -x -q --timeout 300 --timeout-method thread > $OUT/${TAG}_fullsize.log 2>&1 || { tail -40 $OUT/${TAG}_fullsize.log; exit 1; }
tail -2 $OUT/${TAG}_fullsize.log
