#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3/sgab2
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_fused_layers.py > $OUT/pytest_fused.log 2>&1 || { tail -30 $OUT/pytest_fused.log; exit 1; }
tail -1 $OUT/pytest_fused.log
echo "default"; timeout -k 10 200 python3 tools/bench_layers.py --json $OUT/default.json || exit 1
for v in ${VARIANTS:-sg_s4 sg_s16 sg_s8all fp_b2k fp_b2k8 fp_b4k8}; do
  echo $v; PN2HIP_LIB=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_$v.so timeout -k 10 200 python3 tools/bench_layers.py --json $OUT/$v.json || exit 1
done
