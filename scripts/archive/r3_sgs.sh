#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3/sgs
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused_layers.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
timeout -k 10 100 python3 tools/bench_layers.py || exit 1
PN2HIP_LIB=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_v_sgs.so timeout -k 10 100 python3 tools/bench_layers.py || exit 1
done
