#!/bin/bash
# Round 5: attention reduction A/B (tasks in flight, blocks per CU, non-temporal K/V loads).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/attn2
mkdir -p $OUT
for v in main nt ntb8 ntb32 ntb4 ntt1 main nt; do
  if [ "$v" = main ]; then L=""; else L=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_v_$v.so; fi
  PN2HIP_LIB=$L timeout -k 10 120 python3 tools/bench_attn.py > $OUT/$v.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  cat $OUT/$v.json
done
PN2HIP_LIB=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_v_nt.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused_layers.py -x -q --timeout 200 --timeout-method thread -k "attention" > $OUT/tests_nt.log 2>&1 || { tail -30 $OUT/tests_nt.log; exit 1; }
tail -1 $OUT/tests_nt.log
