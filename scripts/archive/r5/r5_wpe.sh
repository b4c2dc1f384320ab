#!/bin/bash
# Round 5: the fused MLP kernels with a one-wave-per-SIMD register budget (no spills) vs two.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/wpe
mkdir -p $OUT
for v in main wpe1; do
  if [ "$v" = main ]; then L=""; else L=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_v_$v.so; fi
  PN2HIP_LIB=$L timeout -k 10 200 python3 tools/bench_mlp.py > $OUT/$v.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  echo "$v $(python3 -c "
import json,sys
r=[json.loads(l) for l in open(sys.argv[1])]
print({x.get('layer','total'): x.get('us', x.get('total_us')) for x in r})" $OUT/$v.jsonl)"
done
