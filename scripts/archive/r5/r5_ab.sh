#!/bin/bash
# Round 5: A/B of library variants (build/libpn2hip_v_<name>.so; "main" = the product build):
# tools/bench_nn.py (FP4 search / fused paths, checked equal), tools/bench_side.py cfg2.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/ab_${AB_TAG:-x}
mkdir -p $OUT
for v in "$@"; do
  if [ "$v" = main ]; then L=""; else L=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_v_$v.so; fi
  for tool in ${AB_TOOLS:-bench_nn bench_side}; do
    PN2HIP_LIB=$L timeout -k 10 200 python3 tools/$tool.py > $OUT/${tool}_$v.json 2> $OUT/${tool}_$v.err || { tail -20 $OUT/${tool}_$v.err; exit 1; }
    echo "$v $tool $(tail -1 $OUT/${tool}_$v.json | cut -c1-600)"
  done
done
