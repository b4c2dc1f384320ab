#!/bin/bash
# Round 5: the SA2-4 sampler chain, A/B of library variants (tools/bench_chain.py).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/chain
mkdir -p $OUT
for v in "$@"; do
  if [ "$v" = main ]; then L=""; else L=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_v_$v.so; fi
  PN2HIP_LIB=$L timeout -k 10 120 python3 tools/bench_chain.py > $OUT/chain_$v.json 2> $OUT/chain_$v.err || { tail -20 $OUT/chain_$v.err; exit 1; }
  echo "$v $(cat $OUT/chain_$v.json)"
done
