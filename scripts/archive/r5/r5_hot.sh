#!/bin/bash
# Round 5: the hot-set chain stages -- parity of the chain, then tools/bench_chain.py A/B
# (main = the hot-set build, v9 = the v9 bodies, others = csrc/build variants), then the
# stamped build's rounds (tools/stamp_chain.py) when built.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r5/hot}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "chain or golden" > $OUT/pytest_chain.log 2>&1 || { tail -30 $OUT/pytest_chain.log; exit 1; }
tail -2 $OUT/pytest_chain.log
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_a_fullsize.py -k "stack_full_size or golden" > $OUT/pytest_full.log 2>&1 || { tail -30 $OUT/pytest_full.log; exit 1; }
tail -2 $OUT/pytest_full.log
for v in "$@"; do
  if [ "$v" = main ]; then L=""; else L=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_v_$v.so; fi
  PN2HIP_LIB=$L timeout -k 10 120 python3 tools/bench_chain.py > $OUT/chain_$v.json 2> $OUT/chain_$v.err || { tail -20 $OUT/chain_$v.err; exit 1; }
  echo "$v $(cat $OUT/chain_$v.json)"
done
H=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_v_hst.so
if [ -f $H ]; then
  PN2HIP_LIB=$H timeout -k 10 120 python3 tools/stamp_chain.py > $OUT/stamp_chain.json 2> $OUT/stamp_chain.err || { tail -20 $OUT/stamp_chain.err; exit 1; }
fi
