#!/bin/bash
# Round 6: tools/bench_side.py (each task of the step alone) for the product and the
# whole-library A/B builds in build/ab_<name> (AB="name ..."), CONFIG, interleaved REPS times.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6/side}
mkdir -p $OUT
D=pointcloud-segmentation-attention_amd/csrc/build
for r in $(seq 1 ${REPS:-1}); do
  for v in main ${AB:-}; do
    E=""
    [ "$v" != main ] && E="PN2HIP_LIB=$D/ab_$v/libpn2hip.so PN2TORCH_LIB=$D/ab_$v/libpn2torch.so"
    env $E timeout -k 10 300 python3 tools/bench_side.py --config ${CONFIG:-cfg2} --json $OUT/side_${CONFIG:-cfg2}_${v}_$r.json > $OUT/side_${v}_$r.log 2>&1 || { tail -20 $OUT/side_${v}_$r.log; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/side_${CONFIG:-cfg2}_${v}_$r.json')); print('$v', {k: v['us'] for k, v in d.items() if isinstance(v, dict)}, d['side_sum_us'])"
  done
done
