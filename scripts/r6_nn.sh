#!/bin/bash
# Round 6: FP4 search A/B (tools/bench_nn.py, product vs VARIANTS libs, interleaved REPS times),
# then the FP parity tests against the product library.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r6/nn}
mkdir -p $OUT
for r in $(seq 1 ${REPS:-2}); do
  timeout -k 10 300 python3 tools/bench_nn.py > $OUT/nn_main_$r.json 2> $OUT/nn_main_$r.err || { tail -20 $OUT/nn_main_$r.err; exit 1; }
  for v in ${VARIANTS:-}; do
    PN2HIP_LIB=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_v_$v.so timeout -k 10 300 python3 tools/bench_nn.py > $OUT/nn_${v}_$r.json 2> $OUT/nn_${v}_$r.err || { tail -20 $OUT/nn_${v}_$r.err; exit 1; }
  done
done
for f in $OUT/nn_*.json; do echo "$f $(cat $f)"; done
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu $TESTS > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
