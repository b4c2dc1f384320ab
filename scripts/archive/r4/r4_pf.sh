#!/bin/bash
# Round 4: the grouping's vector phase gathering the next chunk before storing this one
# (PN2_SG_PREFETCH=1, main) against the round-4 vector phase (nopf).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/pf
mkdir -p $OUT
B=pointcloud-segmentation-attention_amd/csrc/build
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_fused_layers.py tests/test_gpu_a_fullsize.py -k "layers or stack_full_size or pipeline" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in main nopf; do
  l=""; [ $v != main ] && l=$B/libpn2hip_v_$v.so
  for c in cfg2 cfg3; do
    PN2HIP_LIB=$l timeout -k 10 200 python3 tools/bench_layers.py --config $c --json $OUT/layers_${c}_$v.json > $OUT/layers_${c}_$v.log 2>&1 || { tail -20 $OUT/layers_${c}_$v.log; exit 1; }
    grep -i "one launch\|ball_group_layers\|SA2..SA4" $OUT/layers_${c}_$v.log | head -3
  done
done
run() {  # name, lib, bench args
  n=$1; l=$2; shift 2
  PN2HIP_LIB=$l timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --latency-reps 5 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), d.get('verified'), round(d.get('latency_ms_per_batch',0),3))"
}
run main ""
run nopf $B/libpn2hip_v_nopf.so
run side_main "" --diag-only side --no-verify
run side_nopf $B/libpn2hip_v_nopf.so --diag-only side --no-verify
run cfg5_main "" --config cfg5
run cfg5_nopf $B/libpn2hip_v_nopf.so --config cfg5
run main2 ""
run nopf2 $B/libpn2hip_v_nopf.so
