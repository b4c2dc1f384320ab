#!/bin/bash
# Round 5: FP4 (fp_grid_fused_kernel) with 256 / 512 / 1024 threads per workgroup (-DPN2_FPG_BLOCK):
# parity of each build, then bench_fp4 and bench_side cfg2/cfg3.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/fb
mkdir -p $OUT
for v in main fb512 fb1024; do
  if [ "$v" = main ]; then L=""; else L=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_v_$v.so; fi
  PN2HIP_LIB=$L timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "fp_grid_fused or fps_chain_grid" > $OUT/tests_$v.log 2>&1 || { tail -30 $OUT/tests_$v.log; exit 1; }
  echo "$v $(tail -1 $OUT/tests_$v.log)"
  PN2HIP_LIB=$L timeout -k 10 200 python3 tools/bench_fp4.py > $OUT/fp4_$v.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  echo "$v $(cat $OUT/fp4_$v.json)"
  for c in cfg2 cfg3; do
    PN2HIP_LIB=$L timeout -k 10 200 python3 tools/bench_side.py --config $c --fp4-known-grid off > $OUT/side_${c}_$v.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k: d[k]['us'] for k in d if isinstance(d[k], dict) and 'fp' in k}, d['side_sum_us'])" $OUT/side_${c}_$v.json "$v $c"
  done
done
