#!/bin/bash
# Round 5: FP4's known grid from the SA1 sampler (pn2_fps_chain_grid / pn2_fp_grid_fused_known):
# parity tests, standalone FP4 / sampler timings, bench_side with and without, pipeline A/B.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/kgrid
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 280 --timeout-method thread \
  -k "fps_chain or fp_grid_fused or three_nn_grid or pipelined or graph_replay or side_stream" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python3 tools/bench_fp4.py > $OUT/bench_fp4.json 2> $OUT/bench_fp4.err || { tail -20 $OUT/bench_fp4.err; exit 1; }
cat $OUT/bench_fp4.json
for c in cfg2 cfg3; do
  timeout -k 10 200 python3 tools/bench_side.py --config $c > $OUT/side_$c.json 2>> $OUT/side.err || { tail -20 $OUT/side.err; exit 1; }
  timeout -k 10 200 python3 tools/bench_side.py --config $c --no-sampler-grid > $OUT/side_${c}_off.json 2>> $OUT/side.err || { tail -20 $OUT/side.err; exit 1; }
  echo "$c on  $(cut -c1-400 $OUT/side_$c.json)"
  echo "$c off $(cut -c1-400 $OUT/side_${c}_off.json)"
done
for rep in 1 2; do
  for c in cfg2 cfg3; do
    for mode in on off; do
      F=""; [ $mode = off ] && F=--no-sampler-grid
      timeout -k 10 300 python3 bench.py --config $c --steps 500 --warmup 50 --e2e-steps 0 --no-cpu-baseline $F > $OUT/bench_${c}_${mode}_$rep.json 2> $OUT/bench_${c}_${mode}_$rep.err || { tail -20 $OUT/bench_${c}_${mode}_$rep.err; exit 1; }
      echo "$c $mode $rep $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('verified'))" $OUT/bench_${c}_${mode}_$rep.json)"
    done
  done
done
# the driver's default command
timeout -k 10 400 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('default', d['value'], d['ms_per_step'], d.get('verified'), d.get('e2e',{}).get('value') if isinstance(d.get('e2e'),dict) else d.get('e2e'))" $OUT/bench_default.json
