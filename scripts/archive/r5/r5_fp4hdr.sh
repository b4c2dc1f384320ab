#!/bin/bash
# Round 5: DPP wave min/max (grid.h) and the fp32 header of FP4's own grid: parity, stamps,
# standalone times, bench_side and the cfg2 pipeline.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5/fp4hdr
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_a_fullsize.py -x -q --timeout 280 --timeout-method thread \
  -k "grid or fp_ or three_nn or fps_chain or fullsize" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
PN2HIP_LIB=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_v_fpgst.so timeout -k 10 120 python3 tools/stamp_fp4.py > $OUT/stamps.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/stamps.json')); print({k: {p: v['mean'] for p, v in d[k].items() if isinstance(v, dict) and p not in ('start','end')} for k in d})"
timeout -k 10 120 python3 tools/bench_fp4.py > $OUT/fp4.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/fp4.json
timeout -k 10 120 python3 tools/bench_gridbuild.py > $OUT/gb.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/gb.json
timeout -k 10 200 python3 tools/bench_side.py --config cfg2 > $OUT/side_cfg2.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print({k: d[k]['us'] for k in d if isinstance(d[k], dict)}, d['side_sum_us'])" $OUT/side_cfg2.json
timeout -k 10 300 python3 bench.py --config cfg2 --steps 500 --warmup 50 --e2e-steps 0 --no-cpu-baseline > $OUT/b_cfg2.json 2> $OUT/b_cfg2.err || { tail -20 $OUT/b_cfg2.err; exit 1; }
echo "cfg2 500 $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],4), d.get('verified'))" $OUT/b_cfg2.json)"
