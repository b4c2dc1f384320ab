#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3/chain
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "fps_chain or fps_vs_oracle or golden" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  timeout -k 10 100 python3 tools/bench_chain_tail.py || exit 1
  PN2HIP_LIB=pointcloud-segmentation-attention_amd/csrc/build/libpn2hip_v_rc0.so timeout -k 10 100 python3 tools/bench_chain_tail.py || exit 1
done
for c in cfg2 cfg3; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --e2e-steps 0 > $OUT/bench_$c.json 2> $OUT/e.err || { tail -20 $OUT/e.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
done
