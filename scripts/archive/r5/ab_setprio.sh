#!/bin/bash
# A/B of s_setprio 3 on the samplers' loops (csrc/build_prio/libpn2hip.so, built with
# -DPN2_FPS_PRIO=3 at its own loop placement) against the product library, in-step.
# Build the variant first: place_sa1_loop.py --flags "<Makefile FLAGS> -DPN2_FPS_PRIO=3" --out
# csrc/build_prio/sa1_pad.h, then hipcc -DPN2_FPS_PRIO=3 -DPN2_SA1_PAD=<k> -c fps.hip and link
# it with the other build/*.o into csrc/build_prio/libpn2hip.so.
set -e
P=pointcloud-segmentation-attention_amd
mkdir -p gpurun_out
cp $P/libpn2hip.so gpurun_out/lib_base.so
for r in 1 2 3; do
  for v in base prio; do
    if [ $v = prio ]; then cp $P/csrc/build_prio/libpn2hip.so $P/libpn2hip.so; else cp gpurun_out/lib_base.so $P/libpn2hip.so; fi
    timeout -k 10 120 python bench.py --steps 50 --warmup 10 --e2e-steps 0 > gpurun_out/ab_$v$r.json 2>/dev/null
    python -c "import json;d=json.load(open('gpurun_out/ab_$v$r.json'));print('$v',$r,round(d['value']),round(d['roofline']['ns_per_iteration'],1))"
  done
done
for v in base prio; do
  if [ $v = prio ]; then cp $P/csrc/build_prio/libpn2hip.so $P/libpn2hip.so; else cp gpurun_out/lib_base.so $P/libpn2hip.so; fi
  timeout -k 10 180 python bench.py --steps 30 --warmup 5 --model > gpurun_out/ab_model_$v.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/ab_model_$v.json'));print('model $v',round(d['value']))"
done
cp $P/csrc/build_prio/libpn2hip.so $P/libpn2hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q -k "fps or random_sa" --timeout 120 --timeout-method thread 2>&1 | tail -1
cp gpurun_out/lib_base.so $P/libpn2hip.so
