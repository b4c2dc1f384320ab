#!/bin/bash
# Round 4: buffer-set reuse ordered by GPU wait packets (--set-waits gpu: the host runs ahead)
# against the host blocking on the set's lane-end events (host, the default so far).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4/setwaits
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_a_fullsize.py -k "pipeline" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
run() {  # name, bench args
  n=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --e2e-steps 0 --latency-reps 5 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { tail -20 $OUT/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$n.json')); print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), d.get('verified'), d.get('fault_status'), round(d.get('latency_ms_per_batch',0),3), d['host'])"
}
run host
run gpu --set-waits gpu
for i in 1 2 3 4; do
  run drv_host_$i --steps 20 --warmup 5
  run drv_gpu_$i --steps 20 --warmup 5 --set-waits gpu
done
run cfg3_host --config cfg3
run cfg3_gpu --config cfg3 --set-waits gpu
run cfg5_host --config cfg5
run cfg5_gpu --config cfg5 --set-waits gpu
run host2
run gpu2 --set-waits gpu
