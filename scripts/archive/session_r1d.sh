#!/bin/bash
# Round-1 GPU session: reference golden vectors, parity, bench (forked and single stream),
# rocprof kernel trace and PMC traffic passes. Every GPU step has its own time limit and the
# script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== golden vectors from the reference kernels"
timeout -k 10 400 python tests/golden/make_golden_gpu.py gpurun_out/golden > gpurun_out/golden_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/golden_gpu.log; [ $rc -eq 0 ] || exit $rc
cp gpurun_out/golden/*.npz tests/golden/
echo "== single-stream bench"
timeout -k 10 300 python bench.py --no-overlap --no-cpu-baseline > gpurun_out/bench_serial_r1d.json 2> gpurun_out/bench_serial_r1d.err
rc=$?; cat gpurun_out/bench_serial_r1d.json; [ $rc -eq 0 ] || exit $rc
TAG=r1d bash scripts/gpu_check.sh
