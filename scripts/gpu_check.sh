#!/bin/bash
# One GPU-box session: parity tests, a short bench, a rocprofv3 kernel-trace summary.
# Each GPU step has its own time limit; a crash / timeout (exit code other than 0 or 1)
# ends the script before anything else touches the GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-r1}
export TMPDIR=/tmp
rc_ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }

echo "== build check (prebuilt .so must be present)"; ls -la pointcloud-segmentation-attention_amd/*.so oracle/*.so oracle/_ref/*.so || exit 3

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "== pytest -m gpu"
  timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -rf --timeout 600 ${PYTEST_ARGS:-} > $OUT/pytest_gpu_$TAG.log 2>&1
  rc=$?; tail -30 $OUT/pytest_gpu_$TAG.log; echo "pytest rc=$rc"
  rc_ok $rc || exit $rc
fi

if [ "${SKIP_BENCH:-0}" != "1" ]; then
  echo "== bench"
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:-} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
  rc=$?; cat $OUT/bench_$TAG.json; tail -5 $OUT/bench_$TAG.err; echo "bench rc=$rc"
  [ $rc -eq 0 ] || exit $rc
fi

if [ "${SKIP_PROF:-0}" != "1" ]; then
  echo "== rocprofv3 kernel trace"
  timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 ${BENCH_ARGS:-} > $OUT/prof_$TAG.log 2>&1
  rc=$?; tail -5 $OUT/prof_$TAG.log; echo "rocprof rc=$rc"
  find $OUT/prof_$TAG -name "*stats*" | head
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${SKIP_PMC:-0}" != "1" ]; then
  # HBM traffic counters, one counter per pass (FETCH_SIZE and WRITE_SIZE do not fit one
  # TCC pass on gfx950), kernel trace only -- never combined with runtime/sys tracing.
  for C in FETCH_SIZE WRITE_SIZE; do
    echo "== rocprofv3 --pmc $C"
    timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_${C}_$TAG -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-steps 0 ${BENCH_ARGS:-} > $OUT/pmc_${C}_$TAG.log 2>&1
    rc=$?; tail -3 $OUT/pmc_${C}_$TAG.log; echo "pmc $C rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
  python3 tools/pmc_summary.py $OUT/pmc_FETCH_SIZE_$TAG $OUT/pmc_WRITE_SIZE_$TAG > $OUT/pmc_traffic_$TAG.json
  cat $OUT/pmc_traffic_$TAG.json | head -40
fi
echo "== done"
