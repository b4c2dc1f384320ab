set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x -k "ball or golden or stack or graph or overlap or sample_and_group" > gpurun_out/pytest_bq_r1f.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_bq_r1f.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r1f.json 2> gpurun_out/bench_r1f.err; rc=$?; cat gpurun_out/bench_r1f.json; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r1f -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_r1f.log 2>&1; rc=$?; tail -2 gpurun_out/prof_r1f.log; exit $rc
