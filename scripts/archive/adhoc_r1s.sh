set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -q -x -k "chain or stack or graph or overlap or pipelined" > gpurun_out/pytest_r1s.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r1s.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r1s.json 2> gpurun_out/bench_r1s.err; rc=$?; cut -c1-250 gpurun_out/bench_r1s.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r1s -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_r1s.log 2>&1; rc=$?; tail -1 gpurun_out/prof_r1s.log; [ $rc -eq 0 ] || exit $rc
python tools/timeline.py $(find gpurun_out/prof_r1s -name "*kernel_trace.csv" | head -1) | tail -3
