set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x -k "ball or nn or fp or golden or stack or graph or overlap or sample_and_group or interp" > gpurun_out/pytest_nn_r1h.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_nn_r1h.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r1h.json 2> gpurun_out/bench_r1h.err; rc=$?; cat gpurun_out/bench_r1h.json; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r1h -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_r1h.log 2>&1; rc=$?; tail -2 gpurun_out/prof_r1h.log; exit $rc
