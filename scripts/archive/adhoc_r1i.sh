set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x -k "stack or graph or overlap or golden" > gpurun_out/pytest_r1i.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_r1i.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r1i.json 2> gpurun_out/bench_r1i.err; rc=$?; cat gpurun_out/bench_r1i.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --eager > gpurun_out/bench_eager_r1i.json 2> gpurun_out/bench_eager_r1i.err; rc=$?; cat gpurun_out/bench_eager_r1i.json; [ $rc -eq 0 ] || exit $rc
for c in cfg3 cfg5; do timeout -k 10 300 python bench.py --no-cpu-baseline --config $c > gpurun_out/bench_${c}_r1i.json 2> gpurun_out/bench_${c}_r1i.err || exit $?; cat gpurun_out/bench_${c}_r1i.json; done
