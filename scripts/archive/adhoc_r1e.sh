set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x -k "fps or golden or stack or graph or overlap" > gpurun_out/pytest_fps_r1e.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_fps_r1e.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/tune_fps.py > gpurun_out/tune_fps10.jsonl 2> gpurun_out/tune_fps10.err; rc=$?; tail -2 gpurun_out/tune_fps10.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/stamp_fps.py > gpurun_out/stamp9.log 2>&1; rc=$?; tail -8 gpurun_out/stamp9.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r1e.json 2> gpurun_out/bench_r1e.err; rc=$?; cat gpurun_out/bench_r1e.json; exit $rc
