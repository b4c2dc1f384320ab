set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TUNE_ONLY=95-95 TUNE_SIZES=1024:256,4096:512,8192:1024 timeout -k 10 300 python tools/tune_fps.py > gpurun_out/tune_r1ae.jsonl 2> gpurun_out/tune_r1ae.err; rc=$?; [ $rc -eq 0 ] || { tail -3 gpurun_out/tune_r1ae.err; exit $rc; }
grep '"best": true' gpurun_out/tune_r1ae.jsonl | cut -c1-120
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_r1ae.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r1ae.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r1ae.json 2> gpurun_out/bench_r1ae.err; rc=$?; cut -c1-200 gpurun_out/bench_r1ae.json; exit $rc
