set -u
mkdir -p gpurun_out
timeout -k 10 400 python tests/golden/make_golden_gpu.py gpurun_out/golden > gpurun_out/golden_gpu_r1q.log 2>&1; rc=$?; tail -3 gpurun_out/golden_gpu_r1q.log; [ $rc -eq 0 ] || exit $rc
cp gpurun_out/golden/*.npz tests/golden/
timeout -k 10 400 python -m pytest tests -m gpu -q -x -k "knn or select or attention or golden or sample_and_group" > gpurun_out/pytest_r1q.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_r1q.log; exit $rc
