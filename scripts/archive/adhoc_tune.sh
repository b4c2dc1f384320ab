set -u
mkdir -p gpurun_out
TAG=${TAG:-x}
timeout -k 10 600 python tools/tune_fps.py > gpurun_out/tune_fps_$TAG.jsonl 2> gpurun_out/tune_fps_$TAG.err; rc=$?; tail -2 gpurun_out/tune_fps_$TAG.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/stamp_fps.py > gpurun_out/stamp_$TAG.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/stamp_$TAG.log | tail -6; exit $rc
