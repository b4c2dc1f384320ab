set -u
mkdir -p gpurun_out
timeout -k 10 300 python tools/pad_fps.py > gpurun_out/pad_fps.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/pad_fps.log; exit $rc
