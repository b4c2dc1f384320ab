set -u
mkdir -p gpurun_out
timeout -k 10 200 python tools/stamp_fps.py > gpurun_out/stamp_r1ag.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/stamp_r1ag.log; exit $rc
