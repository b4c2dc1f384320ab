set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TUNE_ONLY=91-96 TUNE_SIZES=128:32,256:64,512:128,1024:256,2048:256,4096:512,8192:1024,16384:512 timeout -k 10 400 python tools/tune_fps.py > gpurun_out/tune_r1u.jsonl 2> gpurun_out/tune_r1u.err; rc=$?; tail -2 gpurun_out/tune_r1u.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/stamp_fps.py > gpurun_out/stamp_r1u.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/stamp_r1u.log; exit $rc
