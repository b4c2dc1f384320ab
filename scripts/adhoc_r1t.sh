set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TUNE_ONLY=95-95 TUNE_SIZES=1024:256,4096:512,8192:1024 timeout -k 10 400 python tools/tune_fps.py > gpurun_out/tune_r1ad.jsonl 2> gpurun_out/tune_r1ad.err; rc=$?; tail -2 gpurun_out/tune_r1ad.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/stamp_fps.py > gpurun_out/stamp_r1ad.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/stamp_r1ad.log; exit $rc
