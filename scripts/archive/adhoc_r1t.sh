set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TUNE_ONLY=91-95 TUNE_SIZES=16384:512 timeout -k 10 400 python tools/tune_fps.py > gpurun_out/tune_r1al.jsonl 2> gpurun_out/tune_r1al.err; rc=$?; tail -2 gpurun_out/tune_r1al.err; [ $rc -eq 0 ] || exit $rc
exit 0
