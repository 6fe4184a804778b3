set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_window_classes.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pt_wc.log 2>&1; rc=$?; tail -25 gpurun_out/pt_wc.log; [ $rc -eq 0 ] || exit $rc
