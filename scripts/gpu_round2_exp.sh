set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_region_compact.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_region.log 2>&1; rc=$?; tail -3 gpurun_out/pt_region.log; [ $rc -eq 0 ] || exit $rc
bash scripts/exp_bench.sh base || exit $?
