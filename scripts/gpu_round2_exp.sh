set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_region_compact.py tests/test_gpu_parity.py tests/test_gpu_lateness.py tests/test_gpu_restore.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pt_region.log 2>&1; rc=$?; tail -3 gpurun_out/pt_region.log; [ $rc -eq 0 ] || exit $rc
bash scripts/exp_bench.sh base || exit $?
KRE="k_rgn_apply" TAG=instmix2 PMC_PGRPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY" bash scripts/pmc_kernel.sh
