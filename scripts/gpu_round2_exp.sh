set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_region_compact.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_region.log 2>&1; rc=$?; tail -3 gpurun_out/pt_region.log; [ $rc -eq 0 ] || exit $rc
bash scripts/exp_bench.sh base aw6 p1w6 fsu2 || exit $?
timeout -k 10 300 python -u scripts/configs_bench.py --only ysb > gpurun_out/ysb.json 2> gpurun_out/ysb.err || { tail -20 gpurun_out/ysb.err; exit 7; }
cat gpurun_out/ysb.json
KRE="k_rgn" TAG=instmix PMC_PGRPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES" bash scripts/pmc_kernel.sh
