#!/bin/bash
# One GPU session of round-4 checks and measurements (steps as in r4_steps.sh: a step ending
# 0 or 1 lets the next one run; anything else stops here).  BATCH picks the set.
set -u
mkdir -p gpurun_out/r4
case "${BATCH:-a}" in
a)
  bash scripts/r4_steps.sh \
    "GW_SB_EXP=3 GW_SESSION_PATH=region timeout -k 10 200 python -u -m pytest -x -q -s --timeout 150 -m gpu tests/test_gpu_session_region.py -k f64 > gpurun_out/r4/sbdiag.log 2>&1; grep -E 'sb\\]|passed|failed' gpurun_out/r4/sbdiag.log | head -20" \
    "TESTS=tests/test_gpu_staged_ingest.py TEST_TIMEOUT=300 PER_TEST=200 TAG=stg NOBENCH=1 bash scripts/r4_check.sh" \
    "VARIANTS='base d3=GW_LIB_PATH=/root/repo/flink_amd/libgpuwin_d3.so d3u2=GW_LIB_PATH=/root/repo/flink_amd/libgpuwin_d3u2.so' RUNS=2 bash scripts/r4_ab.sh" \
    "GW_HOST_PROFILE=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-host-fed > gpurun_out/r4/bench_hp.json 2> gpurun_out/r4/bench_hp.err && grep 'gw host' gpurun_out/r4/bench_hp.err" \
    "timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-host-fed --no-kernel-timing > gpurun_out/r4/bench_nkt.json 2> gpurun_out/r4/bench_nkt.err && python3 scripts/json_field.py gpurun_out/r4/bench_nkt.json value" \
    "timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4/bench_hf3.json 2> gpurun_out/r4/bench_hf3.err && python3 scripts/json_field.py gpurun_out/r4/bench_hf3.json host_fed.value; python3 scripts/json_field.py gpurun_out/r4/bench_hf3.json host_fed.h2d_gbs" \
    "CONFIGS='sessions wordcount q7_first q7_maxby' bash scripts/r4_configs.sh"
  ;;
b)
  bash scripts/r4_steps.sh \
    "TESTS='tests/test_gpu_headline.py tests/test_gpu_region_narrow.py tests/test_gpu_session_region.py' TEST_TIMEOUT=500 PER_TEST=400 TAG=b NOBENCH=1 bash scripts/r4_check.sh" \
    "VARIANTS='base' RUNS=3 bash scripts/r4_ab.sh" \
    "GW_HOST_PROFILE=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-host-fed > gpurun_out/r4/bench_hp2.json 2> gpurun_out/r4/bench_hp2.err && grep 'gw host' gpurun_out/r4/bench_hp2.err" \
    "GW_HOST_PROFILE=1 timeout -k 10 200 python -u bench.py --events-per-pane 10000000 --steps 100 --warmup 20 --no-cpu-baseline --no-host-fed > gpurun_out/r4/bench_hp10.json 2> gpurun_out/r4/bench_hp10.err && grep 'gw host' gpurun_out/r4/bench_hp10.err && python3 scripts/json_field.py gpurun_out/r4/bench_hp10.json value"
  ;;
c)
  bash scripts/r4_steps.sh \
    "TESTS='tests/test_gpu_session_keyed.py tests/test_gpu_multirank.py' K='session or keyed or sentinel or colliding or punts' TEST_TIMEOUT=400 PER_TEST=150 TAG=keyed NOBENCH=1 bash scripts/r4_check.sh" \
    "CONFIGS=sessions NO_E10M=1 bash scripts/r4_configs.sh"
  ;;
d)
  bash scripts/r4_steps.sh \
    "timeout -k 10 120 python -u scripts/h2d_probe.py && HSA_ENABLE_SDMA=0 timeout -k 10 120 python -u scripts/h2d_probe.py" \
    "HSA_ENABLE_SDMA=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4/bench_hf_nosdma.json 2> gpurun_out/r4/bench_hf_nosdma.err; python3 scripts/json_field.py gpurun_out/r4/bench_hf_nosdma.json host_fed.value; python3 scripts/json_field.py gpurun_out/r4/bench_hf_nosdma.json host_fed.h2d_gbs" \
    "GW_DRAIN_DEBUG=1 GW_STAGE_STREAMS=2 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4/bench_hf_s2.json 2> gpurun_out/r4/bench_hf_s2.err; python3 scripts/json_field.py gpurun_out/r4/bench_hf_s2.json host_fed.value; python3 scripts/json_field.py gpurun_out/r4/bench_hf_s2.json host_fed.h2d_gbs; grep drain gpurun_out/r4/bench_hf_s2.err | sed -E 's/[0-9]+ rows/N rows/' | sort | uniq -c" \
    "GW_STAGE_STREAMS=4 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4/bench_hf_s4.json 2> gpurun_out/r4/bench_hf_s4.err; python3 scripts/json_field.py gpurun_out/r4/bench_hf_s4.json host_fed.value; python3 scripts/json_field.py gpurun_out/r4/bench_hf_s4.json host_fed.h2d_gbs" \
    "timeout -k 10 500 python -u scripts/configs_bench.py --only wordcount,ysb,q7,sessions,q7_first,q7_maxby > gpurun_out/r4/configs_plain.log 2> gpurun_out/r4/configs_plain.err; grep -c '^{' gpurun_out/r4/configs_plain.log"
  ;;
e)
  bash scripts/r4_steps.sh \
    "timeout -k 10 120 python -u scripts/h2d_probe.py" \
    "GW_HOST_PROFILE=1 timeout -k 10 300 python -u scripts/configs_bench.py --only q7 --no-cpu-baseline > gpurun_out/r4/q7_hp.log 2> gpurun_out/r4/q7_hp.err; grep 'gw host' gpurun_out/r4/q7_hp.err; python3 scripts/json_field.py gpurun_out/r4/q7_hp.log value" \
    "CONFIGS='q7 ysb' bash scripts/r4_configs.sh"
  ;;
f)
  export TMPDIR=/tmp
  bash scripts/r4_steps.sh \
    "timeout -k 10 300 rocprofv3 --memory-copy-trace --kernel-trace -d gpurun_out/r4/hf_trace -o run --output-format csv -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --host-fed-steps 21 > gpurun_out/r4/hf_trace.json 2> gpurun_out/r4/hf_trace.err; python3 scripts/json_field.py gpurun_out/r4/hf_trace.json host_fed.value; ls gpurun_out/r4/hf_trace; python3 scripts/copy_timeline.py gpurun_out/r4/hf_trace/run_memory_copy_trace.csv | tail -45"
  ;;
g)
  bash scripts/r4_steps.sh \
    "GW_HOST_PROFILE=1 timeout -k 10 300 python -u scripts/configs_bench.py --only q7 --no-cpu-baseline > gpurun_out/r4/q7_hp2.log 2> gpurun_out/r4/q7_hp2.err; grep 'gw host' gpurun_out/r4/q7_hp2.err; python3 scripts/json_field.py gpurun_out/r4/q7_hp2.log value" \
    "timeout -k 10 400 python -u bench.py > gpurun_out/r4/bench_final.json 2> gpurun_out/r4/bench_final.err; python3 scripts/json_field.py gpurun_out/r4/bench_final.json value; python3 scripts/json_field.py gpurun_out/r4/bench_final.json roofline.frac; python3 scripts/json_field.py gpurun_out/r4/bench_final.json host_fed.value" \
    "TAG=r4hl timeout -k 10 700 bash scripts/headline_profile.sh > gpurun_out/r4/hl_profile.log 2>&1; tail -30 gpurun_out/r4/hl_profile.log"
  ;;
h)
  bash scripts/r4_steps.sh \
    "TESTS=tests/test_gpu_staged_ingest.py TEST_TIMEOUT=300 PER_TEST=150 TAG=stg2 NOBENCH=1 bash scripts/r4_check.sh" \
    "timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r4/bench_hf5.json 2> gpurun_out/r4/bench_hf5.err; python3 scripts/json_field.py gpurun_out/r4/bench_hf5.json value; python3 scripts/json_field.py gpurun_out/r4/bench_hf5.json host_fed.value; python3 scripts/json_field.py gpurun_out/r4/bench_hf5.json host_fed.h2d_gbs"
  ;;
full)
  bash scripts/r4_steps.sh \
    "TESTS=tests TEST_TIMEOUT=1000 PER_TEST=300 TAG=full2 NOBENCH=1 bash scripts/r4_check.sh" \
    "timeout -k 10 200 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r4/smoke.log 2>&1; tail -5 gpurun_out/r4/smoke.log"
  ;;
i)
  bash scripts/r4_steps.sh \
    "TESTS=tests K='session or count' TEST_TIMEOUT=700 PER_TEST=300 TAG=sess_mirror NOBENCH=1 bash scripts/r4_check.sh" \
    "timeout -k 10 300 python -u scripts/configs_bench.py --only sessions > gpurun_out/r4/sess_mirror.log 2> gpurun_out/r4/sess_mirror.err; python3 scripts/json_field.py gpurun_out/r4/sess_mirror.log value; python3 scripts/json_field.py gpurun_out/r4/sess_mirror.log roofline.device_ms_per_step" \
    "GW_SESSION_PATH=keyed timeout -k 10 300 python -u scripts/configs_bench.py --only sessions --no-cpu-baseline > gpurun_out/r4/sess_mirror_keyed.log 2> gpurun_out/r4/sess_mirror_keyed.err; python3 scripts/json_field.py gpurun_out/r4/sess_mirror_keyed.log value" \
    "VARIANTS='base p2d=GW_LIB_PATH=/root/repo/flink_amd/libgpuwin_p2d.so' RUNS=2 bash scripts/r4_ab.sh"
  ;;
j)
  bash scripts/r4_steps.sh \
    "TESTS='tests/test_gpu_session_deferred.py' TEST_TIMEOUT=300 PER_TEST=150 TAG=sdefer NOBENCH=1 bash scripts/r4_check.sh" \
    "TESTS=tests K='session or count or multirank or staged' TEST_TIMEOUT=700 PER_TEST=300 TAG=sess_defer NOBENCH=1 bash scripts/r4_check.sh" \
    "timeout -k 10 300 python -u scripts/configs_bench.py --only sessions > gpurun_out/r4/sess_defer.log 2> gpurun_out/r4/sess_defer.err; python3 scripts/json_field.py gpurun_out/r4/sess_defer.log value; python3 scripts/json_field.py gpurun_out/r4/sess_defer.log roofline.device_ms_per_step; python3 scripts/json_field.py gpurun_out/r4/sess_defer.log ms_per_step" \
    "CONFIGS=sessions NO_E10M=1 bash scripts/r4_configs.sh"
  ;;
k)
  bash scripts/r4_steps.sh \
    "TESTS='tests/test_gpu_session_deferred.py' TEST_TIMEOUT=300 PER_TEST=150 TAG=sdefer2 NOBENCH=1 bash scripts/r4_check.sh" \
    "TESTS=tests K='session or count or multirank or staged' TEST_TIMEOUT=700 PER_TEST=300 TAG=sess_defer2 NOBENCH=1 bash scripts/r4_check.sh"
  ;;
l)
  bash scripts/r4_steps.sh \
    "VARIANTS='base rs512=GW_LIB_PATH=/root/repo/flink_amd/libgpuwin_rs512.so rs256=GW_LIB_PATH=/root/repo/flink_amd/libgpuwin_rs256.so' RUNS=2 bash scripts/r4_ab.sh"
  ;;
*)
  echo "unknown BATCH"; exit 2 ;;
esac
