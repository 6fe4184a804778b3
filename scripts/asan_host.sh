#!/bin/bash
# Host-side AddressSanitizer run of libgpuwin's CPU-only entry points (no GPU needed; runs here).
# gw_runtime.cpp is rebuilt with ASan on the host side only (-Xarch_host), linked with the
# in-tree kernel objects into /tmp/gw_asan/libgpuwin.so, and the CPU tests that reach host
# parsers (snapshot slicing / key remap on damaged blobs, ABI exports, reference snapshot keys)
# run against it through GW_LIB_PATH with the clang ASan runtime preloaded.
set -eu
cd "$(dirname "$0")/.."
python -m flink_amd.build >/dev/null
D=/tmp/gw_asan
mkdir -p $D
ROCM=${ROCM_PATH:-/opt/rocm}
ASAN_RT=$(ls $ROCM/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
$ROCM/bin/hipcc -O1 -g -w -fPIC -std=c++17 --offload-arch=gfx950 -Xarch_host -fsanitize=address \
  -Xarch_host -fno-omit-frame-pointer -x hip -c flink_amd/csrc/gw_runtime.cpp -o $D/gw_runtime.o
OBJS=$(ls flink_amd/_build/*.o | grep -v gw_runtime.cpp.o)
$ROCM/bin/hipcc --offload-arch=gfx950 -shared -fPIC -shared-libasan -fsanitize=address -o $D/libgpuwin.so \
  $D/gw_runtime.o $OBJS -L$ROCM/lib -lrccl -Wl,-rpath,$ROCM/lib
GW_LIB_PATH=$D/libgpuwin.so LD_PRELOAD=$ASAN_RT ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 \
  python -m pytest -q -p no:cacheprovider tests/test_snapshot_fuzz.py tests/test_snapshot_slice.py tests/test_abi.py tests/test_refsnap_oracle.py "$@"
