"""CPU-side checks of the C ABI: libgpuwin.so loads, exports every entry point that
include/gpuwin.h declares, and its stateless key-group helpers are bit-exact with the
oracle and the reference's key-group golden vector.  No compute calls (no GPU here)."""
import ctypes
import os
import re

import numpy as np
import pytest

from flink_amd import _native as N
from flink_amd import windowing as W
from tests.harness import load_golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "gpuwin.h")).read()
    return sorted(set(re.findall(r"\b(gw_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = N.lib()
    decl = declared_symbols()
    assert len(decl) >= 25
    missing = [s for s in decl if not hasattr(L, s)]
    assert missing == []
    assert sorted(N.EXPORTS) == decl


def test_abi_version():
    assert N.lib().gw_abi_version() == 3


def test_config_struct_layout_matches_header():
    # gw_config: 2x int32, 5x int64, 6x int32, 2x int64 with natural alignment
    assert ctypes.sizeof(N.GwConfig) == 8 + 40 + 24 + 16
    assert N.GwConfig.agg.offset == 48
    assert N.GwConfig.capacity_hint.offset == 72


def test_key_group_kat_through_library():
    g = load_golden("key_groups.json")
    for key, group in g["string_keys"]:
        assert W.assign_to_key_group(key, g["max_parallelism"]) == group


def test_murmur_and_long_hash_match_oracle(oracle_lib):
    L, O = N.lib(), oracle_lib.lib()
    rng = np.random.default_rng(3)
    for v in rng.integers(-(1 << 31), (1 << 31) - 1, 2000).tolist() + [0, -1, 1, -(1 << 31), (1 << 31) - 1]:
        assert L.gw_murmur_hash(v) == O.wo_murmur_hash(v)
    for v in rng.integers(-(1 << 63), (1 << 63) - 1, 2000, dtype=np.int64).tolist() + [-(1 << 63), (1 << 63) - 1]:
        assert L.gw_java_long_hash(v) == O.wo_long_hash(v)
    for p in [1, 2, 4, 8]:
        for kg in range(128):
            assert L.gw_operator_for_key_group(128, p, kg) == O.wo_operator_index_for_key_group(128, p, kg)
    for p in [1, 3, 100, 1000, 30000]:
        assert L.gw_default_max_parallelism(p) == O.wo_default_max_parallelism(p)


def test_java_string_hash():
    assert W.java_string_hash("") == 0
    assert W.java_string_hash("a") == 97
    assert W.java_string_hash("key1") == 3288498
    assert W.java_string_hash("polygenelubricants") == -(1 << 31)


def test_invalid_configs_raise_like_the_reference():
    with pytest.raises(ValueError):
        W.TumblingEventTimeWindows.of(1000, 1000)
    with pytest.raises(ValueError):
        W.SlidingEventTimeWindows.of(1000, 100, -100)
    with pytest.raises(ValueError):
        W.EventTimeSessionWindows.with_gap(0)
    with pytest.raises(ValueError):
        W.GpuWindowOperator(W.TumblingEventTimeWindows.of(10), "sum_i64", allowed_lateness=-1)


def test_create_fails_cleanly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    op = W.GpuWindowOperator(W.TumblingEventTimeWindows.of(1000), "sum_i64")
    with pytest.raises(N.GpuWinError):
        op.open()


def test_missing_library_fails_loudly(tmp_path):
    """No CPU fallback: with the library absent, the product path raises NativeLibraryError
    at the first use (a fresh process, so this one's loaded library is not involved)."""
    import subprocess
    import sys
    code = ("from flink_amd import _native as N\n"
            "from flink_amd import windowing as W\n"
            "try:\n    N.lib()\nexcept N.NativeLibraryError as e:\n    print('raised', 'no CPU fallback' in str(e))\n")
    env = dict(os.environ, GW_LIB_PATH=str(tmp_path / "libgpuwin.so"))
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "raised True"


def test_grouping_sort_refuses_counts_beyond_its_prefix_field():
    """gw_sort.hip keeps a tile's per-digit prefix in 30 bits of its look-back word: the sort
    returns hipErrorInvalidValue for n >= 2^30 before any launch (host-side guard; the session,
    count-window and re-fire callers split or refuse such batches), instead of spilling the
    prefix into the flag bits."""
    L = N.lib()
    p = ctypes.c_void_p
    for sym in ("_ZN2gw14sort_pairs_u32EPjS0_S0_S0_liiPvP12ihipStream_tPib",
                "_ZN2gw14sort_pairs_u64EPmPjS0_S1_liiPvP12ihipStream_tPib"):
        f = getattr(L, sym)
        f.restype = ctypes.c_int
        f.argtypes = [p, p, p, p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, p, p, ctypes.POINTER(ctypes.c_int),
                      ctypes.c_bool]
        alt = ctypes.c_int(-1)
        for n in (1 << 30, (1 << 31) - 1, 1 << 40):
            assert f(None, None, None, None, n, 0, 26, None, None, ctypes.byref(alt), False) == 1  # hipErrorInvalidValue
            assert alt.value == 0
