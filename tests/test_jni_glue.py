"""The JNI glue (integration/jni/native/gw_jni.c) compiled against a test-only JNI header and a
fake JNIEnv (tests/jni/), then called from Python: the per-key-group slicing GpuWindowOperator
.snapshotState uses, and the status -> Java exception mapping (GW_E_INVALID ->
IllegalArgumentException, other errors -> RuntimeException with gw_last_error's text)."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

from flink_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_snapshot_slice import make_blob  # noqa: E402

CLS = "Java_org_apache_flink_streaming_runtime_operators_windowing_gpu_GpuWindowOperator_"


@pytest.fixture(scope="module")
def jni(tmp_path_factory):
    N.lib()
    out = str(tmp_path_factory.mktemp("jni") / "libgw_jni_test.so")
    fl = os.path.join(ROOT, "flink_amd")
    cmd = ["gcc", "-shared", "-fPIC", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
           "-I" + os.path.join(ROOT, "tests", "jni"), "-I" + os.path.join(ROOT, "include"),
           os.path.join(ROOT, "integration", "jni", "native", "gw_jni.c"), os.path.join(ROOT, "tests", "jni", "fake_env.c"),
           "-L" + fl, "-lgpuwin", "-Wl,-rpath," + fl, "-o", out]
    subprocess.run(cmd, check=True, capture_output=True)
    L = ctypes.CDLL(out)
    p = ctypes.c_void_p
    L.fake_env.restype = p
    L.fake_bytes_new.restype = p
    L.fake_bytes_new.argtypes = [p, ctypes.c_int32]
    L.fake_bytes_len.argtypes = [p]
    L.fake_bytes_data.restype = p
    L.fake_bytes_data.argtypes = [p]
    L.fake_bytes_free.argtypes = [p]
    getattr(L, CLS + "nativeSliceKeyGroup").restype = p
    getattr(L, CLS + "nativeSliceKeyGroup").argtypes = [p, p, p, ctypes.c_int32]
    f = getattr(L, CLS + "nativeCreate")
    f.restype = ctypes.c_int64
    f.argtypes = [p, p] + [ctypes.c_int32, ctypes.c_int32] + [ctypes.c_int64] * 5 + [ctypes.c_int32] * 6 + \
        [ctypes.c_int64] * 2
    return L


def exception(L):
    c, m = ctypes.create_string_buffer(256), ctypes.create_string_buffer(1024)
    return (c.value.decode(), m.value.decode()) if L.fake_exception(c, m, 256) else None


@pytest.mark.parametrize("version,words", [(1, 4), (2, 6), (3, 10)])
def test_native_slice_key_group_matches_library(jni, version, words):
    blob, offs, ent = make_blob(version, words, 64, 95, lambda k: k % 4, seed=11)
    env = jni.fake_env()
    arr = jni.fake_bytes_new(blob, len(blob))
    for kg in range(64, 96):
        out = getattr(jni, CLS + "nativeSliceKeyGroup")(env, None, arr, kg)
        assert exception(jni) is None
        got = ctypes.string_at(jni.fake_bytes_data(out), jni.fake_bytes_len(out))
        assert got == N.snapshot_slice(blob, kg)
        i = kg - 64
        assert np.array_equal(np.frombuffer(got[112:], np.int64).reshape(-1, words), ent[offs[i]:offs[i + 1]])
        jni.fake_bytes_free(out)
    # a key group outside the blob: IllegalArgumentException, no array
    assert getattr(jni, CLS + "nativeSliceKeyGroup")(env, None, arr, 3) is None
    exc = exception(jni)
    assert exc is not None and exc[0] == "java/lang/IllegalArgumentException"
    jni.fake_bytes_free(arr)


def test_native_create_maps_status_to_java_exceptions(jni):
    env = jni.fake_env()
    create = getattr(jni, CLS + "nativeCreate")
    # tumbling size 0: invalid in Flink (IllegalArgumentException)
    assert create(env, None, 0, 0, 0, 0, 0, 0, 0, 1, 128, 1, 0, 0, 0, 1 << 16, 1 << 16) == 0
    exc = exception(jni)
    assert exc is not None and exc[0] == "java/lang/IllegalArgumentException" and "abs(offset) < size" in exc[1]


XCLS = "Java_org_apache_flink_streaming_runtime_operators_windowing_gpu_GpuKeyByExchange_"


def test_exchange_glue_maps_invalid_arguments(jni):
    """GpuKeyByExchange.nativeCreate with an impossible layout (rank outside the ranks, or
    max parallelism below the parallelism) fails before touching a device and raises
    IllegalArgumentException, as KeyGroupRangeAssignment's checks do."""
    p = ctypes.c_void_p
    create = getattr(jni, XCLS + "nativeCreate")
    create.restype = ctypes.c_int64
    create.argtypes = [p, p, ctypes.c_int32, ctypes.c_int32, p, ctypes.c_int32, ctypes.c_int32]
    env = jni.fake_env()
    idbuf = ctypes.create_string_buffer(128)
    for nranks, rank, maxp in ((2, 2, 128), (0, 0, 128), (4, 0, 2)):
        assert create(env, None, nranks, rank, ctypes.cast(idbuf, p), 0, maxp) == 0
        exc = exception(jni)
        assert exc is not None and exc[0] == "java/lang/IllegalArgumentException"


def test_exchange_set_timeout_glue(jni):
    """GpuKeyByExchange.setTimeout: a missing exchange or a negative bound is
    IllegalArgumentException (an aborted exchange's GW_E_STATE maps to IllegalStateException)."""
    p = ctypes.c_void_p
    st = getattr(jni, XCLS + "nativeSetTimeout")
    st.restype = None
    st.argtypes = [p, p, ctypes.c_int64, ctypes.c_int64]
    env = jni.fake_env()
    st(env, None, 0, 5000)
    exc = exception(jni)
    assert exc is not None and exc[0] == "java/lang/IllegalArgumentException"


def _payload_fns(jni):
    p, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    ing = getattr(jni, CLS + "nativeIngestPayload")
    ing.restype = None
    ing.argtypes = [p, p, i64, i32, p, p, p, p, p]
    dr = getattr(jni, CLS + "nativeDrainPayload")
    dr.restype = i32
    dr.argtypes = [p, p, i64, p, p, p, p, p, i32]
    adv = getattr(jni, CLS + "nativeAdvanceWatermark")
    adv.restype = i64
    adv.argtypes = [p, p, i64, i64]
    return ing, dr, adv


def test_payload_glue_null_handle(jni):
    """nativeIngestPayload on no handle: gw_ingest_payload's GW_E_INVALID -> IllegalArgumentException."""
    ing, _, _ = _payload_fns(jni)
    env = jni.fake_env()
    col = np.zeros(4, np.int64)
    ing(env, None, 0, 4, col.ctypes.data, None, col.ctypes.data, col.ctypes.data, col.ctypes.data)
    exc = exception(jni)
    assert exc is not None and exc[0] == "java/lang/IllegalArgumentException"


@pytest.mark.gpu
def test_payload_glue_positional_rows(jni):
    """GpuWindowOperator's Tuple3+ positional path through the glue on a GPU: payload = arrival
    sequence, each row's payload = the sequence of its window's first element (min over the
    window's records in arrival order), result = the window's sum."""
    ing, dr, adv = _payload_fns(jni)
    env = jni.fake_env()
    create = getattr(jni, CLS + "nativeCreate")
    h = create(env, None, 0, 0, 100, 0, 0, 0, 0, 1, 128, 1, 0, 0, N.FLAG_FIRST_ELEMENT, 1 << 16, 1 << 16)
    assert h and exception(jni) is None
    rng = np.random.default_rng(3)
    n = 5000
    keys = rng.integers(0, 50, n).astype(np.int64)
    ts = rng.integers(0, 1000, n).astype(np.int64)
    vals = rng.integers(-1000, 1000, n).astype(np.int64)
    seq = np.arange(n, dtype=np.int64)
    try:
        ing(env, None, h, n, keys.ctypes.data, None, ts.ctypes.data, vals.ctypes.data, seq.ctypes.data)
        assert exception(jni) is None
        fired = adv(env, None, h, (1 << 63) - 1)
        assert exception(jni) is None
        cols = [np.zeros(fired, np.int64) for _ in range(5)]
        got = dr(env, None, h, *[c.ctypes.data for c in cols], fired)
        assert got == fired and exception(jni) is None
    finally:
        getattr(jni, CLS + "nativeDestroy")(env, None, ctypes.c_int64(h))
    exp = {}
    for i in range(n):
        w = (int(keys[i]), int(ts[i]) // 100 * 100)
        s, first = exp.get(w, (0, i))
        exp[w] = (s + int(vals[i]), first)
    k, s, e, r, pl = cols
    assert len(k) == len(exp)
    for j in range(len(k)):
        assert (int(r[j]), int(pl[j])) == exp[(int(k[j]), int(s[j]))]
        assert e[j] == s[j] + 100


def test_java_natives_have_jni_entry_points():
    """Every `native` method GpuWindowOperator.java / GpuKeyByExchange.java declares has its
    JNI function in gw_jni.c (the names the JVM binds: Java_<class path>_<method>)."""
    import re
    jdir = os.path.join(ROOT, "integration", "jni", "java", "org", "apache", "flink", "streaming", "runtime",
                        "operators", "windowing", "gpu")
    csrc = open(os.path.join(ROOT, "integration", "jni", "native", "gw_jni.c")).read()
    for cls, macro in (("GpuWindowOperator", "CLS"), ("GpuKeyByExchange", "XCLS")):
        src = open(os.path.join(jdir, cls + ".java")).read()
        natives = set(re.findall(r"\bnative\s+[\w\[\]<>]+\s+(native\w+)\s*\(", src))
        assert natives, cls
        defined = set(re.findall(macro + r"\((native\w+)\)", csrc))
        assert natives <= defined, f"{cls}: no JNI function for {sorted(natives - defined)}"


def _key_fns(jni):
    p = ctypes.c_void_p
    ks = getattr(jni, CLS + "nativeSnapshotKeys")
    ks.restype = p
    ks.argtypes = [p, p, p]
    rm = getattr(jni, CLS + "nativeRemapKeys")
    rm.restype = None
    rm.argtypes = [p, p, p, p, p]
    jni.fake_longs_new.restype = p
    jni.fake_longs_new.argtypes = [p, ctypes.c_int32]
    jni.fake_longs_data.restype = p
    jni.fake_longs_data.argtypes = [p]
    return ks, rm


def test_key_table_glue_on_a_reference_snapshot(jni):
    """snapshotState's key table and initializeState's remap through the glue, on the
    reference's own reduce-event-time snapshot (String keys, tests/refsnap.py)."""
    from flink_amd.windowing import java_string_hash
    from tests import heapsnap, refsnap
    ks, rm = _key_fns(jni)
    ref = refsnap.parse(open(refsnap.migration_fixtures()["2.1"], "rb").read())
    blob = refsnap.to_gpuwin_blob(ref, {"key1": 0, "key2": 1}, java_string_hash, N.AGGS["sum_i32"],
                                  N.ASSIGNERS["tumbling"], 3000, 3000)
    env = jni.fake_env()
    arr = jni.fake_bytes_new(blob, len(blob))
    ids = ks(env, None, arr)
    assert exception(jni) is None and jni.fake_bytes_len(ids) == 2
    assert list(np.ctypeslib.as_array(ctypes.cast(jni.fake_longs_data(ids), ctypes.POINTER(ctypes.c_int64)),
                                      (2,))) == [0, 1]
    frm = np.array([0, 1], np.int64)
    to = np.array([41, 7], np.int64)
    fa, ta = jni.fake_longs_new(frm.ctypes.data, 2), jni.fake_longs_new(to.ctypes.data, 2)
    rm(env, None, arr, fa, ta)
    assert exception(jni) is None
    moved = ctypes.string_at(jni.fake_bytes_data(arr), len(blob))
    st = heapsnap.parse(moved, "sum_i32")[0]["state"]
    assert sorted(k for _, _, k, _, _ in st) == [7, 7, 41]
    # from[] not ascending: IllegalArgumentException
    rm(env, None, arr, ta, fa)
    exc = exception(jni)
    assert exc is not None and exc[0] == "java/lang/IllegalArgumentException"
    for a in (arr, ids, fa, ta):
        jni.fake_bytes_free(a)


@pytest.mark.gpu
def test_ingest_glue_with_key_hashes(jni):
    """nativeIngest with a keyHashes column (String keys as dictionary ids, as the Java operator
    passes them): state is filed under the key group of String.hashCode -- the snapshot blob
    carries the hashes -- and with GW_FLAG_CHECK_KEY_GROUPS a subtask rejects a foreign key."""
    from flink_amd.windowing import assign_to_key_group, java_string_hash, compute_key_group_range_for_operator_index
    from tests import heapsnap
    p, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    ing = getattr(jni, CLS + "nativeIngest")
    ing.restype = None
    ing.argtypes = [p, p, i64, i32, p, p, p, p]
    adv = getattr(jni, CLS + "nativeAdvanceWatermark")
    adv.restype = i64
    adv.argtypes = [p, p, i64, i64]
    snap = getattr(jni, CLS + "nativeSnapshot")
    snap.restype = p
    snap.argtypes = [p, p, i64, i32, i32]
    create = getattr(jni, CLS + "nativeCreate")
    env = jni.fake_env()
    words = [f"word{i}" for i in range(300)]
    lo, hi = compute_key_group_range_for_operator_index(128, 2, 1)
    mine = [w for w in words if lo <= assign_to_key_group(w, 128) <= hi]
    other = [w for w in words if not lo <= assign_to_key_group(w, 128) <= hi]
    h = create(env, None, 0, 0, 1000, 0, 0, 0, 0, 1, 128, 2, 1, 0, N.FLAG_CHECK_KEY_GROUPS, 1 << 12, 1 << 16)
    assert h and exception(jni) is None
    try:
        n = 4000
        rng = np.random.default_rng(8)
        sel = rng.integers(0, len(mine), n)
        keys = sel.astype(np.int64)
        hashes = np.array([java_string_hash(mine[i]) for i in sel], np.int32)
        ts = rng.integers(0, 1500, n).astype(np.int64)
        vals = rng.integers(-50, 50, n).astype(np.int64)
        ing(env, None, h, n, keys.ctypes.data, hashes.ctypes.data, ts.ctypes.data, vals.ctypes.data)
        assert exception(jni) is None
        blob_arr = snap(env, None, h, lo, hi)
        assert exception(jni) is None
        blob = ctypes.string_at(jni.fake_bytes_data(blob_arr), jni.fake_bytes_len(blob_arr))
        jni.fake_bytes_free(blob_arr)
        parsed = heapsnap.parse(blob, "sum_i64")
        seen = 0
        for kg, sec in parsed.items():
            for s, e, k, acc, kh in sec["state"]:
                assert kh == java_string_hash(mine[k]) and assign_to_key_group(mine[k], 128) == kg
                seen += 1
        assert seen > 0
        # a key of the other subtask: the batch fails (IllegalArgumentException text of the reference)
        bad = np.array([10 ** 6], np.int64)  # a new id (id 0 already has its own hash)
        bh = np.array([java_string_hash(other[0])], np.int32)
        ing(env, None, h, 1, bad.ctypes.data, bh.ctypes.data, ts.ctypes.data, vals.ctypes.data)
        exc = exception(jni)
        assert exc is not None and "is not in KeyGroupRange" in exc[1]
    finally:
        getattr(jni, CLS + "nativeDestroy")(env, None, ctypes.c_int64(h))


def _fe_blob(entries, agg="sum_i64", kg=0):
    """A first-element blob (flags bit 1): entries (start, end, key, acc, payload), no timers."""
    import struct
    pay = struct.pack(">i", len(entries))
    for s, e, k, a, p in entries:
        pay += struct.pack(">qqqqq", s, e, k, a, p)
    pay += struct.pack(">ii", 0, 0)
    hdr = struct.pack("<4sIii5q4i3q", b"GWS1", 4, N.AGGS[agg], N.ASSIGNERS["tumbling"], 100, 100, 0, 0, 2,
                      128, kg, kg, 0, 0, 0, len(pay))
    return hdr + struct.pack("<2q", 0, len(pay)) + pay


def test_payload_table_glue(jni):
    """snapshotState's first-element table and initializeState's payload remap through the glue
    (gw_snapshot_payloads / gw_snapshot_remap_payloads)."""
    p = ctypes.c_void_p
    sp = getattr(jni, CLS + "nativeSnapshotPayloads")
    sp.restype = p
    sp.argtypes = [p, p, p, p]
    rp = getattr(jni, CLS + "nativeRemapPayloads")
    rp.restype = None
    rp.argtypes = [p, p, p, p, p]
    _key_fns(jni)
    blob = _fe_blob([(0, 100, 5, 7, 41), (100, 200, 5, 9, 12), (0, 100, 6, 1, 41)])
    env = jni.fake_env()
    arr = jni.fake_bytes_new(blob, len(blob))
    mx = jni.fake_longs_new(np.zeros(1, np.int64).ctypes.data, 1)
    out = sp(env, None, arr, mx)
    assert exception(jni) is None and jni.fake_bytes_len(out) == 2
    L = lambda a, n: list(np.ctypeslib.as_array(ctypes.cast(jni.fake_longs_data(a), ctypes.POINTER(ctypes.c_int64)), (n,)))
    assert L(out, 2) == [12, 41] and L(mx, 1) == [200]
    frm, to = np.array([12, 41], np.int64), np.array([3, 4], np.int64)
    fa, ta = jni.fake_longs_new(frm.ctypes.data, 2), jni.fake_longs_new(to.ctypes.data, 2)
    rp(env, None, arr, fa, ta)
    assert exception(jni) is None
    moved = ctypes.string_at(jni.fake_bytes_data(arr), len(blob))
    assert moved == _fe_blob([(0, 100, 5, 7, 4), (100, 200, 5, 9, 3), (0, 100, 6, 1, 4)])
    # a blob without payloads: IllegalArgumentException
    plain = bytearray(blob)
    plain[48:56] = (0).to_bytes(8, "little")
    parr = jni.fake_bytes_new(bytes(plain), len(plain))
    assert sp(env, None, parr, mx) is None
    assert exception(jni)[0] == "java/lang/IllegalArgumentException"
    for a in (arr, out, mx, fa, ta, parr):
        jni.fake_bytes_free(a)


def test_native_stagger_offset(jni):
    """GpuWindowOperator's staggered handle: nativeStaggerOffset at the first element's processing
    time (TumblingEventTimeWindowsTest.testWindowAssignmentWithStagger: NATURAL, size 5000, 150 ->
    windows from 150); a bad argument is an IllegalArgumentException."""
    f = getattr(jni, CLS + "nativeStaggerOffset")
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_int64,
                  ctypes.c_int64]
    env = jni.fake_env()
    assert f(env, None, 2, 150, 0.0, 5000, 0) == 150 and exception(jni) is None      # NATURAL
    assert f(env, None, 1, 0, 0.5, 5000, 4000) == 1500 and exception(jni) is None    # RANDOM
    assert f(env, None, 0, 999, 0.7, 5000, -100) == -100 and exception(jni) is None  # ALIGNED
    f(env, None, 1, 0, 1.5, 5000, 0)
    exc = exception(jni)
    assert exc is not None and exc[0] == "java/lang/IllegalArgumentException"
