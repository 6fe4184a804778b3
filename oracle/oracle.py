"""ctypes wrapper of the CPU restatement oracle — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module; it is the checker, never the thing measured or shipped.  The product
path (flink_amd/, libgpuwin.so) does not import it and fails loudly without its
own HIP extension.

The oracle restates Flink's WindowOperator record by record (see
oracle/flink_oracle.c for per-function reference citations) and is pinned by the
reference's own golden vectors in tests/golden/ (tests/test_oracle_golden.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libflink_oracle.so")

INT64_MIN = -(1 << 63)
INT64_MAX = (1 << 63) - 1

ASSIGNERS = {"tumbling": 0, "sliding": 1, "session": 2, "count_tumbling": 3, "count_sliding": 4}
TRIGGERS = {"event_time": 0, "purging_event_time": 1}
AGGS = {
    "count": 0, "sum_i64": 1, "sum_f64": 2, "min_i64": 3, "max_i64": 4,
    "min_f64": 5, "max_f64": 6, "avg_i64": 7, "avg_f64": 8, "sum_i32": 9,
}
DOUBLE_RESULT = {"sum_f64", "min_f64", "max_f64", "avg_i64", "avg_f64"}
DOUBLE_INPUT = {"sum_f64", "min_f64", "max_f64", "avg_f64"}


class GwConfig(ctypes.Structure):
    """Mirror of gw_config in include/gpuwin.h."""
    _fields_ = [
        ("assigner", ctypes.c_int32), ("trigger", ctypes.c_int32),
        ("size", ctypes.c_int64), ("slide", ctypes.c_int64), ("offset", ctypes.c_int64),
        ("gap", ctypes.c_int64), ("allowed_lateness", ctypes.c_int64),
        ("agg", ctypes.c_int32), ("max_parallelism", ctypes.c_int32),
        ("parallelism", ctypes.c_int32), ("operator_index", ctypes.c_int32),
        ("device", ctypes.c_int32), ("flags", ctypes.c_int32),
        ("capacity_hint", ctypes.c_int64), ("max_batch", ctypes.c_int64),
    ]


def make_config(assigner="tumbling", size=0, slide=0, offset=0, gap=0, lateness=0,
                agg="sum_i64", trigger="event_time", max_parallelism=128, parallelism=1,
                operator_index=0, device=0, flags=0, capacity_hint=0, max_batch=0) -> GwConfig:
    c = GwConfig()
    c.assigner = ASSIGNERS[assigner]
    c.trigger = TRIGGERS[trigger]
    c.size, c.slide, c.offset, c.gap = size, slide, offset, gap
    c.allowed_lateness = lateness
    c.agg = AGGS[agg]
    c.max_parallelism, c.parallelism, c.operator_index = max_parallelism, parallelism, operator_index
    c.device, c.flags, c.capacity_hint, c.max_batch = device, flags, capacity_hint, max_batch
    return c


class GwRecordLayout(ctypes.Structure):
    """include/gpuwin.h gw_record_layout."""
    _fields_ = [("nfields", ctypes.c_int32), ("key_field", ctypes.c_int32), ("value_field", ctypes.c_int32),
                ("types", ctypes.c_char * 8)]


class GwDecodeResult(ctypes.Structure):
    _fields_ = [("records", ctypes.c_int64), ("watermarks", ctypes.c_int64), ("consumed", ctypes.c_int64),
                ("skipped", ctypes.c_int64)]


def decode_stream(data: bytes, types: str, key_field: int, value_field: int = -1):
    """Sequential decode of one channel's serialized elements (wo_decode_stream).
    Returns (rc, key, ts, value_bits, wm_pos, wm_val, result)."""
    lay = GwRecordLayout()
    lay.nfields, lay.key_field, lay.value_field = len(types), key_field, value_field
    lay.types = types.encode()
    n = len(data)
    cap = n // 6 + 1
    key, ts, val = (np.zeros(cap, dtype=np.int64) for _ in range(3))
    wp, wv = np.zeros(cap, dtype=np.int64), np.zeros(cap, dtype=np.int64)
    res = GwDecodeResult()
    buf = np.frombuffer(data, dtype=np.uint8) if n else np.zeros(1, dtype=np.uint8)
    rc = lib().wo_decode_stream(buf.ctypes.data, n, ctypes.byref(lay), key.ctypes.data, ts.ctypes.data,
                                val.ctypes.data, cap, wp.ctypes.data, wv.ctypes.data, cap, ctypes.byref(res))
    r, w = res.records, res.watermarks
    return rc, key[:r], ts[:r], val[:r], wp[:w], wv[:w], res


def build(force: bool = False) -> str:
    deps = [os.path.join(_HERE, f) for f in ("flink_oracle.c", "flink_oracle.h", "Makefile")]
    deps.append(os.path.join(os.path.dirname(_HERE), "include", "gpuwin.h"))
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < max(map(os.path.getmtime, deps)):
        subprocess.run(["make", "-C", _HERE, "-s"], check=True)
    return _LIB_PATH


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        i32, i64, p = ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p
        P64 = ctypes.POINTER(ctypes.c_int64)
        for name, res, args in [
            ("wo_murmur_hash", i32, [i32]), ("wo_bit_mix", i32, [i32]),
            ("wo_long_to_int_with_bit_mixing", i32, [i64]), ("wo_long_hash", i32, [i64]),
            ("wo_string_hash", i32, [p, i64]), ("wo_assign_to_key_group", i32, [i32, i32]),
            ("wo_operator_index_for_key_group", i32, [i32, i32, i32]),
            ("wo_key_group_range", None, [i32, i32, i32, ctypes.POINTER(i32), ctypes.POINTER(i32)]),
            ("wo_default_max_parallelism", i32, [i32]),
            ("wo_window_start_with_offset", i64, [i64, i64, i64]),
            ("wo_assign_windows", ctypes.c_int, [ctypes.POINTER(GwConfig), i64, P64, P64, ctypes.c_int]),
            ("wo_merge_windows", ctypes.c_int, [ctypes.c_int, P64, P64, ctypes.POINTER(i32), P64, P64]),
            ("wo_validate", ctypes.c_int, [ctypes.POINTER(GwConfig)]),
            ("wo_create", p, [ctypes.POINTER(GwConfig)]), ("wo_destroy", None, [p]),
            ("wo_process_element", ctypes.c_int, [p, i64, i64, i64]),
            ("wo_process_batch", ctypes.c_int, [p, i64, p, p, p]),
            ("wo_process_watermark", ctypes.c_int, [p, i64]),
            ("wo_set_key_hashes", ctypes.c_int, [p, i64, p, p]),
            ("wo_output_count", i64, [p]), ("wo_drain", i64, [p, p, p, p, p, i64]),
            ("wo_drain_seq", i64, [p, p, p, p, p, p, i64]), ("wo_set_arrival", None, [p, i64]),
            ("wo_late_dropped", i64, [p]), ("wo_late_output_count", i64, [p]),
            ("wo_drain_late", i64, [p, p, p, p, i64]), ("wo_current_watermark", i64, [p]),
            ("wo_state_entries", i64, [p]), ("wo_timer_count", i64, [p]),
            ("wo_session_merges", i64, [p]), ("wo_last_error", ctypes.c_char_p, [p]),
            ("wo_decode_stream", ctypes.c_int, [p, i64, ctypes.POINTER(GwRecordLayout), p, p, p, i64, p, p, i64,
                                                 ctypes.POINTER(GwDecodeResult)]),
            ("wo_run_parallel", i64, [ctypes.POINTER(GwConfig), ctypes.c_int, i64, p, p, p, p, p,
                                       P64, ctypes.POINTER(ctypes.c_double)]),
            ("wo_run_parallel_stream", i64, [ctypes.POINTER(GwConfig), ctypes.c_int, i64, p, p, p, p, p,
                                              P64, ctypes.POINTER(ctypes.c_double)]),
            ("wo_run_parallel_rows", i64, [ctypes.POINTER(GwConfig), ctypes.c_int, i64, p, p, p, p, p, i64,
                                            p, p, p, p, p, ctypes.POINTER(ctypes.c_double)]),
            ("wo_snapshot", i64, [p, i32, i32, p, i64]), ("wo_restore", ctypes.c_int, [p, p, i64]),
            ("wo_acc_bytes", ctypes.c_int, [ctypes.c_int]),
            ("wo_mws_create", p, []), ("wo_mws_destroy", None, [p]),
            ("wo_mws_add", ctypes.c_int, [p, i64, i64, P64, P64]),
            ("wo_mws_state_window", ctypes.c_int, [p, i64, i64, P64]),
            ("wo_mws_retire", ctypes.c_int, [p, i64, i64]),
            ("wo_mws_put", None, [p, i64, i64, i64, i64]),
            ("wo_mws_list", ctypes.c_int, [p, P64, ctypes.c_int]),
            ("wo_run_parallel_wm", i64, [ctypes.POINTER(GwConfig), ctypes.c_int, i64, p, p, p, p, p, p, p,
                                          ctypes.POINTER(ctypes.c_double)]),
        ]:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def java_string_hash(s: str) -> int:
    """JDK String.hashCode over UTF-16 code units (via the oracle)."""
    units = np.frombuffer(s.encode("utf-16-le"), dtype=np.uint16).copy()
    return lib().wo_string_hash(units.ctypes.data, len(units))


def _p(a: np.ndarray):
    return a.ctypes.data if a is not None else None


class OracleError(RuntimeError):
    pass


class MergingWindowSet:
    """The oracle's MergingWindowSet of session windows (MergingWindowSet.java:77-224), driven the
    way MergingWindowSetTest drives the reference's (test hook)."""

    def __init__(self, restored=()):
        self._h = lib().wo_mws_create()
        for (s, e), (ss, se) in restored:  # the constructor reading its ListState
            lib().wo_mws_put(self._h, s, e, ss, se)

    def close(self):
        if self._h:
            lib().wo_mws_destroy(self._h)
            self._h = None

    def add_window(self, w):
        """-> (result window, merge) with merge None when the MergeFunction did not run, else
        {"target": w, "state_window": w, "sources": [w], "merged_state_windows": [w]}."""
        res = (ctypes.c_int64 * 2)()
        info = (ctypes.c_int64 * 600)()
        rc = lib().wo_mws_add(self._h, w[0], w[1], res, info)
        if rc:
            raise OracleError(f"addWindow failed: {rc}")
        result = (res[0], res[1])
        if not info[0]:
            return result, None
        q = 5
        ns = info[q]; q += 1
        src = [(info[q + 2 * i], info[q + 2 * i + 1]) for i in range(ns)]; q += 2 * ns
        nm = info[q]; q += 1
        msw = [(info[q + 2 * i], info[q + 2 * i + 1]) for i in range(nm)]
        return result, {"target": (info[1], info[2]), "state_window": (info[3], info[4]), "sources": src,
                        "merged_state_windows": msw}

    def state_window(self, w):
        out = (ctypes.c_int64 * 2)()
        return (out[0], out[1]) if lib().wo_mws_state_window(self._h, w[0], w[1], out) else None

    def retire(self, w):
        if lib().wo_mws_retire(self._h, w[0], w[1]):
            raise OracleError(f"Window {w} is not in in-flight window set.")

    def persisted(self):
        out = (ctypes.c_int64 * 4096)()
        n = lib().wo_mws_list(self._h, out, 1024)
        return sorted(((out[4 * i], out[4 * i + 1]), (out[4 * i + 2], out[4 * i + 3])) for i in range(n))


class OracleOperator:
    """One reference WindowOperator instance (one keyed subtask)."""

    def __init__(self, cfg: GwConfig):
        self.cfg = cfg
        self._h = lib().wo_create(ctypes.byref(cfg))
        if not self._h:
            raise OracleError("invalid window operator configuration")

    def close(self):
        if self._h:
            lib().wo_destroy(self._h)
            self._h = None

    __del__ = close

    def _check(self, rc):
        if rc != 0:
            raise OracleError(f"oracle error {rc}: {lib().wo_last_error(self._h).decode()}")

    def process_element(self, key: int, ts: int, value_bits: int = 0):
        self._check(lib().wo_process_element(self._h, key, ts, value_bits))

    def process_batch(self, key: np.ndarray, ts: np.ndarray, value_bits: np.ndarray | None):
        key = np.ascontiguousarray(key, dtype=np.int64)
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        vb = None if value_bits is None else np.ascontiguousarray(value_bits).view(np.int64)
        self._check(lib().wo_process_batch(self._h, len(key), _p(key), _p(ts), _p(vb)))

    def process_watermark(self, wm: int):
        self._check(lib().wo_process_watermark(self._h, wm))

    def set_key_hashes(self, key: np.ndarray, hashes: np.ndarray):
        """key.hashCode() of caller key ids (String / Integer / ... keys): key groups and the
        snapshot's key hashes follow it."""
        key = np.ascontiguousarray(key, dtype=np.int64)
        hashes = np.ascontiguousarray(hashes, dtype=np.int32)
        self._check(lib().wo_set_key_hashes(self._h, len(key), _p(key), _p(hashes)))

    def drain(self):
        n = lib().wo_output_count(self._h)
        k = np.empty(n, np.int64); s = np.empty(n, np.int64)
        e = np.empty(n, np.int64); r = np.empty(n, np.int64)
        got = lib().wo_drain(self._h, _p(k), _p(s), _p(e), _p(r), n)
        assert got == n
        return k, s, e, r

    def set_arrival(self, next_seq: int):
        lib().wo_set_arrival(self._h, next_seq)

    def drain_seq(self):
        """drain() plus each row's element: its arrival number over every processed record
        (minBy / maxBy with GW_FLAG_BY_FIELD; ComparableAggregator.java:88-95)."""
        n = lib().wo_output_count(self._h)
        k, s, e, r, q = (np.empty(n, np.int64) for _ in range(5))
        got = lib().wo_drain_seq(self._h, _p(k), _p(s), _p(e), _p(r), _p(q), n)
        assert got == n
        return k, s, e, r, q

    def snapshot(self, key_group_range=None) -> bytes:
        """Keyed state of key groups [lo, hi] (default all) in the heap backend's per-key-group
        layout (blob version 4; oracle/flink_oracle.c wo_snapshot)."""
        lo, hi = key_group_range if key_group_range is not None else (0, (self.cfg.max_parallelism or 128) - 1)
        n = lib().wo_snapshot(self._h, lo, hi, None, 0)
        if n < 0:
            raise OracleError(f"snapshot failed: {n}")
        buf = ctypes.create_string_buffer(n)
        m = lib().wo_snapshot(self._h, lo, hi, buf, n)
        assert m == n
        return buf.raw[:n]

    def restore(self, blobs):
        if isinstance(blobs, (bytes, bytearray)):
            blobs = [blobs]
        for b in blobs:
            self._check(lib().wo_restore(self._h, bytes(b), len(b)))

    @property
    def late_dropped(self) -> int:
        return lib().wo_late_dropped(self._h)

    def drain_late(self):
        """The late-data side output so far: (key, ts, value_bits) columns."""
        n = lib().wo_late_output_count(self._h)
        k, t, v = (np.empty(n, np.int64) for _ in range(3))
        got = lib().wo_drain_late(self._h, _p(k), _p(t), _p(v), n)
        assert got == n
        return k, t, v

    @property
    def state_entries(self) -> int:
        return lib().wo_state_entries(self._h)

    @property
    def session_merges(self) -> int:
        return lib().wo_session_merges(self._h)


def run_parallel(cfg: GwConfig, threads: int, batch_len, wm, key, ts, value_bits, final_watermark=True):
    """Multi-threaded CPU baseline (one operator per simulated Flink subtask); without
    final_watermark only the stream's own watermarks run (no MAX_WATERMARK at the end)."""
    batch_len = np.ascontiguousarray(batch_len, dtype=np.int64)
    wm = np.ascontiguousarray(wm, dtype=np.int64)
    key = np.ascontiguousarray(key, dtype=np.int64)
    ts = np.ascontiguousarray(ts, dtype=np.int64)
    vb = None if value_bits is None else np.ascontiguousarray(value_bits).view(np.int64)
    cs = ctypes.c_int64(0)
    sec = ctypes.c_double(0)
    fn = lib().wo_run_parallel if final_watermark else lib().wo_run_parallel_stream
    rows = fn(ctypes.byref(cfg), threads, len(batch_len), _p(batch_len), _p(wm), _p(key), _p(ts), _p(vb),
              ctypes.byref(cs), ctypes.byref(sec))
    if rows < 0:
        raise OracleError(f"parallel oracle failed: {rows}")
    return rows, cs.value, sec.value


def rows_hash_sum(k, s, e, r) -> int:
    """The oracle's order-independent row checksum (wo_run_parallel): the sum over rows of
    (key * 0x9e3779b97f4a7c15) ^ (start * 31) ^ (end * 17) ^ result, mod 2^64, as int64."""
    k, s, e, r = (np.ascontiguousarray(c).view(np.uint64) for c in (k, s, e, r))
    with np.errstate(over="ignore"):
        h = (k * np.uint64(0x9E3779B97F4A7C15)) ^ (s * np.uint64(31)) ^ (e * np.uint64(17)) ^ r
        tot = h.sum(dtype=np.uint64) if h.size else np.uint64(0)
    return int(np.array(tot, dtype=np.uint64).view(np.int64))


def run_parallel_wm(cfg: GwConfig, threads: int, batch_len, wm, key, ts, value_bits):
    """run_parallel with per-watermark results: (rows[nb + 1], checksum[nb + 1], seconds),
    the last entry for the final MAX_WATERMARK; checksum as rows_hash_sum."""
    batch_len = np.ascontiguousarray(batch_len, dtype=np.int64)
    wm = np.ascontiguousarray(wm, dtype=np.int64)
    key = np.ascontiguousarray(key, dtype=np.int64)
    ts = np.ascontiguousarray(ts, dtype=np.int64)
    vb = None if value_bits is None else np.ascontiguousarray(value_bits).view(np.int64)
    nb = len(batch_len)
    rows = np.zeros(nb + 1, np.int64)
    cs = np.zeros(nb + 1, np.int64)
    sec = ctypes.c_double(0)
    rc = lib().wo_run_parallel_wm(ctypes.byref(cfg), threads, nb, _p(batch_len), _p(wm), _p(key), _p(ts), _p(vb),
                                  _p(rows), _p(cs), ctypes.byref(sec))
    if rc < 0:
        raise OracleError(f"parallel oracle failed: {rc}")
    return rows, cs, sec.value


def run_parallel_rows(cfg: GwConfig, threads: int, batch_len, wm, key, ts, value_bits, cap: int):
    """run_parallel keeping every fired row: (key, start, end, result bits, watermark index)
    numpy columns (index len(batch_len) = the final MAX_WATERMARK), seconds."""
    batch_len = np.ascontiguousarray(batch_len, dtype=np.int64)
    wm = np.ascontiguousarray(wm, dtype=np.int64)
    key = np.ascontiguousarray(key, dtype=np.int64)
    ts = np.ascontiguousarray(ts, dtype=np.int64)
    vb = None if value_bits is None else np.ascontiguousarray(value_bits).view(np.int64)
    k, s, e, r = (np.empty(cap, np.int64) for _ in range(4))
    w = np.empty(cap, np.int32)
    sec = ctypes.c_double(0)
    n = lib().wo_run_parallel_rows(ctypes.byref(cfg), threads, len(batch_len), _p(batch_len), _p(wm), _p(key),
                                   _p(ts), _p(vb), cap, _p(k), _p(s), _p(e), _p(r), _p(w), ctypes.byref(sec))
    if n < 0:
        raise OracleError(f"parallel oracle failed: {n}")
    return k[:n], s[:n], e[:n], r[:n], w[:n], sec.value
