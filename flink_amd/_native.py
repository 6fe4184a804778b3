"""ctypes binding of libgpuwin.so (include/gpuwin.h).

The product path has no CPU fallback: if the HIP library is missing or cannot be
loaded, import-time use fails loudly with NativeLibraryError.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# GW_LIB_PATH: an experiment build of the same library (flink_amd.build --define ... --out ...)
LIB_PATH = os.environ.get("GW_LIB_PATH") or os.path.join(HERE, "libgpuwin.so")

GW_OK = 0
ERRORS = {
    -1: "GW_E_INVALID", -2: "GW_E_UNSUPPORTED", -3: "GW_E_DEVICE", -4: "GW_E_OOM",
    -5: "GW_E_OUTPUT_FULL", -6: "GW_E_NO_TIMESTAMP", -7: "GW_E_RANGE", -8: "GW_E_STATE",
}
GW_E_INVALID, GW_E_UNSUPPORTED, GW_E_DEVICE, GW_E_OOM, GW_E_OUTPUT_FULL = -1, -2, -3, -4, -5
GW_E_NO_TIMESTAMP, GW_E_RANGE, GW_E_STATE = -6, -7, -8
STAGE_VALUE, STAGE_KEY_HASH = 1, 2

ASSIGNERS = {"tumbling": 0, "sliding": 1, "session": 2, "count_tumbling": 3, "count_sliding": 4}
TRIGGERS = {"event_time": 0, "purging_event_time": 1}
AGGS = {
    "count": 0, "sum_i64": 1, "sum_f64": 2, "min_i64": 3, "max_i64": 4,
    "min_f64": 5, "max_f64": 6, "avg_i64": 7, "avg_f64": 8, "sum_i32": 9,
}
DOUBLE_RESULT = {"sum_f64", "min_f64", "max_f64", "avg_i64", "avg_f64"}
DOUBLE_INPUT = {"sum_f64", "min_f64", "max_f64", "avg_f64"}

FLAG_FORCE_LDS_PREAGG = 1
FLAG_NO_LDS_PREAGG = 2
FLAG_CHECK_KEY_GROUPS = 4
FLAG_FORCE_REGION = 8
FLAG_NO_REGION = 16
FLAG_NO_BUFFER = 32
FLAG_LATE_SIDE_OUTPUT = 64
FLAG_FIRST_ELEMENT = 128
FLAG_NO_NARROW = 256
FLAG_BY_FIELD = 512
FLAG_BY_LAST = 1024

EXPORTS = [
    "gw_create", "gw_destroy", "gw_last_error", "gw_abi_version", "gw_ingest", "gw_ingest_device",
    "gw_advance_watermark", "gw_flush", "gw_snapshot", "gw_restore", "gw_snapshot_slice", "gw_end_input", "gw_pending_rows", "gw_drain", "gw_rows_device",
    "gw_clear_rows", "gw_late_dropped", "gw_pending_late", "gw_drain_late", "gw_get_stats", "gw_synchronize", "gw_stream",
    "gw_kernel_time_ms", "gw_enable_kernel_timing", "gw_java_long_hash", "gw_murmur_hash",
    "gw_key_group_for_hash", "gw_operator_for_key_group", "gw_default_max_parallelism",
    "gw_key_groups_device", "gw_partition_scratch_bytes", "gw_partition_device",
    "gw_decode_serialized", "gw_ingest_serialized", "gw_ingest_serialized_device",
    "gw_exchange_unique_id", "gw_exchange_create", "gw_exchange_destroy", "gw_exchange_set_timeout", "gw_exchange_batch", "gw_exchange_begin", "gw_exchange_finish",
    "gw_exchange_min_watermark", "gw_exchange_last_error", "gw_exchange_counts", "gw_exchange_plan",
    "gw_window_stagger_offset", "gw_stage_alloc", "gw_stage_columns", "gw_ingest_stage", "gw_stage_send",
    "gw_ingest_payload", "gw_ingest_payload_device", "gw_drain_payload",
    "gw_snapshot_keys", "gw_snapshot_remap_keys", "gw_snapshot_payloads", "gw_snapshot_remap_payloads",
    "gw_pack_geom_init", "gw_pack_records", "gw_unpack_records", "gw_partition_packed_device", "gw_partition_regions_device", "gw_unpack_device",
    "gw_select_lookup_device",
    "gw_exchange_enable_packing", "gw_exchange_last_packed", "gw_exchange_plan_packed",
    "gw_exchange_set_unpack", "gw_exchange_last_words", "gw_ingest_packed_device",
]
EXCHANGE_ID_BYTES = 128
EXCHANGE_RECV_SETS = 3  # gpuwin.h GW_EXCHANGE_RECV_SETS


class GwRecordLayout(ctypes.Structure):
    """gw_record_layout: the Tuple value type of the serialized records."""
    _fields_ = [("nfields", ctypes.c_int32), ("key_field", ctypes.c_int32), ("value_field", ctypes.c_int32),
                ("types", ctypes.c_char * 8)]


class GwDecodeResult(ctypes.Structure):
    _fields_ = [("records", ctypes.c_int64), ("watermarks", ctypes.c_int64), ("consumed", ctypes.c_int64),
                ("skipped", ctypes.c_int64)]


def record_layout(types: str, key_field: int, value_field: int = -1) -> GwRecordLayout:
    """types: JVM type codes of the Tuple fields, e.g. "JJ" for Tuple2<Long, Long>."""
    lay = GwRecordLayout()
    lay.nfields, lay.key_field, lay.value_field = len(types), key_field, value_field
    lay.types = types.encode()
    return lay


class GwPackGeom(ctypes.Structure):
    """gw_pack_geom: packed exchange records (include/gpuwin.h)."""
    _fields_ = [("pane", ctypes.c_int64), ("offset", ctypes.c_int64), ("base_pane", ctypes.c_int64),
                ("enabled", ctypes.c_int32), ("pad", ctypes.c_int32)]


class NativeLibraryError(RuntimeError):
    pass


class GpuWinError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class GwConfig(ctypes.Structure):
    _fields_ = [
        ("assigner", ctypes.c_int32), ("trigger", ctypes.c_int32),
        ("size", ctypes.c_int64), ("slide", ctypes.c_int64), ("offset", ctypes.c_int64),
        ("gap", ctypes.c_int64), ("allowed_lateness", ctypes.c_int64),
        ("agg", ctypes.c_int32), ("max_parallelism", ctypes.c_int32),
        ("parallelism", ctypes.c_int32), ("operator_index", ctypes.c_int32),
        ("device", ctypes.c_int32), ("flags", ctypes.c_int32),
        ("capacity_hint", ctypes.c_int64), ("max_batch", ctypes.c_int64),
    ]


class GwStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in (
        "events_in", "late_dropped", "rows_fired", "live_keys", "table_capacity", "table_bytes",
        "deferred", "batches", "fires", "rehashes", "preagg_batches", "session_merges", "applies",
        "region_format", "session_punted", "session_slow")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


_lib = None


def lib() -> ctypes.CDLL:
    """Load libgpuwin.so (built in-tree by flink_amd.build); raise if absent."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: torch bundles its own libamdhip64.so.7 (same SONAME as
    # /opt/rocm's).  Whichever is loaded first serves both, and torch only initialises
    # with its own, so import torch first when it is installed (plumbing only; the
    # library itself has no torch dependency and binds whatever runtime is loaded).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryError(
            f"{LIB_PATH} not found: build it with `python -m flink_amd.build` (hipcc, gfx950). "
            "There is no CPU fallback on the product path.")
    try:
        L = ctypes.CDLL(LIB_PATH)
    except OSError as e:
        raise NativeLibraryError(f"cannot load {LIB_PATH}: {e}") from e
    i32, i64, p, c_int = ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int
    P64 = ctypes.POINTER(ctypes.c_int64)
    sig = {
        "gw_create": (c_int, [ctypes.POINTER(GwConfig), ctypes.POINTER(p)]),
        "gw_destroy": (c_int, [p]),
        "gw_last_error": (ctypes.c_char_p, [p]),
        "gw_abi_version": (c_int, []),
        "gw_ingest": (c_int, [p, i64, p, p, p, p]),
        "gw_ingest_device": (c_int, [p, i64, p, p, p, p, p]),
        "gw_advance_watermark": (c_int, [p, i64, P64]),
        "gw_flush": (c_int, [p]),
        "gw_snapshot": (c_int, [p, i32, i32, p, i64, P64]),
        "gw_restore": (c_int, [p, p, i64]),
        "gw_snapshot_slice": (c_int, [p, i64, i32, p, i64, P64]),
        "gw_snapshot_keys": (c_int, [p, i64, p, i64, P64]),
        "gw_snapshot_remap_keys": (c_int, [p, i64, p, p, i64]),
        "gw_snapshot_payloads": (c_int, [p, i64, p, i64, P64, P64]),
        "gw_snapshot_remap_payloads": (c_int, [p, i64, p, p, i64]),
        "gw_end_input": (c_int, [p, P64]),
        "gw_pending_rows": (c_int, [p, P64]),
        "gw_drain": (c_int, [p, p, p, p, p, i64, P64]),
        "gw_ingest_payload": (c_int, [p, i64, p, p, p, p, p]),
        "gw_ingest_payload_device": (c_int, [p, i64, p, p, p, p, p, p]),
        "gw_drain_payload": (c_int, [p, p, p, p, p, p, i64, P64]),
        "gw_rows_device": (c_int, [p, ctypes.POINTER(p), ctypes.POINTER(p), ctypes.POINTER(p),
                                   ctypes.POINTER(p), P64]),
        "gw_clear_rows": (c_int, [p]),
        "gw_late_dropped": (i64, [p]),
        "gw_pending_late": (c_int, [p, P64]),
        "gw_drain_late": (c_int, [p, p, p, p, i64, P64]),
        "gw_get_stats": (c_int, [p, ctypes.POINTER(GwStats)]),
        "gw_synchronize": (c_int, [p]),
        "gw_stream": (p, [p]),
        "gw_kernel_time_ms": (c_int, [p, c_int, ctypes.POINTER(ctypes.c_double), P64]),
        "gw_enable_kernel_timing": (c_int, [p, c_int]),
        "gw_java_long_hash": (i32, [i64]),
        "gw_murmur_hash": (i32, [i32]),
        "gw_key_group_for_hash": (i32, [i32, i32]),
        "gw_operator_for_key_group": (i32, [i32, i32, i32]),
        "gw_default_max_parallelism": (i32, [i32]),
        "gw_key_groups_device": (c_int, [i64, p, p, i32, i32, p, p, p]),
        "gw_partition_scratch_bytes": (i64, [i64, i32]),
        "gw_partition_device": (c_int, [i64, p, p, p, p, i32, i32, p, p, p, p, p, p]),
        "gw_decode_serialized": (c_int, [p, i64, ctypes.POINTER(GwRecordLayout), p, p, p, i64, p, p, i64,
                                         ctypes.POINTER(GwDecodeResult), p]),
        "gw_ingest_serialized": (c_int, [p, p, i64, ctypes.POINTER(GwRecordLayout), P64, P64]),
        "gw_ingest_serialized_device": (c_int, [p, p, i64, ctypes.POINTER(GwRecordLayout), p, P64, P64]),
        "gw_exchange_unique_id": (c_int, [p]),
        "gw_exchange_create": (c_int, [ctypes.POINTER(p), i32, i32, p, i32, i32]),
        "gw_exchange_destroy": (None, [p]),
        "gw_exchange_set_timeout": (c_int, [p, i64]),
        "gw_exchange_batch": (c_int, [p, i64, p, p, p, p, i64, P64, ctypes.POINTER(p), ctypes.POINTER(p),
                                      ctypes.POINTER(p), ctypes.POINTER(p), P64, ctypes.POINTER(p), p]),
        "gw_exchange_begin": (c_int, [p, i64, p, p, p, p, i64, p]),
        "gw_exchange_finish": (c_int, [p, P64, ctypes.POINTER(p), ctypes.POINTER(p), ctypes.POINTER(p),
                                       ctypes.POINTER(p), P64, ctypes.POINTER(p), p]),
        "gw_exchange_counts": (c_int, [p, p, p]),
        "gw_exchange_plan": (c_int, [i32, p, p, i64, i64, p, p, p, p, P64, P64]),
        "gw_window_stagger_offset": (c_int, [i32, i64, ctypes.c_double, i64, i64, P64]),
        "gw_stage_alloc": (c_int, [p, i32, i64]),
        "gw_stage_columns": (c_int, [p, i32, ctypes.POINTER(p), ctypes.POINTER(p), ctypes.POINTER(p), ctypes.POINTER(p)]),
        "gw_ingest_stage": (c_int, [p, i32, i64, i32]),
        "gw_stage_send": (c_int, [p, i32, i64, i32]),
        "gw_exchange_min_watermark": (c_int, [p, i64, P64, p]),
        "gw_exchange_last_error": (ctypes.c_char_p, [p]),
        "gw_pack_geom_init": (c_int, [ctypes.POINTER(GwPackGeom), i64, i64, i64, i64]),
        "gw_pack_records": (c_int, [i64, p, p, p, ctypes.POINTER(GwPackGeom), p, p]),
        "gw_unpack_records": (c_int, [i64, p, ctypes.POINTER(GwPackGeom), p, p, p]),
        "gw_partition_packed_device": (c_int, [i64, p, p, p, i32, i32, ctypes.POINTER(GwPackGeom), p, p, p, p, p, p,
                                               p]),
        "gw_partition_regions_device": (c_int, [i64, p, p, p, i32, i32, ctypes.POINTER(GwPackGeom), i64, p, p, p,
                                                p, p, p, p]),
        "gw_unpack_device": (c_int, [i64, p, ctypes.POINTER(GwPackGeom), p, p, p, p]),
        "gw_select_lookup_device": (c_int, [i64, p, i64, p, p, i64, p, p, p, ctypes.POINTER(ctypes.c_int64), p]),
        "gw_exchange_enable_packing": (c_int, [p, i64, i64, i64, i32]),
        "gw_exchange_last_packed": (i64, [p]),
        "gw_exchange_plan_packed": (c_int, [i32, p, p, p, p, p, p, P64, P64]),
        "gw_exchange_set_unpack": (c_int, [p, i32]),
        "gw_exchange_last_words": (c_int, [p, P64, ctypes.POINTER(p), ctypes.POINTER(GwPackGeom)]),
        "gw_ingest_packed_device": (c_int, [p, i64, p, p, p, i64, p, ctypes.POINTER(GwPackGeom), p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return _lib


def check(rc: int, handle=None):
    if rc != GW_OK:
        msg = lib().gw_last_error(handle)
        raise GpuWinError(rc, msg.decode() if msg else "")
    return rc


def snapshot_slice(blob: bytes, kg: int) -> bytes:
    """The part of a gw_snapshot blob that belongs to key group kg, as a blob of its own
    (gw_snapshot_slice: what GpuWindowOperator writes per key group)."""
    n = ctypes.c_int64(0)
    check(lib().gw_snapshot_slice(blob, len(blob), kg, None, 0, ctypes.byref(n)))
    out = ctypes.create_string_buffer(n.value)
    check(lib().gw_snapshot_slice(blob, len(blob), kg, out, n.value, ctypes.byref(n)))
    return out.raw[:n.value]


def snapshot_keys(blob: bytes):
    """The distinct keys (int64 ids) a snapshot blob names, ascending (gw_snapshot_keys)."""
    import numpy as np
    n = ctypes.c_int64(0)
    check(lib().gw_snapshot_keys(blob, len(blob), None, 0, ctypes.byref(n)))
    out = np.empty(n.value, np.int64)
    if n.value:
        check(lib().gw_snapshot_keys(blob, len(blob), out.ctypes.data, n.value, ctypes.byref(n)))
    return out


def snapshot_remap_keys(blob: bytes, mapping: dict) -> bytes:
    """A copy of blob with every key k in mapping replaced by mapping[k] (gw_snapshot_remap_keys)."""
    import numpy as np
    buf = ctypes.create_string_buffer(bytes(blob), len(blob))
    src = np.asarray(sorted(mapping), dtype=np.int64)
    dst = np.asarray([mapping[int(k)] for k in src], dtype=np.int64)
    check(lib().gw_snapshot_remap_keys(buf, len(blob), src.ctypes.data, dst.ctypes.data, len(src)))
    return buf.raw[:len(blob)]


MSG_WORDS = 4  # exchange message per peer: (records, watermark, column mask, packed records)


def exchange_plan(sent_msg, recv_msg, cols_mask: int, wm: int):
    """gw_exchange_plan (host only): per-peer (send_off, send_cnt, recv_off, recv_cnt), total
    received, minimum watermark from this rank's sent / received (records, watermark, mask,
    packed records) messages (int64[nranks * 4] each)."""
    import numpy as np
    sm = np.ascontiguousarray(sent_msg, dtype=np.int64)
    rm = np.ascontiguousarray(recv_msg, dtype=np.int64)
    P = len(sm) // MSG_WORDS
    out = [np.zeros(P, np.int64) for _ in range(4)]
    tot, wmin = ctypes.c_int64(), ctypes.c_int64()
    rc = lib().gw_exchange_plan(P, sm.ctypes.data, rm.ctypes.data, int(cols_mask), int(wm),
                                *[o.ctypes.data for o in out], ctypes.byref(tot), ctypes.byref(wmin))
    check(rc)
    return out, tot.value, wmin.value


def exchange_plan_packed(sent_msg, recv_msg):
    """gw_exchange_plan_packed: per-peer (send_packed, recv_other_off, recv_packed_off,
    recv_packed), total other, total packed."""
    import numpy as np
    sm = np.ascontiguousarray(sent_msg, dtype=np.int64)
    rm = np.ascontiguousarray(recv_msg, dtype=np.int64)
    P = len(sm) // MSG_WORDS
    out = [np.zeros(P, np.int64) for _ in range(4)]
    to, tp = ctypes.c_int64(), ctypes.c_int64()
    check(lib().gw_exchange_plan_packed(P, sm.ctypes.data, rm.ctypes.data, *[o.ctypes.data for o in out],
                                        ctypes.byref(to), ctypes.byref(tp)))
    return out, to.value, tp.value


def pack_geom(size: int, slide: int, offset: int, watermark: int):
    """gw_pack_geom_init; None when the geometry does not pack (size < slide, no watermark yet)."""
    g = GwPackGeom()
    rc = lib().gw_pack_geom_init(ctypes.byref(g), int(size), int(slide), int(offset), int(watermark))
    if rc == GW_E_UNSUPPORTED:
        return None
    check(rc)
    return g


def pack_records(keys, ts, vals, g: GwPackGeom):
    """gw_pack_records (host): (words uint64[n], fits bool[n])."""
    import numpy as np
    keys = np.ascontiguousarray(keys, np.int64)
    ts = np.ascontiguousarray(ts, np.int64)
    vals = None if vals is None else np.ascontiguousarray(vals, np.int64)
    n = keys.size
    w = np.zeros(n, np.uint64)
    f = np.zeros(n, np.uint8)
    check(lib().gw_pack_records(n, keys.ctypes.data, ts.ctypes.data, None if vals is None else vals.ctypes.data,
                                ctypes.byref(g), w.ctypes.data, f.ctypes.data))
    return w, f.astype(bool)


def unpack_records(words, g: GwPackGeom, with_values: bool = True):
    """gw_unpack_records (host): (keys, ts, values or None)."""
    import numpy as np
    words = np.ascontiguousarray(words, np.uint64)
    n = words.size
    k, t = np.zeros(n, np.int64), np.zeros(n, np.int64)
    v = np.zeros(n, np.int64) if with_values else None
    check(lib().gw_unpack_records(n, words.ctypes.data, ctypes.byref(g), k.ctypes.data, t.ctypes.data,
                                  None if v is None else v.ctypes.data))
    return k, t, v
