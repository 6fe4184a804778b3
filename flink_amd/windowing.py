"""Host-side mirror of the reference's keyed event-time window operator interface.

Names, argument meaning and error behaviour follow Flink's DataStream windowing API
so a job (or a harness test) reads the same:

  * assigners   TumblingEventTimeWindows.of / SlidingEventTimeWindows.of /
                EventTimeSessionWindows.with_gap
                (flink-runtime/.../streaming/api/windowing/assigners/*.java,
                 flink-streaming-java/.../EventTimeSessionWindows.java)
  * triggers    EventTimeTrigger.create(), PurgingTrigger.of(...)
  * operator    GpuWindowOperator — the OneInputStreamOperator slot of WindowOperator
                (RS/runtime/operators/windowing/WindowOperator.java:102): open,
                process_element, process_watermark, end_input, close.  Records between
                two watermarks are batched into columns and handed to libgpuwin.so in one
                gw_ingest call; process_watermark fires through gw_advance_watermark.
  * errors      invalid configurations raise ValueError (IllegalArgumentException in
                the reference), runtime failures raise GpuWinError (the task fails).

Every call goes to the HIP library; there is no CPU path here.
"""
from __future__ import annotations

import ctypes
import struct
import time
from dataclasses import dataclass
from typing import Any, Callable, Iterable, List, Optional

import numpy as np

from . import _native as N

LONG_MIN = -(1 << 63)
LONG_MAX = (1 << 63) - 1


# --------------------------------------------------------------------------- time
class Duration:
    """java.time.Duration stand-in: milliseconds."""

    @staticmethod
    def of_millis(ms: int) -> int:
        return int(ms)

    @staticmethod
    def of_seconds(s: int) -> int:
        return int(s) * 1000

    @staticmethod
    def of_minutes(m: int) -> int:
        return int(m) * 60_000


# ---------------------------------------------------------------------- assigners
class WindowAssigner:
    kind = ""

    def config(self) -> dict:
        raise NotImplementedError


class WindowStagger:
    """WindowStagger (RS/api/windowing/assigners/WindowStagger.java:27-60): ALIGNED (0), RANDOM
    (U(0, size)) or NATURAL (the processing time's offset into its window), drawn at the first
    element; gw_window_stagger_offset computes the resulting window offset."""
    ALIGNED, RANDOM, NATURAL = 0, 1, 2

    @staticmethod
    def window_offset(stagger: int, processing_time: int, size: int, global_offset: int,
                      random01: Optional[float] = None) -> int:
        """(global_offset + stagger offset) % size, as TumblingEventTimeWindows.assignWindows
        uses it (TumblingEventTimeWindows.java:72-79)."""
        import random
        r = random.random() if random01 is None else float(random01)
        out = ctypes.c_int64(0)
        N.check(N.lib().gw_window_stagger_offset(int(stagger), int(processing_time), r, int(size), int(global_offset),
                                                 ctypes.byref(out)))
        return out.value


class TumblingEventTimeWindows(WindowAssigner):
    """TumblingEventTimeWindows.of(size[, offset[, stagger]])."""
    kind = "tumbling"

    def __init__(self, size: int, offset: int = 0, stagger: int = WindowStagger.ALIGNED):
        if abs(offset) >= size:  # TumblingEventTimeWindows.java:55-62
            raise ValueError("TumblingEventTimeWindows parameters must satisfy abs(offset) < size")
        self.size, self.offset, self.stagger = int(size), int(offset), int(stagger)

    @staticmethod
    def of(size: int, offset: int = 0, stagger: int = WindowStagger.ALIGNED) -> "TumblingEventTimeWindows":
        return TumblingEventTimeWindows(size, offset, stagger)

    def config(self):
        return dict(assigner="tumbling", size=self.size, slide=self.size, offset=self.offset)


class SlidingEventTimeWindows(WindowAssigner):
    kind = "sliding"
    MAX_WINDOW_NUM = 10_000_000

    def __init__(self, size: int, slide: int, offset: int = 0):
        if abs(offset) >= slide or size <= 0:  # SlidingEventTimeWindows.java:57-70
            raise ValueError("SlidingEventTimeWindows parameters must satisfy abs(offset) < slide and size > 0")
        if size // slide > self.MAX_WINDOW_NUM:
            raise ValueError(f"SlidingEventTimeWindows parameters must satisfy size / slide <= {self.MAX_WINDOW_NUM}")
        self.size, self.slide, self.offset = int(size), int(slide), int(offset)

    @staticmethod
    def of(size: int, slide: int, offset: int = 0) -> "SlidingEventTimeWindows":
        return SlidingEventTimeWindows(size, slide, offset)

    def config(self):
        return dict(assigner="sliding", size=self.size, slide=self.slide, offset=self.offset)


class EventTimeSessionWindows(WindowAssigner):
    kind = "session"

    def __init__(self, gap: int):
        if gap <= 0:  # EventTimeSessionWindows.java:52-53
            raise ValueError("EventTimeSessionWindows parameters must satisfy 0 < size")
        self.gap = int(gap)

    @staticmethod
    def with_gap(gap: int) -> "EventTimeSessionWindows":
        return EventTimeSessionWindows(gap)

    withGap = with_gap

    def config(self):
        return dict(assigner="session", gap=self.gap)


class CountWindows(WindowAssigner):
    """KeyedStream.countWindow(size[, slide]) — GlobalWindows with
    PurgingTrigger(CountTrigger(size)), or CountEvictor(size) + CountTrigger(slide)
    (RS/api/datastream/KeyedStream.java:676-690).  Rows are (key, first element ordinal,
    end ordinal, result) and come out of process_batch itself."""
    kind = "count"

    def __init__(self, size: int, slide: Optional[int] = None):
        if size <= 0 or (slide is not None and slide <= 0):
            raise ValueError("count windows need size > 0 and slide > 0")
        self.size, self.slide = int(size), (int(slide) if slide is not None else None)

    @staticmethod
    def of(size: int, slide: Optional[int] = None) -> "CountWindows":
        return CountWindows(size, slide)

    def config(self):
        if self.slide is None:
            return dict(assigner="count_tumbling", size=self.size, slide=self.size)
        return dict(assigner="count_sliding", size=self.size, slide=self.slide)


# ----------------------------------------------------------------------- triggers
class EventTimeTrigger:
    name = "event_time"

    @staticmethod
    def create() -> "EventTimeTrigger":
        return EventTimeTrigger()


class PurgingTrigger:
    def __init__(self, nested):
        if not isinstance(nested, EventTimeTrigger):
            raise ValueError("only PurgingTrigger.of(EventTimeTrigger) is on the GPU path")
        self.name = "purging_event_time"

    @staticmethod
    def of(nested) -> "PurgingTrigger":
        return PurgingTrigger(nested)


# ------------------------------------------------------------------ stream elements
@dataclass
class StreamRecord:
    value: Any
    timestamp: int


@dataclass
class Watermark:
    timestamp: int


MAX_WATERMARK = Watermark(LONG_MAX)


def java_string_hash(s: str) -> int:
    """JDK String.hashCode (UTF-16 code units, int arithmetic)."""
    h = 0
    data = s.encode("utf-16-le")
    for i in range(0, len(data), 2):
        h = (31 * h + (data[i] | (data[i + 1] << 8))) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


def java_hash(key) -> int:
    """key.hashCode() for the key types the path supports."""
    if isinstance(key, bool):
        return 1231 if key else 1237
    if isinstance(key, int):
        if -(1 << 31) <= key < (1 << 31):
            return key  # Integer.hashCode
        return N.lib().gw_java_long_hash(key)
    if isinstance(key, str):
        return java_string_hash(key)
    raise TypeError(f"unsupported key type {type(key).__name__}")


def assign_to_key_group(key, max_parallelism: int) -> int:
    """KeyGroupRangeAssignment.assignToKeyGroup (bit-exact, via libgpuwin.so)."""
    return N.lib().gw_key_group_for_hash(java_hash(key), max_parallelism)


def compute_operator_index_for_key_group(max_parallelism: int, parallelism: int, key_group: int) -> int:
    return N.lib().gw_operator_for_key_group(max_parallelism, parallelism, key_group)


def compute_key_group_range_for_operator_index(max_parallelism: int, parallelism: int, index: int):
    """KeyGroupRangeAssignment.computeKeyGroupRangeForOperatorIndex (:93-106)."""
    start = (index * max_parallelism + parallelism - 1) // parallelism
    end = ((index + 1) * max_parallelism - 1) // parallelism
    return start, end


def compute_default_max_parallelism(parallelism: int) -> int:
    return N.lib().gw_default_max_parallelism(parallelism)


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def select_lookup_device(sel, sel_value: int, idx, dictionary, ts, key_out, ts_out, stream) -> int:
    """gw_select_lookup_device over device tensors (int64): the records with sel == sel_value,
    in arrival order, as (dictionary[idx], ts) into key_out / ts_out; returns their number.  The
    filter + projection + static-table join a job chains ahead of keyBy (YSB's view filter
    and ad -> campaign join), fused on the device."""
    n_out = ctypes.c_int64(0)
    N.check(N.lib().gw_select_lookup_device(sel.numel(), sel.data_ptr(), int(sel_value), idx.data_ptr(),
                                             dictionary.data_ptr(), dictionary.numel(), ts.data_ptr(),
                                             key_out.data_ptr(), ts_out.data_ptr(), ctypes.byref(n_out), stream))
    return int(n_out.value)


# ------------------------------------------------------------------------ operator
class GpuWindowOperator:
    """Keyed event-time window operator on one MI355X (one Flink subtask).

    aggregate: one of count, sum_i64, sum_i32, sum_f64, min_i64, max_i64, min_f64,
    max_f64, avg_i64, avg_f64 (the closed set of include/gpuwin.h).
    key_selector / value_selector extract key and aggregated field from a record
    value (defaults: value[0] and value[1], i.e. Tuple2 f0 / f1).
    """

    def __init__(self, assigner: WindowAssigner, aggregate: str, allowed_lateness: int = 0,
                 trigger=None, key_selector: Callable = None, value_selector: Callable = None,
                 max_parallelism: int = 128, parallelism: int = 1, operator_index: int = 0,
                 device: int = 0, capacity_hint: int = 0, max_batch: int = 1 << 22, flags: int = 0,
                 window_function: Optional[Callable] = None, processing_time: Optional[Callable[[], int]] = None):
        if aggregate not in N.AGGS:
            raise ValueError(f"unknown aggregate {aggregate!r}")
        if allowed_lateness < 0:
            raise ValueError("The allowed lateness cannot be negative.")
        self.assigner = assigner
        self.aggregate = aggregate
        self.trigger = trigger or EventTimeTrigger.create()
        self.key_selector = key_selector or (lambda v: v[0])
        self.value_selector = value_selector or (lambda v: v[1])
        self.is_double_out = aggregate in N.DOUBLE_RESULT
        self.is_double_in = aggregate in N.DOUBLE_INPUT
        c = N.GwConfig()
        a = assigner.config()
        c.assigner = N.ASSIGNERS[a["assigner"]]
        c.trigger = N.TRIGGERS[self.trigger.name]
        c.size, c.slide, c.offset = a.get("size", 0), a.get("slide", 0), a.get("offset", 0)
        c.gap = a.get("gap", 0)
        c.allowed_lateness = allowed_lateness
        c.agg = N.AGGS[aggregate]
        c.max_parallelism, c.parallelism, c.operator_index = max_parallelism, parallelism, operator_index
        c.device, c.flags, c.capacity_hint, c.max_batch = device, flags, capacity_hint, max_batch
        self.cfg = c
        self._h = None
        self._keys_in: dict = {}
        self._keys_out: list = []
        self._hash_out: list = []  # key.hashCode() per dictionary id (gw_ingest key_hash)
        self._int_keys = True
        self._buf_k: List[int] = []
        self._buf_t: List[int] = []
        self._buf_v: List = []
        # payload handles (FLAG_FIRST_ELEMENT / FLAG_BY_FIELD) on the record-at-a-time surface:
        # each element is kept on the host and its index travels as the payload
        self._payload = bool(flags & (N.FLAG_FIRST_ELEMENT | N.FLAG_BY_FIELD))
        self._by = bool(flags & N.FLAG_BY_FIELD)
        self._elems: list = []
        self._buf_p: List[int] = []
        self.output: list = []
        # reduce / aggregate(..., ProcessWindowFunction): window_function(key, (start, end), [result],
        # out) per fired window, out a list the emitted values go to (InternalSingleValueProcess-
        # WindowFunction: a one-element Iterable of the pre-aggregated result, output stamped
        # window.maxTimestamp())
        self.window_function = window_function
        # processing-time clock in ms (ProcessingTimeService.getCurrentProcessingTime): a staggered
        # tumbling assigner draws its stagger at the first element
        self.processing_time = processing_time or (lambda: time.time_ns() // 1_000_000)
        self._stagger = getattr(assigner, "stagger", WindowStagger.ALIGNED)
        self._deferred = False        # staggered: the handle is created at the first element
        self._deferred_wm = LONG_MIN  # watermarks seen before it
        self._stagger_time = None

    # lifecycle -------------------------------------------------------------
    def open(self):
        if self._stagger != WindowStagger.ALIGNED:
            # TumblingEventTimeWindows draws its stagger at the first element (:72-79): the
            # handle, whose windows need the offset, is created then
            WindowStagger.window_offset(self._stagger, 0, self.cfg.size, self.cfg.offset, 0.0)  # validates
            self._deferred = True
            return self
        return self._create()

    def _create(self):
        h = ctypes.c_void_p()
        rc = N.lib().gw_create(ctypes.byref(self.cfg), ctypes.byref(h))
        if rc == -1:
            raise ValueError(N.lib().gw_last_error(None).decode())
        N.check(rc, None)
        self._h = h
        return self

    def _ensure_handle(self):
        """A staggered operator's first element: draw the stagger at the processing time the
        first element arrived, create the handle with (offset + stagger) % size, replay the
        watermark seen so far (no state yet: it fires nothing)."""
        if not self._deferred:
            return
        now = self._stagger_time if self._stagger_time is not None else self.processing_time()
        self.cfg.offset = WindowStagger.window_offset(self._stagger, now, self.cfg.size, self.cfg.offset)
        self._deferred = False
        self._create()
        if self._deferred_wm != LONG_MIN:
            self.advance_watermark(self._deferred_wm)

    def close(self):
        if self._h:
            N.lib().gw_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self.open() if self._h is None else self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    # keys --------------------------------------------------------------------
    def _encode_key(self, key) -> int:
        """Long keys go to the GPU as they are (the device computes Long.hashCode); any
        other key type gets a dictionary id, and its key.hashCode() travels in the key_hash
        column so key groups, snapshots and rescaling follow the key's own hash."""
        if isinstance(key, int) and not isinstance(key, bool) and LONG_MIN <= key <= LONG_MAX and self._int_keys \
                and not self._keys_out:
            return key
        self._int_keys = False
        kid = self._keys_in.get(key)
        if kid is None:
            kid = len(self._keys_out)
            self._keys_in[key] = kid
            self._keys_out.append(key)
            self._hash_out.append(java_hash(key))
        return kid

    def _decode_key(self, kid: int):
        return kid if self._int_keys else self._keys_out[kid]

    # record-at-a-time surface (StreamRecord / Watermark) ----------------------
    def process_element(self, record: StreamRecord):
        if self._deferred and self._stagger_time is None:
            self._stagger_time = self.processing_time()  # the stagger is drawn at the first element
        v = record.value
        self._buf_k.append(self._encode_key(self.key_selector(v)))
        self._buf_t.append(int(record.timestamp))
        self._buf_v.append(self.value_selector(v) if self.aggregate != "count" else 0)
        if self._payload:
            self._buf_p.append(len(self._elems))
            self._elems.append(v)

    def _flush(self):
        if not self._buf_k:
            return
        k = np.asarray(self._buf_k, dtype=np.int64)
        t = np.asarray(self._buf_t, dtype=np.int64)
        if self.is_double_in:
            v = np.asarray(self._buf_v, dtype=np.float64).view(np.int64)
        else:
            v = np.asarray(self._buf_v, dtype=np.int64)
        self._buf_k, self._buf_t, self._buf_v = [], [], []
        h = None if self._int_keys else np.asarray(self._hash_out, dtype=np.int32)[k]
        if self._payload:
            p = np.asarray(self._buf_p, dtype=np.int64)
            self._buf_p = []
            self.process_batch_payload(k, t, v, p, key_hashes=h)
        else:
            self.process_batch(k, t, v, key_hashes=h)

    def process_watermark(self, wm):
        ts = wm.timestamp if isinstance(wm, Watermark) else int(wm)
        self._flush()
        self.advance_watermark(ts)
        if self._payload:
            # minBy / maxBy emit the element itself (ComparableAggregator.java:88-95); positional
            # aggregates the first element beside the result
            k, s, e, r, pl = self.drain_payload()
            for i in range(len(k)):
                el = self._elems[int(pl[i])]
                val = el if self._by else (self._decode_key(int(k[i])), int(s[i]), int(e[i]), r[i], el)
                self.output.append(StreamRecord(val, int(e[i]) - 1))
            self.output.append(Watermark(ts))
            return
        k, s, e, r = self.drain()
        for i in range(len(k)):
            res = r[i]
            key, start, end = self._decode_key(int(k[i])), int(s[i]), int(e[i])
            if self.window_function is not None:
                out: list = []
                self.window_function(key, (start, end), [res], out)
                self.output.extend(StreamRecord(x, end - 1) for x in out)
            else:
                self.output.append(StreamRecord((key, start, end, res), end - 1))
        self.output.append(Watermark(ts))

    def end_input(self):
        """BoundedOneInput.endInput followed by MAX_WATERMARK."""
        self.process_watermark(MAX_WATERMARK)

    def get_output(self):
        out, self.output = self.output, []
        return out

    # columnar surface ------------------------------------------------------------
    def process_batch(self, keys: np.ndarray, timestamps: np.ndarray, values: Optional[np.ndarray] = None,
                      key_hashes: Optional[np.ndarray] = None):
        self._ensure_handle()
        keys = np.ascontiguousarray(keys, dtype=np.int64)
        timestamps = np.ascontiguousarray(timestamps, dtype=np.int64)
        if values is not None:
            values = np.ascontiguousarray(values)
            if values.dtype == np.float64:
                values = values.view(np.int64)
            values = values.astype(np.int64, copy=False)
        if key_hashes is not None:
            key_hashes = np.ascontiguousarray(key_hashes, dtype=np.int32)
        if len(keys) != len(timestamps) or (values is not None and len(values) != len(keys)):
            raise ValueError("column lengths differ")
        rc = N.lib().gw_ingest(self._h, len(keys), _ptr(keys), _ptr(key_hashes), _ptr(timestamps), _ptr(values))
        N.check(rc, self._h)

    # first-element rows (flags=FLAG_FIRST_ELEMENT) ------------------------------------
    def process_batch_payload(self, keys, timestamps, values, payload, key_hashes=None):
        """Records with a 64-bit payload each (the Tuple's non-aggregated fields, packed by the
        caller); rows carry the payload of their window's first element in arrival order, as
        SumAggregator / ComparableAggregator keep it (gw_ingest_payload)."""
        self._ensure_handle()
        keys = np.ascontiguousarray(keys, dtype=np.int64)
        timestamps = np.ascontiguousarray(timestamps, dtype=np.int64)
        values = np.ascontiguousarray(values)
        values = values.view(np.int64) if values.dtype == np.float64 else values.astype(np.int64, copy=False)
        payload = np.ascontiguousarray(payload, dtype=np.int64)
        if key_hashes is not None:
            key_hashes = np.ascontiguousarray(key_hashes, dtype=np.int32)
        if not (len(keys) == len(timestamps) == len(values) == len(payload)):
            raise ValueError("column lengths differ")
        N.check(N.lib().gw_ingest_payload(self._h, len(keys), _ptr(keys), _ptr(key_hashes), _ptr(timestamps),
                                          _ptr(values), _ptr(payload)), self._h)

    def process_batch_payload_device(self, keys, timestamps, values, payload, stream=None):
        """Same, with torch device columns produced on `stream` (default: torch's current)."""
        self._ensure_handle()
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(keys.device).cuda_stream
        p = [ctypes.c_void_p(x.data_ptr()) for x in (keys, timestamps, values, payload)]
        N.check(N.lib().gw_ingest_payload_device(self._h, keys.numel(), p[0], None, p[1], p[2], p[3],
                                                 ctypes.c_void_p(stream) if stream else None), self._h)

    def drain_payload(self):
        """All pending rows as numpy (key, start, end, result, payload) columns."""
        n = self.pending_rows()
        k, s, e, r, pl = (np.empty(n, np.int64) for _ in range(5))
        got = ctypes.c_int64(0)
        if n:
            N.check(N.lib().gw_drain_payload(self._h, _ptr(k), _ptr(s), _ptr(e), _ptr(r), _ptr(pl), n,
                                             ctypes.byref(got)), self._h)
            assert got.value == n
        if self.is_double_out:
            r = r.view(np.float64)
        return k, s, e, r, pl

    # network-buffer surface -----------------------------------------------------------
    def process_serialized(self, data: bytes, layout: "N.GwRecordLayout") -> tuple:
        """Decode and process one input channel's serialized elements (records and
        watermarks) on the GPU (gw_ingest_serialized).  Returns (consumed, rows_fired):
        bytes past `consumed` belong to an element spanning into the next buffer and must
        be passed again, prepended to it."""
        self._ensure_handle()
        consumed, fired = ctypes.c_int64(0), ctypes.c_int64(0)
        buf = ctypes.create_string_buffer(bytes(data), len(data)) if data else None
        N.check(N.lib().gw_ingest_serialized(self._h, buf, len(data), ctypes.byref(layout), ctypes.byref(consumed),
                                             ctypes.byref(fired)), self._h)
        return consumed.value, fired.value

    def process_serialized_device(self, data, layout: "N.GwRecordLayout", stream=None) -> tuple:
        """Same, with the bytes in a device uint8 tensor."""
        self._ensure_handle()
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(data.device).cuda_stream
        consumed, fired = ctypes.c_int64(0), ctypes.c_int64(0)
        N.check(N.lib().gw_ingest_serialized_device(self._h, ctypes.c_void_p(data.data_ptr()), data.numel(),
                                                    ctypes.byref(layout),
                                                    ctypes.c_void_p(stream) if stream else None,
                                                    ctypes.byref(consumed), ctypes.byref(fired)), self._h)
        return consumed.value, fired.value

    def process_buffers(self, buffers, layout: "N.GwRecordLayout") -> int:
        """Feed network buffers in order, carrying a spanning record's bytes over to the next
        buffer (SpanningWrapper).  Returns the rows fired."""
        carry = b""
        fired = 0
        for b in buffers:
            data = carry + bytes(b)
            used, f = self.process_serialized(data, layout)
            carry = data[used:]
            fired += f
        if carry:
            raise N.GpuWinError(-1, f"{len(carry)} bytes of an incomplete element at the end of the input")
        return fired

    # staged host ingest (gw_stage_*): pinned library-owned columns filled in place ------------
    def stage_alloc(self, slots: int, cap: int):
        """`slots` pinned column slots of `cap` records (gw_stage_alloc)."""
        self._ensure_handle()
        N.check(N.lib().gw_stage_alloc(self._h, int(slots), int(cap)), self._h)
        self._stage_cap = int(cap)

    def stage_columns(self, slot: int):
        """Slot `slot`'s (key int64, key_hash int32, ts int64, value int64) columns as numpy arrays
        over the pinned memory, once the slot's previous transfer has read it."""
        p = [ctypes.c_void_p() for _ in range(4)]
        N.check(N.lib().gw_stage_columns(self._h, int(slot), *[ctypes.byref(x) for x in p]), self._h)
        cap = self._stage_cap

        def arr(ptr, ct):
            return np.ctypeslib.as_array(ctypes.cast(ptr.value, ctypes.POINTER(ct)), shape=(cap,))
        return arr(p[0], ctypes.c_int64), arr(p[1], ctypes.c_int32), arr(p[2], ctypes.c_int64), arr(p[3], ctypes.c_int64)

    def ingest_stage(self, slot: int, n: int, with_value: bool = True, with_key_hash: bool = False):
        """The slot's first n records (gw_ingest_stage)."""
        cols = (N.STAGE_VALUE if with_value else 0) | (N.STAGE_KEY_HASH if with_key_hash else 0)
        N.check(N.lib().gw_ingest_stage(self._h, int(slot), int(n), cols), self._h)

    def stage_send(self, slot: int, n: int, with_value: bool = True, with_key_hash: bool = False):
        """Send the slot's first n records over PCIe ahead of their gw_ingest_stage (gw_stage_send):
        up to two batches ahead (three device buffers); ingest_stage calls must follow the send
        order."""
        cols = (N.STAGE_VALUE if with_value else 0) | (N.STAGE_KEY_HASH if with_key_hash else 0)
        N.check(N.lib().gw_stage_send(self._h, int(slot), int(n), cols), self._h)

    def process_batch_device(self, keys, timestamps, values=None, stream=None):
        """Columns already in HBM (torch tensors or raw device pointers)."""
        self._ensure_handle()
        def p(x):
            if x is None:
                return None
            return ctypes.c_void_p(x if isinstance(x, int) else x.data_ptr())
        n = keys if isinstance(keys, int) else keys.numel()
        if isinstance(keys, int):
            raise ValueError("pass tensors, or use process_batch_device_ptr for raw pointers")
        if stream is None:  # the columns were produced on PyTorch's current stream
            import torch
            stream = torch.cuda.current_stream(keys.device).cuda_stream
        rc = N.lib().gw_ingest_device(self._h, n, p(keys), None, p(timestamps), p(values),
                                      ctypes.c_void_p(stream) if stream else None)
        N.check(rc, self._h)

    def process_batch_device_ptr(self, n: int, key_ptr: int, ts_ptr: int, val_ptr: Optional[int], stream=None):
        self._ensure_handle()
        rc = N.lib().gw_ingest_device(self._h, n, ctypes.c_void_p(key_ptr), None, ctypes.c_void_p(ts_ptr),
                                      ctypes.c_void_p(val_ptr) if val_ptr else None,
                                      ctypes.c_void_p(stream) if stream else None)
        N.check(rc, self._h)

    def process_batch_packed_device_ptr(self, n_other: int, key_ptr, ts_ptr, val_ptr, n_words: int, words_ptr,
                                        geom, stream=None):
        """gw_ingest_packed_device: n_other column records followed by n_words packed exchange
        words (NativeKeyByExchange.last_words)."""
        self._ensure_handle()
        vp = lambda x: ctypes.c_void_p(x) if x else None
        rc = N.lib().gw_ingest_packed_device(self._h, n_other, vp(key_ptr), vp(ts_ptr), vp(val_ptr), n_words,
                                             vp(words_ptr), ctypes.byref(geom), vp(stream))
        N.check(rc, self._h)

    def advance_watermark(self, wm: int) -> int:
        if self._deferred:  # staggered, no element yet: nothing can fire
            self._deferred_wm = max(self._deferred_wm, int(wm))
            return 0
        fired = ctypes.c_int64(0)
        N.check(N.lib().gw_advance_watermark(self._h, int(wm), ctypes.byref(fired)), self._h)
        return fired.value

    def flush(self):
        """Apply every buffered record to the window state (gw_flush); firing does this
        by itself, a snapshot or a timing boundary calls it explicitly."""
        if self._deferred:
            return
        N.check(N.lib().gw_flush(self._h), self._h)

    # checkpointing ----------------------------------------------------------------
    def snapshot_state(self, key_group_range=None) -> bytes:
        """Keyed window state of the key groups [lo, hi] (default: all), as one blob
        (StreamOperator.snapshotState; restore with initialize_state)."""
        lo, hi = key_group_range if key_group_range is not None else (0, self.cfg.max_parallelism - 1)
        if self._deferred:  # staggered, no element yet: no window state
            tmp = GpuWindowOperator(TumblingEventTimeWindows.of(self.cfg.size, self.cfg.offset), self.aggregate,
                                    self.cfg.allowed_lateness, self.trigger, max_parallelism=self.cfg.max_parallelism,
                                    device=self.cfg.device, capacity_hint=16, max_batch=16,
                                    flags=self.cfg.flags).open()
            try:
                return tmp.snapshot_state(key_group_range)
            finally:
                tmp.close()
        n = ctypes.c_int64(0)
        N.check(N.lib().gw_snapshot(self._h, lo, hi, None, 0, ctypes.byref(n)), self._h)
        buf = ctypes.create_string_buffer(n.value)
        N.check(N.lib().gw_snapshot(self._h, lo, hi, buf, n.value, ctypes.byref(n)), self._h)
        return buf.raw[:n.value]

    def initialize_state(self, blobs):
        """Restore one or more snapshot blobs (e.g. the key-group ranges of several
        subtasks after rescaling) before processing (StreamOperator.initializeState).
        A keyed snapshot (snapshot_state_keyed) gets its keys re-encoded through this
        operator's dictionary first."""
        if isinstance(blobs, (bytes, bytearray)):
            blobs = [blobs]
        if self._deferred:
            self._adopt_restored_stagger(blobs)
        if self._deferred:  # no restored window state: the stagger is drawn at the first element
            return
        for b in blobs:
            b = bytes(b)
            if b[:4] == KEYED_MAGIC:
                b = self._rekey(b)
            N.check(N.lib().gw_restore(self._h, b, len(b)), self._h)

    def _adopt_restored_stagger(self, blobs):
        """A staggered tumbling operator restored from window state keeps the stagger the state
        was written under: the blobs' window offset (header), which is (offset + stagger) %
        size of the operator that wrote them.  The reference draws a new stagger after a restore
        (TumblingEventTimeWindows.java:72-79: staggerOffset starts out null) and keeps the
        restored windows at their old alignment beside it; one handle holds one alignment, so
        the old draw is reused -- for RANDOM a valid draw of the same distribution, for NATURAL
        the first element's processing time of the run that wrote the state.  Blobs without
        state leave the operator to draw at its first element; blobs of one restore carrying
        different staggers (subtasks' independent draws merged by a rescale) are refused."""
        offs = set()
        for b in blobs:
            b = bytes(b)
            if b[:4] == KEYED_MAGIC:
                b = unpack_keyed_snapshot(b)[0]
            hdr = struct.unpack_from("<4sIii5q4i3q", b, 0)
            nk = hdr[11] - hdr[10] + 1
            if hdr[15] > 12 * nk:  # payload beyond the empty sections (n = m = t = 0) of each key group
                offs.add(int(hdr[6]))
        if len(offs) > 1:
            raise N.GpuWinError(N.GW_E_UNSUPPORTED, "restoring window state of staggered tumbling operators "
                                f"drawn with different staggers (window offsets {sorted(offs)}) into one")
        if offs:
            self.cfg.offset = offs.pop()
            self._deferred = False
            self._create()

    def snapshot_state_keyed(self, key_group_range=None) -> bytes:
        """snapshot_state plus the real keys behind the dictionary ids its entries name, as
        GpuWindowOperator.snapshotState writes them through the key serializer: any
        operator (another process, another dictionary) restores it."""
        blob = self.snapshot_state(key_group_range)
        ids = N.snapshot_keys(blob)
        return pack_keyed_snapshot(blob, {int(i): self._decode_key(int(i)) for i in ids})

    def _rekey(self, wrapped: bytes) -> bytes:
        blob, keys = unpack_keyed_snapshot(wrapped)
        if self._int_keys and all(isinstance(k, int) for k in keys.values()) and not self._keys_out:
            return N.snapshot_remap_keys(blob, {i: k for i, k in keys.items()})
        if not self._keys_out:
            self._int_keys = False
        return N.snapshot_remap_keys(blob, {i: self._encode_key(k) for i, k in keys.items()})

    def pending_rows(self) -> int:
        if self._deferred:
            return 0
        n = ctypes.c_int64(0)
        N.check(N.lib().gw_pending_rows(self._h, ctypes.byref(n)), self._h)
        return n.value

    def drain(self, out=None):
        """All pending fired rows as numpy (key, start, end, result) columns.  `out`: four int64
        numpy arrays to fill (e.g. over pinned memory, which the D2H then writes directly);
        views of their first n entries are returned."""
        n = self.pending_rows()
        if out is not None:
            if any(len(x) < n for x in out):
                raise ValueError(f"drain: out arrays hold fewer than the {n} pending rows")
            k, s, e, r = (x[:n] for x in out)
        else:
            k = np.empty(n, np.int64)
            s = np.empty(n, np.int64)
            e = np.empty(n, np.int64)
            r = np.empty(n, np.int64)
        got = ctypes.c_int64(0)
        if n:
            rc = N.lib().gw_drain(self._h, _ptr(k), _ptr(s), _ptr(e), _ptr(r), n, ctypes.byref(got))
            N.check(rc, self._h)
            assert got.value == n
        if self.is_double_out:
            r = r.view(np.float64)
        return k, s, e, r

    def clear_rows(self):
        if self._deferred:
            return
        N.check(N.lib().gw_clear_rows(self._h), self._h)

    def rows_device(self):
        p = [ctypes.c_void_p() for _ in range(4)]
        n = ctypes.c_int64(0)
        rc = N.lib().gw_rows_device(self._h, *[ctypes.byref(x) for x in p], ctypes.byref(n))
        N.check(rc, self._h)
        return [x.value for x in p], n.value

    def drain_late(self):
        """The late-data side output (flags=FLAG_LATE_SIDE_OUTPUT, WindowedStream.sideOutputLateData):
        the late records since the last call, as (key, timestamp, value bits) numpy columns."""
        if self._deferred:
            return tuple(np.empty(0, np.int64) for _ in range(3))
        n = ctypes.c_int64(0)
        N.check(N.lib().gw_pending_late(self._h, ctypes.byref(n)), self._h)
        k, t, v = (np.empty(n.value, np.int64) for _ in range(3))
        got = ctypes.c_int64(0)
        if n.value:
            N.check(N.lib().gw_drain_late(self._h, _ptr(k), _ptr(t), _ptr(v), n.value, ctypes.byref(got)), self._h)
            assert got.value == n.value
        return k, t, v

    @property
    def num_late_records_dropped(self) -> int:
        return 0 if self._deferred else N.lib().gw_late_dropped(self._h)

    def stats(self) -> dict:
        s = N.GwStats()
        if self._deferred:
            return s.as_dict()
        N.check(N.lib().gw_get_stats(self._h, ctypes.byref(s)), self._h)
        return s.as_dict()

    def stream(self) -> int:
        return N.lib().gw_stream(self._h)

    def enable_kernel_timing(self, on=True):
        """True / 1: time every launch; k > 1: time region pass 1 on every k-th batch only."""
        k = int(on) if not isinstance(on, bool) else (1 if on else 0)
        N.check(N.lib().gw_enable_kernel_timing(self._h, k), self._h)

    def kernel_time_ms(self, which: int = 0):
        ms = ctypes.c_double(0)
        n = ctypes.c_int64(0)
        N.check(N.lib().gw_kernel_time_ms(self._h, which, ctypes.byref(ms), ctypes.byref(n)), self._h)
        return ms.value, n.value

    def synchronize(self):
        if self._deferred:
            return
        N.check(N.lib().gw_synchronize(self._h), self._h)


# -------------------------------------------------------------- DataStream surface
class WindowedStream:
    """keyBy(...).window(assigner) — WindowedStream (RS/api/datastream/WindowedStream.java:84-96)."""

    def __init__(self, keyed: "KeyedStream", assigner: WindowAssigner):
        self.keyed = keyed
        self.assigner = assigner
        self._lateness = 0
        self._trigger = None

    def allowed_lateness(self, ms: int) -> "WindowedStream":
        if ms < 0:
            raise ValueError("The allowed lateness cannot be negative.")
        self._lateness = ms
        return self

    allowedLateness = allowed_lateness

    def trigger(self, trig) -> "WindowedStream":
        self._trigger = trig
        return self

    def _op(self, agg, field, flags=0, window_function=None):
        kw = dict(self.keyed.env.op_kwargs)
        kw["flags"] = kw.get("flags", 0) | flags
        if window_function is not None:
            kw["window_function"] = window_function
        return GpuWindowOperator(self.assigner, agg, self._lateness, self._trigger, self.keyed.key_selector,
                                 (lambda v: v[field]) if field is not None else (lambda v: 0), **kw)

    # WindowedStream.sum / min / max (:660, :687, :788) on a typed field, aggregate (:310)
    def sum(self, field: int, kind: str = "i64") -> "DataStreamResult":
        return DataStreamResult(self, self._op(f"sum_{kind}", field))

    def min(self, field: int, kind: str = "i64") -> "DataStreamResult":
        return DataStreamResult(self, self._op(f"min_{kind}", field))

    def max(self, field: int, kind: str = "i64") -> "DataStreamResult":
        return DataStreamResult(self, self._op(f"max_{kind}", field))

    # reduce / aggregate with a window function (WindowedStream.java:224-276, 342-526): the
    # pre-aggregated result of each fired window goes through window_function(key, (start, end),
    # [result], out); `reduce` names the built-in ReduceFunction of the closed set ("sum_i64", ...)
    def reduce(self, function: str, field: int, window_function: Optional[Callable] = None) -> "DataStreamResult":
        return DataStreamResult(self, self._op(function, field, window_function=window_function))

    def process(self, function: str, field: Optional[int], window_function: Callable) -> "DataStreamResult":
        """aggregate(AggregateFunction, ProcessWindowFunction) with the closed-set aggregate."""
        return DataStreamResult(self, self._op(function, field, window_function=window_function))

    # WindowedStream.minBy / maxBy (:725-771): the element with the smallest / largest field,
    # the first of equal ones (first=True) or the last
    def min_by(self, field: int, first: bool = True, kind: str = "i64") -> "DataStreamResult":
        return DataStreamResult(self, self._op(f"min_{kind}", field, N.FLAG_BY_FIELD | (0 if first else N.FLAG_BY_LAST)))

    def max_by(self, field: int, first: bool = True, kind: str = "i64") -> "DataStreamResult":
        return DataStreamResult(self, self._op(f"max_{kind}", field, N.FLAG_BY_FIELD | (0 if first else N.FLAG_BY_LAST)))

    minBy = min_by
    maxBy = max_by

    def aggregate(self, function: str, field: Optional[int] = None,
                  window_function: Optional[Callable] = None) -> "DataStreamResult":
        return DataStreamResult(self, self._op(function, field, window_function=window_function))

    def count(self) -> "DataStreamResult":
        return DataStreamResult(self, self._op("count", None))


class DataStreamResult:
    def __init__(self, ws: WindowedStream, op: GpuWindowOperator):
        self.ws, self.op = ws, op

    def execute_and_collect(self) -> list:
        """Run the bounded source through the operator, like env.execute() on a MiniCluster
        with parallelism 1; returns the fired StreamRecords (watermarks dropped)."""
        env = self.ws.keyed.env
        out = []
        with self.op:
            for el in env.elements:
                if isinstance(el, Watermark):
                    self.op.process_watermark(el)
                else:
                    self.op.process_element(el)
            self.op.end_input()
            out = [r for r in self.op.get_output() if isinstance(r, StreamRecord)]
        return out


class KeyedStream:
    def __init__(self, env, key_selector):
        self.env, self.key_selector = env, key_selector

    def window(self, assigner: WindowAssigner) -> WindowedStream:
        return WindowedStream(self, assigner)

    def count_window(self, size: int, slide: Optional[int] = None) -> WindowedStream:
        """KeyedStream.countWindow (KeyedStream.java:676-690)."""
        return WindowedStream(self, CountWindows(size, slide))

    countWindow = count_window


class DataStream:
    def __init__(self, env):
        self.env = env

    def key_by(self, key_selector) -> KeyedStream:
        return KeyedStream(self.env, key_selector)

    keyBy = key_by


class StreamExecutionEnvironment:
    """Minimal local environment: a bounded, timestamped source (list of StreamRecord and
    Watermark elements) feeding one GPU window operator."""

    def __init__(self, **op_kwargs):
        self.elements: list = []
        self.op_kwargs = op_kwargs

    @staticmethod
    def get_execution_environment(**op_kwargs) -> "StreamExecutionEnvironment":
        return StreamExecutionEnvironment(**op_kwargs)

    def from_elements(self, elements: Iterable) -> DataStream:
        self.elements = list(elements)
        return DataStream(self)


# Keyed snapshot: a gw_snapshot blob plus its key table (id -> key), what the Java operator
# writes per key group (the blob, then the keys through the key serializer).
KEYED_MAGIC = b"GWK1"


def pack_keyed_snapshot(blob: bytes, keys: dict) -> bytes:
    out = [KEYED_MAGIC, struct.pack("<qq", len(blob), len(keys)), blob]
    for kid, key in sorted(keys.items()):
        if isinstance(key, str):
            tag, body = b"s", key.encode("utf-8")
        elif isinstance(key, bool):
            tag, body = b"z", b"\x01" if key else b"\x00"
        elif isinstance(key, int):
            tag, body = b"j", struct.pack("<q", key)
        else:
            raise TypeError(f"unsupported key type {type(key).__name__}")
        out.append(struct.pack("<q", kid) + tag + struct.pack("<i", len(body)) + body)
    return b"".join(out)


def unpack_keyed_snapshot(data: bytes):
    if data[:4] != KEYED_MAGIC:
        raise ValueError("not a keyed snapshot")
    nb, nk = struct.unpack_from("<qq", data, 4)
    p = 20
    blob = data[p:p + nb]
    p += nb
    keys = {}
    for _ in range(nk):
        kid, = struct.unpack_from("<q", data, p)
        tag = data[p + 8:p + 9]
        ln, = struct.unpack_from("<i", data, p + 9)
        body = data[p + 13:p + 13 + ln]
        p += 13 + ln
        keys[kid] = body.decode("utf-8") if tag == b"s" else (body == b"\x01" if tag == b"z" else
                                                               struct.unpack("<q", body)[0])
    if p != len(data):
        raise ValueError("trailing bytes in a keyed snapshot")
    return blob, keys


def result_value(bits: int, is_double: bool):
    if is_double:
        return struct.unpack("<d", struct.pack("<q", int(bits)))[0]
    return int(bits)
