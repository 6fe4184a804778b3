"""Shared test helpers: replay a reference harness test (tests/golden/operator_harness.json)
against an operator backend, the way KeyedOneInputStreamOperatorTestHarness drives
WindowOperator (processElement / processWatermark, then compare sorted output —
TestHarnessUtil.assertOutputEqualsSorted, flink-runtime/src/test/.../TestHarnessUtil.java:61)."""
import json
import os
import struct

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def config_kwargs(cfg):
    kw = dict(assigner=cfg["assigner"], size=cfg.get("size", 0), slide=cfg.get("slide", 0),
              offset=cfg.get("offset", 0), gap=cfg.get("gap", 0), lateness=cfg.get("lateness", 0),
              agg=cfg["agg"], trigger=cfg.get("trigger", "event_time"))
    if kw["assigner"] == "tumbling":
        kw["slide"] = kw["size"]
    return kw


class KeyDictionary:
    """String keys -> dense int64 ids (+ Java String.hashCode for key groups)."""

    def __init__(self):
        self.ids, self.names = {}, []

    def id(self, k):
        if k not in self.ids:
            self.ids[k] = len(self.names)
            self.names.append(k)
        return self.ids[k]


def bits_to_result(bits, is_double):
    if is_double:
        return struct.unpack("<d", struct.pack("<q", int(bits)))[0]
    return int(bits)


def replay(test, make_backend, is_double=False, side_output=False):
    """Drive a backend through one golden harness test; returns list of mismatches.
    side_output: run with the late-data side output (WindowedStream.sideOutputLateData) and
    compare it with the test's "side" records; without it those records are counted in
    numLateRecordsDropped ("late")."""
    keys = KeyDictionary()
    be = make_backend(test["config"], side_output=side_output) if side_output else make_backend(test["config"])
    errors = []
    pin_window = any(row[3] is not None for op in test["ops"] if op[0] == "w" for row in op[2])
    for op in test["ops"]:
        if op[0] == "e":
            _, k, v, ts = op
            be.process_element(keys.id(k), ts, v)
        elif op[0] == "snapshot":
            # testHarness.snapshot -> close -> new harness -> initializeState -> open
            # (WindowOperatorTest.java:169-177); backends without it just continue
            if hasattr(be, "snapshot_restore"):
                be.snapshot_restore()
        elif op[0] == "w":
            _, wm, expected = op
            be.process_watermark(wm)
            k, s, e, r = be.drain()
            got = sorted((keys.names[int(k[i])], bits_to_result(r[i], is_double), int(e[i]) - 1,
                          int(s[i]), int(e[i])) for i in range(len(k)))
            n_ = 5 if pin_window else 3
            g_cmp = sorted(g[:n_] for g in got)
            e_cmp = sorted(tuple(x)[:n_] for x in expected)
            if g_cmp != e_cmp:
                errors.append(f"wm {wm}: got {g_cmp} expected {e_cmp}")
    if side_output:
        k, t, v = be.drain_late()
        got = sorted((keys.names[int(k[i])], int(v[i]), int(t[i])) for i in range(len(k)))
        exp = sorted(tuple(x) for x in test["side"])
        if got != exp:
            errors.append(f"side output {got} expected {exp}")
        if be.late_dropped != 0:
            errors.append(f"late_dropped {be.late_dropped} != 0 with a side output")
    elif be.late_dropped != test.get("late", 0):
        errors.append(f"late_dropped {be.late_dropped} != {test.get('late', 0)}")
    return errors


# ---- the ITCase closed-form stream (EventTimeWindowCheckpointingITCase) --------------
# Generator :798-822: for seq s in [0, n): for key i in [0, keys): (i, s)@s; then
# watermark s - 4*elementsPerWindow/3.  Validator :749-771: window sum = sum of
# i in [start, min(end, n)) with i > 0.

def itcase_stream(num_keys, n, window):
    trailing = 4 * window // 3
    keys = np.tile(np.arange(num_keys, dtype=np.int64), n)
    ts = np.repeat(np.arange(n, dtype=np.int64), num_keys)
    batch_len = np.full(n, num_keys, dtype=np.int64)
    wm = np.arange(n, dtype=np.int64) - trailing
    return keys, ts, ts.copy(), batch_len, wm


def itcase_expected_sum(start, end, n):
    hi = min(end, n)
    lo = max(start, 1)
    if hi <= lo:
        return 0
    return (lo + hi - 1) * (hi - lo) // 2
