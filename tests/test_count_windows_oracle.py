"""Count windows, CPU side: the oracle's element-list restatement
(oracle/flink_oracle.c count_process_element) against the reference's golden vector
(EvictingWindowOperatorTest.testCountTrigger, tests/golden/count_windows.json) and against
an independent pure-Python restatement of CountTrigger + CountEvictor / PurgingTrigger."""
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
KEYS = {"key1": 1, "key2": 2}


def golden():
    return json.load(open(os.path.join(HERE, "golden", "count_windows.json")))["tests"]


@pytest.mark.parametrize("case", golden(), ids=lambda c: c["name"])
def test_oracle_count_windows_golden(oracle_lib, case):
    op = oracle_lib.OracleOperator(oracle_lib.make_config(**case["config"]))
    expected = []
    got = []
    for g in case["groups"]:
        keys = np.array([KEYS[k] for k, _ in g["elements"]], dtype=np.int64)
        vals = np.array([v for _, v in g["elements"]], dtype=np.int64)
        op.process_batch(keys, np.zeros_like(keys), vals)
        k, s, e, r = op.drain()
        got += list(zip(k.tolist(), r.tolist()))
        expected += [(KEYS[k], v) for k, v in g["expected"]]
        assert sorted(got) == sorted(expected)
    op.process_watermark((1 << 63) - 1)  # GlobalWindows: MAX_WATERMARK fires nothing
    assert len(op.drain()[0]) == 0


def py_count_windows(keys, vals, size, slide, agg):
    """CountTrigger.onElement + (CountEvictor.evictBefore | PurgingTrigger), element by element."""
    state = {}
    rows = []
    for k, v in zip(keys.tolist(), vals.tolist()):
        st = state.setdefault(k, {"trig": 0, "total": 0, "vals": []})
        st["vals"].append(v)
        st["total"] += 1
        st["trig"] += 1
        if st["trig"] < (slide if slide else size):
            continue
        st["trig"] = 0
        if slide:
            st["vals"] = st["vals"][-size:]
        w = st["vals"]
        if agg == "count":
            r = len(w)
        elif agg == "sum_i64":
            r = (sum(w) + (1 << 63)) % (1 << 64) - (1 << 63)
        elif agg == "min_i64":
            r = min(w)
        elif agg == "max_i64":
            r = max(w)
        else:
            raise ValueError(agg)
        rows.append((k, st["total"] - len(w), st["total"], r))
        if not slide:
            st["vals"] = []
    return rows


CONFIGS = [(5, None), (4, 2), (250, 150), (3, 5), (1, None), (6, 4)]


@pytest.mark.parametrize("size,slide", CONFIGS)
@pytest.mark.parametrize("agg", ["count", "sum_i64", "min_i64", "max_i64"])
def test_oracle_count_windows_match_python(oracle_lib, size, slide, agg):
    rng = np.random.default_rng(size * 31 + (slide or 0))
    n = 4000 if size < 100 else 30000
    keys = rng.integers(0, 7, n).astype(np.int64)
    vals = rng.integers(-1000, 1000, n).astype(np.int64)
    kw = dict(assigner="count_sliding" if slide else "count_tumbling", size=size, slide=slide or size, agg=agg)
    op = oracle_lib.OracleOperator(oracle_lib.make_config(**kw))
    op.process_batch(keys, np.zeros_like(keys), vals)
    k, s, e, r = op.drain()
    assert list(zip(k.tolist(), s.tolist(), e.tolist(), r.tolist())) == py_count_windows(keys, vals, size, slide, agg)
