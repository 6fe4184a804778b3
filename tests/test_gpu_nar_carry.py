"""The nar2 carry (gw_runtime.cpp flush_buffer): on a narrow two-pass table a
fire's flush applies only the ring positions the fire needs and keeps the other positions'
P2-bucketed records in a second output set until the next flush.  Every path that reads or
reshapes the table applies them first.  Against the oracle, with carry on (this process) and
carry off (GW_NAR_CARRY=0, a child process running the same scenario), bit-exact:

* a snapshot taken after each fire (records carried), restored into a fresh operator that
  finishes the stream beside an oracle restored from the oracle's snapshot at the same point;
* a table that grows (and regions that spill) while records are carried: a
  2^19-slot table (1.5M key ids, ~400K live per window);
* early batches whose records are older than the ring base (the first fires move the base
  backwards: records of the second batch precede the first's).
Both runs' rows hash to the same value (oracle.rows_hash_sum)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from flink_amd import _native as N
from flink_amd import windowing as W

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KW = dict(assigner="sliding", size=2000, slide=500, agg="sum_i64")
SNAP_AT = (7, 13)


def stream():
    rng = np.random.default_rng(53)
    nb, batches_n = 60_000, 20
    n = nb * batches_n
    keys = rng.integers(0, 1_500_000, n).astype(np.int64)
    ts = 5_000 + np.arange(n, dtype=np.int64) * 250 // nb - rng.integers(0, 200, n)
    ts[nb:2 * nb] -= 2_500  # the second batch precedes the first: older than the ring base
    vals = rng.integers(-(10 ** 6), 10 ** 6, n).astype(np.int64)
    batches = []
    for b in range(batches_n):
        lo, hi = b * nb, (b + 1) * nb
        wm = int(ts[:hi].max()) - 300 - 1 if b >= 2 else W.LONG_MIN
        batches.append((lo, hi, wm))
    return keys, ts, vals, batches


def rows_of(op):
    k, s, e, r = op.drain()
    return np.stack([k, s, e, r.view(np.int64)], axis=1)


def ora_rows(ora):
    return np.stack(ora.drain()[:4], axis=1).astype(np.int64)


def sort_rows(parts):
    a = np.concatenate(parts) if parts else np.zeros((0, 4), np.int64)
    return a[np.lexsort(a.T[::-1])]


class _NoOracle:
    """Stands in for the oracle in the carry-off child: its rows are compared by digest with
    the parent's, which checked them against the oracle."""

    def __getattr__(self, name):
        return lambda *a, **k: None

    def drain(self):
        return [np.zeros(0, np.int64)] * 4

    late_dropped = 0


def run_scenario(with_oracle=True):
    """-> (rows of the uninterrupted run, rows of each restored continuation, the oracle's
    rows for both, late counts, formats seen)."""
    from oracle import oracle as O
    keys, ts, vals, batches = stream()
    mk = lambda: W.GpuWindowOperator(W.SlidingEventTimeWindows.of(2000, 500), "sum_i64", capacity_hint=300_000,
                                     flags=N.FLAG_FORCE_REGION).open()
    op = mk()
    new_ora = (lambda: O.OracleOperator(O.make_config(**KW))) if with_oracle else _NoOracle
    ora = new_ora()
    g, o, fmts, snaps = [], [], [], {}
    for b, (lo, hi, wm) in enumerate(batches):
        op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
        ora.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
        fmts.append(op.stats()["region_format"])
        op.advance_watermark(wm)
        ora.process_watermark(wm)
        g.append(rows_of(op))
        o.append(ora_rows(ora))
        if b in SNAP_AT:
            snaps[b] = (op.snapshot_state(), ora.snapshot())
    op.advance_watermark(W.LONG_MAX)
    ora.process_watermark(W.LONG_MAX)
    g.append(rows_of(op))
    o.append(ora_rows(ora))
    late = (op.num_late_records_dropped, ora.late_dropped)
    st = op.stats()
    op.close()
    ora.close()
    cont = []
    for b, (blob, oblob) in snaps.items():
        op2 = mk()
        op2.initialize_state(blob)
        ora2 = new_ora()
        ora2.restore(oblob)
        g2, o2 = [], []
        for lo, hi, wm in batches[b + 1:]:
            op2.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
            ora2.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
            op2.advance_watermark(wm)
            ora2.process_watermark(wm)
            g2.append(rows_of(op2))
            o2.append(ora_rows(ora2))
        op2.advance_watermark(W.LONG_MAX)
        ora2.process_watermark(W.LONG_MAX)
        g2.append(rows_of(op2))
        o2.append(ora_rows(ora2))
        cont.append((sort_rows(g2), sort_rows(o2), op2.num_late_records_dropped, ora2.late_dropped))
        op2.close()
        ora2.close()
    return sort_rows(g), sort_rows(o), late, fmts, st, cont


def digest(rows):
    a = np.asarray(rows, np.int64).reshape(-1, 4)
    return [int(a.shape[0]), int((a * np.array([3, 5, 7, 11], np.int64)).sum())]


def check(res, with_oracle=True):
    g, o, late, fmts, st, cont = res
    if with_oracle:
        assert late[0] == late[1]
        assert np.array_equal(g, o) and len(g) > 0
    assert 2 in fmts  # narrow records
    assert st["rehashes"] > 0  # the table grew under the stream
    for g2, o2, l2, lo2 in cont:
        if not with_oracle:
            continue
        assert l2 == lo2
        assert np.array_equal(g2, o2) and len(g2) > 0
    return {"rows": digest(g), "cont": [digest(c[0]) for c in cont]}


def test_carry_snapshot_growth_and_early_rebase(oracle_lib):
    mine = check(run_scenario())
    env = dict(os.environ, GW_NAR_CARRY="0")
    code = ("import json, sys; sys.path.insert(0, %r); sys.path.insert(0, %r); "
            "import test_gpu_nar_carry as t; print('RESULT', json.dumps(t.check(t.run_scenario(False), False)))"
            % (ROOT, os.path.join(ROOT, "tests")))
    p = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=None,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-3000:]
    other = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")][-1][7:])
    assert other == mine  # carry on and carry off: the same rows
