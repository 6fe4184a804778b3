"""Throughput of the BASELINE.json configs other than the headline (bench.py measures
Nexmark Q5), one GPU, synthetic data generated in HBM, with the oracle ("port") timed on
the host cores over a bounded prefix of the same stream.  One JSON line per config.

    python scripts/configs_bench.py [--only ysb,q7,sessions,wordcount] [--steps 10]

  wordcount  WindowWordCount (flink-examples-streaming .../windowing/WindowWordCount.java:
             121-149): tokens keyed by word (String.hashCode of Zipf(1.1) words over a 50k
             vocabulary), countWindow(250, 150).sum(1)
  ysb        Yahoo Streaming Benchmark shape (streaming-benchmarks AdvertisingTopologyNative):
             events (ad_id, event_type, event_time) over 1000 ads of 100 campaigns (10 ads
             each), filter(event_type == "view") (1/3 of the events), project + join
             ad_id -> campaign_id (the Redis lookup, a device gather here), keyBy(campaign)
             10 s tumbling count; ts 1 ms per 100k events, disorder <= 50 ms, watermark every
             200 ms.  The filter and the join run on the GPU inside the timed region; `value`
             counts raw events (before the filter), `operator_events` the window operator's
  q7         Nexmark Q7/Q8 shape at one GPU: 10M keys, 10 s tumbling max(price)
  q7_first   the same stream as a positional max(2) on Tuple3<auction, bidder, price>: rows
             carry the window's first bid's bidder (GW_FLAG_FIRST_ELEMENT; no CPU baseline,
             the oracle has no first-element rows)
  q7_maxby   the same stream as maxBy(2) on Tuple3<auction, bidder, price>: rows carry the
             highest bid itself, the first of equal prices (GW_FLAG_BY_FIELD)
  sessions   event-time sessions, gap 10 s, avg(f64) over 12.5M keys (one GPU's share of
             100M keys on 8 GPUs); keys come in four groups, each active 5 s out of 20 s, so
             sessions close and fire
"""
import argparse
import gc
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import MASK63, splitmix64  # noqa: E402
from flink_amd import _native as N  # noqa: E402
from flink_amd import windowing as W  # noqa: E402


def gen(name, nb, steps, dev):
    """Returns (assigner kwargs, agg, keys, ts, vals, watermarks)."""
    n = nb * steps
    idx = torch.arange(n, device=dev, dtype=torch.int64)
    r = splitmix64(idx, 0x5EED0000 + {"wordcount": 1, "ysb": 2, "q7": 7, "q7_first": 7, "q7_maxby": 7, "sessions": 5}[name]) & MASK63
    if name == "wordcount":
        rng = np.random.default_rng(7)
        vocab = 50_000
        hashes = np.array([W.java_string_hash(f"word{i}") for i in range(vocab)], dtype=np.int64)
        p = 1.0 / np.arange(1, vocab + 1) ** 1.1
        cdf = torch.from_numpy(np.cumsum(p / p.sum())).to(dev)
        u = (r % (1 << 53)).to(torch.float64) / float(1 << 53)
        ranks = torch.searchsorted(cdf, u).clamp_(max=vocab - 1)
        keys = torch.from_numpy(hashes).to(dev)[ranks]
        ts = torch.zeros(n, dtype=torch.int64, device=dev)
        vals = torch.ones(n, dtype=torch.int64, device=dev)
        wms = [0] * steps
        return dict(assigner="count_sliding", size=250, slide=150), "sum_i32", keys, ts, vals, wms
    if name == "ysb":
        # raw events: ad index into the 1000-ad table and event type (0 = view, 1 = click,
        # 2 = purchase); the campaign ids are random 64-bit ids like YSB's UUIDs
        ad = r % 1000
        etype = (splitmix64(idx, 76) & MASK63) % 3
        base = idx // 100_000
        ts = base - (splitmix64(idx, 77) & MASK63) % 51
        wms = [int((b + 1) * nb // 100_000) - 50 - 1 for b in range(steps)]
        campaigns = splitmix64(torch.arange(100, device=dev, dtype=torch.int64), 0xCA11) & MASK63
        ad_campaign = campaigns.repeat_interleave(10)  # ad i belongs to campaign i // 10
        return dict(assigner="tumbling", size=10_000), "count", (ad, etype, ad_campaign), ts, None, wms
    if name in ("q7", "q7_first", "q7_maxby"):
        keys = r % 10_000_000
        base = idx * 200 // nb
        ts = base - (splitmix64(idx, 78) & MASK63) % 101
        vals = (splitmix64(idx, 79) & MASK63) % 1_000_000
        wms = [int((b + 1) * 200) - 100 - 1 for b in range(steps)]
        return dict(assigner="tumbling", size=10_000), "max_i64", keys, ts, vals, wms
    if name == "sessions":
        K = 12_500_000
        base = idx * 200 // nb
        group = (base // 5000) % 4
        keys = group * (K // 4) + r % (K // 4)
        ts = base - (splitmix64(idx, 80) & MASK63) % 101
        vals = ((splitmix64(idx, 81) & MASK63) % 1_000_000).to(torch.float64) / 1000.0
        wms = [int((b + 1) * 200) - 100 - 1 for b in range(steps)]
        return dict(assigner="session", gap=10_000), "avg_f64", keys, ts, vals.view(torch.int64), wms
    raise ValueError(name)


def run(name, args, dev):
    nb = {"wordcount": 2_000_000, "ysb": 20_000_000, "q7": 10_000_000, "q7_first": 10_000_000,
          "q7_maxby": 10_000_000, "sessions": 10_000_000}[name]
    n_timed = args.steps or {"wordcount": 10, "ysb": 60, "q7": 60, "q7_first": 60, "q7_maxby": 60, "sessions": 100}[name]
    steps = args.warmup + n_timed
    kw, agg, keys, ts, vals, wms = gen(name, nb, steps, dev)
    torch.cuda.synchronize()
    assigner = {"tumbling": lambda: W.TumblingEventTimeWindows.of(kw["size"]),
                "session": lambda: W.EventTimeSessionWindows.with_gap(kw["gap"]),
                "count_sliding": lambda: W.CountWindows.of(kw["size"], kw["slide"])}[kw["assigner"]]()
    cap = {"wordcount": 1 << 16, "ysb": 1024, "q7": 10_000_000, "q7_first": 10_000_000, "q7_maxby": 10_000_000,
           "sessions": 12_500_000}[name]
    first = name in ("q7_first", "q7_maxby")
    op = W.GpuWindowOperator(assigner, agg, capacity_hint=cap, max_batch=nb * 2,
                             flags=(N.FLAG_BY_FIELD if name == "q7_maxby" else N.FLAG_FIRST_ELEMENT) if first else 0).open()
    payload = (splitmix64(torch.arange(keys.numel(), device=dev, dtype=torch.int64), 82) & MASK63) if first else None
    rows = 0
    op_events = 0
    ysb = name == "ysb"
    if ysb:
        ad, etype, ad_campaign = keys
        side = torch.cuda.Stream(device=dev)
        ysb_k = torch.empty(nb, dtype=torch.int64, device=dev)  # the selected batch (device select)
        ysb_t = torch.empty(nb, dtype=torch.int64, device=dev)

    def step(b):
        nonlocal rows, op_events
        lo, hi = b * nb, (b + 1) * nb
        if ysb and args.ysb_select == "device":
            # filter(view) -> project -> join(ad -> campaign) fused on the device, on the
            # operator's stream (gw_select_lookup_device: one read of the columns, the view
            # events written in arrival order; the call returns their number)
            n = W.select_lookup_device(etype[lo:hi], 0, ad[lo:hi], ad_campaign, ts[lo:hi], ysb_k, ysb_t, op.stream())
            N.check(N.lib().gw_ingest_device(op.handle, n, ysb_k.data_ptr(), None, ysb_t.data_ptr(), None,
                                             op.stream()), op.handle)
            op_events += n
        elif ysb:  # the same with torch on a stream of its own: the view events' indices once (one
            # stream compaction and its host sync), then the gathers
            with torch.cuda.stream(side):
                idx = torch.nonzero(etype[lo:hi] == 0).squeeze(1)
                k = ad_campaign[ad[lo:hi][idx]]
                t = ts[lo:hi][idx]
            n = k.numel()
            side.synchronize()
            N.check(N.lib().gw_ingest_device(op.handle, n, k.data_ptr(), None, t.data_ptr(), None, op.stream()),
                    op.handle)
            op_events += n
        elif first:
            op.process_batch_payload_device(keys[lo:hi], ts[lo:hi], vals[lo:hi], payload[lo:hi],
                                            stream=torch.cuda.current_stream(dev).cuda_stream)
            op_events += nb
        else:
            N.check(N.lib().gw_ingest_device(op.handle, nb, keys[lo:hi].data_ptr(), None, ts[lo:hi].data_ptr(),
                                             vals[lo:hi].data_ptr() if vals is not None else None, op.stream()),
                    op.handle)
            op_events += nb
        rows += op.advance_watermark(wms[b])
        rows += op.pending_rows() if kw["assigner"].startswith("count") else 0
        op.clear_rows()

    for b in range(args.warmup):
        step(b)
    op.flush()
    torch.cuda.synchronize()
    rows = 0
    op_events = 0
    op.enable_kernel_timing(True)
    for w in range(3):
        op.kernel_time_ms(w)  # reset
    merges0 = op.stats().get("session_merges", 0)
    t0 = time.perf_counter()
    for b in range(args.warmup, steps):
        step(b)
    op.flush()
    op.synchronize()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kt = [op.kernel_time_ms(w) for w in range(3)]  # (avg ms, launches): ingest, fire, flush/apply
    stats = op.stats()
    op.close()
    merges = stats.get("session_merges", 0) - merges0
    roof = roofline(name, kw, agg, keys, ts, nb, args.warmup, steps, op_events, rows, kt, dt, merges)
    out = {"config": name, "window": kw, "aggregate": agg, "events_per_step": nb, "steps": n_timed,
           "value": nb * n_timed / dt, "unit": "events/s", "ms_per_step": dt * 1e3 / n_timed,
           "operator_events_per_s": op_events / dt,
           "rows_fired": rows, "live_keys": stats.get("live_keys"), "data": "synthetic, generated in HBM",
           "roofline": roof}
    if ysb:
        out["pipeline"] = ("filter(event_type == view) + join(ad_id -> campaign_id) on the GPU ("
                           + ("gw_select_lookup_device" if args.ysb_select == "device" else "torch") + "), then the operator")
    if first:
        out["note"] = ("rows carry the highest bid's payload (one MAX pane operator + 4-column log + per-fire probe)"
                       if name == "q7_maxby" else
                       "rows carry the first element's payload (two pane operators + payload log + join)")
    if not args.no_cpu_baseline and not first:
        if ysb:  # the oracle times the window operator on the filtered, joined stream
            ad, etype, ad_campaign = keys
            view = etype == 0
            keys_o, ts_o = ad_campaign[ad[view]], ts[view]
            cum = torch.cumsum(view.view(-1, nb).sum(1), 0).tolist()
            nb_o = int(cum[0])  # first batch's size (batches are ~nb/3 each)
            blen = view.view(-1, nb).sum(1)
            out["cpu_baseline"] = cpu_baseline(kw, agg, keys_o, ts_o, None, wms, blen, args.cpu_seconds, few_keys=True)
            out["cpu_baseline"]["note"] = "oracle operator over the filtered + joined stream, events after the filter"
        else:
            blen = torch.full((steps,), nb, dtype=torch.int64)
            out["cpu_baseline"] = cpu_baseline(kw, agg, keys, ts, vals, wms, blen, args.cpu_seconds)
    return out


HBM_PEAK_GBS = 8000.0
# What bounds each config at the round's code, and the next kernel target.
BOUND_NOTE = {
    "sessions": "slot sort path: k_sess_prep (one table probe per record), the hand-written radix sort of "
                "(slot, arrival) (gw_sort.hip), k_sess_segment (a key's records replayed in arrival order, one "
                "16-B record gather each and a slot-line read-modify-write per key)",
    "q7": "region pipeline as in the headline (pass 1 + flush), fire at each 10-s window end",
    "q7_first": "two pane operators + the payload log and join",
    "q7_maxby": "MAX pane operator + 4-column log + per-fire probe (k_by_scan)",
    "ysb": "the filter / join ahead of the operator (gw_select_lookup_device) and the operator's few-key pre-aggregation (k_ingest_preagg)",
    "wordcount": "count-window replay (k_cnt_apply) over a Zipf vocabulary: hot keys serialise",
}


def roofline(name, kw, agg, keys, ts, nb, warm, steps, op_events, rows, kt, dt, merges=0):
    """HBM roofline of the operator over the timed steps: algorithmic bytes (SURVEY.md §8d:
    each event's input columns once, each distinct per-batch state entry read and written once,
    each fired row written once with its accumulator read, sessions + 3 S_acc per merge) over
    the operator's device time (HIP events on its stream: ingest + flush/apply + fire).  When
    those launches cover less than 90% of the step (first-element / maxBy handles run log,
    join and scan work beside them; YSB runs the torch filter ahead), frac is taken over the
    step's wall time instead, and frac_basis says which."""
    s_acc = 16 if agg.startswith("avg") else 8
    b_in = 16 if agg == "count" else 24  # key + ts (+ value)
    dsum = 0
    if name == "sessions":
        state = s_acc  # §8(d): S_acc per distinct (key, session) accumulator; + 3 S_acc per merge
        for b in range(warm, steps):
            dsum += int(torch.unique(keys[b * nb:(b + 1) * nb]).numel())
    elif name == "wordcount":
        state = 8 * (2 + kw["size"] // int(np.gcd(kw["size"], kw["slide"])))  # key, meta, the pane ring
        for b in range(warm, steps):
            dsum += int(torch.unique(keys[b * nb:(b + 1) * nb]).numel())
    elif name == "ysb":
        state = s_acc
        dsum = None  # <= 100 campaigns x 2 windows per batch: negligible
    else:
        state = s_acc
        size = kw["size"]
        for b in range(warm, steps):
            comp = keys[b * nb:(b + 1) * nb] * 4096 + ((ts[b * nb:(b + 1) * nb] // size) % 4096)
            dsum += int(torch.unique(comp).numel())
    alg = op_events * b_in + 2 * state * (dsum or 0) + rows * (32 + s_acc) + 3 * s_acc * merges
    dev_ms = sum(ms * n for ms, n in kt)
    share = dev_ms / 1e3 / dt if dt > 0 else 0.0
    basis_s = dev_ms / 1e3 if share >= 0.9 else dt
    achieved = alg / basis_s / 1e9 if basis_s > 0 else 0.0
    formula = f"events x {b_in} B + 2 x {state} B x distinct state entries per batch + rows x {32 + s_acc} B"
    if name == "sessions":
        formula += f" + 3 x {s_acc} B x session merges ({merges})"
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": None,
            "frac_basis": ("operator device time (HIP events)" if share >= 0.9 else
                           f"step wall time: the operator's timed launches are {share:.0%} of the step, not "
                           "the dominant cost"),
            "algorithmic_bytes": alg, "bytes_per_event": alg / max(op_events, 1),
            "formula": formula, "session_merges": merges if name == "sessions" else None,
            "device_ms_per_step": dev_ms / max(steps - warm, 1),
            "device_share_of_step": share,
            "launch_ms": {"ingest": kt[0], "fire": kt[1], "flush": kt[2]},
            "distinct_per_batch": (dsum / max(steps - warm, 1)) if dsum is not None else None,
            "bound_by": BOUND_NOTE.get(name)}


def cpu_baseline(kw, agg, keys, ts, vals, wms, blen, seconds, few_keys=False):
    """The oracle ("port") on the host cores over a bounded sample of the WHOLE timed stream,
    so the sample holds the stream's fires as the GPU's run does: every K-th key's records
    (key % K == 0), or, for a stream of few keys (YSB's 100 campaigns), every K-th record;
    K sized for ~`seconds` of CPU work.  blen: records per watermark batch."""
    from oracle import oracle as O
    from bench import host_cores
    O.build()
    threads = host_cores()[0]
    cfg = O.make_config(agg=agg, max_parallelism=128, **kw)
    blen = blen.to(keys.device)
    bidx = torch.repeat_interleave(torch.arange(blen.numel(), device=keys.device), blen)

    def go(k_sub, max_batches=None):
        nb_ = blen.numel() if max_batches is None else max_batches
        n_ = int(blen[:nb_].sum().item())
        sel = (keys[:n_] % k_sub == 0) if not few_keys else (torch.arange(n_, device=keys.device) % k_sub == 0)
        kk = keys[:n_][sel].cpu().numpy()
        t = ts[:n_][sel].cpu().numpy()
        v = vals[:n_][sel].cpu().numpy() if vals is not None else None
        bl = torch.bincount(bidx[:n_][sel], minlength=nb_).cpu().numpy().astype(np.int64)
        wm = np.array(wms[:nb_], np.int64)
        r, _, sec = O.run_parallel(cfg, threads, bl, wm, kk, t, v)
        return int(bl.sum()), sec, r

    total = int(blen.sum().item())
    n0, s0, _ = go(256, max_batches=min(blen.numel(), 4))
    rate = n0 / max(s0, 1e-6)
    k_sub = max(1, int(np.ceil(total / max(rate * seconds, 1.0))))
    n, sec, r = go(k_sub)
    what = f"every {k_sub}-th record" if few_keys else f"every {k_sub}-th key (key % {k_sub} == 0)"
    return {"value": n / sec, "unit": "events/s", "cores": threads, "kind": "port",
            "sample": f"{what} of the whole GPU stream ({blen.numel()} watermark batches, {n} events), then "
                      f"MAX_WATERMARK: {r} rows fired", "seconds": sec, "rows": r}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="wordcount,ysb,q7,sessions")
    ap.add_argument("--ysb-select", choices=["device", "torch"], default="device",
                    help="YSB's filter + ad -> campaign join: gw_select_lookup_device, or torch ops on a side stream")
    ap.add_argument("--steps", type=int, default=0,
                    help="timed steps (0: per config, long enough that windows / sessions fire: "
                         "wordcount 10, ysb and q7 60 (12 s of event time), sessions 100 (20 s))")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--cpu-seconds", type=float, default=3.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    for name in args.only.split(","):
        print(json.dumps(run(name, args, dev)), flush=True)
        # the previous config's stream (tens of GB) back to the device before the next one
        gc.collect()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
