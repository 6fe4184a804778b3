#!/usr/bin/env python3
"""bench.py — events/sec of keyed sliding-window aggregation on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2], SURVEY.md §8d "Config 3"): Nexmark Q5 shape — keyBy(auction)
.window(SlidingEventTimeWindows.of(10 s, 2 s)) over 10M distinct keys, synthetic bids
(auction = splitmix64(i) mod 10M, value = splitmix64(i') mod 1e6), 100M events per 2-s pane
per GPU, bounded disorder 100 ms, a watermark every 200 ms of event time (= one step).
Aggregate defaults to SUM over int64 (the north star's "keyed sliding-window sum"); --agg count
gives the Q5 count.

One step = one watermark batch: (multi-GPU: partition by key group -> RCCL all-to-all) ->
gw_ingest_device -> gw_advance_watermark (fires every 10th step) -> fired rows consumed
(discarded, like the reference's DiscardingSink).  Inputs are pre-generated in HBM before
the timed region.  N GPUs = N processes, key groups sharded by
KeyGroupRangeAssignment.computeKeyGroupRangeForOperatorIndex, weak scaling (each rank
generates the same number of events over the full key space).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
INGEST_PATH = "region_buffered"  # the ingest pipeline a committed traffic.json must describe

C1 = -7046029254386353131   # 0x9E3779B97F4A7C15 as int64
C2 = -4658895280553007687   # 0xBF58476D1CE4E5B9
C3 = -7723592293110705685   # 0x94D049BB133111EB
MASK63 = (1 << 63) - 1


def splitmix64(idx: torch.Tensor, seed: int) -> torch.Tensor:
    """splitmix64(seed + (i+1)*golden) on int64 tensors (wrapping arithmetic)."""
    z = (idx + 1) * C1 + seed
    z = (z ^ ((z >> 30) & ((1 << 34) - 1))) * C2
    z = (z ^ ((z >> 27) & ((1 << 37) - 1))) * C3
    return z ^ ((z >> 31) & ((1 << 33) - 1))


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--agg", default="sum_i64")
    ap.add_argument("--keys", type=int, default=10_000_000)
    ap.add_argument("--events-per-pane", type=int, default=100_000_000, help="per GPU, per 2-s pane")
    ap.add_argument("--size-ms", type=int, default=10_000)
    ap.add_argument("--slide-ms", type=int, default=2_000)
    ap.add_argument("--wm-interval-ms", type=int, default=200)
    ap.add_argument("--disorder-ms", type=int, default=100)
    ap.add_argument("--exchange", choices=["a2a", "none"], default="a2a",
                    help="a2a: libgpuwin's RCCL keyBy exchange (gw_exchange_*); none: each rank generates "
                         "records of its own key groups only")
    ap.add_argument("--pack", choices=["auto", "unpack", "off"], default="auto",
                    help="auto: the exchange ships records that fit as 8-byte words (gw_exchange_enable_packing; "
                         "integer aggregates) and pass 1 decodes them (gw_ingest_packed_device); unpack: the "
                         "receiver unpacks them to columns first; off: every record as 24 B")
    ap.add_argument("--exchange-stream", choices=["own", "operator"], default="own",
                    help="own: the exchange (partition, all-to-all, sends) on a stream of its own, overlapping "
                         "the operator's kernels; operator: on the operator's stream, serialised with them")
    ap.add_argument("--exchange-ahead", type=int, choices=[1, 2], default=1,
                    help="batches the exchange finishes ahead of the ingest: 1 finishes batch b right before "
                         "its ingest (and begins b+1); 2 finishes b+1 (and begins b+2) before batch b is "
                         "ingested and its watermark fires, so the exchange stream has work queued while the "
                         "fire's flush holds the operator's stream; measured the same as 1 (profiles/r6/exchange/driver/)")
    ap.add_argument("--force-exchange", action="store_true",
                    help="run the RCCL exchange path at N = 1 too (a one-rank communicator: every record comes "
                         "back to this rank) -- a check of the N > 1 code path on one GPU")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-fed", action="store_true",
                    help="skip the host-fed leg (gw_ingest from host columns: pinned staging + H2D)")
    ap.add_argument("--host-fed-steps", type=int, default=21,
                    help="batches of the host-fed leg: the first fire cycle (10) untimed, as a running job's "
                         "buffers are grown by then; the other 11 include a 10M-row fire and drain")
    ap.add_argument("--preagg", choices=["auto", "force", "off"], default="auto")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="no HIP events around the kernels (the roofline fields are then null)")
    ap.add_argument("--checksum", action="store_true",
                    help="drain the fired rows of every step to the host and report the oracle's "
                         "order-independent row checksum (oracle.rows_hash_sum) summed over steps and ranks "
                         "(a check, not a bench setting)")
    ap.add_argument("--oracle-check", action="store_true",
                    help="with --checksum at N=1: also run the CPU oracle over the same stream and report "
                         "per-watermark agreement (short runs only: the oracle does ~1-2M events/s)")
    return ap.parse_args(argv)


def make_stream(nb, steps_total, K, E, slide, disorder, agg, dev, rank=0, world=1, key_partitioned=False,
                maxp=128, t_shift=0):
    """The bench's synthetic Nexmark-Q5 bids in HBM: steps_total watermark batches of nb
    events.  auction = splitmix64(i) mod K (uniform), ts advancing so each `slide` of event
    time holds E events with jitter <= disorder, value = splitmix64(i') mod 1e6.  With
    key_partitioned (N > 1, no exchange) the keys are drawn from this rank's key groups only
    (KeyGroupRangeAssignment.computeKeyGroupRangeForOperatorIndex), so every rank keeps the
    same nb, timestamps and watermarks.  Returns (keys, ts, vals or None, wms): the watermark
    after batch b is BoundedOutOfOrdernessWatermarks' maxTs - bound - 1 over the un-jittered
    maximum, identical on every rank.  t_shift (ms) moves the event-time origin back: the
    watermark of batch b then completes windows where batch b + t_shift / interval would have."""
    from flink_amd import _native as N
    n_all = nb * steps_total
    idx = torch.arange(n_all, device=dev, dtype=torch.int64)
    seed = 0x5EED0005 + 7919 * rank
    draw = splitmix64(idx, seed) & MASK63
    if key_partitioned and world > 1:
        allk = torch.arange(K, device=dev, dtype=torch.int64)
        kg = torch.empty(K, dtype=torch.int32, device=dev)
        owner = torch.empty_like(kg)
        N.check(N.lib().gw_key_groups_device(K, allk.data_ptr(), None, maxp, world, kg.data_ptr(),
                                             owner.data_ptr(), None))
        torch.cuda.synchronize()
        own = allk[owner == rank]
        keys = own[draw % own.numel()]
        del allk, kg, owner, own
    else:
        keys = draw % K
    del draw
    t0_ms = 1_700_000_000_000 - t_shift
    jitter = (splitmix64(idx, seed ^ 0x77) & MASK63) % (disorder + 1)
    ts = t0_ms + (idx * slide) // E - jitter
    vals = None
    if agg != "count":
        v = (splitmix64(idx, seed ^ 0x1234) & MASK63) % 1_000_000
        vals = v.to(torch.float64).view(torch.int64) if agg.endswith("f64") else v
    del idx, jitter
    wms = [t0_ms + (((b + 1) * nb - 1) * slide) // E - disorder - 1 for b in range(steps_total)]
    torch.cuda.synchronize()
    return keys, ts, vals, wms


def make_operator(W, N, args, K, world=1, rank=0, local=0, nb=None):
    """The bench's operator: one GpuWindowOperator subtask over this rank's key groups."""
    flags = {"auto": 0, "force": N.FLAG_FORCE_LDS_PREAGG, "off": N.FLAG_NO_LDS_PREAGG}[args.preagg]
    return W.GpuWindowOperator(W.SlidingEventTimeWindows.of(args.size_ms, args.slide_ms), args.agg,
                               capacity_hint=max(K // world, 1024), max_parallelism=128, parallelism=world,
                               operator_index=rank, device=local, flags=flags, max_batch=nb * 2).open()


class Steps:
    """One step = one watermark batch: (N > 1: the keyBy exchange, pipelined one batch ahead --
    gw_exchange_begin of batch b + 1 (partition + the all-to-all of (count, watermark, columns)),
    then gw_exchange_finish of batch b (its one host wait + grouped send/receive)) ->
    gw_ingest_device -> gw_advance_watermark (fires every 10th step) -> fired rows consumed.
    With `collect` the rows of every watermark are drained to the host and (count, checksum)
    recorded."""

    def __init__(self, op, N, keys, ts, vals, wms, nb, ex=None, collect=False, ex_stream=None, keep_rows=False,
                 ahead=1):
        import ctypes
        self.op, self.N, self.ex, self.ex_stream = op, N, ex, ex_stream
        self.keys, self.ts, self.vals, self.wms, self.nb = keys, ts, vals, wms, nb
        self.collect = collect
        self.per_wm = []  # (rows, checksum) per watermark when collecting
        self.keep_rows = keep_rows  # collect: also keep every watermark's rows (tests' row diff)
        self.rows = []
        self.exch_bytes = 0
        self.begun = -1  # the last batch whose exchange has begun
        self.finished = -1  # ... and finished (its receive columns in self.ready until ingested)
        self.ready = {}
        self.ahead = ahead
        # the host side of a step stays lean (the GPU runs a batch in ~70 us): the library's entry
        # points and each batch's device column pointers resolved once, before any clock
        L = N.lib()
        self._ingest, self._advance, self._clear = L.gw_ingest_device, L.gw_advance_watermark, L.gw_clear_rows
        self._ingest_packed = L.gw_ingest_packed_device
        self._byref = ctypes.byref
        self._h, self._stream = op.handle, op.stream()
        self._fired = ctypes.c_int64(0)
        self._fired_ref = ctypes.byref(self._fired)
        es = keys.element_size()
        self._ptrs = [(keys.data_ptr() + b * nb * es, ts.data_ptr() + b * nb * es,
                       vals.data_ptr() + b * nb * es if vals is not None else None) for b in range(len(wms))]

    def _begin(self, b):
        nb = self.nb
        lo, hi = b * nb, (b + 1) * nb
        v = self.vals[lo:hi] if self.vals is not None else None
        self.ex.begin(self.keys[lo:hi], self.ts[lo:hi], v, stream=self.ex_stream, wm=self.wms[b])
        self.begun = b

    def _finish(self, timed, b_in, rank):
        """gw_exchange_finish of the oldest begun batch; its receive columns (and words) wait
        in self.ready until the batch is ingested."""
        n, pk, pt, pv, _, wmin, ist = self.ex.finish(self.ex_stream)
        if timed:  # bytes this rank sent to its peers (received packed share as the estimate)
            f = self.ex.last_packed() / max(self.nb, 1)
            self.exch_bytes += (self.nb - int(self.ex.counts()[0][rank])) * (8 * f + b_in * (1 - f))
        self.finished += 1
        self.ready[self.finished] = (n, pk, pt, pv, wmin, ist, self.ex.last_words())

    def step(self, b, timed=False, b_in=24, rank=0, last=None):
        """One batch; returns the rows its watermark fired.  last: the last batch of this phase
        (warmup / timed): the exchange begins and finishes batches up to it ahead of the ingest."""
        op, nb, N = self.op, self.nb, self.N
        if self.ex is not None:
            # the native exchange on a stream of its own; the ingest orders through the receive
            # set's hand-off stream, so later batches' partitions and transfers overlap batch b's
            # aggregation on the operator's stream.  Batches up to b + ahead - 1 are finished
            # (their transfers queued) and the one after is begun (partitioned, its counts
            # exchanged) before batch b is ingested: with ahead = 2 the exchange stream holds the
            # next batches' work while a firing watermark's flush and fire hold the operator.
            hi = b + self.ahead - 1
            if last is not None:
                hi = max(b, min(hi, last))
            bh = hi + 1 if (last is not None and hi + 1 <= last) else hi
            while self.finished < hi:  # (the exchange holds at most two begun, unfinished batches)
                while self.begun < min(self.finished + 2, bh):
                    self._begin(self.begun + 1)
                self._finish(timed, b_in, rank)
            while self.begun < bh and self.begun - self.finished < 2:
                self._begin(self.begun + 1)
            n, pk, pt, pv, wmin, ist, (nw, pw, geom) = self.ready.pop(b)
            if nw:  # words kept packed: pass 1 decodes them
                N.check(self._ingest_packed(self._h, n, pk, pt, pv, nw, pw, self._byref(geom), ist), self._h)
            else:
                N.check(self._ingest(self._h, n, pk, None, pt, pv, ist), self._h)
            wm = wmin
        else:
            # columns generated and synchronised before the clock: no producer ordering needed
            pk, pt, pv = self._ptrs[b]
            N.check(self._ingest(self._h, nb, pk, None, pt, pv, self._stream), self._h)
            wm = self.wms[b]
        N.check(self._advance(self._h, wm, self._fired_ref), self._h)
        fired = self._fired.value
        self.consume()
        return fired

    def consume(self):
        if self.collect:
            rows = self.op.drain()
            self.per_wm.append((len(rows[0]), rows_checksum(rows)))
            if self.keep_rows:
                self.rows.append(rows)
        else:
            self.N.check(self._clear(self._h), self._h)  # DiscardingSink


def main(argv=None):
    args = parse(argv)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world == 1 and args.gpus > 1:
        raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    from flink_amd import _native as N
    from flink_amd import windowing as W

    agg = args.agg
    size, slide = args.size_ms, args.slide_ms
    E = args.events_per_pane
    nb = E * args.wm_interval_ms // slide           # events per step per rank
    steps_total = args.warmup + args.steps
    K = args.keys
    maxp = 128
    b_in = 16 if agg == "count" else 24
    s_acc = 16 if agg.startswith("avg") else 8

    t_gen = time.time()
    # The stream's event-time origin is placed so that the last warmup batch's watermark fires:
    # the clock then starts right after a fire (and its flush), and every fire cycle inside the
    # timed steps is a whole cycle of slide / interval batches (a cycle cut by the start of the
    # clock would carry a flush over fewer batches than the steady state).
    t_shift = (args.warmup - 1) * args.wm_interval_ms if args.warmup >= 1 else 0
    keys, ts, vals, wms = make_stream(nb, steps_total, K, E, slide, args.disorder_ms, agg, dev, rank, world,
                                      key_partitioned=args.exchange == "none", maxp=maxp, t_shift=t_shift)
    log(f"rank {rank}: generated {nb * steps_total} events ({nb * steps_total * b_in / 1e9:.1f} GB) "
        f"in {time.time() - t_gen:.1f}s")

    op = make_operator(W, N, args, K, world, rank, local, nb)
    ex = None
    if (world > 1 and args.exchange == "a2a") or args.force_exchange:
        # the product path: libgpuwin's own RCCL exchange, what a JVM task drives;
        # torch.distributed only ships its communicator id and times the run
        from flink_amd.exchange import NativeKeyByExchange
        ex = NativeKeyByExchange(world, rank, max_parallelism=maxp, device=local)
        if args.pack != "off" and not agg.endswith("f64"):
            ex.enable_packing(size, slide, 0, with_values=agg != "count")
            ex.keep_words(args.pack == "auto")
    xs = torch.cuda.Stream(device=dev) if ex is not None and args.exchange_stream == "own" else None
    run = Steps(op, N, keys, ts, vals, wms, nb, ex=ex, collect=args.checksum,
                ex_stream=xs.cuda_stream if xs is not None else (op.stream() if ex is not None else None),
                ahead=args.exchange_ahead)

    # pass 1 timed on every 4th batch (all batches are alike): two event records per timed launch
    # cost host time between batches; the fire and flush timers run on every launch
    op.enable_kernel_timing(0 if args.no_kernel_timing else 4)
    for b in range(args.warmup):
        run.step(b, last=args.warmup - 1)
    op.flush()  # warmup batches still buffered are applied outside the timed region
    for w in (0, 1, 2):
        op.kernel_time_ms(w)  # reset timers after warmup
    st0 = op.stats()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    last = t0
    # Per fire cycle: a watermark that completes windows fires them and synchronises with
    # the device (gw_advance_watermark), so the host clock at the return of such a step
    # closes one cycle of batches + their fire.
    cycles = []
    cyc_t, cyc_steps = t0, 0
    for b in range(args.warmup, steps_total):
        fired = run.step(b, True, b_in, rank, last=steps_total - 1)
        cyc_steps += 1
        if fired:  # the watermark completed windows: gw_advance_watermark fired them and synchronised
            now = time.perf_counter()
            cycles.append({"steps": cyc_steps, "ms": (now - cyc_t) * 1e3,
                           "events_per_s": cyc_steps * nb / max(now - cyc_t, 1e-9)})
            cyc_t, cyc_steps = now, 0
            if rank == 0 and now - last > 30:
                last = now
                log(f"step {b - args.warmup + 1}/{args.steps}")
    op.flush()  # every timed batch is in the window state when the clock stops
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if cyc_steps:
        cycles.append({"steps": cyc_steps, "ms": (time.perf_counter() - cyc_t) * 1e3, "partial": True})
    if dist:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    ingest_ms, ingest_launches = op.kernel_time_ms(0)
    fire_ms, fire_launches = op.kernel_time_ms(1)
    apply_ms, apply_launches = op.kernel_time_ms(2)
    st1 = op.stats()
    events_rank = nb * args.steps
    rows_rank = st1["rows_fired"] - st0["rows_fired"]

    # ------------------------------------------ algorithmic bytes
    # D_b: distinct (key, pane) accumulators each timed batch touches.  Exact on the
    # rank's own generated batches (N=1: the ingested batch itself).
    g = int(np.gcd(size, slide))
    dsum = 0
    for b in range(args.warmup, steps_total):
        lo, hi = b * nb, (b + 1) * nb
        comp = keys[lo:hi] * 4096 + ((ts[lo:hi] // g) % 4096)
        dsum += int(torch.unique(comp).numel())
    ingest_bytes_total = events_rank * b_in + 2 * s_acc * dsum
    fire_bytes_total = rows_rank * (32 + s_acc)
    # The ingest pipeline of one watermark batch: pass 1 per batch (its average over the timed
    # sample of batches) plus its share of the plan / pass 2 / apply launches, which run once
    # per buffer flush.  Device time from HIP events on the operator's stream.
    pipe_ms_total = ingest_ms * args.steps + apply_ms * apply_launches
    per_launch = ingest_bytes_total / max(args.steps, 1)
    pipe_ms = pipe_ms_total / max(args.steps, 1)
    achieved = ingest_bytes_total / (pipe_ms_total / 1e3) / 1e9 if pipe_ms_total > 0 else 0.0
    pipeline_gbs = (ingest_bytes_total + fire_bytes_total) / elapsed / 1e9

    checksum = None
    if args.checksum:
        op.advance_watermark(W.LONG_MAX)  # end of input: everything left fires (outside the clock)
        run.consume()
        checksum = wrap64(sum(c for _, c in run.per_wm))
    tot = torch.tensor([events_rank, rows_rank, checksum or 0], dtype=torch.int64, device=dev)
    if dist:
        dist.all_reduce(tot)
    events_all, rows_all = int(tot[0].item()), int(tot[1].item())
    value = events_all / elapsed

    # ------------------------------------------------------------ CPU baseline
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, keys, ts, vals, wms, nb, agg, size, slide)
    host_fed = None
    if rank == 0 and world == 1 and not args.no_host_fed:
        host_fed = host_fed_leg(args, W, keys, ts, vals, wms, nb, agg, size, slide, K, maxp, local)
    oracle_check = None
    if rank == 0 and world == 1 and args.checksum and args.oracle_check:
        oracle_check = oracle_watermarks(args, keys, ts, vals, wms, nb, run.per_wm)

    if rank == 0:
        out = {
            "metric": "events/sec keyed sliding-window agg at 1/2/4/8 GPUs; % of HBM roofline",
            "value": value,
            "unit": "events/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64" if agg.endswith("f64") else "int64",
            "data": "synthetic (splitmix64 Nexmark-Q5-shaped bids, generated in HBM)",
            "config": {
                "workload": f"nexmark_q5_sliding_{size // 1000}s_{slide // 1000}s_{agg}",
                "keys": K, "events_per_pane_per_gpu": E, "events_per_step_per_gpu": nb,
                "watermark_interval_ms": args.wm_interval_ms, "disorder_ms": args.disorder_ms,
                "window": {"assigner": "sliding", "size_ms": size, "slide_ms": slide},
                "aggregate": agg, "max_parallelism": maxp,
                "parallelism": f"keygroup-sharded x{world}" + (f" ({args.exchange} exchange)" if world > 1 else ""),
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "ingest pipeline per watermark batch (region path: pass 1 k_rgn_p1 per batch + "
                          "plan / pass 2 / k_rgn_apply per buffer flush)",
                "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic_bytes(agg, nb),
                "bytes_per_launch": per_launch, "avg_launch_ms": pipe_ms, "launches": args.steps,
                "pass1_timed_launches": ingest_launches,
                "pass1_avg_ms": ingest_ms, "apply_avg_ms": apply_ms, "apply_launches": apply_launches,
                "pipeline_achieved": pipeline_gbs, "pipeline_frac": pipeline_gbs / HBM_PEAK_GBS,
                "fire_avg_launch_ms": fire_ms, "fire_launches": fire_launches,
                "d_over_n": dsum / max(events_rank, 1),
            },
            "rows_fired": rows_all,
            "fire_cycles": cycles,
            "host_fed": host_fed,
            "cpu_baseline": cpu,
        }
        if args.checksum:
            out["rows_checksum"] = int(tot[2].item())
            out["checksum_note"] = ("oracle.rows_hash_sum over every row fired, warmup and the final "
                                    "MAX_WATERMARK included, summed over ranks (mod 2^64)")
        if oracle_check is not None:
            out["oracle_check"] = oracle_check
        if world > 1 or ex is not None:
            pk = args.pack != "off" and not agg.endswith("f64")
            out["exchange_gbs_per_gpu"] = run.exch_bytes / elapsed / 1e9
            drv = f"{args.exchange_ahead} batch(es) finished ahead of the ingest"
            out["exchange_path"] = (f"gw_exchange_begin / gw_exchange_finish {drv} (libgpuwin RCCL: "
                                    "partition, one all-to-all of (count, watermark, columns, packed count), one "
                                    "bounded host wait, grouped send/recv per batch" + ((", 8-B packed words decoded by pass 1" if args.pack == "auto"
                                                    else ", 8-B packed words unpacked to columns") if pk
                                                   else ", 24-B records") + ")"
                                    if ex is not None else "none (key-partitioned source)")
        print(json.dumps(out), flush=True)
    if ex is not None:
        ex.close()
    op.close()
    if dist:
        dist.destroy_process_group()


def oracle_watermarks(args, keys, ts, vals, wms, nb, per_wm):
    """The CPU oracle (oracle/, test infrastructure) over the same stream and watermarks,
    compared per watermark with the GPU's (row count, checksum); outside every timed region."""
    from oracle import oracle as O
    O.build()
    threads, _ = host_cores()
    cfg = O.make_config(assigner="sliding", size=args.size_ms, slide=args.slide_ms, agg=args.agg,
                        max_parallelism=128)
    nbat = len(wms)
    rows, cs, sec = O.run_parallel_wm(cfg, threads, np.full(nbat, nb, np.int64), np.array(wms, np.int64),
                                      keys.cpu().numpy(), ts.cpu().numpy(),
                                      vals.cpu().numpy() if vals is not None else None)
    ora = [(int(r), int(c)) for r, c in zip(rows, cs)]
    bad = [i for i, (g, o) in enumerate(zip(per_wm, ora)) if g != o]
    return {"watermarks": len(ora), "match": not bad and len(per_wm) == len(ora), "mismatched": bad[:10],
            "oracle_checksum": wrap64(sum(c for _, c in ora)),
            "oracle_seconds": sec, "oracle_threads": threads}


def rows_checksum(rows) -> int:
    """The oracle's order-independent row checksum (oracle.rows_hash_sum: the sum over rows
    of (key * 0x9e3779b97f4a7c15) ^ (start * 31) ^ (end * 17) ^ result bits, mod 2^64)."""
    k, s, e, r = (np.ascontiguousarray(c).view(np.uint64) for c in rows)
    with np.errstate(over="ignore"):
        h = (k * np.uint64(0x9E3779B97F4A7C15)) ^ (s * np.uint64(31)) ^ (e * np.uint64(17)) ^ r
        tot = h.sum(dtype=np.uint64) if h.size else np.uint64(0)
    return int(np.array(tot, dtype=np.uint64).view(np.int64))


def wrap64(x: int) -> int:
    """x mod 2^64 as a signed int64."""
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >= (1 << 63) else x


def traffic_bytes(agg, nb):
    """HBM bytes per k_ingest launch from the newest committed PMC pass of this workload
    (profiles/<round>/traffic.json: FETCH_SIZE x2 + WRITE_SIZE, gfx950 corrections);
    None when no pass matches this aggregate / batch size."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "traffic.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("agg") == agg and d.get("events_per_launch") == nb and d.get("path") == INGEST_PATH:
            return d["traffic_bytes_per_launch"]
    return None


def host_fed_leg(args, W, keys, ts, vals, wms, nb, agg, size, slide, K, maxp, local):
    """The north star's host path, as the JVM operator drives it (GpuWindowOperator.java): each
    batch's columns sit in library-owned pinned slots the operator fills in place
    (gw_stage_columns; filled here from the generated stream before the clock, as the JVM's
    processElement calls would have), gw_ingest_stage sends them over PCIe on a copy stream
    (overlapping the previous batch's kernels), gw_advance_watermark fires, and every fired row
    is drained to host memory (gw_drain) before the next batch, as processWatermark emits them.
    A fresh operator over the first --host-fed-steps batches of the stream, the first fire
    cycle untimed (its first fire grows the row buffers and the deferred list, which a running
    job has done long before); PCIe-inclusive events/s (never the bench's `value`)."""
    H = max(2, min(args.host_fed_steps, len(wms)))
    warm = max(1, min(10, H - 2))
    op = W.GpuWindowOperator(W.SlidingEventTimeWindows.of(size, slide), agg, capacity_hint=K,
                             max_parallelism=maxp, device=local, max_batch=nb).open()
    try:
        op.stage_alloc(H, nb)
        for b in range(H):
            k, _, t, v = op.stage_columns(b)
            lo, hi = b * nb, (b + 1) * nb
            k[:nb] = keys[lo:hi].cpu().numpy()
            t[:nb] = ts[lo:hi].cpu().numpy()
            if vals is not None:
                v[:nb] = vals[lo:hi].cpu().numpy()
        with_value = vals is not None
        # the rows land in pinned host memory (the D2H writes them directly, no bounce copy), as
        # a JVM operator emitting from library-owned row buffers would read them
        out = [torch.empty(K + nb, dtype=torch.int64, pin_memory=True).numpy() for _ in range(4)]
        for b in range(warm):  # untimed: the first fire cycle
            op.ingest_stage(b, nb, with_value)
            op.advance_watermark(wms[b])
            op.drain(out)
        op.synchronize()
        rows = 0
        drain_s = 0.0
        t0 = time.perf_counter()
        for b in range(warm, min(H, warm + 2)):
            op.stage_send(b, nb, with_value)
        for b in range(warm, H):
            op.ingest_stage(b, nb, with_value)  # sent ahead: its H2D overlapped earlier batches
            if b + 2 < H:
                op.stage_send(b + 2, nb, with_value)  # batches b+1, b+2 over PCIe while b runs / drains
            if op.advance_watermark(wms[b]):
                td = time.perf_counter()
                rows += len(op.drain(out)[0])  # processWatermark: the rows reach the host first
                drain_s += time.perf_counter() - td
        op.flush()
        op.synchronize()
        sec = time.perf_counter() - t0
    finally:
        op.close()
    n = (H - warm) * nb
    bpe = 16 if vals is None else 24
    return {"value": n / sec, "unit": "events/s", "batches": H - warm, "untimed_batches": warm, "events": n,
            "bytes_per_event_h2d": bpe,
            "h2d_gbs": n * bpe / sec / 1e9, "rows_drained": rows, "drain_seconds": drain_s, "seconds": sec,
            "path": "library-owned pinned slots filled in place (gw_stage_columns) -> gw_stage_send of batches b+1 "
                    "and b+2 (H2D on a copy stream, three device buffers in turn) while batch b is ingested (gw_ingest_stage), "
                    "fired and its rows drained (gw_drain into pinned host arrays, D2H direct)"}


def host_cores():
    """Host cores this process can use: the CPUs it may run on, capped by the cgroup CPU
    quota (a container's share of a bigger machine; os.cpu_count() reports the machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    note = f"sched_getaffinity={n}"
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]  # cgroup v2
        if q != "max":
            quota = int(q) / int(p)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / p
        except (OSError, ValueError):
            pass
    if quota is not None:
        note += f", cgroup cpu quota={quota:g}"
        n = max(1, min(n, int(quota)))
    return n, note


def cpu_baseline(args, keys, ts, vals, wms, nb, agg, size, slide):
    """CPU restatement of Flink's operator (oracle/, 'port') on the host cores: one operator
    per simulated subtask thread (parallelism = the host CPUs this process may run on, SURVEY.md
    §8d), over a bounded sample of the same stream that holds whole fire cycles: the records of
    every K-th auction (key % K == 0) in the batches up to and including the stream's second
    firing watermark -- each batch followed by its watermark, as the GPU's timed steps run -- so
    the reference's timer pops, emits and purges are in the sample as they are in the GPU's
    timed region.  K is sized for ~cpu_baseline_seconds of CPU work; a key subset keeps the
    per-key state small, which only flatters the CPU."""
    try:
        from oracle import oracle as O
        O.build()
    except Exception as e:  # noqa: BLE001
        return {"value": None, "unit": "events/s", "cores": 0, "kind": "port", "sample": f"unavailable: {e}"}
    threads, cores_note = host_cores()
    cfg = O.make_config(assigner="sliding", size=size, slide=slide, agg=agg, max_parallelism=128)
    # batches whose watermark completes windows: the count of windows with end - 1 <= wm grows
    nfired = [(w + 1 - size) // slide for w in wms]
    fires = [b for b in range(1, len(wms)) if nfired[b] > nfired[b - 1]]
    first_fire = fires[0] if fires else len(wms) - 1
    last_b = fires[1] if len(fires) > 1 else first_fire  # the second firing watermark's batch

    def run(nbatches, ksub):
        n = nbatches * nb
        k = keys[:n]
        sel = (k % ksub) == 0
        kk = k[sel].cpu().numpy()
        t = ts[:n][sel].cpu().numpy()
        v = vals[:n][sel].cpu().numpy() if vals is not None else None
        blen = torch.stack([sel[b * nb:(b + 1) * nb].sum() for b in range(nbatches)]).cpu().numpy().astype(np.int64)
        wm = np.array(wms[:nbatches], np.int64)
        rows, _, sec = O.run_parallel(cfg, threads, blen, wm, kk, t, v, final_watermark=False)
        return int(blen.sum()), sec, rows

    # calibrate on the first batch of a 1/64 key subset, then size the subset for the sample
    n0, s0, _ = run(1, 64)
    rate0 = n0 / max(s0, 1e-6)
    ksub = max(1, int(np.ceil((last_b + 1) * nb / max(rate0 * args.cpu_baseline_seconds, 1.0))))
    n, sec, rows = run(last_b + 1, ksub)
    sample = (f"every {ksub}-th auction (key % {ksub} == 0) of the GPU stream over its first {last_b + 1} "
              f"watermark batches ({n} events), each batch followed by its watermark: two firing watermarks "
              f"(batches {first_fire} and {last_b}), {rows} rows fired")
    return {"value": n / sec, "unit": "events/s", "cores": threads, "kind": "port", "sample": sample,
            "seconds": sec, "rows": rows, "key_subset": ksub, "nproc": os.cpu_count(), "cores_source": cores_note}


if __name__ == "__main__":
    main()
