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


def parse():
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
                    help="a2a: RCCL all-to-all keyBy exchange; none: each rank generates only its own key groups")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-fed", action="store_true",
                    help="skip the host-fed leg (gw_ingest from host columns: pinned staging + H2D)")
    ap.add_argument("--host-fed-steps", type=int, default=4)
    ap.add_argument("--preagg", choices=["auto", "force", "off"], default="auto")
    ap.add_argument("--producer-stream", choices=["auto", "torch", "handle"], default="auto",
                    help="stream gw_ingest_device orders after: the exchange output's (torch) stream, or, "
                         "for columns generated and synchronised before the clock starts, none (handle)")
    ap.add_argument("--torch-stream", choices=["side", "default"], default="side",
                    help="stream the step's torch work (exchange) runs on")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="no HIP events around the kernels (the roofline fields are then null)")
    ap.add_argument("--overlap", choices=["on", "off"], default="on",
                    help="on: double-buffered receive columns, so batch b+1's partition and all-to-all "
                         "run while the operator still aggregates batch b; off: every step ordered "
                         "after the previous ingest's reads")
    ap.add_argument("--checksum", action="store_true",
                    help="drain the fired rows to the host and report an order-independent checksum "
                         "(key, start, end, result) summed over ranks (a check, not a bench setting)")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl = RCCL over xGMI; gloo = host-staged rehearsal (several ranks may share one GPU)")
    return ap.parse_args()


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
    local = local % max(torch.cuda.device_count(), 1)  # rehearsal: ranks may share a GPU
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

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

    # ------------------------------------------------------------------ data
    t_gen = time.time()
    n_all = nb * steps_total
    idx = torch.arange(n_all, device=dev, dtype=torch.int64)
    seed = 0x5EED0005 + 7919 * rank
    keys = (splitmix64(idx, seed) & MASK63) % K
    if args.exchange == "none" and world > 1:
        # key-partitioned source: remap every key onto this rank's key groups
        kg = torch.empty(n_all, dtype=torch.int32, device=dev)
        owner = torch.empty_like(kg)
        N.check(N.lib().gw_key_groups_device(n_all, keys.data_ptr(), None, maxp, world, kg.data_ptr(),
                                             owner.data_ptr(), None))
        torch.cuda.synchronize()
        keys = keys[owner == rank]
        n_all = keys.numel() // steps_total * steps_total
        keys = keys[:n_all]
        nb = n_all // steps_total
        idx = torch.arange(n_all, device=dev, dtype=torch.int64)
    t0_ms = 1_700_000_000_000
    jitter = (splitmix64(idx, seed ^ 0x77) & MASK63) % (args.disorder_ms + 1)
    ts = t0_ms + (idx * slide) // E - jitter
    vals = None
    if agg != "count":
        v = (splitmix64(idx, seed ^ 0x1234) & MASK63) % 1_000_000
        vals = v.to(torch.float64).view(torch.int64) if agg.endswith("f64") else v
    del idx, jitter
    # watermark after step b: BoundedOutOfOrdernessWatermarks (maxTs - bound - 1) over the
    # un-jittered maximum, identical on every rank
    wms = [t0_ms + (((b + 1) * nb - 1) * slide) // E - args.disorder_ms - 1 for b in range(steps_total)]
    torch.cuda.synchronize()
    log(f"rank {rank}: generated {n_all} events ({n_all * b_in / 1e9:.1f} GB) in {time.time() - t_gen:.1f}s")

    flags = {"auto": 0, "force": N.FLAG_FORCE_LDS_PREAGG, "off": N.FLAG_NO_LDS_PREAGG}[args.preagg]
    op = W.GpuWindowOperator(W.SlidingEventTimeWindows.of(size, slide), agg, capacity_hint=max(K // world, 1024),
                             max_parallelism=maxp, parallelism=world, operator_index=rank, device=local,
                             flags=flags, max_batch=nb * 2).open()
    # The step's torch work (exchange partition + all-to-all) runs on a dedicated stream: the
    # ingest's cross-stream ordering against a non-default stream is cheap, against the
    # legacy default stream it costs ~25 us per step.
    side = torch.cuda.Stream(device=dev) if args.torch_stream == "side" else torch.cuda.current_stream(dev)
    cur = side.cuda_stream

    ex = None
    native_ex = False
    if world > 1 and args.exchange == "a2a" and args.dist_backend == "nccl":
        # the product path: libgpuwin's own RCCL exchange (gw_exchange_*), what a JVM task
        # drives; torch.distributed only ships its communicator id and times the run
        from flink_amd.exchange import NativeKeyByExchange
        ex = NativeKeyByExchange(world, rank, max_parallelism=maxp, device=local)
        native_ex = True
    elif world > 1:
        # gloo rehearsal (several ranks may share one GPU): the torch.distributed exchange
        from flink_amd.exchange import KeyByExchange
        ex = KeyByExchange(world, rank, max_parallelism=maxp, device=dev)

    exch_bytes = 0
    rows_sum = 0
    # Exchanged columns are produced on torch's stream inside each step, so the ingest orders
    # itself after it (and torch's stream after the read).  Columns generated in HBM before
    # the clock starts (synchronised above) need no ordering: pass the handle's own stream.
    exchanged = ex is not None and args.exchange == "a2a"
    use_torch = args.producer_stream == "torch" or (args.producer_stream == "auto" and exchanged)
    prod = cur if use_torch else op.stream()
    # Overlapped exchange: two sets of receive columns used in turn.  The all-to-all of
    # batch b writes set b%2 once the ingest of batch b-2 has read it (ev_read), and the
    # ingest orders itself through a hand-off stream that nothing else uses, so the
    # exchange stream never waits for the ingest of the batch just before it.
    overlap = exchanged and not native_ex and args.overlap == "on" and args.producer_stream != "handle"
    if overlap:
        cap = nb * 2  # received records per step: ~nb for uniform keys (max_batch above)
        ncols = 3 if vals is not None else 2
        bufs = [[torch.empty(cap, dtype=torch.int64, device=dev) for _ in range(ncols)] + [None] * (3 - ncols)
                for _ in range(2)]
        handoff = torch.cuda.Stream(device=dev)
        ev_read = [None, None]

    def step(b, timed):
        if not exchanged:  # nothing of the step runs on a torch stream
            return step_on_side(b, timed)
        with torch.cuda.stream(side):
            return step_on_side(b, timed)

    def step_on_side(b, timed):
        nonlocal exch_bytes, rows_sum
        lo, hi = b * nb, (b + 1) * nb
        k, t, v = keys[lo:hi], ts[lo:hi], (vals[lo:hi] if vals is not None else None)
        if native_ex:
            # partition + one all-to-all of (count, watermark, columns) + one host wait +
            # grouped send/receive, all on `cur`; the ingest orders through the receive set's
            # hand-off stream, so the next batch's exchange overlaps this batch's aggregation
            n, pk, pt, pv, _, wmin, ist = ex.exchange(k, t, v, stream=cur, wm=wms[b])
            if timed:
                exch_bytes += (nb - int(ex.counts()[0][rank])) * b_in
            N.check(N.lib().gw_ingest_device(op.handle, n, pk, None, pt, pv, ist), op.handle)
            op.advance_watermark(wmin)
            if args.checksum:
                rows_sum = (rows_sum + rows_checksum(op.drain())) % (1 << 56)
            op.clear_rows()  # DiscardingSink
            return None
        if ex is not None and args.exchange == "a2a":
            pk, pt, pv, counts = ex.partition(k, t, v, stream=cur)
            if overlap:
                s = b % 2
                (k, t, v), n_recv = ex.exchange_partitioned([pk, pt, pv], counts, out=bufs[s], out_ready=ev_read[s])
                handoff.wait_event(side.record_event())
            else:
                (k, t, v), n_recv = ex.exchange_partitioned([pk, pt, pv], counts)
            if timed:
                exch_bytes += (nb - ex.last_send_counts[rank]) * b_in
        n = k.numel()
        N.check(N.lib().gw_ingest_device(op.handle, n, k.data_ptr(), None, t.data_ptr(),
                                         v.data_ptr() if v is not None else None,
                                         handoff.cuda_stream if overlap else prod), op.handle)
        if overlap:
            ev_read[b % 2] = handoff.record_event()  # the ingest's reads of set b%2 are done
        wm = wms[b]
        if ex is not None:
            wm = ex.combine_watermark(wm)  # StatusWatermarkValve: min over inputs
        op.advance_watermark(wm)
        if args.checksum:
            rows_sum = (rows_sum + rows_checksum(op.drain())) % (1 << 56)
        op.clear_rows()  # DiscardingSink
        return k, t

    op.enable_kernel_timing(not args.no_kernel_timing)
    for b in range(args.warmup):
        step(b, False)
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
    cyc_t, cyc_steps, fires_seen = t0, 0, op.stats()["fires"]
    for b in range(args.warmup, steps_total):
        step(b, True)
        cyc_steps += 1
        f = op.stats()["fires"]
        if f != fires_seen:
            now = time.perf_counter()
            cycles.append({"steps": cyc_steps, "ms": (now - cyc_t) * 1e3,
                           "events_per_s": cyc_steps * nb / max(now - cyc_t, 1e-9)})
            cyc_t, cyc_steps, fires_seen = now, 0, f
        if rank == 0 and time.perf_counter() - last > 30:
            last = time.perf_counter()
            log(f"step {b - args.warmup + 1}/{args.steps}")
    op.flush()  # every timed batch is in the window state when the clock stops
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if cyc_steps:
        cycles.append({"steps": cyc_steps, "ms": (time.perf_counter() - cyc_t) * 1e3, "partial": True})
    if dist:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
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
    # The ingest pipeline of one watermark batch: pass 1 (k_part_hist/cols/scatter) per
    # batch, plus its share of pass 2 + k_rgn_apply, which run once per fire over the
    # buffered batches.  Device time from HIP events on the operator's stream.
    pipe_ms_total = ingest_ms * ingest_launches + apply_ms * apply_launches
    per_launch = ingest_bytes_total / max(ingest_launches, 1)
    pipe_ms = pipe_ms_total / max(ingest_launches, 1)
    achieved = ingest_bytes_total / (pipe_ms_total / 1e3) / 1e9 if pipe_ms_total > 0 else 0.0
    pipeline_gbs = (ingest_bytes_total + fire_bytes_total) / elapsed / 1e9

    if args.checksum:
        rows_sum = (rows_sum + rows_checksum(op.drain())) % (1 << 56)
    tot = torch.tensor([events_rank, rows_rank, rows_sum], dtype=torch.int64,
                       device=dev if args.dist_backend == "nccl" else "cpu")
    if dist:
        dist.all_reduce(tot)
    events_all, rows_all = int(tot[0].item()), int(tot[1].item())
    rows_sum = int(tot[2].item()) % (1 << 56)
    value = events_all / elapsed

    # ------------------------------------------------------------ CPU baseline
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, keys, ts, vals, wms, nb, agg, size, slide)
    host_fed = None
    if rank == 0 and world == 1 and not args.no_host_fed:
        host_fed = host_fed_leg(args, W, keys, ts, vals, wms, nb, agg, size, slide, K, maxp, local)

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
                "kernel": "ingest pipeline per watermark batch (region path: pass 1 k_part_* per batch + "
                          "pass 2 / k_rgn_apply per buffer flush)",
                "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic_bytes(agg, nb),
                "bytes_per_launch": per_launch, "avg_launch_ms": pipe_ms, "launches": ingest_launches,
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
            out["rows_checksum"] = rows_sum
        if world > 1:
            out["exchange_gbs_per_gpu"] = exch_bytes / elapsed / 1e9
            out["exchange_path"] = ("gw_exchange_batch (libgpuwin RCCL: partition, one all-to-all of "
                                    "(count, watermark, columns), one host wait, grouped send/recv per batch)"
                                    if native_ex else "torch.distributed KeyByExchange (gloo rehearsal)")
        print(json.dumps(out), flush=True)
    op.close()
    if dist:
        dist.destroy_process_group()


def rows_checksum(rows) -> int:
    """Order-independent checksum of fired rows: sum of a 64-bit mix of each (key, start,
    end, result), mod 2^56 (results compared by their bit pattern)."""
    k, s, e, r = (np.ascontiguousarray(c).view(np.uint64) for c in rows)
    with np.errstate(over="ignore"):
        h = k * np.uint64(0x9E3779B97F4A7C15) ^ s * np.uint64(0xBF58476D1CE4E5B9) \
            ^ e * np.uint64(0x94D049BB133111EB) ^ r * np.uint64(0xD6E8FEB86659FD93)
        h ^= h >> np.uint64(31)
    return int((h & np.uint64((1 << 56) - 1)).astype(object).sum() % (1 << 56)) if h.size else 0


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
    """The north star's host path: columns in (pageable) host memory -> gw_ingest, which
    copies them into the handle's pinned staging and then over PCIe into HBM, then the
    watermark.  A fresh operator over the first --host-fed-steps batches of the same stream;
    PCIe-inclusive events/s (never the bench's `value`)."""
    H = max(1, min(args.host_fed_steps, len(wms)))
    hk = keys[:H * nb].cpu().numpy()
    ht = ts[:H * nb].cpu().numpy()
    hv = vals[:H * nb].cpu().numpy() if vals is not None else None
    op = W.GpuWindowOperator(W.SlidingEventTimeWindows.of(size, slide), agg, capacity_hint=K,
                             max_parallelism=maxp, device=local, max_batch=nb).open()
    try:
        op.process_batch(hk[:nb], ht[:nb], hv[:nb] if hv is not None else None)  # warm: staging allocation
        op.advance_watermark(wms[0])
        op.clear_rows()
        op.synchronize()
        t0 = time.perf_counter()
        for b in range(1, H):
            lo, hi = b * nb, (b + 1) * nb
            op.process_batch(hk[lo:hi], ht[lo:hi], hv[lo:hi] if hv is not None else None)
            op.advance_watermark(wms[b])
            op.clear_rows()
        op.flush()
        op.synchronize()
        sec = time.perf_counter() - t0
    finally:
        op.close()
    n = (H - 1) * nb
    return {"value": n / sec if n else None, "unit": "events/s", "batches": H - 1, "events": n,
            "bytes_per_event_h2d": 16 if vals is None else 24,
            "path": "gw_ingest (memcpy into pinned staging + hipMemcpyAsync H2D) + gw_advance_watermark"}


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
    per simulated subtask thread over the first watermark batches of the same stream, at the
    stream's own cadence (each batch followed by its watermark, no final MAX_WATERMARK: what
    the GPU's timed steps do).  Parallelism = the host CPUs this process may run on
    (parallelism = nproc)."""
    try:
        from oracle import oracle as O
        O.build()
    except Exception as e:  # noqa: BLE001
        return {"value": None, "unit": "events/s", "cores": 0, "kind": "port", "sample": f"unavailable: {e}"}
    threads, cores_note = host_cores()
    cfg = O.make_config(assigner="sliding", size=size, slide=slide, agg=agg, max_parallelism=128)

    def run(nbatches, per_batch):
        n = nbatches * per_batch
        k = keys[:n].cpu().numpy()
        t = ts[:n].cpu().numpy()
        v = vals[:n].cpu().numpy() if vals is not None else None
        blen = np.full(nbatches, per_batch, np.int64)
        wm = np.array(wms[:nbatches], np.int64) if per_batch == nb else \
            np.array([int(t[(b + 1) * per_batch - 1]) - args.disorder_ms - 1 for b in range(nbatches)], np.int64)
        rows, _, sec = O.run_parallel(cfg, threads, blen, wm, k, t, v, final_watermark=False)
        return n, sec, rows

    # calibrate on 1/50 of a step, then size the sample for ~cpu_baseline_seconds in whole
    # watermark batches of the stream (at least one)
    n0, s0, _ = run(1, max(nb // 50, 10000))
    rate0 = n0 / max(s0, 1e-6)
    nbatches = max(1, min(len(wms), int(round(rate0 * args.cpu_baseline_seconds / nb))))
    n, sec, rows = run(nbatches, nb)
    sample = (f"first {nbatches} watermark batches ({n} events) of the GPU stream, each followed by its "
              f"watermark (no final MAX_WATERMARK), {rows} rows fired")
    return {"value": n / sec, "unit": "events/s", "cores": threads, "kind": "port", "sample": sample,
            "seconds": sec, "rows": rows, "nproc": os.cpu_count(), "cores_source": cores_note}


if __name__ == "__main__":
    main()
