"""keyBy exchange across GPUs: key-group partition on the device + RCCL all-to-all.

Replaces the reference's keyBy shuffle — KeyGroupStreamPartitioner.selectChannel
(flink-runtime/.../streaming/runtime/partitioner/KeyGroupStreamPartitioner.java:55-64)
feeding RecordWriter / Netty (RR/io/network/api/writer/RecordWriter.java:108-158) — with
one columnar all-to-all per watermark batch over xGMI (torch.distributed "nccl" = RCCL).
Each GPU owns the key groups computeKeyGroupRangeForOperatorIndex(maxP, N, rank)
(flink-runtime/.../runtime/state/KeyGroupRangeAssignment.java:93-106).

The watermark combine (StatusWatermarkValve.inputWatermark, min over input channels,
RS/runtime/watermarkstatus/StatusWatermarkValve.java:153-185) is an all-reduce(MIN).
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from . import _native as N


def owners_np(keys, max_parallelism: int, parallelism: int):
    """Owner subtask of int64 keys on the host (vectorised KeyGroupRangeAssignment.
    assignKeyToParallelOperator: Long.hashCode, MathUtils.murmurHash, key group * p / maxP;
    KeyGroupRangeAssignment.java:63-77,124-127, MathUtils.java:137-155) -- the host partition
    of KeyByExchange.exchange_packed; the device partition is gw_keygroups.hip."""
    import numpy as np
    u = np.ascontiguousarray(keys, np.int64).view(np.uint64)
    c = (u ^ (u >> np.uint64(32))).astype(np.uint32)
    with np.errstate(over="ignore"):
        c = (c * np.uint32(0xcc9e2d51)).astype(np.uint32)
        c = ((c << np.uint32(15)) | (c >> np.uint32(17))).astype(np.uint32)
        c = (c * np.uint32(0x1b873593)).astype(np.uint32)
        c = ((c << np.uint32(13)) | (c >> np.uint32(19))).astype(np.uint32)
        c = (c * np.uint32(5) + np.uint32(0xe6546b64)).astype(np.uint32)
        c ^= np.uint32(4)
        c ^= c >> np.uint32(16)
        c = (c * np.uint32(0x85ebca6b)).astype(np.uint32)
        c ^= c >> np.uint32(13)
        c = (c * np.uint32(0xc2b2ae35)).astype(np.uint32)
        c ^= c >> np.uint32(16)
    r = c.view(np.int32).astype(np.int64)
    r = np.where(r >= 0, r, np.where(r == -(1 << 31), 0, -r))
    return (r % max_parallelism) * parallelism // max_parallelism


class KeyByExchange:
    def __init__(self, parallelism: int, rank: int, max_parallelism: int = 128, group=None,
                 device: Optional[torch.device] = None):
        if not (1 <= parallelism <= max_parallelism):
            raise ValueError("Maximum parallelism must not be smaller than parallelism.")
        self.p, self.rank, self.maxp, self.group = parallelism, rank, max_parallelism, group
        self.device = device
        self._scratch = None
        self._bufs = {}
        # Watermarks are control-plane data: combining them over a host (gloo) group keeps
        # the per-batch minimum off the GPU streams (an RCCL all-reduce + .item() would
        # wait for the column all-to-all queued before it).
        self._wm_group = None
        if dist.is_initialized() and dist.get_backend(group) != "gloo":
            self._wm_group = dist.new_group(backend="gloo")
        self.last_send_counts: list = []

    # ---------------------------------------------------------------- partition
    def partition(self, keys: torch.Tensor, ts: torch.Tensor, vals: Optional[torch.Tensor],
                  key_hashes: Optional[torch.Tensor] = None, stream=None):
        """Stable device partition of the columns by owner subtask; returns the grouped
        columns and the per-destination counts (device int64[p])."""
        if not keys.is_cuda:
            raise ValueError("KeyByExchange.partition runs on the GPU (libgpuwin.so); got host tensors")
        n = keys.numel()
        need = N.lib().gw_partition_scratch_bytes(n, self.p)
        if self._scratch is None or self._scratch.numel() < need:
            self._scratch = torch.empty(need, dtype=torch.uint8, device=keys.device)
        pk = torch.empty_like(keys)
        pt = torch.empty_like(ts)
        pv = torch.empty_like(vals) if vals is not None else None
        counts = torch.empty(self.p, dtype=torch.int64, device=keys.device)
        ptr = lambda t: t.data_ptr() if t is not None else None
        s = stream if stream is not None else torch.cuda.current_stream(keys.device).cuda_stream
        N.check(N.lib().gw_partition_device(n, ptr(keys), ptr(key_hashes), ptr(ts), ptr(vals), self.maxp, self.p,
                                            ptr(pk), ptr(pt), ptr(pv), ptr(counts), ptr(self._scratch), s))
        return pk, pt, pv, counts

    # ---------------------------------------------------------------- exchange
    def exchange_partitioned(self, cols: Sequence[Optional[torch.Tensor]], send_counts: torch.Tensor,
                             out: Optional[Sequence[Optional[torch.Tensor]]] = None,
                             out_ready: Optional[torch.cuda.Event] = None) -> Tuple[list, int]:
        """All-to-all of already partitioned columns (any backend: RCCL on GPU tensors,
        gloo on CPU tensors).  send_counts[d] = records for rank d.

        ``out`` (optional): persistent receive columns, one per input column, each with
        capacity for the received records; the result columns are their leading slices.
        ``out_ready``: an event the current stream waits for before the column exchange
        writes into ``out`` (the consumer's read of the previous contents), so a caller can
        double-buffer the receive side instead of ordering every step after the consumer."""
        staged = dist.get_backend(self.group) == "gloo" and send_counts.is_cuda
        if staged:  # rehearsal on one GPU: gloo moves host tensors only
            dev = send_counts.device
            send_counts = send_counts.cpu()
            cols = [c.cpu() if c is not None else None for c in cols]
        recv_counts = torch.empty_like(send_counts)
        dist.all_to_all_single(recv_counts, send_counts, group=self.group)
        sc = send_counts.tolist()
        rc = recv_counts.tolist()
        self.last_send_counts = sc
        total = int(sum(rc))
        if out is not None:
            for c, o in zip(cols, out):
                if c is not None and (o is None or o.numel() < total):
                    raise ValueError(f"receive buffer holds {0 if o is None else o.numel()} records, "
                                     f"the exchange delivers {total}")
            if out_ready is not None:
                torch.cuda.current_stream().wait_event(out_ready)
        res = []
        for i, c in enumerate(cols):
            if c is None:
                res.append(None)
                continue
            if out is not None and not staged:
                r = out[i][:total]
            else:
                r = torch.empty(total, dtype=c.dtype, device=c.device)
            dist.all_to_all_single(r, c, rc, sc, group=self.group)
            if staged:
                r = out[i][:total].copy_(r) if out is not None else r.to(dev)
            res.append(r)
        return res, total

    def exchange(self, keys, ts, vals, key_hashes=None):
        pk, pt, pv, counts = self.partition(keys, ts, vals, key_hashes)
        (rk, rt, rv), _ = self.exchange_partitioned([pk, pt, pv], counts)
        return rk, rt, rv

    # ---------------------------------------------------------------- packed exchange
    def exchange_packed(self, keys: torch.Tensor, ts: torch.Tensor, vals: Optional[torch.Tensor], geom, wm: int):
        """The packed protocol of gw_exchange_batch (include/gpuwin.h gw_pack_geom) over
        torch.distributed point-to-point transfers: records that fit travel as 8-byte words,
        the rest as (key, ts, value).  geom: N.pack_geom(size, slide, offset, watermark before
        the batch) -- the same on every rank -- or None (nothing packs).  The partition runs on
        the device for GPU tensors (gw_partition_packed_device), on the host otherwise
        (gw_pack_records + a stable sort by (owner, does not fit)); the receiver unpacks the
        words behind the other records, as gw_exchange_batch does.  Returns host numpy
        (keys, ts, values, packed records received, minimum watermark over the ranks)."""
        import numpy as np
        M, P = N.MSG_WORDS, self.p
        n = keys.numel()
        has_v = vals is not None
        ptr = lambda t: t.data_ptr() if t is not None else None
        if geom is not None and keys.is_cuda:
            dev = keys.device
            need = N.lib().gw_partition_scratch_bytes(max(n, 1), 2 * P)
            if self._scratch is None or self._scratch.numel() < need:
                self._scratch = torch.empty(need, dtype=torch.uint8, device=dev)
            words = torch.empty(n, dtype=torch.int64, device=dev)
            pk, pt = torch.empty_like(keys), torch.empty_like(ts)
            pv = torch.empty_like(vals) if has_v else None
            counts = torch.empty(2 * P, dtype=torch.int64, device=dev)
            N.check(N.lib().gw_partition_packed_device(n, ptr(keys), ptr(ts), ptr(vals), self.maxp, P, geom,
                                                       ptr(words), ptr(pk), ptr(pt), ptr(pv), ptr(counts),
                                                       ptr(self._scratch), torch.cuda.current_stream(dev).cuda_stream))
            torch.cuda.synchronize(dev)
            words, pk, pt = words.cpu().numpy().view(np.uint64), pk.cpu().numpy(), pt.cpu().numpy()
            pv = pv.cpu().numpy() if has_v else None
            c2 = counts.cpu().numpy().reshape(P, 2)
        else:
            k, t = keys.cpu().numpy(), ts.cpu().numpy()
            v = vals.cpu().numpy() if has_v else None
            own = owners_np(k, self.maxp, P)
            if geom is not None:
                w, fits = N.pack_records(k, t, v, geom)
            else:
                w, fits = np.zeros(n, np.uint64), np.zeros(n, bool)
            bucket = 2 * own + (~fits).astype(np.int64)
            order = np.argsort(bucket, kind="stable")
            words, pk, pt = w[order], k[order], t[order]
            pv = v[order] if has_v else None
            c2 = np.bincount(bucket, minlength=2 * P).reshape(P, 2)
        mask = (1 if has_v else 0) | (4 if geom is not None else 0)
        msg = torch.zeros(P, M, dtype=torch.int64)
        msg[:, 0] = torch.from_numpy(c2.sum(1))
        msg[:, 1] = int(wm)
        msg[:, 2] = mask
        msg[:, 3] = torch.from_numpy(c2[:, 0].copy())
        rmsg = torch.empty_like(msg)
        dist.all_to_all_single(rmsg.view(-1), msg.view(-1), group=self.group)
        sm, rm = msg.view(-1).numpy(), rmsg.view(-1).numpy()
        (so, sc, ro, rc), total, wmin = N.exchange_plan(sm, rm, mask, int(wm))
        (sp, rwo, rpo, rp), tw, tp = N.exchange_plan_packed(sm, rm)
        self.last_send_counts = sc.tolist()

        def move(src, dst, s_off, s_cnt, r_off, r_cnt):
            reqs = []
            for q in range(P):
                if q == self.rank:
                    dst[r_off[q]:r_off[q] + r_cnt[q]] = src[s_off[q]:s_off[q] + s_cnt[q]]
                    continue
                if s_cnt[q]:
                    reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(src[s_off[q]:s_off[q] + s_cnt[q]])),
                                           q, group=self.group))
                if r_cnt[q]:
                    reqs.append(dist.irecv(torch.from_numpy(dst[r_off[q]:r_off[q] + r_cnt[q]]), q, group=self.group))
            for x in reqs:
                x.wait()

        rw = np.zeros(tp, np.int64)
        move(words.view(np.int64), rw, so, sp, rpo, rp)  # words as int64: gloo has no uint64
        other_s = so + sp
        other_n_s, other_n_r = sc - sp, rc - rp
        out = []
        for col in (pk, pt, pv):
            if col is None:
                out.append(None)
                continue
            r = np.zeros(total, np.int64)
            move(col, r, other_s, other_n_s, rwo, other_n_r)
            out.append(r)
        if tp:
            kk, tt, vv = N.unpack_records(rw.view(np.uint64), geom, has_v)
            out[0][tw:], out[1][tw:] = kk, tt
            if has_v:
                out[2][tw:] = vv
        return out[0], out[1], out[2], tp, wmin

    # ---------------------------------------------------------------- watermark
    def combine_watermark(self, wm: int) -> int:
        """Minimum over all ranks (StatusWatermarkValve), on a host (gloo) group."""
        t = torch.tensor([wm], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self._wm_group if self._wm_group is not None else self.group)
        return int(t.item())

    def key_group_range(self):
        start = (self.rank * self.maxp + self.p - 1) // self.p
        end = ((self.rank + 1) * self.maxp - 1) // self.p
        return start, end


class NativeKeyByExchange:
    """The same exchange through libgpuwin's own RCCL communicator (gw_exchange_*,
    include/gpuwin.h): the C-ABI path a JVM task drives.  torch.distributed, when
    initialized, only carries the 128-byte communicator id from rank 0 to the others
    (a JVM job would use its own rendezvous)."""

    def __init__(self, parallelism: int, rank: int, max_parallelism: int = 128, device: int = 0,
                 uid: Optional[bytes] = None, group=None):
        import ctypes
        if not (1 <= parallelism <= max_parallelism):
            raise ValueError("Maximum parallelism must not be smaller than parallelism.")
        L = N.lib()
        if uid is None:
            buf = ctypes.create_string_buffer(N.EXCHANGE_ID_BYTES)
            if rank == 0:
                N.check(L.gw_exchange_unique_id(buf))
            if parallelism > 1:
                obj = [buf.raw if rank == 0 else None]
                dist.broadcast_object_list(obj, src=0, group=group)
                buf = ctypes.create_string_buffer(obj[0], N.EXCHANGE_ID_BYTES)
        else:
            buf = ctypes.create_string_buffer(uid, N.EXCHANGE_ID_BYTES)
        h = ctypes.c_void_p()
        rc = L.gw_exchange_create(ctypes.byref(h), parallelism, rank, buf, device, max_parallelism)
        if rc != N.GW_OK:
            raise N.GpuWinError(rc, "gw_exchange_create failed")
        self._h = h
        self.p, self.rank, self.maxp, self.device = parallelism, rank, max_parallelism, device

    def set_timeout(self, timeout_ms: int):
        """gw_exchange_set_timeout: the bound of every host wait (0: none).  On expiry or an
        asynchronous RCCL error the communicator is aborted and the call raises GW_E_STATE."""
        self._check(N.lib().gw_exchange_set_timeout(self._h, int(timeout_ms)))

    def close(self):
        if getattr(self, "_h", None):
            N.lib().gw_exchange_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != N.GW_OK:
            msg = N.lib().gw_exchange_last_error(self._h)
            raise N.GpuWinError(rc, msg.decode() if msg else "")

    def exchange(self, keys: torch.Tensor, ts: torch.Tensor, vals: Optional[torch.Tensor] = None,
                 key_hashes: Optional[torch.Tensor] = None, stream=None, wm: int = -(1 << 63)):
        """One watermark batch (gw_exchange_batch): -> (n, key_ptr, ts_ptr, value_ptr, key_hash_ptr,
        min watermark over the ranks, ingest stream).  The pointers are device columns of the
        records this rank owns (valid until the next-but-one call); pass the ingest stream as
        the producer stream of gw_ingest_device (GpuWindowOperator.process_batch_device_ptr)."""
        import ctypes
        s = stream if stream is not None else torch.cuda.current_stream(keys.device).cuda_stream
        ptr = lambda t: t.data_ptr() if t is not None else None
        n_out, wm_out = ctypes.c_int64(), ctypes.c_int64()
        ok, oh, ot, ov, ist = (ctypes.c_void_p() for _ in range(5))
        self._check(N.lib().gw_exchange_batch(self._h, keys.numel(), ptr(keys), ptr(key_hashes), ptr(ts), ptr(vals),
                                              int(wm), ctypes.byref(n_out), ctypes.byref(ok), ctypes.byref(oh),
                                              ctypes.byref(ot), ctypes.byref(ov), ctypes.byref(wm_out),
                                              ctypes.byref(ist), s))
        return n_out.value, ok.value, ot.value, ov.value, oh.value, wm_out.value, ist.value

    def begin(self, keys: torch.Tensor, ts: torch.Tensor, vals: Optional[torch.Tensor] = None,
              key_hashes: Optional[torch.Tensor] = None, stream=None, wm: int = -(1 << 63)):
        """gw_exchange_begin: partition a batch and queue its count all-to-all (no host wait).
        The input columns must stay untouched until the batch is finished."""
        s = stream if stream is not None else torch.cuda.current_stream(keys.device).cuda_stream
        ptr = lambda t: t.data_ptr() if t is not None else None
        self._check(N.lib().gw_exchange_begin(self._h, keys.numel(), ptr(keys), ptr(key_hashes), ptr(ts), ptr(vals),
                                              int(wm), s))

    def finish(self, stream):
        """gw_exchange_finish: the oldest begun batch -> what exchange() returns."""
        import ctypes
        n_out, wm_out = ctypes.c_int64(), ctypes.c_int64()
        ok, oh, ot, ov, ist = (ctypes.c_void_p() for _ in range(5))
        self._check(N.lib().gw_exchange_finish(self._h, ctypes.byref(n_out), ctypes.byref(ok), ctypes.byref(oh),
                                               ctypes.byref(ot), ctypes.byref(ov), ctypes.byref(wm_out),
                                               ctypes.byref(ist), stream))
        return n_out.value, ok.value, ot.value, ov.value, oh.value, wm_out.value, ist.value

    def enable_packing(self, size: int, slide: int, offset: int = 0, with_values: bool = True):
        """gw_exchange_enable_packing: later batches ship the records that fit as 8-byte words."""
        self._check(N.lib().gw_exchange_enable_packing(self._h, int(size), int(slide), int(offset),
                                                       1 if with_values else 0))

    def keep_words(self, keep: bool = True):
        """gw_exchange_set_unpack(!keep): received words stay packed for gw_ingest_packed_device."""
        self._check(N.lib().gw_exchange_set_unpack(self._h, 0 if keep else 1))

    def last_words(self):
        """(n_words, device pointer, GwPackGeom) of the last batch's words kept packed."""
        import ctypes
        n, w, g = ctypes.c_int64(), ctypes.c_void_p(), N.GwPackGeom()
        self._check(N.lib().gw_exchange_last_words(self._h, ctypes.byref(n), ctypes.byref(w), ctypes.byref(g)))
        return n.value, w.value, g

    def last_packed(self) -> int:
        """Records this rank received packed in the last batch."""
        return int(N.lib().gw_exchange_last_packed(self._h))

    def counts(self):
        """(send, receive) record counts per peer of the last batch."""
        import ctypes
        import numpy as np
        sc, rc = np.zeros(self.p, np.int64), np.zeros(self.p, np.int64)
        self._check(N.lib().gw_exchange_counts(self._h, sc.ctypes.data, rc.ctypes.data))
        return sc, rc

    def combine_watermark(self, wm: int, stream=None) -> int:
        import ctypes
        out = ctypes.c_int64()
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        self._check(N.lib().gw_exchange_min_watermark(self._h, int(wm), ctypes.byref(out), s))
        return out.value
