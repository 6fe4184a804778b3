"""Host-side cost per watermark step of the bench loop (ingest / advance / clear), with
the same operator configuration as bench.py, on a small batch so the GPU is never the
bottleneck."""
import ctypes
import sys
import time

import torch

sys.path.insert(0, ".")
from flink_amd import _native as N  # noqa: E402
from flink_amd import windowing as W  # noqa: E402

torch.cuda.set_device(0)
n = 1 << 17
steps = 400
K = 10_000_000
keys = torch.randint(0, K, (steps * n,), device="cuda", dtype=torch.int64)
ts = 1_700_000_000_000 + torch.arange(steps * n, device="cuda", dtype=torch.int64) // 1000
vals = torch.ones_like(keys)
op = W.GpuWindowOperator(W.SlidingEventTimeWindows.of(10_000_000, 2_000_000), "sum_i64", capacity_hint=K,
                         max_batch=n * 2, flags=N.FLAG_FORCE_REGION).open()
cur = torch.cuda.current_stream().cuda_stream
L = N.lib()
for timing in (False, True):
    op.enable_kernel_timing(timing)
    t_ing = t_adv = t_clr = t_sl = 0.0
    for b in range(steps):
        a0 = time.perf_counter()
        lo, hi = b * n, (b + 1) * n
        k, t, v = keys[lo:hi], ts[lo:hi], vals[lo:hi]
        a1 = time.perf_counter()
        N.check(L.gw_ingest_device(op.handle, n, k.data_ptr(), None, t.data_ptr(), v.data_ptr(), cur), op.handle)
        a2 = time.perf_counter()
        op.advance_watermark(int(1_700_000_000_000 + hi // 1000 - 200))
        a3 = time.perf_counter()
        op.clear_rows()
        a4 = time.perf_counter()
        if b >= 20:
            t_sl += a1 - a0; t_ing += a2 - a1; t_adv += a3 - a2; t_clr += a4 - a3
    m = steps - 20
    print(f"timing={timing}: per step us: slice {t_sl / m * 1e6:.1f} ingest {t_ing / m * 1e6:.1f} "
          f"advance {t_adv / m * 1e6:.1f} clear {t_clr / m * 1e6:.1f}", flush=True)
op.close()
