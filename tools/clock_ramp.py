"""Untimed back-to-back shading before a measurement: the MI355X clock ramps over the first ~40 ms
of launches (kernel trace: 2.05 -> 1.75 ms per cfg3 pass), see bench.py --ramp-ms."""
import time

import torch


def clock_ramp(ctx, gb, out, ms: float = 200.0) -> int:
    t0 = time.perf_counter()
    n = 0
    while True:
        ctx.shade(gb, out)
        n += 1
        if n % 8 == 0:
            torch.cuda.synchronize()
            if time.perf_counter() - t0 >= ms / 1e3:
                return n
