"""Kernel time vs light count on a fixed G-buffer: separates the per-pixel fixed cost (V, BRDF
invariants, ambient, tonemap, gamma) from the per-light cost. Prints one line per light count.

    python tools/light_sweep.py [--width 3840 --height 2160] [--ibl] [--flags 16]
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from physically_based_renderer_amd import _native as N  # noqa: E402
from physically_based_renderer_amd import scenes as S  # noqa: E402
from physically_based_renderer_amd.renderer import GBuffer, PassConstants, ShadingContext  # noqa: E402
from clock_ramp import clock_ramp  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--ibl", action="store_true")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--flags", type=int, default=0, help="extra pass flags, e.g. 16 = PBR_FLAG_FAITHFUL")
    ap.add_argument("--counts", type=int, nargs="+", default=[0, 1, 2, 4, 8, 16, 32, 64])
    ap.add_argument("--no-floor", action="store_true")
    a = ap.parse_args()
    cfg = S.CONFIGS[3].with_size(a.width, a.height)
    planes, _ = S.fill_gbuffer_host(cfg)
    base = S.scene_pass(cfg.with_size(a.width, a.height))
    lights = S.scene_pass(S.CONFIGS[3]).light_array()
    dev = torch.device("cuda", 0)
    gb = GBuffer.from_host(planes, dev)
    out = torch.empty((a.height, a.width, 4), device=dev)
    px = a.width * a.height
    with ShadingContext(0) as ctx:
        ctx.set_env_map(S.env_map())
        ctx.set_pass(base)
        clock_ramp(ctx, gb, out)
        prev = None
        for n in a.counts:
            pc = PassConstants(eye_pos_w=base.eye_pos_w, num_point_lights=n, lights_array=lights[:max(n, 1)],
                               ambient_mode=N.PBR_AMBIENT_IBL_DIFFUSE if a.ibl else N.PBR_AMBIENT_CONSTANT,
                               flags=a.flags)
            ctx.set_pass(pc)
            for _ in range(3):
                ctx.shade(gb, out)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
            for e0, e1 in ev:
                e0.record()
                ctx.shade(gb, out)
                e1.record()
            torch.cuda.synchronize()
            ms = float(np.median([e0.elapsed_time(e1) for e0, e1 in ev]))
            slope = "" if prev is None else f"  +{(ms - prev[1]) / (n - prev[0]) * 1e6 / px * 1e3:.3f} ps/px/light"
            print(f"lights {n:3d}: {ms:.4f} ms  {px / ms / 1e3:9.1f} Mpix/s{slope}", flush=True)
            prev = (n, ms)
        # Memory floor for the same bytes: read the 11 planes the constant-ambient pass reads (sum over planes,
        # 44 B/px in, 4 B/px out) and write the 16 B/px RGBA output (fill), each timed alone.
        def timed(fn):
            for _ in range(3):
                fn()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
            for e0, e1 in ev:
                e0.record()
                fn()
                e1.record()
            torch.cuda.synchronize()
            return float(np.median([e0.elapsed_time(e1) for e0, e1 in ev]))
        if a.no_floor:
            return
        src = gb.planes[:11]
        acc = torch.empty((a.height, a.width), device=dev)
        t_rd = timed(lambda: torch.sum(src, dim=0, out=acc))
        t_wr = timed(lambda: out.fill_(0.5))
        print(f"memory floor: read 11 planes {t_rd:.4f} ms ({44 * px / t_rd / 1e6:.0f} GB/s), write RGBA "
              f"{t_wr:.4f} ms ({16 * px / t_wr / 1e6:.0f} GB/s), sum {t_rd + t_wr:.4f} ms", flush=True)


if __name__ == "__main__":
    main()
