"""Tail-effect probe: time one config's pass at several frame heights (same width, scene, lights, mode) and print
ms, Mpix/s and the number of waves against the device's wave slots, to see whether a frame whose wave count is
just above a multiple of the resident slots pays for a nearly empty last round.
usage: python tools/tail_probe.py [--config 2] [--heights 960 1024 1080 1152] [--flags 16] [--reps 100]"""
import argparse
import json
import os
import sys
from dataclasses import replace

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--heights", type=int, nargs="+", default=[960, 1024, 1040, 1080, 1120, 1152])
    ap.add_argument("--flags", type=int, default=16)
    ap.add_argument("--reps", type=int, default=100)
    a = ap.parse_args()
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import numpy as np
    import torch

    from clock_ramp import clock_ramp
    from physically_based_renderer_amd import scenes as S
    from physically_based_renderer_amd.renderer import GBuffer, ShadingContext

    dev = torch.device("cuda", 0)
    base = S.CONFIGS[a.config]
    with ShadingContext(0) as ctx:
        for h in a.heights:
            cfg = replace(base, height=h)
            planes, _ = S.fill_gbuffer_host(cfg)
            pc = S.scene_pass(cfg)
            pc.flags = int(pc.flags) | a.flags
            gb = GBuffer.from_host(planes, dev)
            out = torch.empty((cfg.height, cfg.width, 4), device=dev)
            ctx.set_pass(pc)
            if pc.ambient_mode:
                ctx.set_env_map(S.env_map())
            clock_ramp(ctx, gb, out)
            stream = torch.cuda.current_stream(dev)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
            for s, e in ev:
                s.record(stream)
                ctx.shade(gb, out, stream)
                e.record(stream)
            torch.cuda.synchronize()
            ms = float(np.median([s.elapsed_time(e) for s, e in ev]))
            waves = ((cfg.width + 63) // 64) * ((h + 1) // 2)
            print(json.dumps({"config": a.config, "width": cfg.width, "height": h, "waves": waves,
                              "median_ms": ms, "mpix_s": cfg.width * h / ms / 1e3,
                              "ns_per_wave": ms * 1e6 / waves}), flush=True)
            del gb, out


if __name__ == "__main__":
    main()
