"""Where config 4's time goes (256 point lights, tiled culling, F0 plane, ~5 lights per tile).

Times, with HIP events on the launch stream, config 4 and variants that remove one cost at a time:
every light culled away (fixed per-pixel cost + culling), no lights (fixed cost only), no F0 plane,
and the config-3 G-buffer with the same mean light count unculled. Also prints the per-tile survivor
distribution computed on the host from the tile AABBs.

    python tools/cfg4_probe.py [--reps 30]
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


def time_pass(ctx, gb, out, pc, reps):
    """Median launch time of `reps` back-to-back passes (events recorded between launches, one sync)."""
    ctx.set_pass(pc)
    for _ in range(3):
        ctx.shade(gb, out)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in ev:
        e0.record()
        ctx.shade(gb, out)
        e1.record()
    torch.cuda.synchronize()
    return float(np.median([e0.elapsed_time(e1) for e0, e1 in ev]))


def tile_survivors(planes, lights, tw=64, th=2, radius=100.01):
    h, w = planes.shape[1:]
    p = planes[0:3].reshape(3, h // th, th, w // tw, tw)
    lo = p.min(axis=(2, 4)).reshape(3, -1).T
    hi = p.max(axis=(2, 4)).reshape(3, -1).T
    pos = lights[:, 8:11]
    cnt = np.zeros(lo.shape[0], dtype=np.int64)
    for lp in pos:
        d = np.maximum(np.maximum(lo - lp, lp - hi), 0.0)
        cnt += (np.sqrt((d * d).sum(1)) <= radius)
    return cnt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    cfg4 = S.CONFIGS[4]
    planes, _ = S.fill_gbuffer_host(cfg4)
    base = S.scene_pass(cfg4)
    lights = base.light_array()
    cnt = tile_survivors(planes, lights)
    print(f"tiles {cnt.size}: survivors mean {cnt.mean():.2f} p50 {np.median(cnt):.0f} p99 "
          f"{np.percentile(cnt, 99):.0f} max {cnt.max()}", flush=True)
    dev = torch.device("cuda", 0)
    gb = GBuffer.from_host(planes, dev)
    out = torch.empty((cfg4.height, cfg4.width, 4), device=dev)
    far = lights.copy()
    far[:, 9] += 1.0e4  # every light > 100 units above the plane: all culled
    f0c = N.PBR_FLAG_F0_PLANE | N.PBR_FLAG_TILED_CULLING

    def pc(arr, n, flags):
        return PassConstants(eye_pos_w=base.eye_pos_w, ambient_light=base.ambient_light, num_point_lights=n,
                             lights_array=arr[:max(n, 1)], ambient_mode=N.PBR_AMBIENT_CONSTANT, flags=flags)

    rows = [
        ("cfg4 as benchmarked", pc(lights, 256, f0c)),
        ("all 256 lights culled away", pc(far, 256, f0c)),
        ("0 lights, F0 plane, culling on", pc(lights, 0, f0c)),
        ("0 lights, F0 plane", pc(lights, 0, N.PBR_FLAG_F0_PLANE)),
        ("0 lights, metallic workflow", pc(lights, 0, 0)),
    ]
    with ShadingContext(0) as ctx:
        ctx.set_pass(rows[0][1])
        clock_ramp(ctx, gb, out)
        for name, p in rows:
            ms = time_pass(ctx, gb, out, p, a.reps)
            extra = ""
            if p.flags & N.PBR_FLAG_TILED_CULLING:
                s, t = ctx.cull_stats()
                extra = f"  L_in {s / max(t, 1):.2f}"
            print(f"{name:32s} {ms:8.4f} ms  {cfg4.width * cfg4.height / ms / 1e3:9.1f} Mpix/s{extra}", flush=True)
        cfg3 = S.CONFIGS[3]
        p3, _ = S.fill_gbuffer_host(cfg3)
        gb3 = GBuffer.from_host(p3, dev)
        l3 = S.scene_pass(cfg3).light_array()
        for n in (0, 5, 8):
            p = PassConstants(eye_pos_w=S.scene_pass(cfg3).eye_pos_w, num_point_lights=n, lights_array=l3[:max(n, 1)],
                              ambient_mode=N.PBR_AMBIENT_CONSTANT)
            ms = time_pass(ctx, gb3, out, p, a.reps)
            print(f"{'cfg3 G-buffer, %d lights' % n:32s} {ms:8.4f} ms  {cfg3.width * cfg3.height / ms / 1e3:9.1f} Mpix/s",
                  flush=True)


if __name__ == "__main__":
    main()
