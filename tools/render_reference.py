"""Render the reference's 58-sphere scene end to end on the GPU (ray-cast G-buffer fill, PS on the
spheres, sky pass behind, fused RGBA8 back buffer) and write it as PNG.

    python tools/render_reference.py [--width 1920 --height 1080] [--overview] [--ibl] [--out path.png]
"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from physically_based_renderer_amd import _native as N, envmap, image_io  # noqa: E402
from physically_based_renderer_amd import scenes as S  # noqa: E402
from physically_based_renderer_amd.renderer import GBuffer, ShadingContext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--overview", action="store_true", help="back the camera off to show all 58 spheres")
    ap.add_argument("--ibl", action="store_true", help="diffuse IBL ambient (Chelsea_Stairs) instead of 0.03")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "reference_scene.png"))
    a = ap.parse_args()
    cfg = S.REFERENCE_SCENE.with_size(a.width, a.height)
    if a.overview:
        cfg = cfg.with_camera(*S.OVERVIEW_CAMERA)
    t0 = time.perf_counter()
    planes, cov = S.fill_gbuffer_host_coverage(cfg)
    t_fill = time.perf_counter() - t0
    pc = S.scene_pass(cfg)
    dev = torch.device("cuda", 0)
    with ShadingContext(0) as ctx:
        if a.ibl:
            pc.ambient_mode = N.PBR_AMBIENT_IBL_DIFFUSE
            ctx.set_env_map(S.env_map())
        ctx.set_pass(pc)
        ctx.set_sky_map(envmap.procedural_sky_rgba16(512, 256))
        gb = GBuffer.from_host(planes, dev)
        cv = torch.from_numpy(cov).to(dev)
        img = ctx.shade_frame(gb, coverage=cv, fmt=N.PBR_OUTPUT_RGBA8_UNORM)
        t1 = time.perf_counter()
        while time.perf_counter() - t1 < 0.2:  # GPU clock ramp (bench.py --ramp-ms)
            for _ in range(8):
                ctx.shade_frame(gb, img, coverage=cv, fmt=N.PBR_OUTPUT_RGBA8_UNORM)
            torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
        for e0, e1 in ev:
            e0.record()
            ctx.shade_frame(gb, img, coverage=cv, fmt=N.PBR_OUTPUT_RGBA8_UNORM)
            e1.record()
        torch.cuda.synchronize()
        t_shade = sorted(e0.elapsed_time(e1) for e0, e1 in ev)[len(ev) // 2] / 1e3
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    image_io.write_png_rgba8(a.out, img)
    print(f"{cfg.width}x{cfg.height} covered {cov.mean():.3f}: host fill {t_fill * 1e3:.1f} ms, "
          f"shade+sky+RGBA8 {t_shade * 1e3:.4f} ms (median of 50, HIP events) = "
          f"{cfg.width * cfg.height / t_shade / 1e6:.0f} Mpix/s -> {a.out}")


if __name__ == "__main__":
    main()
