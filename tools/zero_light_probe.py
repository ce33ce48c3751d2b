"""Shade the cfg3 G-buffer with N lights (default 0), a few times: a target for rocprofv3 --pmc runs
that isolate the per-pixel fixed cost."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from physically_based_renderer_amd import _native as N  # noqa: E402
from physically_based_renderer_amd import scenes as S  # noqa: E402
from physically_based_renderer_amd.renderer import GBuffer, PassConstants, ShadingContext  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 0
ibl = len(sys.argv) > 2 and sys.argv[2] == "ibl"
cfg = S.CONFIGS[3]
planes, _ = S.fill_gbuffer_host(cfg)
lights = S.scene_pass(cfg).light_array()
dev = torch.device("cuda", 0)
gb = GBuffer.from_host(planes, dev)
out = torch.empty((cfg.height, cfg.width, 4), device=dev)
with ShadingContext(0) as ctx:
    ctx.set_env_map(S.env_map())
    ctx.set_pass(PassConstants(num_point_lights=n, lights_array=lights[:max(n, 1)],
                               ambient_mode=N.PBR_AMBIENT_IBL_DIFFUSE if ibl else N.PBR_AMBIENT_CONSTANT))
    for _ in range(5):
        ctx.shade(gb, out)
    torch.cuda.synchronize()
print("done")
