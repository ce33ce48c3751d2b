"""Pass statistics (pbr_last_pass_stats) and the fast-path window, pixel by pixel.

The fast path (exact Markstein divisions and 5-op sqrt, pbr_device_math.h) is only exact inside a
window; a pixel whose values leave it for some light must be re-evaluated by the exact path. The
bit-identity tests elsewhere compare frames, which cannot show a window test that is silently missing
when the fast result happens to round the same. Here the window is driven on purpose and the number of
pixels the kernel sent to the exact path is read back and compared with the count the geometry
implies — separately for the two pixels of a work-item's pair, for waves on the lean loop and on the
general loop, and for a light that is out of range.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from physically_based_renderer_amd import _native as N
from physically_based_renderer_amd import scenes as S
from physically_based_renderer_amd.renderer import GBuffer, PassConstants

pytestmark = pytest.mark.gpu

EYE = (0.0, 5.0, -5.0)


def grazing_gbuffer(kind_a, kind_b, non_lean_waves=False):
    """A 128x8 G-buffer (two 64x8 workgroups) of up-facing pixels (N = +y, roughness 1, albedo 0.5,
    metallic 0: every wave is on the lean loop unless `non_lean_waves`).

    kind_a / kind_b: (H, W) bool masks of the pixels placed so that a light grazes them:
      * A: P.y = 1 - 2^-24 under light 0 at (0, 1, 99) (in range): L.y = 2^-24, N.L ~ 2^-30.6, so
        NDF*G ~ 2^-31.6 is in (0, 2^-30): outside the division window of the specular term;
      * B: P.y = 2 - 2^-23 under light 1 at (0, 2, 150) (out of range, d > 100): the same grazing
        product for a light the pixel does not see (its lane carries a zero-attenuated term that is
        +-0 only inside the window, so the pixel must go to the exact path as well);
    every other pixel sits at P.y = 0, well lit by light 0 (N.L ~ 0.01)."""
    h, w = 8, 128
    p = np.zeros((15, h, w), np.float32)
    xs = np.arange(w, dtype=np.float32)
    p[0] = (xs - 64.0) * 0.25          # P.x in 0 or [2^-2, 16]: inside the position window
    p[1] = np.where(kind_a, np.float32(1.0 - 2.0 ** -24), np.where(kind_b, np.float32(2.0 - 2.0 ** -23), 0.0))
    p[2] = 0.0
    p[4] = 1.0                          # N = (0, 1, 0)
    p[6:9] = 0.5                        # albedo
    p[9] = 0.0                          # metallic
    p[10] = 1.0                         # roughness: k = 0.5, a^2 = 1
    p[11] = 1.0
    p[12:15] = 0.04                     # F0 plane (used with PBR_FLAG_F0_PLANE only)
    if non_lean_waves:
        p[13, :, 5::64] = 0.0           # a zero F0 component in every wave of both workgroups: general loop
    lights = np.zeros((2, 12), np.float32)
    lights[0, 0:3] = 40.0
    lights[0, 8:11] = (0.0, 1.0, 99.0)
    lights[1, 0:3] = 40.0
    lights[1, 8:11] = (0.0, 2.0, 150.0)
    return p, lights


def shade(ctx, p, lights, flags, device):
    pc = PassConstants(eye_pos_w=EYE, num_point_lights=2, flags=flags, lights_array=lights)
    ctx.set_pass(pc)
    out = ctx.shade(GBuffer.from_host(p, device))
    torch.cuda.synchronize()
    return out.cpu().numpy(), ctx.pass_stats()


@pytest.mark.parametrize("pattern", ["odd_a", "even_a", "odd_b", "even_b", "mixed"])
@pytest.mark.parametrize("non_lean", [False, True])
def test_exact_pixels_follow_the_window(pattern, non_lean, shading_ctx, gpu):
    h, w = 8, 128
    yy, xx = np.mgrid[0:h, 0:w]
    rng = np.random.default_rng(7)
    if pattern == "mixed":
        r = rng.uniform(size=(h, w))
        kind_a, kind_b = r < 0.1, (r >= 0.1) & (r < 0.2)
    else:
        sel = (xx % 2 == 1) if pattern.startswith("odd") else (xx % 2 == 0)
        sel &= (yy + xx // 2) % 3 == 0  # not every pair of the row
        kind_a, kind_b = (sel, np.zeros_like(sel)) if pattern.endswith("_a") else (np.zeros_like(sel), sel)
    p, lights = grazing_gbuffer(kind_a, kind_b, non_lean)
    flags = N.PBR_FLAG_F0_PLANE if non_lean else 0
    fast, st = shade(shading_ctx, p, lights, flags, gpu)
    expected = int(kind_a.sum() + kind_b.sum())
    assert st["workgroups"] == 2 and st["culled"] == 0
    assert st["exact_pixels"] == expected, (pattern, non_lean, st)
    exact, st_x = shade(shading_ctx, p, lights, flags | N.PBR_FLAG_EXACT_ONLY, gpu)
    assert st_x["exact_pixels"] == h * w
    assert O.bit_equal(fast, exact).all()
    ref = O.shade(list(p), O.OraclePass(eye=EYE, n_point=2, use_f0_plane=non_lean), lights, None, n_threads=4)
    assert O.rel_err(fast, ref).max() <= 1e-5


def test_pass_stats_on_scene_configs(shading_ctx, gpu):
    """cfg3 (no culling) and cfg4 (tiled culling) at reduced size: the record counts, culling stats equal
    pbr_last_cull_stats, and EXACT_ONLY sends every pixel to the exact path."""
    for cid, size in ((3, (256, 64)), (4, (512, 128))):
        cfg = S.CONFIGS[cid].with_size(*size)
        planes, _ = S.fill_gbuffer_host(cfg)
        pc = S.scene_pass(cfg)
        shading_ctx.set_pass(pc)
        if pc.ambient_mode:
            shading_ctx.set_env_map(S.env_map())
        gb = GBuffer.from_host(planes, gpu)
        shading_ctx.shade(gb)
        st = shading_ctx.pass_stats()
        kept, tiles = shading_ctx.cull_stats()
        assert st["workgroups"] == ((size[0] + 63) // 64) * ((size[1] + 7) // 8)
        culled = bool(pc.flags & N.PBR_FLAG_TILED_CULLING)
        assert st["culled"] == int(culled)
        assert (st["cull_tile_lights"], st["cull_tiles"]) == (kept, tiles)
        if culled:
            assert tiles == st["workgroups"] * 4  # four 64x2 waves per workgroup, all covered
        else:
            assert (kept, tiles) == (0, 0)
        print(f"cfg{cid} {size}: {st}")
        assert st["exact_pixels"] <= size[0] * size[1] // 1000  # scene data stays in the window
        from physically_based_renderer_amd.renderer import PassConstants as PC
        shading_ctx.set_pass(PC(**{**pc.__dict__, "flags": pc.flags | N.PBR_FLAG_EXACT_ONLY}))
        shading_ctx.shade(gb)
        assert shading_ctx.pass_stats()["exact_pixels"] == size[0] * size[1]
