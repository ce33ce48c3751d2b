"""GPU parity of pbr_shade_frame: the sky pass on background pixels (Skybox.hlsl:37-49), R8G8B8A8_UNORM
output (d3dApp.h:124, D3D FLOAT -> UNORM), fp32 (HDR) textures, against the oracle and the frame
golden vectors (tests/golden/frame_*.npz, made by the reference build).

Bars: background (sky) pixels bit-identical (every op on that path is IEEE or glibc's own
algorithm); geometry pixels within the north_star tolerance 1e-5; RGBA8 channels equal to the
oracle's, or one code apart where the fp32 value sits within the tolerance of a rounding boundary.
"""
import os

import numpy as np
import pytest
import torch

from conftest import frame_golden_names, load_frame_golden, oracle_pass_from_constants, oracle_pass_from_meta
from oracle import oracle as O
from physically_based_renderer_amd import _native as N
from physically_based_renderer_amd import envmap
from physically_based_renderer_amd import scenes as S
from physically_based_renderer_amd.renderer import GBuffer, PassConstants

pytestmark = pytest.mark.gpu

REL_TOL = 1e-5


def unorm8_np(c):
    """D3D FLOAT -> UNORM8 in numpy fp32 (same ops as oracle_unorm8)."""
    c = np.asarray(c, np.float32)
    c = np.where(np.isnan(c), np.float32(0), c)
    c = np.clip(c, np.float32(0), np.float32(1)).astype(np.float32)
    return (c * np.float32(255) + np.float32(0.5)).astype(np.float32).astype(np.uint8)


def pass_from_meta(meta, lights):
    flags = (N.PBR_FLAG_F0_PLANE if meta["use_f0_plane"] else 0) | (N.PBR_FLAG_APPLY_AO if meta["apply_ao"] else 0)
    return PassConstants(eye_pos_w=meta["eye"], ambient_light=meta["ambient"], fresnel_r0=meta["fresnel_r0"],
                         opacity=meta["opacity"], num_dir_lights=meta["n_dir"], num_point_lights=meta["n_point"],
                         num_spot_lights=meta["n_spot"], ambient_mode=meta["ambient_mode"], flags=flags,
                         lights_array=lights)


def run_frame(ctx, gpu, planes, pc, env, sky, coverage, fmt):
    ctx.set_pass(pc)
    if env is not None:
        ctx.set_env_map(env)
    if sky is not None:
        ctx.set_sky_map(sky)
    cov = None if coverage is None else torch.from_numpy(np.ascontiguousarray(coverage, np.uint8)).to(gpu)
    out = ctx.shade_frame(GBuffer.from_host(planes, gpu), coverage=cov, fmt=fmt)
    torch.cuda.synchronize()
    return out.cpu().numpy()


def check(got, ref, coverage, fmt, name):
    bg = np.ones(got.shape[:2], bool) if coverage is None else coverage == 0
    if fmt == N.PBR_OUTPUT_RGBA8_UNORM:
        d = np.abs(got.astype(np.int16) - ref.astype(np.int16))
        print(f"{name}: rgba8 exact={np.mean(d == 0):.6f} max_code_diff={d.max()}")
        assert d.max() <= 1
        assert (d[bg] == 0).all()
    else:
        e = O.rel_err(got, ref)
        print(f"{name}: max_rel={e.max():.3g} bit_exact={O.bit_equal(got, ref).mean():.6f}")
        assert e.max() <= REL_TOL
        assert O.bit_equal(got[bg], ref[bg]).all()


@pytest.mark.parametrize("name", frame_golden_names())
def test_frame_golden_vectors_on_gpu(name, shading_ctx, gpu, env_map):
    g = load_frame_golden(name, env_map)
    pc = pass_from_meta(g["meta"], g["lights"])
    got = run_frame(shading_ctx, gpu, g["planes"], pc, g["env"], g["sky"], g["coverage"], g["meta"]["format"])
    check(got, g["expected"], g["coverage"], g["meta"]["format"], name)


def test_frame_without_coverage_equals_shade_gbuffer(shading_ctx, gpu):
    cfg = S.CONFIGS[3].with_size(512, 48)
    planes, _ = S.fill_gbuffer_host(cfg)
    pc = S.scene_pass(cfg)
    shading_ctx.set_pass(pc)
    shading_ctx.set_env_map(S.env_map())
    gb = GBuffer.from_host(planes, gpu)
    a = shading_ctx.shade(gb).cpu().numpy()
    b = shading_ctx.shade_frame(gb).cpu().numpy()
    c = shading_ctx.shade_frame(gb, fmt=N.PBR_OUTPUT_RGBA8_UNORM).cpu().numpy()
    assert O.bit_equal(a, b).all()
    assert np.array_equal(c, unorm8_np(a))  # the fused conversion == converting the fp32 frame


def test_sphere_frame_with_sky(shading_ctx, gpu):
    """Config 1's 256x256 sphere with its background given to the sky pass: coverage from the fill,
    background normals = the view ray (the sky dome's direction), RGBA8 and fp32 against the oracle."""
    cfg = S.CONFIGS[1]
    planes, covered = S.fill_gbuffer_host(cfg)
    planes2, cov = S.fill_gbuffer_host_coverage(cfg)
    assert np.array_equal(planes.view(np.uint32), planes2.view(np.uint32))
    assert int(cov.sum()) == covered and 0 < covered < cfg.width * cfg.height
    pc = S.scene_pass(cfg)
    sky = envmap.procedural_sky_rgba16(128, 64)
    for fmt in (N.PBR_OUTPUT_RGBA32F, N.PBR_OUTPUT_RGBA8_UNORM):
        got = run_frame(shading_ctx, gpu, planes, pc, None, sky, cov, fmt)
        ref = O.shade_frame(list(planes), oracle_pass_from_constants(pc), pc.light_array(), None, sky, cov,
                            O.OUTPUT_RGBA8 if fmt == N.PBR_OUTPUT_RGBA8_UNORM else O.OUTPUT_RGBA32F, n_threads=8)
        check(got, ref, cov, fmt, f"cfg1 sphere + sky fmt={fmt}")


def test_all_background_and_culled_mixed(shading_ctx, gpu):
    """All-sky frames skip the light loop; a culled pass with background tiles equals the unculled one."""
    cfg = S.CONFIGS[4].with_size(512, 64)
    planes, _ = S.fill_gbuffer_host(cfg)
    pc = S.scene_pass(cfg)
    sky = envmap.procedural_sky_rgba16(96, 48)
    cov0 = np.zeros((64, 512), np.uint8)
    got = run_frame(shading_ctx, gpu, planes, pc, None, sky, cov0, N.PBR_OUTPUT_RGBA32F)
    ref = O.shade_frame(list(planes), oracle_pass_from_constants(pc), pc.light_array(), None, sky, cov0,
                        O.OUTPUT_RGBA32F, n_threads=8)
    assert O.bit_equal(got, ref).all()
    rng = np.random.default_rng(3)
    cov = np.ones((64, 512), np.uint8)
    cov[:, 128:256] = 0  # two whole 64-pixel tile columns of sky
    cov[rng.uniform(size=cov.shape) < 0.1] = 0
    planes[0:3, cov == 0] = np.nan  # background positions are never read for shading or culling
    culled = run_frame(shading_ctx, gpu, planes, pc, None, sky, cov, N.PBR_OUTPUT_RGBA32F)
    kept, tiles = shading_ctx.cull_stats()
    pc_full = PassConstants(**{**pc.__dict__, "flags": pc.flags & ~N.PBR_FLAG_TILED_CULLING})
    full = run_frame(shading_ctx, gpu, planes, pc_full, None, sky, cov, N.PBR_OUTPUT_RGBA32F)
    assert O.bit_equal(culled, full).all()
    tile_w, tile_h = (32, 8) if os.environ.get("PBR_PIXELS_PER_THREAD") == "1" else (64, 2)  # culling unit
    assert tiles == (512 // tile_w - 128 // tile_w) * (64 // tile_h)  # the all-sky tiles did no lighting
    ref = O.shade_frame(list(planes), oracle_pass_from_constants(pc), pc.light_array(), None, sky, cov,
                        O.OUTPUT_RGBA32F, n_threads=8)
    check(culled, ref, cov, N.PBR_OUTPUT_RGBA32F, "cfg4 strip, sky tiles + NaN background, culled")


def test_hdr_env_f32_upload(shading_ctx, gpu):
    """pbr_set_env_map_f32 / pbr_set_sky_map_f32: HDR texels used as given."""
    cfg = S.CONFIGS[3].with_size(384, 32)
    planes, _ = S.fill_gbuffer_host(cfg)
    pc = S.scene_pass(cfg)
    rng = np.random.default_rng(5)
    env = (rng.uniform(0, 1, (90, 180, 4)) ** 4 * 60).astype(np.float32)
    sky = (rng.uniform(0, 1, (45, 90, 4)) ** 4 * 30).astype(np.float32)
    cov = (rng.uniform(size=(32, 384)) > 0.3).astype(np.uint8)
    got = run_frame(shading_ctx, gpu, planes, pc, env, sky, cov, N.PBR_OUTPUT_RGBA32F)
    ref = O.shade_frame(list(planes), oracle_pass_from_constants(pc), pc.light_array(), env, sky, cov,
                        O.OUTPUT_RGBA32F, n_threads=8)
    check(got, ref, cov, N.PBR_OUTPUT_RGBA32F, "cfg3 strip, HDR env + HDR sky")


def test_frame_error_paths(gpu):
    from physically_based_renderer_amd.renderer import ShadingContext

    ctx = ShadingContext(0)
    gb = GBuffer(torch.zeros((15, 8, 8), device=gpu))
    ctx.set_pass(PassConstants())
    cov = torch.zeros((8, 8), dtype=torch.uint8, device=gpu)
    with pytest.raises(N.PbrError) as ei:
        ctx.shade_frame(gb, coverage=cov)  # background pixels but no sky map
    assert ei.value.status == -6
    f = N.FrameDesc()
    out = torch.empty((8, 8, 4), device=gpu)
    f.out, f.out_row_stride, f.format = out.data_ptr(), 8, 7
    g = gb.to_c()
    assert ctx.lib.pbr_shade_frame(ctx.handle, g, f, None) == -1  # unknown format
    f.format, f.out = N.PBR_OUTPUT_RGBA32F, out.data_ptr() + 4
    assert ctx.lib.pbr_shade_frame(ctx.handle, g, f, None) == -1  # misaligned RGBA32F output
    f.format = N.PBR_OUTPUT_RGBA8_UNORM
    assert ctx.lib.pbr_shade_frame(ctx.handle, g, f, None) == 0  # 4-byte aligned is enough for RGBA8
    torch.cuda.synchronize()
    with pytest.raises(ValueError):
        ctx.set_sky_map(np.zeros((4, 4, 4), np.int32))
    ctx.close()


@pytest.mark.parametrize("camera", [None, "overview"])
def test_reference_scene_frame(camera, shading_ctx, gpu):
    """The reference's own scene end to end: ray-cast G-buffer with coverage, PS on the
    58 spheres under the 4 directional lights, sky pass behind, RGBA8 back buffer."""
    cfg = S.REFERENCE_SCENE.with_size(640, 360)
    if camera:
        cfg = cfg.with_camera(*S.OVERVIEW_CAMERA)
    planes, cov = S.fill_gbuffer_host_coverage(cfg)
    pc = S.scene_pass(cfg)
    sky = envmap.procedural_sky_rgba16(256, 128)
    for fmt in (N.PBR_OUTPUT_RGBA32F, N.PBR_OUTPUT_RGBA8_UNORM):
        got = run_frame(shading_ctx, gpu, planes, pc, None, sky, cov, fmt)
        ref = O.shade_frame(list(planes), oracle_pass_from_constants(pc), pc.light_array(), None, sky, cov,
                            O.OUTPUT_RGBA8 if fmt == N.PBR_OUTPUT_RGBA8_UNORM else O.OUTPUT_RGBA32F, n_threads=8)
        check(got, ref, cov, fmt, f"reference scene camera={camera} fmt={fmt}")


def test_one_pixel_layout_matches_pair_layout(gpu, env_map):
    """The 1-pixel-per-work-item kernel (PBR_PIXELS_PER_THREAD=1, 32x8 tiles) is bit-identical to the
    default pixel-pair kernel: plain, culled, with background pixels and RGBA8 output, and under
    EXACT_ONLY."""
    from physically_based_renderer_amd.renderer import ShadingContext

    cfg = S.CONFIGS[4].with_size(300, 40)  # partial tiles in both layouts
    planes, _ = S.fill_gbuffer_host(cfg)
    rng = np.random.default_rng(11)
    cov = (rng.uniform(size=(40, 300)) > 0.2).astype(np.uint8)
    sky = envmap.procedural_sky_rgba16(64, 32)
    pc = S.scene_pass(cfg)
    old = os.environ.get("PBR_PIXELS_PER_THREAD")
    try:
        results = []
        for layout in ("2", "1"):
            os.environ["PBR_PIXELS_PER_THREAD"] = layout
            ctx = ShadingContext(0)
            outs = []
            for flags in (pc.flags, pc.flags & ~N.PBR_FLAG_TILED_CULLING, pc.flags | N.PBR_FLAG_EXACT_ONLY):
                p2 = PassConstants(**{**pc.__dict__, "flags": flags, "ambient_mode": N.PBR_AMBIENT_IBL_DIFFUSE})
                for fmt in (N.PBR_OUTPUT_RGBA32F, N.PBR_OUTPUT_RGBA8_UNORM):
                    outs.append(run_frame(ctx, gpu, planes, p2, env_map, sky, cov, fmt))
            ctx.close()
            results.append(outs)
        for a, b in zip(*results):
            assert (np.array_equal(a, b) if a.dtype == np.uint8 else O.bit_equal(a, b).all())
    finally:
        if old is None:
            os.environ.pop("PBR_PIXELS_PER_THREAD", None)
        else:
            os.environ["PBR_PIXELS_PER_THREAD"] = old
