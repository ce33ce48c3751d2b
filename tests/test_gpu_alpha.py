"""PBR_FLAG_ALPHA_TEST on the GPU: the reference's ALPHA_TEST permutation (Default.hlsl:111-113).

Every kernel that can run the pass -- the lean pair kernel (uniform loops, no sky pass), the monolithic pair
kernel (PBR_LEAN=0, and every pass with a sky pass), the wave-balanced kernels (>= 22 / 18 point lights), tiled
culling and the one-pixel layout -- must keep a pixel's output untouched where clip(fragOpacity - 0.1f) discards
it and write alpha = fragOpacity elsewhere: bit-identical to the reference build's golden vectors in the exact
mode, within 1e-5 (same discarded set) in the faithful mode.
"""
import os

import numpy as np
import pytest
import torch

from conftest import alpha_golden_names, load_alpha_golden, oracle_pass_from_constants
from oracle import oracle as O
from physically_based_renderer_amd import _native as N
from physically_based_renderer_amd.renderer import GBuffer, PassConstants, ShadingContext

pytestmark = pytest.mark.gpu

REL_TOL = 1e-5


def context(**env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return ShadingContext(0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


VARIANTS = {"default": {}, "monolithic": {"PBR_LEAN": 0}, "one_pixel": {"PBR_PIXELS_PER_THREAD": 1}}


@pytest.fixture(scope="module", params=list(VARIANTS))
def variant_ctx(request, gpu):
    ctx = context(**VARIANTS[request.param])
    yield ctx
    ctx.close()


def pass_for(meta, lights, extra=0):
    flags = N.PBR_FLAG_ALPHA_TEST | (N.PBR_FLAG_F0_PLANE if meta["use_f0_plane"] else 0) | extra
    return PassConstants(eye_pos_w=meta["eye"], ambient_light=meta["ambient"], fresnel_r0=meta["fresnel_r0"],
                         opacity=meta["opacity"], num_dir_lights=meta["n_dir"], num_point_lights=meta["n_point"],
                         num_spot_lights=meta["n_spot"], ambient_mode=meta["ambient_mode"], flags=flags,
                         lights_array=lights)


def run(ctx, gpu, planes, opacity, pc, env=None, sky=None, coverage=None, fmt=N.PBR_OUTPUT_RGBA32F):
    ctx.set_pass(pc)
    if env is not None:
        ctx.set_env_map(env)
    gb = GBuffer.from_host(planes, gpu, opacity=opacity)
    if fmt == N.PBR_OUTPUT_RGBA8_UNORM:
        out = torch.full((gb.height, gb.width, 4), O.UNTOUCHED_U8, dtype=torch.uint8, device=gpu)
    else:
        out = torch.full((gb.height, gb.width, 4), O.UNTOUCHED_F32, dtype=torch.float32, device=gpu)
    if sky is not None or coverage is not None or fmt != N.PBR_OUTPUT_RGBA32F:
        if sky is not None:
            ctx.set_sky_map(sky)
        cov = None if coverage is None else torch.from_numpy(np.ascontiguousarray(coverage, np.uint8)).to(gpu)
        ctx.shade_frame(gb, out, coverage=cov, fmt=fmt)
    else:
        ctx.shade(gb, out)
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("name", alpha_golden_names())
def test_alpha_golden_on_gpu(name, variant_ctx, gpu, env_map):
    g = load_alpha_golden(name, env_map)
    pc = pass_for(g["meta"], g["lights"])
    got = run(variant_ctx, gpu, g["planes"], g["opacity"], pc, g["env"], g["sky"], g["coverage"])
    exp = g["expected"]
    assert np.array_equal(got[..., 3] == O.UNTOUCHED_F32, exp[..., 3] == O.UNTOUCHED_F32)  # same discards
    e = O.rel_err(got, exp)
    print(f"{name}: max_rel={e.max():.3g} bit-identical {O.bit_equal(got, exp).mean():.6f}")
    assert e.max() <= REL_TOL
    assert O.bit_equal(got, exp).mean() >= 0.999


@pytest.mark.parametrize("name", alpha_golden_names())
def test_alpha_golden_faithful(name, gpu, env_map):
    g = load_alpha_golden(name, env_map)
    pc = pass_for(g["meta"], g["lights"], N.PBR_FLAG_FAITHFUL)
    with ShadingContext(0) as ctx:
        got = run(ctx, gpu, g["planes"], g["opacity"], pc, g["env"], g["sky"], g["coverage"])
    exp = g["expected"]
    assert np.array_equal(got[..., 3] == O.UNTOUCHED_F32, exp[..., 3] == O.UNTOUCHED_F32)
    assert O.rel_err(got, exp).max() <= REL_TOL


def scene(rng, h, w, n_point):
    p = np.zeros((15, h, w), np.float32)
    p[0:3] = rng.uniform(-10, 10, (3, h, w))
    n = rng.normal(size=(3, h, w))
    p[3:6] = n / np.linalg.norm(n, axis=0)
    p[6:15] = rng.uniform(0.01, 1, (9, h, w))
    op = rng.uniform(0.0, 0.25, (h, w)).astype(np.float32)
    lights = np.zeros((n_point, 12), np.float32)
    lights[:, 0:3] = rng.uniform(1, 50, (n_point, 3))
    lights[:, 8:11] = rng.uniform(-20, 20, (n_point, 3))
    return p, op, lights


@pytest.mark.parametrize("n_point,flags", [(24, N.PBR_FLAG_FAITHFUL), (24, 0), (40, N.PBR_FLAG_TILED_CULLING),
                                           (8, N.PBR_FLAG_APPLY_AO)])
def test_alpha_kernels_vs_oracle(n_point, flags, gpu):
    """The balanced kernels (24 point lights: both modes), tiled culling and the AO extension."""
    rng = np.random.default_rng(n_point + flags)
    p, op, lights = scene(rng, 40, 200, n_point)
    p[11] = rng.uniform(0, 1, p[11].shape)
    pc = PassConstants(eye_pos_w=(0.0, 2.0, -30.0), num_point_lights=n_point, lights_array=lights,
                       flags=N.PBR_FLAG_ALPHA_TEST | flags, opacity=0.5)
    with ShadingContext(0) as ctx:
        got = run(ctx, gpu, p, op, pc)
        stats = ctx.pass_stats()
    ref = O.shade(list(p) + [op], oracle_pass_from_constants(pc), lights)
    if n_point >= 22 and not flags & N.PBR_FLAG_TILED_CULLING:
        assert stats["backface_tests"] > 0  # the balanced kernel ran
    assert np.array_equal(got[..., 3] == O.UNTOUCHED_F32, ref[..., 3] == O.UNTOUCHED_F32)
    assert O.rel_err(got, ref).max() <= REL_TOL
    if not flags & N.PBR_FLAG_FAITHFUL:
        assert O.bit_equal(got, ref).mean() >= 0.999


def test_alpha_rgba8_frame(gpu, env_map):
    g = load_alpha_golden("alpha_test_frame_sky", env_map)
    pc = pass_for(g["meta"], g["lights"])
    with ShadingContext(0) as ctx:
        got = run(ctx, gpu, g["planes"], g["opacity"], pc, g["env"], g["sky"], g["coverage"], N.PBR_OUTPUT_RGBA8_UNORM)
    f32 = g["expected"]
    discarded = f32[..., 3] == O.UNTOUCHED_F32
    assert (got[discarded] == O.UNTOUCHED_U8).all()
    assert np.abs(got[~discarded].astype(int) - O.unorm8(f32[~discarded]).astype(int)).max() <= 1


def test_alpha_flag_needs_the_plane(gpu):
    rng = np.random.default_rng(5)
    p, op, lights = scene(rng, 8, 64, 2)
    pc = PassConstants(num_point_lights=2, lights_array=lights, flags=N.PBR_FLAG_ALPHA_TEST)
    with ShadingContext(0) as ctx:
        ctx.set_pass(pc)
        with pytest.raises(RuntimeError):
            ctx.shade(GBuffer.from_host(p, gpu))
