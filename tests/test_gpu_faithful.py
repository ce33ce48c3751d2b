"""PBR_FLAG_FAITHFUL (tolerance mode): hardware-reciprocal divisions in the well-conditioned BRDF terms.

Bar (north_star): |gpu - cpu| <= 1e-5 * |cpu| per RGBA channel against the CPU oracle of the reference
math. The mode is not bit-identical by design, so each test also shows that it ran (some channels differ
from the exact default) or, where its host preconditions fail, that the pass stayed exact (bit-identical
to the default mode).
"""
import numpy as np
import pytest
import torch

from conftest import golden_names, load_golden, oracle_pass_from_constants
from oracle import oracle as O
from physically_based_renderer_amd import _native as N
from physically_based_renderer_amd import scenes as S
from physically_based_renderer_amd.renderer import GBuffer, PassConstants

pytestmark = pytest.mark.gpu

REL_TOL = 1e-5


def with_flags(pc, add=0, remove=0):
    return PassConstants(**{**pc.__dict__, "flags": (pc.flags | add) & ~remove})


def shade(ctx, gb, pc, env):
    ctx.set_pass(pc)
    if env is not None:
        ctx.set_env_map(env)
    out = ctx.shade(gb)
    torch.cuda.synchronize()
    return out.cpu().numpy()


# cfg4's normal-mapped material plane has waves outside the lean conditions (|N|^2 > 1 + 2^-20, zero F0
# components), which stay on the exact loop: the mode need not show there.
@pytest.mark.parametrize("cid,size,row_step,active", [(2, None, 1, True), (3, None, 8, True), (4, None, 8, False),
                                                      (3, (1024, 128), 1, True)])
def test_faithful_config_within_tolerance(cid, size, row_step, active, shading_ctx, gpu):
    cfg = S.CONFIGS[cid] if size is None else S.CONFIGS[cid].with_size(*size)
    planes, _ = S.fill_gbuffer_host(cfg)
    pc = S.scene_pass(cfg)
    env = S.env_map() if pc.ambient_mode == N.PBR_AMBIENT_IBL_DIFFUSE else None
    gb = GBuffer.from_host(planes, gpu)
    fast = shade(shading_ctx, gb, with_flags(pc, N.PBR_FLAG_FAITHFUL), env)
    exact = shade(shading_ctx, gb, pc, env)
    ref = O.shade(list(np.ascontiguousarray(planes[:, ::row_step])), oracle_pass_from_constants(pc),
                  pc.light_array(), env, n_threads=16)
    e = O.rel_err(fast[::row_step], ref)
    same = O.bit_equal(fast, exact).mean()
    print(f"{cfg.name} {cfg.width}x{cfg.height}: faithful max_rel={e.max():.3g} "
          f"bit-identical to exact {same:.4f}")
    assert e.max() <= REL_TOL
    if active:
        assert same < 1.0  # the faithful loop ran
    assert O.rel_err(exact[::row_step], ref).max() <= REL_TOL


@pytest.mark.parametrize("name", golden_names())
def test_faithful_golden_vectors(name, shading_ctx, gpu, env_map):
    """The golden fixtures (edge pixels with NaN/inf/subnormals/|N| > 1 included): waves outside the
    mode's conditions stay exact, the rest are within the tolerance."""
    from test_gpu_parity import pass_from_meta

    planes, lights, meta, expected = load_golden(name)
    pc = with_flags(pass_from_meta(meta, lights), N.PBR_FLAG_FAITHFUL)
    gb = GBuffer.from_host(planes, gpu)
    got = shade(shading_ctx, gb, pc, env_map if meta["env"] else None)
    e = O.rel_err(got, expected)
    print(f"{name}: faithful max_rel={e.max():.3g}")
    assert e.max() <= REL_TOL
    assert np.array_equal(np.isnan(got), np.isnan(expected))


@pytest.mark.parametrize("case", ["negative_strength", "negative_ambient", "exact_only", "65_lights"])
def test_faithful_preconditions_keep_the_pass_exact(case, shading_ctx, gpu):
    """Where a light term could be negative (strength, ambient) or the sum is longer than the bound
    allows (> 64 lights) the error bound does not hold: the host turns the mode off and the frame
    equals the default (exact) mode bit for bit."""
    import dataclasses

    cfg = S.CONFIGS[2].with_size(512, 64)
    if case == "65_lights":
        cfg = dataclasses.replace(cfg, n_lights=65)
    planes, _ = S.fill_gbuffer_host(cfg)
    pc = S.scene_pass(cfg)
    if case == "negative_strength":
        arr = pc.light_array().copy()
        arr[3, 1] = -1.0
        pc = PassConstants(**{**pc.__dict__, "lights_array": arr})
    elif case == "negative_ambient":
        pc = PassConstants(**{**pc.__dict__, "ambient_light": (0.03, -0.01, 0.03)})
    extra = N.PBR_FLAG_EXACT_ONLY if case == "exact_only" else 0
    gb = GBuffer.from_host(planes, gpu)
    exact = shade(shading_ctx, gb, with_flags(pc, extra), None)
    fast = shade(shading_ctx, gb, with_flags(pc, N.PBR_FLAG_FAITHFUL | extra), None)
    assert O.bit_equal(fast, exact).all()


def test_faithful_negative_albedo_waves_stay_exact(shading_ctx, gpu):
    """Per-wave condition: a pixel pair with a negative albedo or F0 > 1 keeps its wave on the exact loop."""
    cfg = S.CONFIGS[2].with_size(256, 16)
    planes, _ = S.fill_gbuffer_host(cfg)
    pc = S.scene_pass(cfg)
    planes = planes.copy()
    # every wave (64x2 pixels) gets one pixel with a negative albedo channel
    planes[7, ::2, ::64] = -0.25
    gb = GBuffer.from_host(planes, gpu)
    exact = shade(shading_ctx, gb, pc, None)
    fast = shade(shading_ctx, gb, with_flags(pc, N.PBR_FLAG_FAITHFUL), None)
    assert O.bit_equal(fast, exact).all()
