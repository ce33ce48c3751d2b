"""The lean pair kernel (shade_lean_kernel, shade_kernels.hip).

Uniform-loop passes without a sky pass run the lean kernel: the monolithic kernel's per-wave choice of fast
loops, every settled pixel finished and stored, then, per pixel, the IEEE path for the pixels the fast loop
sends to the exact re-pass. The bar: every frame and every pass statistic identical to the monolithic kernel's
(PBR_LEAN=0), and within the north-star 1e-5 of the CPU oracle (exact mode: bit-identical but for the documented
x^5 residue). The adversarial G-buffers put each kind of rare pixel (outside the fast window, outside the
faithful conditions, too close to a light, on the eye) next to lean and non-lean (normal-mapped) waves, at a
ragged size whose last tile row has a wave wholly outside the frame.
"""
import os

import numpy as np
import pytest
import torch

from conftest import oracle_pass_from_constants
from oracle import oracle as O
from physically_based_renderer_amd import _native as N
from physically_based_renderer_amd import scenes as S
from physically_based_renderer_amd.renderer import GBuffer, PassConstants, ShadingContext

pytestmark = pytest.mark.gpu

REL_TOL = 1e-5


def context(lean: bool) -> ShadingContext:
    old = os.environ.get("PBR_LEAN")
    os.environ["PBR_LEAN"] = "1" if lean else "0"
    try:
        return ShadingContext(0)  # the context reads PBR_LEAN when it is created
    finally:
        if old is None:
            del os.environ["PBR_LEAN"]
        else:
            os.environ["PBR_LEAN"] = old


@pytest.fixture(scope="module")
def lean_ctx(gpu):
    ctx = context(True)
    yield ctx
    ctx.close()


@pytest.fixture(scope="module")
def mono_ctx(gpu):
    ctx = context(False)
    yield ctx
    ctx.close()


def with_flags(pc, add=0):
    return PassConstants(**{**pc.__dict__, "flags": pc.flags | add})


def run(ctx, gb, pc, env):
    ctx.set_pass(pc)
    if env is not None:
        ctx.set_env_map(env)
    out = ctx.shade(gb)
    torch.cuda.synchronize()
    return out.cpu().numpy(), ctx.pass_stats()


def adversarial(cid, width, height, seed=7):
    """A config's G-buffer at a ragged size with pixels for the exact path."""
    cfg = S.CONFIGS[cid].with_size(width, height)
    planes, _ = S.fill_gbuffer_host(cfg)
    pc = S.scene_pass(cfg)
    p = planes.copy()
    rng = np.random.default_rng(seed)
    lights = pc.light_array()
    hit = lambda: (int(rng.integers(0, height)), int(rng.integers(0, width)))  # noqa: E731
    for _ in range(6):  # outside the fast window: a NaN normal, a huge position
        y, x = hit()
        p[3, y, x] = np.nan
        y, x = hit()
        p[0, y, x] = 3.0e7
    for _ in range(6):  # a negative albedo (faithful precondition; exact mode keeps the wave)
        y, x = hit()
        p[6, y, x] = -0.25
    for _ in range(6):  # 0.004 from a point light: the faithful window (dist >= 0.01) sends the pixel to the re-pass
        y, x = hit()
        p[0:3, y, x] = lights[int(rng.integers(0, len(lights))), 8:11] + np.float32(0.004)
    y, x = hit()  # on the eye: V = 0/0 (the fast normalize's window)
    p[0:3, y, x] = np.asarray(pc.eye_pos_w, np.float32)
    # Normal-mapped rows (|N| != 1): non-lean waves that the lean kernel shades itself.
    p[3:6, 0:2, :] *= np.float32(1.01)
    return cfg, p, pc


@pytest.mark.parametrize("cid", [2, 4])
@pytest.mark.parametrize("faithful", [True, False])
def test_lean_config_frame_equals_monolithic(cid, faithful, lean_ctx, mono_ctx, gpu):
    cfg = S.CONFIGS[cid]
    planes, _ = S.fill_gbuffer_host(cfg)
    pc = S.scene_pass(cfg)
    if faithful:
        pc = with_flags(pc, N.PBR_FLAG_FAITHFUL)
    env = S.env_map() if pc.ambient_mode == N.PBR_AMBIENT_IBL_DIFFUSE else None
    gb = GBuffer.from_host(planes, gpu)
    a, sa = run(lean_ctx, gb, pc, env)
    b, sb = run(mono_ctx, gb, pc, env)
    print(f"{cfg.name} faithful={faithful}: stats {sa}")
    assert O.bit_equal(a, b).all()
    assert sa == sb


@pytest.mark.parametrize("cid,width,height", [(2, 1000, 37), (4, 517, 45)])
@pytest.mark.parametrize("faithful", [True, False])
def test_lean_rare_pixels(cid, width, height, faithful, lean_ctx, mono_ctx, gpu):
    cfg, p, pc = adversarial(cid, width, height)
    if faithful:
        pc = with_flags(pc, N.PBR_FLAG_FAITHFUL)
    env = S.env_map() if pc.ambient_mode == N.PBR_AMBIENT_IBL_DIFFUSE else None
    gb = GBuffer.from_host(p, gpu)
    b, sb = run(mono_ctx, gb, pc, env)
    assert sb["exact_pixels"] > 0  # the frame does send pixels to the exact path
    frames = []
    for _ in range(3):  # repeated passes agree
        a, sa = run(lean_ctx, gb, pc, env)
        frames.append(a)
        assert O.bit_equal(a, b).all()
        assert sa == sb
    ref = O.shade(list(np.ascontiguousarray(p)), oracle_pass_from_constants(pc), pc.light_array(), env, n_threads=16)
    e = O.rel_err(frames[0], ref)
    print(f"cfg{cid} {width}x{height} faithful={faithful}: max_rel={np.nanmax(e):.3g} "
          f"exact_pixels={sb['exact_pixels']} bit-identical to the oracle {O.bit_equal(frames[0], ref).mean():.6f}")
    assert np.nanmax(e) <= REL_TOL
    if not faithful:
        assert O.bit_equal(frames[0], ref).mean() >= 0.9999


def test_lean_passes_on_two_streams(lean_ctx, mono_ctx, gpu):
    """Passes with rare pixels queued on two streams without host syncs (per-stream statistics records)."""
    cfg, p, pc = adversarial(2, 640, 64, seed=11)
    gb = GBuffer.from_host(p, gpu)
    ref, _ = run(mono_ctx, gb, pc, None)
    s1, s2 = torch.cuda.Stream(gpu), torch.cuda.Stream(gpu)
    torch.cuda.synchronize()
    lean_ctx.set_pass(pc)
    outs = []
    for i in range(8):
        st = s1 if i % 2 == 0 else s2
        with torch.cuda.stream(st):
            outs.append(lean_ctx.shade(gb, stream=st))
    torch.cuda.synchronize()
    for o in outs:
        assert O.bit_equal(o.cpu().numpy(), ref).all()


def light_set(pc, kind):
    """Config 4's light list recombined (48-byte records: strength, spot power, direction, pad, position, pad):
    '300pt' -- 300 point lights (the culled walk's first 256 tested on the positions lean_wave preloads, the rest
    by survivor_masks); '2dir_40pt' -- two directional lights ahead of 40 point lights (the preloaded indices
    offset by n_dir, a partial chunk); '100pt_20spot' -- spot lights after the points (no preloaded survivors)."""
    pts = pc.light_array()[: pc.num_point_lights]
    n_dir, n_pt, n_sp = {"300pt": (0, 300, 0), "2dir_40pt": (2, 40, 0), "100pt_20spot": (0, 100, 20)}[kind]
    pt = np.concatenate([pts, pts[: max(n_pt - len(pts), 0)].copy()])[:n_pt]
    pt[len(pts):, 8:11] += np.float32(3.0)  # the repeated lights moved off their originals
    dirs = np.zeros((n_dir, 12), np.float32)
    dirs[:, 0:3] = (0.6, 0.5, 0.4)
    dirs[:, 4:7] = np.asarray([(0.57735026, -0.57735026, 0.57735026), (-0.6, -0.8, 0.0)], np.float32)[:n_dir]
    spots = pts[:n_sp].copy()
    spots[:, 3] = 8.0  # spot power
    spots[:, 4:7] = (0.0, -1.0, 0.0)
    spots[:, 8:11] += np.float32(1.5)
    arr = np.concatenate([dirs, pt, spots]).astype(np.float32)
    return PassConstants(**{**pc.__dict__, "num_dir_lights": n_dir, "num_point_lights": n_pt,
                            "num_spot_lights": n_sp, "lights": [], "lights_array": arr})


@pytest.mark.parametrize("kind", ["300pt", "2dir_40pt", "100pt_20spot"])
@pytest.mark.parametrize("faithful", [True, False])
def test_lean_culled_light_sets(kind, faithful, lean_ctx, mono_ctx, gpu):
    """The culled lean kernel's survivor masks (preloaded for the first 256 point lights when the pass has no spot
    lights) on light sets config 4 does not have: frames and statistics identical to the monolithic kernel's, and
    within the bar of the oracle (exact mode bit-identical but for the x^5 residue)."""
    cfg = S.CONFIGS[4].with_size(517, 45)
    planes, _ = S.fill_gbuffer_host(cfg)
    pc = light_set(S.scene_pass(cfg), kind)
    if faithful:
        pc = with_flags(pc, N.PBR_FLAG_FAITHFUL)
    gb = GBuffer.from_host(planes, gpu)
    a, sa = run(lean_ctx, gb, pc, None)
    assert "shade_lean_kernel" in lean_ctx.last_kernel()
    b, sb = run(mono_ctx, gb, pc, None)
    assert sa["cull_tiles"] > 0 and sa["cull_tile_lights"] > 0  # the pass culled
    assert O.bit_equal(a, b).all()
    assert sa == sb
    ref = O.shade(list(np.ascontiguousarray(planes)), oracle_pass_from_constants(pc), pc.light_array(), None,
                  n_threads=16)
    e = O.rel_err(a, ref)
    print(f"{kind} faithful={faithful}: stats {sa} max_rel={np.nanmax(e):.3g} "
          f"bit-identical {O.bit_equal(a, ref).mean():.6f}")
    assert np.nanmax(e) <= REL_TOL
    if not faithful:
        assert O.bit_equal(a, ref).mean() >= 0.9999
