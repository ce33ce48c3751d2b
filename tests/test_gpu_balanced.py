"""Wave-balanced point-light lists (pbr_balanced.h): back-face rejection + cross-lane rebalancing.

The balanced kernel evaluates each live (pixel, light) item with the same operations as the packed uniform
loop and skips only items whose reference term is +-0.
* Faithful passes: it sums each pixel's live terms in two interleaved partial sums, so its frames differ from
  the unbalanced faithful kernel's by the association of the sum only: both must be within the north-star
  1e-5 of the oracle, and within a few ulps of each other.
* Exact (default) passes: each pixel's sum continues from its directional lights through its live point
  lights in light order, so the frames are bit-identical to the unbalanced kernel's and to the oracle's.
The contexts here choose the path through PBR_BALANCED_MIN, which pbr_context_create reads (0 = never
balanced, 1 = every untiled pass with point lights only).
"""
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
ASSOC_TOL = 64 * 2.0 ** -23  # <= 64 summed non-negative terms: re-association moves the sum by <= 1 ulp per term


def close(a, b):
    """Frames that differ only by the association of the light sum (NaN == NaN)."""
    return O.rel_err(a, b).max() <= ASSOC_TOL


@pytest.fixture(scope="module")
def ctx_pair(gpu):
    """(balanced, unbalanced) shading contexts."""
    import os

    old = os.environ.get("PBR_BALANCED_MIN")
    os.environ["PBR_BALANCED_MIN"] = "1"
    bal = ShadingContext(0)
    os.environ["PBR_BALANCED_MIN"] = "0"
    plain = ShadingContext(0)
    if old is None:
        del os.environ["PBR_BALANCED_MIN"]
    else:
        os.environ["PBR_BALANCED_MIN"] = old
    yield bal, plain
    bal.close()
    plain.close()


def faithful(pc):
    return PassConstants(**{**pc.__dict__, "flags": pc.flags | N.PBR_FLAG_FAITHFUL})


def exact(pc):
    return PassConstants(**{**pc.__dict__, "flags": pc.flags & ~N.PBR_FLAG_FAITHFUL})


MODES = ["faithful", "exact"]


def check_mode(mode, got, want, ref):
    """Faithful: the association bound against the unbalanced frame and 1e-5 against the oracle; exact: the
    same bits as both (NaN payloads aside)."""
    if mode == "exact":
        assert O.bit_equal(got, want).all()
        assert O.bit_equal(got, ref).all()
    else:
        assert close(got, want)
        assert O.rel_err(got, ref).max() <= REL_TOL


def run(ctx, gb, pc, env=None):
    ctx.set_pass(pc)
    if env is not None:
        ctx.set_env_map(env)
    out = ctx.shade(gb)
    torch.cuda.synchronize()
    return out.cpu().numpy(), ctx.pass_stats()["exact_pixels"]


@pytest.mark.parametrize("cid,size", [(2, (1920, 256)), (3, (1024, 256)), (3, (1000, 77)), (1, None)])
def test_balanced_equals_unbalanced_and_oracle(cid, size, ctx_pair, gpu, env_map):
    """Scene configs (odd sizes included: partial waves and tiles): same frames up to the sum's association,
    same redo sets."""
    cfg = S.CONFIGS[cid] if size is None else S.CONFIGS[cid].with_size(*size)
    planes, _ = S.fill_gbuffer_host(cfg)
    pc = faithful(S.scene_pass(cfg))
    env = env_map if pc.ambient_mode == N.PBR_AMBIENT_IBL_DIFFUSE else None
    gb = GBuffer.from_host(planes, gpu)
    bal, plain = ctx_pair
    got, redo_b = run(bal, gb, pc, env)
    want, redo_p = run(plain, gb, pc, env)
    ref = O.shade(list(planes), oracle_pass_from_constants(pc), pc.light_array(), env, n_threads=16)
    e = O.rel_err(got, ref)
    print(f"{cfg.name} {cfg.width}x{cfg.height}: balanced max_rel={e.max():.3g}, redo {redo_b} vs {redo_p}")
    assert close(got, want)
    assert redo_b == redo_p
    assert e.max() <= REL_TOL


def _scene(rng, w, h, n_lights):
    n = w * h
    pos = np.stack([rng.uniform(-10, 10, n), rng.uniform(-10, 10, n), rng.uniform(0, 10, n)], 1)
    nrm = rng.normal(size=(n, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    planes = np.zeros((15, h, w), np.float32)
    planes[0:3] = pos.T.reshape(3, h, w)
    planes[3:6] = nrm.T.reshape(3, h, w)
    planes[6:9] = rng.uniform(0, 1, (3, h, w))
    planes[9] = rng.uniform(0, 1, (h, w))
    planes[10] = rng.uniform(0, 1, (h, w))
    planes[11] = 1.0
    lights = np.zeros((n_lights, 12), np.float32)
    lights[:, 0:3] = rng.uniform(0, 100, (n_lights, 3))
    lights[:, 8:11] = np.stack([rng.uniform(-20, 20, n_lights), rng.uniform(-20, 20, n_lights),
                                rng.uniform(-20, 0, n_lights)], 1)
    return planes, lights


@pytest.mark.parametrize("mode", MODES)
def test_balanced_back_face_edges(mode, ctx_pair, gpu):
    """Items at the edges of the back-face test:
    * L == -V exactly (eye, pixel and light collinear, pixel facing the eye): the reference's
      H = normalize(V + L) is NaN, but max(dot(N, H), 0) and saturate(dot(H, V)) map it to 0 and with
      N.L = -1 the term is +0, so the item is skipped (the unbalanced loop sends the pixel to the exact
      re-pass instead, for its |V + L| window: same bits, different redo counts);
    * the pixel on a light (l == 0: the reference's L = 0 / 0 is NaN, absorbed the same way; the item stays
      live through the test's 2^-120 seed and the dist window sends the pixel to the exact re-pass);
    * N.L within a few ulps of 0 (lights in the pixel's tangent plane, slightly behind / in front);
    * a light beyond the 100-unit range behind the pixel, and lights 1e-3 behind it."""
    rng = np.random.default_rng(7)
    w, h, nl = 128, 4, 20
    planes, lights = _scene(rng, w, h, nl)
    eye = np.array([0.0, 0.0, -5.0], np.float32)
    # row 0: pixels on the z axis facing the eye, a light straight behind each (L == -V exactly)
    for x in range(0, 16):
        z = np.float32(x * 0.5)
        planes[0:3, 0, x] = (0.0, 0.0, z)
        planes[3:6, 0, x] = (0.0, 0.0, -1.0)
    lights[0, 8:11] = (0.0, 0.0, 20.0)
    # row 1: pixels exactly on light 1 and on light 2
    planes[0:3, 1, 0] = lights[1, 8:11]
    planes[0:3, 1, 1] = lights[2, 8:11]
    # row 2: tangent-plane lights: N = +y, light j at the pixel's height +- a few ulps
    for x in range(0, 32):
        p = np.array([x * 0.25 - 4.0, 1.0, 2.0], np.float32)
        planes[0:3, 2, x] = p
        planes[3:6, 2, x] = (0.0, 1.0, 0.0)
    for j, dy in zip(range(3, 9), (0.0, 1e-7, -1e-7, 1e-6, -1e-6, 3e-5)):
        lights[j, 8:11] = (5.0, np.float32(1.0) + np.float32(dy), 2.5)
    # row 3: lights just behind (1e-3) and far behind (150) the pixel
    planes[0:3, 3, 0] = (1.0, 1.0, 1.0)
    planes[3:6, 3, 0] = (0.0, 0.0, -1.0)
    lights[9, 8:11] = (1.0, 1.0, 1.001)
    lights[10, 8:11] = (1.0, 1.0, 151.0)
    flags = N.PBR_FLAG_FAITHFUL if mode == "faithful" else 0
    pc = PassConstants(eye_pos_w=tuple(eye), num_point_lights=nl, lights_array=lights, flags=flags)
    gb = GBuffer.from_host(planes, gpu)
    bal, plain = ctx_pair
    got, redo_b = run(bal, gb, pc)
    want, redo_p = run(plain, gb, pc)
    ref = O.shade(list(planes), oracle_pass_from_constants(pc), pc.light_array(), None, n_threads=4)
    print(f"edges ({mode}): redo {redo_b} vs {redo_p}; NaN pixels {int(np.isnan(ref[..., 0]).sum())}")
    assert np.isfinite(ref[0, :16]).all()  # the L == -V pixels: the NaN H is absorbed by maxNum
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    assert redo_b <= redo_p
    check_mode(mode, got, want, ref)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("n_lights", [1, 31, 32, 33, 63, 64])
def test_balanced_light_counts(n_lights, mode, ctx_pair, gpu):
    """Mask-word boundaries (32 lights per word) and the one-light pass."""
    rng = np.random.default_rng(100 + n_lights)
    planes, lights = _scene(rng, 256, 8, n_lights)
    flags = N.PBR_FLAG_FAITHFUL if mode == "faithful" else 0
    pc = PassConstants(num_point_lights=n_lights, lights_array=lights, flags=flags)
    gb = GBuffer.from_host(planes, gpu)
    bal, plain = ctx_pair
    got, _ = run(bal, gb, pc)
    want, _ = run(plain, gb, pc)
    ref = O.shade(list(planes), oracle_pass_from_constants(pc), pc.light_array(), None, n_threads=4)
    check_mode(mode, got, want, ref)


@pytest.mark.parametrize("cid,size", [(2, (1920, 256)), (3, (1024, 256)), (3, (1000, 77))])
def test_balanced_exact_scene_configs(cid, size, ctx_pair, gpu, env_map):
    """Exact (default) passes of the scene configs: bit-identical to the uniform loop and to the oracle."""
    cfg = S.CONFIGS[cid].with_size(*size)
    planes, _ = S.fill_gbuffer_host(cfg)
    pc = exact(S.scene_pass(cfg))
    env = env_map if pc.ambient_mode == N.PBR_AMBIENT_IBL_DIFFUSE else None
    gb = GBuffer.from_host(planes, gpu)
    bal, plain = ctx_pair
    got, redo_b = run(bal, gb, pc, env)
    want, redo_p = run(plain, gb, pc, env)
    ref = O.shade(list(planes), oracle_pass_from_constants(pc), pc.light_array(), env, n_threads=16)
    print(f"{cfg.name} {cfg.width}x{cfg.height} exact: redo {redo_b} vs {redo_p}")
    assert redo_b <= redo_p
    check_mode("exact", got, want, ref)


@pytest.mark.parametrize("mode", MODES)
def test_balanced_after_directional_lights(mode, ctx_pair, gpu):
    """Directional lights ahead of the point lights: faithful passes add the balanced point-light sums to the
    directional ones; exact passes keep the uniform loop (the host gate: the balanced exact variant has no
    directional loop), so both modes must still match."""
    rng = np.random.default_rng(11)
    nd, npt = 3, 40
    planes, lights = _scene(rng, 384, 8, nd + npt)
    d = rng.normal(size=(nd, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    lights[:nd, 4:7] = d
    lights[:nd, 8:11] = 0.0
    flags = N.PBR_FLAG_FAITHFUL if mode == "faithful" else 0
    pc = PassConstants(num_dir_lights=nd, num_point_lights=npt, lights_array=lights, flags=flags)
    gb = GBuffer.from_host(planes, gpu)
    bal, plain = ctx_pair
    got, redo_b = run(bal, gb, pc)
    want, redo_p = run(plain, gb, pc)
    ref = O.shade(list(planes), oracle_pass_from_constants(pc), pc.light_array(), None, n_threads=4)
    assert redo_b <= redo_p
    check_mode(mode, got, want, ref)


@pytest.mark.parametrize("mode", MODES)
def test_balanced_range_cut_in_pass1(mode, ctx_pair, gpu):
    """The range cut `if (d > 100) return 0` (LightingUtil.hlsl:131) as pass 1 applies it (balanced_pass1): lights
    beyond 100.1 of a wave's whole box are dropped for the wave, lights within 99.9 of every corner are kept, and a
    light whose range boundary crosses the box is decided per pixel by the reference's own test, dot(l, l) > 10000
    (beyond_range). Waves (64 x 2 pixels each) here:
    * rows 0-1: a small cluster, 22 lights within 40 units, 2 lights ~300 units away (dropped whole);
    * rows 2-3: pixels facing light 0 at exactly 100 + k 2^-17 (k in [-16, 16)) from it -- the cut at ulp
      granularity -- and the rest of the row nearby (light 0 crosses this box);
    * rows 4-7: positions spread over a 300-unit box (most lights cross it).
    Exact mode: bit-identical to the uniform loop and the oracle; faithful: 1e-5 of the oracle."""
    rng = np.random.default_rng(23)
    w, h, nl = 128, 8, 24
    planes, lights = _scene(rng, w, h, nl)
    planes[0:3, 0:2] = rng.uniform(-2, 2, (3, 2, w))
    lights[:nl - 2, 8:11] = rng.uniform(-20, 20, (nl - 2, 3))
    lights[nl - 2:, 8:11] = (300.0, 0.0, 0.0), (0.0, -290.0, 10.0)
    lights[0, 8:11] = (100.0, 0.0, 0.0)
    k = np.arange(-16, 16, dtype=np.float32)
    for r in (2, 3):
        planes[0:3, r] = rng.uniform(-1, 1, (3, w))
        planes[0, r, :32] = -k * np.float32(2.0 ** -17)  # l.x = 100 + k ulp(100), l.y = l.z = 0
        planes[1:3, r, :32] = 0.0
        planes[3:6, r, :32] = np.array([1.0, 0.0, 0.0], np.float32)[:, None]
    planes[0:3, 4:8] = rng.uniform(-150, 150, (3, 4, w))
    flags = N.PBR_FLAG_FAITHFUL if mode == "faithful" else 0
    pc = PassConstants(num_point_lights=nl, lights_array=lights, flags=flags)
    gb = GBuffer.from_host(planes, gpu)
    bal, plain = ctx_pair
    got, redo_b = run(bal, gb, pc)
    st = bal.pass_stats()
    want, redo_p = run(plain, gb, pc)
    ref = O.shade(list(planes), oracle_pass_from_constants(pc), pc.light_array(), None, n_threads=4)
    # the cut is exercised: light 0 alone reaches half of the straddling pixels
    only0 = PassConstants(num_point_lights=1, lights_array=lights[:1], flags=flags)
    row = np.ascontiguousarray(planes[:, 2:3, :32])
    ref0 = O.shade(list(row), oracle_pass_from_constants(only0), only0.light_array(), None)
    dark0 = O.shade(list(row), oracle_pass_from_constants(PassConstants(flags=flags)), None, None)
    lit0 = ~np.all(ref0[0] == dark0[0], axis=-1)
    assert 0 < lit0.sum() < 32
    print(f"range cut ({mode}): light terms {st['light_terms']} of {st['backface_tests']} tests, redo {redo_b} vs {redo_p}")
    assert st["light_terms"] < st["backface_tests"] // 2  # the far lights and the 300-unit waves' cut items are gone
    assert redo_b <= redo_p
    check_mode(mode, got, want, ref)


@pytest.mark.parametrize("top", [2.0 ** 50, 2.0 ** 51, 1.0e30])
def test_balanced_exact_strength_bound(top, ctx_pair, gpu):
    """The exact balanced items run brdf_x2's QUARTER form (N / 4, k / 4, 16 (a^2 - 1), 16 N.V, 4x strengths: exact
    power-of-two scalings, pbr_balanced.h), whose 4x radiance the host bounds: every point strength within 2^50
    (pbr_context.hip, points_quarter_ok), else the uniform exact loop. Strengths spanning 2^-20 .. `top` (one light
    at `top`, one negative, others over 20 decades): bit-identical to the uniform loop and the oracle either way, and
    the balanced kernel runs exactly when the bound holds."""
    rng = np.random.default_rng(71)
    nl = 24
    planes, lights = _scene(rng, 256, 8, nl)
    lights[:, 0:3] = (10.0 ** rng.uniform(-6, 14, (nl, 3))).astype(np.float32)
    lights[3, 0:3] = (top, 1.0, 2.0 ** -20)
    lights[7, 0:3] = (-5.0e3, 0.0, -2.0 ** -30)  # negative and zero strengths scale exactly too
    pc = PassConstants(num_point_lights=nl, lights_array=lights, flags=0)
    gb = GBuffer.from_host(planes, gpu)
    bal, plain = ctx_pair
    got, redo_b = run(bal, gb, pc)
    kernel = bal.last_kernel()
    want, redo_p = run(plain, gb, pc)
    ref = O.shade(list(planes), oracle_pass_from_constants(pc), pc.light_array(), None, n_threads=4)
    print(f"strengths up to {top:g}: {kernel}, redo {redo_b} vs {redo_p}")
    assert kernel.endswith(", 2>") == (top <= 2.0 ** 50)
    assert redo_b <= redo_p
    check_mode("exact", got, want, ref)


def test_balanced_light_outside_window_sends_all_to_exact(ctx_pair, gpu):
    """A light whose position is outside the fast-path window (|x| > 2^20): every pixel is redone exactly,
    as in the uniform loop (frames bit-identical to the oracle there)."""
    rng = np.random.default_rng(5)
    planes, lights = _scene(rng, 128, 4, 20)
    lights[7, 8] = 3.0e6
    pc = PassConstants(num_point_lights=20, lights_array=lights, flags=N.PBR_FLAG_FAITHFUL)
    gb = GBuffer.from_host(planes, gpu)
    bal, plain = ctx_pair
    got, redo_b = run(bal, gb, pc)
    want, redo_p = run(plain, gb, pc)
    assert redo_b == redo_p == 128 * 4
    assert close(got, want)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("n_on_light", [1, 3, 8, 9, 20, 64])
def test_balanced_repass_after_stores(n_on_light, mode, ctx_pair, gpu):
    """The balanced kernels re-pass their exact pixels after the wave's stores (shade_kernels.hip, repass_exact):
    up to kLanesRepassMax (8) pixels one at a time with the lanes splitting the lights, more with every lane
    taking its own pixels. Pixels placed exactly on a light (the reference's L = 0 / 0: NaN, absorbed by the
    maxNum clamps; the balanced pass's distance window sends them to the re-pass) in one wave of 128 pixels, the
    other waves of the frame untouched: the re-passed pixels, the pixels around them that the wave stored first
    and the redo count all as the uniform loop and the oracle have them."""
    rng = np.random.default_rng(300 + n_on_light)
    w, h, nl = 128, 8, 64
    planes, lights = _scene(rng, w, h, nl)
    # wave 1 of tile 0 covers rows 2-3, columns 0-63 (64 lanes x 2 pixels): put n pixels of it on lights
    cols = rng.permutation(64 * 2)[:n_on_light]
    for i, c in enumerate(cols):
        x, y = int(c % 64), 2 + int(c // 64)
        planes[0:3, y, x] = lights[i % nl, 8:11]
    flags = N.PBR_FLAG_FAITHFUL if mode == "faithful" else 0
    pc = PassConstants(num_point_lights=nl, lights_array=lights, flags=flags)
    gb = GBuffer.from_host(planes, gpu)
    bal, plain = ctx_pair
    got, redo_b = run(bal, gb, pc)
    assert ", false, 1>" in bal.last_kernel() or ", false, 2>" in bal.last_kernel(), bal.last_kernel()
    want, redo_p = run(plain, gb, pc)
    ref = O.shade(list(planes), oracle_pass_from_constants(pc), pc.light_array(), None, n_threads=4)
    print(f"repass ({mode}, {n_on_light} on lights): redo {redo_b} vs {redo_p}, kernel {bal.last_kernel()}")
    assert redo_b >= n_on_light  # every pixel on a light is redone (the rest of the scene stays in the window)
    assert redo_b <= redo_p
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    check_mode(mode, got, want, ref)


@pytest.fixture(scope="module")
def ctx_default(gpu):
    """A context with the built-in per-mode minimums (PBR_BALANCED_MIN unset)."""
    import os

    old = os.environ.pop("PBR_BALANCED_MIN", None)
    ctx = ShadingContext(0)
    if old is not None:
        os.environ["PBR_BALANCED_MIN"] = old
    yield ctx
    ctx.close()


@pytest.mark.parametrize("mode,n_lights", [("faithful", 21), ("faithful", 22), ("exact", 17), ("exact", 18)])
def test_default_balancing_minimum(mode, n_lights, ctx_default, ctx_pair, gpu):
    """The built-in minimums (faithful 22, exact 18 point lights; pbr_context.hip): one light below a minimum
    the default context runs the uniform loop (its frame has the uniform kernel's bits), at the minimum it
    runs the balanced lists; both match the oracle at the mode's bar."""
    rng = np.random.default_rng(500 + n_lights)
    planes, lights = _scene(rng, 256, 8, n_lights)
    flags = N.PBR_FLAG_FAITHFUL if mode == "faithful" else 0
    pc = PassConstants(num_point_lights=n_lights, lights_array=lights, flags=flags)
    gb = GBuffer.from_host(planes, gpu)
    bal, plain = ctx_pair
    got, _ = run(ctx_default, gb, pc)
    want_plain, _ = run(plain, gb, pc)
    want_bal, _ = run(bal, gb, pc)
    ref = O.shade(list(planes), oracle_pass_from_constants(pc), pc.light_array(), None, n_threads=4)
    minimum = 22 if mode == "faithful" else 18
    expect = want_bal if n_lights >= minimum else want_plain
    assert O.bit_equal(got, expect).all()
    check_mode(mode, got, want_plain, ref)


@pytest.mark.parametrize("mode", MODES)
def test_balanced_distance_window_in_pass1(mode, ctx_pair, gpu):
    """The items' distance window (faithful dist >= 0.01, exact >= 2^-20: point_or_spot_*_x2) as pass 1 decides it
    (balanced_pass1: a light whose nearest box point is >= 1.02 x the window from the wave's box needs no test; for
    another one each pixel with the light live runs the item's own test, and a failing pixel is redone on the exact
    path). Row 0: pixels facing light 0 at distances straddling 0.01 and 2^-20 (and on it); row 1: the same distances
    behind the pixels (N.L < 0: the items are skipped, no redo is needed); rows 2-3: ordinary pixels of the same
    waves, farther away. Exact: bit-identical to the uniform loop and the oracle; faithful: 1e-5 of the oracle."""
    rng = np.random.default_rng(31)
    w, h, nl = 128, 4, 24
    planes, lights = _scene(rng, w, h, nl)
    lights[0, 8:11] = (1.0, 2.0, 3.0)
    dists = np.array([0.0, 2.0 ** -21, 2.0 ** -20, 1.5 * 2.0 ** -20, 1e-3, 0.0099, 0.00999999, 0.01, 0.01000001,
                      0.0101, 0.0102, 0.0103, 0.011, 0.02, 0.05, 0.5], np.float32)
    for r, side in ((0, 1.0), (1, -1.0)):
        planes[0:3, r, :16] = np.array([1.0, 2.0, 3.0], np.float32)[:, None]
        planes[2, r, :16] = np.float32(3.0) - dists  # light 0 at +dist along z from the pixel
        planes[3:6, r, :16] = np.array([0.0, 0.0, side], np.float32)[:, None]
    flags = N.PBR_FLAG_FAITHFUL if mode == "faithful" else 0
    pc = PassConstants(num_point_lights=nl, lights_array=lights, flags=flags)
    gb = GBuffer.from_host(planes, gpu)
    bal, plain = ctx_pair
    got, redo_b = run(bal, gb, pc)
    want, redo_p = run(plain, gb, pc)
    ref = O.shade(list(planes), oracle_pass_from_constants(pc), pc.light_array(), None, n_threads=4)
    print(f"distance window ({mode}): redo {redo_b} vs {redo_p}")
    assert 0 < redo_b <= redo_p  # the pixels facing light 0 within the window are redone
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    check_mode(mode, got, want, ref)


@pytest.mark.parametrize("heavy", [0.78, 0.5, 0.95])
def test_balanced_faithful_uneven_waves(heavy, ctx_pair, gpu):
    """Waves whose pixels' live counts are far from even (the case the ranking pairs up): `heavy` of the pixels (more
    on later rows) face all 64 lights, the rest face none, and a fifth take random normals. Within 1e-5 of the oracle
    and within the association bound of the unbalanced kernel."""
    rng = np.random.default_rng(int(heavy * 1000))
    w, h, nl = 256, 8, 64
    planes, lights = _scene(rng, w, h, nl)
    lights[:, 8:11] = np.stack([rng.uniform(-20, 20, nl), rng.uniform(-20, 20, nl), rng.uniform(-30, -15, nl)], 1)
    planes[2] = rng.uniform(0, 5, (h, w))
    face = rng.uniform(0, 1, (h, w)) < heavy * (0.6 + 0.1 * np.arange(h))[:, None]
    randn = rng.uniform(0, 1, (h, w)) < 0.2
    planes[3:6] = np.where(face, np.array([0.0, 0.0, -1.0], np.float32)[:, None, None],
                           np.array([0.0, 0.0, 1.0], np.float32)[:, None, None])
    rn = rng.normal(size=(3, h, w)).astype(np.float32)
    rn /= np.linalg.norm(rn, axis=0, keepdims=True)
    planes[3:6] = np.where(randn, rn, planes[3:6])
    pc = PassConstants(num_point_lights=nl, lights_array=lights, flags=N.PBR_FLAG_FAITHFUL)
    gb = GBuffer.from_host(planes, gpu)
    bal, plain = ctx_pair
    got, redo_b = run(bal, gb, pc)
    st = bal.pass_stats()
    want, redo_p = run(plain, gb, pc)
    ref = O.shade(list(planes), oracle_pass_from_constants(pc), pc.light_array(), None, n_threads=4)
    e = O.rel_err(got, ref)
    print(f"uneven waves (heavy {heavy}): max_rel {e.max():.3g}, light terms {st['light_terms']}, redo {redo_b}")
    assert redo_b <= redo_p
    assert close(got, want)
    assert e.max() <= REL_TOL
