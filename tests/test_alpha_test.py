"""The ALPHA_TEST permutation on the CPU: the C oracle against the reference build's golden vectors.

The reference compiles Default.hlsl a sixth time with ALPHA_TEST = 1 (alphaTestedPS, PBRApp.cpp:750-765):
fragOpacity is sampled from the opacity map and clip(fragOpacity - 0.1f) discards the fragment when that is
negative (Default.hlsl:111-113); a kept pixel's alpha is fragOpacity (Default.hlsl:160). A discarded pixel
leaves the render target as it was, so every output buffer here starts as oracle.UNTOUCHED_F32 / _U8.
tests/golden/alpha_test_*.npz were made by oracle/_ref (the reference's PS text compiled with ALPHA_TEST = 1).
"""
import os

import numpy as np
import pytest

from conftest import alpha_golden_names, load_alpha_golden, oracle_pass_from_meta
from oracle import oracle as O

DEFAULT_HLSL = "/root/reference/Source/Shaders/Default.hlsl"


def oracle_alpha(g, fmt=O.OUTPUT_RGBA32F, fn=None):
    ps = oracle_pass_from_meta(g["meta"])
    planes = list(g["planes"]) + [g["opacity"]]
    if g["coverage"] is not None or fn is not None:
        f = fn or O.shade_frame
        return f(planes, ps, g["lights"], g["env"], g["sky"], g["coverage"], fmt)
    return O.shade(planes, ps, g["lights"], g["env"])


@pytest.mark.parametrize("name", alpha_golden_names())
def test_oracle_matches_alpha_golden(name, env_map):
    g = load_alpha_golden(name, env_map)
    got = oracle_alpha(g)
    assert O.bit_equal(got, g["expected"]).all()


def test_alpha_golden_set():
    names = alpha_golden_names()
    assert {"alpha_test_const", "alpha_test_ibl_f0plane", "alpha_test_frame_sky"} <= set(names)
    for n in names:
        g = load_alpha_golden(n)
        kept = g["expected"][..., 3] != O.UNTOUCHED_F32
        assert 0 < kept.sum() < kept.size  # both outcomes occur


def test_alpha_known_answers(env_map):
    """clip(fragOpacity - 0.1f): the subtraction in fp32, then < 0 (NaN and +0 are kept)."""
    g = load_alpha_golden("alpha_test_const", env_map)
    out = oracle_alpha(g)
    op = g["opacity"][0, :11]
    kept = out[0, :11, 3] != O.UNTOUCHED_F32
    want = ~((op - np.float32(0.1)) < 0)  # NaN compares false: kept
    assert np.array_equal(kept, want)
    # 0.1f itself kept, the float below it discarded, the float above kept; 0, -0 and -inf discarded
    assert list(kept[:5]) == [True, False, True, False, False]
    assert kept[5] and np.isnan(out[0, 5, 3])  # NaN opacity: kept, alpha NaN
    assert out[0, 6, 3] == np.float32(1.5) and out[0, 9, 3] == np.inf and not kept[10]
    shaded = out[..., 3] != O.UNTOUCHED_F32
    assert np.array_equal(out[..., 3][shaded], g["opacity"][shaded], equal_nan=True)  # alpha = fragOpacity


def test_alpha_frame_sky_pixels_are_not_tested(env_map):
    g = load_alpha_golden("alpha_test_frame_sky", env_map)
    out = oracle_alpha(g)
    bg = g["coverage"] == 0
    assert (out[bg][:, 3] == 1.0).all()  # the sky PS has no clip: every background pixel is written, alpha 1
    assert (out[~bg][:, 3] == O.UNTOUCHED_F32).any()


def test_alpha_rgba8_untouched_bytes(env_map):
    g = load_alpha_golden("alpha_test_frame_sky", env_map)
    out = oracle_alpha(g, O.OUTPUT_RGBA8)
    ref = oracle_alpha(g)
    discarded = ref[..., 3] == O.UNTOUCHED_F32
    assert (out[discarded] == O.UNTOUCHED_U8).all()
    assert np.array_equal(out[~discarded], O.unorm8(ref[~discarded]))


def test_alpha_test_off_ignores_opacity(env_map):
    g = load_alpha_golden("alpha_test_const", env_map)
    ps = oracle_pass_from_meta(g["meta"])
    ps.alpha_test = False
    a = O.shade(list(g["planes"]), ps, g["lights"], None)
    b = O.shade(list(g["planes"]) + [g["opacity"]], ps, g["lights"], None)
    assert O.bit_equal(a, b).all() and (a[..., 3] == np.float32(ps.opacity)).all()


@pytest.mark.skipif(not os.path.exists(DEFAULT_HLSL) or not O.ref_available(), reason="reference tree absent")
def test_reference_source_has_the_clip():
    src = open(DEFAULT_HLSL).read()
    assert "clip(fragOpacity - 0.1f);" in src and "g_TextureArray[11].Sample(g_SamPointWrap, TexCoord).r" in src


@pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built (needs /root/reference)")
@pytest.mark.parametrize("seed,amb,f0,fmt", [(1, O.AMBIENT_CONSTANT, False, O.OUTPUT_RGBA32F),
                                             (2, O.AMBIENT_IBL_DIFFUSE, True, O.OUTPUT_RGBA8),
                                             (3, O.AMBIENT_IBL_DIFFUSE, False, O.OUTPUT_RGBA32F)])
def test_oracle_matches_reference_build_alpha_random(seed, amb, f0, fmt, env_map):
    rng = np.random.default_rng(seed)
    h, w = 24, 64
    p = np.zeros((15, h, w), np.float32)
    p[0:3] = rng.uniform(-10, 10, (3, h, w))
    n = rng.normal(size=(3, h, w))
    p[3:6] = n / np.linalg.norm(n, axis=0)
    p[6:15] = rng.uniform(0, 1, (9, h, w))
    op = rng.uniform(-0.1, 0.4, (h, w)).astype(np.float32)
    cov = (rng.uniform(size=(h, w)) > 0.2).astype(np.uint8)
    lights = np.zeros((10, 12), np.float32)
    lights[:, 0:3] = rng.uniform(0, 50, (10, 3))
    lights[:, 3] = 16.0
    lights[:, 4:7] = rng.normal(size=(10, 3))
    lights[:, 8:11] = rng.uniform(-20, 20, (10, 3))
    ps = O.OraclePass(n_dir=2, n_point=6, n_spot=2, ambient_mode=amb, use_f0_plane=f0, alpha_test=True, opacity=0.5)
    sky = (rng.uniform(size=(16, 32, 4)) * 65535).astype(np.uint16)
    planes = list(p) + [op]
    a = O.shade_frame(planes, ps, lights, env_map, sky, cov, fmt)
    b = O.shade_frame_ref(planes, ps, lights, env_map, sky, cov, fmt)
    assert O.bit_equal(a, b).all() if fmt == O.OUTPUT_RGBA32F else np.array_equal(a, b)
