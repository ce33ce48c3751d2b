"""The oracle (oracle/pbr_oracle.c) against the golden vectors made by the reference's own shader text
compiled as C++ (oracle/_ref: Default.hlsl's PS with Core.hlsl and LightingUtil.hlsl, Skybox.hlsl's PS;
oracle/strip_hlsl.py, tests/golden/gen_golden.py).

Bar: bit equality (NaN == NaN), since both run the same fp32 operations in the same order on the
same libm. When /root/reference is present the reference build is also re-run here on fresh random
inputs (this container only; the GPU box has no reference).
"""
import numpy as np
import pytest

from conftest import frame_golden_names, golden_names, load_frame_golden, load_golden, oracle_pass_from_meta
from oracle import oracle as O


@pytest.mark.parametrize("name", golden_names())
def test_oracle_matches_golden(name, env_map):
    planes, lights, meta, expected = load_golden(name)
    ps = oracle_pass_from_meta(meta)
    env = env_map if meta["env"] else None
    got = O.shade(list(planes), ps, lights, env, n_threads=4)
    eq = O.bit_equal(got, expected)
    assert eq.all(), f"{name}: {int((~eq).sum())} channels differ, max rel {O.rel_err(got, expected).max():.3g}"


def test_golden_set_covers_paths():
    metas = [load_golden(n)[2] for n in golden_names()]
    assert any(m["n_dir"] == 4 and m["n_point"] == 0 for m in metas)  # reference scene
    assert any(m["ambient_mode"] == O.AMBIENT_IBL_DIFFUSE for m in metas)
    assert any(m["use_f0_plane"] for m in metas)
    assert any(m["apply_ao"] for m in metas)
    assert any(m["n_spot"] > 0 for m in metas)
    assert any(m["n_point"] > 16 for m in metas)  # beyond the reference's MAX_LIGHTS
    assert any(m["n_dir"] + m["n_point"] + m["n_spot"] == 0 for m in metas)


def test_golden_edges_contain_nan_cases():
    _, _, _, expected = load_golden("edges_constant")
    assert np.isnan(expected).any()  # degenerate inputs keep the reference's NaN behaviour


@pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref needs /root/reference (build container only)")
@pytest.mark.parametrize("counts,mode,f0,ao", [((4, 0, 0), 0, False, False), ((0, 1, 0), 0, False, False),
                                               ((0, 8, 0), 1, False, False), ((4, 8, 4), 0, True, False),
                                               ((2, 40, 3), 1, True, True), ((0, 300, 0), 0, False, False)])
def test_oracle_matches_reference_build_random(counts, mode, f0, ao, env_map):
    rng = np.random.default_rng(sum(counts) * 7 + mode)
    h, w = 32, 64
    p = np.zeros((O.NUM_PLANES, h, w), np.float32)
    p[0:3] = rng.uniform(-30, 30, (3, h, w))
    n = rng.normal(size=(3, h, w))
    p[3:6] = n / np.linalg.norm(n, axis=0)
    p[6:15] = rng.uniform(-0.1, 1.2, (9, h, w))
    lights = np.zeros((sum(counts), 12), np.float32)
    lights[:, 0:3] = rng.uniform(0, 80, (sum(counts), 3))
    lights[:, 3] = rng.uniform(0, 100, sum(counts))
    d = rng.normal(size=(sum(counts), 3))
    lights[:, 4:7] = d / np.linalg.norm(d, axis=1, keepdims=True)
    lights[:, 8:11] = rng.uniform(-60, 60, (sum(counts), 3))
    ps = O.OraclePass(n_dir=counts[0], n_point=counts[1], n_spot=counts[2], ambient_mode=mode, use_f0_plane=f0,
                      apply_ao=ao)
    env = env_map if mode else None
    a = O.shade(list(p), ps, lights, env, n_threads=2)
    b = O.shade_ref(list(p), ps, lights, env)
    assert O.bit_equal(a, b).all()


@pytest.mark.parametrize("name", frame_golden_names())
def test_oracle_matches_frame_golden(name, env_map):
    """pbr_shade_frame's oracle (sky pass, RGBA8, HDR env) against the reference build's output."""
    g = load_frame_golden(name, env_map)
    ps = oracle_pass_from_meta(g["meta"])
    got = O.shade_frame(list(g["planes"]), ps, g["lights"], g["env"], g["sky"], g["coverage"], g["meta"]["format"],
                        n_threads=3)
    if g["meta"]["format"] == O.OUTPUT_RGBA8:
        assert got.dtype == np.uint8 and np.array_equal(got, g["expected"])
    else:
        assert O.bit_equal(got, g["expected"]).all()
    bg = g["coverage"] == 0
    assert bg.any() and (~bg).any()
    if g["meta"]["format"] == O.OUTPUT_RGBA32F:
        assert (got[bg][:, 3] == 1.0).all()  # Skybox.hlsl:49 alpha


def test_frame_without_coverage_equals_shade(env_map):
    """oracle_shade_frame with no coverage plane and RGBA32F output is oracle_shade."""
    planes, lights, meta, expected = load_golden("mixed_ibl_ao")
    ps = oracle_pass_from_meta(meta)
    got = O.shade_frame(list(planes), ps, lights, env_map, None, None, O.OUTPUT_RGBA32F, n_threads=2)
    assert O.bit_equal(got, expected).all()


def test_unorm8_known_answers():
    """D3D FLOAT -> UNORM8: NaN -> 0, clamp, c*255 + 0.5 (fp32), truncate."""
    # one ulp below 0.5/255: c*255 = 0.49999997, + 0.5 rounds to 1.0 in fp32 -> 1 (not 0)
    c = np.array([np.nan, -np.inf, -1.0, -0.0, 0.0, 0.5 / 255, np.nextafter(np.float32(0.5 / 255), np.float32(0)),
                  1.5 / 255, 0.5, 1.0, 2.0, np.inf, 254.5 / 255, 0.49996], np.float32)
    want = [0, 0, 0, 0, 0, 1, 1, 2, 128, 255, 255, 255, 255, 127]
    got = O.unorm8(c)
    assert got.tolist() == want, got.tolist()


@pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref needs /root/reference (build container only)")
@pytest.mark.parametrize("fmt", [O.OUTPUT_RGBA32F, O.OUTPUT_RGBA8])
def test_frame_oracle_matches_reference_build_random(fmt, env_map):
    rng = np.random.default_rng(99 + fmt)
    h, w = 24, 48
    p = np.zeros((O.NUM_PLANES, h, w), np.float32)
    p[0:3] = rng.uniform(-30, 30, (3, h, w))
    n = rng.normal(size=(3, h, w))
    p[3:6] = n / np.linalg.norm(n, axis=0) * rng.uniform(0.5, 3.0, (1, h, w))
    p[6:15] = rng.uniform(-0.1, 1.2, (9, h, w))
    cov = (rng.uniform(size=(h, w)) > 0.5).astype(np.uint8)
    sky = rng.uniform(0, 5, (20, 40, 4)).astype(np.float32)  # an fp32 HDR sky
    lights = np.zeros((6, 12), np.float32)
    lights[:, 0:3] = rng.uniform(0, 80, (6, 3))
    lights[:, 8:11] = rng.uniform(-40, 40, (6, 3))
    ps = O.OraclePass(n_point=6, ambient_mode=1)
    a = O.shade_frame(list(p), ps, lights, env_map, sky, cov, fmt, n_threads=2)
    b = O.shade_frame_ref(list(p), ps, lights, env_map, sky, cov, fmt)
    assert (np.array_equal(a, b) if fmt == O.OUTPUT_RGBA8 else O.bit_equal(a, b).all())


# ---- the reference build itself: the compiled PS / Skybox PS text (oracle/strip_hlsl.py) ------------------

@pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref needs /root/reference (build container only)")
@pytest.mark.parametrize("name", golden_names())
def test_reference_build_reproduces_golden(name, env_map):
    """oracle/_ref -- Default.hlsl's PS (or its revived IBL block) compiled from the reference text --
    reproduces every committed golden bit for bit."""
    planes, lights, meta, expected = load_golden(name)
    ps = oracle_pass_from_meta(meta)
    got = O.shade_ref(list(planes), ps, lights, env_map if meta["env"] else None)
    assert O.bit_equal(got, expected).all()


@pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref needs /root/reference (build container only)")
@pytest.mark.parametrize("name", frame_golden_names())
def test_reference_build_reproduces_frame_golden(name, env_map):
    g = load_frame_golden(name, env_map)
    ps = oracle_pass_from_meta(g["meta"])
    got = O.shade_frame_ref(list(g["planes"]), ps, g["lights"], g["env"], g["sky"], g["coverage"], g["meta"]["format"])
    assert (np.array_equal(got, g["expected"]) if g["meta"]["format"] == O.OUTPUT_RGBA8
            else O.bit_equal(got, g["expected"]).all())


@pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref needs /root/reference (build container only)")
def test_reference_build_shipped_permutation_equals_runtime_counts():
    """Core.hlsl's own 4/0/0 permutation (compile-time counts) and the runtime-count build agree: the
    harness runs the shipped one for a 4-directional-light pass, the runtime one for 4 dir + 0-strength
    point light appended (which adds +0 to every channel, ComputeLighting order)."""
    planes, lights, meta, expected = load_golden("reference_scene_red_spheres")
    ps = oracle_pass_from_meta(meta)
    assert (ps.n_dir, ps.n_point, ps.n_spot) == (4, 0, 0)
    shipped = O.shade_ref(list(planes), ps, lights)
    extra = np.concatenate([lights, np.zeros((1, 12), np.float32)])
    extra[-1, 8:11] = 1e6  # beyond the 100-unit range: the reference returns exactly 0 (LightingUtil.hlsl:131)
    ps2 = O.OraclePass(**{**ps.__dict__, "n_point": 1})
    runtime = O.shade_ref(list(planes), ps2, extra)
    assert O.bit_equal(shipped, runtime).all() and O.bit_equal(shipped, expected).all()


def test_strip_hlsl_rules_are_syntax_only(tmp_path):
    """The transform on a miniature of the reference's syntax: every rule fires, and a mismatched count
    fails loudly (so a changed reference text cannot pass silently)."""
    import importlib.util
    import os

    spec = importlib.util.spec_from_file_location("strip_hlsl", os.path.join(O.HERE, "strip_hlsl.py"))
    sh = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sh)
    src = ("Texture2D g_Tex[2] : register(t0);\nSamplerState g_S : register(s0);\n"
           "cbuffer cbPass : register(b1)\n{\n    float3 g_Eye;\n    Light g_Lights[MAX_LIGHTS];\n};\n"
           "struct VertexOut { float4 PosH : SV_POSITION; float3 PosW : POSITION; };\n"
           "float4 PS(VertexOut pin) : SV_Target\n{\n    VertexOut v = (VertexOut)0.0f;\n"
           "    return float4(g_Tex[0].Sample(g_S, pin.PosW.xy).rgb, 1.0f);\n}\n")
    sh.EXPECT["mini"] = dict(register=3, cbuffer=1, resources=2, semantics=2, sv_target=1, swizzles=2, zero_cast=1,
                             capacity=1)
    out = sh.common(src, "mini")
    assert "register" not in out and ": SV_Target" not in out and "cbuffer" not in out
    assert "inline namespace cbPass {" in out and "PBR_HLSL_GLOBAL float3 g_Eye;" in out
    assert "PBR_HLSL_GLOBAL Light g_Lights[PBR_ORACLE_MAX_LIGHTS];" in out
    assert "PBR_HLSL_GLOBAL Texture2D g_Tex[2];" in out and "PBR_HLSL_GLOBAL SamplerState g_S;" in out
    assert ".xy()" in out and ".rgb()" in out and "VertexOut{}" in out
    # a rule that fires a different number of times than the reference text implies is an error
    sh.EXPECT["mini"]["swizzles"] = 3
    with pytest.raises(SystemExit):
        sh.common(src, "mini")
