"""Known-answer and property checks of the reference semantics, on the CPU oracle (the GPU kernel is
held to the oracle by tests/test_gpu_parity.py). Each cites the reference line it exercises."""
import numpy as np

from oracle import oracle as O


def planes(h=1, w=8, **vals):
    p = np.zeros((O.NUM_PLANES, h, w), np.float32)
    p[5] = -1.0  # N = (0, 0, -1): facing the eye at z = -5
    p[6:9] = 0.5
    p[10] = 0.5
    p[11] = 1.0
    for k, v in vals.items():
        p[O.PLANE_NAMES.index(k)] = v
    return p


def light(strength=(1, 1, 1), pos=(0, 0, -3), direction=(0, 0, 1), spot=64.0):
    return [*strength, spot, *direction, 0.0, *pos, 0.0]


def shade(p, lights, **kw):
    kw.setdefault("n_point", len(lights))
    return O.shade(list(p), O.OraclePass(**kw), np.array(lights, np.float32).reshape(-1, 12))


def test_ambient_only_formula():
    """No lights: c = 0.03*albedo; c/(c+1); pow(c, 1/2.2) (Default.hlsl:150-155)."""
    p = planes()
    p[6] = np.linspace(0, 1, 8, dtype=np.float32)
    out = O.shade(list(p), O.OraclePass(), None)
    c = np.float32(0.03) * p[6, 0]
    c = c / (c + np.float32(1))
    exp = np.power(c.astype(np.float32), np.float32(1.0) / np.float32(2.2), dtype=np.float32)
    assert np.allclose(out[0, :, 0], exp, rtol=2e-7, atol=0)
    assert (out[..., 3] == 1.0).all()


def test_roughness_clamp_at_0_05_only_in_ndf():
    """DistributionGGX clamps roughness to 0.05 (LightingUtil.hlsl:51) but GeometrySchlickGGX uses the
    raw value (:66): roughness 0 and 0.05 therefore differ only through k."""
    mirror = light(pos=(-1.0, 0.0, -5.0))  # eye at (1, 0, -5): H = N, NdotL = NdotV < 1 so k matters
    a = shade(planes(rough=0.0), [mirror], eye=(1.0, 0.0, -5.0))
    b = shade(planes(rough=0.05), [mirror], eye=(1.0, 0.0, -5.0))
    c = shade(planes(rough=0.02), [mirror], eye=(1.0, 0.0, -5.0))
    assert not np.array_equal(a, b)
    assert np.isfinite(a).all() and np.isfinite(c).all()


def test_range_cut_exactly_at_100():
    """`if (d > 100) return 0` (LightingUtil.hlsl:131): d == 100 is lit, d just above is not."""
    p = planes(w=3, nx=1.0, nz=0.0)  # N faces +x, towards the light
    p[0, 0, :] = [0.0, -1e-5, 0.0]
    far = light(strength=(1e4, 1e4, 1e4), pos=(100.0, 0.0, 0.0))
    lit = shade(p, [far])
    base = O.shade(list(p), O.OraclePass(), None)
    assert not np.array_equal(lit[0, 0], base[0, 0])  # exactly 100 away: contributes
    assert np.array_equal(lit[0, 1], base[0, 1])  # 100.00001 away: culled, output = ambient only


def test_light_behind_surface_adds_nothing():
    """NdotL <= 0 makes the BRDF's final factor max(dot(N,L),0) = 0 (LightingUtil.hlsl:102-103)."""
    p = planes()
    behind = light(strength=(50, 50, 50), pos=(0, 0, 5))
    assert np.array_equal(shade(p, [behind]), O.shade(list(p), O.OraclePass(), None))


def test_light_order_and_type_ranges():
    """ComputeLighting sums dir, then point, then spot (LightingUtil.hlsl:176-199)."""
    p = planes(w=4)
    p[0:3] = np.random.default_rng(1).uniform(-1, 1, (3, 1, 4))
    L = [light(strength=(0.3, 0.3, 0.3), direction=(0.0, 0.0, 1.0)), light(pos=(1, 2, -3)),
         light(pos=(0, 3, -2), direction=(0, -1, 0), spot=4.0)]
    out = O.shade(list(p), O.OraclePass(n_dir=1, n_point=1, n_spot=1), np.array(L, np.float32))
    # spot light with SpotPower 0: pow(x, 0) = 1 -> identical to a point light
    L0 = [light(pos=(0, 3, -2), direction=(0, -1, 0), spot=0.0)]
    as_spot = O.shade(list(p), O.OraclePass(n_spot=1), np.array(L0, np.float32))
    as_point = O.shade(list(p), O.OraclePass(n_point=1), np.array(L0, np.float32))
    assert np.array_equal(as_spot, as_point)
    assert np.isfinite(out).all()


def test_ao_is_ignored_unless_requested():
    """The reference never reads its AO slot (Default.hlsl:150; Material.h:54)."""
    p = planes()
    p[11] = 0.0
    a = O.shade(list(p), O.OraclePass(), None)
    p[11] = 1.0
    b = O.shade(list(p), O.OraclePass(apply_ao=True), None)
    assert np.array_equal(a, b)


def test_degenerate_vectors_are_absorbed_by_maxnum():
    """Under D3D10+ max/saturate (IEEE maxNum: a NaN operand yields the other one) a NaN from
    normalize(0) is clamped before it can reach the output: a pixel at the eye (V = 0/0,
    Default.hlsl:53) and a light exactly on the pixel (L = 0/0, LightingUtil.hlsl:134) both shade to
    the ambient term alone. A NaN material input is not clamped and reaches RGB."""
    base = O.shade(list(planes()), O.OraclePass(), None)
    p = planes()
    p[2] = -5.0
    at_eye = shade(p, [light()])
    assert np.isfinite(at_eye).all()
    assert np.array_equal(shade(planes(), [light(pos=(0.0, 0.0, 0.0))]), base)
    nan_rough = shade(planes(rough=float("nan")), [light()])
    assert np.isnan(nan_rough[..., :3]).all() and (nan_rough[..., 3] == 1.0).all()
