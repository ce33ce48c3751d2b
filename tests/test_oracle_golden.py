"""The oracle (oracle/pbr_oracle.c) against the golden vectors made by the reference's own
LightingUtil.hlsl compiled as C++ (oracle/_ref, tests/golden/gen_golden.py).

Bar: bit equality (NaN == NaN), since both run the same fp32 operations in the same order on the
same libm. When /root/reference is present the reference build is also re-run here on fresh random
inputs (this container only; the GPU box has no reference).
"""
import numpy as np
import pytest

from conftest import golden_names, load_golden, oracle_pass_from_meta
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
