"""Shared fixtures. `-m gpu` tests need an MI355X; everything else runs on CPU.

The oracle (oracle/liboracle.so) and the product library (physically_based_renderer_amd/_lib/
libpbrshade.so) are built on first use if the in-tree .so files are missing.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")


def _ensure_built():
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "liboracle.so"], check=True)
    if not os.path.exists(os.path.join(ROOT, "physically_based_renderer_amd", "_lib", "libpbrshade.so")):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "physically_based_renderer_amd", "csrc")],
                       check=True)


_ensure_built()


def golden_names():
    """Fixtures of the PS path (oracle_shade / pbr_shade_gbuffer), ALPHA_TEST fixtures excluded."""
    return sorted(f[:-4] for f in os.listdir(GOLDEN_DIR)
                  if f.endswith(".npz") and not f.startswith(("frame_", "alpha_test_")))


def alpha_golden_names():
    """Fixtures of the ALPHA_TEST permutation (Default.hlsl:111-113): planes + opacity plane."""
    return sorted(f[:-4] for f in os.listdir(GOLDEN_DIR) if f.endswith(".npz") and f.startswith("alpha_test_"))


def load_alpha_golden(name, env_png=None):
    """dict(planes (15,H,W), opacity (H,W), lights, meta, expected, coverage or None, sky (uint16) or None, env)."""
    z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"))  # numeric arrays only: allow_pickle stays False
    meta = json.loads(str(z["meta"]))
    return dict(planes=z["planes"], opacity=z["opacity"], lights=z["lights"], meta=meta, expected=z["expected"],
                coverage=z["coverage"] if "coverage" in z.files else None,
                sky=z["sky_u16"] if "sky_u16" in z.files else None, env=env_png if meta["env"] else None)


def frame_golden_names():
    """Fixtures of the frame path (sky pass, RGBA8 output, HDR env: pbr_shade_frame)."""
    return sorted(f[:-4] for f in os.listdir(GOLDEN_DIR) if f.endswith(".npz") and f.startswith("frame_"))


def load_frame_golden(name, env_png=None):
    """dict(planes, lights, meta, expected, coverage, sky (uint16), env (uint16 / float32 / None))."""
    z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"))  # numeric arrays only: allow_pickle stays False
    meta = json.loads(str(z["meta"]))
    if "env_f32" in z.files:
        env = z["env_f32"]
    elif meta["env"]:
        env = env_png
    else:
        env = None
    return dict(planes=z["planes"], lights=z["lights"], meta=meta, expected=z["expected"], coverage=z["coverage"],
                sky=z["sky_u16"], env=env)


def load_golden(name):
    """(planes (15,H,W) f32, lights (n,12) f32, meta dict, expected (H,W,4) f32)."""
    z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"))  # numeric arrays only: allow_pickle stays False
    meta = json.loads(str(z["meta"]))
    return z["planes"], z["lights"], meta, z["expected"]


def oracle_pass_from_meta(meta):
    from oracle import oracle as O

    return O.OraclePass(eye=tuple(meta["eye"]), ambient=tuple(meta["ambient"]),
                        fresnel_r0=tuple(meta["fresnel_r0"]), opacity=meta["opacity"], n_dir=meta["n_dir"],
                        n_point=meta["n_point"], n_spot=meta["n_spot"], ambient_mode=meta["ambient_mode"],
                        use_f0_plane=meta["use_f0_plane"], apply_ao=meta["apply_ao"],
                        alpha_test=meta.get("alpha_test", False))


def oracle_pass_from_constants(pc):
    """oracle.OraclePass for a renderer.PassConstants."""
    from oracle import oracle as O

    return O.OraclePass(eye=tuple(pc.eye_pos_w), ambient=tuple(pc.ambient_light), fresnel_r0=tuple(pc.fresnel_r0),
                        opacity=pc.opacity, n_dir=pc.num_dir_lights, n_point=pc.num_point_lights,
                        n_spot=pc.num_spot_lights, ambient_mode=pc.ambient_mode,
                        use_f0_plane=bool(pc.flags & 1), apply_ao=bool(pc.flags & 2),
                        alpha_test=bool(pc.flags & 32))


@pytest.fixture(scope="session")
def env_map():
    from physically_based_renderer_amd import envmap

    return envmap.load_chelsea_stairs_env()


def gpu_available():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not gpu_available():
        pytest.fail("GPU test run without a visible HIP device")
    import torch

    return torch.device("cuda", 0)


@pytest.fixture(scope="session")
def shading_ctx(gpu):
    from physically_based_renderer_amd import ShadingContext

    ctx = ShadingContext(0)
    yield ctx
    ctx.close()
