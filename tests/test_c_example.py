"""examples/shade_sphere.c: the C ABI driven from plain C (no Python, no PyTorch).

CPU: the example compiles as C11 against include/pbr/pbr_shade.h and links libpbrshade.so.
GPU: it renders the RGBA8 frame (lit sphere + sky through pbr_shade_frame); the G-buffer it dumps is
shaded again by the CPU oracle, and the two frames must agree to the byte.
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from physically_based_renderer_amd import _native as N

EXAMPLE = os.path.join(ROOT, "examples", "shade_sphere.c")


def build_example(out_dir):
    exe = os.path.join(out_dir, "shade_sphere")
    lib_dir = os.path.dirname(N.LIB_PATH)
    cmd = ["gcc", "-std=c11", "-O2", "-Wall", "-Wextra", "-Werror=implicit-function-declaration",
           "-D__HIP_PLATFORM_AMD__", "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include", EXAMPLE,
           "-L", lib_dir, "-lpbrshade", "-L", "/opt/rocm/lib", "-lamdhip64", "-lm", f"-Wl,-rpath,{lib_dir}",
           "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def test_example_compiles_as_c11(tmp_path):
    build_example(str(tmp_path))


@pytest.mark.gpu
def test_example_frame_equals_oracle(tmp_path, gpu):
    from oracle import oracle as O

    exe = build_example(str(tmp_path))
    dump = str(tmp_path / "frame.bin")
    w, h = 320, 180
    r = subprocess.run([exe, "--width", str(w), "--height", str(h), "--out", str(tmp_path / "sphere.ppm"),
                        "--dump", dump], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    print(r.stdout.strip())
    raw = open(dump, "rb").read()
    dims = np.frombuffer(raw[:16], np.int32)
    assert tuple(dims[:2]) == (w, h)
    sw, sh = int(dims[2]), int(dims[3])
    n = w * h
    off = 16
    planes = np.frombuffer(raw, np.float32, 15 * n, off).reshape(15, h, w)
    off += 4 * 15 * n
    cov = np.frombuffer(raw, np.uint8, n, off).reshape(h, w)
    off += n
    sky = np.frombuffer(raw, np.uint16, 4 * sw * sh, off).reshape(sh, sw, 4)
    off += 2 * 4 * sw * sh
    frame = np.frombuffer(raw, np.uint8, 4 * n, off).reshape(h, w, 4)
    assert 0 < cov.sum() < n  # sphere and sky both present
    d = 0.57735
    lights = np.zeros((4, 12), np.float32)
    lights[:, 0:3] = 0.25
    lights[:, 3] = 64.0
    lights[:, 4:7] = [[d, d, d], [d, -d, d], [-d, d, d], [-d, -d, d]]
    opass = O.OraclePass(eye=(0.0, 0.0, -5.0), ambient=(0.03, 0.03, 0.03), fresnel_r0=(0.04, 0.04, 0.04),
                         opacity=1.0, n_dir=4, n_point=0, n_spot=0, ambient_mode=0, use_f0_plane=False,
                         apply_ao=False)
    ref = O.shade_frame(list(planes), opass, lights, None, sky, cov, O.OUTPUT_RGBA8, n_threads=8)
    assert (frame == ref).all(), f"{int((frame != ref).sum())} bytes differ"
