"""Host-side logic: G-buffer fill determinism and partition independence, scene constants,
env-map ingest, row-band partitioning."""
import ctypes
import os

import numpy as np
import pytest

from physically_based_renderer_amd import _native as N
from physically_based_renderer_amd import dist as D
from physically_based_renderer_amd import envmap
from physically_based_renderer_amd import scenes as S


@pytest.mark.parametrize("cid", [1, 2, 3, 4, 5])
def test_fill_is_partition_independent(cid):
    cfg = S.CONFIGS[cid].with_size(200, 48) if cid != 1 else S.CONFIGS[1]
    full, cov = S.fill_gbuffer_host(cfg, n_threads=3)
    parts = [S.fill_gbuffer_host(cfg, r0, r1, n_threads=2)[0] for r0, r1 in [(0, 7), (7, 30), (30, cfg.height)]]
    assert np.array_equal(np.concatenate(parts, axis=1).view(np.uint32), full.view(np.uint32))
    again, cov2 = S.fill_gbuffer_host(cfg, n_threads=1)
    assert np.array_equal(again.view(np.uint32), full.view(np.uint32)) and cov == cov2
    assert np.isfinite(full).all()


def test_random_covered_ranges():
    cfg = S.CONFIGS[2].with_size(256, 64)
    p, cov = S.fill_gbuffer_host(cfg)
    assert cov == 256 * 64
    assert p[0].min() >= -10 and p[0].max() < 10 and p[2].min() >= 0 and p[2].max() < 10
    nl = np.sqrt((p[3:6].astype(np.float64) ** 2).sum(0))
    assert np.allclose(nl, 1.0, atol=1e-6)
    assert (p[9] >= 0).all() and (p[9] <= 1).all() and (p[11] == 1).all()
    # F0 plane = lerp(0.04, albedo, metallic) in fp32 (Default.hlsl:94-95)
    f0 = np.float32(0.04) + p[9] * (p[6] - np.float32(0.04))
    assert np.array_equal(f0.view(np.uint32), p[12].view(np.uint32))


def test_sphere_scene_coverage_and_normals():
    p, cov = S.fill_gbuffer_host(S.CONFIGS[1])
    hit = p[6] > 0  # background albedo is 0
    assert cov == int(hit.sum()) and 10000 < cov < 15000
    r = np.sqrt((p[0:3, hit].astype(np.float64) ** 2).sum(0))
    assert np.allclose(r, 1.0, atol=1e-5)
    assert (p[2, hit] < 0).all()  # the visible hemisphere faces the eye at z = -5


def test_plane_scene_uses_all_materials():
    cfg = S.CONFIGS[4].with_size(1024, 512)
    p, _ = S.fill_gbuffer_host(cfg)
    assert (p[1] == 0).all()
    assert abs(p[2].max() - 500) < 1 and abs(p[2].min() + 500) < 1
    assert len(np.unique(p[6][::64, ::64])) >= 5
    assert (p[9] > 0).any()  # metal_bare metalness map


@pytest.mark.parametrize("cid,n", [(1, 1), (2, 8), (3, 64), (4, 256), (5, 64)])
def test_scene_pass(cid, n):
    pc = S.scene_pass(S.CONFIGS[cid])
    assert pc.num_point_lights == n and pc.num_dir_lights == 0 and pc.num_spot_lights == 0
    L = pc.light_array()
    assert L.shape == (n, 12)
    assert np.allclose(pc.ambient_light, 0.03) and np.allclose(pc.fresnel_r0, 0.04) and pc.opacity == 1.0
    if cid in (2, 3, 5):
        assert (np.abs(L[:, 8:10]) <= 20).all() and (L[:, 10] <= 0).all() and (L[:, 0:3] < 100).all()
    if cid == 1:
        assert L[0, 8:11].tolist() == [20.0, 20.0, -20.0] and L[0, 0] == 100.0
    assert pc.ambient_mode == S.CONFIGS[cid].ambient_mode


def test_fill_rejects_bad_arguments():
    cfg = S.CONFIGS[2].with_size(16, 16)
    with pytest.raises(N.PbrError):
        S.fill_gbuffer_host(cfg, 10, 5)
    with pytest.raises(N.PbrError):
        S.fill_gbuffer_host(cfg, 0, 17)


def test_env_png16_decode_matches_pil_8bit_and_survey_stats():
    env = envmap.load_chelsea_stairs_env()
    assert env.shape == (180, 360, 4) and env.dtype == np.uint16
    assert (env[..., 3] == 65535).all()
    assert env[..., :3].min() == 300 and env[..., :3].max() == 65535
    try:
        from PIL import Image
    except ImportError:
        pytest.skip("PIL absent")
    p8 = np.asarray(Image.open(envmap.CHELSEA_STAIRS_ENV))
    assert np.array_equal(p8.astype(np.uint16), env[..., :3] >> 8)  # PIL truncates 16-bit to 8-bit


def _png(w, h, depth, color, rows_bytes, filt):
    import struct
    import zlib

    raw = b"".join(bytes([filt]) + r for r in rows_bytes)

    def chunk(t, b):
        return struct.pack(">I", len(b)) + t + b + struct.pack(">I", zlib.crc32(t + b) & 0xFFFFFFFF)

    return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, color, 0, 0, 0))
            + chunk(b"IDAT", zlib.compress(raw)) + chunk(b"IEND", b""))


def test_png_decoder_filters_and_formats():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 65536, (5, 7, 3), dtype=np.uint16)
    be = img.astype(">u2").tobytes()
    rows = [be[i * 42:(i + 1) * 42] for i in range(5)]
    dec = envmap.decode_png_rgba16(_png(7, 5, 16, 2, rows, 0))
    assert np.array_equal(dec[..., :3], img) and (dec[..., 3] == 65535).all()
    # Sub filter: encode row bytes as differences to the pixel 6 bytes to the left
    sub_rows = []
    for r in rows:
        a = np.frombuffer(r, np.uint8).astype(np.int32)
        d = a.copy()
        d[6:] = (a[6:] - a[:-6]) & 0xFF
        sub_rows.append(d.astype(np.uint8).tobytes())
    assert np.array_equal(envmap.decode_png_rgba16(_png(7, 5, 16, 2, sub_rows, 1))[..., :3], img)
    gray8 = rng.integers(0, 256, (3, 4), dtype=np.uint8)
    g = envmap.decode_png_rgba16(_png(4, 3, 8, 0, [gray8[i].tobytes() for i in range(3)], 0))
    assert np.array_equal(g[..., 0], gray8.astype(np.uint16) * 257) and np.array_equal(g[..., 0], g[..., 2])


@pytest.mark.parametrize("height,world", [(8192, 8), (2160, 1), (2160, 2), (2160, 7), (100, 3), (8, 4), (0, 2)])
def test_band_partition_covers_rows_once(height, world):
    bands = D.all_bands(height, world)
    assert bands[0].row_begin == 0 and bands[-1].row_end == height
    for a, b in zip(bands, bands[1:]):
        assert a.row_end == b.row_begin
    for b in bands:
        assert 0 <= b.rows <= b.rows_max
        if b.row_end < height:
            assert b.row_begin % 8 == 0 and b.row_end % 8 == 0
    if height == 8192 and world == 8:
        assert all(b.rows == 1024 for b in bands)


def test_libm_port_matches_host_glibc(tmp_path):
    """libm_f32.h (the kernel's atan2f/asinf for WorldToSkyUV, LightingUtil.hlsl:216-225, and powf for
    Fresnel, spot cone and gamma) restated on the host must equal glibc bit for bit (this also pins
    the host: the oracle's powf is glibc's x86-64 FMA variant). tools/libm_port_check.c without
    --quick is the exhaustive version of this check, tests/test_gpu_probes.py the device one."""
    import os
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "lpc")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fno-builtin", "-I",
                    os.path.join(root, "physically_based_renderer_amd", "csrc"),
                    os.path.join(root, "tools", "libm_port_check.c"), "-o", exe, "-lm", "-lpthread"], check=True)
    out = subprocess.run([exe, "--quick"], check=True, capture_output=True, text=True).stdout
    print(out)
    assert out.count("mismatches 0") == 7, out


def test_libm_pair_forms_match_host_glibc(tmp_path):
    """libm_f32_x2.h, the branch-free pair forms of atan2f / asinf the shading kernels' diffuse IBL runs, compiled
    for the host: glibc's bits wherever they do not flag an element for the scalar function, and flagged exactly
    where that is needed. tools/libm_x2_check.cpp without --quick is the exhaustive version (every float of
    asinf's domain, every finite atan2f(y, 1), 2e9 random pairs: 0 mismatches), tests/test_gpu_probes.py the
    device one."""
    import os
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "lx2")
    subprocess.run(["/opt/rocm/llvm/bin/clang++", "-std=c++17", "-O2", "-ffp-contract=off", "-fno-builtin", "-I",
                    os.path.join(root, "physically_based_renderer_amd", "csrc"),
                    os.path.join(root, "tools", "libm_x2_check.cpp"), "-o", exe, "-lm", "-lpthread"], check=True)
    r = subprocess.run([exe, "--quick"], capture_output=True, text=True)
    print(r.stdout)
    assert r.returncode == 0 and r.stdout.count(" 0 mismatches  0 special-flag errors") == 5, r.stdout


def _rgbe_expected(rgbe):
    e = rgbe[..., 3].astype(np.int64)
    return np.where(e[..., None] > 0, rgbe[..., :3].astype(np.float64) * np.ldexp(1.0, e[..., None] - 136),
                    0.0).astype(np.float32)


@pytest.mark.parametrize("w", [8, 37, 300])
def test_hdr_rle_decode_known_answer(w):
    """RGBE decode (c = mantissa * 2^(e-136), e = 0 -> 0) through new-style RLE scanlines with runs,
    literals and run/literal boundaries."""
    rng = np.random.default_rng(w)
    rgbe = rng.integers(0, 256, (6, w, 4)).astype(np.uint8)
    rgbe[1, :] = rgbe[1, :1]  # whole-row runs
    rgbe[2, ::3, 3] = 0  # zero exponents
    rgbe[3, : w // 2] = rgbe[3, :1]
    out = envmap.decode_hdr_rgba32f(envmap.encode_hdr_rle(rgbe))
    assert out.shape == (6, w, 4) and out.dtype == np.float32
    assert np.array_equal(out[..., :3], _rgbe_expected(rgbe)) and (out[..., 3] == 1.0).all()


def test_hdr_flat_and_bad_inputs():
    rgbe = np.array([[[128, 64, 32, 129], [255, 0, 1, 0], [1, 2, 3, 200]]], np.uint8)  # w = 3 < 8: flat rows
    data = b"#?RGBE\nGAMMA=1\n\n-Y 1 +X 3\n" + rgbe.tobytes()
    out = envmap.decode_hdr_rgba32f(data)
    assert np.array_equal(out[..., :3], _rgbe_expected(rgbe))
    assert out[0, 0, 0] == 1.0  # 128 * 2^(129-136)
    for bad in (b"P6\n", b"#?RADIANCE\nFORMAT=32-bit_rle_xyze\n\n-Y 1 +X 3\n" + rgbe.tobytes(),
                b"#?RADIANCE\n\n+Y 1 +X 3\n" + rgbe.tobytes(), b"#?RADIANCE\n\n-Y 2 +X 3\n" + rgbe.tobytes()):
        with pytest.raises(ValueError):
            envmap.decode_hdr_rgba32f(bad)


REF_HDR = "/root/reference/Assets/Chelsea_Stairs/Chelsea_Stairs_Env.hdr"


@pytest.mark.skipif(not os.path.exists(REF_HDR), reason="reference assets only in the build container")
def test_hdr_decodes_reference_env_asset():
    """The reference's Chelsea_Stairs_Env.hdr (read in place, never copied): 360x180, HDR range, and
    spatially the same image as the 16-bit PNG the IBL path samples."""
    hdr = envmap.decode_hdr_rgba32f(REF_HDR)
    png = envmap.load_chelsea_stairs_env().astype(np.float64) / 65535.0
    assert hdr.shape == (180, 360, 4) and np.isfinite(hdr).all()
    assert hdr[..., :3].max() > 10.0 and hdr[..., :3].min() >= 0.0
    assert np.corrcoef(hdr[..., 1].ravel(), png[..., 1].ravel())[0, 1] > 0.5


def test_procedural_sky_is_deterministic_unorm16():
    a, b = envmap.procedural_sky_rgba16(64, 32), envmap.procedural_sky_rgba16(64, 32)
    assert a.dtype == np.uint16 and a.shape == (32, 64, 4) and np.array_equal(a, b)
    assert (a[..., 3] == 65535).all() and a[..., :3].std() > 1000


def test_png_writer_round_trips_through_decoder(tmp_path):
    from physically_based_renderer_amd import image_io

    rng = np.random.default_rng(4)
    img = rng.integers(0, 256, (7, 13, 4)).astype(np.uint8)
    path = str(tmp_path / "f.png")
    image_io.write_png_rgba8(path, img)
    back = envmap.decode_png_rgba16(path)
    assert np.array_equal(back, img.astype(np.uint16) * 257)  # exact UNORM8 -> UNORM16 widening
    with pytest.raises(ValueError):
        image_io.encode_png_rgba8(img.astype(np.float32))


@pytest.mark.parametrize("camera", [None, "overview"])
def test_reference_scene_fill(camera):
    """The 58-sphere reference scene: partition-independent fill with coverage, finite geometry,
    F0 resolved per material permutation, the reference's four directional lights."""
    cfg = S.REFERENCE_SCENE.with_size(320, 180)
    if camera:
        cfg = cfg.with_camera(*S.OVERVIEW_CAMERA)
    full, cov = S.fill_gbuffer_host_coverage(cfg, n_threads=3)
    parts = [S.fill_gbuffer_host_coverage(cfg, r0, r1, n_threads=2) for r0, r1 in [(0, 41), (41, 100), (100, 180)]]
    assert np.array_equal(np.concatenate([p for p, _ in parts], axis=1).view(np.uint32), full.view(np.uint32))
    assert np.array_equal(np.concatenate([c for _, c in parts], axis=0), cov)
    planes, covered = S.fill_gbuffer_host(cfg)
    assert np.array_equal(planes.view(np.uint32), full.view(np.uint32)) and covered == int(cov.sum())
    assert 0 < covered < cfg.width * cfg.height and np.isfinite(full).all()
    g = cov == 1
    red = g & (full[6] == 1.0) & (full[7] == 0.0) & (full[8] == 0.0)
    assert red.any()  # textureless red spheres: F0 = lerp(0.04, albedo, metallic) (Default.hlsl:94-95)
    m = full[9][red]
    np.testing.assert_array_equal(full[12][red], (np.float32(0.04) + m * (np.float32(1.0) - np.float32(0.04))))
    bg = ~g  # background normal planes carry the unit view direction
    nrm = np.sqrt((full[3:6, bg].astype(np.float64) ** 2).sum(0))
    assert np.allclose(nrm, 1.0, atol=1e-6)
    pc = S.scene_pass(cfg)
    assert (pc.num_dir_lights, pc.num_point_lights) == (4, 0) and pc.flags & N.PBR_FLAG_F0_PLANE
    L = pc.light_array()
    assert np.allclose(np.abs(L[:, 4:7]), 0.57735) and np.allclose(L[:, 0:3], 0.25)


def test_div_pi_is_exact(tmp_path):
    """pbr_device_math.h div_pi: fma(x, zh, x*zl) == x / 3.14159265359f for every significand (two
    binades cover every significand and exponent parity; other exponents scale exactly)."""
    import subprocess

    src = tmp_path / "dp.c"
    src.write_text(r'''
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
int main(void) {
    const float pi = 3.14159265359f, zh = 0x1.45f306p-2f, zl = 0x1.11be6cp-28f;
    if (zh != 1.0f / pi || zl != (float)(1.0 / (double)pi - (double)zh)) { puts("constants"); return 1; }
    unsigned long long bad = 0;
    for (uint32_t m = 0; m < (1u << 24); ++m) {
        uint32_t u = 0x3f800000u + m; float x; memcpy(&x, &u, 4);
        if (fmaf(x, zh, x * zl) != x / pi) ++bad;
    }
    printf("%llu\n", bad);
    return 0;
}''')
    exe = str(tmp_path / "dp")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", str(src), "-o", exe, "-lm"], check=True)
    assert subprocess.run([exe], capture_output=True, text=True, check=True).stdout.strip() == "0"


def test_gbuffer_accepts_row_interleaved_planes():
    """A (H, 15, W) tensor viewed as (15, H, W): plane stride W < H * row stride, yet no two planes share an
    element. GBuffer takes it (the planes are read-only, so no layout is refused for overlap) and hands the
    kernel the right plane bases and row stride."""
    import torch

    from physically_based_renderer_amd.renderer import GBuffer

    h, w = 5, 8
    inter = torch.arange(h * 15 * w, dtype=torch.float32).reshape(h, 15, w).permute(1, 0, 2)
    gb = GBuffer(inter)
    c = gb.to_c()
    assert (gb.height, gb.width, gb.row_stride) == (h, w, 15 * w)
    base = inter.data_ptr()
    assert c.pos_w[0] == base and c.normal_w[0] == base + 3 * w * 4 and c.f0[2] == base + 14 * w * 4
    assert c.row_stride == 15 * w
    with pytest.raises(ValueError):
        GBuffer(torch.zeros((15, h, w), dtype=torch.float32)[:, :, ::2])  # rows must be contiguous
