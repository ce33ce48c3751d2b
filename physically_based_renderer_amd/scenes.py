"""The BASELINE.json configurations as G-buffer scenes (host fill through ``pbr_gbuffer_fill``).

    1  256x256,   1 point light, rustediron sphere (CPU plumbing case)
    2  1920x1080, 8 point lights, rustediron material
    3  3840x2160, 64 point lights + diffuse IBL (Chelsea_Stairs)      <- the bench workload
    4  3840x2160, 256 point lights, tiled light culling, *_1K materials, F0 plane
    5  8192x8192, 64 point lights + IBL, row bands across GPUs + RCCL gather

plus REFERENCE_SCENE: the reference's own 58-sphere scene under its 4 directional lights,
ray-cast from a camera, with background pixels for the sky pass.

All inputs are synthetic but deterministic functions of (global pixel, seed); see DESIGN.md.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, replace
from typing import Optional

import numpy as np

from . import _native as N
from . import envmap
from .renderer import GBuffer, PassConstants

ASSET_DIR = envmap.ASSET_DIR


@dataclass(frozen=True)
class SceneConfig:
    cid: int
    name: str
    kind: int
    width: int
    height: int
    n_lights: int
    ambient_mode: int
    flags: int
    seed: int
    camera: Optional[tuple] = None  # (eye xyz, target xyz, fov_y) for the reference scene; None = its default

    def with_size(self, width: int, height: int) -> "SceneConfig":
        return replace(self, width=width, height=height)

    def with_camera(self, eye, target, fov_y: float = float(np.pi / 4)) -> "SceneConfig":
        return replace(self, camera=(tuple(eye), tuple(target), float(fov_y)))


CONFIGS = {
    1: SceneConfig(1, "cfg1_256x256_sphere_rustediron_1pt", N.PBR_SCENE_SPHERE_RUSTEDIRON, 256, 256, 1,
                   N.PBR_AMBIENT_CONSTANT, 0, 0x5EED0001),
    2: SceneConfig(2, "cfg2_1920x1080_rustediron_8pt", N.PBR_SCENE_RANDOM_COVERED, 1920, 1080, 8,
                   N.PBR_AMBIENT_CONSTANT, 0, 0x5EED0002),
    3: SceneConfig(3, "cfg3_3840x2160_64pt_ibl_chelsea", N.PBR_SCENE_RANDOM_COVERED, 3840, 2160, 64,
                   N.PBR_AMBIENT_IBL_DIFFUSE, 0, 0x5EED0003),
    4: SceneConfig(4, "cfg4_3840x2160_256pt_tiled_materials", N.PBR_SCENE_PLANE_MATERIALS, 3840, 2160, 256,
                   N.PBR_AMBIENT_CONSTANT, N.PBR_FLAG_F0_PLANE | N.PBR_FLAG_TILED_CULLING, 0x5EED0004),
    5: SceneConfig(5, "cfg5_8192x8192_64pt_ibl_rowbands", N.PBR_SCENE_RANDOM_COVERED, 8192, 8192, 64,
                   N.PBR_AMBIENT_IBL_DIFFUSE, 0, 0x5EED0005),
}


# The reference scene (PBRApp.cpp:964-973, 1016-1068), F0 resolved into the plane by the fill. Its
# default camera is BuildCamera's (eye (0, 0, -5) looking down +z, PBRApp.cpp:652-659); OVERVIEW_CAMERA
# backs off to show all 58 spheres.
REFERENCE_SCENE = SceneConfig(0, "reference_58_spheres", N.PBR_SCENE_REFERENCE_SPHERES, 1280, 720, 4,
                              N.PBR_AMBIENT_CONSTANT, N.PBR_FLAG_F0_PLANE, 0x5EED0000)
OVERVIEW_CAMERA = ((0.0, -7.0, -30.0), (0.0, -7.0, 0.0), float(np.pi / 4))


class Assets:
    """Texture tiles committed under assets/ (tools/make_assets.py), kept alive for the C fill."""

    _instance: Optional["Assets"] = None

    def __init__(self):
        rust = np.load(os.path.join(ASSET_DIR, "rustediron_256.npz"))
        mats = np.load(os.path.join(ASSET_DIR, "materials_1k_64.npz"))
        self.rust_metallic = np.ascontiguousarray(rust["metallic"], np.uint8)
        self.rust_roughness = np.ascontiguousarray(rust["roughness"], np.uint8)
        self.mat_albedo = np.ascontiguousarray(mats["albedo"], np.uint8)
        self.mat_specular = np.ascontiguousarray(mats["specular"], np.uint8)
        self.mat_roughness = np.ascontiguousarray(mats["roughness"], np.uint8)
        self.mat_metallic = np.ascontiguousarray(mats["metallic"], np.uint8)
        self.mat_has_metallic = np.ascontiguousarray(mats["has_metallic"], np.uint8)
        self.mat_normal = np.ascontiguousarray(mats["normal"], np.uint8)
        self.material_names = [str(s) for s in mats["names"]]
        self.env = envmap.load_chelsea_stairs_env()
        a = N.SceneAssets()
        a.rust_metallic = self.rust_metallic.ctypes.data
        a.rust_roughness = self.rust_roughness.ctypes.data
        a.rust_size = self.rust_metallic.shape[0]
        a.mat_albedo = self.mat_albedo.ctypes.data
        a.mat_specular = self.mat_specular.ctypes.data
        a.mat_roughness = self.mat_roughness.ctypes.data
        a.mat_metallic = self.mat_metallic.ctypes.data
        a.mat_has_metallic = self.mat_has_metallic.ctypes.data
        a.mat_normal = self.mat_normal.ctypes.data
        a.num_materials = self.mat_albedo.shape[0]
        a.mat_size = self.mat_albedo.shape[1]
        self.c = a

    @classmethod
    def get(cls) -> "Assets":
        if cls._instance is None:
            cls._instance = Assets()
        return cls._instance


def _scene_desc(cfg: SceneConfig, assets: Assets) -> N.SceneDesc:
    d = N.SceneDesc()
    d.kind, d.width, d.height, d.seed = cfg.kind, cfg.width, cfg.height, cfg.seed
    d.assets = ctypes.pointer(assets.c)
    if cfg.camera is not None:
        cam = N.Camera()
        cam.eye[:] = [float(v) for v in cfg.camera[0]]
        cam.target[:] = [float(v) for v in cfg.camera[1]]
        cam.fov_y = float(cfg.camera[2])
        d._camera_keep = cam  # the pointer below must not outlive it
        d.camera = ctypes.pointer(cam)
    return d


def fill_gbuffer_host(cfg: SceneConfig, row_begin: int = 0, row_end: Optional[int] = None,
                      out: Optional[np.ndarray] = None, n_threads: int = 0):
    """Host planes (15, rows, width) for rows [row_begin, row_end); returns (planes, covered_px)."""
    assets = Assets.get()
    row_end = cfg.height if row_end is None else row_end
    rows = row_end - row_begin
    if rows < 0 or row_begin < 0 or row_end > cfg.height:
        raise N.PbrError(-1, "pbr_gbuffer_fill", f"rows [{row_begin}, {row_end}) outside [0, {cfg.height})")
    if out is None:
        out = np.empty((N.NUM_PLANES, rows, cfg.width), np.float32)
    if rows == 0:
        return out, 0
    assert out.dtype == np.float32 and out.shape[0] == N.NUM_PLANES and out.shape[1] >= rows
    assert out.strides[2] == 4 and out.strides[0] % 4 == 0
    ptrs = (ctypes.c_void_p * N.NUM_PLANES)(*[out[i].ctypes.data for i in range(N.NUM_PLANES)])
    nt = n_threads or min(16, os.cpu_count() or 1)
    d = _scene_desc(cfg, assets)
    covered = N.lib().pbr_gbuffer_fill(ctypes.byref(d), row_begin, row_end, ptrs, out.strides[1] // 4, nt)
    N.check(int(covered), "pbr_gbuffer_fill")
    return out, int(covered)


def fill_gbuffer_host_coverage(cfg: SceneConfig, row_begin: int = 0, row_end: Optional[int] = None,
                               n_threads: int = 0):
    """(planes (15, rows, width) float32, coverage (rows, width) uint8: 1 geometry / 0 background)."""
    assets = Assets.get()
    row_end = cfg.height if row_end is None else row_end
    rows = row_end - row_begin
    if rows < 0 or row_begin < 0 or row_end > cfg.height:
        raise N.PbrError(-1, "pbr_gbuffer_fill_coverage", f"rows [{row_begin}, {row_end}) outside [0, {cfg.height})")
    out = np.empty((N.NUM_PLANES, rows, cfg.width), np.float32)
    cov = np.empty((rows, cfg.width), np.uint8)
    if rows == 0:
        return out, cov
    ptrs = (ctypes.c_void_p * N.NUM_PLANES)(*[out[i].ctypes.data for i in range(N.NUM_PLANES)])
    nt = n_threads or min(16, os.cpu_count() or 1)
    d = _scene_desc(cfg, assets)
    r = N.lib().pbr_gbuffer_fill_coverage(ctypes.byref(d), row_begin, row_end, ptrs, cfg.width, cov.ctypes.data,
                                          cfg.width, nt)
    N.check(int(r), "pbr_gbuffer_fill_coverage")
    return out, cov


def scene_pass(cfg: SceneConfig) -> PassConstants:
    """Pass constants + light list of a config (pbr_scene_pass), with its ambient mode and flags."""
    assets = Assets.get()
    d = _scene_desc(cfg, assets)
    lights = (N.Light * max(cfg.n_lights, 1))()
    p = N.PassDesc()
    N.check(N.lib().pbr_scene_pass(ctypes.byref(d), cfg.n_lights, lights, ctypes.byref(p)), "pbr_scene_pass")
    arr = np.frombuffer(lights, dtype=np.float32).reshape(-1, 12)[: cfg.n_lights].copy()
    pc = PassConstants.from_c(p, arr)
    pc.ambient_mode = cfg.ambient_mode
    pc.flags = int(pc.flags) | cfg.flags
    return pc


def build_gbuffer(cfg: SceneConfig, device, row_begin: int = 0, row_end: Optional[int] = None,
                  n_threads: int = 0) -> GBuffer:
    """Fill rows on the host (pinned staging) and upload them; returns the device G-buffer."""
    import torch

    row_end = cfg.height if row_end is None else row_end
    rows = row_end - row_begin
    staging = torch.empty((N.NUM_PLANES, rows, cfg.width), dtype=torch.float32, pin_memory=True)
    fill_gbuffer_host(cfg, row_begin, row_end, out=staging.numpy(), n_threads=n_threads)
    dev = staging.to(device, non_blocking=True)
    torch.cuda.current_stream(device).synchronize()
    return GBuffer(dev)


def env_map() -> np.ndarray:
    return Assets.get().env
