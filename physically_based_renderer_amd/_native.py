"""ctypes binding of ``include/pbr/pbr_shade.h`` (libpbrshade.so, built in-tree for gfx950).

There is no fallback: if the HIP library is missing or fails to load, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import re

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
# PBR_LIB_PATH overrides the in-tree library (development A/B of kernel builds only).
LIB_PATH = os.environ.get("PBR_LIB_PATH") or os.path.join(PKG_DIR, "_lib", "libpbrshade.so")
HEADER_PATH = os.path.join(REPO_DIR, "include", "pbr", "pbr_shade.h")
CSRC_DIR = os.path.join(PKG_DIR, "csrc")

PBR_OK = 0
PBR_ERR_INVALID_ARGUMENT = -1
PBR_ERR_NO_DEVICE = -2
PBR_ERR_OUT_OF_MEMORY = -3
PBR_ERR_LAUNCH = -4
PBR_ERR_HIP = -5
PBR_ERR_NOT_READY = -6
PBR_ERR_UNSUPPORTED = -7
PBR_MAX_LIGHTS = 4096
PBR_AMBIENT_CONSTANT = 0
PBR_AMBIENT_IBL_DIFFUSE = 1
PBR_FLAG_F0_PLANE = 1 << 0
PBR_FLAG_APPLY_AO = 1 << 1
PBR_FLAG_TILED_CULLING = 1 << 2
PBR_FLAG_EXACT_ONLY = 1 << 3
PBR_FLAG_FAITHFUL = 1 << 4  # tolerance mode (pbr_shade.h): within 1e-5, not bit-identical
PBR_FLAG_ALPHA_TEST = 1 << 5  # ALPHA_TEST permutation (Default.hlsl:111-113): clip on the opacity plane
PBR_OUTPUT_RGBA32F = 0
PBR_OUTPUT_RGBA8_UNORM = 1
PBR_SCENE_SPHERE_RUSTEDIRON = 1
PBR_SCENE_RANDOM_COVERED = 2
PBR_SCENE_PLANE_MATERIALS = 4
PBR_SCENE_REFERENCE_SPHERES = 5

NUM_PLANES = 15
PLANE_NAMES = ("px", "py", "pz", "nx", "ny", "nz", "ar", "ag", "ab",
               "metal", "rough", "ao", "f0r", "f0g", "f0b")


class PbrError(RuntimeError):
    def __init__(self, status: int, what: str, detail: str = ""):
        self.status = status
        msg = f"{what} failed: {status_string(status)} ({status})"
        if detail:
            msg += f": {detail}"
        super().__init__(msg)


class Light(ctypes.Structure):
    """The reference cbuffer `Light` (LightingUtil.hlsl:9-17), 48 bytes."""
    _fields_ = [
        ("strength", ctypes.c_float * 3),
        ("spot_power", ctypes.c_float),
        ("direction", ctypes.c_float * 3),
        ("pad0", ctypes.c_float),
        ("position", ctypes.c_float * 3),
        ("pad1", ctypes.c_float),
    ]


class PassDesc(ctypes.Structure):
    _fields_ = [
        ("eye_pos_w", ctypes.c_float * 3),
        ("ambient_light", ctypes.c_float * 3),
        ("fresnel_r0", ctypes.c_float * 3),
        ("opacity", ctypes.c_float),
        ("num_dir_lights", ctypes.c_int32),
        ("num_point_lights", ctypes.c_int32),
        ("num_spot_lights", ctypes.c_int32),
        ("ambient_mode", ctypes.c_int32),
        ("flags", ctypes.c_uint32),
        ("lights", ctypes.POINTER(Light)),
    ]


class GBufferSoA(ctypes.Structure):
    _fields_ = [
        ("pos_w", ctypes.c_void_p * 3),
        ("normal_w", ctypes.c_void_p * 3),
        ("albedo", ctypes.c_void_p * 3),
        ("metallic", ctypes.c_void_p),
        ("roughness", ctypes.c_void_p),
        ("ao", ctypes.c_void_p),
        ("f0", ctypes.c_void_p * 3),
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("row_stride", ctypes.c_int64),
        ("opacity", ctypes.c_void_p),  # ABI 6: PBR_FLAG_ALPHA_TEST's opacity plane
    ]


class FrameDesc(ctypes.Structure):
    _fields_ = [
        ("out", ctypes.c_void_p),
        ("out_row_stride", ctypes.c_int64),
        ("format", ctypes.c_int32),
        ("pad0", ctypes.c_int32),
        ("coverage", ctypes.c_void_p),
        ("coverage_row_stride", ctypes.c_int64),
    ]


class SceneAssets(ctypes.Structure):
    _fields_ = [
        ("rust_metallic", ctypes.c_void_p),
        ("rust_roughness", ctypes.c_void_p),
        ("rust_size", ctypes.c_int32),
        ("mat_albedo", ctypes.c_void_p),
        ("mat_specular", ctypes.c_void_p),
        ("mat_roughness", ctypes.c_void_p),
        ("mat_metallic", ctypes.c_void_p),
        ("mat_has_metallic", ctypes.c_void_p),
        ("mat_normal", ctypes.c_void_p),
        ("num_materials", ctypes.c_int32),
        ("mat_size", ctypes.c_int32),
    ]


class Camera(ctypes.Structure):
    _fields_ = [
        ("eye", ctypes.c_float * 3),
        ("target", ctypes.c_float * 3),
        ("fov_y", ctypes.c_float),
        ("pad0", ctypes.c_float),
    ]


class PassStats(ctypes.Structure):
    """pbr_pass_stats: statistics of the last shading pass."""
    _fields_ = [
        ("workgroups", ctypes.c_int64),
        ("culled", ctypes.c_int64),
        ("cull_tiles", ctypes.c_int64),
        ("cull_tile_lights", ctypes.c_int64),
        ("exact_pixels", ctypes.c_int64),
        ("light_terms", ctypes.c_int64),
        ("geometry_pixels", ctypes.c_int64),
        ("backface_tests", ctypes.c_int64),
    ]


class SceneDesc(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int32),
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("assets", ctypes.POINTER(SceneAssets)),
        ("camera", ctypes.POINTER(Camera)),
    ]


# name -> (restype, argtypes); every symbol declared in the header must appear here.
SIGNATURES = {
    "pbr_context_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "pbr_context_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "pbr_set_pass": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(PassDesc), ctypes.c_void_p]),
    "pbr_set_env_map": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_void_p]),
    "pbr_shade_gbuffer": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(GBufferSoA), ctypes.c_void_p,
                                         ctypes.c_int64, ctypes.c_void_p]),
    "pbr_set_env_map_f32": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                           ctypes.c_void_p]),
    "pbr_set_sky_map": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_void_p]),
    "pbr_set_sky_map_f32": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                           ctypes.c_void_p]),
    "pbr_shade_frame": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(GBufferSoA), ctypes.POINTER(FrameDesc),
                                       ctypes.c_void_p]),
    "pbr_last_cull_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64),
                                           ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p]),
    "pbr_last_pass_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(PassStats), ctypes.c_void_p]),
    "pbr_last_pass_kernel": (ctypes.c_char_p, [ctypes.c_void_p, ctypes.c_void_p]),
    "pbr_debug_bounds": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "pbr_gbuffer_fill": (ctypes.c_int64, [ctypes.POINTER(SceneDesc), ctypes.c_int32, ctypes.c_int32,
                                          ctypes.POINTER(ctypes.c_void_p), ctypes.c_int64, ctypes.c_int32]),
    "pbr_gbuffer_fill_coverage": (ctypes.c_int64, [ctypes.POINTER(SceneDesc), ctypes.c_int32, ctypes.c_int32,
                                                   ctypes.POINTER(ctypes.c_void_p), ctypes.c_int64, ctypes.c_void_p,
                                                   ctypes.c_int64, ctypes.c_int32]),
    "pbr_scene_pass": (ctypes.c_int, [ctypes.POINTER(SceneDesc), ctypes.c_int32, ctypes.POINTER(Light),
                                      ctypes.POINTER(PassDesc)]),
    "pbr_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "pbr_last_error": (ctypes.c_char_p, [ctypes.c_void_p]),
    "pbr_abi_version": (ctypes.c_int, []),
    "pbr_build_info": (ctypes.c_char_p, []),
}

_lib = None


def header_symbols(path: str = HEADER_PATH) -> list:
    """Function names declared in the public header (for the ABI-coverage test)."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pbr_[a-z_0-9]+)\s*\(", text)))


def lib() -> ctypes.CDLL:
    """Load libpbrshade.so. Raises (never falls back) if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `make -C {CSRC_DIR}` or __graft_entry__.build()")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if "PBR_LIB_PATH" in os.environ and not hasattr(handle, name):
                continue  # development A/B against an older build: bind what it exports
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def kernel_sources_sha(csrc_dir: str = CSRC_DIR) -> str:
    """sha256 (first 16 hex digits) of the sources libpbrshade.so is built from (csrc/*.hip, *.h, *.cpp, the
    Makefile) and the public header (_sources.py): the stamp every object of a build carries (build_info) and that
    committed profiles (profiles/pmc_summary.json) are keyed by."""
    from ._sources import sources_sha

    return sources_sha(csrc_dir, HEADER_PATH)


# The product build: every unit compiled by the Makefile's default target from one checkout (no EXTRA flags, no
# debug / profiling / experiment switches). Anything else -- the bounds-checked build, an ASan build, a development
# variant (tools/build_variant.sh), `make EXTRA=...` -- carries another flavor in pbr_build_info.
PRODUCT_FLAVOR = "product"


def build_info() -> dict:
    """What the LOADED library was built from (pbr_build_info, ABI 9): per compilation unit the sources stamp, the
    build flavor, its extra compiler flags and the value of every build switch, plus a summary -- `sources_sha` (the
    units' common stamp, None if they differ), `flavor` (likewise) and `path`. Libraries older than ABI 9 report
    {"sources_sha": None, "flavor": None, "units": []}."""
    import json

    handle = lib()
    if not hasattr(handle, "pbr_build_info"):
        return {"path": LIB_PATH, "sources_sha": None, "flavor": None, "units": [], "abi": handle.pbr_abi_version()}
    info = json.loads(handle.pbr_build_info().decode())
    shas = {u["sources_sha"] for u in info["units"]}
    flavors = {u["flavor"] for u in info["units"]}
    info.update(path=os.path.abspath(LIB_PATH), sources_sha=shas.pop() if len(shas) == 1 else None,
                flavor=flavors.pop() if len(flavors) == 1 else None)
    return info


def build_problems(info: dict = None, tree_sha: str = None) -> list:
    """Why the loaded library is not provably the product build of this checkout (empty = it is): units compiled
    from different source states, a stamp other than the checkout's, or a non-product flavor (debug, profiling,
    experiment or EXTRA flags)."""
    info = build_info() if info is None else info
    tree_sha = kernel_sources_sha() if tree_sha is None else tree_sha
    bad = []
    if not info["units"]:
        return ["the library reports no build info (ABI < 9)"]
    if info["sources_sha"] is None:
        bad.append("units built from different sources: " + ", ".join(f"{u['unit']}={u['sources_sha']}"
                                                                       for u in info["units"]))
    elif info["sources_sha"] != tree_sha:
        bad.append(f"library built from sources {info['sources_sha']}, checkout is {tree_sha}")
    for u in info["units"]:
        if u["flavor"] != PRODUCT_FLAVOR:
            bad.append(f"unit {u['unit']} is a {u['flavor']!r} build")
    return bad


def status_string(status: int) -> str:
    try:
        return lib().pbr_strerror(int(status)).decode()
    except Exception:  # pragma: no cover - the message path must never mask the original error
        return "unknown"


def check(status: int, what: str, ctx=None) -> int:
    if status < 0:
        detail = ""
        if ctx:
            detail = (lib().pbr_last_error(ctx) or b"").decode()
        raise PbrError(int(status), what, detail)
    return status
