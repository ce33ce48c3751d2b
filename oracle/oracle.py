"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY (ctypes front for the parity checker).

Loads ``oracle/liboracle.so`` (plain-C restatement, pbr_oracle.c) or ``oracle/_ref/libpbr_ref.so``
(the reference's own pixel-shader text -- Default.hlsl's PS with Core.hlsl and LightingUtil.hlsl, and
Skybox.hlsl's PS -- compiled as C++: strip_hlsl.py + ref_harness.cpp). Only tests/,
``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg may import this module; the product
package never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# PBR_ORACLE_LIB: another build of the same C restatement (the sanitizer build of `make asan`, tests only).
ORACLE_SO = os.environ.get("PBR_ORACLE_LIB") or os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libpbr_ref.so")
REFERENCE_SHADER = "/root/reference/Source/Shaders/LightingUtil.hlsl"

NUM_PLANES = 15  # the product's G-buffer planes
C_PLANES = 16    # pbr_oracle.h ORACLE_NUM_PLANES: + the ALPHA_TEST opacity plane (ORACLE_OPACITY; callers may omit it)
PLANE_NAMES = ("px", "py", "pz", "nx", "ny", "nz", "ar", "ag", "ab",
               "metal", "rough", "ao", "f0r", "f0g", "f0b", "opacity")
# What the output buffers hold before a pass: pixels the ALPHA_TEST permutation's clip discards keep it.
UNTOUCHED_F32 = -1.0
UNTOUCHED_U8 = 7
AMBIENT_CONSTANT = 0
AMBIENT_IBL_DIFFUSE = 1


class _Pass(ctypes.Structure):
    _fields_ = [
        ("eye", ctypes.c_float * 3),
        ("ambient", ctypes.c_float * 3),
        ("fresnel_r0", ctypes.c_float * 3),
        ("opacity", ctypes.c_float),
        ("n_dir", ctypes.c_int32),
        ("n_point", ctypes.c_int32),
        ("n_spot", ctypes.c_int32),
        ("ambient_mode", ctypes.c_int32),
        ("use_f0_plane", ctypes.c_int32),
        ("apply_ao", ctypes.c_int32),
        ("alpha_test", ctypes.c_int32),
    ]


@dataclass
class OraclePass:
    """Per-frame constants, mirroring cbPass/cbMaterial (Core.hlsl:35-81)."""
    eye: tuple = (0.0, 0.0, -5.0)
    ambient: tuple = (0.03, 0.03, 0.03)
    fresnel_r0: tuple = (0.04, 0.04, 0.04)
    opacity: float = 1.0
    n_dir: int = 0
    n_point: int = 0
    n_spot: int = 0
    ambient_mode: int = AMBIENT_CONSTANT
    use_f0_plane: bool = False
    apply_ao: bool = False
    alpha_test: bool = False  # ALPHA_TEST permutation (Default.hlsl:111-113): needs the opacity plane

    def to_c(self) -> _Pass:
        p = _Pass()
        p.eye[:] = [float(v) for v in self.eye]
        p.ambient[:] = [float(v) for v in self.ambient]
        p.fresnel_r0[:] = [float(v) for v in self.fresnel_r0]
        p.opacity = float(self.opacity)
        p.n_dir, p.n_point, p.n_spot = int(self.n_dir), int(self.n_point), int(self.n_spot)
        p.ambient_mode = int(self.ambient_mode)
        p.use_f0_plane = int(bool(self.use_f0_plane))
        p.apply_ao = int(bool(self.apply_ao))
        p.alpha_test = int(bool(self.alpha_test))
        return p


_libs: dict = {}


def build(ref: bool = False) -> None:
    """Compile liboracle.so (and, when /root/reference exists and ref=True, _ref/libpbr_ref.so)."""
    targets = ["liboracle.so"]
    if ref and os.path.exists(REFERENCE_SHADER):
        targets.append("ref")
    subprocess.run(["make", "-s", "-C", HERE] + targets, check=True)


def _load(path: str, sym: str):
    if path not in _libs:
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C {HERE}`")
        lib = ctypes.CDLL(path)
        fn = getattr(lib, sym)
        fn.restype = ctypes.c_int
        fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p),
                       ctypes.POINTER(_Pass), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                       ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]
        _libs[path] = fn
    return _libs[path]


def ref_available() -> bool:
    return os.path.exists(REF_SO)


def _shade(fn, planes, opass: OraclePass, lights, env, n_threads: int) -> np.ndarray:
    """planes: sequence of NUM_PLANES arrays (or None), each (H, W) float32 C-contiguous."""
    planes = list(planes) + [None] * (C_PLANES - len(planes))  # 15: no opacity plane
    assert len(planes) == C_PLANES
    ref_plane = next(p for p in planes if p is not None)
    h, w = ref_plane.shape
    keep = []
    ptrs = (ctypes.c_void_p * C_PLANES)()
    for i, p in enumerate(planes):
        if p is None:
            ptrs[i] = None
            continue
        a = np.ascontiguousarray(p, dtype=np.float32)
        assert a.shape == (h, w)
        keep.append(a)
        ptrs[i] = a.ctypes.data
    n_lights = opass.n_dir + opass.n_point + opass.n_spot
    lights_arr = np.ascontiguousarray(lights, dtype=np.float32).reshape(-1, 12) if n_lights else np.zeros((1, 12), np.float32)
    assert lights_arr.shape[0] >= n_lights
    env_ptr, ew, eh = None, 0, 0
    if env is not None:
        env_arr = np.ascontiguousarray(env, dtype=np.uint16)
        assert env_arr.ndim == 3 and env_arr.shape[2] == 4
        eh, ew = env_arr.shape[:2]
        keep.append(env_arr)
        env_ptr = env_arr.ctypes.data
    out = np.full((h, w, 4), UNTOUCHED_F32, np.float32)
    cp = opass.to_c()
    rc = fn(w, h, w, ptrs, ctypes.byref(cp), lights_arr.ctypes.data, env_ptr, ew, eh,
            out.ctypes.data, w, int(n_threads))
    if rc != 0:
        raise ValueError(f"oracle rejected arguments (rc={rc})")
    return out


def shade(planes, opass: OraclePass, lights=None, env=None, n_threads: int = 1) -> np.ndarray:
    """The C restatement (pbr_oracle.c)."""
    return _shade(_load(ORACLE_SO, "oracle_shade"), planes, opass, lights, env, n_threads)


def shade_ref(planes, opass: OraclePass, lights=None, env=None) -> np.ndarray:
    """The reference's Default.hlsl PS compiled as C++ (oracle/_ref); this container and the travelling build."""
    return _shade(_load(REF_SO, "ref_shade"), planes, opass, lights, env, 1)


def rel_err(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Per-channel relative error |a-b| / max(|b|, 1e-30); NaN==NaN counts as 0, NaN vs number as inf."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        e = np.abs(a.astype(np.float64) - b.astype(np.float64)) / np.maximum(np.abs(b.astype(np.float64)), 1e-30)
    e = np.where(na & nb, 0.0, e)
    e = np.where(na ^ nb, np.inf, e)
    same_inf = np.isinf(a) & np.isinf(b) & (a == b)
    return np.where(same_inf, 0.0, e)


class _Frame(ctypes.Structure):
    _fields_ = [
        ("env_rgba", ctypes.c_void_p),
        ("env_w", ctypes.c_int32),
        ("env_h", ctypes.c_int32),
        ("sky_rgba", ctypes.c_void_p),
        ("sky_w", ctypes.c_int32),
        ("sky_h", ctypes.c_int32),
        ("coverage", ctypes.c_void_p),
        ("coverage_stride", ctypes.c_int64),
        ("format", ctypes.c_int32),
        ("pad0", ctypes.c_int32),
    ]


OUTPUT_RGBA32F = 0
OUTPUT_RGBA8 = 1


def decode_unorm16(texels: np.ndarray) -> np.ndarray:
    """R16G16B16A16_UNORM -> RGBA fp32 exactly as the C oracle does ((float)u / 65535.0f)."""
    lib = ctypes.CDLL(ORACLE_SO)
    src = np.ascontiguousarray(texels, dtype=np.uint16)
    dst = np.empty(src.shape, np.float32)
    lib.oracle_decode_unorm16.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    lib.oracle_decode_unorm16(src.ctypes.data, src.size, dst.ctypes.data)
    return dst


def _texture(t):
    """An RGBA texture for the frame entry: uint16 UNORM (decoded here) or float32, (h, w, 4)."""
    if t is None:
        return None
    a = np.asarray(t)
    if a.dtype == np.uint16:
        a = decode_unorm16(a)
    a = np.ascontiguousarray(a, dtype=np.float32)
    assert a.ndim == 3 and a.shape[2] == 4
    return a


def _shade_frame(fn, planes, opass: OraclePass, lights, env, sky, coverage, fmt, n_threads):
    planes = list(planes) + [None] * (C_PLANES - len(planes))  # 15: no opacity plane
    assert len(planes) == C_PLANES
    ref_plane = next(p for p in planes if p is not None)
    h, w = ref_plane.shape
    keep = []
    ptrs = (ctypes.c_void_p * C_PLANES)()
    for i, p in enumerate(planes):
        if p is None:
            ptrs[i] = None
            continue
        a = np.ascontiguousarray(p, dtype=np.float32)
        assert a.shape == (h, w)
        keep.append(a)
        ptrs[i] = a.ctypes.data
    n_lights = opass.n_dir + opass.n_point + opass.n_spot
    lights_arr = np.ascontiguousarray(lights, dtype=np.float32).reshape(-1, 12) if n_lights else np.zeros((1, 12), np.float32)
    fr = _Frame()
    env_a, sky_a = _texture(env), _texture(sky)
    keep += [env_a, sky_a]
    if env_a is not None:
        fr.env_rgba, fr.env_h, fr.env_w = env_a.ctypes.data, env_a.shape[0], env_a.shape[1]
    if sky_a is not None:
        fr.sky_rgba, fr.sky_h, fr.sky_w = sky_a.ctypes.data, sky_a.shape[0], sky_a.shape[1]
    if coverage is not None:
        cov = np.ascontiguousarray(coverage, dtype=np.uint8)
        assert cov.shape == (h, w)
        keep.append(cov)
        fr.coverage, fr.coverage_stride = cov.ctypes.data, w
    fr.format = int(fmt)
    out = (np.full((h, w, 4), UNTOUCHED_U8, np.uint8) if fmt == OUTPUT_RGBA8
           else np.full((h, w, 4), UNTOUCHED_F32, np.float32))
    cp = opass.to_c()
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p),
                   ctypes.POINTER(_Pass), ctypes.c_void_p, ctypes.POINTER(_Frame), ctypes.c_void_p, ctypes.c_int64,
                   ctypes.c_int]
    rc = fn(w, h, w, ptrs, ctypes.byref(cp), lights_arr.ctypes.data, ctypes.byref(fr), out.ctypes.data, w,
            int(n_threads))
    if rc != 0:
        raise ValueError(f"oracle rejected arguments (rc={rc})")
    return out


def shade_frame(planes, opass: OraclePass, lights=None, env=None, sky=None, coverage=None, fmt=OUTPUT_RGBA32F,
                n_threads: int = 1) -> np.ndarray:
    """PS + the sky pass on background pixels (coverage == 0), RGBA fp32 or RGBA8 (pbr_oracle.c)."""
    return _shade_frame(ctypes.CDLL(ORACLE_SO).oracle_shade_frame, planes, opass, lights, env, sky, coverage, fmt,
                        n_threads)


def shade_frame_ref(planes, opass: OraclePass, lights=None, env=None, sky=None, coverage=None,
                    fmt=OUTPUT_RGBA32F) -> np.ndarray:
    """The same through the reference's own LightingUtil.hlsl (oracle/_ref); this container only."""
    return _shade_frame(ctypes.CDLL(REF_SO).ref_shade_frame, planes, opass, lights, env, sky, coverage, fmt, 1)


def unorm8(c: np.ndarray) -> np.ndarray:
    """D3D FLOAT -> UNORM8 of the C oracle, element-wise (oracle_unorm8)."""
    lib = ctypes.CDLL(ORACLE_SO)
    lib.oracle_unorm8.restype = ctypes.c_uint8
    lib.oracle_unorm8.argtypes = [ctypes.c_float]
    flat = np.asarray(c, np.float32).ravel()
    return np.array([lib.oracle_unorm8(float(v)) for v in flat], np.uint8).reshape(np.shape(c))


def bit_equal(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Elementwise bit equality, treating any NaN as equal to any NaN."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
