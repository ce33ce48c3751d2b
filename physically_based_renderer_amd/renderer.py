"""Host-side mirror of the reference's shading interface, over the C ABI of libpbrshade.so.

The reference drives its pixel shader through D3D12: per-frame constants in ``PassConstants``
(``Source/App/FrameResource.h:19-44``) holding ``Light Lights[MaxLights]`` (``d3dUtil.h:144-152``),
per-material constants (``Material.h:10-29``), then ``DrawIndexedInstanced`` (``PBRApp.cpp:1133``).
Here the same roles are:

  =====================================  ==============================================
  reference                              this module
  =====================================  ==============================================
  ``Light`` (strength/spotpower/dir/pos)  :class:`Light` (same fields, same defaults)
  ``PassConstants`` + light-count defines :class:`PassConstants`
  ``UpdateMainPassCB`` / ``CopyData``     :meth:`ShadingContext.set_pass`
  sky_env SRV (t1)                        :meth:`ShadingContext.set_env_map`
  sky_box SRV (t0) + Skybox.hlsl pass     :meth:`ShadingContext.set_sky_map`, ``coverage``
  ``DrawIndexedInstanced(PS)``            :meth:`ShadingContext.shade`
  PS + sky dome into the R8G8B8A8 target  :meth:`ShadingContext.shade_frame`
  =====================================  ==============================================

PyTorch is used only for device memory and streams. Every shading call runs the gfx950 kernel;
there is no CPU path.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np
import torch

from . import _native as N


@dataclass
class Light:
    """``struct Light`` (LightingUtil.hlsl:9-17) with the C++ defaults of d3dUtil.h:144-152."""
    strength: Sequence[float] = (0.5, 0.5, 0.5)
    spot_power: float = 64.0
    direction: Sequence[float] = (0.0, -1.0, 0.0)
    position: Sequence[float] = (0.0, 0.0, 0.0)

    def to_c(self) -> N.Light:
        c = N.Light()
        c.strength[:] = [float(v) for v in self.strength]
        c.spot_power = float(self.spot_power)
        c.direction[:] = [float(v) for v in self.direction]
        c.position[:] = [float(v) for v in self.position]
        return c


@dataclass
class PassConstants:
    """Shading subset of cbPass / cbMaterial (Core.hlsl:35-81) plus the NUM_*_LIGHTS defines.

    ``lights`` are ordered directional, point, spot (ComputeLighting, LightingUtil.hlsl:176-199);
    alternatively pass ``lights_array`` as an (n, 12) float32 array in the 48-byte layout.
    """
    eye_pos_w: Sequence[float] = (0.0, 0.0, -5.0)
    ambient_light: Sequence[float] = (0.03, 0.03, 0.03)
    fresnel_r0: Sequence[float] = (0.04, 0.04, 0.04)
    opacity: float = 1.0
    num_dir_lights: int = 0
    num_point_lights: int = 0
    num_spot_lights: int = 0
    ambient_mode: int = N.PBR_AMBIENT_CONSTANT
    flags: int = 0
    lights: Sequence[Light] = field(default_factory=list)
    lights_array: Optional[np.ndarray] = None

    @property
    def num_lights(self) -> int:
        return self.num_dir_lights + self.num_point_lights + self.num_spot_lights

    def light_array(self) -> np.ndarray:
        if self.lights_array is not None:
            arr = np.ascontiguousarray(self.lights_array, dtype=np.float32).reshape(-1, 12)
        else:
            arr = np.zeros((len(self.lights), 12), np.float32)
            for i, L in enumerate(self.lights):
                arr[i, 0:3] = L.strength
                arr[i, 3] = L.spot_power
                arr[i, 4:7] = L.direction
                arr[i, 8:11] = L.position
        if arr.shape[0] < self.num_lights:
            raise ValueError(f"{self.num_lights} lights declared, {arr.shape[0]} given")
        return arr

    def to_c(self, keepalive: list) -> N.PassDesc:
        p = N.PassDesc()
        p.eye_pos_w[:] = [float(v) for v in self.eye_pos_w]
        p.ambient_light[:] = [float(v) for v in self.ambient_light]
        p.fresnel_r0[:] = [float(v) for v in self.fresnel_r0]
        p.opacity = float(self.opacity)
        p.num_dir_lights = int(self.num_dir_lights)
        p.num_point_lights = int(self.num_point_lights)
        p.num_spot_lights = int(self.num_spot_lights)
        p.ambient_mode = int(self.ambient_mode)
        p.flags = int(self.flags)
        arr = self.light_array()
        keepalive.append(arr)
        p.lights = ctypes.cast(arr.ctypes.data, ctypes.POINTER(N.Light)) if arr.size else None
        return p

    @classmethod
    def from_c(cls, p: N.PassDesc, lights: np.ndarray) -> "PassConstants":
        return cls(eye_pos_w=tuple(p.eye_pos_w), ambient_light=tuple(p.ambient_light),
                   fresnel_r0=tuple(p.fresnel_r0), opacity=p.opacity, num_dir_lights=p.num_dir_lights,
                   num_point_lights=p.num_point_lights, num_spot_lights=p.num_spot_lights,
                   ambient_mode=p.ambient_mode, flags=p.flags, lights_array=np.array(lights, np.float32))


class GBuffer:
    """Structure-of-arrays G-buffer: one (15, H, row_stride) fp32 tensor, plane order
    pos xyz, normal xyz, albedo rgb, metallic, roughness, ao, f0 rgb (pbr_gbuffer_soa), and, for the
    ALPHA_TEST permutation (PBR_FLAG_ALPHA_TEST), an (H, row_stride) opacity plane with the same row stride."""

    def __init__(self, planes: torch.Tensor, width: Optional[int] = None, opacity: Optional[torch.Tensor] = None):
        if planes.dim() != 3 or planes.shape[0] != N.NUM_PLANES or planes.dtype != torch.float32:
            raise ValueError("planes must be a (15, H, W) float32 tensor")
        if planes.stride(2) != 1:
            raise ValueError("planes rows must be contiguous")
        if opacity is not None and (opacity.dim() != 2 or opacity.dtype != torch.float32 or
                                    opacity.shape[0] != planes.shape[1] or opacity.shape[1] < planes.shape[2] or
                                    opacity.stride(1) != 1 or opacity.stride(0) != planes.stride(1) or
                                    opacity.device != planes.device):
            raise ValueError("opacity must be an (H, W) float32 plane with the planes' row stride and device")
        self.planes = planes
        self.opacity = opacity
        self.height = planes.shape[1]
        self.width = planes.shape[2] if width is None else width
        self.row_stride = planes.stride(1)

    @classmethod
    def from_host(cls, planes: np.ndarray, device, opacity: Optional[np.ndarray] = None) -> "GBuffer":
        t = torch.from_numpy(np.ascontiguousarray(planes, dtype=np.float32))
        o = None if opacity is None else torch.from_numpy(np.ascontiguousarray(opacity, dtype=np.float32)).to(device)
        return cls(t.to(device), opacity=o)

    def rows(self, r0: int, r1: int) -> "GBuffer":
        """A row band (a view: shading it writes only those rows)."""
        return GBuffer(self.planes[:, r0:r1, :], self.width, None if self.opacity is None else self.opacity[r0:r1])

    def to_c(self) -> N.GBufferSoA:
        g = N.GBufferSoA()
        base = self.planes.data_ptr()
        ps = self.planes.stride(0) * 4
        ptr = [base + i * ps for i in range(N.NUM_PLANES)]
        g.pos_w[:] = ptr[0:3]
        g.normal_w[:] = ptr[3:6]
        g.albedo[:] = ptr[6:9]
        g.metallic, g.roughness, g.ao = ptr[9], ptr[10], ptr[11]
        g.f0[:] = ptr[12:15]
        g.width, g.height, g.row_stride = int(self.width), int(self.height), int(self.row_stride)
        g.opacity = None if self.opacity is None else self.opacity.data_ptr()
        return g


def _stream_handle(stream) -> int:
    if stream is None:
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream) if hasattr(stream, "cuda_stream") else int(stream)


class ShadingContext:
    """One ``pbr_context`` on one device."""

    def __init__(self, device: int = 0):
        self.lib = N.lib()
        self.device = int(device)
        h = ctypes.c_void_p()
        N.check(self.lib.pbr_context_create(self.device, ctypes.byref(h)), "pbr_context_create")
        self._h = h
        self.pass_constants: Optional[PassConstants] = None

    @property
    def handle(self):
        return self._h

    def close(self) -> None:
        if self._h:
            self.lib.pbr_context_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_pass(self, pc: PassConstants, stream=None) -> None:
        keep: list = []
        p = pc.to_c(keep)
        N.check(self.lib.pbr_set_pass(self._h, ctypes.byref(p), ctypes.c_void_p(_stream_handle(stream))),
                "pbr_set_pass", self._h)
        self.pass_constants = pc

    def _set_texture(self, name: str, texels: np.ndarray, stream) -> None:
        if texels.dtype == np.uint16:
            fn, t = name, np.ascontiguousarray(texels)
        elif texels.dtype == np.float32:
            fn, t = name + "_f32", np.ascontiguousarray(texels)
        else:
            raise ValueError(f"{name}: texels must be uint16 (R16G16B16A16_UNORM) or float32 RGBA")
        if t.ndim != 3 or t.shape[2] != 4:
            raise ValueError(f"{name}: texels must be (h, w, 4)")
        N.check(getattr(self.lib, fn)(self._h, t.ctypes.data, t.shape[1], t.shape[0],
                                      ctypes.c_void_p(_stream_handle(stream))), fn, self._h)

    def set_env_map(self, texels: np.ndarray, stream=None) -> None:
        """IBL environment (g_SkyArray[1]): (h, w, 4) uint16 UNORM or float32 (e.g. a decoded .hdr)."""
        self._set_texture("pbr_set_env_map", texels, stream)

    def set_sky_map(self, texels: np.ndarray, stream=None) -> None:
        """Sky texture (g_SkyArray[0]) sampled for background pixels: uint16 UNORM or float32 RGBA."""
        self._set_texture("pbr_set_sky_map", texels, stream)

    def _check_device(self, *tensors) -> None:
        """Every tensor handed to the kernel must live on this context's device: a foreign pointer would be
        dereferenced by the kernel (peer access or a fault)."""
        want = torch.device("cuda", self.device)
        for t in tensors:
            if t is not None and t.device != want:
                raise ValueError(f"tensor on {t.device}, but this ShadingContext shades on {want}")

    def shade(self, gb: GBuffer, out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
        """Shade every pixel of ``gb`` into ``out`` ((H, >=W, 4) fp32 on the device), asynchronously."""
        self._check_device(gb.planes, gb.opacity, out)
        if out is None:
            out = torch.empty((gb.height, gb.width, 4), dtype=torch.float32, device=gb.planes.device)
        if out.dtype != torch.float32 or out.dim() != 3 or out.shape[2] != 4 or out.stride(2) != 1 or out.stride(1) != 4:
            raise ValueError("out must be (H, W, 4) float32 with contiguous pixels")
        if out.shape[0] < gb.height or out.shape[1] < gb.width:
            raise ValueError("out is smaller than the G-buffer")
        g = gb.to_c()
        N.check(self.lib.pbr_shade_gbuffer(self._h, ctypes.byref(g), ctypes.c_void_p(out.data_ptr()),
                                           out.stride(0) // 4, ctypes.c_void_p(_stream_handle(stream))),
                "pbr_shade_gbuffer", self._h)
        return out

    def shade_frame(self, gb: GBuffer, out: Optional[torch.Tensor] = None, coverage: Optional[torch.Tensor] = None,
                    fmt: int = N.PBR_OUTPUT_RGBA32F, stream=None) -> torch.Tensor:
        """Shade ``gb`` with the sky pass on background pixels (``coverage`` == 0; (H, >=W) uint8 on the
        device) into ``out``: (H, W, 4) float32 for RGBA32F or (H, W, 4) uint8 for RGBA8_UNORM."""
        self._check_device(gb.planes, gb.opacity, out, coverage)
        dev = gb.planes.device
        if fmt == N.PBR_OUTPUT_RGBA8_UNORM:
            dtype, px_bytes = torch.uint8, 4
        elif fmt == N.PBR_OUTPUT_RGBA32F:
            dtype, px_bytes = torch.float32, 16
        else:
            raise ValueError("unknown output format")
        if out is None:
            out = torch.empty((gb.height, gb.width, 4), dtype=dtype, device=dev)
        if out.dtype != dtype or out.dim() != 3 or out.shape[2] != 4 or out.stride(2) != 1 or out.stride(1) != 4:
            raise ValueError("out must be (H, W, 4) with contiguous pixels of the format's dtype")
        if out.shape[0] < gb.height or out.shape[1] < gb.width:
            raise ValueError("out is smaller than the G-buffer")
        f = N.FrameDesc()
        f.out = out.data_ptr()
        f.out_row_stride = out.stride(0) // 4
        f.format = int(fmt)
        if coverage is not None:
            if coverage.dtype != torch.uint8 or coverage.dim() != 2 or coverage.stride(1) != 1:
                raise ValueError("coverage must be a (H, W) uint8 tensor with contiguous rows")
            if coverage.shape[0] < gb.height or coverage.shape[1] < gb.width:
                raise ValueError("coverage is smaller than the G-buffer")
            f.coverage = coverage.data_ptr()
            f.coverage_row_stride = coverage.stride(0)
        g = gb.to_c()
        N.check(self.lib.pbr_shade_frame(self._h, ctypes.byref(g), ctypes.byref(f),
                                         ctypes.c_void_p(_stream_handle(stream))), "pbr_shade_frame", self._h)
        return out

    def pass_stats(self, stream=None) -> dict:
        """pbr_last_pass_stats of the last pass on ``stream`` as a dict (workgroups, culled, cull_tiles,
        cull_tile_lights, exact_pixels, light_terms, geometry_pixels, backface_tests)."""
        st = N.PassStats()
        N.check(self.lib.pbr_last_pass_stats(self._h, ctypes.byref(st), ctypes.c_void_p(_stream_handle(stream))),
                "pbr_last_pass_stats", self._h)
        return {name: getattr(st, name) for name, _ in N.PassStats._fields_}

    def last_kernel(self, stream=None) -> str:
        """pbr_last_pass_kernel: the kernel the last pass on ``stream`` launched, as rocprofv3 names it without
        its argument list ("" before the first pass)."""
        fn = getattr(self.lib, "pbr_last_pass_kernel", None)  # absent only from older A/B builds (PBR_LIB_PATH)
        return "" if fn is None else (fn(self._h, ctypes.c_void_p(_stream_handle(stream))) or b"").decode()

    def debug_bounds(self, reset: bool = True) -> dict:
        """pbr_debug_bounds of a bounds-checked build (PBR_DEBUG_BOUNDS, loaded through PBR_LIB_PATH): synchronises
        the device and returns {class name: last offending index} for every violated index class (empty: none),
        then clears the flags when ``reset``. Raises PbrError(PBR_ERR_UNSUPPORTED) on a product build."""
        flags = (ctypes.c_uint32 * 16)()
        N.check(self.lib.pbr_debug_bounds(self._h, flags, int(reset)), "pbr_debug_bounds", self._h)
        names = ("gbuffer", "output", "coverage", "texel", "light", "lds")
        return {n: int(flags[8 + c]) for c, n in enumerate(names) if flags[c]}

    def cull_stats(self, stream=None):
        """(sum of surviving point/spot lights over tiles, tiles) of the last pass ((0, 0) unless it culled)."""
        s, t = ctypes.c_int64(), ctypes.c_int64()
        N.check(self.lib.pbr_last_cull_stats(self._h, ctypes.byref(s), ctypes.byref(t),
                                             ctypes.c_void_p(_stream_handle(stream))), "pbr_last_cull_stats", self._h)
        return s.value, t.value
