"""physically_based_renderer_amd -- MI355X (gfx950) G-buffer shading for trevordblack/Physically_Based_Renderer.

The hot path is the reference's pixel shader (Source/Shaders/Default.hlsl:47-161 +
LightingUtil.hlsl:35-225) as hand-written HIP kernels behind the C ABI of include/pbr/pbr_shade.h.
"""
from . import _native
from ._native import PbrError
from .renderer import GBuffer, Light, PassConstants, ShadingContext

__all__ = ["GBuffer", "Light", "PassConstants", "PbrError", "ShadingContext", "_native"]
