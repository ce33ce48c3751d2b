"""Writing presented frames: R8G8B8A8_UNORM (the reference's back buffer, d3dApp.h:124, presented by
PBRApp::Draw, PBRApp.cpp:274-279) as PNG, so a frame of pbr_shade_frame can be compared with the
reference's screenshots (Samples/*.png) by eye or by tooling. Plain zlib; filter type 0 per row.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np


def _chunk(kind: bytes, body: bytes) -> bytes:
    return struct.pack(">I", len(body)) + kind + body + struct.pack(">I", zlib.crc32(kind + body) & 0xFFFFFFFF)


def encode_png_rgba8(rgba: np.ndarray, level: int = 6) -> bytes:
    """(H, W, 4) uint8 RGBA -> PNG bytes (8-bit RGBA, non-interlaced)."""
    a = np.ascontiguousarray(rgba)
    if a.dtype != np.uint8 or a.ndim != 3 or a.shape[2] != 4:
        raise ValueError("expected an (H, W, 4) uint8 array")
    h, w, _ = a.shape
    raw = np.zeros((h, 1 + 4 * w), np.uint8)  # filter byte 0 (None) + the row
    raw[:, 1:] = a.reshape(h, 4 * w)
    return (b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 0))
            + _chunk(b"IDAT", zlib.compress(raw.tobytes(), level)) + _chunk(b"IEND", b""))


def write_png_rgba8(path: str, rgba) -> None:
    """Write an (H, W, 4) uint8 frame (numpy array or a torch tensor on any device) as PNG."""
    if hasattr(rgba, "detach"):
        rgba = rgba.detach().cpu().numpy()
    with open(path, "wb") as f:
        f.write(encode_png_rgba8(np.asarray(rgba)))
