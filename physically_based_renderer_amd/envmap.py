"""Environment-map ingest: exact 16-bit PNG decode (zlib + PNG row filters) to R16G16B16A16_UNORM.

The reference loads ``*_Env.png`` through WIC as ``R16G16B16A16_UNORM`` with no sRGB decode
(``Source/3rdParty/DirectXTK12/WICTextureLoader.cpp:312-367``; ``Source/App/PBRApp.cpp:1205-1210``)
and samples it with ``g_SamLinearWrap`` (``PBRApp.cpp:1157-1162``) in the (commented-out) diffuse-IBL
block of ``Default.hlsl:140-149``. PIL truncates 16-bit PNGs to 8 bits, so this module decodes the
stream itself; the shading kernel consumes the u16 texels (value / 65535).
"""
from __future__ import annotations

import os
import struct
import zlib

import numpy as np

ASSET_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets")
CHELSEA_STAIRS_ENV = os.path.join(ASSET_DIR, "Chelsea_Stairs_Env.png")

_PNG_SIG = b"\x89PNG\r\n\x1a\n"
_CHANNELS = {0: 1, 2: 3, 4: 2, 6: 4}  # color type -> samples per pixel (no palette support)


def _unfilter(raw: bytes, h: int, stride: int, bpp: int) -> np.ndarray:
    out = np.zeros((h, stride), np.uint8)
    prev = np.zeros(stride, np.int32)
    pos = 0
    for y in range(h):
        ftype = raw[pos]
        line = np.frombuffer(raw, np.uint8, stride, pos + 1).astype(np.int32)
        pos += 1 + stride
        if ftype == 0:
            cur = line
        elif ftype == 2:  # Up
            cur = (line + prev) & 0xFF
        else:
            cur = line.copy()
            if ftype == 1:  # Sub
                for i in range(bpp, stride):
                    cur[i] = (cur[i] + cur[i - bpp]) & 0xFF
            elif ftype == 3:  # Average
                for i in range(stride):
                    left = cur[i - bpp] if i >= bpp else 0
                    cur[i] = (cur[i] + ((left + prev[i]) >> 1)) & 0xFF
            elif ftype == 4:  # Paeth
                for i in range(stride):
                    a = cur[i - bpp] if i >= bpp else 0
                    b = prev[i]
                    c = prev[i - bpp] if i >= bpp else 0
                    p = a + b - c
                    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                    pred = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
                    cur[i] = (cur[i] + pred) & 0xFF
            else:
                raise ValueError(f"bad PNG filter type {ftype} on row {y}")
        out[y] = cur
        prev = cur
    return out


def decode_png_rgba16(path_or_bytes) -> np.ndarray:
    """Decode a non-interlaced 8/16-bit gray/RGB/RGBA PNG to an (h, w, 4) uint16 UNORM array.

    8-bit inputs are widened by x257 (exact UNORM8 -> UNORM16); missing channels follow the DXGI
    expansion (gray -> rrr, alpha -> 65535).
    """
    data = path_or_bytes if isinstance(path_or_bytes, (bytes, bytearray)) else open(path_or_bytes, "rb").read()
    if data[:8] != _PNG_SIG:
        raise ValueError("not a PNG")
    pos, idat, ihdr = 8, [], None
    while pos < len(data):
        n, ctype = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        if ctype == b"IHDR":
            ihdr = struct.unpack(">IIBBBBB", body)
        elif ctype == b"IDAT":
            idat.append(body)
        elif ctype == b"IEND":
            break
        pos += 12 + n
    if ihdr is None:
        raise ValueError("PNG without IHDR")
    w, h, depth, color, _comp, _filt, interlace = ihdr
    if interlace != 0 or color not in _CHANNELS or depth not in (8, 16):
        raise ValueError(f"unsupported PNG (depth={depth}, color={color}, interlace={interlace})")
    ch = _CHANNELS[color]
    bps = depth // 8
    raw = zlib.decompress(b"".join(idat))
    stride = w * ch * bps
    if len(raw) != h * (stride + 1):
        raise ValueError("PNG data size mismatch")
    rows = _unfilter(raw, h, stride, ch * bps)
    if depth == 16:
        px = rows.reshape(h, w * ch, 2).astype(np.uint16)
        px = ((px[..., 0] << 8) | px[..., 1]).reshape(h, w, ch)
    else:
        px = rows.reshape(h, w, ch).astype(np.uint16) * 257
    out = np.empty((h, w, 4), np.uint16)
    if ch in (1, 2):
        out[..., 0] = out[..., 1] = out[..., 2] = px[..., 0]
    else:
        out[..., :3] = px[..., :3]
    out[..., 3] = px[..., ch - 1] if ch in (2, 4) else 65535
    return out


def load_chelsea_stairs_env() -> np.ndarray:
    """The Chelsea_Stairs 360x180 diffuse environment (BASELINE configs 3 and 5)."""
    return decode_png_rgba16(CHELSEA_STAIRS_ENV)
