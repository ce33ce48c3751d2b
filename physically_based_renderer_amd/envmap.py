"""Environment-map ingest: exact 16-bit PNG decode (zlib + PNG row filters) to R16G16B16A16_UNORM,
Radiance RGBE ``.hdr`` decode to RGBA fp32, and a procedural sky texture.

The reference loads ``*_Env.png`` through WIC as ``R16G16B16A16_UNORM`` with no sRGB decode
(``Source/3rdParty/DirectXTK12/WICTextureLoader.cpp:312-367``; ``Source/App/PBRApp.cpp:1205-1210``)
and samples it with ``g_SamLinearWrap`` (``PBRApp.cpp:1157-1162``) in the (commented-out) diffuse-IBL
block of ``Default.hlsl:140-149``. PIL truncates 16-bit PNGs to 8 bits, so this module decodes the
stream itself; the shading kernel consumes the u16 texels (value / 65535).

Every sIBL set in ``Assets/`` also ships a Radiance ``*_Env.hdr`` (the ``EVfile`` of its ``.ibl``
descriptor). The reference never loads them (WIC has no RGBE codec); :func:`decode_hdr_rgba32f`
reads them for ``pbr_set_env_map_f32`` / ``pbr_set_sky_map_f32`` with the RGBE convention of
``rgbe.c`` as most loaders use it: ``c = mantissa * 2**(e - 136)``, ``e == 0`` -> 0.
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


def _rle_channel(buf: bytes, pos: int, width: int) -> tuple:
    """One channel of a new-style RLE scanline: (values uint8[width], new pos)."""
    out = np.empty(width, np.uint8)
    x = 0
    while x < width:
        if pos >= len(buf):
            raise ValueError("truncated RLE scanline")
        n = buf[pos]
        pos += 1
        if n > 128:  # a run of n - 128 copies of the next byte
            n -= 128
            if n > width - x or pos >= len(buf):
                raise ValueError("bad RLE run")
            out[x:x + n] = buf[pos]
            pos += 1
        else:  # n literal bytes
            if n == 0 or n > width - x or pos + n > len(buf):
                raise ValueError("bad RLE literal")
            out[x:x + n] = np.frombuffer(buf, np.uint8, n, pos)
            pos += n
        x += n
    return out, pos


def decode_hdr_rgba32f(data) -> np.ndarray:
    """Decode a Radiance RGBE image (``#?RADIANCE`` / ``#?RGBE``, ``FORMAT=32-bit_rle_rgbe``,
    resolution ``-Y H +X W``; new-style RLE or flat scanlines) to (H, W, 4) float32 RGBA, alpha 1.
    ``data`` is a path or the file's bytes."""
    buf = open(data, "rb").read() if isinstance(data, (str, os.PathLike)) else bytes(data)
    if not (buf.startswith(b"#?RADIANCE") or buf.startswith(b"#?RGBE")):
        raise ValueError("not a Radiance .hdr file")
    pos = 0
    fmt = None
    while True:  # header lines up to the blank line
        end = buf.index(b"\n", pos)
        line = buf[pos:end].strip()
        pos = end + 1
        if not line:
            break
        if line.startswith(b"FORMAT="):
            fmt = line[7:]
    if fmt not in (None, b"32-bit_rle_rgbe"):
        raise ValueError(f"unsupported .hdr format {fmt!r}")
    end = buf.index(b"\n", pos)
    res = buf[pos:end].split()
    pos = end + 1
    if len(res) != 4 or res[0] != b"-Y" or res[2] != b"+X":
        raise ValueError(f"unsupported .hdr orientation {b' '.join(res)!r}")
    h, w = int(res[1]), int(res[3])
    if h <= 0 or w <= 0:
        raise ValueError("bad .hdr size")
    rgbe = np.empty((h, w, 4), np.uint8)
    for y in range(h):
        rle = (8 <= w < 32768 and pos + 4 <= len(buf) and buf[pos] == 2 and buf[pos + 1] == 2
               and not (buf[pos + 2] & 0x80))
        if rle:
            if (buf[pos + 2] << 8 | buf[pos + 3]) != w:
                raise ValueError("RLE scanline width mismatch")
            pos += 4
            for c in range(4):
                rgbe[y, :, c], pos = _rle_channel(buf, pos, w)
        else:  # flat scanline
            if pos + 4 * w > len(buf):
                raise ValueError("truncated flat scanline")
            rgbe[y] = np.frombuffer(buf, np.uint8, 4 * w, pos).reshape(w, 4)
            pos += 4 * w
    e = rgbe[..., 3].astype(np.int32)
    scale = np.where(e > 0, np.ldexp(np.float64(1.0), e - 136), 0.0)
    out = np.empty((h, w, 4), np.float32)
    out[..., :3] = (rgbe[..., :3].astype(np.float64) * scale[..., None]).astype(np.float32)
    out[..., 3] = 1.0
    return out


def encode_hdr_rle(rgbe: np.ndarray) -> bytes:
    """Encode (H, W, 4) uint8 RGBE texels as a new-style RLE Radiance file (runs of >= 3 equal bytes
    become runs). Used to build decoder fixtures."""
    h, w, _ = rgbe.shape
    out = bytearray(b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n" + f"-Y {h} +X {w}\n".encode())
    for y in range(h):
        out += bytes([2, 2, w >> 8, w & 0xFF])
        for c in range(4):
            row = rgbe[y, :, c]
            x = 0
            while x < w:
                r = 1
                while x + r < w and r < 127 and row[x + r] == row[x]:
                    r += 1
                if r >= 3:
                    out += bytes([128 + r, int(row[x])])
                    x += r
                    continue
                start = x
                while x < w and x - start < 128:
                    if x + 2 < w and row[x] == row[x + 1] == row[x + 2]:
                        break
                    x += 1
                out += bytes([x - start]) + bytes(row[start:x].tolist())
    return bytes(out)


def procedural_sky_rgba16(width: int = 256, height: int = 128, seed: int = 7) -> np.ndarray:
    """A deterministic R16G16B16A16_UNORM sky texture (gradient horizon, a bright sun disc, texel noise)
    standing in for the reference's sky_box image, which is not part of its asset tree."""
    rng = np.random.default_rng(seed)
    v = (np.arange(height) + 0.5) / height
    u = (np.arange(width) + 0.5) / width
    uu, vv = np.meshgrid(u, v)
    base = np.stack([0.25 + 0.6 * (1 - vv), 0.35 + 0.5 * (1 - vv), 0.55 + 0.4 * (1 - vv)], -1)
    sun = np.exp(-(((uu - 0.3) * 8) ** 2 + ((vv - 0.3) * 8) ** 2))[..., None] * np.array([0.9, 0.8, 0.5])
    c = np.clip(base * (0.8 + 0.4 * vv[..., None]) + sun + rng.uniform(-0.02, 0.02, (height, width, 3)), 0, 1)
    out = np.empty((height, width, 4), np.uint16)
    out[..., :3] = np.round(c * 65535).astype(np.uint16)
    out[..., 3] = 65535
    return out
