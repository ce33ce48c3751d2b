"""Derive the small input assets the GPU box needs from /root/reference/Assets (run here only).

/root/reference does not travel to the GPU box, so the shading inputs are committed as reduced data
files under physically_based_renderer_amd/assets/:
  * Chelsea_Stairs_Env.png      the 360x180 16-bit environment, byte-for-byte (decoded by envmap.py)
  * rustediron_256.npz          rustediron2_metallic/roughness (2048^2 u8 gray), every 8th texel
  * materials_1k_64.npz         the seven *_1K material sets the reference loads
                                (PBRApp.cpp:1270-1463): albedo, specular, roughness, normal and
                                (Metal_Bare only) metalness, every 16th texel of the 1024^2 JPEGs
JPEG decode is PIL/libjpeg (parity unpinned vs WIC, +-1 LSB); it only changes G-buffer content, which
both the GPU path and the oracle consume identically.
"""
import os
import shutil
import sys

import numpy as np
from PIL import Image

REF = "/root/reference/Assets"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "physically_based_renderer_amd", "assets")

MATERIALS = [  # (name, dir, file stem, has metalness)  PBRApp.cpp:892-962 order
    ("brick_modern", "Brick_Modern_1K", "semlcibb_8K", False),
    ("concrete_dirty", "Concrete_Dirty_1K", "rm4kshp_4K", False),
    ("concrete_rough", "Concrete_Rough_1K", "sdbhdd3b_8K", False),
    ("grass_wild", "Grass_Wild_1K", "sfknaeoa_8K", False),
    ("metal_bare", "Metal_Bare_1K", "se2abbvc_8K", True),
    ("soil_mud", "Soil_Mud_1K", "pjDtB2_8K", False),
    ("stone_wall", "Stone_Wall_1K", "scpgdgca_8K", False),
]


def rgb(path, step):
    return np.asarray(Image.open(path).convert("RGB"))[::step, ::step].copy()


def main():
    if not os.path.isdir(REF):
        sys.exit("needs /root/reference/Assets")
    os.makedirs(OUT, exist_ok=True)
    shutil.copyfile(os.path.join(REF, "Chelsea_Stairs", "Chelsea_Stairs_Env.png"),
                    os.path.join(OUT, "Chelsea_Stairs_Env.png"))

    met = np.asarray(Image.open(os.path.join(REF, "rustediron", "rustediron2_metallic.png")))[::8, ::8]
    rough = np.asarray(Image.open(os.path.join(REF, "rustediron", "rustediron2_roughness.png")))[::8, ::8]
    np.savez_compressed(os.path.join(OUT, "rustediron_256.npz"), metallic=met.astype(np.uint8),
                        roughness=rough.astype(np.uint8))

    step = 16
    n = 1024 // step
    albedo = np.zeros((7, n, n, 3), np.uint8)
    spec = np.zeros((7, n, n, 3), np.uint8)
    roughm = np.zeros((7, n, n), np.uint8)
    metal = np.zeros((7, n, n), np.uint8)
    normal = np.zeros((7, n, n, 3), np.uint8)
    has_metal = np.zeros(7, np.uint8)
    for i, (_name, d, stem, hm) in enumerate(MATERIALS):
        base = os.path.join(REF, d, stem)
        albedo[i] = rgb(base + "_Albedo.jpg", step)
        spec[i] = rgb(base + "_Specular.jpg", step)
        roughm[i] = rgb(base + "_Roughness.jpg", step)[..., 0]  # Sample(...).r, Default.hlsl:99
        normal[i] = rgb(base + "_Normal.jpg", step)
        if hm:
            metal[i] = rgb(base + "_Metalness.jpg", step)[..., 0]  # Default.hlsl:86
            has_metal[i] = 1
    np.savez_compressed(os.path.join(OUT, "materials_1k_64.npz"), albedo=albedo, specular=spec,
                        roughness=roughm, metallic=metal, has_metallic=has_metal, normal=normal,
                        names=np.array([m[0] for m in MATERIALS]))
    for f in sorted(os.listdir(OUT)):
        print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
