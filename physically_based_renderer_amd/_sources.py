"""The revision stamp of libpbrshade.so's sources (no imports beyond the standard library).

sources_sha() is the sha256 (first 16 hex digits) of csrc/*.hip, *.h, *.cpp, the Makefile and the public header. The
Makefile runs this file to embed the stamp in every object it compiles (pbr_build_info, ABI 9); bench.py and the
profile tools compare the stamp of the library a process actually loaded with the stamp of the checkout.

    python3 physically_based_renderer_amd/_sources.py      # prints the stamp of this checkout
"""
from __future__ import annotations

import hashlib
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC_DIR = os.path.join(PKG_DIR, "csrc")
HEADER_PATH = os.path.join(os.path.dirname(PKG_DIR), "include", "pbr", "pbr_shade.h")


def sources_sha(csrc_dir: str = CSRC_DIR, header: str = HEADER_PATH) -> str:
    h = hashlib.sha256()
    names = sorted(n for n in os.listdir(csrc_dir) if n.endswith((".hip", ".h", ".cpp")) or n == "Makefile")
    for path in [os.path.join(csrc_dir, n) for n in names] + [header]:
        h.update(os.path.basename(path).encode() + b"\0")
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(sources_sha())
