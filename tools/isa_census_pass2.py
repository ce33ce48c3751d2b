"""Static instruction census of the wave-balanced faithful kernel's pass 2: the loop that walks
each lane's live lights two at a time (pbr_balanced.h, lighting_balanced_points), split into its main path -- the
two (pixel, light) items, the list bookkeeping, the window tests -- and the block that runs when a lane's pixel is
done (hand-back + next record), by instruction class, with the SIMD cycles of each class (DESIGN.md §5 measured
costs: packed fp32 / compare / select / fp64 4, plain fp32 and integer 2, transcendental 8; s_nop and SALU issue on
other units).

The loop is found in the device assembly (`make -C physically_based_renderer_amd/csrc asm`, or hipcc -S of
shade_kernels_bal.hip) as the block range that holds the item pair's twelve LDS reads (`ds_read_b32 ... offset:1360`,
the sixth structure-of-arrays row) up to the branch back to its header.

usage: python tools/isa_census_pass2.py [asm] [kernel-symbol-prefix]
"""
import re
import sys
from collections import Counter

ASM = sys.argv[1] if len(sys.argv) > 1 else "build/obj/shade_kernels_bal.s"
KERNEL = sys.argv[2] if len(sys.argv) > 2 else "_ZN3pbr17shade_tile_kernelILi1ELb0ELb0ELb0ELi1E"

CLASSES = [
    ("transcendental", re.compile(r"^v_(rcp|rsq|sqrt|exp|log|sin|cos)_")),
    ("fp64", re.compile(r"^v_(fma|mul|add)_f64|^v_cvt_f(64_f32|32_f64)")),
    ("packed fp32", re.compile(r"^v_pk_")),
    ("compare", re.compile(r"^v_cmp")),
    ("select/min/max", re.compile(r"^v_(cndmask|max|min|med3)")),
    ("plain fp32", re.compile(r"^v_(fma|mul|add|sub|subrev|fmac|ldexp|frexp|div_|trunc|floor|fract|cvt)_f32")),
    ("integer / mask", re.compile(r"^v_")),
    ("LDS", re.compile(r"^ds_")),
    ("SALU", re.compile(r"^s_(?!nop|waitcnt|cbranch|branch)")),
    ("s_nop / waitcnt", re.compile(r"^s_(nop|waitcnt)")),
    ("branch", re.compile(r"^s_(cbranch|branch)")),
]
CYCLES = {"packed fp32": 4, "compare": 4, "select/min/max": 4, "fp64": 4, "plain fp32": 2, "integer / mask": 2,
          "transcendental": 8}


def classify(op):
    for name, rx in CLASSES:
        if rx.search(op):
            return name
    return "other"


def kernel_lines(path, prefix):
    out, on = [], False
    for line in open(path):
        if not on and line.startswith(prefix) and line.rstrip().endswith(":") is False and ":" in line:
            on = line.split(":")[0].startswith(prefix)
            continue
        if on:
            if line.startswith(".Lfunc_end"):
                break
            out.append(line.rstrip("\n"))
    return out


def census(block):
    c = Counter()
    for t in block:
        t = t.strip()
        if not t or t.startswith((";", ".")):
            continue
        c[classify(t.split()[0])] += 1
    return c


def blocks_of(lines):
    """[(label, comment, [lines])] in layout order; the kernel's first block is unlabelled."""
    out, cur = [], ("<entry>", "", [])
    for l in lines:
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):?(.*)$", l)
        if m:
            out.append(cur)
            cur = (m.group(1), m.group(2), [])
        else:
            cur[2].append(l)
    out.append(cur)
    return out


def main():
    lines = kernel_lines(ASM, KERNEL)
    bl = blocks_of(lines)
    ri = next(k for k, b in enumerate(bl) if any("offset:1360" in l for l in b[2]))
    hk = max(k for k in range(ri + 1) if "Loop Header" in bl[k][1])
    hdr = bl[hk][0].lstrip(".")  # e.g. LBB8_612 -> the blocks of its loop carry "Header=BB8_612"
    tag = "Header=" + hdr[1:]
    # (a nested loop -- the faithful pieces' advance -- carries "Parent Loop BB8_612" on its blocks)
    loop = [b for k, b in enumerate(bl) if k == hk or tag in b[1] or ("Parent Loop " + hdr[1:]) in b[1]]
    # main path: the header and the fall-through blocks that follow it up to the one holding the done-mask compare
    main_blocks, k = [], hk
    while True:
        main_blocks.append(bl[k])
        if any("v_cmp_eq_u64" in l for l in bl[k][2]):
            break
        k += 1
    kinds = {"main path": [l for b in main_blocks for l in b[2]], "pixel done (hand-back, next record)": [],
             "grazing band (glibc x^5)": [], "control": []}
    names = {b[0] for b in main_blocks}
    for b in loop:
        if b[0] in names:
            continue
        if any(re.search(r"v_(fma|mul|add)_f64|v_cvt_f64", l) for l in b[2]):
            kinds["grazing band (glibc x^5)"] += b[2]
        elif any(l.strip().startswith("ds_") for l in b[2]):
            kinds["pixel done (hand-back, next record)"] += b[2]
        else:
            kinds["control"] += b[2]
    cen = {k: census(v) for k, v in kinds.items()}
    print(f"kernel {KERNEL}...: pass-2 loop (header .{hdr}, {len(loop)} blocks, {len(main_blocks)} on the main path)")
    hdr_row = f"{'class':18s}" + "".join(f"{k[:22]:>24s}" for k in cen)
    print(hdr_row)
    allc = [name for name, _ in CLASSES] + ["other"]
    for name in allc:
        if any(c[name] for c in cen.values()):
            print(f"{name:18s}" + "".join(f"{c[name]:24d}" for c in cen.values()))
    print(f"{'VALU instructions':18s}" + "".join(f"{sum(c[n] for n in CYCLES):24d}" for c in cen.values()))
    print(f"{'VALU SIMD cycles':18s}" + "".join(f"{sum(c[n] * w for n, w in CYCLES.items()):24d}" for c in cen.values()))


if __name__ == "__main__":
    main()
