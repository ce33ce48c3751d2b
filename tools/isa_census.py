"""Instruction census of the shading kernel's light loops.

Reads the device assembly `make -C physically_based_renderer_amd/csrc asm` writes, takes one kernel
(default: the config-3 kernel, shade_tile_kernel<IBL, no F0 plane, no AO, no culling>), finds its loops
(a block range closed by a branch back to an earlier label) and counts each loop body's instructions by
class: packed fp32 (v_pk_*), other fp32 VALU, transcendental seeds (v_rcp/v_rsq/v_sqrt/v_exp/v_log),
compares, selects/med3/max, fp64, integer VALU, SALU, memory. A light loop executes its body once per
pixel pair and light, so the counts are per pair and light. SIMD-cycle weights per wave64 instruction are
the ones measured on gfx950: packed / cmp / cndmask / max / med3 / fp64 4, plain fp32 2,
transcendental 8.

usage: python tools/isa_census.py [asm] [kernel-substring]
"""
import re
import sys

ASM = sys.argv[1] if len(sys.argv) > 1 else "build/obj/shade_kernels.s"
KERNEL = sys.argv[2] if len(sys.argv) > 2 else "_ZN3pbr17shade_tile_kernelILi1ELb0ELb0ELb0E"

CLASSES = [
    ("trans", re.compile(r"^v_(rcp|rsq|sqrt|exp|log|sin|cos)_")),
    ("fp64", re.compile(r"^v_(fma|mul|add|cvt_f64|cvt_f32_f64|ldexp)_f64|^v_cvt_f64_f32|^v_cvt_f32_f64|^v_fma_f64|^v_mul_f64|^v_add_f64")),
    ("packed", re.compile(r"^v_pk_")),
    ("cmp", re.compile(r"^v_cmp")),
    ("sel", re.compile(r"^v_(cndmask|max|min|med3)_")),
    ("fp32", re.compile(r"^v_(fma|mul|add|sub|subrev|fmac|mac|ldexp|frexp|div_|trunc|floor|fract|cvt)")),
    ("ivalu", re.compile(r"^v_")),
    ("salu", re.compile(r"^s_(?!nop|waitcnt|cbranch|branch|load|buffer|endpgm|barrier|setprio|sleep)")),
    ("smem", re.compile(r"^s_(load|buffer)")),
    ("vmem", re.compile(r"^(global|buffer|scratch|flat)_")),
    ("lds", re.compile(r"^ds_")),
    ("nop", re.compile(r"^s_(nop|waitcnt)")),
    ("branch", re.compile(r"^s_(cbranch|branch)")),
]
CYCLES = {"packed": 4, "fp32": 2, "trans": 8, "cmp": 4, "sel": 4, "fp64": 4, "ivalu": 2}


def kernel_lines(path, name):
    out, on = [], False
    for line in open(path):
        if line.startswith(name) and line.rstrip().endswith(name.split()[0] + line[len(name):].split(":")[0] + ":") or (line.startswith(name) and ":" in line and not on):
            on = True
            continue
        if on:
            if line.startswith(".Lfunc_end"):
                break
            out.append(line.rstrip("\n"))
    return out


def classify(op):
    for c, rx in CLASSES:
        if rx.search(op):
            return c
    return "other"


def main():
    lines = kernel_lines(ASM, KERNEL)
    labels = {}
    insts = []  # (line_index, opcode, text)
    for i, l in enumerate(lines):
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            labels[m.group(1)] = len(insts)
            continue
        t = l.strip()
        if not t or t.startswith((";", ".")):
            continue
        insts.append((i, t.split()[0], t))
    loops = []
    for k, (_, op, t) in enumerate(insts):
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = t.split()[-1]
            if tgt in labels and labels[tgt] <= k:
                loops.append((labels[tgt], k))
    print(f"kernel {KERNEL}: {len(insts)} instructions, {len(loops)} loops")
    hdr = ["start", "len", "packed", "fp32", "trans", "cmp", "sel", "fp64", "ivalu", "salu", "smem", "vmem", "nop",
           "branch", "other", "valu", "cycles"]
    print(" ".join(f"{h:>7}" for h in hdr))
    for a, b in loops:
        cnt = {}
        for _, op, _t in insts[a:b + 1]:
            c = classify(op)
            cnt[c] = cnt.get(c, 0) + 1
        valu = sum(cnt.get(c, 0) for c in CYCLES)
        cyc = sum(cnt.get(c, 0) * w for c, w in CYCLES.items())
        row = [a, b - a + 1] + [cnt.get(h, 0) for h in hdr[2:15]] + [valu, cyc]
        print(" ".join(f"{v:>7}" for v in row))


if __name__ == "__main__":
    main()
