"""List scratch (spill) instructions of one kernel in the device assembly, with the enclosing loop depth.
usage: python tools/spills.py [asm] [kernel-substring]"""
import sys
asm = sys.argv[1] if len(sys.argv) > 1 else "build/obj/shade_kernels.s"
name = sys.argv[2] if len(sys.argv) > 2 else "_ZN3pbr17shade_tile_kernelILi1ELb0ELb0ELb0E"
s = open(asm).read()
i = s.index("\n" + name) + 1
j = s.index(".Lfunc_end", i)
lines = s[i:j].split("\n")
depth = 0
for n, l in enumerate(lines):
    if "Loop Header" in l or "in Loop" in l:
        pass
    if "scratch_" in l:
        ctx = ""
        for k in range(n, max(0, n - 400), -1):
            if lines[k].startswith(".LBB") or lines[k].startswith("; %bb"):
                ctx = lines[k].strip()
                break
        print(n, l.strip(), "|", ctx[:90])
