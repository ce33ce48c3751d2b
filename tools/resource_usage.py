"""Tabulate the compiler's kernel-resource-usage remarks (make -C physically_based_renderer_amd/csrc
resource-usage > report.txt 2>&1): one line per kernel with VGPRs, scratch bytes per lane, LDS bytes per block
and occupancy (waves per SIMD), kernel names demangled to their template arguments.
usage: python tools/resource_usage.py report.txt [name-substring]"""
import re
import sys

FIELDS = {"VGPRs": "vgpr", "ScratchSize [bytes/lane]": "scratch", "LDS Size [bytes/block]": "lds",
          "Occupancy [waves/SIMD]": "occ", "VGPRs Spill": "vspill"}


def parse(text):
    kernels, cur = [], None
    for line in text.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            kernels.append(cur)
            continue
        m = re.search(r"remark:\s+([^:]+(?:\[[^\]]*\])?): (\S+) \[-Rpass", line)
        if m and cur is not None and m.group(1).strip() in FIELDS:
            cur[FIELDS[m.group(1).strip()]] = m.group(2)
    return kernels


def short(name):
    m = re.match(r"_ZN3pbr\d+(\w+?)I(.*?)EEvNS_", name)
    if not m:
        return name[:60]
    args = re.findall(r"L([ib])(\d)E", m.group(2))
    return f"{m.group(1)}<{','.join(('true' if v == '1' else 'false') if t == 'b' else v for t, v in args)}>"


def main():
    kernels = parse(open(sys.argv[1], errors="replace").read())
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    print(f"{'kernel':58s} {'VGPR':>5s} {'scratch':>7s} {'LDS':>6s} {'occ':>4s}")
    for k in kernels:
        if sub in k["name"]:
            print(f"{short(k['name']):58s} {k.get('vgpr', '?'):>5s} {k.get('scratch', '?'):>7s} "
                  f"{k.get('lds', '?'):>6s} {k.get('occ', '?'):>4s}")


if __name__ == "__main__":
    main()
