"""Phase census of a pair kernel (VERDICT r05 "next round" item 1): every VALU instruction of the kernel's hot path,
labelled with the phase it belongs to and weighted by how often the phase runs per wave.

Input: the device assembly of a census build (PBR_CENSUS=1: the kernel sources mark where each phase begins with
PBR_PHASE(name), an assembly comment fenced by scheduling barriers, shade_kernels.h), e.g.
    hipcc ... -DPBR_CENSUS=1 --cuda-device-only -S csrc/shade_kernels_bal.hip -o build/obj/census_bal.s

Method. The kernel carries every path of its template (directional lights, the exact fallbacks, the sky pass); only
some run on a given workload. The tool builds the control-flow graph of the kernel's blocks and, for each pair of
consecutive markers of the path (`--path`, default the balanced faithful path of config 3), takes the blocks that lie
on a path from the one marker to the next without crossing another marker. Those blocks are split into
  * always: blocks every execution of the phase passes through (dominators of the next marker in the region's
    graph) -- straight-line code;
  * divergent: blocks entered under an EXEC mask (`s_and_saveexec` / `s_cbranch_execz`: a per-lane `if` whose
    body the wave runs whenever one lane takes it; counted as executed, which is what happens on data with mixed
    lanes);
  * uniform-rare: blocks behind a wave-uniform branch (`s_cbranch_scc*` / `vcc*`) that is not the phase's main line
    (fallbacks, special-value paths): listed, not counted;
  * cold: blocks holding IEEE-division sequences or fp64 glibc polynomials (FMAs: the rare-lane patches), and code
    after a PBR_COLD marker (fallbacks and other modes' branches): not counted.
Loops (pass 2) are weighted by their iteration count per wave (`--weights pass2=34.7`, from the balanced phase
profile / pass statistics); every other phase runs once per wave. Classes and SIMD-cycle weights follow
tools/isa_census_pass2.py (DESIGN.md §5's measured costs); `v_writelane` / `v_readlane` (SGPR spills to VGPR lanes and
uniform reads) and `v_mov` are counted as their own classes.

usage: python tools/isa_census_phases.py ASM [--kernel PREFIX] [--weights pass2=34.7] [--total 6459]
"""
import argparse
import re
from collections import Counter, defaultdict

CLASSES = [
    ("transcendental", re.compile(r"^v_(rcp|rsq|sqrt|exp|log|sin|cos)_")),
    ("fp64", re.compile(r"^v_(fma|mul|add)_f64|^v_cvt_f(64_f32|32_f64)")),
    ("packed fp32", re.compile(r"^v_pk_(fma|mul|add)_f32")),
    ("fp32 arith", re.compile(r"^v_(fma|fmac|mul|add|sub|subrev|mac)_f32|^v_(ldexp|frexp|fract|trunc|floor|rndne|div_)")),
    ("compare", re.compile(r"^v_cmp")),
    ("select", re.compile(r"^v_cndmask")),
    ("min/max/med3", re.compile(r"^v_(max|min|med3)")),
    ("lane move (readlane/writelane/readfirstlane)", re.compile(r"^v_(readlane|writelane|readfirstlane)")),
    ("move", re.compile(r"^v_(mov|pk_mov|accvgpr)")),
    ("integer/bit", re.compile(r"^v_")),
    ("LDS", re.compile(r"^ds_")),
    ("VMEM", re.compile(r"^(global|buffer|flat|scratch)_")),
    ("SMEM", re.compile(r"^s_(load|buffer_load|store|dcache)")),
    ("s_nop/waitcnt", re.compile(r"^s_(nop|waitcnt)")),
    ("branch", re.compile(r"^s_(cbranch|branch|setpc)")),
    ("SALU", re.compile(r"^s_")),
]
VALU = ["transcendental", "fp64", "packed fp32", "fp32 arith", "compare", "select", "min/max/med3",
        "lane move (readlane/writelane/readfirstlane)", "move", "integer/bit"]
FP = {"transcendental", "packed fp32", "fp32 arith"}  # fp32 arithmetic (the FLOP-carrying classes)
CYCLES = {"packed fp32": 4, "compare": 4, "select": 4, "min/max/med3": 4, "fp64": 4, "fp32 arith": 2,
          "integer/bit": 2, "transcendental": 8, "move": 2, "lane move (readlane/writelane/readfirstlane)": 2}
DEFAULT_PATH = ["entry", "load_window", "pass1", "invariants", "rank", "pass2", "handback", "invariants2",
                "stats_repass", "finish_setup", "ibl", "finish", "store"]


def classify(op):
    for name, rx in CLASSES:
        if rx.search(op):
            return name
    return "other"


def kernel_lines(path, prefix):
    out, on = [], False
    for line in open(path):
        if not on and line.startswith(prefix) and ":" in line:
            on = True
            continue
        if on:
            if line.startswith(".Lfunc_end"):
                break
            out.append(line.rstrip("\n"))
    return out


class Block:
    def __init__(self, label, comment):
        self.label, self.comment = label, comment
        self.items = []  # ("insn", op, text) | ("phase", name)
        self.succ = []

    def insns(self):
        return [x for x in self.items if x[0] == "insn"]


def parse(lines):
    blocks, cur = [], Block("<entry>", "")
    for l in lines:
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):?(.*)$", l)
        if m:
            blocks.append(cur)
            cur = Block(m.group(1).lstrip(".").replace("; %", ""), m.group(2))
            continue
        t = l.strip()
        pm = re.match(r"^; @phase (\S+)", t)
        if pm:
            cur.items.append(("phase", pm.group(1)))
            continue
        if not t or t.startswith((";", ".")):
            continue
        op = t.split()[0]
        cur.items.append(("insn", op, t))
    blocks.append(cur)
    index = {b.label: k for k, b in enumerate(blocks)}
    for k, b in enumerate(blocks):
        ins = b.insns()
        falls = True
        for _, op, t in ins[-3:]:
            if op.startswith("s_cbranch") or op == "s_branch":
                target = t.split()[1].lstrip(".")
                if target in index:
                    b.succ.append(index[target])
            if op in ("s_branch", "s_endpgm", "s_setpc_b64"):
                falls = False
        if falls and k + 1 < len(blocks):
            b.succ.append(k + 1)
    return blocks


def is_cold(b):
    ops = [op for _, op, _ in b.insns()]
    if any(op.startswith(("v_div_scale", "v_div_fmas", "v_div_fixup")) for op in ops):
        return True  # an IEEE division: the exact fallback's sequence
    if sum(1 for op in ops if re.match(r"v_fmac?_f64", op)) >= 3:
        return True  # fp64 polynomial (FMAs): glibc's powf patched in for rare lanes (the exact x^5's plain fp64
        # products, v_mul_f64 only, are the exact kernel's main path)
    return False


def guard_kind(blocks, pred, b):
    """How block b is entered from pred: 'exec' (divergent if), 'uniform' (scc / vcc branch) or 'fall'."""
    ins = blocks[pred].insns()
    for _, op, t in ins[-3:]:
        if op.startswith("s_cbranch_exec"):
            return "exec"
        if op.startswith("s_cbranch_scc") or op.startswith("s_cbranch_vcc"):
            return "uniform"
    return "fall"


def region(blocks, start, stop_names, start_name):
    """Blocks reachable from the marker block `start` (from the marker on) to the block holding the next path marker,
    without passing another marker. Returns (blocks, the end block index or None)."""
    marker_blocks = {k for k, b in enumerate(blocks) if any(x[0] == "phase" for x in b.items)}
    seen, stack, ends = set(), [start], set()
    while stack:
        k = stack.pop()
        if k in seen:
            continue
        seen.add(k)
        names = [x[1] for x in blocks[k].items if x[0] == "phase"]
        if k != start and names:
            if names[0] in stop_names:
                ends.add(k)
            continue  # another marker: the region ends here
        if k == start and names and names[-1] != start_name:
            # the start block holds a later marker too (a phase with no code): stop
            ends.add(k)
            continue
        for s in blocks[k].succ:
            if not is_cold(blocks[s]):
                stack.append(s)
    # keep only blocks from which an end is reachable (inside the region)
    rev = defaultdict(set)
    for k in seen:
        for s in blocks[k].succ:
            if s in seen:
                rev[s].add(k)
    back, stack = set(), list(ends)
    while stack:
        k = stack.pop()
        if k in back:
            continue
        back.add(k)
        stack.extend(rev[k])
    return sorted(seen & back), ends


def dominators_of(blocks, nodes, start, end):
    """Blocks on every path from start to end inside `nodes` (iterative dominator sets)."""
    nodes = set(nodes)
    preds = defaultdict(set)
    for k in nodes:
        for s in blocks[k].succ:
            if s in nodes:
                preds[s].add(k)
    dom = {k: set(nodes) for k in nodes}
    dom[start] = {start}
    changed = True
    while changed:
        changed = False
        for k in sorted(nodes):
            if k == start:
                continue
            ps = [dom[p] for p in preds[k]]
            new = ({k} | set.intersection(*ps)) if ps else {k}
            if new != dom[k]:
                dom[k], changed = new, True
    return dom.get(end, set())


def phase_part(block, phase, where):
    """The instructions of `block` that belong to `phase`: after its marker (where='start'), before the next marker
    (where='end'), or all of them."""
    out, on = [], where != "start"
    for x in block.items:
        if x[0] == "phase":
            if where == "start":
                on = x[1] == phase
            elif where == "end":
                break
            else:
                on = x[1] == phase
            continue
        if on:
            out.append(x)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--kernel", default="_ZN3pbr17shade_tile_kernelILi1ELb0ELb0ELb0ELi1E")
    ap.add_argument("--path", nargs="+", default=DEFAULT_PATH)
    ap.add_argument("--weights", nargs="*", default=["pass2=34.7"], help="phase=executions per wave")
    ap.add_argument("--total", type=float, default=None, help="measured SQ_INSTS_VALU per wave, for the check")
    a = ap.parse_args()
    weights = {k: float(v) for k, v in (w.split("=") for w in a.weights)}
    blocks = parse(kernel_lines(a.asm, a.kernel))
    where = {}
    for k, b in enumerate(blocks):
        for x in b.items:
            if x[0] == "phase":
                where.setdefault(x[1], k)
    print(f"kernel {a.kernel}...: {len(blocks)} blocks, {sum(len(b.insns()) for b in blocks)} instructions; "
          f"phase markers found: {sorted(where)}")
    rows, detail = [], []
    extra_once = {}
    cond_blocks = defaultdict(list)

    def loop_counts(blocks, nodes, start, end, ph):
        """Per-iteration VALU of the loop inside the region (its blocks carry 'Loop Header' / 'in Loop' comments):
        blocks on every path from the header to the latch, plus divergent bodies; blocks behind a uniform branch
        inside the loop (the lane-done hand-over) are returned apart; blocks outside the loop run once."""
        inloop = [k for k in nodes if "Loop" in blocks[k].comment]
        header = min(inloop)
        latch = max(k for k in inloop if header in blocks[k].succ)
        dom = dominators_of(blocks, inloop, header, latch)
        preds = defaultdict(set)
        for k in inloop:
            for s_ in blocks[k].succ:
                preds[s_].add(k)
        per, once, cond = Counter(), Counter(), Counter()
        for k in nodes:
            items = (phase_part(blocks[k], ph, "start") if k == start else
                     phase_part(blocks[k], ph, "end") if k == end else [x for x in blocks[k].items if x[0] == "insn"])
            c = Counter(classify(op) for _, op, _ in [x for x in items if x[0] == "insn"])
            if k not in inloop:
                once += c
            elif k in dom:
                per += c
            else:
                kinds = {guard_kind(blocks, p, k) for p in preds[k]}
                if "uniform" in kinds:
                    cond += c
                    nv = sum(c[n] for n in VALU)
                    if nv:
                        first = [x[2] for x in items if x[0] == "insn" and x[2].startswith("v_")][:3]
                        cond_blocks[ph].append((blocks[k].label, nv, "; ".join(first)))
                else:
                    per += c
        return per, once, cond
    total_w, total_fp_w = 0.0, 0.0
    for i, ph in enumerate(a.path):
        if ph not in where:
            print(f"phase {ph}: no marker")
            continue
        start = where[ph]
        nxt = a.path[i + 1:i + 2]
        nodes, ends = region(blocks, start, set(nxt) if nxt else set(), ph)
        if not nxt:  # the last phase: every block reachable from the marker
            nodes, ends = region(blocks, start, {"__none__"}, ph)
            nodes = sorted(set(nodes) | {start})
        end = min(ends) if ends else None
        dom = dominators_of(blocks, nodes, start, end) if end is not None else {start}
        preds = defaultdict(set)
        for k in nodes:
            for s in blocks[k].succ:
                preds[s].add(k)
        cat = {"always": Counter(), "divergent": Counter(), "uniform-rare": Counter()}
        listed = []
        for k in nodes:
            b = blocks[k]
            part = "start" if k == start else ("end" if k == end else "all")
            if k == start and k == end:
                # both markers in one block: the code between them
                items, on = [], False
                for x in b.items:
                    if x[0] == "phase":
                        on = x[1] == ph
                        continue
                    if on:
                        items.append(x)
            else:
                items = phase_part(b, ph, part)
            c = Counter(classify(op) for _, op, _ in [x for x in items if x[0] == "insn"])
            if k in dom or k == start:
                kind = "always"
            else:
                kinds = {guard_kind(blocks, p, k) for p in preds[k] if p in nodes}
                kind = "divergent" if kinds <= {"exec", "fall"} and "exec" in kinds else (
                    "uniform-rare" if "uniform" in kinds else "divergent")
            cat[kind] += c
            nv = sum(c[n] for n in VALU)
            if nv and kind != "always":
                first = [t for x in items if x[0] == "insn" for t in [x[2]] if t.startswith("v_")][:3]
                listed.append((kind, b.label, nv, "; ".join(first)))
        cold = sorted({s for k in nodes for s in blocks[k].succ if is_cold(blocks[s])})
        w = weights.get(ph, 1.0)
        counted = cat["always"] + cat["divergent"]
        if w != 1.0:  # a loop phase: per iteration = the loop's blocks; the rest of the region runs once
            counted, once, cond = loop_counts(blocks, nodes, start, end, ph)
            cat = {"always": counted, "divergent": Counter(), "uniform-rare": cond}
            pre = sum(once[n] for n in VALU)
            extra_once[ph] = pre
            listed = [("per-pixel-done", lbl, n, f) for lbl, n, f in cond_blocks[ph]]
        nv = sum(counted[n] for n in VALU)
        nfp = sum(counted[n] for n in VALU if n in FP)
        cyc = sum(counted[n] * CYCLES.get(n, 0) for n in VALU)
        total_w += nv * w + extra_once.get(ph, 0)
        total_fp_w += nfp * w
        rows.append((ph, w, counted, nv, nfp, cyc))
        detail.append((ph, cat, listed, cold, len(nodes)))
    # table
    shown = [n for n in VALU if any(r[2][n] for r in rows)]
    print()
    print("Per execution of each phase (always + divergent blocks), VALU instructions by class:")
    print(f"{'phase':14s}{'runs/wave':>10s}" + "".join(f"{n[:12]:>13s}" for n in shown) + f"{'VALU':>8s}{'non-FP':>8s}"
          f"{'cycles':>8s}{'VALU/wave':>11s}{'nonFP/wave':>11s}")
    for ph, w, c, nv, nfp, cyc in rows:
        print(f"{ph:14s}{w:10.1f}" + "".join(f"{c[n]:13d}" for n in shown) +
              f"{nv:8d}{nv - nfp:8d}{cyc:8d}{nv * w:11.0f}{(nv - nfp) * w:11.0f}")
    print(f"{'total':14s}{'':10s}" + "".join(f"{'':13s}" for n in shown) + f"{'':8s}{'':8s}{'':8s}{total_w:11.0f}"
          f"{total_w - total_fp_w:11.0f}")
    if a.total:
        print(f"measured SQ_INSTS_VALU per wave: {a.total:.0f}; this census accounts for {total_w / a.total:.3f} of it")
    print()
    print("Blocks counted as divergent (run when any lane takes them) and uniform-rare (not counted), per phase:")
    for ph, cat, listed, cold, n in detail:
        nr = sum(cat["uniform-rare"][x] for x in VALU)
        print(f"  {ph}: {n} blocks; uniform-rare VALU {nr}; cold successors (IEEE division / fp64 glibc, not counted): "
              f"{len(cold)}")
        for kind, label, nv, first in sorted(listed, key=lambda t: -t[2])[:8]:
            print(f"    {kind:12s} {label:10s} {nv:4d} VALU  {first[:100]}")


if __name__ == "__main__":
    main()
