"""Per-wave dynamic instruction classes of a workload from tools/valu_class_pmc.sh (two --pmc passes): the VALU
instructions by class (rocprofv3 SQ_INSTS_VALU_<class>; gfx950 counts a packed fp32 op in its class once), their SIMD
cycles at DESIGN.md §5's measured costs, SALU and LDS, and the hardware's FP32 FLOP count where the pass recorded it.
usage: python tools/valu_class_summary.py <tag> [<out.json>]"""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from pmc_summarize import per_kernel  # noqa: E402


def main():
    tag = sys.argv[1]
    src = os.path.join(ROOT, "gpurun_out", f"vclass_{tag}")
    c = {}
    for part in ("a", "b"):
        hits = sorted(glob.glob(f"{src}/{part}/**/*counter_collection.csv", recursive=True))
        if not hits:
            raise SystemExit(f"missing {src}/{part}")
        c.update(per_kernel(hits[0]))
    waves = c["SQ_WAVES"]
    per_wave = {k: v / waves for k, v in sorted(c.items()) if k != "SQ_WAVES"}
    classes = {k[len("SQ_INSTS_VALU_"):]: v for k, v in per_wave.items() if k.startswith("SQ_INSTS_VALU_")}
    named = sum(classes.values())
    out = {"tag": tag, "waves_per_launch": waves, "per_wave": per_wave,
           "valu_per_wave": per_wave.get("SQ_INSTS_VALU"), "valu_classes_per_wave": classes,
           "valu_unclassified_per_wave": per_wave.get("SQ_INSTS_VALU", 0) - named,
           "note": "SQ_INSTS_VALU_<class>: ADD/MUL/FMA/TRANS per width, INT32/INT64, CVT; the remainder (moves, "
                   "compares, selects, bit ops, max/min/med3) is unclassified by the hardware counters"}
    text = json.dumps(out, indent=1)
    print(text)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text + "\n")


if __name__ == "__main__":
    main()
