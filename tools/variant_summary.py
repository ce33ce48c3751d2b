"""Per-wave instruction counts of development builds from tools/variant_pmc.sh (not part of the product).

    python tools/variant_summary.py gpurun_out/vpmc_v0 gpurun_out/vpmc_v1 ...

For each directory: the workload kernel's dispatches (the most frequent kernel name with the largest grid), the
counters summed per dispatch and divided by SQ_WAVES: VALU / SALU / LDS / VMEM-read instructions per wave, and
SQ_ACTIVE_INST_VALU / SQ_BUSY_CYCLES.
"""
import csv
import os
import sys
from collections import defaultdict


def summarize(d):
    path = os.path.join(d, "pmc_counter_collection.csv")
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for row in csv.DictReader(open(path)):
        k = row["Dispatch_Id"]
        names[k] = row["Kernel_Name"]
        per[k][row["Counter_Name"]] += float(row["Counter_Value"])
    # the workload kernel: the dispatches with the most waves
    big = max(per.values(), key=lambda c: c.get("SQ_WAVES", 0))["SQ_WAVES"]
    ds = [k for k in per if per[k].get("SQ_WAVES", 0) >= 0.99 * big]
    tot = defaultdict(float)
    for k in ds:
        for c, v in per[k].items():
            tot[c] += v / len(ds)
    w = tot["SQ_WAVES"]
    return {"dispatches": len(ds), "kernel": names[ds[0]][:60], "waves": w,
            "valu_per_wave": tot["SQ_INSTS_VALU"] / w, "salu_per_wave": tot["SQ_INSTS_SALU"] / w,
            "lds_per_wave": tot["SQ_INSTS_LDS"] / w, "vmem_rd_per_wave": tot["SQ_INSTS_VMEM_RD"] / w,
            "valu_busy": tot["SQ_ACTIVE_INST_VALU"] / max(tot["SQ_BUSY_CYCLES"], 1),
            "wave_cycles_per_wave": tot["SQ_WAVE_CYCLES"] / w}


def main():
    print(f"{'build':24s} {'waves':>8s} {'VALU/w':>9s} {'SALU/w':>8s} {'LDS/w':>7s} {'VMEMrd/w':>9s} {'cyc/w':>9s}")
    for d in sys.argv[1:]:
        s = summarize(d)
        print(f"{os.path.basename(d):24s} {s['waves']:8.0f} {s['valu_per_wave']:9.1f} {s['salu_per_wave']:8.1f} "
              f"{s['lds_per_wave']:7.1f} {s['vmem_rd_per_wave']:9.1f} {s['wave_cycles_per_wave']:9.0f}  {s['kernel']}")


if __name__ == "__main__":
    main()
