"""Summarise tools/wait_pmc.sh (gpurun_out/wait_c<N>_<mode>/): per config, each counter over SQ_WAVE_CYCLES and
the in-flight level per instruction (SQ_INST_LEVEL_x / SQ_INSTS_x) of scalar (SMEM), vector-read (VMEM) and LDS
instructions, over the workload's first six shading dispatches (bench.py --steps 5 --warmup 1 --ramp-ms 0).
usage: python tools/wait_summary.py <out.json> <config_mode>..."""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    out, tags = sys.argv[1], sys.argv[2:]
    res = {}
    for t in tags:
        p = glob.glob(os.path.join(ROOT, "gpurun_out", f"wait_{t}", "**", "*counter_collection.csv"), recursive=True)[0]
        shutil.copy(p, os.path.join(os.path.dirname(out), f"wait_pmc_{t}.csv"))
        rows = [r for r in csv.DictReader(open(p)) if "shade_" in r["Kernel_Name"]]
        ds = sorted({int(r["Dispatch_Id"]) for r in rows})[:6]
        v = {}
        for r in rows:
            if int(r["Dispatch_Id"]) in ds:
                v.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        v = {k: sum(x) / len(x) for k, x in v.items()}
        wc = v["SQ_WAVE_CYCLES"]
        res[t] = {"kernel": rows[0]["Kernel_Name"].split("(")[0],
                  "per_wave_cycle": {k: round(x / wc, 4) for k, x in sorted(v.items()) if k != "SQ_WAVE_CYCLES"},
                  "level_per_inst": {k: round(v[f"SQ_INST_LEVEL_{k}"] / max(v["SQ_INSTS_" + ("VMEM_RD" if k == "VMEM" else k)], 1), 2)
                                     for k in ("SMEM", "VMEM", "LDS")},
                  "vmem_over_smem_level": round(v["SQ_INST_LEVEL_VMEM"] / max(v["SQ_INST_LEVEL_SMEM"], 1), 1)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
