"""Turn tools/profile_round.sh output (gpurun_out/prof_<tag>) into the committed evidence:
profiles/<tag>/{kernel_stats,pmc_*}.csv and the per-workload entry of profiles/pmc_summary.json
that bench.py reads for roofline.traffic.

HBM bytes per launch = FETCH_SIZE x 2 + WRITE_SIZE (KiB; gfx950 FETCH_SIZE reports half of a
coalesced read, MI355X_MICROARCH.md "HBM"), averaged over the shading kernel's dispatches.
usage: python tools/pmc_summarize.py <tag> <workload> <pixels> <bytes_per_px> <lights> <revision> [<profiles subdir>]
The entry's kernel_sources_sha is the stamp of the library the PROFILED process loaded (the bench line's `library`,
pbr_build_info): a profile of a development, debug or stale build (library.problems non-empty) is refused, and the
stamp never comes from the files of the checkout that summarises it.
"""
import csv
import glob
import json
import os
import shutil
import sys

N_SIMD = 256 * 4  # MI355X: 256 CUs x 4 SIMDs
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# Entry fields that are not measurements and survive a re-profile of the same library (anything else is replaced).
CARRIED = ("note",)


def library_stamp(bench_line: dict) -> tuple:
    """(sources stamp, library record) of the library the profiled bench process loaded; raises SystemExit when that
    was not the product build of its checkout, or when the line predates pbr_build_info."""
    lib = (bench_line or {}).get("library")
    if not lib or not lib.get("sources_sha"):
        raise SystemExit("the profiled bench line names no library build (pbr_build_info): cannot stamp the profile")
    if lib.get("problems"):
        raise SystemExit("the profiled library is not a product build: " + "; ".join(lib["problems"]))
    return lib["sources_sha"], {k: lib[k] for k in ("path", "sources_sha", "flavor", "tree_sources_sha") if k in lib}


def find(pattern):
    hits = sorted(glob.glob(pattern, recursive=True))
    if not hits:
        raise SystemExit(f"missing {pattern}")
    return hits[0]


# The --pmc passes run bench.py --steps 5 --warmup 1 --ramp-ms 0 (profile_round.sh): the workload's launches are
# the first six shading dispatches; later ones (the N = 1 line's config-5 scale anchor) are another workload.
PMC_LAUNCHES = 6


def per_kernel(path, kernel=("shade_tile", "shade_lean"), launches=PMC_LAUNCHES):
    vals = {}
    with open(path) as f:
        rows = [r for r in csv.DictReader(f) if any(k in r.get("Kernel_Name", r.get("Name", "")) for k in kernel)]
    dispatches = sorted({int(r["Dispatch_Id"]) for r in rows})[:launches]
    for row in rows:
        if int(row["Dispatch_Id"]) in dispatches:
            vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    tag, workload, pixels, bpp, lights, revision = sys.argv[1:7]
    pixels, bpp, lights = int(pixels), int(bpp), int(lights)
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst_tag = sys.argv[7] if len(sys.argv) > 7 else tag
    dst = os.path.join(ROOT, "profiles", dst_tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(find(f"{src}/kt/**/*kernel_stats.csv"), os.path.join(dst, f"kernel_stats_{workload}.csv"))
    shutil.copy(os.path.join(src, "kt.log"), os.path.join(dst, f"bench_{workload}.log"))
    counters = {}
    for name in ("fetch", "write", "sq", "busy"):
        p = find(f"{src}/pmc_{name}/**/*counter_collection.csv")
        shutil.copy(p, os.path.join(dst, f"pmc_{name}_{workload}.csv"))
        counters.update(per_kernel(p))
    bench = None
    for line in open(os.path.join(src, "kt.log")):
        if line.startswith("{"):
            bench = json.loads(line)
    stamp, library = library_stamp(bench)
    hbm = counters["FETCH_SIZE"] * 2 * 1024 + counters["WRITE_SIZE"] * 1024
    alg = pixels * bpp
    entry = {
        "hbm_bytes_per_launch": hbm,
        "fetch_size_kib": counters["FETCH_SIZE"],
        "write_size_kib": counters["WRITE_SIZE"],
        "correction": "FETCH_SIZE x2 (gfx950 reports half of a coalesced read: MI355X_MICROARCH.md HBM); "
                      "WRITE_SIZE as reported; KiB",
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": hbm / alg,
        "sq": {k: v for k, v in sorted(counters.items()) if k.startswith(("SQ_", "GRBM_"))},
        "valu_insts_per_pixel_light": counters["SQ_INSTS_VALU"] * 64 / pixels / max(lights, 1),
        # SQ_ACTIVE_INST_VALU counts quad-cycles summed over waves; GRBM_GUI_ACTIVE is summed over the 8
        # XCDs (MI355X_MICROARCH.md): VALU-issue cycles per SIMD over kernel cycles.
        "valu_issue_busy": counters["SQ_ACTIVE_INST_VALU"] * 4 / N_SIMD / (counters["GRBM_GUI_ACTIVE"] / 8),
        "source": f"profiles/{dst_tag}/pmc_*_{workload}.csv (rocprofv3 --pmc, separate passes, bench.py --steps 5)",
        "kernel_revision": revision,
        # bench.py quotes traffic / valu_issue_busy only while the library it loads carries this stamp
        "kernel_sources_sha": stamp,
        "library": library,
        "kernel": bench["roofline"].get("kernel"),
        # the balanced exact kernel reads the G-buffer pair again after its light loop (+44 B/px)
        "pair_reread": str(bench["roofline"].get("kernel", "")).endswith(", 2>"),
    }
    # Kernel trace of the bench run itself: mean launch time over the timed steps (the last K launches;
    # the clock-ramp and warm-up launches come first) next to the bench's own HIP-event average.
    trace = find(f"{src}/kt/**/*kernel_trace.csv")
    shutil.copy(trace, os.path.join(dst, f"kernel_trace_{workload}.csv"))
    with open(trace) as f:
        durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in csv.DictReader(f)
                if "shade_tile" in r["Kernel_Name"] or "shade_lean" in r["Kernel_Name"]]
    # launch order of bench.py: clock ramp, warm-up steps, the K timed steps, then (exact leg, scale anchor)
    k = bench["steps"] if bench else len(durs)
    first = bench["clock_ramp"]["launches"] + bench["warmup"] if bench else len(durs) - k
    timed = durs[first:first + k]
    entry["kernel_trace"] = {
        "launches": len(durs), "mean_ms_all": sum(durs) / len(durs),
        "mean_ms_timed_steps": sum(timed) / len(timed), "timed_steps": len(timed), "first_timed_launch": first,
        "bench_avg_launch_ms": bench["roofline"]["avg_launch_ms"] if bench else None,
        "bench_value": bench["value"] if bench else None,
    }
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    summary = json.load(open(path)) if os.path.exists(path) else {}
    old = summary.get(workload, {})
    if old.get("kernel_sources_sha") == stamp:  # hand-written notes survive a re-profile of the same library only
        for k in CARRIED:
            if k in old:
                entry.setdefault(k, old[k])
    summary[workload] = entry
    json.dump(summary, open(path, "w"), indent=1)
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main()
