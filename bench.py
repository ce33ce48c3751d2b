#!/usr/bin/env python3
"""Headline benchmark: shaded pixels/s and achieved HBM GB/s of the G-buffer shading pass.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C]

N = 1: BASELINE config 3 -- a 3840x2160 G-buffer, 64 point lights + diffuse IBL (Chelsea_Stairs),
one step = one shading pass over the whole frame (inputs resident in HBM before timing).
N > 1 (launched by torch.distributed.run, one rank per GPU, RCCL): BASELINE config 5 geometry --
an 8192-wide frame of 1024 rows per rank (8192x8192 at N = 8); one step = every rank shades its
row band and the bands are gathered to rank 0 (pipelined: the gather of frame k overlaps the shading
of frame k+1) as the presented R8G8B8A8_UNORM frame (--output; shading is fp32 at every N). Weak
scaling: per-GPU work is fixed.

Rank 0 prints one JSON line ("Measurement"). The cpu_baseline leg times the CPU
oracle (oracle/, test infrastructure) on a bounded row sample of the same frame and doubles as a
parity check of the sampled rows.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from physically_based_renderer_amd import _native as N  # noqa: E402
from physically_based_renderer_amd import dist as D  # noqa: E402
from physically_based_renderer_amd import scenes as S  # noqa: E402
from physically_based_renderer_amd.renderer import ShadingContext  # noqa: E402

METRIC = "shaded pixels/sec (Mpix/s) + achieved HBM GB/s, 4K G-buffer, 64 lights"
HBM_PEAK_GBPS = 8000.0     # MI355X_MICROARCH.md, chip-level parameters (spec)
FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md, vector FP32 (spec)
# Algorithmic FLOP per pixel (+,-,*,/,sqrt,pow = 1 each after parity-safe hoisting):
# base 27 + 20 hoisted BRDF invariants + 91 per point light + 87 for the diffuse IBL.
FLOP_BASE, FLOP_HOIST, FLOP_POINT, FLOP_IBL = 27, 20, 91, 87
FLOP_RANGE_TEST = 9  # per light and tile under tiled culling (box distance + compare)
# The north-star parity bar: RGBA within 1e-5 relative fp32 per channel of the reference CPU evaluation (NaN where
# it has NaN). RGBA8 output: a 1e-5 relative difference can move a code by one where c * 255 + 0.5 sits on an
# integer, so codes may differ by at most 1.
PARITY_REL_TOL = 1e-5
PARITY_RGBA8_CODE_TOL = 1
EXIT_PARITY = 3  # bench.py's exit status when the checked frame misses the bar (no metric line is printed)
EXIT_PROVENANCE = 4  # ... when the loaded library is not the product build of this checkout (without --dev)
# Environment variables that only route the transport of the multi-rank run; every other PBR_* variable changes which
# library or kernel runs (PBR_LIB_PATH, PBR_BALANCED_MIN, PBR_LEAN, PBR_PIXELS_PER_THREAD, ...): a development setting.
ENV_NEUTRAL = ("PBR_DIST_TIMEOUT_S", "PBR_DIST_INIT_METHOD")
# Version of the line's keys, bumped when a key changes meaning (6: hbm_gbps = the kernel's own bytes, hbm_gbps_model
# = SURVEY 8(d)'s; pcie_h2d_gbps = the warm link rate, pcie_h2d_first_gbps = the first copy; roofline.bound_unit,
# frac_profile, launch_vs_profile). Lines without the key are rounds 1-5.
LINE_SCHEMA = 6


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def bytes_per_pixel(pc, out_bytes: int = 16) -> int:
    """Algorithmic HBM bytes per shaded pixel, SURVEY 8(d)'s model: the 12 G-buffer planes of the north star's
    G-buffer (position, normal, albedo, metallic, roughness, AO: 48 B), + the F0 plane (12 B) when the pass reads it,
    + the RGBA write (16 B fp32, 4 B RGBA8): 64 B/px for configs 1-3 and 5, 76 B/px for config 4."""
    planes = 12
    if pc.flags & N.PBR_FLAG_F0_PLANE:
        planes += 3
    return planes * 4 + out_bytes


def bytes_read_per_pixel(pc, out_bytes: int = 16) -> int:
    """The bytes the kernel itself moves per pixel: the AO plane only with PBR_FLAG_APPLY_AO (the reference never
    reads its AO slot), so 60 B/px where 8(d) counts 64."""
    planes = 11  # pos xyz, normal xyz, albedo rgb, metallic, roughness
    if pc.flags & N.PBR_FLAG_APPLY_AO:
        planes += 1
    if pc.flags & N.PBR_FLAG_F0_PLANE:
        planes += 3
    return planes * 4 + out_bytes


def library_provenance(dev: bool) -> dict:
    """The build the process LOADED (pbr_build_info, ABI 9) against this checkout: its sources stamp, flavor and units,
    the checkout's stamp, and the reasons it is not the product build of this checkout (`problems`: units of
    different sources, another checkout, a debug / variant / EXTRA-flags build, PBR_* development overrides in the
    environment). Empty problems = the measured binary is the one the committed sources describe."""
    info = N.build_info()
    tree = N.kernel_sources_sha()
    problems = N.build_problems(info, tree)
    overrides = {k: v for k, v in sorted(os.environ.items()) if k.startswith("PBR_") and k not in ENV_NEUTRAL}
    if overrides:
        problems.append("development environment overrides: " + ", ".join(f"{k}={v}" for k, v in overrides.items()))
    if os.path.abspath(N.LIB_PATH) != os.path.abspath(os.path.join(N.PKG_DIR, "_lib", "libpbrshade.so")):
        problems.append(f"not the in-tree library: {N.LIB_PATH}")
    return {"path": os.path.relpath(os.path.abspath(N.LIB_PATH), ROOT), "sources_sha": info.get("sources_sha"),
            "flavor": info.get("flavor"), "tree_sources_sha": tree, "problems": problems, "dev": dev,
            "units": [{k: u[k] for k in ("unit", "sources_sha", "flavor", "cflags")} for u in info.get("units", [])],
            "env_overrides": overrides}


FLOP_DIR = FLOP_POINT - 17  # 74 per directional light (no distance / attenuation)
FLOP_BACKFACE_TEST = 8  # the wave-balanced lists' pass-1 test: 4 FMAs per (pixel, point light)


def flops_per_pixel(pc, lights_per_tile=None, tile_px: int = 128) -> float:
    """Algorithmic FLOP per pixel, SURVEY 8(d)'s model: every light of the pass for every pixel
    (LightingUtil.hlsl:176-199 sums them all). With tiled culling only the lights that survive a tile are
    shaded (base + L_in per-light BRDFs); the 9-FLOP range test of every point/spot light is
    counted once per culling tile (the unit that runs it), not per pixel."""
    n_ps = pc.num_point_lights + pc.num_spot_lights
    f = FLOP_BASE + FLOP_HOIST
    if pc.flags & N.PBR_FLAG_TILED_CULLING and lights_per_tile is not None:
        f += FLOP_POINT * lights_per_tile + FLOP_RANGE_TEST * n_ps / tile_px
    else:
        f += FLOP_POINT * n_ps
    f += FLOP_DIR * pc.num_dir_lights
    if pc.ambient_mode == N.PBR_AMBIENT_IBL_DIFFUSE:
        f += FLOP_IBL
    return round(f, 2)


def executed_flops_per_pixel(pc, st: dict, px: int) -> float:
    """FLOP per pixel of the work the pass executed, from its own statistics (pbr_last_pass_stats): the
    per-pixel part for every geometry pixel, 91 / 74 FLOP per point / directional light term the light loops
    evaluated (the wave-balanced lists skip back-facing terms, tiled culling skips out-of-range lights: neither
    is credited), the lists' back-face tests and the culling range tests. Skipped work is never counted."""
    geo = st["geometry_pixels"]
    dir_terms = pc.num_dir_lights * geo
    f = (FLOP_BASE + FLOP_HOIST + (FLOP_IBL if pc.ambient_mode == N.PBR_AMBIENT_IBL_DIFFUSE else 0)) * geo
    f += FLOP_POINT * (st["light_terms"] - dir_terms) + FLOP_DIR * dir_terms
    f += FLOP_BACKFACE_TEST * st["backface_tests"]
    if st["culled"]:
        f += FLOP_RANGE_TEST * (pc.num_point_lights + pc.num_spot_lights) * st["cull_tiles"]
    return round(f / max(px, 1), 2)


def load_pmc(workload: str, head: str, path: str = os.path.join(ROOT, "profiles", "pmc_summary.json")):
    """(HBM bytes per launch, VALU-issue busy fraction, provenance) from the committed rocprofv3 PMC summary of
    this workload (profiles/pmc_summary.json, tools/pmc_summarize.py). The counters are quoted only when the
    summary's kernel_sources_sha -- the stamp of the library the profiled process loaded -- equals `head`, the stamp of
    the library this process loaded (pbr_build_info); otherwise (a kernel changed since the profile, or an unstamped
    profile) they are None and the provenance says so."""
    try:
        with open(path) as f:
            e = json.load(f).get(workload)
    except (OSError, ValueError):
        e = None
    if e is None:
        return None, None, {"profile": None, "kernel_sources_sha": head}
    prov = {"profile": e.get("source"), "profile_kernel_sources_sha": e.get("kernel_sources_sha"),
            "kernel_sources_sha": head, "profile_revision": e.get("kernel_revision")}
    # The profiled box's own kernel time (rocprofv3 kernel trace, mean over the profiled run's timed launches): counter
    # ratios transfer between boxes, durations do not, so the line shows which box its traffic figure came from.
    kt = e.get("kernel_trace") or {}
    if kt.get("mean_ms_timed_steps") is not None:
        prov["profile_kernel_mean_ms"] = round(float(kt["mean_ms_timed_steps"]), 4)
    if e.get("kernel_sources_sha") != head:
        prov["stale"] = True
        return None, None, prov
    try:
        busy = e.get("valu_issue_busy")
        return float(e["hbm_bytes_per_launch"]), (None if busy is None else round(float(busy), 3)), prov
    except (KeyError, TypeError, ValueError):
        return None, None, prov


def roofline_block(fpp, fpp_exec, bpp, bpp_read, px, avg_kernel_s, median_kernel_ms, traffic, valu_busy, pmc_prov,
                   kernel_name, stats) -> dict:
    """The line's `roofline` object for the dominant kernel (one launch = one pass over `px` pixels).

    At 64 lights the arithmetic intensity (fpp / bpp ~ 93 FLOP/B) is 5x the ridge point, so the FP32 vector (VALU) roof
    bounds the kernel: 157.3 TF (MI355X_MICROARCH.md). There is no matrix op on this path: `bound` keeps the
    contract's vocabulary ("mfma" = the compute roof, "hbm") and `bound_unit` names the unit that roof really is
    ("valu" or "hbm"). `frac` comes from this run's HIP events; `frac_profile` from the committed profile's kernel-trace
    mean (pmc.profile_kernel_mean_ms, the box the traffic counters came from), and `launch_vs_profile` is this run's
    mean launch over that one: boxes of this pool differ by up to ~5% for one build."""
    compute_bound = fpp / bpp > FP32_PEAK_TFLOPS * 1e12 / (HBM_PEAK_GBPS * 1e9)
    achieved = bpp * px / avg_kernel_s / 1e9
    hbm = {"achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBPS, 5),
           "bytes_per_px": bpp, "bytes_per_px_read": bpp_read,
           "achieved_read": round(bpp_read * px / avg_kernel_s / 1e9, 2)}
    tflops = fpp * px / avg_kernel_s / 1e12
    tflops_exec = fpp_exec * px / avg_kernel_s / 1e12
    prof_ms = (pmc_prov or {}).get("profile_kernel_mean_ms")
    quoted = prof_ms is not None and not (pmc_prov or {}).get("stale")
    frac_profile = None
    if quoted:
        frac_profile = (round(fpp * px / (prof_ms / 1e3) / 1e12 / FP32_PEAK_TFLOPS, 4) if compute_bound else
                        round(bpp * px / (prof_ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 5))
    return {
        "bound": "mfma" if compute_bound else "hbm",
        "bound_unit": "valu" if compute_bound else "hbm",
        "achieved": round(tflops, 3) if compute_bound else hbm["achieved"],
        "peak": FP32_PEAK_TFLOPS if compute_bound else HBM_PEAK_GBPS,
        "unit": "TFLOP/s" if compute_bound else "GB/s",
        "frac": round(tflops / FP32_PEAK_TFLOPS, 4) if compute_bound else hbm["frac"],
        "frac_profile": frac_profile,
        "launch_vs_profile": round(avg_kernel_s * 1e3 / prof_ms, 4) if quoted else None,
        "traffic": traffic,
        "compute_unit": "valu (fp32 vector ALU; no MFMA on this path)" if compute_bound else None,
        "kernel": kernel_name, "avg_launch_ms": round(avg_kernel_s * 1e3, 4),
        "median_launch_ms": round(median_kernel_ms, 4),
        "flop_per_px": fpp, "bytes_per_px": bpp, "bytes_per_px_read": bpp_read, "px_per_launch": px,
        "executed_flop_per_px": fpp_exec,
        "achieved_executed": round(tflops_exec, 3),
        "frac_executed": round(tflops_exec / FP32_PEAK_TFLOPS, 4),
        "pass_stats": {k: stats[k] for k in ("geometry_pixels", "light_terms", "backface_tests",
                                             "cull_tiles", "exact_pixels")},
        "hbm": hbm,
        "valu_issue_busy": valu_busy,
        "pmc": pmc_prov,
        "note": ("bound: the contract's vocabulary ('mfma' = the compute roof); bound_unit: the unit that roof is -- "
                 "the FP32 vector ALU (VALU, 157.3 TF packed; no matrix op on this path); frac / achieved count SURVEY "
                 "8(d)'s algorithmic-model FLOPs (every light for every pixel, which the kernel does not all evaluate) "
                 "over this run's HIP-event launch mean; frac_profile the same over the committed profile's kernel-trace "
                 "mean (pmc.profile_kernel_mean_ms; launch_vs_profile = this box / the profiled box); frac_executed / "
                 "achieved_executed are the utilisation figure: only the terms the kernel evaluated (pass_stats: "
                 "back-facing terms skipped by the wave-balanced lists and culled lights are not credited; the "
                 "lists' back-face tests are); kernel = pbr_last_pass_kernel; traffic = rocprofv3 "
                 "FETCH_SIZE x2 + WRITE_SIZE bytes per launch and valu_issue_busy = SQ_ACTIVE_INST_VALU over "
                 "kernel cycles, from profiles/pmc_summary.json, quoted only when its kernel_sources_sha "
                 "equals this build's (pmc)"),
    }


def host_cpu_budget() -> dict:
    """The host cores this process may use: the affinity mask, the whole machine (os.cpu_count), and the
    cgroup CPU quota (cpu.max, in CPUs) when one caps the container below its affinity. `used` = the
    threads the CPU baseline runs: the affinity count, capped by the quota (threads beyond the quota
    would only be throttled)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    used = aff if quota is None else max(1, min(aff, int(quota)))
    return {"affinity": aff, "os_cpu_count": os.cpu_count(), "cgroup_cpu_quota": quota, "used": used}


def oracle_pass_of(pc):
    from oracle import oracle as O  # test infrastructure: the checker / CPU baseline only

    return O.OraclePass(eye=tuple(pc.eye_pos_w), ambient=tuple(pc.ambient_light), fresnel_r0=tuple(pc.fresnel_r0),
                        opacity=pc.opacity, n_dir=pc.num_dir_lights, n_point=pc.num_point_lights,
                        n_spot=pc.num_spot_lights, ambient_mode=pc.ambient_mode,
                        use_f0_plane=bool(pc.flags & N.PBR_FLAG_F0_PLANE),
                        apply_ao=bool(pc.flags & N.PBR_FLAG_APPLY_AO))


def cpu_shade(planes, pc, env, threads: int, use_ref: bool, rgba8: bool):
    """The CPU shader path over (15, rows, W) host planes in the bench's output format: the reference's own
    shader text built for the host (oracle/_ref, one row band per thread; ctypes releases the GIL) or the C
    restatement (oracle/pbr_oracle.c, pthreads)."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle as O  # test infrastructure: the checker / CPU baseline only

    ops, lights = oracle_pass_of(pc), pc.light_array()
    fmt = O.OUTPUT_RGBA8 if rgba8 else O.OUTPUT_RGBA32F
    if not use_ref:
        return O.shade_frame(list(planes), ops, lights, env, None, None, fmt, n_threads=threads)
    edges = np.linspace(0, planes.shape[1], threads + 1).astype(int)
    bands = [np.ascontiguousarray(planes[:, a:b]) for a, b in zip(edges[:-1], edges[1:]) if b > a]
    with ThreadPoolExecutor(len(bands)) as ex:
        parts = ex.map(lambda b: O.shade_frame_ref(list(b), ops, lights, env, None, None, fmt), bands)
        return np.concatenate(list(parts), axis=0)


def parity_of(got, ref, rgba8: bool) -> dict:
    """fp32: max relative error per channel (NaN == NaN) and the bit-identical fraction; RGBA8: the largest
    code difference and the identical fraction (a 1e-5 relative difference can move a code by one where
    c * 255 + 0.5 sits on an integer)."""
    from oracle import oracle as O  # test infrastructure: the checker only

    if rgba8:
        d = np.abs(got.astype(np.int32) - ref.astype(np.int32))
        return {"parity_max_code_diff": int(d.max()) if d.size else 0,
                "parity_bit_exact_frac": round(float((d == 0).mean()) if d.size else 1.0, 6)}
    return {"parity_max_rel": float(O.rel_err(got, ref).max()) if got.size else 0.0,
            "parity_bit_exact_frac": round(float(O.bit_equal(got, ref).mean()) if got.size else 1.0, 6)}


def parity_failures(line: dict) -> list:
    """Every parity result in a bench line that misses the north-star bar: the CPU leg's frame check
    (parity_max_rel / parity_max_code_diff; a NaN where the reference has none, or the reverse, is an infinite
    relative error), the exact leg's, the assembled frame's at N > 1 and its band checksums. Empty = all pass."""
    bad = []

    def check(where: str, p: dict):
        rel, code = p.get("parity_max_rel"), p.get("parity_max_code_diff")
        if rel is not None and not rel <= PARITY_REL_TOL:  # NaN-safe: NaN or inf fails
            bad.append(f"{where}parity_max_rel {rel} > {PARITY_REL_TOL}")
        if code is not None and not code <= PARITY_RGBA8_CODE_TOL:
            bad.append(f"{where}parity_max_code_diff {code} > {PARITY_RGBA8_CODE_TOL}")

    check("", line)
    if isinstance(line.get("exact_mode"), dict):
        check("exact_mode.", line["exact_mode"])
    if isinstance(line.get("gathered_frame_parity"), dict):
        check("gathered_frame_parity.", line["gathered_frame_parity"])
    if line.get("gather_checksums_match") is False:
        bad.append("gather_checksums_match false")
    return bad


def emit_line(line: dict) -> int:
    """Print the bench line on stdout and return 0 -- unless a parity check in it failed: then the line goes to
    stderr with the failures, nothing is printed on stdout (no throughput is published for a wrong frame) and the
    exit status is EXIT_PARITY."""
    bad = parity_failures(line)
    checked = any(k in line for k in ("parity_max_rel", "parity_max_code_diff", "gathered_frame_parity"))
    line = {**line, "parity_checked": checked, "parity_ok": not bad if checked else None}
    if bad:
        log("PARITY FAILURE: " + "; ".join(bad))
        print(json.dumps({**line, "parity_failures": bad}), file=sys.stderr, flush=True)
        return EXIT_PARITY
    print(json.dumps(line), flush=True)
    return 0


def cpu_baseline(cfg, planes_host, pc, env, gpu_frame, budget_rows: int, kind: str = "auto", rgba8: bool = False):
    """Time the reference CPU shader path on every k-th row of the frame (rank 0, N = 1) and check parity
    there. kind "reference": the reference's own pixel shader (Default.hlsl PS + Core.hlsl + LightingUtil.hlsl)
    compiled as C++ (oracle/_ref, built in the build container; nothing under /root/reference is read at run
    time), one row band per host thread; kind "port": the C restatement oracle/pbr_oracle.c (pthreads). "auto"
    takes the reference build when it is present. Both are test infrastructure, used here only as the CPU
    baseline and the checker. Threads: every core of the affinity mask (capped by a cgroup quota)."""
    from oracle import oracle as O  # test infrastructure: the checker / CPU baseline only

    use_ref = kind == "reference" or (kind == "auto" and O.ref_available())
    budget = host_cpu_budget()
    n_threads = budget["used"]
    step = max(1, cfg.height // budget_rows) if budget_rows > 0 else 1
    sample = np.ascontiguousarray(planes_host[:, ::step])
    t0 = time.perf_counter()
    ref = cpu_shade(sample, pc, env, n_threads, use_ref, rgba8)
    dt = time.perf_counter() - t0
    px = sample.shape[1] * sample.shape[2]
    # single-thread rate on the first 8 sampled rows (single-thread and all-core)
    one = np.ascontiguousarray(sample[:, :8])
    t1 = time.perf_counter()
    cpu_shade(one, pc, env, 1, use_ref, rgba8)
    st = one.shape[1] * one.shape[2] / (time.perf_counter() - t1) / 1e6
    parity = parity_of(gpu_frame[::step], ref, rgba8)
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    what = ("oracle/_ref/libpbr_ref.so: the reference's Default.hlsl PS (+ Core/LightingUtil.hlsl) compiled as "
            f"C++ (g++ -O2 -ffp-contract=off), {n_threads} host threads over row bands" if use_ref else
            f"oracle/pbr_oracle.c, -O2 -ffp-contract=off, {n_threads} pthreads")
    return {
        "value": round(px / dt / 1e6, 4), "unit": "Mpix/s", "cores": n_threads,
        "host_cpus": budget,
        "kind": "reference" if use_ref else "port",
        "cpu_model": model,
        "single_thread_value": round(st, 4),
        "sample": (f"every {step}th row of" if step > 1 else "all rows of") +
                  f" the same {cfg.width}x{cfg.height} frame ({px} px, {dt:.2f} s wall), {what}",
    }, parity, (step, ref)


def gathered_parity(cfg, pc, env, frame: np.ndarray, world: int, rows_per_band: int, rgba8: bool) -> dict:
    """Rank 0 at N > 1: the assembled frame against the CPU oracle on `rows_per_band` rows of every rank's
    band (spread over the band; the G-buffer rows are refilled on the host, the fill being a function of
    the global pixel). Untimed."""
    from oracle import oracle as O  # test infrastructure: the checker only

    rows = []
    for r in range(world):
        b = D.band_rows(cfg.height, world, r)
        rows += sorted({b.row_begin + (k * b.rows) // rows_per_band for k in range(rows_per_band)} if b.rows else [])
    planes = np.concatenate([S.fill_gbuffer_host(cfg, y, y + 1)[0] for y in rows], axis=1)
    ref = cpu_shade(planes, pc, env, host_cpu_budget()["used"], O.ref_available(), rgba8)
    return {"rows_checked": len(rows), **parity_of(frame[rows], ref, rgba8)}


def time_exact_mode(ctx, pc, gb, out, stream, args, fmt, rgba8, px):
    """The same pass with PBR_FLAG_FAITHFUL cleared (correctly rounded, bit-identical to the oracle), timed
    like the headline: warm-up, then K launches between synchronisations with HIP events around each.
    Leaves the exact-mode frame in `out`."""
    from physically_based_renderer_amd.renderer import PassConstants

    ctx.set_pass(PassConstants(**{**pc.__dict__, "flags": int(pc.flags) & ~N.PBR_FLAG_FAITHFUL}))

    def one():
        if rgba8:
            ctx.shade_frame(gb, out, fmt=fmt, stream=stream)
        else:
            ctx.shade(gb, out, stream)

    for _ in range(max(args.warmup, 3)):
        one()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for a, b in ev:
        a.record(stream)
        one()
        b.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ms = [a.elapsed_time(b) for a, b in ev]
    ctx.set_pass(pc)
    return {"value": round(px * args.steps / wall / 1e6, 2), "ms_per_step": round(wall / args.steps * 1e3, 4),
            "avg_launch_ms": round(float(np.mean(ms)), 4), "median_launch_ms": round(float(np.median(ms)), 4)}


def make_workload(cfg, band, mode: str, device, apply_ao: bool = False):
    """The pass constants, env map and resident G-buffer rows of `band` of frame `cfg` (host fill into
    pinned staging, one upload). Returns (pc, env, staging, gb, fill_s, (first_upload_s, warm_upload_s)).
    The first upload of the process pays the device allocation and the first DMA use of the pinned pages
    (tools/h2d_probe.py, profiles/r04/h2d_probe.log: ~5 GB/s); the same copy again into the resident buffer
    runs at the link rate (~57 GB/s), which is what a frame loop re-uploading its G-buffer would see."""
    from physically_based_renderer_amd.renderer import GBuffer

    t0 = time.perf_counter()
    pc = S.scene_pass(cfg)
    if mode == "faithful":
        pc.flags = int(pc.flags) | N.PBR_FLAG_FAITHFUL
    if apply_ao:  # the AO extension (ambient *= AO, PBR_FLAG_APPLY_AO): the kernel reads the AO plane too
        pc.flags = int(pc.flags) | N.PBR_FLAG_APPLY_AO
    env = S.env_map() if pc.ambient_mode == N.PBR_AMBIENT_IBL_DIFFUSE else None
    staging = torch.empty((N.NUM_PLANES, band.rows, cfg.width), dtype=torch.float32, pin_memory=True)
    S.fill_gbuffer_host(cfg, band.row_begin, band.row_end, out=staging.numpy())
    t_fill = time.perf_counter() - t0
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    planes_dev = staging.to(device, non_blocking=True)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    planes_dev.copy_(staging, non_blocking=True)
    torch.cuda.synchronize()
    return pc, env, staging, GBuffer(planes_dev), t_fill, (t2 - t1, time.perf_counter() - t2)


def shade_steps(shade_into, outs, stream, warmup: int, steps: int, gather=None, in_group=False):
    """W untimed warm-up steps, then exactly K timed steps between barrier + synchronize on both sides. A
    step shades into one of two output slots; with `gather`, the slot is then gathered to rank 0 (pipelined:
    the gather of frame k overlaps the shading of frame k + 1; a slot is reused only after its gather).
    Each shading launch is bracketed by HIP events on the launch stream. Returns (wall s, [launch ms])."""
    pending = [[], []]

    def step(k: int, ev=None):
        slot = k % 2
        D.BandGather.wait(pending[slot])  # the gather that last read this slot (stream-side wait)
        if ev is not None:
            ev[0].record(stream)
        shade_into(outs[slot])
        if ev is not None:
            ev[1].record(stream)
        if gather is not None:
            pending[slot] = gather.start(outs[slot])

    for k in range(warmup):
        step(k)
    for p in pending:
        D.BandGather.wait(p)
    pending = [[], []]
    torch.cuda.synchronize()
    if in_group:
        dist.barrier()
    torch.cuda.synchronize()
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t_start = time.perf_counter()
    for k in range(steps):
        step(k, events[k])
    for p in pending:
        D.BandGather.wait(p)
    torch.cuda.synchronize()
    if in_group:
        dist.barrier()
    torch.cuda.synchronize()
    return time.perf_counter() - t_start, [a.elapsed_time(b) for a, b in events]


def clock_ramp(shade_into, out, ramp_ms: float) -> dict:
    """Untimed back-to-back shading passes for `ramp_ms` (synchronised every 8 launches), so that timed steps run
    at settled GPU clocks (the kernel trace shows the clock ramping over the first ~40 ms of launches). Not a step."""
    t0 = time.perf_counter()
    n = 0
    while ramp_ms > 0:
        shade_into(out)
        n += 1
        if n % 8 == 0:
            torch.cuda.synchronize()
            if time.perf_counter() - t0 >= ramp_ms / 1e3:
                break
    return {"ms": round((time.perf_counter() - t0) * 1e3, 1), "launches": n}


def band_anchor(ctx, args, world: int, device, stream, resident=None) -> dict:
    """The scaling anchor: ONE rank's config-5 band (8192 x rows_per_rank, RGBA8, the run's mode) shaded alone
    -- no gather, no other rank -- timed like a step. It is the per-GPU work of every point of the 1/2/4/8-GPU
    curve, so `efficiency_vs_anchor` = (value / N) / anchor compares identical per-rank geometry. At N > 1 the
    rank's own resident band (`resident` = (gb, outs)); at N = 1 (headline config 3) the band is built here."""
    rows = args.rows_per_rank
    cfg5 = S.CONFIGS[5].with_size(8192, rows * world)
    if resident is None:
        pc5, env5, _, gb, _, _ = make_workload(cfg5, D.band_rows(rows, 1, 0), args.mode, device)
        ctx.set_pass(pc5, stream)
        if env5 is not None:
            ctx.set_env_map(env5, stream)
        outs = [torch.empty((rows, cfg5.width, 4), dtype=torch.uint8, device=device) for _ in range(2)]
    else:
        gb, outs = resident

    def shade_into(o):
        ctx.shade_frame(gb, o, fmt=N.PBR_OUTPUT_RGBA8_UNORM, stream=stream)

    # The same clock ramp as the headline before the warm-up: the anchor is timed at settled clocks like every
    # point of the curve it anchors (measured cold, it read 6% low and overstated efficiency_vs_anchor).
    ramp = clock_ramp(shade_into, outs[0], args.ramp_ms)
    wall, ms = shade_steps(shade_into, outs, stream, max(args.warmup, 3), args.steps)
    px = cfg5.width * rows
    return {"workload": f"{cfg5.name}_band{rows}", "output": "rgba8", "mode": args.mode, "px_per_step": px,
            "value": round(px * args.steps / wall / 1e6, 2), "ms_per_step": round(wall / args.steps * 1e3, 4),
            "shade_ms": round(float(np.mean(ms)), 4), "clock_ramp": ramp}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--ramp-ms", type=float, default=200.0,
                    help="untimed back-to-back shading before the warm-up steps, so the timed steps run at "
                         "settled GPU clocks (DVFS: the first ~40 ms of launches run 2.05 -> 1.75 ms, "
                         "profiles/r01 kernel trace); not a step, no gather")
    ap.add_argument("--config", type=int, default=0, help="BASELINE config id (default 3 at N=1, 5 at N>1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-anchor", action="store_true",
                    help="skip the scaling anchor (one rank's config-5 band shaded alone, scale_anchor)")
    ap.add_argument("--rows-per-rank", type=int, default=1024,
                    help="config 5 band height per rank (1024 = the BASELINE geometry: 8192x8192 at N = 8; "
                         "smaller only for rehearsing the multi-rank path). The same band at every N, N = 1 "
                         "included, so per-GPU work is identical across the scaling curve")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (the benchmark); gloo = host-staged gather, for exercising the "
                         "multi-rank path on one GPU")
    ap.add_argument("--output", default="auto", choices=["auto", "rgba32f", "rgba8"],
                    help="output format: fp32 RGBA or the reference's R8G8B8A8_UNORM back buffer (fused conversion). "
                         "auto = rgba32f for the single-GPU configs 1-4 (the frame the parity check reads), rgba8 "
                         "for config 5 at every N (the presented frame rank 0 assembles; an fp32 band is 134 MB "
                         "per xGMI link per frame, longer than the band's shading, DESIGN.md section 7). "
                         "--output rgba32f with config 5 gathers fp32 and checks the assembled frame against the "
                         "oracle")
    ap.add_argument("--mode", default="faithful", choices=["exact", "faithful"],
                    help="faithful (default) = PBR_FLAG_FAITHFUL: hardware reciprocals (<= 1 ulp; D3D allows 2.5 ulp "
                         "for fp32 division) in the well-conditioned BRDF divisions, exact GGX/Fresnel chain, within "
                         "the north-star 1e-5 (measured in the line: parity_max_rel); exact = correctly rounded "
                         "reference semantics, bit-identical to the oracle.")
    ap.add_argument("--exact-leg", action="store_true",
                    help="N = 1, faithful mode: also time the exact mode on the same G-buffer and report it as exact_mode "
                         "(off by default so that a kernel trace of the default command holds only the headline launches)")
    ap.add_argument("--cpu-kind", default="auto", choices=["auto", "reference", "port"],
                    help="CPU baseline: the reference's own shader source compiled for the host (oracle/_ref) or the "
                         "C restatement (oracle/pbr_oracle.c); auto = the reference build when present")
    ap.add_argument("--cpu-rows", type=int, default=0,
                    help="rows in the CPU-baseline sample (0 = the whole frame or band)")
    ap.add_argument("--inject-parity-breach", type=float, default=0.0, metavar="REL",
                    help="test only: scale one channel of the checked frame by (1 + REL) before the parity check, "
                         "to show that a frame off the 1e-5 bar is refused (exit status 3, no metric line)")
    ap.add_argument("--parity-rows", type=int, default=8,
                    help="N > 1: rows per band of the assembled frame checked against the oracle (0 = none)")
    ap.add_argument("--apply-ao", action="store_true",
                    help="shade with PBR_FLAG_APPLY_AO (ambient *= AO): the north star's G-buffer AO plane is read "
                         "(64 B/px, SURVEY 8(d)'s model); the reference itself never reads its AO slot (SURVEY F4), so "
                         "the default pass does not")
    ap.add_argument("--dev", action="store_true",
                    help="measure a library that is not the product build of this checkout (a variant, a debug or stale "
                         "build, PBR_* overrides): the line is printed with library.problems listed; without --dev such "
                         "a run exits 4 and prints no metric line")
    args = ap.parse_args()

    # Which binary is measured (pbr_build_info): decided before anything runs, on any host.
    library = library_provenance(args.dev)
    if library["problems"] and not args.dev:
        log("REFUSED: the loaded library is not the product build of this checkout: " + "; ".join(library["problems"]))
        log("(rebuild with `make -C physically_based_renderer_amd/csrc`, or pass --dev to measure it anyway)")
        return EXIT_PROVENANCE
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a HIP device")
    n_dev = torch.cuda.device_count()
    local_env = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dist_backend == "nccl" and local_env >= n_dev:
        raise SystemExit(f"LOCAL_RANK {local_env} but only {n_dev} visible GPU(s): RCCL needs one GPU per rank")
    torch.cuda.set_device(local_env % n_dev)
    # Under torch.distributed.run (WORLD_SIZE set) the process group is created at every world size, N = 1
    # included, so the N = 1 line runs the same RCCL init, band gather and checksum collective as N = 8.
    rank, world, local = D.init_from_env(args.dist_backend, always="WORLD_SIZE" in os.environ)
    in_group = dist.is_initialized()
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE {world}; using {world}")
    device = torch.device("cuda", local % n_dev)

    cid = args.config or (3 if world == 1 else 5)
    cfg = S.CONFIGS[cid]
    banded = cid == 5  # BASELINE config 5: row bands of --rows-per-rank rows, gathered to rank 0
    if banded:
        cfg = cfg.with_size(8192, args.rows_per_rank * world)
    band = D.band_rows(cfg.height, world, rank)
    workload = f"{cfg.name}" + (f"_band{args.rows_per_rank}" if banded else "")

    pc, env, staging, gb, t_fill, t_upload = make_workload(cfg, band, args.mode, device, args.apply_ao)
    ctx = ShadingContext(device.index)
    stream = torch.cuda.current_stream(device)
    ctx.set_pass(pc, stream)
    if env is not None:
        ctx.set_env_map(env, stream)
    log(f"rank {rank}/{world}: {workload} rows [{band.row_begin},{band.row_end}) fill {t_fill:.2f}s "
        f"upload {t_upload[0] * 1e3:.1f} ms first ({staging.numel() * 4 / t_upload[0] / 1e9:.1f} GB/s H2D), "
        f"{t_upload[1] * 1e3:.1f} ms again ({staging.numel() * 4 / t_upload[1] / 1e9:.1f} GB/s)"
        + (f", process group {dist.get_backend()}" if in_group else ""))

    output = args.output if args.output != "auto" else ("rgba8" if banded else "rgba32f")
    rgba8 = output == "rgba8"
    out_dtype = torch.uint8 if rgba8 else torch.float32
    fmt = N.PBR_OUTPUT_RGBA8_UNORM if rgba8 else N.PBR_OUTPUT_RGBA32F
    outs = [torch.empty((band.rows_max, cfg.width, 4), dtype=out_dtype, device=device) for _ in range(2)]
    gather = D.BandGather(band, cfg.width, device, dtype=out_dtype) if banded else None

    def shade_into(o):
        if rgba8:
            ctx.shade_frame(gb, o, fmt=fmt, stream=stream)
        else:
            ctx.shade(gb, o, stream)

    # GPU clock ramp (see --ramp-ms): full shading passes, untimed, before the W warm-up steps.
    ramp = clock_ramp(shade_into, outs[0], args.ramp_ms)
    elapsed, kernel_ms = shade_steps(shade_into, outs, stream, args.warmup, args.steps, gather, in_group)

    # The executed work of the last timed pass (pbr_last_pass_stats; every timed pass shades the same input).
    stats = ctx.pass_stats(stream)
    kernel_name = ctx.last_kernel(stream)
    cull_note = {}
    if pc.flags & N.PBR_FLAG_TILED_CULLING:
        cull_note = {"lights_per_tile": round(stats["cull_tile_lights"] / max(stats["cull_tiles"], 1), 3),
                     "tiles": stats["cull_tiles"]}

    coll_dev = device if args.dist_backend == "nccl" else torch.device("cpu")
    gather_note = {}
    if gather is not None:
        # The gather alone (no shading), timed the same way: the exchange cost the pipelined step hides.
        torch.cuda.synchronize()
        if in_group:
            dist.barrier()
        tg = time.perf_counter()
        for k in range(args.steps):
            D.BandGather.wait(gather.start(outs[k % 2]))
        torch.cuda.synchronize()
        if in_group:
            dist.barrier()
        gather_ms = (time.perf_counter() - tg) / args.steps * 1e3
        # Property check of the assembled image: each rank's band checksum (int64 sum of the 32-bit words,
        # exact) must equal the checksum of the slot rank 0 received -- an all_gather on the device (RCCL).
        last = outs[(args.steps - 1) % 2][: band.rows].contiguous()
        mine = last.view(torch.int32).to(torch.int64).sum().reshape(1).to(coll_dev)
        sums = [torch.zeros(1, dtype=torch.int64, device=coll_dev) for _ in range(world)]
        if in_group:
            dist.all_gather(sums, mine)
        else:
            sums = [mine]
        gather_ok = None
        if rank == 0:
            got = [gather.frame[r, : D.band_rows(cfg.height, world, r).rows].contiguous().view(torch.int32)
                   .to(torch.int64).sum() for r in range(world)]
            gather_ok = all(int(g.item()) == int(s_.item()) for g, s_ in zip(got, sums))
        gather_note = {
            "gather": ("batched isend/irecv star to rank 0 (RCCL over xGMI), pipelined with the next frame"
                       if in_group and args.dist_backend == "nccl" else
                       "host-staged gloo gather (test mode)" if in_group else "rank 0's own band: device copy"),
            "process_group": dist.get_backend() if in_group else None,
            "gather_checksums_match": gather_ok, "gather_ms": round(gather_ms, 4),
            "shade_ms": round(float(np.mean(kernel_ms)), 4)}

    el = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
    if in_group and world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    total_px = cfg.width * cfg.height
    value = total_px * args.steps / elapsed / 1e6

    if rank == 0:
        avg_kernel_s = float(np.mean(kernel_ms)) / 1e3
        median_kernel_ms = float(np.median(kernel_ms))
        band_px = cfg.width * band.rows
        bpp = bytes_per_pixel(pc, 4 if rgba8 else 16)
        bpp_read = bytes_read_per_pixel(pc, 4 if rgba8 else 16)
        achieved_read = bpp_read * band_px / avg_kernel_s / 1e9  # the bytes the kernel moves (hbm_gbps)
        achieved_model = bpp * band_px / avg_kernel_s / 1e9  # SURVEY 8(d)'s model (roofline.hbm.achieved)
        traffic, valu_busy, pmc_prov = load_pmc(workload + ("_ao" if pc.flags & N.PBR_FLAG_APPLY_AO else "")
                                                + ("_rgba8" if rgba8 and not banded else "")
                                                + ("_faithful" if args.mode == "faithful" else ""),
                                                library["sources_sha"])
        tile_px = 256 if os.environ.get("PBR_PIXELS_PER_THREAD") == "1" else 128  # culling unit: 32x8 / 64x2
        fpp = flops_per_pixel(pc, cull_note.get("lights_per_tile"), tile_px)
        fpp_exec = executed_flops_per_pixel(pc, stats, band_px)
        roofline = roofline_block(fpp, fpp_exec, bpp, bpp_read, band_px, avg_kernel_s, median_kernel_ms, traffic,
                                  valu_busy, pmc_prov, kernel_name, stats)
        cpu = None
        parity = {}
        exact_leg = None
        frame = outs[0][: band.rows].cpu().numpy() if world == 1 else None  # the timed mode's frame
        if frame is not None and args.inject_parity_breach:  # test only: the largest channel, scaled
            frame = frame.copy()
            flat = frame.reshape(-1)
            k = int(np.argmax(np.where(np.isfinite(flat), np.abs(flat.astype(np.float64)), 0.0)))
            flat[k] = flat[k] * (1.0 + args.inject_parity_breach) if not rgba8 else (int(flat[k]) + 2) % 256
        exact_frame = None
        assembled = gather.assembled(cfg.height).cpu().numpy() if world > 1 and gather is not None else None
        # The scaling anchor runs right after the timed steps, on a warm GPU, before the host-side legs (the CPU
        # baseline and the parity checks leave the GPU idle for seconds); it ramps the clock itself as well.
        scale = {}
        if not args.no_anchor:
            anchor = band_anchor(ctx, args, world, device, stream, (gb, outs) if banded and rgba8 else None)
            scale = {"scale_anchor": anchor}
            if world > 1:
                per_rank = value / world
                scale.update({"per_rank_mpix_s": round(per_rank, 2),
                              "efficiency_vs_anchor": round(per_rank / anchor["value"], 4)})
            ctx.set_pass(pc, stream)  # the anchor set its own pass (config 5 geometry, same lights and mode)
            if env is not None:
                ctx.set_env_map(env, stream)
        if world == 1 and args.mode == "faithful" and args.exact_leg:
            exact_leg = time_exact_mode(ctx, pc, gb, outs[0], stream, args, fmt, rgba8, band_px)
            exact_frame = outs[0][: band.rows].cpu().numpy()
        if world == 1 and not args.no_cpu_baseline:
            cpu, parity, (step_, ref) = cpu_baseline(cfg, staging.numpy(), pc, env, frame, args.cpu_rows,
                                                    args.cpu_kind, rgba8)
            if exact_frame is not None:
                exact_leg.update(parity_of(exact_frame[::step_], ref, rgba8))
        elif world > 1 and assembled is not None and args.parity_rows > 0:
            parity = {"gathered_frame_parity": gathered_parity(cfg, pc, env, assembled, world, args.parity_rows,
                                                               rgba8)}
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "Mpix/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "clock_ramp": ramp,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "output": output, "mode": args.mode,
            "library": library,
            "data": "synthetic deterministic G-buffer (splitmix64 per pixel; rustediron metal/rough tiles; "
                    "Chelsea_Stairs 16-bit env)",
            "config": {"workload": workload, "width": cfg.width, "height": cfg.height,
                       "rows_per_rank": band.rows, "point_lights": pc.num_point_lights,
                       "ambient": "ibl_diffuse" if pc.ambient_mode else "constant",
                       "tiled_culling": bool(pc.flags & N.PBR_FLAG_TILED_CULLING),
                       "apply_ao": bool(pc.flags & N.PBR_FLAG_APPLY_AO),
                       "parallelism": f"row-bands x{world}"},
            # HBM GB/s of the headline metric: the bytes the kernel itself reads and writes per launch (the 11 planes
            # it reads + the RGBA write) over the HIP-event launch mean; hbm_gbps_model counts SURVEY 8(d)'s 12-plane
            # model (with the AO plane the default pass never reads) -- the roofline.hbm figure
            "hbm_gbps": round(achieved_read, 2),
            "hbm_gbps_model": round(achieved_model, 2),
            "roofline": roofline,
            "cpu_baseline": cpu,
            **parity, **gather_note, **cull_note, **scale,
            **({"exact_mode": exact_leg} if exact_leg is not None else {}),
            # pinned staging -> HBM: pcie_h2d_gbps = the copy repeated into the resident buffer (the
            # link rate; this key's meaning in round 4 and from round 6); pcie_h2d_first_gbps = the process's first
            # copy (device allocation + first DMA use of the pinned pages). Line schema 6 (line_schema).
            "pcie_h2d_gbps": round(staging.numel() * 4 / t_upload[1] / 1e9, 2),
            "pcie_h2d_first_gbps": round(staging.numel() * 4 / t_upload[0] / 1e9, 2),
            "line_schema": LINE_SCHEMA,
        }
        rc = emit_line(out)
    else:
        rc = 0
    ctx.close()
    if in_group:
        dist.destroy_process_group()
    return rc


if __name__ == "__main__":
    sys.exit(main())
