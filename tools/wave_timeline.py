"""Per-wave timeline of the pair kernel (development tool): when each wave starts, when its G-buffer pair
arrives, how long its light loops and finish take, and how full every SIMD is over the launch.

Needs a library built with -DPBR_WAVE_TIMELINE=1, passed as PBR_LIB_PATH:
    make -C physically_based_renderer_amd/csrc OUTDIR=$PWD/build/tl OBJDIR=$PWD/build/tl/obj EXTRA=-DPBR_WAVE_TIMELINE=1
    PBR_LIB_PATH=build/tl/libpbrshade.so python tools/wave_timeline.py --config 2 [--mode faithful] [--json out]

Stamps (shade_kernels.hip, PBR_WAVE_TIMELINE): s_memrealtime (100 MHz, chip-wide) at entry, when the pair's
planes have arrived (s_waitcnt vmcnt(0) in the debug build), at the start and end of the light loops and after
the stores are issued; HW_ID / XCC_ID name the SIMD and wave slot.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

TICK_NS = 10.0  # s_memrealtime: 100 MHz


def block_idle(tl: np.ndarray, waves_per_block: int = 4) -> dict:
    """Multi-wave workgroups (the tile kernel: 4 waves, one per SIMD; row = block * 4 + wave): a workgroup's LDS is
    released when its last wave ends, and with LDS-limited occupancy no new workgroup starts on the CU before that,
    so each wave's slot idles from its own end to its workgroup's last end. Returns that idle time as a fraction of
    the waves' lifetimes, and the spread of the waves' lifetimes inside a workgroup."""
    n = (len(tl) // waves_per_block) * waves_per_block
    t = tl[:n, 1:6].astype(np.int64).reshape(-1, waves_per_block, 5)
    ok = (t[:, :, 0] != 0).all(axis=1)
    t = t[ok] * TICK_NS / 1e3
    entry, done = t[:, :, 0], t[:, :, 4]
    life = done - entry
    idle = done.max(axis=1, keepdims=True) - done
    return {"blocks": int(ok.sum()), "idle_over_life": round(float(idle.sum() / life.sum()), 4),
            "idle_us_mean_per_wave": round(float(idle.mean()), 3),
            "life_spread_in_block_us_mean": round(float((life.max(axis=1) - life.min(axis=1)).mean()), 3),
            "entry_spread_in_block_us_mean": round(float((entry.max(axis=1) - entry.min(axis=1)).mean()), 3)}


def analyse(tl: np.ndarray, name: str) -> dict:
    """tl: (waves, 8) uint64 stamps of one launch (rows of waves that never ran are zero)."""
    blk = block_idle(tl)
    tl = tl[tl[:, 1] != 0]
    hw, xcc = (tl[:, 0] & 0xFFFFFFFF).astype(np.int64), ((tl[:, 0] >> 32) & 0xFFFF).astype(np.int64)
    flags = (tl[:, 0] >> 48).astype(np.int64)  # shade_lean_kernel: 1 = pixels re-passed, 2 = not a faithful wave
    t = tl[:, 1:6].astype(np.int64)
    t0 = t[:, 0].min()
    t = (t - t0) * TICK_NS / 1e3  # us from the first wave's entry
    entry, loaded, loop0, loop1, done = t.T
    cyc = (tl[:, 7].astype(np.int64) - tl[:, 6].astype(np.int64))
    simd = xcc * 4096 + ((hw >> 4) & 0xFFF)  # simd, pipe, cu, sh, se within the XCD
    end = done.max()
    n_simd = len(np.unique(simd))
    life = done - entry
    # residency: waves resident per SIMD averaged over the launch
    resid = life.sum() / (n_simd * end)
    # per SIMD, sorted by entry: the gap from a wave's end to the next wave starting in the same slot
    slot = simd * 16 + (hw & 0xF)
    order = np.lexsort((entry, slot))
    s_sorted, e_sorted, d_sorted = slot[order], entry[order], done[order]
    same = s_sorted[1:] == s_sorted[:-1]
    gaps = (e_sorted[1:] - d_sorted[:-1])[same]
    # first-round dispatch: entries in the first 1.5 x (median life) window
    bins = np.arange(0, end + 1.0, 1.0)
    phase = {k: np.zeros(len(bins) - 1) for k in ("load", "pre", "loop", "finish")}
    for k, (a, b) in {"load": (entry, loaded), "pre": (loaded, loop0), "loop": (loop0, loop1),
                      "finish": (loop1, done)}.items():
        # time-weighted count of waves in the phase per 1-us bin
        lo, hi = np.clip(a, 0, end), np.clip(b, 0, end)
        for i in range(len(bins) - 1):
            phase[k][i] = np.clip(np.minimum(hi, bins[i + 1]) - np.maximum(lo, bins[i]), 0, None).sum()
    waves_per_simd = np.bincount(np.unique(simd, return_inverse=True)[1])
    out = {
        "workload": name, "waves": int(len(tl)), "simds": int(n_simd), "launch_us": round(float(end), 2),
        "block_idle": blk,
        "waves_per_simd": {"mean": round(float(waves_per_simd.mean()), 2), "min": int(waves_per_simd.min()),
                           "max": int(waves_per_simd.max())},
        "mean_resident_waves_per_simd": round(float(resid), 3),
        "wave_life_us": {"mean": round(float(life.mean()), 3), "p10": round(float(np.percentile(life, 10)), 3),
                         "p90": round(float(np.percentile(life, 90)), 3)},
        "wave_cycles_mean": round(float(cyc.mean()), 0),
        "phase_us_mean": {"load": round(float((loaded - entry).mean()), 3),
                          "pre_loop": round(float((loop0 - loaded).mean()), 3),
                          "loop": round(float((loop1 - loop0).mean()), 3),
                          "finish": round(float((done - loop1).mean()), 3)},
        "slot_refill_gap_us": {"mean": round(float(gaps.mean()), 3) if gaps.size else None,
                               "p90": round(float(np.percentile(gaps, 90)), 3) if gaps.size else None},
        "last_entry_us": round(float(entry.max()), 2),
        "first_round_entries_within_us": round(float(np.sort(entry)[min(len(entry) - 1, 4 * n_simd - 1)]), 3),
        "wave_life_max_us": round(float(life.max()), 3),
        # the waves that end last: when they entered and how long they lived
        "last_to_end": [{"entry_us": round(float(entry[i]), 2), "life_us": round(float(life[i]), 2),
                         "loop_us": round(float(loop1[i] - loop0[i]), 2), "after_loop_us": round(float(done[i] - loop1[i]), 2),
                         "flags": int(flags[i])} for i in np.argsort(done)[-8:]],
        "flagged": {str(f): {"waves": int((flags == f).sum()), "life_us_mean": round(float(life[flags == f].mean()), 2),
                             "after_loop_us_mean": round(float((done - loop1)[flags == f].mean()), 2)}
                    for f in np.unique(flags)},
        # chip-wide: waves per SIMD in each phase, per 1-us bin
        "timeline_per_simd": {k: [round(float(v) / n_simd, 2) for v in phase[k]] for k in phase},
    }
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--mode", default="faithful", choices=["faithful", "exact"])
    ap.add_argument("--ramp-ms", type=float, default=300.0, help="untimed back-to-back launches first (clock ramp)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import torch

    from clock_ramp import clock_ramp
    from physically_based_renderer_amd import _native as N
    from physically_based_renderer_amd import scenes as S
    from physically_based_renderer_amd.renderer import GBuffer, ShadingContext

    cfg = S.CONFIGS[a.config]
    planes, _ = S.fill_gbuffer_host(cfg)
    pc = S.scene_pass(cfg)
    if a.mode == "faithful":
        pc.flags = int(pc.flags) | N.PBR_FLAG_FAITHFUL
    dev = torch.device("cuda", 0)
    gb = GBuffer.from_host(planes, dev)
    out = torch.empty((cfg.height, cfg.width, 4), device=dev)
    lib = N.lib()
    f = lib.pbr_debug_wave_timeline
    f.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    waves = ((cfg.width + 63) // 64) * ((cfg.height + 7) // 8) * 4
    buf = torch.zeros((waves, 8), dtype=torch.int64, device=dev)
    res = {}
    with ShadingContext(0) as ctx:
        ctx.set_pass(pc)
        if pc.ambient_mode:
            ctx.set_env_map(S.env_map())
        assert f(buf.data_ptr(), waves) == 0, "library not built with PBR_WAVE_TIMELINE"
        clock_ramp(ctx, gb, out, a.ramp_ms)
        torch.cuda.synchronize()
        buf.zero_()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        ctx.shade(gb, out)
        ev[1].record()
        torch.cuda.synchronize()
        assert f(None, 0) == 0
        res = analyse(buf.cpu().numpy().view(np.uint64), f"{cfg.name}_{a.mode}")
        res["event_ms"] = round(ev[0].elapsed_time(ev[1]), 4)
    tl = res.pop("timeline_per_simd")
    print(json.dumps(res, indent=1))
    print("us  " + "  ".join(f"{k:>6s}" for k in tl))
    for i in range(len(tl["load"])):
        print(f"{i:3d} " + "  ".join(f"{tl[k][i]:6.2f}" for k in tl))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump({**res, "timeline_per_simd": tl}, fh)


if __name__ == "__main__":
    main()
