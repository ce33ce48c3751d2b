"""Same-box A/B timing of kernel builds (development tool; not part of the product or the tests).

    python tools/ab_bench.py --libs A.so B.so[@ENV=VALUE,...] [--configs 3 4 2] [--rounds 2] [--reps 30]

Each (round, lib, config) runs in a fresh subprocess with PBR_LIB_PATH pointing at that build: the
G-buffer is filled, the clock ramped (tools/clock_ramp.py), then `reps` launches are timed with HIP
events on the launch stream and the median is printed. Rounds alternate the libraries (A B A B ...)
so that clock drift on the box affects both alike. Every run also checks the frame against the first
library's frame (bit-identical or not) through a checksum of the fp32 bit patterns.
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(lib: str, cid: int, reps: int, flags: int = 0) -> dict:
    label = lib
    if "@" in lib:  # "build.so@NAME=VALUE,NAME=VALUE": environment for this leg (e.g. PBR_BALANCED_MIN=0)
        lib, envs = lib.split("@", 1)
        for kv in envs.split(","):
            k, v = kv.split("=", 1)
            os.environ[k] = v
    os.environ["PBR_LIB_PATH"] = os.path.abspath(lib)
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import numpy as np
    import torch

    from clock_ramp import clock_ramp
    from physically_based_renderer_amd import scenes as S
    from physically_based_renderer_amd.renderer import GBuffer, ShadingContext

    cfg = S.CONFIGS[cid]
    planes, _ = S.fill_gbuffer_host(cfg)
    pc = S.scene_pass(cfg)
    pc.flags = int(pc.flags) | flags
    dev = torch.device("cuda", 0)
    gb = GBuffer.from_host(planes, dev)
    out = torch.empty((cfg.height, cfg.width, 4), device=dev)
    with ShadingContext(0) as ctx:
        ctx.set_pass(pc)
        if pc.ambient_mode:
            ctx.set_env_map(S.env_map())
        clock_ramp(ctx, gb, out)
        stream = torch.cuda.current_stream(dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for a, b in ev:
            a.record(stream)
            ctx.shade(gb, out, stream)
            b.record(stream)
        torch.cuda.synchronize()
        ms = [a.elapsed_time(b) for a, b in ev]
        bits = out.view(torch.int32).to(torch.int64)
        csum = int((bits * (torch.arange(bits.numel(), device=dev, dtype=torch.int64).view(bits.shape) % 65521 + 1)).sum())
    return {"lib": label, "config": cid, "median_ms": float(np.median(ms)), "min_ms": float(np.min(ms)),
            "mpix_s": cfg.width * cfg.height / float(np.median(ms)) / 1e3, "checksum": csum}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--configs", nargs="+", type=int, default=[3])
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--flags", type=int, default=0, help="extra pass flags, e.g. 16 = PBR_FLAG_FAITHFUL")
    ap.add_argument("--one", nargs=2, help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.one:
        print(json.dumps(one(a.one[0], int(a.one[1]), a.reps, a.flags)), flush=True)
        return
    results = {}
    for r in range(a.rounds):
        order = a.libs if r % 2 == 0 else list(reversed(a.libs))
        for cid in a.configs:
            for lib in order:
                p = subprocess.run([sys.executable, __file__, "--libs", lib, "--reps", str(a.reps), "--flags", str(a.flags),
                                    "--one", lib, str(cid)],
                                   capture_output=True, text=True, timeout=300)
                if p.returncode != 0:
                    print(p.stdout, p.stderr, file=sys.stderr)
                    raise SystemExit(f"{lib} config {cid}: exit {p.returncode}")
                res = json.loads(p.stdout.strip().splitlines()[-1])
                results.setdefault((cid, lib), []).append(res)
                print(json.dumps(res), flush=True)
    print("summary (median of per-run medians):")
    for cid in a.configs:
        base = None
        ref_sum = results[(cid, a.libs[0])][0]["checksum"]
        for lib in a.libs:
            ms = sorted(x["median_ms"] for x in results[(cid, lib)])
            med = ms[len(ms) // 2]
            base = base or med
            same = all(x["checksum"] == ref_sum for x in results[(cid, lib)])
            print(f"  cfg{cid} {lib:28s} {med:.4f} ms  ({base / med:.4f}x vs first)  "
                  f"frame {'==' if same else '!='} first lib's")


if __name__ == "__main__":
    main()
