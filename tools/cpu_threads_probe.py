"""CPU-baseline thread sweep (development tool; evidence for bench.py's host_cpu_budget policy).

    python tools/cpu_threads_probe.py [--rows 270] [--threads 1 8 16 32 64]

Times bench.py's CPU leg (the reference's pixel shader built for the host, oracle/_ref, one row band per
thread) on the same rows of the config-3 frame at each thread count and prints one JSON line per count,
together with the affinity mask, os.cpu_count() and the cgroup quota. Under a cgroup quota, threads beyond it
share the same CPU time, so the rate should stop rising at the quota.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402
from physically_based_renderer_amd import scenes as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=270)
    ap.add_argument("--threads", type=int, nargs="+", default=[1, 8, 16, 32, 64])
    a = ap.parse_args()
    from oracle import oracle as O  # test infrastructure: the CPU leg being timed

    cfg = S.CONFIGS[3]
    planes, _ = S.fill_gbuffer_host(cfg)
    sample = np.ascontiguousarray(planes[:, : a.rows])
    pc = S.scene_pass(cfg)
    env = S.env_map()
    use_ref = O.ref_available()
    print(json.dumps({"host_cpus": bench.host_cpu_budget(), "kind": "reference" if use_ref else "port",
                      "sample_px": int(sample.shape[1] * sample.shape[2])}), flush=True)
    for n in a.threads:
        t0 = time.perf_counter()
        bench.cpu_shade(sample, pc, env, n, use_ref, False)
        dt = time.perf_counter() - t0
        print(json.dumps({"threads": n, "seconds": round(dt, 3),
                          "mpix_s": round(sample.shape[1] * sample.shape[2] / dt / 1e6, 4)}), flush=True)


if __name__ == "__main__":
    main()
