"""Host -> HBM upload rate of a G-buffer (development tool; VERDICT r03 asked why bench.py's pcie_h2d_gbps read
3 GB/s). Uploads the 15-plane config-3 G-buffer (498 MB) several ways and prints one JSON line per way:

  pinned_first     torch pinned staging filled by pbr_gbuffer_fill, the first .to(device) of the process (what
                   bench.py times)
  pinned_again     the same copy repeated (DMA engine, page tables and the driver's pinned-buffer state warm)
  pinned_chunked   8 row chunks, each its own copy, on the same stream
  pageable         the fill into plain (pageable) numpy memory, uploaded with torch.from_numpy(..).to(device)
  pinned_into      copy_ into a preallocated device tensor (no allocation inside the timed region)

usage: python tools/h2d_probe.py [--rows 2160] [--repeat 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2160)
    ap.add_argument("--repeat", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch

    from physically_based_renderer_amd import _native as N
    from physically_based_renderer_amd import scenes as S

    cfg = S.CONFIGS[3].with_size(3840, a.rows)
    dev = torch.device("cuda", 0)
    shape = (N.NUM_PLANES, cfg.height, cfg.width)
    nbytes = int(np.prod(shape)) * 4

    def timed(name, fn, extra=None):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"way": name, "bytes": nbytes, "ms": round(dt * 1e3, 2), "gbps": round(nbytes / dt / 1e9, 2),
                          **(extra or {})}), flush=True)
        return out

    t0 = time.perf_counter()
    staging = torch.empty(shape, dtype=torch.float32, pin_memory=True)
    t_alloc = time.perf_counter() - t0
    S.fill_gbuffer_host(cfg, out=staging.numpy())
    print(json.dumps({"way": "pinned_alloc", "ms": round(t_alloc * 1e3, 2), "is_pinned": staging.is_pinned()}))
    d = timed("pinned_first", lambda: staging.to(dev, non_blocking=True))
    for _ in range(a.repeat):
        del d
        d = timed("pinned_again", lambda: staging.to(dev, non_blocking=True))
    dst = torch.empty(shape, dtype=torch.float32, device=dev)
    for _ in range(a.repeat):
        timed("pinned_into", lambda: dst.copy_(staging, non_blocking=True))

    def chunked():
        k = 8
        edges = np.linspace(0, cfg.height, k + 1).astype(int)
        for r0, r1 in zip(edges[:-1], edges[1:]):
            dst[:, r0:r1].copy_(staging[:, r0:r1], non_blocking=True)
    for _ in range(a.repeat):
        timed("pinned_chunked_8", chunked)
    host = np.empty(shape, np.float32)
    S.fill_gbuffer_host(cfg, out=host)
    for _ in range(a.repeat):
        timed("pageable", lambda: dst.copy_(torch.from_numpy(host)))
    assert torch.equal(dst.cpu(), staging)


if __name__ == "__main__":
    main()
