"""The multi-rank path with the HIP kernel: several ranks share the one GPU of the test box (gloo,
host-staged gather; the benchmark itself uses RCCL, one GPU per rank).

SURVEY §4 item 6: the gathered image must equal the single-GPU image bit for bit, run as 8 ranks over
fewer devices. Also rehearses bench.py's own N > 1 leg (partition, pipelined gather, band checksums,
max-over-ranks timing) under torch.distributed.run.
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu

WIDTH, HEIGHT = 200, 203  # ragged: bands of 8-row tiles plus a short tail


# Rendezvous without a pre-picked TCP port (a port probed free here and bound later by the ranks can be taken in
# between): the spawned ranks meet in a file store (PBR_DIST_INIT_METHOD), torchrun runs --standalone (it picks its
# own free port for its rendezvous and hands it to the ranks).
TORCHRUN = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--standalone", "--local-addr", "127.0.0.1"]


def _worker(rank, world, init, q):
    sys.path.insert(0, ROOT)
    os.environ.update(PBR_DIST_INIT_METHOD=init, RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from physically_based_renderer_amd import dist as D
    from physically_based_renderer_amd import scenes as S
    from physically_based_renderer_amd.renderer import ShadingContext

    D.init_from_env("gloo")
    dev = torch.device("cuda", 0)
    cfg = S.CONFIGS[3].with_size(WIDTH, HEIGHT)
    band = D.band_rows(cfg.height, world, rank)
    gb = S.build_gbuffer(cfg, dev, band.row_begin, band.row_end, n_threads=2)
    slot = torch.zeros((band.rows_max, cfg.width, 4), dtype=torch.float32, device=dev)
    with ShadingContext(0) as ctx:
        ctx.set_pass(S.scene_pass(cfg))
        ctx.set_env_map(S.env_map())
        ctx.shade(gb, slot[: band.rows])
        torch.cuda.synchronize()
    g = D.BandGather(band, cfg.width, dev)
    D.BandGather.wait(g.start(slot))
    frame = g.assembled(cfg.height)
    if rank == 0:
        q.put(frame.cpu().numpy().copy())
        q.close()
        q.join_thread()  # flushed before the process can end
    dist.barrier()
    dist.destroy_process_group()


def test_eight_ranks_on_one_gpu_equal_single_frame(gpu):
    from physically_based_renderer_amd import scenes as S
    from physically_based_renderer_amd.renderer import ShadingContext

    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.TemporaryDirectory(prefix="pbr_rdzv_") as tmp:
        procs = [ctx.Process(target=_worker, args=(r, world, "file://" + os.path.join(tmp, "store"), q))
                 for r in range(world)]
        for p in procs:
            p.start()
        frame = q.get(timeout=300)
        for p in procs:
            p.join(timeout=120)
            assert p.exitcode == 0
    cfg = S.CONFIGS[3].with_size(WIDTH, HEIGHT)
    with ShadingContext(0) as sc:
        sc.set_pass(S.scene_pass(cfg))
        sc.set_env_map(S.env_map())
        whole = sc.shade(S.build_gbuffer(cfg, gpu)).cpu().numpy()
    assert frame.shape == whole.shape
    assert np.array_equal(frame.view(np.uint32), whole.view(np.uint32))


def test_bench_multi_rank_rehearsal(gpu):
    """bench.py at N = 4 (gloo, the one GPU shared): one JSON line from rank 0 with the gathered bands'
    checksums matching and the per-rank band geometry of config 5."""
    cmd = TORCHRUN + ["--nproc-per-node", "4", os.path.join(ROOT, "bench.py"),
           "--gpus", "4", "--steps", "3", "--warmup", "1", "--ramp-ms", "0", "--dist-backend", "gloo",
           "--rows-per-rank", "64"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT,
                       env={**os.environ, "OMP_NUM_THREADS": "2"})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    d = lines[0]
    assert d["n_gpus"] == 4 and d["scaling"] == "weak"
    assert d["gather_checksums_match"] is True
    assert d["config"]["workload"].startswith("cfg5_8192x8192_64pt_ibl_rowbands")
    assert d["config"]["rows_per_rank"] == 64 and d["config"]["width"] == 8192
    assert d["value"] > 0 and d["cpu_baseline"] is None
    assert d["output"] == "rgba8"  # config 5 gathers the presented back-buffer format by default
    gp = d["gathered_frame_parity"]  # sampled rows of every band against the CPU oracle
    assert gp["rows_checked"] == 4 * 8 and gp["parity_max_code_diff"] <= 1
    assert d["shade_ms"] > 0 and d["gather_ms"] > 0
    # the scaling anchor: rank 0's own band (identical per-rank geometry at every N) shaded alone
    a = d["scale_anchor"]
    assert a["workload"] == d["config"]["workload"] + "_band64" or a["workload"].endswith("_band64")
    assert a["px_per_step"] == 8192 * 64 and a["output"] == "rgba8" and a["mode"] == d["mode"]
    assert d["per_rank_mpix_s"] == pytest.approx(d["value"] / 4, abs=0.01)
    assert d["efficiency_vs_anchor"] == pytest.approx(d["per_rank_mpix_s"] / a["value"], rel=1e-3)


def _bench_torchrun(nproc, extra, timeout=600):
    cmd = TORCHRUN + ["--nproc-per-node", str(nproc), os.path.join(ROOT, "bench.py"),
           "--gpus", str(nproc), "--steps", "3", "--warmup", "1", "--ramp-ms", "0"] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT,
                       env={**os.environ, "OMP_NUM_THREADS": "2"})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    return lines[0]


def test_bench_fp32_gather_parity_multi_rank(gpu):
    """--output rgba32f at N = 3 (gloo on the one GPU): the fp32 bands are gathered and rank 0 checks the
    assembled frame against the CPU oracle on 8 rows of every band (faithful mode: within 1e-5)."""
    d = _bench_torchrun(3, ["--dist-backend", "gloo", "--rows-per-rank", "64", "--output", "rgba32f"])
    assert d["output"] == "rgba32f" and d["gather_checksums_match"] is True
    gp = d["gathered_frame_parity"]
    assert gp["rows_checked"] == 24 and gp["parity_max_rel"] <= 1e-5


def test_bench_rccl_single_rank(gpu):
    """The RCCL path that runs on a one-GPU box: torch.distributed.run with one rank creates the nccl (RCCL)
    process group with device_id, gathers rank 0's band, runs the device-side checksum all_gather and the
    max-over-ranks all_reduce on RCCL, and tears the communicator down -- the same calls as at N = 8."""
    d = _bench_torchrun(1, ["--config", "5", "--rows-per-rank", "64", "--dist-backend", "nccl",
                            "--no-cpu-baseline"])
    assert d["process_group"] == "nccl" and d["gather_checksums_match"] is True
    assert d["n_gpus"] == 1 and d["config"]["rows_per_rank"] == 64 and d["output"] == "rgba8"


def test_bench_config5_one_gpu_is_the_per_rank_workload(gpu):
    """`bench.py --gpus 1 --config 5`: the same 8192 x 1024 band and RGBA8 output each rank of the N = 8 run
    shades (so the 1 -> 8 curve compares equal work), with the CPU leg on a row sample of that band."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--config", "5", "--steps",
                        "3", "--warmup", "1", "--ramp-ms", "0", "--cpu-rows", "16", "--cpu-kind", "port"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert d["config"]["width"] == 8192 and d["config"]["height"] == 1024 and d["config"]["rows_per_rank"] == 1024
    assert d["output"] == "rgba8" and d["gather_checksums_match"] is True and d["process_group"] is None
    assert d["cpu_baseline"]["kind"] == "port" and d["parity_max_code_diff"] <= 1


def test_bench_default_line_carries_anchor_and_executed_roofline(gpu):
    """`bench.py --gpus 1` (config 3): the line carries the scaling anchor -- one rank's config-5 band of
    --rows-per-rank rows, RGBA8, the same mode -- and both roofline fractions, the executed one counting only
    the terms the pass evaluated (the wave-balanced lists skip back-facing ones)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "3", "--warmup",
                        "1", "--ramp-ms", "0", "--no-cpu-baseline", "--rows-per-rank", "64"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert d["config"]["workload"] == "cfg3_3840x2160_64pt_ibl_chelsea" and d["n_gpus"] == 1
    a = d["scale_anchor"]
    assert a["workload"] == "cfg5_8192x8192_64pt_ibl_rowbands_band64" or a["workload"].endswith("_band64")
    assert a["px_per_step"] == 8192 * 64 and a["output"] == "rgba8" and a["value"] > 0 and a["shade_ms"] > 0
    assert a["clock_ramp"] == {"ms": 0.0, "launches": 0}  # --ramp-ms 0: the anchor ramps like the headline
    rf = d["roofline"]
    assert rf["bound"] == "mfma" and rf["flop_per_px"] == 5958
    st = rf["pass_stats"]
    # nearly every wave is lean and builds the lists (64 back-face tests per pixel); the rest run the uniform loop
    assert st["geometry_pixels"] == 3840 * 2160 and 0.99 * 64 * 3840 * 2160 <= st["backface_tests"] <= 64 * 3840 * 2160
    assert 0.3 * 64 * 3840 * 2160 < st["light_terms"] < 0.7 * 64 * 3840 * 2160
    assert rf["executed_flop_per_px"] < rf["flop_per_px"] and 0 < rf["frac_executed"] < rf["frac"]
    assert rf["pmc"]["kernel_sources_sha"] and (rf["traffic"] is None) == bool(rf["pmc"].get("stale"))


def test_bench_exits_nonzero_on_a_parity_breach(gpu):
    """The real bench process refuses a frame off the 1e-5 bar: with one channel of the checked frame scaled by
    1 + 2e-5 it exits with bench.EXIT_PARITY and prints no metric line; the same run without the injection
    prints its line with parity_ok true."""
    import bench

    base = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--config", "1", "--steps", "3",
            "--warmup", "1", "--ramp-ms", "0", "--no-anchor", "--cpu-kind", "port"]
    r = subprocess.run(base + ["--inject-parity-breach", "2e-5"], capture_output=True, text=True, timeout=600,
                       cwd=ROOT)
    assert r.returncode == bench.EXIT_PARITY, r.stderr[-3000:]
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")] and "PARITY FAILURE" in r.stderr
    r = subprocess.run(base, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert d["parity_ok"] is True and d["parity_checked"] is True and d["parity_max_rel"] <= 1e-5
